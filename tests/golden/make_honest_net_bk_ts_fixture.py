"""Extract the reference's recorded B_k and Tailstorm honest-clique rows (k in {4, 8, 16},
activation delays 30 and 600) from data/honest_net.tsv into a fixture. Their Parany worker
states are unknown (the chains pass through SPar/STree tasks, see make_honest_net_chains.py),
so tests/test_oracle_clique.py compares them statistically with keyed oracle tasks.
Data only: inputs (protocol, k, scheme, selection, delay, nodes, activations) and outputs
(reward per node, head progress).

Run here (the container that has /root/reference):
    python tests/golden/make_honest_net_bk_ts_fixture.py
"""

import csv
import json
import pathlib

SRC = pathlib.Path("/root/reference/data/honest_net.tsv")
OUT = pathlib.Path(__file__).with_name("honest_net_bk_ts_rows.json")


def main():
    rows = []
    with SRC.open() as f:
        for ln, r in enumerate(csv.DictReader(f, delimiter="\t"), start=2):
            if r["protocol"] not in ("bk", "tailstorm") or r["k"] not in ("4", "8", "16"):
                continue
            if r["activation_delay"] not in ("30.", "600."):
                continue
            rows.append(dict(line=ln, protocol=r["protocol"], k=int(r["k"]),
                             incentive_scheme=r["incentive_scheme"],
                             subblock_selection=r["subblock_selection"] or None,
                             activation_delay=float(r["activation_delay"]),
                             nodes=len(r["compute"].split("|")),
                             activations=int(r["number_activations"]),
                             reward=[float(x) for x in r["reward"].split("|")],
                             head_progress=float(r["head_progress"])))
    OUT.write_text(json.dumps({"source": "data/honest_net.tsv", "rows": rows}, indent=1) + "\n")
    print(f"wrote {len(rows)} rows to {OUT}")


if __name__ == "__main__":
    main()
