"""Extract the reference's own recorded honest-clique outputs (Nakamoto, Ethereum) into a
fixture.

Source: /root/reference/data/honest_net.tsv, written by the reference's batch runner
(experiments/simulate/honest_net.ml over models.ml:3-28 honest_clique: 10 nodes with compute
1..10, uniform 0.5..1.5 propagation delays, 10,000 activations per task). Every task there
starts from OCaml's default Random state. Only data columns are kept: inputs (protocol,
incentive scheme, activation delay, nodes, activations) and outputs (activations and
reward per node, head time / progress / height). The Ethereum rows carry an empty
`protocol` column in the TSV; they are the Byzantium rows (heaviest_chain, work, 2 uncles).

Run here (the container that has /root/reference):  python tests/golden/make_honest_net_fixture.py
"""

import csv
import json
import pathlib

SRC = pathlib.Path("/root/reference/data/honest_net.tsv")
OUT = pathlib.Path(__file__).with_name("honest_net_clique.json")


def main():
    rows = []
    with SRC.open() as f:
        for ln, row in enumerate(csv.DictReader(f, delimiter="\t"), start=2):
            if row["protocol"] == "nakamoto":
                proto, scheme = "nakamoto", None
            elif row["protocol"] in ("", "ethereum") and row["preference"] == "heaviest_chain":
                proto, scheme = "ethereum", row["incentive_scheme"]
            else:
                continue
            rows.append(
                dict(
                    line=ln,
                    protocol=proto,
                    incentive_scheme=scheme,
                    activation_delay=float(row["activation_delay"]),
                    nodes=len(row["compute"].split("|")),
                    activations=int(row["number_activations"]),
                    activations_per_node=[int(x) for x in row["activations"].split("|")],
                    reward=[float(x) for x in row["reward"].split("|")],
                    head_time=row["head_time"],
                    head_progress=float(row["head_progress"]),
                    head_height=int(row["head_height"]),
                )
            )
    OUT.write_text(json.dumps({"source": "data/honest_net.tsv", "rows": rows}, indent=1) + "\n")
    print(f"wrote {len(rows)} rows to {OUT}")


if __name__ == "__main__":
    main()
