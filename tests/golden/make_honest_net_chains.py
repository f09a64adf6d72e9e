"""Recover the Parany worker chains behind data/honest_net.tsv and write them as a fixture.

The reference's batch runner (experiments/simulate/csv_runner.ml:105-131) farms the tasks of
experiments/simulate/honest_net.ml over forked Parany workers. Each worker starts from OCaml's
default Random state and carries its state from one task to the next, so a row is
reproducible from the default state after replaying the rows its worker ran before it. The
rows are written in completion order, so a worker's previous task is an earlier line.

This script searches those chains with the oracle (the checker; OCaml 4.12 Random replica):
rows are visited in file order; each in-scope row (Nakamoto, Ethereum, B_k, Tailstorm) is
tried from the default state and from the end state of every earlier reproduced row whose
successor is still unknown. A row is accepted only if every recorded output matches bit for
bit (activations and reward of all 10 nodes, head time to the TSV's 12 digits, progress,
height). Chains through out-of-scope rows (spar, stree) cannot be followed.

Output: tests/golden/honest_net_chains.json — per reproduced row, the inputs, the recorded
outputs and the list of earlier lines replayed before it. Data only.

Run here (the container that has /root/reference):
    PYTHONPATH=tests python tests/golden/make_honest_net_chains.py
"""

import csv
import json
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import oracle_py as O  # noqa: E402

SRC = pathlib.Path("/root/reference/data/honest_net.tsv")
OUT = pathlib.Path(__file__).with_name("honest_net_chains.json")
SCHEMES = {"constant": 0, "block": 2, "discount": 1, "punish": 3, "hybrid": 4}  # cpr_hip.h


def spec_of(ln, row):
    p = row["protocol"]
    if p == "nakamoto":
        proto = "nakamoto"
    elif p in ("", "ethereum") and row["preference"] == "heaviest_chain":
        proto = "ethereum"
    elif p in ("bk", "tailstorm"):
        proto = p
    else:
        return None
    return dict(
        line=ln,
        protocol=proto,
        k=int(row["k"]) if row["k"] else None,
        incentive_scheme=row["incentive_scheme"] or None,
        subblock_selection=row["subblock_selection"] or None,
        activation_delay=float(row["activation_delay"]),
        nodes=len(row["compute"].split("|")),
        activations=int(row["number_activations"]),
        activations_per_node=[int(x) for x in row["activations"].split("|")],
        reward=[float(x) for x in row["reward"].split("|")],
        head_time=row["head_time"],
        head_progress=float(row["head_progress"]),
        head_height=int(row["head_height"]),
    )


def run(spec, rng):
    """One Simulator.loop task of `spec` on `rng` (advanced in place)."""
    n, ad, acts = spec["nodes"], spec["activation_delay"], spec["activations"]
    if spec["protocol"] in ("nakamoto", "ethereum"):
        sch = 0 if spec["incentive_scheme"] == "constant" else 1  # Ethereum: Constant/Discount
        return O.clique_task(spec["protocol"], n, ad, acts, scheme=sch, rng=rng)
    sch = SCHEMES[spec["incentive_scheme"]]
    if spec["protocol"] == "bk":
        return O.bk_loop(spec["k"], acts, net="honest-clique", n_nodes=n, activation_delay=ad,
                         scheme=sch, rng=rng)
    return O.ts_loop(spec["k"], acts, net="honest-clique", n_nodes=n, activation_delay=ad,
                     scheme=sch, selection=O.TS_SELECTIONS[spec["subblock_selection"]], rng=rng)


def matches(spec, out):
    return (out["activations"] == spec["activations_per_node"]
            and out["reward"] == spec["reward"]
            and float("%.12g" % out["head_time"]) == float(spec["head_time"])
            and out["head_progress"] == spec["head_progress"]
            and out["head_height"] == spec["head_height"])


def main():
    t0 = time.time()
    with SRC.open() as f:
        specs = [s for s in (spec_of(ln, r) for ln, r in
                             enumerate(csv.DictReader(f, delimiter="\t"), start=2)) if s]
    open_ends = {}  # line -> (end state, chain) of reproduced rows without a known successor
    found = []
    for spec in specs:
        cands = [(None, O.OcamlRandom(), [])] + [
            (ln, st.copy(), ch) for ln, (st, ch) in sorted(open_ends.items())]
        hit = None
        for pred, rng, chain in cands:
            if matches(spec, run(spec, rng)):
                hit = (pred, rng, chain)
                break
        if hit is None:
            print(f"line {spec['line']:4d} {spec['protocol']:9s} k={spec['k']} -", flush=True)
            continue
        pred, rng, chain = hit
        if pred is not None:
            del open_ends[pred]
        chain = chain + ([pred] if pred is not None else [])
        open_ends[spec["line"]] = (rng, chain)
        found.append(dict(spec, chain=chain))
        print(f"line {spec['line']:4d} {spec['protocol']:9s} k={spec['k']} after {chain}",
              flush=True)
    OUT.write_text(json.dumps({"source": "data/honest_net.tsv", "rows": found}, indent=1) + "\n")
    print(f"wrote {len(found)} of {len(specs)} in-scope rows to {OUT} ({time.time() - t0:.0f} s)")


if __name__ == "__main__":
    main()
