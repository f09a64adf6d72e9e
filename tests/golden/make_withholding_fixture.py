"""Extract the reference's own recorded Nakamoto two-agents outputs into a fixture.

Source: /root/reference/data/withholding.tsv, written by the reference's batch runner
(experiments/simulate/withholding.ml + csv_runner.ml:244-265, 10,000 activations per task,
tasks run back to back in Parany workers so the OCaml Random state carries over).
Only data columns are kept: inputs (alpha, policy), and outputs (activations per node,
reward per node, head_time, head_progress). `prior_tasks` is how many two-agents tasks
(alpha < 0.5) ran before this row in the same worker, found by tests/test_oracle_kat.py's
search and verified there.

Run here (the container that has /root/reference):  python tests/golden/make_withholding_fixture.py
"""

import csv
import json
import pathlib

SRC = pathlib.Path("/root/reference/data/withholding.tsv")
OUT = pathlib.Path(__file__).with_name("withholding_nakamoto_two_agents.json")

# rows 2-13 start from the default state, 14-23,26,27 after one task, 24,25,210,249 after two
PRIOR = {**{ln: 0 for ln in range(2, 14)}, **{ln: 1 for ln in list(range(14, 24)) + [26, 27]},
         24: 2, 25: 2, 210: 2, 249: 2}
POLICY = {"ssz-honest": "honest", "ssz-simple": "simple", "ssz-eyal-sirer-2014": "eyal-sirer-2014",
          "ssz-sapirshtein-2016-sm1": "sapirshtein-2016-sm1"}


def main():
    rows = []
    with SRC.open() as f:
        for ln, row in enumerate(csv.DictReader(f, delimiter="\t"), start=2):
            if row["network"] != "two-agents" or row["protocol"] != "nakamoto":
                continue
            rows.append(
                dict(
                    line=ln,
                    alpha=float(row["compute"].split("|")[0]),
                    policy=POLICY[row["strategy"]],
                    activations=int(row["number_activations"]),
                    prior_tasks=PRIOR[ln],
                    activations_per_node=[int(x) for x in row["activations"].split("|")],
                    reward=[float(x) for x in row["reward"].split("|")],
                    head_time=row["head_time"],
                    head_progress=float(row["head_progress"]),
                )
            )
    OUT.write_text(json.dumps({"source": "data/withholding.tsv", "rows": rows}, indent=1) + "\n")
    print(f"wrote {len(rows)} rows to {OUT}")


if __name__ == "__main__":
    main()
