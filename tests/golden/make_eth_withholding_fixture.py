"""Extract the reference's recorded Ethereum two-agents outputs into a fixture.

Source: /root/reference/data/withholding.tsv (experiments/simulate/withholding.ml, 10,000
activations per task, Byzantium parameters, ethereum_ssz policies). These rows started
from OCaml Random states that cannot be recovered, so they are one Monte
Carlo sample each: tests/test_oracle_eth.py compares them statistically. Only data
columns are kept.

Run here (the container that has /root/reference):
    python tests/golden/make_eth_withholding_fixture.py
"""

import csv
import json
import pathlib

SRC = pathlib.Path("/root/reference/data/withholding.tsv")
OUT = pathlib.Path(__file__).with_name("withholding_ethereum_two_agents.json")


def main():
    rows = []
    with SRC.open() as f:
        for ln, row in enumerate(csv.DictReader(f, delimiter="\t"), start=2):
            if row["network"] != "two-agents" or row["incentive_scheme"] == "":
                continue
            if row["preference"] == "" or row["protocol"] not in ("", "ethereum"):
                continue
            rows.append(
                dict(
                    line=ln,
                    alpha=float(row["compute"].split("|")[0]),
                    policy=row["strategy"].replace("ssz-", ""),
                    incentive_scheme=row["incentive_scheme"],
                    activations=int(row["number_activations"]),
                    activations_per_node=[int(x) for x in row["activations"].split("|")],
                    reward=[float(x) for x in row["reward"].split("|")],
                    head_progress=float(row["head_progress"]),
                    head_height=int(float(row["head_height"])),
                )
            )
    OUT.write_text(json.dumps({"source": "data/withholding.tsv", "rows": rows}, indent=1) + "\n")
    print(f"wrote {len(rows)} rows to {OUT}")


if __name__ == "__main__":
    main()
