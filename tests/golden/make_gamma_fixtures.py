"""Extract the reference's own recorded outputs on the selfish-mining (gamma) network.

1. withholding_nakamoto_gamma.json — the 112 Nakamoto `gamma-*` rows of
   /root/reference/data/withholding.tsv, written by the reference's batch runner
   (experiments/simulate/withholding.ml:29-52 + models.ml:54-84: Network.T.selfish_mining
   with activation delay 1, defender message delay 1e-4, defenders = max 2 ceil(1/(1-gamma)),
   the nakamoto_ssz attacker as node 0, Simulator.loop of 10,000 activations,
   csv_runner.ml:244-265). Their OCaml Random start states are unknown (Parany workers), so
   they are statistical anchors: inputs (alpha, gamma, defenders, policy) and outputs
   (activations and reward per node, head time, progress, height, miner).
2. rl_results_seq_hc.json — the `gamma*_seq_hc` columns of
   experiments/rl-eval/rl-results.csv: for cpr-v0 Nakamoto (defenders = 42, episode_len
   2048, eval-policies.ipynb), the best mean over the hard-coded policies
   {sapirshtein-2016-sm1, honest} of episode_reward_attacker / episode_progress over 100
   episodes (rl-results-condensed.ipynb `best_models`, rpp_mean).

Only data columns are kept. Run here (the container that has /root/reference):
    python tests/golden/make_gamma_fixtures.py
"""

import csv
import json
import pathlib

REF = pathlib.Path("/root/reference")
HERE = pathlib.Path(__file__).parent
POLICY = {"ssz-honest": "honest", "ssz-simple": "simple", "ssz-eyal-sirer-2014": "eyal-sirer-2014",
          "ssz-sapirshtein-2016-sm1": "sapirshtein-2016-sm1"}


def withholding_gamma():
    rows = []
    with (REF / "data" / "withholding.tsv").open() as f:
        for ln, row in enumerate(csv.DictReader(f, delimiter="\t"), start=2):
            if not row["network"].startswith("gamma-") or row["protocol"] != "nakamoto":
                continue
            compute = [float(x) for x in row["compute"].split("|")]
            rows.append(dict(
                line=ln,
                alpha=compute[0],
                gamma=float(row["network"][len("gamma-"):]),
                defenders=len(compute) - 1,
                policy=POLICY[row["strategy"]],
                activations=int(row["number_activations"]),
                activations_per_node=[int(x) for x in row["activations"].split("|")],
                reward=[float(x) for x in row["reward"].split("|")],
                head_time=row["head_time"],
                head_progress=float(row["head_progress"]),
                head_height=int(row["head_height"]),
                head_miner=int(row["head_miner"]),
            ))
    out = HERE / "withholding_nakamoto_gamma.json"
    out.write_text(json.dumps({"source": "data/withholding.tsv", "msg_delay": 1e-4,
                               "rows": rows}, indent=1) + "\n")
    print(f"wrote {len(rows)} rows to {out}")


def rl_results():
    rows = []
    with (REF / "experiments" / "rl-eval" / "rl-results.csv").open() as f:
        for row in csv.DictReader(f):
            for g, gamma in (("gamma05", 0.05), ("gamma50", 0.5), ("gamma95", 0.95)):
                rows.append(dict(alpha=float(row["alpha"]), gamma=gamma,
                                 rpp_mean=float(row[f"{g}_seq_hc"])))
    out = HERE / "rl_results_seq_hc.json"
    out.write_text(json.dumps({
        "source": "experiments/rl-eval/rl-results.csv (gamma*_seq_hc)",
        "env": "cpr_gym:cpr-v0 nakamoto, defenders 42, episode_len 2048, 100 episodes",
        "policies": ["sapirshtein-2016-sm1", "honest"],
        "statistic": "max over policies of mean(episode_reward_attacker / episode_progress)",
        "rows": rows}, indent=1) + "\n")
    print(f"wrote {len(rows)} rows to {out}")


if __name__ == "__main__":
    withholding_gamma()
    rl_results()
