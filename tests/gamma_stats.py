"""Statistical anchors on the selfish-mining (gamma) network: the reference's own recorded
outputs (tests/golden/make_gamma_fixtures.py) against independently seeded runs of the
same configuration. Shared by the oracle tests (CPU) and the device tests (-m gpu).

A recorded row is one draw of its task's outcome distribution, so for each output x the
check is |z| < bound with z = (x_ref - mean) / (sd * sqrt(1 + 1/N)) over N keyed tasks.
"""

import json
import math
import pathlib

import numpy as np

GOLDEN = pathlib.Path(__file__).parent / "golden"
POLICY_ID = {"honest": 0, "simple": 1, "eyal-sirer-2014": 2, "sapirshtein-2016-sm1": 3}


def withholding_rows():
    return json.loads((GOLDEN / "withholding_nakamoto_gamma.json").read_text())["rows"]


def rl_rows():
    return json.loads((GOLDEN / "rl_results_seq_hc.json").read_text())["rows"]


def row_config(make_config, L, row, seed):
    """cpr_config of a withholding gamma row (models.ml:54-84, withholding.ml:44-52)."""
    cfg, _ = make_config(alpha=row["alpha"], gamma=row["gamma"], defenders=row["defenders"],
                         policy=POLICY_ID[row["policy"]], mode=L.MODE_LOOP,
                         activations=row["activations"], propagation_delay=1e-4, seed=seed)
    return cfg


def z_score(ref, sample):
    sample = np.asarray(sample, dtype=np.float64)
    n = len(sample)
    mean = float(sample.mean())
    sd = float(sample.std(ddof=1))
    if sd == 0.0:
        return 0.0 if ref == mean else math.inf
    return (ref - mean) / (sd * math.sqrt(1.0 + 1.0 / n))


def rank_z(ref, sample):
    """Distribution-free z: the normal quantile of the sample's two-sided mid-rank tail
    probability at ref. The attacker's reward at gamma = 0 is heavy tailed (it is the length
    of the private fork still ahead when the loop ends), where mean/sd z-scores mislead.
    When ref lies outside the sample's range the tail is unresolved and the mean/sd z is
    returned instead."""
    from statistics import NormalDist

    sample = np.asarray(sample, dtype=np.float64)
    n = len(sample)
    above = int((sample > ref).sum())
    below = int((sample < ref).sum())
    equal = n - above - below
    if (above + equal == 0) or (below + equal == 0):
        return z_score(ref, sample)
    p_up = (above + 0.5 * equal) / n    # P(X > ref) + P(X = ref) / 2
    p_lo = (below + 0.5 * equal) / n
    p = min(p_up, p_lo)
    if p >= 0.5:
        return 0.0
    z = NormalDist().inv_cdf(1.0 - p)
    return z if p_up < p_lo else -z


OUTPUTS = ("reward_attacker", "reward_defender", "progress", "head_time")


def withholding_values(row):
    return {"reward_attacker": row["reward"][0], "reward_defender": sum(row["reward"][1:]),
            "progress": row["head_progress"], "head_time": float(row["head_time"])}


def record_values(rec):
    return {"reward_attacker": rec["reward_attacker"], "reward_defender": rec["reward_defender"],
            "progress": rec["progress"], "head_time": rec["chain_time"]}


def withholding_z(row, rec, stat=z_score, outputs=OUTPUTS):
    """z of attacker reward, defender reward (sum), progress and head time of one row
    against a record array (cpr_episode_record dtype) of N tasks."""
    ref, got = withholding_values(row), record_values(rec)
    return {k: stat(ref[k], got[k]) for k in outputs}


def rpp_z(ref, rpp_by_policy):
    """rl-results seq_hc: the reference reports the best mean over policies of
    episode_reward_attacker / episode_progress over 100 episodes; compare it with the best
    of ours, z over the reference's 100-episode standard error plus ours."""
    best = max(rpp_by_policy, key=lambda p: float(np.mean(rpp_by_policy[p])))
    x = np.asarray(rpp_by_policy[best], dtype=np.float64)
    se = math.sqrt(x.var(ddof=1) / 100.0 + x.var(ddof=1) / len(x))
    return best, float(x.mean()), (ref - float(x.mean())) / se
