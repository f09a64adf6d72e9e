"""Batch experiments in the reference's TSV format, run on the device.

The reference's simulate experiments (experiments/simulate/honest_net.ml, withholding.ml)
build a list of Simulator.loop tasks — a network, a protocol, optionally an attack — run
each one (csv_runner.ml:56-98) and write one row per task with Info.pp_rows
(simulator/lib/info.ml:24-58) as a tab-separated file. Here every task runs as one episode
of a libcpr_hip batch in LOOP mode; the per-node `activations` and `reward` columns come
from cpr_node_outputs (the head's per-node reward array, simulator.ml:377-388).

Randomness is the keyed stream: episode e of a task is a pure function of
(seed, e), so rows are reproducible but not the reference's OCaml Random draws (the tests
replay those through traces). Tasks whose protocol has no device engine (SPar, STree) are
not generated; a task the device flags (CPR_ST_REFERENCE_RAISES / CPR_ST_CAPACITY) becomes
an `error` row, as csv_runner.ml:83-101 writes for an exception.

    python -m cpr_amd.csv_runner honest_net out.tsv --activations 10000
    python -m cpr_amd.csv_runner withholding out.tsv --activations 10000
"""

import argparse
import math
import sys
import time
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L

# ---------------------------------------------------------------- simulator/lib/info.ml


def string_of_float(x):
    """OCaml's string_of_float: "%.12g", plus a trailing "." when the result would read as
    an integer (Stdlib.valid_float_lexem)."""
    x = float(x)
    if math.isnan(x):
        return "nan"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    s = "%.12g" % x
    return s if any(c not in "0123456789-" for c in s) else s + "."


def string_of_value(v):
    """Info.string_of_value (info.ml:7-12)."""
    if isinstance(v, (bool, np.bool_)):
        return "true" if v else "false"
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if isinstance(v, (float, np.floating)):
        return string_of_float(v)
    return str(v)


def pp_rows(rows, sep="\t"):
    """Info.pp_rows (info.ml:24-58): a header of every key in order of first appearance,
    then one line per row, empty fields where a row lacks a key (a key repeated within a
    row keeps its last value)."""
    cols, idx = [], {}
    for r in rows:
        for k, _ in r:
            if k not in idx:
                idx[k] = len(cols)
                cols.append(k)
    lines = [sep.join(cols)]
    for r in rows:
        a = [""] * len(cols)
        for k, v in r:
            a[idx[k]] = string_of_value(v)
        lines.append(sep.join(a))
    return "\n".join(lines) + "\n"


def save_rows_as_tsv(filename, rows):
    """csv_runner.ml:16-29."""
    with open(filename, "w") as f:
        f.write(pp_rows(rows, sep="\t"))


def _join(xs, f):
    """csv_runner.ml:31-35 array / floatarray columns: values joined by "|"."""
    return "|".join(f(x) for x in xs)


# ---------------------------------------------------------------- protocols and attacks


@dataclass
class Protocol:
    """A protocol on the device with its Protocol.info (nakamoto.ml:6-9, ethereum.ml:57-64,
    bk.ml:21-24, tailstorm.ml:45-52)."""

    proto: int
    info: list
    k: int = 8
    scheme: int = L.REWARD_CONSTANT
    selection: int = L.SELECT_HEURISTIC

    def head_info(self, rec):
        """Referee.info of the head (nakamoto.ml:22-27, ethereum.ml:92-95, bk.ml:53-58,
        tailstorm.ml:89-94)."""
        h = int(rec["head_height"])
        if self.proto == L.PROTO_NAKAMOTO:
            m = int(rec["head_miner"])
            return [("height", h), ("miner", str(m) if m >= 0 else "n/a")]
        if self.proto == L.PROTO_ETHEREUM:
            return [("height", h), ("work", int(rec["head_work"]))]
        if self.proto == L.PROTO_BK:
            return [("kind", "block"), ("height", h)]
        return [("kind", "summary"), ("height", h)]


_SCHEMES = {"constant": L.REWARD_CONSTANT, "discount": L.REWARD_DISCOUNT,
            "block": L.REWARD_BLOCK, "punish": L.REWARD_PUNISH, "hybrid": L.REWARD_HYBRID}
_SELECTIONS = {"altruistic": L.SELECT_ALTRUISTIC, "heuristic": L.SELECT_HEURISTIC,
               "optimal": L.SELECT_OPTIMAL}


def nakamoto():
    return Protocol(L.PROTO_NAKAMOTO, [("family", "nakamoto")])


def ethereum(incentive_scheme="discount"):
    return Protocol(L.PROTO_ETHEREUM,
                    [("preference", "heaviest_chain"), ("progress", "work"), ("max_uncles", 2),
                     ("incentive_scheme", incentive_scheme)],
                    scheme=_SCHEMES[incentive_scheme])


def bk(k, incentive_scheme):
    return Protocol(L.PROTO_BK, [("family", "bk"), ("k", k), ("incentive_scheme", incentive_scheme)],
                    k=k, scheme=_SCHEMES[incentive_scheme])


def tailstorm(k, incentive_scheme, subblock_selection):
    return Protocol(L.PROTO_TAILSTORM,
                    [("family", "tailstorm"), ("k", k), ("incentive_scheme", incentive_scheme),
                     ("subblock_selection", subblock_selection)],
                    k=k, scheme=_SCHEMES[incentive_scheme],
                    selection=_SELECTIONS[subblock_selection])


# attack spaces with unit observations (nakamoto_ssz.ml:15-21 and the ethereum_ssz,
# bk_ssz, tailstorm_ssz equivalents) and their policy collections in registry order
_SSZ_LIKE = "SSZ'16-like attack space with unit observations"
ATTACK_SPACES = {
    L.PROTO_NAKAMOTO: ("ssz-unitobs", "SSZ'16 attack space with unit observations", [
        ("honest", "emulate honest behaviour", L.POLICY_HONEST),
        ("simple", "simple withholding policy", L.POLICY_SIMPLE),
        ("eyal-sirer-2014", "Eyal and Sirer 2014", L.POLICY_EYAL_SIRER_2014),
        ("sapirshtein-2016-sm1", "Sapirshtein et al. 2016, SM1", L.POLICY_SAPIRSHTEIN_2016_SM1),
    ]),  # nakamoto_ssz.ml:342-350
    L.PROTO_ETHEREUM: ("ssz-unitobs", _SSZ_LIKE, [
        ("honest", "emulate honest behaviour", L.ETH_POLICY_HONEST),
        ("selfish_release", "ad-hoc selfish policy w/ release on adopt",
         L.ETH_POLICY_SELFISH_RELEASE),
        ("selfish_discard", "ad-hoc selfish policy w/ discard on adopt",
         L.ETH_POLICY_SELFISH_DISCARD),
        ("fn19", "Feng and Niu. Selfish mining in Ethereum. ICDCS '19.", L.ETH_POLICY_FN19),
        ("fn19pkel", "Improved? version of Feng and Niu @ ICDCS '19.", L.ETH_POLICY_FN19PKEL),
    ]),  # ethereum_ssz.ml:523-538
    L.PROTO_BK: ("ssz-unitobs", _SSZ_LIKE, [
        ("honest", "emulate honest behaviour", L.BK_POLICY_HONEST),
        ("get-ahead", "release private block a.s.a.p.", L.BK_POLICY_GET_AHEAD),
        ("minor-delay", "override public block a.s.a.p.", L.BK_POLICY_MINOR_DELAY),
        ("avoid-loss", "override public head just before defender catches up",
         L.BK_POLICY_AVOID_LOSS),
    ]),  # bk_ssz.ml:404-415
    L.PROTO_TAILSTORM: ("ssz-unitobs", _SSZ_LIKE, [
        ("honest", "emulate honest behaviour", L.TS_POLICY_HONEST),
        ("get-ahead", "release private block a.s.a.p.", L.TS_POLICY_GET_AHEAD),
        ("minor-delay", "override public block a.s.a.p.", L.TS_POLICY_MINOR_DELAY),
        ("avoid-loss", "override public head just before defender catches up",
         L.TS_POLICY_AVOID_LOSS),
        ("avoid-loss-a", "override public head just before defender catches up",
         L.TS_POLICY_AVOID_LOSS_A),
        ("avoid-loss-b", "override public head just before defender catches up",
         L.TS_POLICY_AVOID_LOSS_B),
        ("long-delay", "override public head just before defender catches up",
         L.TS_POLICY_LONG_DELAY),
    ]),  # tailstorm_ssz.ml:449-471
}


@dataclass
class Attack:
    """withholding.ml:8-15: key = space key ^ "-" ^ policy key, info = space info ^ "; " ^
    policy info."""

    key: str
    info: str
    policy: int


def attacks(protocol):
    space, sinfo, pols = ATTACK_SPACES[protocol.proto]
    return [Attack(f"{space}-{k}", f"{sinfo}; {i}", pid) for k, i, pid in pols]


# ---------------------------------------------------------------- networks (models.ml)


@dataclass
class Network:
    key: str
    info: str
    activation_delay: float
    compute: list
    cfg: dict = field(default_factory=dict)


def honest_clique(n, activation_delay):
    """models.ml:3-28: compute 1..n, uniform [0.5, 1.5) link delays."""
    return Network(f"honest-clique-{n}",
                   f"{n} nodes, compute 1..{n}, simple dissemination, uniform propagation "
                   "delay 0.5 .. 1.5", float(activation_delay), [float(i + 1) for i in range(n)],
                   dict(network=L.NET_HONEST_CLIQUE, defenders=n, alpha=0.0, gamma=0.0))


def two_agents(alpha):
    """models.ml:30-47 (Network.T.two_agents, activation delay 1)."""
    return Network("two-agents", f"2 nodes, alpha={alpha:g}, no propagation delays", 1.0,
                   [alpha, 1.0 - alpha], dict(network=L.NET_TWO_AGENTS, alpha=alpha, gamma=0.0))


def selfish_mining(alpha, gamma, defenders=None, msg_delay=1e-4):
    """models.ml:54-84 with withholding.ml:44-52's defenders = max 2 ceil(1/(1-gamma))."""
    if defenders is None:
        defenders = max(2, int(math.ceil(1.0 / (1.0 - gamma))))
    return Network(f"gamma-{gamma:g}",
                   f"1 attacker, alpha={alpha:g}, {defenders} symmetric defenders, constant "
                   f"propagation delays modeling gamma={gamma:g}. with defender message delay "
                   f"{msg_delay:g})", 1.0,
                   [alpha] + [(1.0 - alpha) / defenders] * defenders,
                   dict(network=L.NET_SELFISH_MINING, defenders=defenders, alpha=alpha,
                        gamma=gamma, propagation_delay=msg_delay))


@dataclass
class Task:
    """csv_runner.ml:3-14."""

    activations: int
    network: Network
    protocol: Protocol
    attack: Attack = None


def config_of(task, seed=0):
    from . import device

    p, n = task.protocol, task.network
    return device.make_config(
        protocol=p.proto, mode=L.MODE_LOOP, activations=task.activations, seed=seed,
        activation_delay=n.activation_delay, k=p.k, reward_scheme=p.scheme,
        subblock_selection=p.selection,
        policy=task.attack.policy if task.attack is not None else 0, **n.cfg)


def prepare_row(task):
    """csv_runner.ml:37-54."""
    a = task.attack
    return ([("network", task.network.key), ("network_description", task.network.info),
             ("activation_delay", float(task.network.activation_delay)),
             ("compute", _join(task.network.compute, string_of_float)),
             ("number_activations", int(task.activations)),
             ("strategy", a.key if a is not None else "none"),
             ("strategy_description", a.info if a is not None else ""),
             ("version", L.lib().cpr_version().decode())]
            + [("protocol" if k == "family" else k, v) for k, v in task.protocol.info])


def result_row(task, rec, acts, rews, duration):
    """csv_runner.ml:56-101 for one finished episode: rec one cpr_episode_record, acts and
    rews its per-node rows."""
    row = prepare_row(task)
    st = int(rec["status"])
    if st & L.ST_INVALID:
        what = ("the reference simulator raises an exception" if st & L.ST_REFERENCE_RAISES
                else "device lane capacity exceeded" if st & L.ST_CAPACITY
                else "trace too short")
        return row + [("error", what), ("machine_duration_s", float(duration))]
    return (row
            + [("machine_duration_s", float(duration)),
               ("activations", _join(acts, lambda x: str(int(x)))),
               ("reward", _join(rews, string_of_float)),
               ("head_time", float(rec["chain_time"])),
               ("head_progress", float(rec["progress"]))]
            + [("head_" + k, v) for k, v in task.protocol.head_info(rec)])


def run(tasks, ctx=None, seed=0, first_episode=0, progress=None):
    """Run every task as one keyed episode (task i: episode first_episode + i) and return
    the rows."""
    from . import device

    ctx = ctx or device.default_context()
    rows = []
    for i, t in enumerate(tasks):
        t0 = time.perf_counter()
        cfg, keep = config_of(t, seed)
        b = device.Batch(cfg, ctx=ctx, keep=keep)
        try:
            rec, acts, rews = b.node_outputs(1, first_episode + i)
        finally:
            b.close()
        rows.append(result_row(t, rec[0], acts[0], rews[0], time.perf_counter() - t0))
        if progress:
            progress(i + 1, len(tasks))
    return rows


# ---------------------------------------------------------------- task lists


def honest_net_tasks(n_activations):
    """honest_net.ml:4-42 without SPar / STree (no device engine)."""
    protocols = [nakamoto(), ethereum("discount")]
    for k in [1, 2, 4, 8, 16, 32]:
        protocols += [bk(k, s) for s in ("block", "constant")]
        sel = "heuristic" if k > 8 else "optimal"
        protocols += [tailstorm(k, s, sel) for s in ("constant", "discount")]
    return [Task(n_activations, honest_clique(10, d), p)
            for p in protocols for d in (30.0, 60.0, 120.0, 300.0, 600.0)]


ALPHAS = [0.1, 0.2, 0.25, 0.33, 0.4, 0.45, 0.5]
GAMMAS = [0.0, 0.5, 0.75, 0.9]


def withholding_tasks(n_activations):
    """withholding.ml:6-80 without SPar / STree: two-agents tasks for every attack space,
    selfish-mining (gamma) tasks for Nakamoto and Ethereum."""
    def over(nets, p):
        return [Task(n_activations, net, p, a) for net in nets for a in attacks(p)]

    two = [two_agents(a) for a in ALPHAS]
    sm = [selfish_mining(a, g) for a in ALPHAS for g in GAMMAS]
    tasks = over(two, nakamoto()) + over(sm, nakamoto())
    tasks += over(two, ethereum("discount")) + over(sm, ethereum("discount"))
    for k in [1, 2, 4, 8, 16, 32]:
        for s in ("block", "constant"):
            tasks += over(two, bk(k, s))
        sel = "heuristic" if k > 8 else "optimal"
        for s in ("constant", "discount"):
            tasks += over(two, tailstorm(k, s, sel))
    return tasks


EXPERIMENTS = {"honest_net": honest_net_tasks, "withholding": withholding_tasks}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("experiment", choices=sorted(EXPERIMENTS))
    ap.add_argument("output", help="name of the TSV output file")
    ap.add_argument("--activations", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--limit", type=int, default=0, help="run only the first N tasks")
    args = ap.parse_args(argv)
    tasks = EXPERIMENTS[args.experiment](args.activations)
    if args.limit:
        tasks = tasks[: args.limit]
    print(f"Run {len(tasks)} simulations on the device", file=sys.stderr)
    rows = run(tasks, seed=args.seed)
    save_rows_as_tsv(args.output, rows)


if __name__ == "__main__":
    main()
