"""ctypes binding of the CPU oracle (oracle/build/liboracle.so) — TEST INFRASTRUCTURE.

The oracle is the checker: a faithful C++ restatement of the reference DES
(oracle/src/des.h). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg load it.
"""

import ctypes
import pathlib
import subprocess

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
LIB = ROOT / "oracle" / "build" / "liboracle.so"

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        import sys

        sys.path.insert(0, str(ROOT))
        from cpr_amd import _lib as C  # struct layouts only (no GPU needed)

        L = ctypes.CDLL(str(LIB))
        P = ctypes.POINTER
        vp = ctypes.c_void_p
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_ocaml_rng_new.restype = vp
        L.oracle_ocaml_rng_new.argtypes = [ctypes.c_long]
        L.oracle_ocaml_rng_free.argtypes = [vp]
        L.oracle_ocaml_rng_copy.restype = vp
        L.oracle_ocaml_rng_copy.argtypes = [vp]
        L.oracle_ocaml_rng_bits.argtypes = [vp]
        L.oracle_ocaml_rng_int.argtypes = [vp, ctypes.c_int32]
        L.oracle_ocaml_rng_float.argtypes = [vp, ctypes.c_double]
        L.oracle_ocaml_rng_float.restype = ctypes.c_double
        L.oracle_keyed_block.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                         ctypes.c_uint32, vp]
        L.oracle_philox_raw.argtypes = [vp, vp, vp]
        L.oracle_cpr_log.argtypes = [ctypes.c_double]
        L.oracle_cpr_log.restype = ctypes.c_double
        L.oracle_u53.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_u53.restype = ctypes.c_double
        L.oracle_nak_policy.argtypes = [ctypes.c_int, vp, vp, ctypes.c_int]
        L.oracle_nak_obs_to_floats.argtypes = [vp, ctypes.c_int, vp]
        L.oracle_nak_obs_of_floats.argtypes = [vp, ctypes.c_int, vp]
        L.oracle_two_agents_task.argtypes = [
            ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double, ctypes.c_int,
            ctypes.c_int, vp, vp, P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_int32),
            P(ctypes.c_uint32),
        ]
        L.oracle_clique_task.argtypes = [
            ctypes.c_int, ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
            ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int, vp,
            vp, P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_int32), P(ctypes.c_int32),
            P(ctypes.c_int32),
        ]
        L.oracle_gym_new.restype = vp
        L.oracle_gym_new.argtypes = [P(C.Config), ctypes.c_int, vp, ctypes.c_uint64]
        L.oracle_gym_free.argtypes = [vp]
        L.oracle_gym_reset.argtypes = [vp, vp]
        L.oracle_gym_obs_fields.argtypes = [vp, vp]
        L.oracle_gym_step.argtypes = [vp, ctypes.c_int, vp, P(ctypes.c_double), P(ctypes.c_int), vp]
        L.oracle_gym_diag.argtypes = [vp]
        L.oracle_gym_diag.restype = ctypes.c_uint32
        L.oracle_run_episodes.argtypes = [P(C.Config), ctypes.c_uint64, ctypes.c_int64, vp,
                                          ctypes.c_int]
        L.oracle_trace_record.restype = vp
        L.oracle_trace_record.argtypes = [P(C.Config), ctypes.c_int, vp, ctypes.c_uint64,
                                          ctypes.c_int64, vp]
        L.oracle_trace_sizes.argtypes = [vp, vp]
        L.oracle_trace_fill.argtypes = [vp] + [vp] * 8
        L.oracle_trace_free.argtypes = [vp]
        L.oracle_trace_replay.argtypes = [P(C.Config), P(C.CTrace), vp]
        L.oracle_node_outputs.argtypes = [P(C.Config), ctypes.c_uint64, ctypes.c_int64, vp,
                                          ctypes.c_int, vp, vp, vp, vp]
        L.oracle_ocaml_sort_ints.argtypes = [vp, ctypes.c_int]
        L.oracle_ocaml_sort_pairs.argtypes = [vp, vp, ctypes.c_int]
        L.oracle_at_most_first_ints.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        L.oracle_eth_dag_new.restype = vp
        L.oracle_eth_dag_new.argtypes = [ctypes.c_int, ctypes.c_int]
        L.oracle_eth_dag_free.argtypes = [vp]
        L.oracle_eth_dag_mine.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, P(ctypes.c_int32)]
        L.oracle_eth_policy.argtypes = [ctypes.c_int, vp, vp, ctypes.c_int]
        L.oracle_eth_obs_to_floats.argtypes = [vp, ctypes.c_int, vp]
        L.oracle_eth_obs_of_floats.argtypes = [vp, ctypes.c_int, vp]
        L.oracle_eth_gym_new.restype = vp
        L.oracle_eth_gym_new.argtypes = [P(C.Config), ctypes.c_int, vp, ctypes.c_uint64]
        L.oracle_eth_gym_free.argtypes = [vp]
        L.oracle_eth_gym_reset.argtypes = [vp, vp]
        L.oracle_eth_gym_obs_fields.argtypes = [vp, vp]
        L.oracle_eth_gym_step.argtypes = [vp, ctypes.c_int, vp, P(ctypes.c_double),
                                          P(ctypes.c_int), vp]
        L.oracle_eth_gym_diag.argtypes = [vp]
        L.oracle_eth_gym_diag.restype = ctypes.c_uint32
        L.oracle_eth_two_agents_task.argtypes = [
            ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, vp, vp, P(ctypes.c_double), P(ctypes.c_double),
            P(ctypes.c_int32), P(ctypes.c_int32), P(ctypes.c_uint32),
        ]
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        raise RuntimeError(lib().oracle_last_error().decode())


class OcamlRandom:
    def __init__(self, seed=-1):
        self.h = lib().oracle_ocaml_rng_new(seed)

    def __del__(self):
        try:
            lib().oracle_ocaml_rng_free(self.h)
        except Exception:
            pass

    def copy(self):
        c = OcamlRandom.__new__(OcamlRandom)
        c.h = lib().oracle_ocaml_rng_copy(self.h)
        return c

    def bits(self):
        return lib().oracle_ocaml_rng_bits(self.h)

    def int(self, n):
        return lib().oracle_ocaml_rng_int(self.h, n)

    def float(self, b):
        return lib().oracle_ocaml_rng_float(self.h, b)


POLICIES = {"honest": 0, "simple": 1, "eyal-sirer-2014": 2, "sapirshtein-2016-sm1": 3}


def two_agents_task(alpha, policy, activations, rng=None, seed=0, episode=0):
    """Simulator.loop task (csv_runner.ml:56-98) on the two-agents network."""
    acts = np.zeros(2, dtype=np.int64)
    rew = np.zeros(2, dtype=np.float64)
    ht, hp = ctypes.c_double(), ctypes.c_double()
    hh, dg = ctypes.c_int32(), ctypes.c_uint32()
    mode = 0 if rng is not None else 1
    check(
        lib().oracle_two_agents_task(
            mode, rng.h if rng is not None else None, seed, episode, alpha,
            POLICIES.get(policy, policy), activations, acts.ctypes.data, rew.ctypes.data,
            ctypes.byref(ht), ctypes.byref(hp), ctypes.byref(hh), ctypes.byref(dg),
        )
    )
    return dict(activations=acts.tolist(), reward=rew.tolist(), head_time=ht.value,
                head_progress=hp.value, head_height=hh.value, diag=dg.value)


def clique_task(protocol, n, activation_delay, activations, scheme=1, lo=0.5, hi=1.5, rng=None,
                seed=0, episode=0):
    """Simulator.loop task on models.ml:3-28 honest_clique (n honest nodes, compute i + 1,
    uniform [lo, hi) link delays); protocol "nakamoto" or "ethereum" (Byzantium, scheme)."""
    acts = np.zeros(n, dtype=np.int64)
    rew = np.zeros(n, dtype=np.float64)
    ht, hp = ctypes.c_double(), ctypes.c_double()
    hh, hm, hw = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    check(
        lib().oracle_clique_task(
            1 if protocol == "ethereum" else 0, 0 if rng is not None else 1,
            rng.h if rng is not None else None, seed, episode, n, activation_delay, lo, hi,
            scheme, activations, acts.ctypes.data, rew.ctypes.data, ctypes.byref(ht),
            ctypes.byref(hp), ctypes.byref(hh), ctypes.byref(hm), ctypes.byref(hw),
        )
    )
    return dict(activations=acts.tolist(), reward=rew.tolist(), head_time=ht.value,
                head_progress=hp.value, head_height=hh.value, head_miner=hm.value,
                head_work=hw.value)


def keyed_block(seed, episode, idx, tag):
    out = np.zeros(4, dtype=np.uint32)
    lib().oracle_keyed_block(seed, episode, idx, tag, out.ctypes.data)
    return out


def philox(ctr, key):
    c = np.asarray(ctr, dtype=np.uint32)
    k = np.asarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    lib().oracle_philox_raw(c.ctypes.data, k.ctypes.data, out.ctypes.data)
    return out


def cpr_log(x):
    return lib().oracle_cpr_log(x)


def u53(a, b):
    return lib().oracle_u53(a, b)


def nak_policy(policy, obs_fields, table=None):
    o = np.asarray(obs_fields, dtype=np.int32)
    if table is not None:
        t = np.ascontiguousarray(table, dtype=np.uint8)
        dim = int(round((t.size // 2) ** 0.5))
        return lib().oracle_nak_policy(policy, o.ctypes.data, t.ctypes.data, dim)
    return lib().oracle_nak_policy(policy, o.ctypes.data, None, 0)


def obs_to_floats(fields, unit):
    o = np.asarray(fields, dtype=np.int32)
    out = np.zeros(4)
    lib().oracle_nak_obs_to_floats(o.ctypes.data, 1 if unit else 0, out.ctypes.data)
    return out


def obs_of_floats(floats, unit):
    f = np.asarray(floats, dtype=np.float64)
    out = np.zeros(4, dtype=np.int32)
    lib().oracle_nak_obs_of_floats(f.ctypes.data, 1 if unit else 0, out.ctypes.data)
    return out


class GymEnv:
    """The oracle's engine.ml restatement (one env, keyed stream or OCaml Random)."""

    INFO_KEYS = [
        "step_reward_attacker", "step_reward_defender", "step_progress", "step_chain_time",
        "step_sim_time", "episode_reward_attacker", "episode_reward_defender",
        "episode_progress", "episode_chain_time", "episode_sim_time", "episode_n_steps",
        "episode_n_activations", "head_height", "head_miner",
    ]

    def __init__(self, config, episode=0, ocaml_rng=None):
        self.cfg = config
        self.h = lib().oracle_gym_new(ctypes.byref(config), 0 if ocaml_rng else 1,
                                      ocaml_rng.h if ocaml_rng else None, episode)
        if not self.h:
            raise ValueError(lib().oracle_last_error().decode())

    def __del__(self):
        try:
            lib().oracle_gym_free(self.h)
        except Exception:
            pass

    def reset(self):
        obs = np.zeros(4)
        check(lib().oracle_gym_reset(self.h, obs.ctypes.data))
        return obs

    def fields(self):
        f = np.zeros(4, dtype=np.int32)
        lib().oracle_gym_obs_fields(self.h, f.ctypes.data)
        return f

    def step(self, action):
        obs = np.zeros(4)
        r = ctypes.c_double()
        d = ctypes.c_int()
        info = np.zeros(14)
        check(lib().oracle_gym_step(self.h, int(action), obs.ctypes.data, ctypes.byref(r),
                                    ctypes.byref(d), info.ctypes.data))
        return obs, r.value, bool(d.value), dict(zip(self.INFO_KEYS, info.tolist()))

    def diag(self):
        return lib().oracle_gym_diag(self.h)


def run_episodes(config, first, n, threads=1):
    from cpr_amd import _lib as C

    rec = np.zeros(n, dtype=C.RECORD_DTYPE)
    check(lib().oracle_run_episodes(ctypes.byref(config), first, n, rec.ctypes.data, threads))
    return rec


def export_traces(config, first, n, rng=None):
    """Run episodes [first, first + n) of `config` in the oracle, logging every draw:
    returns (cpr_amd._lib.Trace, records). rng=None draws from the keyed stream; an
    OcamlRandom draws from that OCaml 4.12 Random state, carried over the episodes in
    order (the reference's own stream, as one Parany worker would)."""
    from cpr_amd import _lib as C

    rec = np.zeros(n, dtype=C.RECORD_DTYPE)
    h = lib().oracle_trace_record(ctypes.byref(config), 0 if rng is not None else 1,
                                  rng.h if rng is not None else None, first, n, rec.ctypes.data)
    if not h:
        raise RuntimeError(lib().oracle_last_error().decode())
    try:
        sz = np.zeros(3, dtype=np.int64)
        lib().oracle_trace_sizes(h, sz.ctypes.data)
        a = {
            "act_offset": np.zeros(n + 1, np.int64), "act_miner": np.zeros(sz[0], np.int32),
            "act_delay": np.zeros(sz[0], np.float64), "pow_offset": np.zeros(n + 1, np.int64),
            "pow_hash": np.zeros(sz[1], np.int32), "link_offset": np.zeros(n + 1, np.int64),
            "link_key": np.zeros(sz[2], np.uint64), "link_delay": np.zeros(sz[2], np.float64),
        }
        lib().oracle_trace_fill(h, *[a[k].ctypes.data for k, _ in C.Trace.ARRAYS])
    finally:
        lib().oracle_trace_free(h)
    return C.Trace(**a), rec


def replay(config, trace):
    """The oracle driven by a trace instead of a generator; record e = trace episode e."""
    from cpr_amd import _lib as C

    rec = np.zeros(trace.n_episodes, dtype=C.RECORD_DTYPE)
    ct = trace.ctrace()
    check(lib().oracle_trace_replay(ctypes.byref(config), ctypes.byref(ct), rec.ctypes.data))
    return rec


def node_outputs(config, n_nodes, first=0, n=0, trace=None):
    """Per-node outputs of loop tasks (the oracle side of cpr_node_outputs): (records,
    activations [n, n_nodes], rewards [n, n_nodes], head_miner [n], -2 = not reported)."""
    from cpr_amd import _lib as C

    if trace is not None:
        n = trace.n_episodes
    rec = np.zeros(n, dtype=C.RECORD_DTYPE)
    acts = np.zeros((n, n_nodes), dtype=np.int64)
    rews = np.zeros((n, n_nodes), dtype=np.float64)
    hm = np.zeros(n, dtype=np.int32)
    ct = trace.ctrace() if trace is not None else None
    check(lib().oracle_node_outputs(ctypes.byref(config), first, n,
                                    ctypes.byref(ct) if ct is not None else None, n_nodes,
                                    rec.ctypes.data, acts.ctypes.data, rews.ctypes.data,
                                    hm.ctypes.data))
    return rec, acts, rews, hm


# ---------------------------------------------------------------- OCaml Array.sort


def ocaml_sort(xs):
    a = np.ascontiguousarray(xs, dtype=np.int32).copy()
    lib().oracle_ocaml_sort_ints(a.ctypes.data, a.size)
    return a.tolist()


def ocaml_sort_pairs(keys, tags):
    k = np.ascontiguousarray(keys, dtype=np.int32).copy()
    t = np.ascontiguousarray(tags, dtype=np.int32).copy()
    lib().oracle_ocaml_sort_pairs(k.ctypes.data, t.ctypes.data, k.size)
    return list(zip(k.tolist(), t.tolist()))


def at_most_first(xs, n):
    a = np.ascontiguousarray(xs, dtype=np.int32).copy()
    m = lib().oracle_at_most_first_ints(a.ctypes.data, a.size, n)
    return a[:m].tolist()


# ---------------------------------------------------------------- Ethereum

ETH_POLICIES = {"honest": 0, "selfish_release": 1, "selfish_discard": 2, "fn19": 3,
                "fn19pkel": 4}
ETH_OBS_FIELDS = ["public_height", "public_work", "private_height", "private_work",
                  "diff_height", "diff_work", "public_orphans", "private_orphans_inclusive",
                  "private_orphans_exclusive", "event"]


class EthDag:
    """Hand-built Ethereum DAG for the validity KATs (ethereum_test.ml:44-77)."""

    def __init__(self, height, work):
        self.h = lib().oracle_eth_dag_new(height, work)
        self.root = 0

    def __del__(self):
        try:
            lib().oracle_eth_dag_free(self.h)
        except Exception:
            pass

    def mine(self, parent, uncles=()):
        u = np.ascontiguousarray(list(uncles) or [0], dtype=np.int32)
        out = ctypes.c_int32()
        ok = lib().oracle_eth_dag_mine(self.h, parent, u.ctypes.data, len(uncles),
                                       ctypes.byref(out))
        return out.value, bool(ok)


def eth_policy(policy, fields, table=None):
    """ethereum_ssz policy by name or id; policy 5 (CPR_ETH_POLICY_TABLE) reads `table`
    (dim x dim x 2 actions)."""
    o = np.ascontiguousarray(fields, dtype=np.int32)
    t = None if table is None else np.ascontiguousarray(table, dtype=np.uint8).ravel()
    dim = 0 if t is None else int(round((t.size // 2) ** 0.5))
    return lib().oracle_eth_policy(ETH_POLICIES.get(policy, policy), o.ctypes.data,
                                   None if t is None else t.ctypes.data, dim)


def eth_obs_to_floats(fields, unit):
    o = np.ascontiguousarray(fields, dtype=np.int32)
    out = np.zeros(10)
    lib().oracle_eth_obs_to_floats(o.ctypes.data, 1 if unit else 0, out.ctypes.data)
    return out


def eth_obs_of_floats(floats, unit):
    f = np.ascontiguousarray(floats, dtype=np.float64)
    out = np.zeros(10, dtype=np.int32)
    lib().oracle_eth_obs_of_floats(f.ctypes.data, 1 if unit else 0, out.ctypes.data)
    return out


class EthGymEnv:
    """The oracle's engine.ml restatement for the ethereum_ssz attack space."""

    INFO_KEYS = GymEnv.INFO_KEYS + ["head_work"]

    def __init__(self, config, episode=0, ocaml_rng=None):
        self.cfg = config
        self.h = lib().oracle_eth_gym_new(ctypes.byref(config), 0 if ocaml_rng else 1,
                                          ocaml_rng.h if ocaml_rng else None, episode)
        if not self.h:
            raise ValueError(lib().oracle_last_error().decode())

    def __del__(self):
        try:
            lib().oracle_eth_gym_free(self.h)
        except Exception:
            pass

    def reset(self):
        obs = np.zeros(10)
        check(lib().oracle_eth_gym_reset(self.h, obs.ctypes.data))
        return obs

    def fields(self):
        f = np.zeros(10, dtype=np.int32)
        lib().oracle_eth_gym_obs_fields(self.h, f.ctypes.data)
        return f

    def step(self, action):
        obs = np.zeros(10)
        r = ctypes.c_double()
        d = ctypes.c_int()
        info = np.zeros(15)
        check(lib().oracle_eth_gym_step(self.h, int(action), obs.ctypes.data, ctypes.byref(r),
                                        ctypes.byref(d), info.ctypes.data))
        return obs, r.value, bool(d.value), dict(zip(self.INFO_KEYS, info.tolist()))

    def diag(self):
        return lib().oracle_eth_gym_diag(self.h)


def eth_two_agents_task(alpha, policy, activations, scheme=1, rng=None, seed=0, episode=0):
    acts = np.zeros(2, dtype=np.int64)
    rew = np.zeros(2, dtype=np.float64)
    ht, hp = ctypes.c_double(), ctypes.c_double()
    hh, hw, dg = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_uint32()
    mode = 0 if rng is not None else 1
    check(
        lib().oracle_eth_two_agents_task(
            mode, rng.h if rng is not None else None, seed, episode, alpha, scheme,
            ETH_POLICIES.get(policy, policy), activations, acts.ctypes.data, rew.ctypes.data,
            ctypes.byref(ht), ctypes.byref(hp), ctypes.byref(hh), ctypes.byref(hw),
            ctypes.byref(dg),
        )
    )
    return dict(activations=acts.tolist(), reward=rew.tolist(), head_time=ht.value,
                head_progress=hp.value, head_height=hh.value, head_work=hw.value,
                diag=dg.value)


# ---------------------------------------------------------------- B_k

BK_POLICIES = {"honest": 0, "get-ahead": 1, "minor-delay": 2, "avoid-loss": 3}
BK_OBS_FIELDS = ["public_blocks", "private_blocks", "diff_blocks", "public_votes",
                 "private_votes_inclusive", "private_votes_exclusive", "lead", "event"]


def _bk_declare(L):
    P = ctypes.POINTER
    vp = ctypes.c_void_p
    from cpr_amd import _lib as C

    L.oracle_bk_policy.argtypes = [ctypes.c_int, vp, ctypes.c_int, vp, ctypes.c_int]
    L.oracle_bk_obs_to_floats.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
    L.oracle_bk_obs_of_floats.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
    L.oracle_bk_obs_range.argtypes = [ctypes.c_int, vp, vp]
    L.oracle_bk_gym_new.restype = vp
    L.oracle_bk_gym_new.argtypes = [P(C.Config), ctypes.c_int, vp, ctypes.c_uint64]
    L.oracle_bk_gym_free.argtypes = [vp]
    L.oracle_bk_gym_reset.argtypes = [vp, vp]
    L.oracle_bk_gym_obs_fields.argtypes = [vp, vp]
    L.oracle_bk_gym_step.argtypes = [vp, ctypes.c_int, vp, P(ctypes.c_double), P(ctypes.c_int),
                                     vp]
    L.oracle_bk_loop.argtypes = [
        ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double,
        ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
        ctypes.c_int, ctypes.c_int, vp, vp, P(ctypes.c_double), P(ctypes.c_double),
        P(ctypes.c_int32), P(ctypes.c_int32), P(ctypes.c_int64),
    ]


def bk_lib():
    L = lib()
    if not getattr(L, "_bk_declared", False):
        _bk_declare(L)
        L._bk_declared = True
    return L


def bk_policy(policy, fields, k, table=None, dim=0):
    o = np.ascontiguousarray(fields, dtype=np.int32)
    if table is not None:
        t = np.ascontiguousarray(table, dtype=np.uint8)
        return bk_lib().oracle_bk_policy(policy, o.ctypes.data, k, t.ctypes.data, dim)
    return bk_lib().oracle_bk_policy(BK_POLICIES.get(policy, policy), o.ctypes.data, k, None, 0)


def bk_obs_to_floats(fields, unit, k):
    o = np.ascontiguousarray(fields, dtype=np.int32)
    out = np.zeros(8)
    bk_lib().oracle_bk_obs_to_floats(o.ctypes.data, 1 if unit else 0, k, out.ctypes.data)
    return out


def bk_obs_of_floats(floats, unit, k):
    f = np.ascontiguousarray(floats, dtype=np.float64)
    out = np.zeros(8, dtype=np.int32)
    bk_lib().oracle_bk_obs_of_floats(f.ctypes.data, 1 if unit else 0, k, out.ctypes.data)
    return out


def bk_obs_range(unit):
    lo, hi = np.zeros(8), np.zeros(8)
    bk_lib().oracle_bk_obs_range(1 if unit else 0, lo.ctypes.data, hi.ctypes.data)
    return lo, hi


class BkGymEnv:
    """The oracle's engine.ml restatement for the bk_ssz attack space."""

    INFO_KEYS = GymEnv.INFO_KEYS + ["n_vertices"]

    def __init__(self, config, episode=0, ocaml_rng=None):
        self.cfg = config
        self.h = bk_lib().oracle_bk_gym_new(ctypes.byref(config), 0 if ocaml_rng else 1,
                                            ocaml_rng.h if ocaml_rng else None, episode)
        if not self.h:
            raise ValueError(lib().oracle_last_error().decode())

    def __del__(self):
        try:
            bk_lib().oracle_bk_gym_free(self.h)
        except Exception:
            pass

    def reset(self):
        obs = np.zeros(8)
        check(bk_lib().oracle_bk_gym_reset(self.h, obs.ctypes.data))
        return obs

    def fields(self):
        f = np.zeros(8, dtype=np.int32)
        bk_lib().oracle_bk_gym_obs_fields(self.h, f.ctypes.data)
        return f

    def step(self, action):
        obs = np.zeros(8)
        r = ctypes.c_double()
        d = ctypes.c_int()
        info = np.zeros(15)
        check(bk_lib().oracle_bk_gym_step(self.h, int(action), obs.ctypes.data, ctypes.byref(r),
                                          ctypes.byref(d), info.ctypes.data))
        return obs, r.value, bool(d.value), dict(zip(self.INFO_KEYS, info.tolist()))


def bk_loop(k, activations, *, net="clique", n_nodes=3, alpha=0.5, activation_delay=1.0,
            prop_ev=1.0, scheme=0, policy=-1, rng=None, seed=0, episode=0):
    """Simulator.loop task for B_k; policy < 0 = all nodes honest."""
    n = 2 if net == "two-agents" else n_nodes
    rew = np.zeros(n)
    acts = np.zeros(n, dtype=np.int64)
    ht, hp = ctypes.c_double(), ctypes.c_double()
    hh, hs, nv = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
    check(bk_lib().oracle_bk_loop(
        {"two-agents": 0, "clique": 1, "honest-clique": 2}[net], n, alpha, activation_delay,
        prop_ev,
        0 if rng is not None else 1, rng.h if rng is not None else None, seed, episode, k,
        scheme, BK_POLICIES.get(policy, policy), activations, rew.ctypes.data,
        acts.ctypes.data, ctypes.byref(ht), ctypes.byref(hp), ctypes.byref(hh),
        ctypes.byref(hs), ctypes.byref(nv)))
    return dict(reward=rew.tolist(), activations=acts.tolist(), head_time=ht.value,
                head_progress=hp.value, head_height=hh.value, head_signer=hs.value,
                n_vertices=nv.value)


# ---------------------------------------------------------------- Tailstorm

TS_POLICIES = {"honest": 0, "get-ahead": 1, "minor-delay": 2, "avoid-loss": 3,
               "avoid-loss-a": 4, "avoid-loss-b": 5, "long-delay": 6}
TS_SCHEMES = {"constant": 0, "discount": 1, "punish": 3, "hybrid": 4}
TS_SELECTIONS = {"altruistic": 0, "heuristic": 1, "optimal": 2}


def ts_lib():
    L = lib()
    if not getattr(L, "_ts_declared", False):
        P = ctypes.POINTER
        vp = ctypes.c_void_p
        from cpr_amd import _lib as C

        L.oracle_ts_policy.argtypes = [ctypes.c_int, vp, ctypes.c_int, vp, ctypes.c_int]
        L.oracle_ts_obs_to_floats.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
        L.oracle_ts_obs_of_floats.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
        L.oracle_n_choose_k.argtypes = [ctypes.c_int64, ctypes.c_int64]
        L.oracle_n_choose_k.restype = ctypes.c_int64
        L.oracle_ts_gym_new.restype = vp
        L.oracle_ts_gym_new.argtypes = [P(C.Config), ctypes.c_int, vp, ctypes.c_uint64]
        L.oracle_ts_gym_free.argtypes = [vp]
        L.oracle_ts_gym_reset.argtypes = [vp, vp]
        L.oracle_ts_gym_obs_fields.argtypes = [vp, vp]
        L.oracle_ts_gym_step.argtypes = [vp, ctypes.c_int, vp, P(ctypes.c_double),
                                         P(ctypes.c_int), vp]
        L.oracle_ts_loop.argtypes = [
            ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double,
            ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, P(ctypes.c_double),
            P(ctypes.c_double), P(ctypes.c_int32), P(ctypes.c_int64),
        ]
        L._ts_declared = True
    return L


def ts_policy(policy, fields, k, table=None):
    """tailstorm_ssz policy by name or id; policy 7 (CPR_TS_POLICY_TABLE) reads `table`
    (dim x dim x (k+1) x (k+1) x 3 actions)."""
    o = np.ascontiguousarray(fields, dtype=np.int32)
    t = None if table is None else np.ascontiguousarray(table, dtype=np.uint8).ravel()
    dim = 0 if t is None else int(round((t.size // (3 * (k + 1) ** 2)) ** 0.5))
    return ts_lib().oracle_ts_policy(TS_POLICIES.get(policy, policy), o.ctypes.data, k,
                                     None if t is None else t.ctypes.data, dim)


def ts_obs_to_floats(fields, unit, k):
    o = np.ascontiguousarray(fields, dtype=np.int32)
    out = np.zeros(10)
    ts_lib().oracle_ts_obs_to_floats(o.ctypes.data, 1 if unit else 0, k, out.ctypes.data)
    return out


def ts_obs_of_floats(floats, unit, k):
    f = np.ascontiguousarray(floats, dtype=np.float64)
    out = np.zeros(10, dtype=np.int32)
    ts_lib().oracle_ts_obs_of_floats(f.ctypes.data, 1 if unit else 0, k, out.ctypes.data)
    return out


def n_choose_k(n, k):
    return ts_lib().oracle_n_choose_k(n, k)


class TsGymEnv:
    """The oracle's engine.ml restatement for the tailstorm_ssz attack space."""

    INFO_KEYS = GymEnv.INFO_KEYS + ["n_vertices"]

    def __init__(self, config, episode=0, ocaml_rng=None):
        self.cfg = config
        self.h = ts_lib().oracle_ts_gym_new(ctypes.byref(config), 0 if ocaml_rng else 1,
                                            ocaml_rng.h if ocaml_rng else None, episode)
        if not self.h:
            raise ValueError(lib().oracle_last_error().decode())

    def __del__(self):
        try:
            ts_lib().oracle_ts_gym_free(self.h)
        except Exception:
            pass

    def reset(self):
        obs = np.zeros(10)
        check(ts_lib().oracle_ts_gym_reset(self.h, obs.ctypes.data))
        return obs

    def fields(self):
        f = np.zeros(10, dtype=np.int32)
        ts_lib().oracle_ts_gym_obs_fields(self.h, f.ctypes.data)
        return f

    def step(self, action):
        obs = np.zeros(10)
        r = ctypes.c_double()
        d = ctypes.c_int()
        info = np.zeros(15)
        check(ts_lib().oracle_ts_gym_step(self.h, int(action), obs.ctypes.data, ctypes.byref(r),
                                          ctypes.byref(d), info.ctypes.data))
        return obs, r.value, bool(d.value), dict(zip(self.INFO_KEYS, info.tolist()))


def ts_loop(k, activations, *, net="clique", n_nodes=3, alpha=0.5, activation_delay=1.0,
            prop_ev=1.0, scheme="discount", selection="heuristic", policy=-1, rng=None, seed=0,
            episode=0):
    n = 2 if net == "two-agents" else n_nodes
    rew = np.zeros(n)
    acts = np.zeros(n, dtype=np.int64)
    ht, hp = ctypes.c_double(), ctypes.c_double()
    hh, nv = ctypes.c_int32(), ctypes.c_int64()
    check(ts_lib().oracle_ts_loop(
        {"two-agents": 0, "clique": 1, "honest-clique": 2}[net], n, alpha, activation_delay,
        prop_ev,
        0 if rng is not None else 1, rng.h if rng is not None else None, seed, episode, k,
        TS_SCHEMES.get(scheme, scheme), TS_SELECTIONS.get(selection, selection),
        TS_POLICIES.get(policy, policy), activations, rew.ctypes.data, acts.ctypes.data,
        ctypes.byref(ht), ctypes.byref(hp), ctypes.byref(hh), ctypes.byref(nv)))
    return dict(reward=rew.tolist(), activations=acts.tolist(), head_time=ht.value,
                head_progress=hp.value, head_height=hh.value, n_vertices=nv.value)


# ---------------- FC'16 abstract model (gym/rust/src/fc16.rs), pure Python (small cases)

FC16_TAG = 0x40000000
FC16_WAIT, FC16_ADOPT, FC16_OVERRIDE, FC16_MATCH = 0, 1, 2, 3
FC16_IRRELEVANT, FC16_RELEVANT, FC16_ACTIVE = 0, 1, 2


def _thr(p):
    t = p * 4294967296.0
    return 0 if t <= 0 else (4294967296 if t >= 4294967296.0 else int(t))


def fc16_policy(policy, a, h, fork, table=None, dim=0):
    """honest / sapirshtein-2016-sm1 on (h, a) / a (a, h, fork) table of action names."""
    if policy == 0:
        return FC16_OVERRIDE if a > h else (FC16_ADOPT if h > a else FC16_WAIT)
    if policy == 1:
        if h > a:
            return FC16_ADOPT
        if h == 1 and a == 1:
            return FC16_MATCH
        if h == a - 1 and h >= 1:
            return FC16_OVERRIDE
        return FC16_WAIT
    return int(table[(min(a, dim - 1) * dim + min(h, dim - 1)) * 3 + fork])


def fc16_episode(seed, episode, alpha, gamma, horizon, policy, table=None, max_steps=1 << 30):
    """One episode of FC16SSZwPT (fc16.rs:74-190) on the keyed stream of fc16_lane.h:
    returns (reward, progress, steps, truncated). The offered actions are [Wait, Adopt,
    Override if a > h, Match if a >= h]; a named action not offered acts as Wait."""
    ta, tg, tt = _thr(alpha), _thr(gamma), _thr(1.0 / horizon)
    dim = 0 if table is None else int(round((len(table) // 3) ** 0.5))
    if int(keyed_block(seed, episode, 0, FC16_TAG | 1)[0]) < ta:
        a, h = 1, 0
    else:
        a, h = 0, 1
    fork, reward, progress, steps = FC16_IRRELEVANT, 0, 0, 0
    j = 0
    while True:
        if j >= max_steps:
            return reward, progress, steps, True
        act = fc16_policy(policy, a, h, fork, table, dim)
        if (act == FC16_OVERRIDE and not a > h) or (act == FC16_MATCH and not a >= h):
            act = FC16_WAIT
        w = keyed_block(seed, episode, j, FC16_TAG)
        mining = int(w[0]) < ta
        r = g = 0
        if act == FC16_ADOPT:  # fc16.rs:131-137
            a, h, fork, g = (1, 0, FC16_IRRELEVANT, h) if mining else (0, 1, FC16_IRRELEVANT, h)
        elif act == FC16_OVERRIDE:  # fc16.rs:116-129
            r = g = h + 1
            a, h, fork = (a - h, 0, FC16_IRRELEVANT) if mining else (a - h - 1, 1, FC16_RELEVANT)
        elif act == FC16_MATCH or fork == FC16_ACTIVE:  # fc16.rs:103-114
            if mining:
                a, fork = a + 1, FC16_ACTIVE
            elif int(w[1]) < tg:
                r = h
                a, h, fork = a - h, 1, FC16_RELEVANT
            else:
                h, fork = h + 1, FC16_RELEVANT
        else:  # fc16.rs:94-101
            if mining:
                a, fork = a + 1, FC16_IRRELEVANT
            else:
                h, fork = h + 1, FC16_RELEVANT
        reward += r
        progress += g
        steps += 1
        term = False
        for i in range(g):  # fc16.rs:178-186, one Bernoulli(1/horizon) per unit of progress
            if i % 4 == 0:
                t = keyed_block(seed, episode, j, FC16_TAG | 0x100000 | (i >> 2))
            if int(t[i % 4]) < tt:
                term = True
                break
        if term:
            return reward, progress, steps, False
        j += 1
