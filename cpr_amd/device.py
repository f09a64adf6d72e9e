"""Device contexts and episode batches over libcpr_hip.

A ``Context`` is one HIP device (one process per GPU, see ``cpr_amd.parallel``); a
``Batch`` is one configuration of the episode engine (protocol, network, attack policy,
alpha/gamma, termination) on that device. ``Batch.run`` fuses the reference's Python
reset/step/policy loop (gym/ocaml/test/test_benchmark.py:5-15, rl-eval) into one kernel
launch; ``Batch.reset``/``Batch.step`` expose the per-step gym API over many lanes.
"""

import ctypes
import math
import os
import warnings

import numpy as np

from . import _lib as L

_default_ctx = {}


class Context:
    def __init__(self, device=0):
        self.device = device
        h = ctypes.c_void_p()
        L.check(L.lib().cpr_ctx_create(device, ctypes.byref(h)))
        self.handle = h

    def close(self):
        if self.handle:
            L.lib().cpr_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def rerun_hbm_retries(self):
        """Cumulative exact re-runs whose event heap outgrew LDS (cpr_rerun_hbm_retries)."""
        v = ctypes.c_int64()
        L.check(L.lib().cpr_rerun_hbm_retries(self.handle, ctypes.byref(v)))
        return v.value

    def rerun_stats(self):
        """Cumulative (episodes, flushes, kernel ms) of exact re-runs on this context
        (cpr_rerun_stats): episodes the fused kernels handed to the exact event engine."""
        e, f, ms = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
        L.check(L.lib().cpr_rerun_stats(self.handle, ctypes.byref(e), ctypes.byref(f),
                                        ctypes.byref(ms)))
        return e.value, f.value, ms.value

    def synchronize(self):
        L.check(L.lib().cpr_synchronize(self.handle))

    def stream_fill(self, seed, episode, idx0, tag, n, with_exp=False):
        """Keyed-stream Philox blocks computed on the device."""
        out = np.zeros((n, 4), dtype=np.uint32)
        ex = np.zeros(n, dtype=np.float64) if with_exp else None
        L.check(
            L.lib().cpr_stream_fill(
                self.handle, seed, episode, idx0, tag, n, L.ptr(out), L.ptr(ex) if with_exp else None
            )
        )
        return (out, ex) if with_exp else out


def default_context():
    dev = int(os.environ.get("LOCAL_RANK", "0"))
    if dev not in _default_ctx:
        n = ctypes.c_int()
        L.check(L.lib().cpr_device_count(ctypes.byref(n)))
        if n.value == 0:
            raise RuntimeError("cpr_amd: no HIP device visible")
        _default_ctx[dev] = Context(dev % n.value)
    return _default_ctx[dev]


def make_config(
    alpha,
    gamma=0.5,
    defenders=None,
    policy=L.POLICY_SAPIRSHTEIN_2016_SM1,
    network=L.NET_SELFISH_MINING,
    mode=L.MODE_GYM,
    activation_delay=1.0,
    propagation_delay=1e-9,
    max_steps=None,
    max_progress=None,
    max_time=None,
    activations=0,
    seed=0,
    unit_observation=True,
    n_lanes=0,
    table=None,
    protocol=L.PROTO_NAKAMOTO,
    reward_scheme=L.REWARD_CONSTANT,
    k=8,
    table_dim=None,
    subblock_selection=1,
    delay_lo=math.nan,
    delay_hi=math.nan,
    horizon=100.0,
):
    """Build a cpr_config. ``defenders=None`` applies the gym's rule
    d = max(2, ceil(1 / (1 - gamma))) (gym/ocaml/cpr_gym/envs.py:70-76).
    B_k tables (protocol=PROTO_BK) hold dim*dim*(k+1)*(k+1)*3 actions
    (include/cpr_hip.h CPR_BK_POLICY_TABLE)."""
    if defenders is None and network == L.NET_SELFISH_MINING:
        if gamma >= 1:
            raise ValueError("gamma must be smaller than 1")
        defenders = max(2, int(math.ceil(1 / (1 - gamma))))
    c = L.Config()
    c.protocol = protocol
    c.reward_scheme = reward_scheme
    c.network = network
    c.mode = mode
    c.policy = policy
    c.unit_observation = 1 if unit_observation else 0
    c.alpha = alpha
    c.gamma = gamma
    c.defenders = defenders or 1
    c.activation_delay = activation_delay
    c.propagation_delay = propagation_delay
    c.max_steps = 0 if max_steps is None else int(max_steps)
    c.max_progress = 0.0 if max_progress is None else float(max_progress)
    c.max_time = 0.0 if max_time is None else float(max_time)
    c.activations = int(activations)
    c.seed = int(seed) & ((1 << 64) - 1)
    c.n_lanes = int(n_lanes)
    c.k = int(k)
    c.subblock_selection = int(subblock_selection)
    c.delay_lo = float(delay_lo)
    c.delay_hi = float(delay_hi)
    c.horizon = float(horizon)
    keep = None
    if table is not None and protocol in (L.PROTO_BK, L.PROTO_TAILSTORM):
        keep = np.ascontiguousarray(table, dtype=np.uint8).ravel()
        per = (k + 1) * (k + 1) * 3
        dim = int(round((keep.size // per) ** 0.5)) if table_dim is None else int(table_dim)
        if dim * dim * per != keep.size:
            raise ValueError("B_k / Tailstorm policy table must have dim*dim*(k+1)*(k+1)*3 "
                             "entries")
        c.policy = L.BK_POLICY_TABLE if protocol == L.PROTO_BK else L.TS_POLICY_TABLE
        c.policy_table = keep.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        c.policy_table_dim = dim
    elif table is not None and protocol == L.PROTO_FC16:
        keep = np.ascontiguousarray(table, dtype=np.uint8).ravel()
        dim = int(round((keep.size // 3) ** 0.5))
        if dim * dim * 3 != keep.size:
            raise ValueError("FC16 policy table must have dim*dim*3 entries")
        c.policy = L.FC16_POLICY_TABLE
        c.policy_table = keep.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        c.policy_table_dim = dim
    elif table is not None and protocol == L.PROTO_ETHEREUM:
        keep = np.ascontiguousarray(table, dtype=np.uint8).ravel()
        dim = int(round((keep.size // 2) ** 0.5))
        if dim * dim * 2 != keep.size:
            raise ValueError("Ethereum policy table must have dim*dim*2 entries")
        c.policy = L.ETH_POLICY_TABLE
        c.policy_table = keep.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        c.policy_table_dim = dim
    elif table is not None:
        keep = np.ascontiguousarray(table, dtype=np.uint8)
        dim = int(round((keep.size // 2) ** 0.5))
        if dim * dim * 2 != keep.size:
            raise ValueError("policy table must have dim*dim*2 entries")
        c.policy = L.POLICY_TABLE
        c.policy_table = keep.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        c.policy_table_dim = dim
    return c, keep


class Batch:
    def __init__(self, config, ctx=None, keep=None):
        self.ctx = ctx or default_context()
        self.config = config
        self._keep = keep
        h = ctypes.c_void_p()
        L.check(L.lib().cpr_batch_create(self.ctx.handle, ctypes.byref(config), ctypes.byref(h)))
        self.handle = h
        self.n_lanes = int(config.n_lanes)
        self.obs_len = self.observation_spec()[0]
        self._coverage_warned = False

    def close(self):
        if self.handle:
            L.lib().cpr_batch_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- fused episodes
    def run(self, n_episodes, first_episode=0, records=False, summary=None):
        s = summary if summary is not None else L.Summary()
        rec = np.zeros(n_episodes, dtype=L.RECORD_DTYPE) if records else None
        L.check(
            L.lib().cpr_run_episodes(
                self.handle, n_episodes, first_episode, ctypes.byref(s), L.ptr(rec), 0
            )
        )
        return (s, rec) if records else s

    def replay(self, trace, records=True, summary=None):
        """Replay an exported activation/delay trace (cpr_replay): record e is trace
        episode e, run with this batch's protocol, mode and policy."""
        s = summary if summary is not None else L.Summary()
        rec = np.zeros(trace.n_episodes, dtype=L.RECORD_DTYPE) if records else None
        ct = trace.ctrace()
        L.check(L.lib().cpr_replay(self.handle, ctypes.byref(ct), ctypes.byref(s), L.ptr(rec), 0))
        return (s, rec) if records else s

    @property
    def n_nodes(self):
        """Nodes of the batch's network: 2, defenders + 1 (attacker first) or the clique."""
        c = self.config
        if c.network == L.NET_TWO_AGENTS:
            return 2
        return int(c.defenders) if c.network == L.NET_HONEST_CLIQUE else int(c.defenders) + 1

    def node_outputs(self, n_episodes=0, first_episode=0, trace=None):
        """Per-node outputs (cpr_node_outputs): (records, activations [n, n_nodes] int64,
        rewards [n, n_nodes] f64) of keyed episodes [first, first + n) or of a trace; the
        `activations` / `reward` columns of a csv_runner.ml row."""
        if trace is not None:
            n_episodes = trace.n_episodes
        nn = self.n_nodes
        rec = np.zeros(n_episodes, dtype=L.RECORD_DTYPE)
        acts = np.zeros((n_episodes, nn), dtype=np.int64)
        rews = np.zeros((n_episodes, nn), dtype=np.float64)
        ct = trace.ctrace() if trace is not None else None
        L.check(L.lib().cpr_node_outputs(
            self.handle, n_episodes, first_episode, ctypes.byref(ct) if ct is not None else None,
            nn, L.ptr(rec), L.ptr(acts), L.ptr(rews)))
        return rec, acts, rews

    def last_launch(self):
        """(kernel_ms, activations) of the last fused-episode launch (HIP events)."""
        ms = ctypes.c_double()
        acts = ctypes.c_int64()
        L.check(L.lib().cpr_last_launch(self.handle, ctypes.byref(ms), ctypes.byref(acts)))
        return ms.value, acts.value

    def launch_shape(self):
        """(lanes, resident lanes) of the last episode-kernel launch (cpr_launch_shape)."""
        lanes = ctypes.c_int64()
        res = ctypes.c_int64()
        L.check(L.lib().cpr_launch_shape(self.handle, ctypes.byref(lanes), ctypes.byref(res)))
        return lanes.value, res.value

    def run_async(self, n_episodes, first_episode, summary_dev_ptr, records_dev_ptr=None):
        L.check(
            L.lib().cpr_run_episodes_async(
                self.handle, n_episodes, first_episode, summary_dev_ptr, records_dev_ptr
            )
        )

    # ---- lockstep gym lanes
    def reset(self, mask=None, episode_ids=None):
        obs = np.zeros((self.n_lanes, self.obs_len), dtype=np.float64)
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        e = None if episode_ids is None else np.ascontiguousarray(episode_ids, dtype=np.uint64)
        L.check(L.lib().cpr_reset(self.handle, L.ptr(m), L.ptr(e), L.ptr(obs)))
        log_steps, _ = self.lockstep_coverage()
        ms = int(self.config.max_steps)
        if log_steps and 0 < ms < 2**30 and log_steps < ms and not self._coverage_warned:
            self._coverage_warned = True
            warnings.warn(f"{self.n_lanes} lockstep lanes x {ms}-step episodes exceed the "
                          f"action-log budget: lanes leaving the closed form after step "
                          f"{log_steps} keep its flags instead of an exact re-run",
                          RuntimeWarning, stacklevel=2)
        return obs

    def lockstep_coverage(self):
        """(action-log steps, exact-engine slots) of the lockstep lanes
        (cpr_lockstep_coverage); (0, 0) before the first reset or without exact lanes."""
        s, k = ctypes.c_int64(), ctypes.c_int64()
        L.check(L.lib().cpr_lockstep_coverage(self.handle, ctypes.byref(s), ctypes.byref(k)))
        return s.value, k.value

    def step(self, actions, with_info=True):
        n = self.n_lanes
        a = np.ascontiguousarray(actions, dtype=np.int32)
        obs = np.zeros((n, self.obs_len), dtype=np.float64)
        rew = np.zeros(n, dtype=np.float64)
        done = np.zeros(n, dtype=np.uint8)
        info = None
        si = None
        if with_info:
            info = {
                "episode_reward_attacker": np.zeros(n),
                "episode_reward_defender": np.zeros(n),
                "episode_progress": np.zeros(n),
                "episode_chain_time": np.zeros(n),
                "episode_sim_time": np.zeros(n),
                "episode_n_steps": np.zeros(n, dtype=np.int64),
                "episode_n_activations": np.zeros(n, dtype=np.int64),
                "head_height": np.zeros(n, dtype=np.int32),
                "head_miner": np.zeros(n, dtype=np.int32),
                "status": np.zeros(n, dtype=np.uint32),
            }
            si = L.StepInfo()
            for k, v in info.items():
                ct = np.ctypeslib.as_ctypes_type(v.dtype)
                setattr(si, k, v.ctypes.data_as(ctypes.POINTER(ct)))
        L.check(
            L.lib().cpr_step(
                self.handle, L.ptr(a), L.ptr(obs), L.ptr(rew), L.ptr(done),
                ctypes.byref(si) if si is not None else None,
            )
        )
        return obs, rew, done.astype(bool), info

    def observe_fields(self):
        f = np.zeros((self.n_lanes, self.obs_len), dtype=np.int32)
        L.check(L.lib().cpr_observe_fields(self.handle, L.ptr(f)))
        return f

    def policy_actions(self, policy, obs):
        o = np.ascontiguousarray(np.atleast_2d(obs), dtype=np.float64)
        if o.shape[1] != self.obs_len:
            raise ValueError("invalid dimensions")
        out = np.zeros(o.shape[0], dtype=np.int32)
        L.check(L.lib().cpr_policy_actions(self.handle, policy, L.ptr(o), o.shape[0], L.ptr(out)))
        return out

    def rollout(self, n_steps, outputs=False, summary=None, device_outputs=None):
        """Device rollout (cpr_rollout): every lane takes n_steps steps with the batch
        policy, auto-resetting finished episodes. ``outputs=True`` returns host arrays
        obs [n_steps, n_lanes, obs_len], reward [n_steps, n_lanes], done [n_steps, n_lanes];
        ``device_outputs=(obs_ptr, reward_ptr, done_ptr)`` writes to caller-owned device
        memory instead. Returns the summary (and the arrays if requested)."""
        s = summary if summary is not None else L.Summary()
        n = self.n_lanes
        if device_outputs is not None:
            o, r, d = (None if x is None else ctypes.c_void_p(int(x)) for x in device_outputs)
            L.check(L.lib().cpr_rollout(self.handle, int(n_steps), o, r, d, 1, ctypes.byref(s)))
            return s
        if not outputs:
            L.check(L.lib().cpr_rollout(self.handle, int(n_steps), None, None, None, 0,
                                        ctypes.byref(s)))
            return s
        obs = np.zeros((n_steps, n, self.obs_len))
        rew = np.zeros((n_steps, n))
        done = np.zeros((n_steps, n), dtype=np.uint8)
        L.check(L.lib().cpr_rollout(self.handle, int(n_steps), L.ptr(obs), L.ptr(rew),
                                    L.ptr(done), 0, ctypes.byref(s)))
        return s, obs, rew, done.astype(bool)

    def observation_spec(self):
        ol = ctypes.c_int32()
        na = ctypes.c_int32()
        low = np.zeros(16)
        high = np.zeros(16)
        L.check(
            L.lib().cpr_observation_spec(
                self.handle, ctypes.byref(ol), ctypes.byref(na), L.ptr(low), L.ptr(high)
            )
        )
        return ol.value, na.value, low[: ol.value], high[: ol.value]


def policy_registry(protocol=L.PROTO_NAKAMOTO):
    """[(name, id)] in the reference's registry order (nakamoto_ssz.ml:342-350)."""
    out = []
    for i in range(L.lib().cpr_policy_count(protocol)):
        pid = ctypes.c_int32()
        name = L.lib().cpr_policy_name(protocol, i, ctypes.byref(pid))
        out.append((name.decode(), pid.value))
    return out
