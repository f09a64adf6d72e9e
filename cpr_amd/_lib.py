"""ctypes binding of libcpr_hip (include/cpr_hip.h).

The shared object is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950). There
is no fallback: if the library is missing or no HIP device is present, the product path
raises instead of silently computing anything on the CPU.
"""

import ctypes
import os
import pathlib

import numpy as np

LIB_PATH = pathlib.Path(__file__).resolve().parent / "libcpr_hip.so"

# enums (include/cpr_hip.h)
CPR_OK = 0
CPR_E_INVALID_ARG = -1
CPR_E_UNSUPPORTED = -2
CPR_E_HIP = -3
CPR_E_CAPACITY = -4
CPR_E_STATE = -5

PROTO_NAKAMOTO = 0
PROTO_ETHEREUM = 1
PROTO_BK = 2
PROTO_TAILSTORM = 3
REWARD_PUNISH = 3
REWARD_HYBRID = 4
SELECT_ALTRUISTIC = 0
SELECT_HEURISTIC = 1
SELECT_OPTIMAL = 2
TS_POLICY_HONEST = 0
TS_POLICY_TABLE = 7  # include/cpr_hip.h, the B_k table layout
TS_POLICY_GET_AHEAD = 1
TS_POLICY_MINOR_DELAY = 2
TS_POLICY_AVOID_LOSS = 3
TS_POLICY_AVOID_LOSS_A = 4
TS_POLICY_AVOID_LOSS_B = 5
TS_POLICY_LONG_DELAY = 6
TS_POLICY_RANDOM = 8  # loop tasks: keyed random Action8 (cpr_protocols.ml:658-782)
REWARD_CONSTANT = 0
REWARD_DISCOUNT = 1
REWARD_BLOCK = 2
BK_POLICY_HONEST = 0
BK_POLICY_GET_AHEAD = 1
BK_POLICY_MINOR_DELAY = 2
BK_POLICY_AVOID_LOSS = 3
BK_POLICY_TABLE = 4
BK_POLICY_RANDOM = 5
ETH_POLICY_HONEST = 0
ETH_POLICY_TABLE = 5  # include/cpr_hip.h: [(pub_h, priv_h) clamped to D][event]
ETH_POLICY_SELFISH_RELEASE = 1
ETH_POLICY_SELFISH_DISCARD = 2
ETH_POLICY_FN19 = 3
ETH_POLICY_FN19PKEL = 4
ETH_POLICY_RANDOM = 6
NET_SELFISH_MINING = 0
NET_TWO_AGENTS = 1
NET_HONEST_CLIQUE = 2
NET_EXP_CLIQUE = 3  # include/cpr_hip.h: attacker + `defenders`, exponential link delays
NET_ABSTRACT_GAMMA = 4  # FLAGGED abstract-gamma mode (include/cpr_hip.h), gamma in [0, 1]
MODE_GYM = 0
MODE_LOOP = 1

POLICY_HONEST = 0
POLICY_SIMPLE = 1
POLICY_EYAL_SIRER_2014 = 2
POLICY_SAPIRSHTEIN_2016_SM1 = 3
POLICY_TABLE = 4
POLICY_RANDOM = 5  # loop tasks on the event engine (cpr_protocols.ml:658-782)

PROTO_FC16 = 4  # gym/rust/src/fc16.rs abstract model (fused episodes)
FC16_POLICY_HONEST = 0
FC16_POLICY_SM1 = 1
FC16_POLICY_TABLE = 2
FC16_WAIT, FC16_ADOPT, FC16_OVERRIDE, FC16_MATCH = 0, 1, 2, 3
ST_TIE = 1
ST_OVERLAP = 2
ST_DEEP_FORK = 4
ST_TIE_UNRESOLVED = 8
ST_STALE_TIME = 16
ST_CAPACITY = 32
ST_REFERENCE_RAISES = 64
ST_TRACE_MISS = 128
ST_EXACT_RERUN = 256
ST_INVALID = ST_CAPACITY | ST_REFERENCE_RAISES | ST_TRACE_MISS  # include/cpr_hip.h
ST_LOCKSTEP_INEXACT = ST_OVERLAP | ST_DEEP_FORK | ST_TIE_UNRESOLVED | ST_STALE_TIME
ABI_VERSION = 11  # include/cpr_hip.h CPR_ABI_VERSION this module's structures follow

HIST_BINS = 64


class Config(ctypes.Structure):
    _fields_ = [
        ("protocol", ctypes.c_int32),
        ("network", ctypes.c_int32),
        ("mode", ctypes.c_int32),
        ("policy", ctypes.c_int32),
        ("policy_table", ctypes.POINTER(ctypes.c_uint8)),
        ("policy_table_dim", ctypes.c_int32),
        ("unit_observation", ctypes.c_int32),
        ("alpha", ctypes.c_double),
        ("gamma", ctypes.c_double),
        ("defenders", ctypes.c_int32),
        ("reward_scheme", ctypes.c_int32),
        ("activation_delay", ctypes.c_double),
        ("propagation_delay", ctypes.c_double),
        ("max_steps", ctypes.c_int64),
        ("max_progress", ctypes.c_double),
        ("max_time", ctypes.c_double),
        ("activations", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("n_lanes", ctypes.c_int64),
        ("k", ctypes.c_int32),
        ("subblock_selection", ctypes.c_int32),
        ("delay_lo", ctypes.c_double),
        ("delay_hi", ctypes.c_double),
        ("horizon", ctypes.c_double),
    ]


class EpisodeRecord(ctypes.Structure):
    _fields_ = [
        ("reward_attacker", ctypes.c_double),
        ("reward_defender", ctypes.c_double),
        ("progress", ctypes.c_double),
        ("chain_time", ctypes.c_double),
        ("sim_time", ctypes.c_double),
        ("n_steps", ctypes.c_int64),
        ("n_activations", ctypes.c_int64),
        ("head_height", ctypes.c_int32),
        ("head_miner", ctypes.c_int32),
        ("status", ctypes.c_uint32),
        ("head_work", ctypes.c_int32),
    ]


RECORD_DTYPE = np.dtype(
    [
        ("reward_attacker", "<f8"),
        ("reward_defender", "<f8"),
        ("progress", "<f8"),
        ("chain_time", "<f8"),
        ("sim_time", "<f8"),
        ("n_steps", "<i8"),
        ("n_activations", "<i8"),
        ("head_height", "<i4"),
        ("head_miner", "<i4"),
        ("status", "<u4"),
        ("head_work", "<i4"),
    ]
)
assert RECORD_DTYPE.itemsize == ctypes.sizeof(EpisodeRecord)


class Summary(ctypes.Structure):
    _fields_ = [
        ("episodes", ctypes.c_int64),
        ("steps", ctypes.c_int64),
        ("activations", ctypes.c_int64),
        ("reward_attacker_fx", ctypes.c_int64),
        ("reward_defender_fx", ctypes.c_int64),
        ("progress_fx", ctypes.c_int64),
        ("rel_revenue_fx", ctypes.c_uint64),
        ("rel_revenue_sq_fx", ctypes.c_uint64),
        ("orphans", ctypes.c_int64),
        ("status_tie", ctypes.c_int64),
        ("status_overlap", ctypes.c_int64),
        ("status_other", ctypes.c_int64),
        ("hist", ctypes.c_int64 * HIST_BINS),
        ("invalid", ctypes.c_int64),
    ]

    FIELDS = [f for f, _ in _fields_ if f != "hist"]

    def to_array(self):
        """int64 vector (fields then histogram) — the RCCL all-reduce payload."""
        head = [getattr(self, f) for f in self.FIELDS]
        head = [x - (1 << 64) if x >= (1 << 63) else x for x in head]
        return np.array(head + list(self.hist), dtype=np.int64)

    @classmethod
    def from_array(cls, a):
        s = cls()
        for i, f in enumerate(cls.FIELDS):
            v = int(a[i])
            if f.startswith("rel_") and v < 0:
                v += 1 << 64
            setattr(s, f, v)
        for i in range(HIST_BINS):
            s.hist[i] = int(a[len(cls.FIELDS) + i])
        return s

    def as_dict(self):
        d = {f: int(getattr(self, f)) for f in self.FIELDS}
        d["hist"] = [int(x) for x in self.hist]
        n = max(1, d["episodes"])
        d["mean_rel_revenue"] = d["rel_revenue_fx"] / 2**32 / n
        d["mean_reward_attacker"] = d["reward_attacker_fx"] / 2**20 / n
        d["mean_progress"] = d["progress_fx"] / 2**20 / n
        return d


class StepInfo(ctypes.Structure):
    _fields_ = [
        ("episode_reward_attacker", ctypes.POINTER(ctypes.c_double)),
        ("episode_reward_defender", ctypes.POINTER(ctypes.c_double)),
        ("episode_progress", ctypes.POINTER(ctypes.c_double)),
        ("episode_chain_time", ctypes.POINTER(ctypes.c_double)),
        ("episode_sim_time", ctypes.POINTER(ctypes.c_double)),
        ("episode_n_steps", ctypes.POINTER(ctypes.c_int64)),
        ("episode_n_activations", ctypes.POINTER(ctypes.c_int64)),
        ("head_height", ctypes.POINTER(ctypes.c_int32)),
        ("head_miner", ctypes.POINTER(ctypes.c_int32)),
        ("status", ctypes.POINTER(ctypes.c_uint32)),
    ]


class CTrace(ctypes.Structure):
    _fields_ = [
        ("n_episodes", ctypes.c_int64),
        ("act_offset", ctypes.c_void_p),
        ("act_miner", ctypes.c_void_p),
        ("act_delay", ctypes.c_void_p),
        ("pow_offset", ctypes.c_void_p),
        ("pow_hash", ctypes.c_void_p),
        ("link_offset", ctypes.c_void_p),
        ("link_key", ctypes.c_void_p),
        ("link_delay", ctypes.c_void_p),
    ]


class Trace:
    """An exported activation/delay trace (cpr_trace, include/cpr_hip.h): CSR numpy arrays
    over episodes. ``ctrace()`` gives the C struct (the arrays must outlive it)."""

    ARRAYS = [
        ("act_offset", np.int64), ("act_miner", np.int32), ("act_delay", np.float64),
        ("pow_offset", np.int64), ("pow_hash", np.int32),
        ("link_offset", np.int64), ("link_key", np.uint64), ("link_delay", np.float64),
    ]

    def __init__(self, **arrays):
        for name, dt in self.ARRAYS:
            setattr(self, name, np.ascontiguousarray(arrays[name], dtype=dt))
        self.n_episodes = len(self.act_offset) - 1

    def episode(self, e):
        """Trace of episode e alone."""
        a0, a1 = self.act_offset[e], self.act_offset[e + 1]
        p0, p1 = self.pow_offset[e], self.pow_offset[e + 1]
        l0, l1 = self.link_offset[e], self.link_offset[e + 1]
        return Trace(act_offset=[0, a1 - a0], act_miner=self.act_miner[a0:a1],
                     act_delay=self.act_delay[a0:a1], pow_offset=[0, p1 - p0],
                     pow_hash=self.pow_hash[p0:p1], link_offset=[0, l1 - l0],
                     link_key=self.link_key[l0:l1], link_delay=self.link_delay[l0:l1])

    def save(self, path):
        np.savez_compressed(path, **{n: getattr(self, n) for n, _ in self.ARRAYS})

    # binary layout written by the OCaml recorder (integration/ocaml/trace_hooks.ml
    # `write`): magic, u32 version, u32 n_episodes, then per array of ARRAYS: u64 count and
    # that many little-endian elements (act_miner / pow_hash as 32-bit ints)
    MAGIC = b"CPRTRACE"
    _WIRE = {"act_offset": "<i8", "act_miner": "<i4", "act_delay": "<f8", "pow_offset": "<i8",
             "pow_hash": "<i4", "link_offset": "<i8", "link_key": "<u8", "link_delay": "<f8"}

    def save_binary(self, path):
        """The OCaml recorder's format (a Python mirror of trace_hooks.ml `write`)."""
        with open(path, "wb") as f:
            f.write(self.MAGIC)
            f.write(np.array([1, self.n_episodes], dtype="<u4").tobytes())
            for name, _ in self.ARRAYS:
                a = np.ascontiguousarray(getattr(self, name), dtype=self._WIRE[name])
                f.write(np.array([len(a)], dtype="<u8").tobytes())
                f.write(a.tobytes())

    @classmethod
    def load(cls, path):
        """An .npz (Trace.save, the oracle's exporter) or the OCaml recorder's binary file."""
        with open(path, "rb") as f:
            head = f.read(len(cls.MAGIC))
        if head != cls.MAGIC:
            with np.load(path, allow_pickle=False) as z:
                return cls(**{n: z[n] for n, _ in cls.ARRAYS})
        raw = open(path, "rb").read()
        ver, n_ep = np.frombuffer(raw, dtype="<u4", count=2, offset=8)
        if ver != 1:
            raise ValueError(f"{path}: trace format version {ver}, expected 1")
        o, arrays = 16, {}
        for name, _ in cls.ARRAYS:
            (cnt,) = np.frombuffer(raw, dtype="<u8", count=1, offset=o)
            o += 8
            dt = np.dtype(cls._WIRE[name])
            arrays[name] = np.frombuffer(raw, dtype=dt, count=int(cnt), offset=o).copy()
            o += int(cnt) * dt.itemsize
        if o != len(raw) or len(arrays["act_offset"]) != n_ep + 1:
            raise ValueError(f"{path}: malformed trace file")
        return cls(**arrays)

    def ctrace(self):
        t = CTrace()
        t.n_episodes = self.n_episodes
        for name, _ in self.ARRAYS:
            setattr(t, name, self.__dict__[name].ctypes.data)
        return t


# every symbol include/cpr_hip.h declares
EXPORTS = [
    "cpr_version",
    "cpr_abi_version",
    "cpr_last_error",
    "cpr_ctx_create",
    "cpr_ctx_destroy",
    "cpr_device_count",
    "cpr_batch_create",
    "cpr_batch_destroy",
    "cpr_run_episodes",
    "cpr_run_episodes_async",
    "cpr_synchronize",
    "cpr_replay",
    "cpr_node_outputs",
    "cpr_last_launch",
    "cpr_launch_shape",
    "cpr_rerun_hbm_retries",
    "cpr_rerun_stats",
    "cpr_lockstep_coverage",
    "cpr_reset",
    "cpr_step",
    "cpr_observe_fields",
    "cpr_rollout",
    "cpr_policy_actions",
    "cpr_observation_spec",
    "cpr_policy_count",
    "cpr_policy_name",
    "cpr_stream_fill",
]


class CprError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


_lib = None


def _declare(L):
    P = ctypes.POINTER
    vp = ctypes.c_void_p
    L.cpr_version.restype = ctypes.c_char_p
    L.cpr_abi_version.restype = ctypes.c_int
    L.cpr_last_error.restype = ctypes.c_char_p
    L.cpr_ctx_create.argtypes = [ctypes.c_int, P(vp)]
    L.cpr_ctx_destroy.argtypes = [vp]
    L.cpr_device_count.argtypes = [P(ctypes.c_int)]
    L.cpr_batch_create.argtypes = [vp, P(Config), P(vp)]
    L.cpr_batch_destroy.argtypes = [vp]
    L.cpr_run_episodes.argtypes = [vp, ctypes.c_int64, ctypes.c_uint64, P(Summary), vp, ctypes.c_int]
    L.cpr_run_episodes_async.argtypes = [vp, ctypes.c_int64, ctypes.c_uint64, vp, vp]
    L.cpr_synchronize.argtypes = [vp]
    L.cpr_replay.argtypes = [vp, P(CTrace), P(Summary), vp, ctypes.c_int]
    L.cpr_node_outputs.argtypes = [vp, ctypes.c_int64, ctypes.c_uint64, vp, ctypes.c_int32, vp,
                                   vp, vp]
    L.cpr_last_launch.argtypes = [vp, P(ctypes.c_double), P(ctypes.c_int64)]
    L.cpr_launch_shape.argtypes = [vp, P(ctypes.c_int64), P(ctypes.c_int64)]
    L.cpr_rerun_hbm_retries.argtypes = [vp, P(ctypes.c_int64)]
    L.cpr_rerun_stats.argtypes = [vp, P(ctypes.c_int64), P(ctypes.c_int64), P(ctypes.c_double)]
    L.cpr_lockstep_coverage.argtypes = [vp, P(ctypes.c_int64), P(ctypes.c_int64)]
    L.cpr_reset.argtypes = [vp, vp, vp, vp]
    L.cpr_step.argtypes = [vp, vp, vp, vp, vp, P(StepInfo)]
    L.cpr_observe_fields.argtypes = [vp, vp]
    L.cpr_rollout.argtypes = [vp, ctypes.c_int64, vp, vp, vp, ctypes.c_int, P(Summary)]
    L.cpr_policy_actions.argtypes = [vp, ctypes.c_int32, vp, ctypes.c_int64, vp]
    L.cpr_observation_spec.argtypes = [vp, P(ctypes.c_int32), P(ctypes.c_int32), vp, vp]
    L.cpr_policy_count.argtypes = [ctypes.c_int32]
    L.cpr_policy_name.restype = ctypes.c_char_p
    L.cpr_policy_name.argtypes = [ctypes.c_int32, ctypes.c_int32, P(ctypes.c_int32)]
    L.cpr_stream_fill.argtypes = [
        vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int64, vp, vp
    ]


def lib():
    """Load libcpr_hip.so (no fallback: raises if it is missing)."""
    global _lib
    if _lib is None:
        path = os.environ.get("CPR_HIP_LIB", str(LIB_PATH))
        if not os.path.exists(path):
            raise ImportError(
                f"libcpr_hip.so not found at {path}; run __graft_entry__.build() (hipcc, gfx950)"
            )
        L = ctypes.CDLL(path)
        _declare(L)
        if L.cpr_abi_version() != ABI_VERSION:
            raise ImportError(f"{path} has ABI {L.cpr_abi_version()}, this module expects "
                              f"{ABI_VERSION}; rebuild with __graft_entry__.build()")
        _lib = L
    return _lib


def check(rc):
    if rc != CPR_OK:
        raise CprError(rc, lib().cpr_last_error().decode())
    return rc


def ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None
