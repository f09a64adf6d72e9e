"""Drop-in for the reference's Python module ``engine`` (simulator/gym/cpr_gym_engine.ml:
310-436): create / reset / step / policies / to_string / n_actions / observation_low /
observation_high over one device lane each. The episode state lives on the GPU; every
step is one launch of the lane state machine (cpr_amd/csrc/*_lane.h).

Randomness: the reference seeds OCaml's Random with ``self_init`` at import
(cpr_gym_engine.ml:39), so it is not reproducible. Here each ``create`` draws a fresh
64-bit seed from ``os.urandom`` unless ``seed=`` is passed (or CPR_SEED is set).
"""

import math
import os
import sys

import numpy as np

from . import __version__
from . import _lib as L
from . import device

cpr_lib_version = f"cpr_amd-{__version__}"

MAX_INT = (1 << 62) - 1  # OCaml max_int on 64-bit

_ACTIONS = ["Adopt", "Override", "Match", "Wait"]  # nakamoto_ssz.ml:116-154
_EVENTS = ["`ProofOfWork", "`Network"]  # ssz_tools.ml:76-80

# per attack space: action names (Variants.to_name, rank order), observation record fields,
# event values (ssz_tools.ml event_to_string)
_ACTION8 = ["Adopt_Prolong", "Override_Prolong", "Match_Prolong", "Wait_Prolong",
            "Adopt_Proceed", "Override_Proceed", "Match_Proceed", "Wait_Proceed"]  # ssz_tools.ml:230-263
_SPACES = {
    L.PROTO_NAKAMOTO: dict(actions=_ACTIONS, events=_EVENTS,
                           fields=["public_blocks", "private_blocks", "diff_blocks", "event"],
                           bools=()),
    L.PROTO_BK: dict(actions=_ACTION8, events=["`Append", "`ProofOfWork", "`Network"],
                     fields=["public_blocks", "private_blocks", "diff_blocks", "public_votes",
                             "private_votes_inclusive", "private_votes_exclusive", "lead",
                             "event"],
                     bools=("lead",)),  # bk_ssz.ml:22-34,123-143
    # ethereum_ssz.ml:21-41,161-263: action i = (action_list[i / 4], uncles_list[i % 4])
    L.PROTO_ETHEREUM: dict(
        actions=[f"{a}, uncles {{own: {o}; foreign: {f}}}"
                 for a in ["Adopt_discard", "Adopt_release", "Override", "Match", "Release1",
                           "Wait"]
                 for o in ("false", "true") for f in ("false", "true")],
        events=_EVENTS,
        fields=["public_height", "public_work", "private_height", "private_work",
                "diff_height", "diff_work", "public_orphans", "private_orphans_inclusive",
                "private_orphans_exclusive", "event"],
        bools=()),
    L.PROTO_TAILSTORM: dict(actions=_ACTION8, events=["`Append", "`ProofOfWork", "`Network"],
                            fields=["public_blocks", "private_blocks", "diff_blocks",
                                    "public_votes", "private_votes_inclusive",
                                    "private_votes_exclusive", "public_depth",
                                    "private_depth_inclusive", "private_depth_exclusive",
                                    "event"],
                            bools=()),  # tailstorm_ssz.ml:22-38,136-157
}


class InstantiatedEnv:
    """Stands in for the reference's "ocaml.instantiated_env" capsule."""

    def __init__(self, proto, params, batch, seed):
        self.proto = proto
        self.params = params
        self.batch = batch
        self.seed = seed
        self.episode = 0
        self._last = None


def _params(alpha, gamma, defenders, activation_delay, max_steps, max_progress, max_time):
    # engine.ml:37-51, messages verbatim
    if math.isnan(activation_delay):
        raise RuntimeError("activation_delay cannot be NaN")
    if math.isnan(alpha):
        raise RuntimeError("alpha cannot be NaN")
    if math.isnan(gamma):
        raise RuntimeError("gamma cannot be NaN")
    if alpha < 0.0 or alpha > 1.0:
        raise RuntimeError("alpha < 0 || alpha > 1")
    if gamma < 0.0 or gamma > 1.0:
        raise RuntimeError("gamma < 0 || gamma > 1")
    if defenders < 1:
        raise RuntimeError("defenders < 0")
    if activation_delay <= 0.0:
        raise RuntimeError("activation_delay <= 0")
    if max_steps <= 0:
        raise RuntimeError("max_steps <= 0")
    if max_progress <= 0.0:
        raise RuntimeError("max_progress <= 0")
    if max_time <= 0.0:
        raise RuntimeError("max_time <= 0")
    return dict(
        alpha=alpha,
        gamma=gamma,
        defenders=defenders,
        activation_delay=activation_delay,
        max_steps=max_steps,
        max_progress=max_progress,
        max_time=max_time,
    )


def create(
    proto,
    alpha,
    gamma,
    defenders,
    activation_delay,
    max_steps=MAX_INT,
    max_progress=math.inf,
    max_time=math.inf,
    seed=None,
):
    p = _params(float(alpha), float(gamma), int(defenders), float(activation_delay),
                int(max_steps), float(max_progress), float(max_time))
    if seed is None:
        seed = int(os.environ["CPR_SEED"]) if "CPR_SEED" in os.environ else \
            int.from_bytes(os.urandom(8), "little")
    cfg, keep = device.make_config(
        protocol=proto.protocol_id,
        k=proto.params.get("k", 8),
        subblock_selection=proto.params.get("selection_id", 1),
        reward_scheme=proto.params.get("reward_scheme", L.REWARD_CONSTANT),
        alpha=p["alpha"],
        gamma=p["gamma"],
        defenders=p["defenders"],
        policy=L.POLICY_HONEST,
        activation_delay=p["activation_delay"],
        max_steps=p["max_steps"],
        max_progress=None if math.isinf(p["max_progress"]) else p["max_progress"],
        max_time=None if math.isinf(p["max_time"]) else p["max_time"],
        seed=seed,
        unit_observation=proto.unit_observation,
        n_lanes=1,
    )
    try:
        batch = device.Batch(cfg, keep=keep)
    except L.CprError as e:
        if e.code == L.CPR_E_INVALID_ARG:
            raise ValueError(str(e)) from None  # network.ml Invalid_argument
        raise
    return InstantiatedEnv(proto, p, batch, seed)


def reset(ienv):
    ienv._last = None
    obs = ienv.batch.reset(episode_ids=np.array([ienv.episode], dtype=np.uint64))
    ienv.episode += 1
    return obs[0].copy()


def _miner_str(m):
    return "n/a" if m < 0 else str(m)


def _space(ienv):
    return _SPACES[ienv.proto.protocol_id]


def step(ienv, action):
    a = int(action)
    if a < 0 or a >= len(_space(ienv)["actions"]):
        raise IndexError("index out of bounds")  # Action.of_int on table (nakamoto_ssz.ml:152)
    obs, rew, done, inf = ienv.batch.step(np.array([a], dtype=np.int32))
    status = int(inf["status"][0])
    if status & L.ST_REFERENCE_RAISES:
        # tailstorm.ml: List.for_all2 in summary dedup (simulator.ml:139-159),
        # Division_by_zero in n_choose_k, assert false in heuristic_quorum
        raise RuntimeError("the reference simulator raises an exception at this step "
                           "(CPR_ST_REFERENCE_RAISES); the episode has no valid outcome")
    if status & L.ST_CAPACITY:
        raise RuntimeError("device lane capacity exceeded (CPR_ST_CAPACITY); the episode's "
                           "outputs are not valid")
    ra = float(inf["episode_reward_attacker"][0])
    rd = float(inf["episode_reward_defender"][0])
    prog = float(inf["episode_progress"][0])
    ct = float(inf["episode_chain_time"][0])
    st = float(inf["episode_sim_time"][0])
    last = ienv._last or (0.0, 0.0, 0.0, 0.0, 0.0)
    # engine.ml:224-241 (key order kept)
    info = {
        "step_reward_attacker": ra - last[0],
        "step_reward_defender": rd - last[1],
        "step_progress": prog - last[2],
        "step_chain_time": ct - last[3],
        "step_sim_time": st - last[4],
        "episode_reward_attacker": ra,
        "episode_reward_defender": rd,
        "episode_progress": prog,
        "episode_chain_time": ct,
        "episode_sim_time": st,
        "episode_n_steps": int(inf["episode_n_steps"][0]),
        "episode_n_activations": int(inf["episode_n_activations"][0]),
    }
    if ienv.proto.protocol_id == L.PROTO_TAILSTORM:
        # tailstorm.ml:45-52 (Protocol.info), :89-94 (Referee.info of a summary)
        info["protocol_family"] = "tailstorm"
        info["protocol_k"] = ienv.proto.params["k"]
        info["protocol_incentive_scheme"] = ienv.proto.params["reward"]
        info["protocol_subblock_selection"] = ienv.proto.params["subblock_selection"]
        info["head_kind"] = "summary"
        info["head_height"] = int(inf["head_height"][0])
    elif ienv.proto.protocol_id == L.PROTO_BK:
        # bk.ml:21-24 (Protocol.info), :53-58 (Referee.info of a block)
        info["protocol_family"] = "bk"
        info["protocol_k"] = ienv.proto.params["k"]
        info["protocol_incentive_scheme"] = ienv.proto.params["reward"]
        info["head_kind"] = "block"
        info["head_height"] = int(inf["head_height"][0])
    elif ienv.proto.protocol_id == L.PROTO_ETHEREUM:
        # ethereum.ml:57-63 (Protocol.info, Byzantium + scheme), :92-95 (Referee.info)
        info["protocol_preference"] = "heaviest_chain"
        info["protocol_progress"] = "work"
        info["protocol_max_uncles"] = "2"
        info["protocol_incentive_scheme"] = ienv.proto.params["reward"]
        info["head_height"] = int(inf["head_height"][0])
        info["head_work"] = int(round(prog))
    else:
        info["protocol_family"] = "nakamoto"
        info["head_height"] = int(inf["head_height"][0])
        info["head_miner"] = _miner_str(int(inf["head_miner"][0]))
    if status & L.ST_LOCKSTEP_INEXACT and not status & L.ST_EXACT_RERUN:
        # Nakamoto lockstep lane outside its closed form that could not move to the exact
        # engine (no free exact slot, or a configuration that engine cannot hold): outputs
        # not exact; not a reference key
        info["device_status"] = status
    ienv._last = (ra, rd, prog, ct, st)
    return obs[0].copy(), float(rew[0]), bool(done[0]), info


def policies(ienv):
    """name -> callable(obs) -> int, in the reference's registry order."""
    out = {}
    n = len(_space(ienv)["fields"])
    for name, pid in device.policy_registry(ienv.proto.protocol_id):

        def fn(obs, _pid=pid):
            o = np.asarray(obs, dtype=np.float64)
            if o.shape != (n,):
                raise ValueError("invalid dimensions")
            return int(ienv.batch.policy_actions(_pid, o)[0])

        out[name] = fn
    return out


def n_actions(ienv):
    return ienv.batch.observation_spec()[1]


def observation_low(ienv):
    return ienv.batch.observation_spec()[2]


def observation_high(ienv):
    return ienv.batch.observation_spec()[3]


def _observe_hum(ienv):
    # Observation.to_string: "field: value" per record field (nakamoto_ssz.ml, bk_ssz.ml:123-143)
    sp = _space(ienv)
    f = ienv.batch.observe_fields()[0]
    lines = []
    for name, v in zip(sp["fields"], f):
        if name == "event":
            lines.append(f"event: {sp['events'][v]}")
        elif name in sp["bools"]:
            lines.append(f"{name}: {'true' if v else 'false'}")
        else:
            lines.append(f"{name}: {v}")
    return "\n".join(lines)


def to_string(ienv):
    # engine.ml:250-257
    actions = " | ".join(f"({i}) {a}" for i, a in enumerate(_space(ienv)["actions"]))
    return "%s; %s; α=%.2f attacker\n%s\nActions: %s" % (
        ienv.proto.description,
        ienv.proto.attack_info,
        ienv.params["alpha"],
        _observe_hum(ienv),
        actions,
    )


# importable as top-level `engine` like the reference's pyml module
sys.modules.setdefault("cpr_amd_engine", sys.modules[__name__])
