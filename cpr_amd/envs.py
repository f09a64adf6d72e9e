"""Gym-style environments over the device engine, mirroring gym/ocaml/cpr_gym/envs.py:
``Core`` (core-v0), ``env_fn`` (cpr-v0, cpr-nakamoto-v0) and a tiny registry. ``gym`` is
not installed in this image, so ``Env``/``Discrete``/``Box`` are minimal local classes
with the same call signatures (reset() -> obs, step(a) -> (obs, r, done, info)).
"""

import warnings

import numpy as np

from . import engine, protocols, wrappers


class Discrete:
    def __init__(self, n, seed=None):
        self.n = int(n)
        self._rng = np.random.default_rng(seed)

    def sample(self):
        return int(self._rng.integers(self.n))

    def contains(self, x):
        return 0 <= int(x) < self.n


class Box:
    def __init__(self, low, high, dtype=np.float64):
        self.low = np.asarray(low, dtype=dtype)
        self.high = np.asarray(high, dtype=dtype)
        self.shape = self.low.shape
        self.dtype = dtype

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))


class Env:
    metadata = {}
    action_space = None
    observation_space = None

    def reset(self):
        raise NotImplementedError

    def step(self, action):
        raise NotImplementedError

    @property
    def unwrapped(self):
        return self


class Core(Env):
    """envs.py:9-96: one episode at a time; each reset builds a fresh engine instance."""

    metadata = {"render.modes": ["ascii"]}

    def __init__(self, proto=None, alpha=0.25, gamma=0.5, activation_delay=1.0, **kwargs):
        if proto is None:
            proto = protocols.nakamoto(unit_observation=True)
        self.core_kwargs = kwargs
        self.core_kwargs["proto"] = proto
        self.core_kwargs["alpha"] = alpha
        self.core_kwargs["gamma"] = gamma
        self.core_kwargs["activation_delay"] = activation_delay
        if not any(k in kwargs for k in ("max_time", "max_progress", "max_steps")):
            raise ValueError(
                "cpr_gym: set at least one of kwargs max_progress, max_steps, and max_time."
            )
        for k in ("max_time", "max_progress", "max_steps"):
            if k in kwargs and kwargs[k] is None:
                kwargs.pop(k)
        self.ocaml_env = None
        Core.reset(self)
        self.action_space = Discrete(engine.n_actions(self.ocaml_env))
        self.observation_space = Box(
            np.array(engine.observation_low(self.ocaml_env)),
            np.array(engine.observation_high(self.ocaml_env)),
        )
        self.version = engine.cpr_lib_version

    def policies(self):
        return engine.policies(self.ocaml_env).keys()

    def policy(self, obs, name="honest"):
        try:
            fn = engine.policies(self.ocaml_env)[name]
        except KeyError:
            raise ValueError(
                name + " is not a valid policy; choose from " + ", ".join(self.policies())
            )
        return fn(obs)

    def reset(self):
        kwargs = dict(self.core_kwargs)
        d = kwargs.pop("defenders", None)
        if d is None:
            g = kwargs["gamma"]
            if g >= 1:
                raise ValueError("gamma must be smaller than 1")
            d = max(2, int(np.ceil(1 / (1 - g))))
            if d >= 100:
                warnings.warn(f"Expensive assumptions: gamma={g} implies defenders>={d}")
        self.ocaml_env = engine.create(defenders=d, **kwargs)
        return np.array(engine.reset(self.ocaml_env))

    def step(self, a):
        obs, r, d, i = engine.step(self.ocaml_env, a)
        return np.array(obs), r, d, i

    def render(self, mode="ascii"):
        print(engine.to_string(self.ocaml_env))


def env_fn(
    protocol="nakamoto",
    protocol_args=None,
    _protocol_args=dict(unit_observation=True),
    activation_delay=1.0,
    episode_len=128,
    alpha=0.45,
    gamma=0.5,
    pretend_alpha=None,
    pretend_gamma=None,
    defenders=None,
    reward="sparse_relative",
    normalize_reward=True,
):
    """envs.py:99-163: Core + AssumptionScheduleWrapper + reward wrapper (+ r/alpha)."""
    ctor = getattr(protocols, protocol)
    args = dict(_protocol_args) if protocol_args is None else {**_protocol_args, **protocol_args}
    reward_wrappers = {
        "sparse_relative": (wrappers.SparseRelativeRewardWrapper, dict(max_steps=episode_len)),
        "sparse_per_progress": (wrappers.SparseRewardPerProgressWrapper, dict(max_steps=episode_len)),
        "dense_per_progress": (
            lambda env: wrappers.DenseRewardPerProgressWrapper(env, episode_len=episode_len),
            dict(max_steps=None),
        ),
    }
    wrap, env_args = reward_wrappers[reward]
    env = Core(proto=ctor(**args), activation_delay=1.0, alpha=0.0, gamma=0.0,
               defenders=defenders, **env_args)
    env = wrappers.AssumptionScheduleWrapper(env, alpha=alpha, gamma=gamma,
                                             pretend_alpha=pretend_alpha,
                                             pretend_gamma=pretend_gamma)
    env.reset()
    env = wrap(env)
    if normalize_reward:
        env = wrappers.MapRewardWrapper(env, lambda r, i: r / i["alpha"])
    return env


_registry = {
    "core-v0": (Core, {}),
    "cpr-v0": (env_fn, {}),
    "cpr-nakamoto-v0": (
        env_fn,
        dict(protocol="nakamoto", _protocol_args=dict(unit_observation=True), reward="sparse_relative"),
    ),
    "cpr-tailstorm-v0": (
        env_fn,
        dict(
            protocol="tailstorm",
            _protocol_args=dict(k=8, reward="discount", subblock_selection="heuristic",
                                unit_observation=True),
            reward="sparse_per_progress",
        ),
    ),
}


def make(env_id, **kwargs):
    """gym.make replacement for the ids registered by envs.py:166-191."""
    env_id = env_id.split(":")[-1]
    ctor, defaults = _registry[env_id]
    return ctor(**{**defaults, **kwargs})
