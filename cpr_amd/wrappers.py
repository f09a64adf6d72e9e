"""Reward and assumption wrappers with the semantics of gym/ocaml/cpr_gym/wrappers.py.

Each wrapper forwards everything to the wrapped env and rewrites one aspect of
reset/step. The formulas (and warnings) follow the reference line by line:
  SparseRelativeRewardWrapper      wrappers.py:8-26
  SparseRewardPerProgressWrapper   wrappers.py:29-51
  DenseRewardPerProgressWrapper    wrappers.py:54-113
  ExtendObservationWrapper         wrappers.py:116-153
  MapRewardWrapper                 wrappers.py:156-169
  AssumptionScheduleWrapper        wrappers.py:172-242
  EpisodeRecorderWrapper           wrappers.py:245-266
  ClearInfoWrapper                 wrappers.py:269-289
"""

import collections
import itertools
import warnings

import numpy as np


class Wrapper:
    def __init__(self, env):
        self.env = env
        self.action_space = env.action_space
        self.observation_space = env.observation_space

    def __getattr__(self, name):
        if name.startswith("__") or name == "env":
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return self.env.unwrapped

    def reset(self):
        return self.env.reset()

    def step(self, action):
        return self.env.step(action)


class SparseRelativeRewardWrapper(Wrapper):
    """Reward = attacker share of the head's rewards, paid once at the end."""

    def step(self, action):
        obs, _, done, info = self.env.step(action)
        reward = 0
        if done:
            total = info["episode_reward_attacker"] + info["episode_reward_defender"]
            reward = info["episode_reward_attacker"] / total if total != 0 else 0
        return obs, reward, done, info


class SparseRewardPerProgressWrapper(Wrapper):
    """Reward = attacker reward per unit of chain progress, paid once at the end."""

    def step(self, action):
        obs, _, done, info = self.env.step(action)
        reward = 0
        if done:
            progress = info["episode_progress"]
            reward = info["episode_reward_attacker"] / progress if progress != 0 else 0
        return obs, reward, done, info


class DenseRewardPerProgressWrapper(Wrapper):
    """Dense variant: end the episode at a target progress, scale step rewards by 1/target
    and correct the last step for overshoot."""

    def __init__(self, env, episode_len=None):
        super().__init__(env)
        self.drpb_max_progress = episode_len
        self.drpb_factor = 1 / self.drpb_max_progress
        core = self.env.unwrapped.core_kwargs
        for k in ("max_steps", "max_time", "max_progress"):
            if k in core:
                core.pop(k, None)
                warnings.warn(
                    f"DenseRewardPerProgressWrapper overwrites argument '{k}' given to wrapped env"
                )
        core["max_steps"] = self.drpb_max_progress * 100
        core["max_progress"] = self.drpb_max_progress

    def reset(self):
        self.drpb_acc = 0
        return self.env.reset()

    def step(self, action):
        obs, reward, done, info = self.env.step(action)
        reward *= self.drpb_factor
        self.drpb_acc += reward
        if done:
            got, want = info["episode_progress"], self.drpb_max_progress
            if got < want:
                warnings.warn(f"observed too little progress: {got}/{want}")
            if got > want * 1.1:
                warnings.warn(f"observed too much progress: {got}/{want}")
            if got != want:
                reward += (want - got) * self.drpb_acc / got
        return obs, reward, done, info


class ExtendObservationWrapper(Wrapper):
    """Append fields computed from (env, info); fields = [(fn, low, high, default)]."""

    def __init__(self, env, fields):
        super().__init__(env)
        from .envs import Box

        self.eow_fields = fields
        self.eow_n = len(fields)
        low = np.array([f[1] for f in fields], dtype=np.float64)
        high = np.array([f[2] for f in fields], dtype=np.float64)
        self.observation_space = Box(
            np.append(self.observation_space.low, low), np.append(self.observation_space.high, high)
        )

    def reset(self):
        return np.append(self.env.reset(), [f[3] for f in self.eow_fields])

    def step(self, action):
        obs, reward, done, info = self.env.step(action)
        extra = [f[0](self, info) for f in self.eow_fields]
        return np.append(obs, extra), reward, done, info

    def policy(self, obs, name="honest"):
        return self.env.policy(obs[: -self.eow_n], name)


class MapRewardWrapper(Wrapper):
    def __init__(self, env, fn):
        super().__init__(env)
        self.mrw_fn = fn

    def step(self, action):
        obs, reward, done, info = self.env.step(action)
        return obs, self.mrw_fn(reward, info), done, info


def _schedule(x):
    if callable(x):
        return x
    try:
        it = itertools.cycle(x)
        return lambda: next(it)
    except TypeError:
        return lambda: x


class AssumptionScheduleWrapper(Wrapper):
    """Draw (alpha, gamma) on every reset, append them (or pretended values) to the
    observation and report them in info."""

    def __init__(self, env, alpha=None, gamma=None, pretend_alpha=None, pretend_gamma=None):
        super().__init__(env)
        from .envs import Box

        self.asw_alpha_fn = _schedule(alpha)
        self.asw_gamma_fn = _schedule(gamma)
        self.asw_pretend_alpha = pretend_alpha
        self.asw_pretend_gamma = pretend_gamma
        self.observation_space = Box(
            np.append(self.observation_space.low, [0.0, 0.0]),
            np.append(self.observation_space.high, [1.0, 1.0]),
        )

    def observation(self, obs):
        a = self.asw_alpha if self.asw_pretend_alpha is None else float(self.asw_pretend_alpha)
        g = self.asw_gamma if self.asw_pretend_gamma is None else float(self.asw_pretend_gamma)
        return np.append(obs, [a, g])

    def policy(self, obs, name="honest"):
        return self.env.policy(obs[:-2], name)

    def reset(self):
        self.asw_alpha = self.asw_alpha_fn()
        self.asw_gamma = self.asw_gamma_fn()
        core = self.env.unwrapped.core_kwargs
        core["alpha"] = self.asw_alpha
        core["gamma"] = self.asw_gamma
        return AssumptionScheduleWrapper.observation(self, self.env.reset())

    def step(self, action):
        obs, reward, done, info = self.env.step(action)
        info["alpha"] = self.asw_alpha
        info["gamma"] = self.asw_gamma
        return AssumptionScheduleWrapper.observation(self, obs), reward, done, info


class EpisodeRecorderWrapper(Wrapper):
    def __init__(self, env, n=42, info_keys=()):
        super().__init__(env)
        self.erw_info_keys = list(info_keys)
        self.erw_history = collections.deque([], maxlen=n)

    def reset(self):
        self.erw_episode_reward = 0
        return self.env.reset()

    def step(self, action):
        obs, reward, done, info = self.env.step(action)
        self.erw_episode_reward += reward
        if done:
            entry = {k: info[k] for k in self.erw_info_keys}
            entry["episode_reward"] = self.erw_episode_reward
            self.erw_history.append(entry)
        return obs, reward, done, info


class ClearInfoWrapper(Wrapper):
    def __init__(self, env, keep_keys=()):
        super().__init__(env)
        self.ciw_keys = list(keep_keys)

    def step(self, action):
        obs, reward, done, info = self.env.step(action)
        return obs, reward, done, {k: info[k] for k in self.ciw_keys if k in info}
