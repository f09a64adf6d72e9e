"""The Python drop-in API on the device (mirrors gym/ocaml/test/test_engine.py,
test_envs.py and test_protocols.py of the reference)."""

import numpy as np
import pytest

from cpr_amd import engine, envs, protocols, wrappers

pytestmark = pytest.mark.gpu


def run_episode(env, policy):
    obs = env.reset()
    done = False
    while not done:
        obs, rew, done, info = env.step(env.policy(obs, policy))
    return obs, rew, done, info


def fuzz_episode(env):
    obs = env.reset()
    done = False
    while not done:
        obs, rew, done, info = env.step(env.action_space.sample())
    return obs, rew, done, info


def test_engine():
    # test_engine.py:4-30
    env = engine.create(proto=protocols.nakamoto(unit_observation=False), alpha=0.33,
                        gamma=0.5, defenders=2, activation_delay=1)
    engine.reset(env)
    obs, rew, done, info = engine.step(env, 0)
    assert not done
    env = engine.create(proto=protocols.nakamoto(unit_observation=True), alpha=0.33,
                        gamma=0.5, defenders=2, activation_delay=1)
    engine.reset(env)
    for _ in range(600):
        obs, rew, done, info = engine.step(env, 3)
    assert not done
    assert info["episode_n_activations"] == 601
    assert list(info)[:12] == [
        "step_reward_attacker", "step_reward_defender", "step_progress", "step_chain_time",
        "step_sim_time", "episode_reward_attacker", "episode_reward_defender",
        "episode_progress", "episode_chain_time", "episode_sim_time", "episode_n_steps",
        "episode_n_activations"]


def test_render_strings(capsys):
    # test_protocols.py:12-20 and test_envs.py:145-152
    envs.Core(max_steps=1000).render()
    assert capsys.readouterr().out.splitlines()[0] == (
        "Nakamoto consensus; SSZ'16 attack space with unit observations; α=0.25 attacker")
    envs.make("cpr_gym:cpr-nakamoto-v0").render()
    out = capsys.readouterr().out.splitlines()
    assert out[0] == "Nakamoto consensus; SSZ'16 attack space with unit observations; α=0.45 attacker"
    assert out[-1] == "Actions: (0) Adopt | (1) Override | (2) Match | (3) Wait"


def test_core_env_policies_and_spaces():
    env = envs.make("core-v0", max_steps=2016)
    assert list(env.policies()) == ["sapirshtein-2016-sm1", "eyal-sirer-2014", "simple", "honest"]
    obs, rew, done, info = run_episode(env, "honest")
    assert done and env.observation_space.contains(obs)
    assert info["episode_n_steps"] == 2016
    fuzz_episode(env)
    with pytest.raises(ValueError):
        env.policy(obs, "no-such-policy")
    with pytest.raises(ValueError):
        engine.policies(env.ocaml_env)["honest"](np.zeros(3))


def test_reward_wrappers():
    # test_envs.py:33-58
    env = wrappers.SparseRelativeRewardWrapper(envs.make("core-v0", max_steps=32))
    for _ in range(5):
        _, r, done, info = run_episode(env, "honest")
        tot = info["episode_reward_attacker"] + info["episode_reward_defender"]
        assert r == pytest.approx(info["episode_reward_attacker"] / tot)
        fuzz_episode(env)
    env = wrappers.SparseRewardPerProgressWrapper(envs.make("core-v0", max_steps=32))
    _, r, _, info = run_episode(env, "honest")
    assert r == pytest.approx(info["episode_reward_attacker"] / info["episode_progress"])
    env = wrappers.DenseRewardPerProgressWrapper(
        envs.make("core-v0", max_progress=None), episode_len=32)
    for _ in range(3):
        run_episode(env, "honest")
        fuzz_episode(env)


def test_assumption_schedule_wrapper():
    # test_envs.py:61-86
    env = wrappers.AssumptionScheduleWrapper(envs.make("core-v0", max_steps=32), alpha=0.33,
                                             gamma=0.1)
    for _ in range(2):
        obs, _, _, i = fuzz_episode(env)
        assert i["alpha"] == 0.33 and i["gamma"] == 0.1
        assert obs[-2] == 0.33 and obs[-1] == 0.1
    env = wrappers.AssumptionScheduleWrapper(env, alpha=[0.1, 0.2, 0.3], gamma=[0.1, 0.5, 0.9])
    seen = set()
    for _ in range(6):
        obs, _, _, i = run_episode(env, "honest")
        assert i["alpha"] == obs[-2] and i["gamma"] == obs[-1]
        seen.add(i["alpha"])
    assert seen == {0.1, 0.2, 0.3}


def test_episode_recorder():
    env = wrappers.EpisodeRecorderWrapper(envs.make("core-v0", max_progress=100), n=10,
                                          info_keys=["head_height"])
    for _ in range(12):
        run_episode(env, "honest")
    assert len(env.erw_history) == 10
    assert all("episode_reward" in e and "head_height" in e for e in env.erw_history)


def test_registered_env_normalized_reward():
    env = envs.make("cpr-nakamoto-v0", episode_len=64, alpha=0.3, gamma=0.5)
    _, r, done, info = run_episode(env, "honest")
    assert done and info["alpha"] == 0.3
    # honest play: relative reward ~ alpha, normalised by alpha -> ~1
    assert 0.0 <= r < 3.0


def test_unsupported_protocol_is_loud():
    with pytest.raises(NotImplementedError):
        protocols.spar(k=8, reward="constant", unit_observation=True)


def test_ethereum_protocol(capsys):
    # gym/ocaml/test/test_protocols.py:77-102
    env = envs.make("cpr_gym:core-v0",
                    proto=protocols.ethereum(reward="discount", unit_observation=True),
                    alpha=0.13, gamma=0.9, defenders=10, max_steps=10000)
    env.render()
    assert capsys.readouterr().out.splitlines()[0] == (
        "Ethereum with heaviest_chain-preference, work-progress, uncle cap 2, "
        "and discount-rewards; "
        "SSZ'16-like attack space with unit observations; α=0.13 attacker")
    obs = env.reset()
    for _ in range(600):
        obs, _, _, _ = env.step(env.policy(obs, "honest"))
    obs = env.reset()
    for _ in range(600):
        obs, _, _, info = env.step(env.policy(obs, "selfish_discard"))
    assert env.observation_space.contains(obs)
    assert env.action_space.n == 24
    assert list(env.policies()) == ["fn19pkel", "fn19", "selfish_discard", "selfish_release",
                                    "honest"]
    assert info["protocol_incentive_scheme"] == "discount"
    assert info["head_work"] == info["episode_progress"]
    env.render()
    out = capsys.readouterr().out.splitlines()
    assert out[1].startswith("public_height: ") and out[10].startswith("event: `")
    assert out[-1].startswith("Actions: (0) Adopt_discard, uncles {own: false; foreign: false}"
                              " | (1) Adopt_discard, uncles {own: false; foreign: true}")
    with pytest.raises(ValueError, match="try 'constant' or 'discount'"):
        protocols.ethereum(reward="block", unit_observation=True)
    fuzz_episode(envs.make("core-v0", proto=protocols.ethereum(reward="constant",
                                                                unit_observation=False),
                           max_steps=300))


def test_bk_protocol(capsys):
    # gym/ocaml/test/test_protocols.py:105-127
    env = envs.make("cpr_gym:core-v0",
                    proto=protocols.bk(k=42, reward="constant", unit_observation=True),
                    alpha=0.33, gamma=0.3, defenders=4, max_steps=10000)
    env.render()
    assert capsys.readouterr().out.splitlines()[0] == (
        "Bₖ with k=42 and constant rewards; "
        "SSZ'16-like attack space with unit observations; α=0.33 attacker")
    obs = env.reset()
    for _ in range(600):
        obs, _, _, _ = env.step(env.policy(obs, "honest"))
    obs = env.reset()
    for _ in range(600):
        obs, _, _, info = env.step(env.policy(obs, "minor-delay"))
    assert info["protocol_k"] == 42
    assert info["protocol_family"] == "bk" and info["head_kind"] == "block"
    assert env.observation_space.contains(obs)
    assert env.action_space.n == 8
    assert list(env.policies()) == ["avoid-loss", "minor-delay", "get-ahead", "honest"]
    env.render()
    out = capsys.readouterr().out.splitlines()
    assert out[-1].startswith("Actions: (0) Adopt_Prolong | (1) Override_Prolong")
    assert out[7] == "lead: false" and out[8].startswith("event: `")
    fuzz_episode(envs.make("core-v0", proto=protocols.bk(k=8, reward="block",
                                                          unit_observation=False),
                           max_steps=300))


def test_bk_policies_and_errors():
    # test_protocols.py:22-47
    for gamma, d, pol in [(0.2, 2, "honest"), (0.5, 3, "minor-delay")]:
        env = envs.make("core-v0", proto=protocols.bk(k=8, reward="constant",
                                                      unit_observation=True),
                        alpha=0.33, gamma=gamma, defenders=d, max_steps=10000)
        obs = env.reset()
        for _ in range(600):
            obs, _, _, _ = env.step(env.policy(obs, pol))
    with pytest.raises(ValueError, match="not a valid parameter choice, try 'block' or 'constant'"):
        protocols.bk(k=8, reward="discount", unit_observation=True)
    env = envs.make("cpr-v0", protocol="bk", protocol_args=dict(k=8, reward="constant"),
                    episode_len=256)
    _, r, done, info = run_episode(env, "avoid-loss")
    assert done and info["episode_n_steps"] == 256 and r >= 0


def test_tailstorm_protocol(capsys):
    # gym/ocaml/test/test_protocols.py:230-261
    env = envs.make("cpr_gym:core-v0",
                    proto=protocols.tailstorm(k=13, reward="discount",
                                              subblock_selection="heuristic",
                                              unit_observation=True),
                    alpha=0.33, gamma=0.8, defenders=5, max_steps=10000)
    env.render()
    assert capsys.readouterr().out.splitlines()[0] == (
        "Tailstorm with k=13, discount rewards, and heuristic sub-block selection; "
        "SSZ'16-like attack space with unit observations; α=0.33 attacker")
    obs = env.reset()
    for _ in range(600):
        obs, _, _, _ = env.step(env.policy(obs, "honest"))
    obs = env.reset()
    for _ in range(600):
        obs, _, _, info = env.step(env.policy(obs, "avoid-loss"))
    assert info["protocol_k"] == 13 and info["head_kind"] == "summary"
    assert env.observation_space.contains(obs)
    assert list(env.policies()) == ["long-delay", "avoid-loss-b", "avoid-loss-a", "avoid-loss",
                                    "minor-delay", "get-ahead", "honest"]


def test_cpr_tailstorm_v0(capsys):
    # gym/ocaml/test/test_envs.py:154-169
    env = envs.make("cpr_gym:cpr-tailstorm-v0")
    env.render()
    assert capsys.readouterr().out.splitlines()[0] == (
        "Tailstorm with k=8, discount rewards, and heuristic sub-block selection; "
        "SSZ'16-like attack space with unit observations; α=0.45 attacker")
    _, r, done, info = run_episode(env, "honest")
    assert done and r >= 0
    fuzz_episode(env)
