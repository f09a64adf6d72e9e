"""Table policies for the device's table-driven Nakamoto path from the selfish-mining MDP.

SURVEY.md §8f rank 4: the reference derives optimal withholding policies offline with its
MDP toolbox — the Sapirshtein et al. (FC'16) Bitcoin model (`mdp/lib/models/fc16sapirshtein.py:
21-205`), explored breadth-first into an explicit MDP (`mdp/lib/compiler.py:6-90`), mapped to
a probabilistically terminating MDP (`mdp/lib/models/aft20barzur.py:244-300` `ptmdp`) and
solved by value iteration (`mdp/lib/explicit_mdp.py:97-177`, used as in
`mdp/sprint-0-explicit-mdps/util.py:6-14`). This module restates that pipeline (same state
order, same transition order, same floating-point accumulation order, same first-best
tie rule) and turns the policy into the `dim * dim * 2` action table that `CPR_POLICY_TABLE`
evaluates on the device (`nakamoto_lane.h` `nak_policy`: index `(h * dim + a) * 2 + event`).

Host-side numpy; nothing here runs per step.
"""

from collections import deque

import numpy as np

# fc16sapirshtein.py:11-19 (same encoding as nakamoto_ssz's Action ranks)
ADOPT, OVERRIDE, MATCH, WAIT = 0, 1, 2, 3
IRRELEVANT, RELEVANT, ACTIVE = 0, 1, 2


class BitcoinSM:
    """fc16sapirshtein.BitcoinSM: states (a, h, fork), actions per state in the model's
    order, transitions as (state, probability, reward, progress)."""

    def __init__(self, alpha, gamma, maximum_fork_length, maximum_dag_size=0):
        if alpha < 0 or alpha >= 0.5:
            raise ValueError("alpha must be between 0 and 0.5")
        if gamma < 0 or gamma > 1:
            raise ValueError("gamma must be between 0 and 1")
        self.alpha, self.gamma = alpha, gamma
        self.mfl, self.mds = maximum_fork_length, maximum_dag_size

    def start(self):  # :60-64
        return [((1, 0, IRRELEVANT), self.alpha), ((0, 1, IRRELEVANT), 1 - self.alpha)]

    def truncated(self, s):  # :66-77
        a, h, _ = s
        if self.mfl > 0 and (a >= self.mfl or h >= self.mfl):
            return True
        return self.mds > 0 and a + h + 1 >= self.mds

    def actions(self, s):  # :79-91
        a, h, fork = s
        acts = []
        if not self.truncated(s):
            acts.append(WAIT)
        if a > h:
            acts.append(OVERRIDE)
        if a >= h and fork == RELEVANT:
            acts.append(MATCH)
        acts.append(ADOPT)
        return acts

    def apply(self, act, s):  # :93-183
        a, h, fork = s
        al, ga = self.alpha, self.gamma
        if act == ADOPT:
            return [((1, 0, IRRELEVANT), al, 0, h), ((0, 1, IRRELEVANT), 1 - al, 0, h)]
        if act == OVERRIDE:
            return [((a - h, 0, IRRELEVANT), al, h + 1, h + 1),
                    ((a - h - 1, 1, RELEVANT), 1 - al, h + 1, h + 1)]
        if act == WAIT and fork != ACTIVE:
            return [((a + 1, h, IRRELEVANT), al, 0, 0.0), ((a, h + 1, RELEVANT), 1 - al, 0, 0)]
        # MATCH, or WAIT while a match is active
        return [((a + 1, h, ACTIVE), al, 0, 0.0),
                ((a - h, 1, RELEVANT), ga * (1 - al), h, h),
                ((a, h + 1, RELEVANT), (1 - ga) * (1 - al), 0, 0)]


def compile_mdp(model):
    """compiler.py:6-90: breadth-first exploration; state ids in discovery order, action ids
    = positions in model.actions(state). Returns (states, tab) with
    tab[s][i] = [(dst, p, reward, progress), ...]."""
    ids, states, tab = {}, [], []
    queue, explored = deque(), set()
    for s, _p in model.start():
        ids[s] = len(states)
        states.append(s)
        tab.append([])
        queue.append(s)
    while queue:
        s = queue.popleft()
        if s in explored:
            continue
        explored.add(s)
        sid = ids[s]
        for act in model.actions(s):
            lst = []
            for to, p, r, prg in model.apply(act, s):
                if to not in ids:
                    ids[to] = len(states)
                    states.append(to)
                    tab.append([])
                    queue.append(to)
                lst.append((ids[to], p, r, prg))
            tab[sid].append(lst)
    return states, tab


def ptmdp(tab, horizon):
    """aft20barzur.py:244-300: one terminal state (the last id); every transition with
    progress > 0 splits into termination with 1 - (1 - 1/H)^progress and the rest."""
    assert horizon > 0
    terminal = len(tab)
    out = []
    for actions in tab:
        new_actions = []
        for lst in actions:
            nl = []
            for dst, p, r, prg in lst:
                if prg == 0.0:
                    nl.append((dst, p, r, prg))
                else:
                    term = 1.0 - ((1.0 - (1.0 / horizon)) ** prg)
                    nl.append((terminal, term * p, 0.0, 0.0))
                    nl.append((dst, (1 - term) * p, r, prg))
            new_actions.append(nl)
        out.append(new_actions)
    out.append([])  # the terminal state has no actions
    return out


def value_iteration(tab, *, stop_delta, discount=1.0, max_iter=0):
    """explicit_mdp.py:97-177 vectorised over states: per (state, action) the transitions
    accumulate in their order, the first action with the strictly best value wins."""
    n = len(tab)
    n_act = max((len(a) for a in tab), default=0)
    n_tr = max((len(l) for a in tab for l in a), default=0)
    dst = np.zeros((n, n_act, n_tr), np.int64)
    prb = np.zeros((n, n_act, n_tr))
    rew = np.zeros((n, n_act, n_tr))
    prg = np.zeros((n, n_act, n_tr))
    valid = np.zeros((n, n_act), bool)
    used = np.zeros((n, n_act, n_tr), bool)
    for s, actions in enumerate(tab):
        for i, lst in enumerate(actions):
            valid[s, i] = True
            for j, (d, p, r, g) in enumerate(lst):
                dst[s, i, j], prb[s, i, j], rew[s, i, j], prg[s, i, j] = d, p, r, g
                used[s, i, j] = True
    value = np.zeros(n)
    progress = np.zeros(n)
    policy = np.zeros(n, np.int64)
    it = 1
    while True:
        this_v = np.zeros((n, n_act))
        this_p = np.zeros((n, n_act))
        for j in range(n_tr):  # += in transition order, as the reference's inner loop
            tv = prb[:, :, j] * (rew[:, :, j] + discount * value[dst[:, :, j]])
            tp = prb[:, :, j] * (prg[:, :, j] + discount * progress[dst[:, :, j]])
            this_v = np.where(used[:, :, j], this_v + tv, this_v)
            this_p = np.where(used[:, :, j], this_p + tp, this_p)
        best_a = np.full(n, -1, np.int64)
        best_v = np.zeros(n)
        best_p = np.zeros(n)
        for i in range(n_act):  # `this_v > best_v or best_a < 0`
            take = valid[:, i] & ((this_v[:, i] > best_v) | (best_a < 0))
            best_a = np.where(take, i, best_a)
            best_v = np.where(take, this_v[:, i], best_v)
            best_p = np.where(take, this_p[:, i], best_p)
        delta = float(np.abs(best_v - value).max()) if n else 0.0
        value, progress, policy = best_v, best_p, best_a
        if max_iter > 0 and it >= max_iter:
            break
        if delta <= stop_delta:
            break
        it += 1
    return dict(vi_policy=policy, vi_value=value, vi_progress=progress, vi_iter=it,
                vi_delta=delta)


def solve(alpha, gamma, *, maximum_fork_length=20, horizon=100, stop_delta=1e-6):
    """The SSZ'16 Bitcoin MDP solved for PTO revenue; returns (model, states, vi)."""
    model = BitcoinSM(alpha, gamma, maximum_fork_length)
    states, tab = compile_mdp(model)
    vi = value_iteration(ptmdp(tab, horizon), stop_delta=stop_delta)
    return model, states, vi


def policy_table(alpha, gamma, *, dim=None, maximum_fork_length=20, horizon=100,
                 stop_delta=1e-6):
    """A `CPR_POLICY_TABLE` for `device.make_config(table=...)`: entry (h, a, event) =
    the MDP's action in state (a, h, IRRELEVANT) for event = ProofOfWork (0) and
    (a, h, RELEVANT) for event = Network (1) — the attacker's view after its own block or a
    defender's block; an active match (ACTIVE) is not observable by nakamoto_ssz and shares
    the ProofOfWork entry. States the MDP does not reach fall back to the other event's entry,
    else to honest play (nakamoto_ssz.ml:275-284)."""
    model, states, vi = solve(alpha, gamma, maximum_fork_length=maximum_fork_length,
                              horizon=horizon, stop_delta=stop_delta)
    dim = maximum_fork_length + 1 if dim is None else dim
    act = {}
    for sid, s in enumerate(states):
        acts = model.actions(s)
        if acts:
            act[s] = acts[int(vi["vi_policy"][sid])]
    table = np.zeros((dim, dim, 2), np.uint8)
    for h in range(dim):
        for a in range(dim):
            honest = OVERRIDE if a > h else (ADOPT if a < h else WAIT)
            for ev, fork, other in ((0, IRRELEVANT, RELEVANT), (1, RELEVANT, IRRELEVANT)):
                x = act.get((a, h, fork), act.get((a, h, other), honest))
                if x == MATCH and ev == 0 and (a, h, fork) not in act:
                    x = honest
                table[h, a, ev] = x
    return table.ravel()


# ---- the FC'16 abstract-model kernel (gym/rust/src/fc16.rs, cpr_amd/csrc/fc16_lane.h)

FC16_WAIT, FC16_ADOPT, FC16_OVERRIDE, FC16_MATCH = 0, 1, 2, 3  # fc16.rs:19-25 names
_FC16_NAME = {WAIT: FC16_WAIT, ADOPT: FC16_ADOPT, OVERRIDE: FC16_OVERRIDE, MATCH: FC16_MATCH}


def fc16_table(alpha, gamma, *, dim=None, maximum_fork_length=20, horizon=100,
               stop_delta=1e-6):
    """A `CPR_FC16_POLICY_TABLE` (entry (a, h, fork) = an action name) from the solved
    SSZ'16 MDP: the MDP's action where it defines one, honest play elsewhere."""
    model, states, vi = solve(alpha, gamma, maximum_fork_length=maximum_fork_length,
                              horizon=horizon, stop_delta=stop_delta)
    dim = maximum_fork_length + 1 if dim is None else dim
    act = {}
    for sid, s in enumerate(states):
        acts = model.actions(s)
        if acts:
            act[s] = _FC16_NAME[acts[int(vi["vi_policy"][sid])]]
    table = np.zeros((dim, dim, 3), np.uint8)
    for a in range(dim):
        for h in range(dim):
            honest = FC16_OVERRIDE if a > h else (FC16_ADOPT if h > a else FC16_WAIT)
            for fork in (IRRELEVANT, RELEVANT, ACTIVE):
                table[a, h, fork] = act.get((a, h, fork), honest)
    return table.ravel()


def _fc16_threshold(p):
    t = p * 4294967296.0
    return 0 if t <= 0 else (4294967296 if t >= 4294967296.0 else int(t))


def fc16_policy_value(alpha, gamma, horizon, table, *, max_states=200_000):
    """Exact expected episode reward and progress of the device's FC16 lane under a table
    policy: the Markov chain of fc16.rs's transitions (a successful match adds reward h and
    progress 0, fc16.rs:109-110; the reward of the step that terminates is kept, fc16.rs:
    174-199) with the lane's draw probabilities (thresholds / 2^32), solved exactly over
    the states the policy reaches. Returns (E[reward], E[progress])."""
    pa = _fc16_threshold(alpha) / 4294967296.0
    pg = _fc16_threshold(gamma) / 4294967296.0
    pt = _fc16_threshold(1.0 / horizon) / 4294967296.0
    table = np.asarray(table, np.uint8).ravel()
    dim = int(round((table.size // 3) ** 0.5))

    def action(s):
        a, h, fork = s
        x = int(table[(min(a, dim - 1) * dim + min(h, dim - 1)) * 3 + fork])
        if (x == FC16_OVERRIDE and not a > h) or (x == FC16_MATCH and not a >= h):
            x = FC16_WAIT
        return x

    def transitions(s):
        a, h, fork = s
        x = action(s)
        if x == FC16_ADOPT:
            return [((1, 0, IRRELEVANT), pa, 0, h), ((0, 1, IRRELEVANT), 1 - pa, 0, h)]
        if x == FC16_OVERRIDE:
            return [((a - h, 0, IRRELEVANT), pa, h + 1, h + 1),
                    ((a - h - 1, 1, RELEVANT), 1 - pa, h + 1, h + 1)]
        if x == FC16_MATCH or fork == ACTIVE:
            return [((a + 1, h, ACTIVE), pa, 0, 0), ((a - h, 1, RELEVANT), (1 - pa) * pg, h, 0),
                    ((a, h + 1, RELEVANT), (1 - pa) * (1 - pg), 0, 0)]
        return [((a + 1, h, IRRELEVANT), pa, 0, 0), ((a, h + 1, RELEVANT), 1 - pa, 0, 0)]

    starts = [(1, 0, IRRELEVANT), (0, 1, IRRELEVANT)]
    ids, order, queue = {}, [], deque(starts)
    for s in starts:
        ids[s] = len(order)
        order.append(s)
    tr = []
    while queue:
        s = queue.popleft()
        row = transitions(s)
        tr.append(row)
        for d, _p, _r, _g in row:
            if d not in ids:
                if len(order) >= max_states:
                    raise ValueError("the policy reaches more than max_states states")
                ids[d] = len(order)
                order.append(d)
                queue.append(d)
    n = len(order)
    m = np.eye(n)
    rhs_r = np.zeros(n)
    rhs_g = np.zeros(n)
    for s_id, row in enumerate(tr):
        for d, p, r, g in row:
            cont = (1.0 - pt) ** g  # no termination draw fires over g units of progress
            m[s_id, ids[d]] -= p * cont
            rhs_r[s_id] += p * r
            rhs_g[s_id] += p * g
    v_r = np.linalg.solve(m, rhs_r)
    v_g = np.linalg.solve(m, rhs_g)
    return (pa * v_r[0] + (1 - pa) * v_r[1], pa * v_g[0] + (1 - pa) * v_g[1])
