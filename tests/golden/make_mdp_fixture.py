"""Golden vectors for cpr_amd/mdp.py from the reference's own MDP toolbox.

Imports /root/reference/mdp (numpy/scipy only; SURVEY.md §8c: importable here) and records,
for a few (alpha, gamma) points of the Sapirshtein FC'16 Bitcoin model, the compiled state
order (mdp/lib/compiler.py), and the PTO value-iteration result (aft20barzur.ptmdp +
explicit_mdp.value_iteration, as mdp/sprint-0-explicit-mdps/util.py:6-14): policy (action
ids), values and iteration count. Data only.

Run here (the container that has /root/reference):  python tests/golden/make_mdp_fixture.py
"""

import json
import pathlib
import sys

sys.path.insert(0, "/root/reference/mdp")
from lib.compiler import Compiler  # noqa: E402
from lib.models import aft20barzur, fc16sapirshtein  # noqa: E402

OUT = pathlib.Path(__file__).with_name("mdp_fc16_vi.json")
POINTS = [(0.25, 0.0, 8, 50, 1e-5), (1 / 3, 0.5, 10, 100, 1e-5), (0.4, 0.9, 12, 100, 1e-4),
          (0.45, 0.5, 10, 200, 1e-4)]


def main():
    cases = []
    for alpha, gamma, mfl, horizon, stop in POINTS:
        model = fc16sapirshtein.BitcoinSM(alpha=alpha, gamma=gamma, maximum_fork_length=mfl)
        c = Compiler(model)
        m = c.mdp()
        states = [None] * len(c.state_map)
        for s, i in c.state_map.items():
            states[i] = [s.a, s.h, s.fork]
        vi = aft20barzur.ptmdp(m, horizon=horizon).value_iteration(
            stop_delta=stop, eps=None, discount=1)
        cases.append(dict(alpha=alpha, gamma=gamma, maximum_fork_length=mfl, horizon=horizon,
                          stop_delta=stop, states=states,
                          vi_policy=[int(x) for x in vi["vi_policy"]],
                          vi_value=[float(x) for x in vi["vi_value"]],
                          vi_iter=int(vi["vi_iter"])))
        print(alpha, gamma, len(states), vi["vi_iter"])
    OUT.write_text(json.dumps({"source": "mdp/lib (fc16sapirshtein, compiler, aft20barzur.ptmdp,"
                                         " explicit_mdp.value_iteration)", "cases": cases}) + "\n")
    print("wrote", OUT, OUT.stat().st_size, "bytes")


if __name__ == "__main__":
    main()
