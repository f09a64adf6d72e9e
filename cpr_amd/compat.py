"""Install this engine under the module names the reference's Python package imports.

gym/ocaml/cpr_gym/__init__.py:55-64 loads cpr_gym_engine.so with PyDLL, starts the OCaml
runtime and then does ``import engine, protocols`` (the pyml-registered modules of
simulator/gym/cpr_gym_engine.ml). Calling ``install()`` first registers cpr_amd's
drop-ins under those names, so gym/ocaml/cpr_gym/envs.py and wrappers.py run unchanged
on the GPU engine.
"""

import sys


def install():
    from . import engine, protocols

    sys.modules["engine"] = engine
    sys.modules["protocols"] = protocols
    return engine, protocols
