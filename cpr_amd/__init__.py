"""cpr_amd — MI355X-native batched episode engine for pkel/cpr's gym hot path.

Layout:
  csrc/        HIP kernels for gfx950 + the C ABI (include/cpr_hip.h) -> libcpr_hip.so
  _lib.py      ctypes binding (no CPU fallback)
  device.py    contexts, batches (fused episodes, lockstep lanes)
  engine.py    drop-in for the reference's `engine` module (cpr_gym_engine.ml:37-163)
  protocols.py drop-in for the reference's `protocols` module (cpr_gym_engine.ml:165-304)
  envs.py      Core env, env_fn and registered ids (gym/ocaml/cpr_gym/envs.py)
  wrappers.py  reward / assumption wrappers (gym/ocaml/cpr_gym/wrappers.py)
  parallel.py  one process per GPU, episode sharding, RCCL all-reduce of batch summaries
"""

__version__ = "0.1.0"
