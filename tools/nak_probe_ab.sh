#!/bin/bash
# Kernel-time A/B of the build/var/*.so variants (tools/nak_probe_variants.py): the
# default bench workload without the CPU leg, one run per variant, via CPR_HIP_LIB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-base cheap_rng cheap_log cheap_both base}; do
  for E in ${EPISODES:-393216}; do
  CPR_HIP_LIB=build/var/$v.so timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu --no-configs ${BENCH_ARGS:-} --episodes $E > gpurun_out/ab_${v}_$E.log 2>&1
  rc=$?; echo "$v $E rc=$rc" >> gpurun_out/ab_status.log; [[ $rc -eq 0 ]] || exit $rc
  python - "$v" "$E" >> gpurun_out/ab_status.log <<'PY'
import json, sys
v, E = sys.argv[1], sys.argv[2]
line = [l for l in open(f"gpurun_out/ab_{v}_{E}.log") if l.startswith("{")][-1]
d = json.loads(line)
print(v, E, "value %.4e" % d["value"], "kernel_ms %.3f" % d["roofline"]["kernel_ms_mean"],
      "abstract %.4e" % d["abstract_gamma_1"]["activations_per_s"])
PY
  done
done
