"""Timing probes for k_run_episodes (not product code): build libcpr_hip variants whose
kernels.hip translation unit has one cost centre replaced by a trivial stand-in, so one
GPU call can time each (tools/nak_probe_ab.sh). The stand-ins break the keyed stream, so
the variants' results are meaningless; only their kernel times are read.

  cheap_rng : Philox4x32-10 -> two multiply-xorshift rounds
  cheap_log : fdlibm cpr_log -> (x - 1) (a negative number, so delays stay positive)
  cheap_both: both
  cheap_link: the link draws (the race at a match: a second Philox per activation in
              which any lane of the wave races) -> a multiply-xorshift hash
  base      : the tree as it is
  tt1w4     : the d = 2 tie-rule kernel at 4 waves/SIMD instead of 5
  tt0       : no tie-rule kernel (d = 2 runs the heap-replay summary-only kernel)
  norace    : cost probe, the d = 2 kernel's races decided without their link draw
  nodefer   : the d = 2 kernel with its races verified eagerly (CPR_DEFER_RACES 0, TT = 1)
  defer*    : the d = 2 kernel with its races deferred (CPR_DEFER_RACES 1, TT = 2)
  nodrain   : cost probe, deferred races never verified (the queue is only emptied)
  nosave    : cost probe, deferred races verified without moving the checkpoint
  rqN       : the deferred races' list with N entries per lane of the wave (RQ_LANE)
  asmfma    : the log polynomial's fma as v_fma_f64 with SGPR coefficients (CPR_FMA_ASM 1,
              the default since r03n; nofma: CPR_FMA_ASM 0)
  g0wN      : the gamma = 0 kernel compiled for at least N waves per SIMD (CPR_G0_WAVES,
              8 by default since r03n)
  *_nock    : cost probe, no checkpoint and no rollback after a verification
  *_nolink  : cost probe, and the verification without its link draws
  *_norb    : cost probe, the checkpoint kept, no rollback code
  *_nosv    : cost probe, the rollback code kept (never run), no checkpoint
  nokeep    : every tie rolls back (no closed-form tie rule in the verification)
  wavesN    : k_run_episodes compiled for N waves per SIMD instead of 4 (VGPR budget 512/N)
  ilp       : the scheduler's max-ILP strategy (-mllvm -amdgpu-sched-strategy=max-ilp)
  biasN     : the scheduler's occupancy-vs-latency bias N (-amdgpu-schedule-metric-bias)

usage: python tools/nak_probe_variants.py [name | name@gitrev ...]  (build/var/<name>.so;
       name@rev builds the csrc/ of that git revision, e.g. prev@HEAD)
"""
import os
import pathlib
import re
import shutil
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
CSRC = ROOT / "cpr_amd" / "csrc"
OUT = ROOT / "build" / "var"

PHILOX_OLD = "#pragma unroll\n  for (int r = 0; r < 10; ++r) {"
PHILOX_NEW = """#if 1  // probe: cheap stand-in
  {
    uint32_t h = c0 * 0x9E3779B9u ^ c1 * 0x85EBCA6Bu ^ c2 * 0xC2B2AE35u ^ c3 ^ k0 ^ k1;
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12;
    return Words4{h, h * 0x297A2D39u, h ^ 0x5BD1E995u, (h >> 7) * 0x68E31DA4u};
  }
#endif
#pragma unroll
  for (int r = 0; r < 10; ++r) {"""
LINK_OLD = """  __host__ __device__ inline double link_u(uint32_t kw, uint32_t off, uint32_t dest) const {
"""
LINK_NEW = LINK_OLD + """    if (1) {  // probe: cheap stand-in for the race's link draw
      uint32_t h = (kw * 0x9E3779B9u) ^ (off * 0x85EBCA6Bu) ^ (dest * 0xC2B2AE35u) ^ e0 ^ k0;
      h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12;
      return (double)h * (1.0 / 4294967296.0);
    }
"""
LOG_OLD = "__host__ __device__ inline double cpr_log(double x) {"
LOG_NEW = LOG_OLD + "\n  return x - 1.0;  // probe: cheap stand-in"


def variant(name, rng, log, rev=None):
    d = ROOT / "cpr_amd" / ("csrc_probe_" + name)  # same depth: ../../include resolves
    if d.exists():
        shutil.rmtree(d)
    shutil.copytree(CSRC, d)
    if rev:  # the csrc/ tree of a git revision instead of the working tree
        for f in d.iterdir():
            blob = subprocess.run(["git", "-C", str(ROOT), "show", f"{rev}:cpr_amd/csrc/{f.name}"],
                                  capture_output=True)
            if blob.returncode == 0:
                f.write_bytes(blob.stdout)
    st = (d / "cpr_stream.h").read_text()
    if rng:
        assert PHILOX_OLD in st
        st = st.replace(PHILOX_OLD, PHILOX_NEW, 1)
    if log:
        assert LOG_OLD in st
        st = st.replace(LOG_OLD, LOG_NEW, 1)
    if "link" in name:
        assert LINK_OLD in st
        st = st.replace(LINK_OLD, LINK_NEW, 1)
    (d / "cpr_stream.h").write_text(st)
    if name.startswith("tt1w4"):  # the d = 2 tie-rule kernel at the 4-wave budget
        k = (d / "kernels.hip").read_text()
        assert "amdgpu_waves_per_eu(TT ? 5 : 4)" in k
        (d / "kernels.hip").write_text(k.replace("amdgpu_waves_per_eu(TT ? 5 : 4)",
                                                 "amdgpu_waves_per_eu(4)"))
    if name.startswith("tt0"):  # no tie-rule kernel: d = 2 runs the heap-replay kernel
        k = (d / "kernels.hip").read_text()
        old = "if (P.d != 2) return k_run_episodes<CPR_MODE_GYM, SeedSource, POL, 0, 1>;"
        assert old in k
        (d / "kernels.hip").write_text(k.replace(old, old.replace("P.d != 2", "true")))
    if name.startswith("tt1d2"):  # the tie-rule kernel with d = 2 a compile-time constant
        k = (d / "kernels.hip").read_text()
        old = "  if (ARR >= 0) P.arrive = ARR;"
        assert old in k
        (d / "kernels.hip").write_text(k.replace(old, old + "\n  if (TT) P.d = 2;"))
    if name.startswith("norace"):  # cost probe: d = 2 races always won by the release
        lane = (d / "nakamoto_lane.h").read_text()
        old = "      for (int32_t i = 0; i < P.d - 1; ++i) {"
        assert old in lane
        lane = lane.replace(old, "      if (TT) { mask = 1ull << (2 - wminer); } else\n" + old, 1)
        (d / "nakamoto_lane.h").write_text(lane)
    if "nodefer" in name:  # races verified eagerly (the TT = 1 kernel)
        k = (d / "kernels.hip").read_text()
        (d / "kernels.hip").write_text("#define CPR_DEFER_RACES 0\n" + k)
    elif "defer" in name:  # races deferred (the TT = 2 kernel) whatever the default
        k = (d / "kernels.hip").read_text()
        (d / "kernels.hip").write_text("#define CPR_DEFER_RACES 1\n" + k)
    if name.startswith("nodrain") or name.startswith("nosave"):
        lane = (d / "nakamoto_lane.h").read_text()
        old = "  bool wrong = false;\n  for (int32_t i = 0; i < L.qn; ++i) {"
        assert old in lane
        if name.startswith("nodrain"):
            lane = lane.replace(old, "  if (1) { L.qn = 0; return; }\n" + old, 1)
        else:
            old2 = "  L.save(M.ck, M.ck_stride);\n}"
            assert old2 in lane
            lane = lane.replace(old2, "}", 1)
        (d / "nakamoto_lane.h").write_text(lane)
    if "asmfma" in name or "nofma" in name:  # the log polynomial's fma (CPR_FMA_ASM)
        st2 = (d / "cpr_stream.h").read_text()
        flag = 0 if "nofma" in name else 1
        (d / "cpr_stream.h").write_text(f"#define CPR_FMA_ASM {flag}\n" + st2)
    m8 = re.search(r"g0w(\d+)", name)
    if m8:  # the gamma = 0 kernel's waves-per-SIMD minimum (CPR_G0_WAVES)
        k = (d / "kernels.hip").read_text()
        (d / "kernels.hip").write_text(f"#define CPR_G0_WAVES {m8.group(1)}\n" + k)
    if "_nock" in name or "_nolink" in name:
        lane = (d / "nakamoto_lane.h").read_text()
        for old, new in [("  if (wrong) {\n    const int32_t k_now", "  if (wrong && false) {\n    const int32_t k_now"),
                         ("  L.save(M.ck, M.ck_stride);\n}\ntemplate <int POL, class St>",
                          "}\ntemplate <int POL, class St>")]:
            assert old in lane, old
            lane = lane.replace(old, new, 1)
        if "_nolink" in name:
            old = "      const double a = t + so.link(e.z, (uint32_t)(rhi - m), j, P.dmax);"
            assert old in lane
            lane = lane.replace(old, "      const double a = t + (double)(e.z ^ so.e0) * 1e-20;", 1)
        (d / "nakamoto_lane.h").write_text(lane)
    if "_norb" in name or "_nosv" in name:
        lane = (d / "nakamoto_lane.h").read_text()
        old = "  if (wrong) {\n    const int32_t k_now"
        assert old in lane
        if "_norb" in name:
            lane = lane.replace(old, "  if (wrong && false) {\n    const int32_t k_now", 1)
        else:
            lane = lane.replace(old, "  if (wrong && L.k < 0) {\n    const int32_t k_now", 1)
            old = "  L.save(M.ck, M.ck_stride);\n}\ntemplate <int POL, class St>"
            assert old in lane
            lane = lane.replace(old, "}\ntemplate <int POL, class St>", 1)
        (d / "nakamoto_lane.h").write_text(lane)
    if "nokeep" in name:
        lane = (d / "nakamoto_lane.h").read_text()
        old = "      const bool kept = v == tb && rlo == rhi &&"
        assert old in lane
        lane = lane.replace(old, "      const bool kept = false && v == tb && rlo == rhi &&", 1)
        (d / "nakamoto_lane.h").write_text(lane)
    m = re.match(r"rq(\d+)", name)
    if m:
        lane = (d / "nakamoto_lane.h").read_text()
        old = re.search(r"constexpr int32_t RQ_LANE = \d+;", lane).group(0)
        (d / "nakamoto_lane.h").write_text(lane.replace(old, f"constexpr int32_t RQ_LANE = {m.group(1)};"))
    m = re.match(r"waves(\d+)", name)
    if m:
        k = (d / "kernels.hip").read_text()
        assert "amdgpu_waves_per_eu(4)" in k
        (d / "kernels.hip").write_text(k.replace("amdgpu_waves_per_eu(4)",
                                                 f"amdgpu_waves_per_eu({m.group(1)})", 1))
    extra = os.environ.get("PROBE_DEFS", "").split()  # e.g. "-DCPR_TT_WAVES=6 -DCPR_RQ_LANE=5"
    if name.startswith("ilp"):
        extra += ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
    m = re.match(r"bias(\d+)", name)
    if m:
        extra += ["-mllvm", f"-amdgpu-schedule-metric-bias={m.group(1)}"]
    tu = os.environ.get("PROBE_TU", "kernels.hip")  # the translation unit rebuilt
    obj = OUT / f"{tu}_{name}.o"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-ffp-contract=off", "-fPIC", f"-I{ROOT / 'include'}", *extra, "-c",
                    str(d / tu), "-o", str(obj)], check=True)
    objs = [str(obj)] + [str(p) for p in sorted((ROOT / "build" / "hip").glob("*.o"))
                         if p.name != f"{tu}.o"]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", *objs,
                    "-o", str(OUT / f"{name}.so")], check=True)
    shutil.rmtree(d)


if __name__ == "__main__":
    OUT.mkdir(parents=True, exist_ok=True)
    names = sys.argv[1:] or ["base", "cheap_rng", "cheap_log", "cheap_both"]
    for n in names:
        rev = n.split("@", 1)[1] if "@" in n else None  # e.g. prev@HEAD~1
        n = n.split("@", 1)[0]
        variant(n, "rng" in n or "both" in n, "log" in n or "both" in n, rev)
        print("built", OUT / f"{n}.so")
