"""Summarise a tools/profile_configs.sh run (gpurun_out/cf_<n>_<pass>/) into
profiles/<tag>_config_pmc.json, the file bench.py's other_configs read their measured
`traffic` from: per config key, over the dispatches of that config's kernel that bench.py
times (every point's launch; for a rollout the last dispatch), HBM bytes per activation
(FETCH_SIZE x1024 x2 gfx950 correction + WRITE_SIZE x1024, MI355X_MICROARCH.md) and VALU
lane-instructions per activation (SQ_INSTS_VALU x 64), plus the kernel-trace durations.

Usage: python tools/summarize_configs.py <tag>
"""
import collections
import csv
import glob
import json
import os
import sys

tag = sys.argv[1]
out = {}
for trace_dir in sorted(glob.glob("gpurun_out/cf_*_trace")):
    n = os.path.basename(trace_dir)[3:-6]
    key = "configs[3]_exp" if n == "3_exp" else f"configs[{n}]"
    log = open(f"gpurun_out/cf_{n}_trace.log").read().strip().splitlines()
    info = json.loads([ln for ln in log if ln.startswith("{")][-1])[key]
    kernel = info["roofline"]["kernel"]
    rollout = "rollout_steps_per_lane" in info
    rows = [r for r in csv.DictReader(open(f"{trace_dir}/run_kernel_trace.csv"))
            if kernel + "<" in r["Kernel_Name"] or r["Kernel_Name"].startswith(kernel + "(")
            or f" {kernel}<" in r["Kernel_Name"] or f"::{kernel}<" in r["Kernel_Name"]
            or f"::{kernel}(" in r["Kernel_Name"]]
    if rollout:
        rows = rows[-1:]
    dur_ms = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows) / 1e6
    acts = info["activations"]
    c = collections.defaultdict(float)
    for p in ("sq", "fetch", "write"):
        f = f"gpurun_out/cf_{n}_{p}/run_counter_collection.csv"
        if not os.path.exists(f):
            continue
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            nm = r["Kernel_Name"]
            if f"::{kernel}<" in nm or f"::{kernel}(" in nm:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        ids = sorted(per)[-1:] if rollout else sorted(per)
        for i in ids:
            for k, v in per[i].items():
                c[k] += v
    s = {"kernel": kernel, "dispatches": len(rows), "trace_kernel_ms": dur_ms,
         "activations": acts, "probe_kernel_ms": info["kernel_ms"]}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rd, wr = c["FETCH_SIZE"] * 1024 * 2, c["WRITE_SIZE"] * 1024
        s["hbm_read_bytes (FETCH_SIZE x1024 x2)"] = rd
        s["hbm_write_bytes (WRITE_SIZE x1024)"] = wr
        s["hbm_bytes_per_activation"] = (rd + wr) / acts
        s["hbm_GB_per_s"] = (rd + wr) / (dur_ms / 1e3) / 1e9 if dur_ms else None
    if "SQ_INSTS_VALU" in c:
        s["valu_lane_ops_per_activation"] = c["SQ_INSTS_VALU"] * 64 / acts
        # the two issue counts on one scale: wave instructions per activation (a VALU wave
        # instruction is 64 lane-ops, a SALU one a single scalar issue; up to round 5 the
        # SALU figure here was the count x 64 under the name salu_instr_per_activation)
        s["valu_wave_instr_per_activation"] = c["SQ_INSTS_VALU"] / acts
        s["salu_wave_instr_per_activation"] = c["SQ_INSTS_SALU"] / acts
        s["salu_over_valu"] = c["SQ_INSTS_SALU"] / c["SQ_INSTS_VALU"] if c["SQ_INSTS_VALU"] else None
        s["wave_wait_any_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        s["valu_issue_frac_of_78.6T"] = (c["SQ_INSTS_VALU"] * 64 / (dur_ms / 1e3) / 7.86432e13
                                         if dur_ms else None)
    s["counters"] = dict(c)
    out[key] = s
json.dump(out, open(f"profiles/{tag}_config_pmc.json", "w"), indent=1)
for k, s in out.items():
    print(k, json.dumps({a: (round(b, 4) if isinstance(b, float) else b)
                         for a, b in s.items() if a != "counters"}))
