"""Summarise a tools/profile_events.sh run (gpurun_out/ev_<probe>_<pass>/) into
profiles/<tag>_event_kernels.json: per probe the measured launch's duration, activations,
instruction mix per activation, LDS bank-conflict ratio, wave wait fractions, HBM bytes
(FETCH_SIZE x 64 B-units x2 gfx950 correction, WRITE_SIZE) and L2 hit rate.

Usage: python tools/summarize_events.py <tag>
"""
import collections
import csv
import glob
import json
import os
import sys

tag = sys.argv[1]
out = {}
for trace_dir in sorted(glob.glob("gpurun_out/ev_*_trace")):
    probe = os.path.basename(trace_dir)[3:-6]
    log = open(f"gpurun_out/ev_{probe}_trace.log").read().strip().splitlines()
    info = json.loads([ln for ln in log if ln.startswith("{")][-1])
    name = info["kernel"].split("<")[0].split(" ")[0]
    rows = [r for r in csv.DictReader(open(f"{trace_dir}/run_kernel_trace.csv"))
            if name in r["Kernel_Name"]]
    last = rows[-1]  # the measured launch follows the warm-up
    dur_ns = int(last["End_Timestamp"]) - int(last["Start_Timestamp"])
    acts = info["activations"]
    c = {}
    for p in ("sq", "fetch", "write", "tcc"):
        f = f"gpurun_out/ev_{probe}_{p}/run_counter_collection.csv"
        if not os.path.exists(f):
            continue
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if name in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        c.update(per[max(per)])
    s = dict(info)
    s["trace_duration_ms"] = dur_ns / 1e6
    s["activations_per_s"] = acts / (dur_ns / 1e9)
    if "SQ_INSTS_VALU" in c:
        s["valu_lane_instr_per_activation"] = c["SQ_INSTS_VALU"] * 64 / acts
        # SALU issues once per wave instruction: a wave count, not scaled by 64 like lane-ops
        s["salu_wave_instr_per_activation"] = c["SQ_INSTS_SALU"] / acts
        s["lds_instr_per_activation"] = c["SQ_INSTS_LDS"] * 64 / acts
        s["lds_bank_conflict_cycles_per_lds_instr"] = (
            c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"] if c["SQ_INSTS_LDS"] else 0.0)
        s["wave_wait_any_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        s["wave_wait_inst_frac"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
        s["valu_issue_frac_of_78.6T"] = c["SQ_INSTS_VALU"] * 64 / (dur_ns / 1e9) / 7.86432e13
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rd = c["FETCH_SIZE"] * 1024 * 2
        wr = c["WRITE_SIZE"] * 1024
        s["hbm_read_bytes (FETCH_SIZE x1024 x2)"] = rd
        s["hbm_write_bytes (WRITE_SIZE x1024)"] = wr
        s["hbm_bytes_per_activation"] = (rd + wr) / acts
        s["hbm_GB_per_s"] = (rd + wr) / (dur_ns / 1e9) / 1e9
    if "TCC_HIT_sum" in c:
        s["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    s["counters"] = c
    out[probe] = s
json.dump(out, open(f"profiles/{tag}_event_kernels.json", "w"), indent=1)
for p, s in out.items():
    print(p, json.dumps({k: (round(v, 4) if isinstance(v, float) else v)
                         for k, v in s.items() if k != "counters"}))
