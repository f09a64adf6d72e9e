"""Summarise a tools/profile.sh run (gpurun_out/prof_*) into profiles/<tag>_*.

Usage: python tools/summarize_profile.py <tag> [episodes_per_launch]
"""
import collections
import csv
import json
import shutil
import sys

import re

tag = sys.argv[1]
eps = int(sys.argv[2]) if len(sys.argv) > 2 else 5242880
K = "k_run_episodes"
# the headline sweep's launches: the sapirshtein-2016-sm1 specialisation on the keyed
# stream (bench.py's abstract-gamma column after the timed sweep runs the generic POL = -1
# instantiation and is left out); bench.py asks for no records, so the summary-only
# specialisation (REC = 0) runs. At gamma = .5 (d = 2, dmax = delta) it defers its races and
# an eager second pass (ListSource) reruns the few episodes a race went otherwise in: a
# point's launch is both kernels, so their times and counters are summed per main dispatch
# (the template's trailing arguments: REC, ARR, TT, LZ; any of them may be printed)
HEADLINE = re.compile(r"k_run_episodes<0, (cpr::)?(Seed|List)Source, 3(, 0(, -?\d+)*)?>")
SECOND = re.compile(r"k_run_episodes<0, (cpr::)?ListSource")


def is_headline(name):
    return HEADLINE.search(name) is not None


def agg(path):
    a = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(path)):
        if K in r["Kernel_Name"] and not is_headline(r["Kernel_Name"]):
            continue
        k = K if is_headline(r["Kernel_Name"]) else r["Kernel_Name"].split("(")[0]
        a[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if not SECOND.search(r["Kernel_Name"]):  # per main dispatch (the second pass adds in)
            n[(k, r["Counter_Name"])] += 1
    return a, n


res = {}
for p in ["prof_pmc_sq", "prof_pmc_fetch", "prof_pmc_write"]:
    a, n = agg(f"gpurun_out/{p}/run_counter_collection.csv")
    for k, v in a.items():
        for c, x in v.items():
            res.setdefault(k, {})[c] = {"sum": x, "dispatches": n[(k, c)], "per_dispatch": x / n[(k, c)]}
tr = list(csv.DictReader(open("gpurun_out/prof_trace/run_kernel_trace.csv")))
main = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr
        if is_headline(r["Kernel_Name"]) and not SECOND.search(r["Kernel_Name"])]
second = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr
          if SECOND.search(r["Kernel_Name"])]
# a point = its main dispatch + its second pass (if any): total time per main dispatch
durs = [sum(main + second) / len(main)] * len(main)
acts = eps * 2017
r = res[K]
s = {
    "kernel": K,
    "dispatches": len(durs),
    "mean_duration_ms": sum(durs) / len(durs) / 1e6,
    "second_pass_dispatches": len(second),
    "second_pass_mean_duration_ms": sum(second) / len(second) / 1e6 if second else 0.0,
    "episodes_per_dispatch": eps,
    "activations_per_dispatch": acts,
    "activations_per_s_in_kernel": acts / (sum(durs) / len(durs) / 1e9),
    # per activation, in the lane's view: every wave instruction (VALU or SALU) is issued
    # once for the 64 lanes' 64 activations, so count x 64 / activations = instructions one
    # lane's activation takes (the figure the 40-op cost model prices); up to round 5 these
    # keys were named *_wave_instr_per_activation
    "valu_lane_instr_per_activation": r["SQ_INSTS_VALU"]["per_dispatch"] * 64 / acts,
    "salu_lane_instr_per_activation": r["SQ_INSTS_SALU"]["per_dispatch"] * 64 / acts,
    "vmem_rd_lane_instr_per_activation": r["SQ_INSTS_VMEM_RD"]["per_dispatch"] * 64 / acts,
    "vmem_wr_lane_instr_per_activation": r["SQ_INSTS_VMEM_WR"]["per_dispatch"] * 64 / acts,
    "valu_lane_ops_per_s": r["SQ_INSTS_VALU"]["per_dispatch"] * 64 / (sum(durs) / len(durs) / 1e9),
    "hbm_read_bytes_per_dispatch (FETCH_SIZE x1024 x2, gfx950 correction)": r["FETCH_SIZE"]["per_dispatch"] * 1024 * 2,
    "hbm_write_bytes_per_dispatch (WRITE_SIZE x1024)": r["WRITE_SIZE"]["per_dispatch"] * 1024,
    "counters": r,
}
# the LDS pass (tools/profile.sh pmc_lds): LDS instructions and bank-conflict cycles of the
# same launches, in a pass of its own
try:
    la, ln = agg("gpurun_out/prof_pmc_lds/run_counter_collection.csv")
    lk = la.get(K, {})
    if "SQ_INSTS_LDS" in lk:
        lds = lk["SQ_INSTS_LDS"] / ln[(K, "SQ_INSTS_LDS")]
        conf = lk.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1, ln.get((K, "SQ_LDS_BANK_CONFLICT"), 1))
        s["lds_lane_instr_per_activation"] = lds * 64 / acts
        s["lds_bank_conflict_cycles_per_lds_instr"] = conf / lds if lds else 0.0
        s["lds_counters"] = {c: {"sum": x, "dispatches": ln[(K, c)]} for c, x in lk.items()}
except FileNotFoundError:
    pass
s["valu_issue_frac_of_78.6T"] = s["valu_lane_ops_per_s"] / 7.86432e13
s["hbm_bytes_per_activation"] = (s["hbm_read_bytes_per_dispatch (FETCH_SIZE x1024 x2, gfx950 correction)"]
                                 + s["hbm_write_bytes_per_dispatch (WRITE_SIZE x1024)"]) / acts
json.dump(s, open(f"profiles/{tag}_pmc_summary.json", "w"), indent=1)
shutil.copy("gpurun_out/prof_trace/run_kernel_stats.csv", f"profiles/{tag}_kernel_stats.csv")
shutil.copy("gpurun_out/bench.log", f"profiles/{tag}_bench.jsonl") if False else None
print(json.dumps({k: v for k, v in s.items() if k not in ("counters", "lds_counters")}, indent=1))
