#!/usr/bin/env python3
"""Per-launch PMC means of one kernel from a profiles/scripts/r06_pmc.sh run, with derived ratios:
    python profiles/scripts/pmc_table.py gpurun_out/pmc_TAG KERNEL_SUBSTRING"""
import collections, csv, glob, os, sys

d, kern = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
c = {k: sum(v) / len(v) for k, v in acc.items()}
dur = []
for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv"))):
    if kern in r["Kernel_Name"]:
        dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
dur.sort()
t = dur[len(dur) // 2] if dur else float("nan")
for k in sorted(c):
    print(f"| {k} | {c[k]:.4g} |")
print(f"| median launch (trace) | {t * 1e3:.4f} ms over {len(dur)} launches |")
if "GRBM_GUI_ACTIVE" in c:
    clk = c["GRBM_GUI_ACTIVE"] / t / 1e9
    print(f"| clock GRBM_GUI_ACTIVE / duration | {clk:.3f} GHz (as counted; XCD-summed counters divide by 8: {clk / 8:.3f}) |")
if "SQ_WAVE_CYCLES" in c:
    print(f"| SQ_WAIT_ANY / SQ_WAVE_CYCLES | {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f} |")
    print(f"| SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES | {c['SQ_ACTIVE_INST_ANY'] / c['SQ_WAVE_CYCLES']:.3f} |")
if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
    simd_cycles = c["GRBM_GUI_ACTIVE"] / 8 * 1024  # per-XCD count x 1024 SIMDs
    print(f"| MFMA busy / (1024 SIMD x cycles) | {c['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cycles:.3f} |")
