#!/usr/bin/env python3
"""Summarise a profiles/scripts/profile.sh run (gpurun_out/prof_TAG) into
profiles/TAG/: the rocprofv3 kernel stats CSV, a per-kernel PMC table, and
pmc.json (HBM bytes per launch of the dominant kernel, read by bench.py).

    python profiles/scripts/summarize.py TAG [KERNEL_SUBSTRING]

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reports half the
bytes of a wide coalesced streaming read on gfx950, so it is doubled;
WRITE_SIZE (KiB) is taken as is.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))


def per_kernel(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        meta[name] = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count",
                                        "Accum_VGPR_Count", "SGPR_Count", "Scratch_Size")}
    return agg, meta


def main():
    tag = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "scan_topk"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    bench = json.load(open(os.path.join(src, "trace_bench.json")))
    counters = {}
    meta = {}
    for p in sorted(os.listdir(src)):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if p.startswith("pmc_") and os.path.exists(f):
            agg, m = per_kernel(f)
            meta.update(m)
            for name, cs in agg.items():
                for c, v in cs.items():
                    counters.setdefault(name, {})[c] = sum(v) / len(v)
    stats = list(csv.DictReader(open(os.path.join(dst, "kernel_stats.csv"))))
    lines = [f"# rocprofv3 summary: {tag}", "",
             f"bench line under `--kernel-trace` (same command): value {bench['value']:.1f} {bench['unit']}, "
             f"config `{bench['config']['workload']}`", "",
             "| kernel | calls | avg µs | share % |", "|---|---|---|---|"]
    for r in stats:
        lines.append(f"| `{r['Name'][:110]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {r['Percentage']} |")
    out = {"tag": tag, "config": bench["config"]["workload"].split(":")[0], "n_gpus": bench["n_gpus"],
           "precision": bench["roofline"].get("precision", "fp32")}
    for name, cs in counters.items():
        if kern not in name:
            continue
        avg_ns = next(float(r["AverageNs"]) for r in stats if r["Name"] == name)
        fetch = cs.get("FETCH_SIZE", 0.0) * 1024 * 2
        write = cs.get("WRITE_SIZE", 0.0) * 1024
        lines += ["", f"## PMC, `{name[:110]}` (mean per launch)", "",
                  f"resources: {json.dumps(meta.get(name, {}))}", "",
                  "| counter | value |", "|---|---|"]
        for c, v in sorted(cs.items()):
            lines.append(f"| {c} | {v:.6g} |")
        clk = cs.get("GRBM_GUI_ACTIVE", 0.0) / 8 / (avg_ns * 1e-9) / 1e9 if "GRBM_GUI_ACTIVE" in cs else None
        lines += ["", f"- HBM read (FETCH_SIZE x2, gfx950 correction): {fetch / 1e9:.4f} GB per launch",
                  f"- HBM write (WRITE_SIZE): {write / 1e9:.6f} GB per launch",
                  f"- HBM traffic / avg duration: {(fetch + write) / (avg_ns * 1e-9) / 1e9:.1f} GB/s"]
        if clk:
            lines.append(f"- effective clock (GRBM_GUI_ACTIVE/8/duration): {clk:.2f} GHz")
        if "TCC_HIT_sum" in cs:
            h, m = cs["TCC_HIT_sum"], cs.get("TCC_MISS_sum", 0.0)
            lines.append(f"- L2 hit rate: {h / max(h + m, 1):.3f}")
        out.update({"kernel": name, "avg_ns": avg_ns, "hbm_read_bytes_per_launch": fetch,
                    "hbm_write_bytes_per_launch": write, "hbm_bytes_per_launch": fetch + write})
    open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
    json.dump(out, open(os.path.join(dst, "pmc.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
