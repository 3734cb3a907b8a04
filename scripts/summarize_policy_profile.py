"""gpurun_out/<tag>/ (scripts/prof_policy.sh) -> profiles/<name>_kernel_stats.csv (rocprofv3 --stats summary)
and profiles/<name>_pmc.json (per-launch SQ counter averages of gr::policy_kernel, per-wave figures, the MFMA
busy fraction).  SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES cycles
(MI355X_MICROARCH.md constants table).

    python scripts/summarize_policy_profile.py <tag> <name> [kernel substring: policy_kernel | policy_f32_kernel]
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag, name, kern="policy_kernel"):
    prof = os.path.join(ROOT, "gpurun_out", tag)
    shutil.copy(os.path.join(prof, "trace", "trace_kernel_stats.csv"),
                os.path.join(ROOT, "profiles", f"{name}_kernel_stats.csv"))
    acc = collections.defaultdict(list)
    kname = None
    for f in glob.glob(os.path.join(prof, "pmc*", "pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                kname = r["Kernel_Name"]
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in acc.items()}
    waves = m.get("SQ_WAVES", 1.0)
    stats = {}
    for r in csv.DictReader(open(os.path.join(prof, "trace", "trace_kernel_stats.csv"))):
        if kern in r["Name"]:
            stats = {"calls": int(r["Calls"]), "average_ns": float(r["AverageNs"])}
    out = {"kernel": kname, "launch_stats": stats, "per_launch": m,
           "per_wave": {k: v / waves for k, v in m.items() if k != "SQ_WAVES"},
           "note": "scripts/bench_policy.py at 65536 envs (actor + critic 16-256-256-out, "
                   + ("fp32 operands, MFMA 16x16x4 f32)" if "f32" in kern else "bf16 MFMA)")}
    if stats:
        flops = 2 * 65536 * 2 * (16 * 256 + 256 * 256 + 256 * 4)
        peak = 157.3e12 if "f32" in kern else 2.5e15
        out["useful_TFLOPs"] = flops / (stats["average_ns"] * 1e-9) / 1e12
        out["frac_of_dense_mfma_peak"] = flops / (stats["average_ns"] * 1e-9) / peak
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_WAVE_CYCLES" in m:
        # two waves share a SIMD: MFMA-busy cycles of both over the wave lifetime (quad-cycles x 4)
        out["mfma_busy_fraction_of_wave_lifetime_per_simd"] = 2 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * m["SQ_WAVE_CYCLES"])
    json.dump(out, open(os.path.join(ROOT, "profiles", f"{name}_pmc.json"), "w"), indent=1)
    print(json.dumps(out["launch_stats"]), out.get("mfma_busy_fraction_of_wave_lifetime_per_simd"))


if __name__ == "__main__":
    main(*sys.argv[1:4])
