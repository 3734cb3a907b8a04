"""gpurun_out/<tag>/ (scripts/prof_camera_valu.sh) -> profiles/<name>_camera_valu.json: per-call averages of the
camera kernel's SQ counters, split into re-render and reuse calls (bimodal in SQ_INSTS_VALU), and the VALU issue
fraction of the re-render calls.

VALU issue fraction = SQ_INSTS_VALU x 2 cycles / (1 024 SIMDs x call cycles at 2.4 GHz): a wave64 fp32 VALU
instruction occupies its SIMD for 2 cycles (MI355X_MICROARCH.md, per-instruction table), so this is the share
of the chip's VALU issue slots the call used (transcendentals, which take longer, make it a lower bound).
SQ_WAVE_CYCLES / SQ_ACTIVE_INST_VALU / SQ_WAIT_ANY / SQ_BUSY_CYCLES count quad-cycles.

    python scripts/summarize_camera_valu.py <tag> <name>
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS, CLOCK_GHZ = 1024, 2.4


def main(tag, name):
    prof = os.path.join(ROOT, "gpurun_out", tag)
    # per-dispatch durations of the camera kernel
    durs = []
    for f in glob.glob(os.path.join(prof, "trace", "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            if "camera_kernel" in r["Kernel_Name"]:
                durs.append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    durs.sort()
    cut = (durs[0] + durs[-1]) / 2
    t_render = [d for d in durs if d > cut]
    t_reuse = [d for d in durs if d <= cut]
    # per-dispatch counters
    disp = collections.defaultdict(dict)
    kname = None
    for f in glob.glob(os.path.join(prof, "pmc*", "pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "camera_kernel" in r["Kernel_Name"]:
                kname = r["Kernel_Name"]
                d = disp[(f, r["Dispatch_Id"])]
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    calls = list(disp.values())
    v = sorted(c["SQ_INSTS_VALU"] for c in calls)
    vcut = (v[0] + v[-1]) / 2
    out = {"kernel": kname, "note": "scripts/bench_camera.py --steps 8 at 65 536 envs, obstacle tracks; calls alternate "
                                    "re-render / reuse (update_period 0.04 s = 2 steps)"}
    for label, sel, ts in (("render", lambda c: c["SQ_INSTS_VALU"] > vcut, t_render),
                           ("reuse", lambda c: c["SQ_INSTS_VALU"] <= vcut, t_reuse)):
        cs = [c for c in calls if sel(c)]
        m = {k: sum(c[k] for c in cs) / len(cs) for k in cs[0]}
        ns = sum(ts) / len(ts)
        cyc = ns * CLOCK_GHZ
        out[label] = {
            "calls_counted": len(cs), "trace_avg_ns": ns, "counters_per_call": m,
            "valu_issue_fraction": m["SQ_INSTS_VALU"] * 2 / (SIMDS * cyc),
            "waves_per_simd_avg": 4 * m["SQ_WAVE_CYCLES"] / (SIMDS * cyc),
            "valu_active_frac_of_wave_cycles": m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"],
            "wait_any_frac_of_wave_cycles": m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"],
            "valu_insts_per_wave": m["SQ_INSTS_VALU"] / m["SQ_WAVES"],
        }
    json.dump(out, open(os.path.join(ROOT, "profiles", f"{name}_camera_valu.json"), "w"), indent=1)
    for label in ("render", "reuse"):
        o = out[label]
        print(label, round(o["trace_avg_ns"] / 1e6, 3), "ms", {k: round(o[k], 3) for k in o if k.endswith(("fraction", "frac_of_wave_cycles", "simd_avg"))})


if __name__ == "__main__":
    main(*sys.argv[1:3])
