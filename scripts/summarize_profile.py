"""Turn a gpurun_out/prof_<tag>/ directory (scripts/gpu_profile.sh) into the
committed evidence under profiles/:

  profiles/<name>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as produced)
  profiles/<name>_pmc.json           per-launch PMC averages of the fused step kernel, with the
                                     MI355X_MICROARCH.md corrections (FETCH_SIZE x2 on gfx950,
                                     SQ_* cycle counters in quad-cycles) and derived ratios
  profiles/pmc_traffic.json          HBM bytes per launch read by bench.py's roofline.traffic

    python scripts/summarize_profile.py <tag> <name> [--num-envs 65536] [--gates 8]
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "gr::step_kernel<true, false, 8, 1>"  # <USE_LDS, OBST, MAXG, LEAN>; --obstacles: <false, true, 0, 1>


def pmc_means(prof):
    acc = collections.defaultdict(list)
    dur = collections.defaultdict(list)
    meta = {}
    for f in glob.glob(os.path.join(prof, "pmc_*", "pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if KERNEL not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[r["Counter_Name"]].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
            meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size",
                                      "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count")}
    mean = {k: sum(v) / len(v) for k, v in acc.items()}
    mean.update({f"duration_ns[{k}]": sum(v) / len(v) for k, v in dur.items()})
    return mean, {k: len(v) for k, v in acc.items()}, meta


def main():
    p = argparse.ArgumentParser()
    p.add_argument("tag")
    p.add_argument("name")
    p.add_argument("--num-envs", type=int, default=65536)
    p.add_argument("--gates", type=int, default=8)
    p.add_argument("--read-bytes", type=int, default=256, help="algorithmic bytes read per env-step")
    p.add_argument("--write-bytes", type=int, default=290, help="algorithmic bytes written per env-step")
    p.add_argument("--obstacles", action="store_true", help="obstacle tracks (kernel <false, true>, +16 B r/w hint)")
    a = p.parse_args()
    global KERNEL
    if a.obstacles:
        KERNEL = "gr::step_kernel<false, true, 0, 1>"
        a.read_bytes += 16
        a.write_bytes += 16
    prof = os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}")
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(prof, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, f"{a.name}_kernel_stats.csv"))
    avg_ns = None
    for r in csv.DictReader(open(stats)):
        if KERNEL in r["Name"]:
            avg_ns = float(r["AverageNs"])
    m, counts, meta = pmc_means(prof)
    n = a.num_envs
    d = {"kernel": f"{KERNEL} (fused step)", "num_envs": n, "gates": a.gates, "obstacles": int(a.obstacles),
         "launches_per_counter": counts, "dispatch": meta, "raw_means": m, "trace_avg_ns": avg_ns}
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        rd = m["FETCH_SIZE"] * 1024 * 2  # KB; gfx950 reports half of a coalesced streaming read
        wr = m["WRITE_SIZE"] * 1024
        d["hbm_bytes_per_launch"] = {"read": rd, "write": wr, "total": rd + wr}
        alg = (a.read_bytes + a.write_bytes) * n
        d["algorithmic_bytes_per_launch"] = alg
        d["traffic_over_algorithmic"] = (rd + wr) / alg
        tpath = os.path.join(out, "pmc_traffic.json")
        key = "obstacles" if a.obstacles else "gates_only"
        allt = json.load(open(tpath)) if os.path.exists(tpath) else {}
        if "bytes_per_launch" in allt:  # old single-entry format
            allt = {}
        allt[key] = {"num_envs": n, "gates": a.gates, "obstacles": int(a.obstacles), "bytes_per_launch": rd + wr,
                     "read": rd, "write": wr, "source": f"profiles/{a.name}_pmc.json"}
        json.dump(allt, open(tpath, "w"), indent=1)
    if "SQ_WAVES" in m:
        waves = m["SQ_WAVES"]
        per = {k: m[k] / waves for k in m if k.startswith("SQ_") and k != "SQ_WAVES"}
        d["per_wave"] = per
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            d["wave_cycles_per_wave"] = wc * 4 / waves  # quad-cycles
            for k in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY"):
                if k in m:
                    d[f"{k}_frac_of_wave_cycles"] = m[k] / wc
    # GRBM_GUI_ACTIVE / 8 / wall is not used as a clock estimate: the guide notes the quotient reads
    # high on dispatches shorter than ~0.3 ms (this kernel runs ~20 us).
    json.dump(d, open(os.path.join(out, f"{a.name}_pmc.json"), "w"), indent=1)
    print(json.dumps({k: d[k] for k in d if k not in ("raw_means", "per_wave", "launches_per_counter")}, indent=1))


if __name__ == "__main__":
    main()
