"""One graph-replayed PPO mini-batch step of the update, kernel by kernel, from a rocprofv3 kernel trace
(`rocprofv3 --kernel-trace --output-format csv -- python3 scripts/prof_update.py --envs 4096 --fused --graph`).

A step is the span from one `mlp_bwd` launch to the next; the last update's 20 steps are taken.  Prints JSON: the
median step's kernels in order (duration, gap before it), the sum of kernel time against the step's period (what is
neither kernel is launch gap), and the periods of all steps.

    python scripts/summarize_update_step.py TRACE.csv [> out.json]
"""
import csv
import json
import re
import statistics
import sys


def short(name):
    return re.sub(r"\(.*", "", name).replace("void ", "")


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "mlp_bwd" in r["Kernel_Name"]]
    last = idx[-21:]  # the last update: 20 step spans between 21 backward launches
    steps = []
    for a, b in zip(last, last[1:]):
        t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
        ks, prev = [], None
        for r in rows[a:b]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            ks.append({"kernel": short(r["Kernel_Name"]), "us": (e - s) / 1e3,
                       "gap_before_us": 0.0 if prev is None else (s - prev) / 1e3})
            prev = e
        steps.append({"period_us": (t1 - t0) / 1e3, "kernels": ks})
    periods = [s["period_us"] for s in steps]
    med = sorted(steps, key=lambda s: s["period_us"])[len(steps) // 2]
    mlp = sum(k["us"] for k in med["kernels"] if k["kernel"].startswith("gr::mlp_"))
    ksum = sum(k["us"] for k in med["kernels"])
    out = {"trace": path, "steps": len(steps), "median_step": med, "kernel_sum_us": ksum,
           "mlp_kernels_us": mlp, "other_kernels_us": ksum - mlp, "gaps_us": med["period_us"] - ksum,
           "periods_us": periods, "period_median_us": statistics.median(periods)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
