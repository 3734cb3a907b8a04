"""Summarise rocprofv3 PMC passes of scripts/time_mlp.py into one JSON per kernel and mini-batch size.

    python scripts/summarize_mlp_pmc.py OUT.json --rows 24576 393216 --trace DIR --pmc DIR [DIR ...] [--label NAME]

time_mlp.py runs each size in turn, so each kernel's dispatches split evenly, in dispatch order, into one group per
entry of --rows.  Per group: the counters' means per dispatch, the wave-cycle split (SQ_ACTIVE_INST_ANY / SQ_WAIT_ANY /
SQ_WAIT_INST_ANY of SQ_WAVE_CYCLES; all quad-cycle counts), LDS bank-conflict cycles per wave, the MFMA count and
its executed flops (16x16x4 f32 = 2 048 flop, 32 cycles each), and from the --trace kernel trace (a run without
counters) the mean duration and the fraction of the fp32 MFMA peak (157.3 TFLOP/s = 1 024 SIMDs x 2.4 GHz x 64)."""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os

PEAK_TFLOPS = 157.3
FLOP_PER_MFMA = 2048


def split(seq, n):
    k = len(seq) // n
    return [seq[i * k:(i + 1) * k] for i in range(n)]


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--rows", type=int, nargs="+", required=True)
    ap.add_argument("--trace", required=True)
    ap.add_argument("--pmc", nargs="+", required=True)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    ngroups = len(a.rows)

    durs = collections.defaultdict(list)
    for f in glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "mlp_" in r["Kernel_Name"]:
                durs[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))

    counters = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in a.pmc:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(dict)  # (kernel, dispatch) -> counter -> value
            for r in csv.DictReader(open(f)):
                if "mlp_" in r["Kernel_Name"]:
                    key = (short(r["Kernel_Name"]), int(r["Dispatch_Id"]))
                    per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            bykern = collections.defaultdict(list)
            for (k, disp), cs in sorted(per.items(), key=lambda kv: kv[0][1]):
                bykern[k].append(cs)
            for k, lst in bykern.items():
                for gi, grp in enumerate(split(lst, ngroups)):
                    for cs in grp:
                        for c, v in cs.items():
                            counters[(k, gi)][c].append(v)

    out = {"source": {"trace": a.trace, "pmc": a.pmc, "label": a.label}, "kernels": {}}
    for (k, gi), cs in sorted(counters.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        rec = {"rows": a.rows[gi], "dispatches": len(next(iter(cs.values()))), "counters": m}
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            rec["wave_cycle_split"] = {c: m[c] / wc for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")
                                       if c in m}
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_WAVES" in m:
            rec["lds_bank_conflict_cycles_per_wave"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_WAVES"]
        if "SQ_INSTS_MFMA" in m:
            rec["mfma_flop"] = m["SQ_INSTS_MFMA"] * FLOP_PER_MFMA
        ds = durs.get(k)
        if ds:
            g = split(ds, ngroups)[gi]
            us = sum(g) / len(g) / 1e3
            rec["trace_us"] = us
            if "mfma_flop" in rec:
                rec["frac_fp32_peak_executed"] = rec["mfma_flop"] / (us * 1e-6) / 1e12 / PEAK_TFLOPS
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                rec["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (us * 1e-6 * 2.4e9 * 1024)
        out["kernels"].setdefault(k, []).append(rec)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for k, recs in out["kernels"].items():
        for r in recs:
            print(k, r["rows"], {x: round(r[x], 3) for x in ("trace_us", "frac_fp32_peak_executed", "mfma_busy_frac",
                                                              "lds_bank_conflict_cycles_per_wave") if x in r},
                  {c: round(v, 3) for c, v in r.get("wave_cycle_split", {}).items()})


if __name__ == "__main__":
    main()
