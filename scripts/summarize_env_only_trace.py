"""The env-only chain's timeline from a rocprofv3 kernel trace of `bench.py --legs policy` (historically scripts/gpu_r4z.sh; today scripts/gpu.sh TAG 'trace 300 cd /tmp && rocprofv3 --kernel-trace ... -- python3 $R/bench.py --legs policy'):
per rollout step the fused fp32 actor (policy_f32_kernel, actor only) and the env step (step_kernel), back to back
in one hipGraph.  Prints and writes the per-step stamps (median actor / step / gap µs, the excerpt of one graph
replay) — the measured form of DESIGN §4e''s argument that the chain is the actor's MFMA time plus the step.

    python scripts/summarize_env_only_trace.py gpurun_out/r4z/envonly profiles/round04_env_only_timeline.json
"""
import csv
import glob
import json
import statistics as st
import sys


def main(d, out):
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    steps = []
    for i in range(1, len(rows)):
        s0, e0, n0 = rows[i - 1]
        s1, e1, n1 = rows[i]
        if "policy_f32_kernel" in n0 and "step_kernel" in n1:
            steps.append({"actor_start": s0, "actor_us": (e0 - s0) / 1e3, "gap_us": (s1 - e0) / 1e3,
                          "step_us": (e1 - s1) / 1e3, "step_end": e1, "actor": n0[:60], "step": n1[:60]})
    # actor-only launches are the ~80 us ones (the actor + critic fp32 leg runs ~150 us)
    a_only = [x for x in steps if x["actor_us"] < 120.0]
    for k in range(1, len(a_only)):
        a_only[k - 1]["to_next_actor_us"] = (a_only[k]["actor_start"] - a_only[k - 1]["step_end"]) / 1e3
    per = [x["actor_us"] + x["gap_us"] + x["step_us"] + x.get("to_next_actor_us", 0.0) for x in a_only[:-1]]
    res = {
        "source": d, "pairs": len(a_only),
        "median_actor_us": st.median(x["actor_us"] for x in a_only),
        "median_actor_to_step_gap_us": st.median(x["gap_us"] for x in a_only),
        "median_step_us": st.median(x["step_us"] for x in a_only),
        "median_step_to_next_actor_gap_us": st.median(x["to_next_actor_us"] for x in a_only[:-1]),
        "median_per_env_step_us": st.median(per),
        "env_steps_per_s_from_stamps": 65536 / (st.median(per) * 1e-6),
        "excerpt": [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in x.items()} for x in a_only[:8]],
    }
    res["actor_fraction"] = res["median_actor_us"] / res["median_per_env_step_us"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "excerpt"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
