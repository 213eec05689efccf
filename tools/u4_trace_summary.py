"""The launches bench.py's U4 line (roofline_evd) times, read from rocprofv3's
kernel trace of the same command: every k_evd_with_mean dispatch of a
9-keypoint batch-1 call (grid 9 x 256: measure_u4's calls) and the
k_vote_mfma dispatch before it on the same queue (the vote over the 16 x 256
hypotheses); the last `samples` of them against the line's medians.
    python tools/u4_trace_summary.py <kernel_trace.csv> <bench line .json> [out.json]"""
import csv
import json
import sys

import numpy as np

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
line = json.loads(open(sys.argv[2]).read())
u4 = line["roofline_evd"]
last_vote = {}
pairs = []
for r in rows:
    name, q = r["Kernel_Name"], r["Queue_Id"]
    if "k_vote_mfma" in name:
        last_vote[q] = r
    elif "k_evd_with_mean" in name and int(r["Grid_Size_X"]) == 9 * 256 and int(r["Grid_Size_Y"]) == 1 and q in last_vote:
        v = last_vote[q]
        pairs.append(((int(v["End_Timestamp"]) - int(v["Start_Timestamp"])) / 1e3,
                      (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
n = int(u4["samples"])
d = np.array(pairs[-n:])
out = {
    "source": "rocprofv3 --kernel-trace of `python3 bench.py --gpus 1 --steps 20 --warmup 5` (tools/prof_bench.sh)",
    "u4_calls_found": len(pairs), "timed_calls": n,
    "vote_median_us": round(float(np.median(d[:, 0])), 3), "vote_mean_us": round(float(d[:, 0].mean()), 3),
    "evd_reduce_median_us": round(float(np.median(d[:, 1])), 3),
    "bench_vote_avg_kernel_ms_same_run": u4["avg_kernel_ms"], "bench_frac_same_run": u4["frac"],
}
out["bench_vs_trace_vote"] = round(u4["avg_kernel_ms"] * 1e3 / out["vote_median_us"], 4)
print(json.dumps(out, indent=1))
if len(sys.argv) > 3:
    json.dump(out, open(sys.argv[3], "w"), indent=1)
