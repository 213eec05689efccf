"""The launches bench.py's U1 roofline times, read from rocprofv3's kernel
trace of the same command: the last U1_TIMED x 100 k_vote_bytes launches
(measure_u1's timed replays), their mean / median duration and the period
start-to-end, beside the mean over every launch of the run.
    python tools/u1_trace_summary.py <kernel_trace.csv> <bench line .json> [out.json]"""
import csv
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from bench import U1_TIMED  # noqa: E402

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
            if r["Kernel_Name"].startswith("k_vote_bytes"))
n = 100 * U1_TIMED
d = np.array([(e - s) / 1e3 for s, e in ev])
t = ev[-n:]
line = json.loads(open(sys.argv[2]).read())
out = {
    "source": "rocprofv3 --kernel-trace of `python3 bench.py --gpus 1 --steps 20 --warmup 5` (tools/prof_bench.sh)",
    "launches_all": len(ev), "mean_us_all": round(float(d.mean()), 3),
    "timed_launches": n, "timed_mean_us": round(float(d[-n:].mean()), 3),
    "timed_median_us": round(float(np.median(d[-n:])), 3),
    "timed_period_us": round((t[-1][1] - t[0][0]) / 1e3 / n, 3),
    "bench_avg_kernel_ms_same_run": line["roofline"]["avg_kernel_ms"],
    "bench_frac_same_run": line["roofline"]["frac"],
}
out["bench_vs_trace_period"] = round(out["bench_avg_kernel_ms_same_run"] * 1e3 / out["timed_period_us"], 4)
print(json.dumps(out, indent=1))
if len(sys.argv) > 3:
    json.dump(out, open(sys.argv[3], "w"), indent=1)
