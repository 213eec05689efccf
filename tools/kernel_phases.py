"""Per-kernel durations from a rocprofv3 kernel trace, split into launches that
ran alone on the device (no other kernel's [start, end) overlaps them) and
launches that overlapped others (the bench's in-flight streams).

    python tools/kernel_phases.py <kernel_trace.csv> [out.json]

The bench's per-kernel figures (hipEvents around eager single-stream calls:
k_vote_count's avg_kernel_ms, U1's back-to-back calls) correspond to the
'alone' rows; rocprof's --stats averages mix both kinds."""
import csv
import json
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].split("<")[0]
             .replace("(anonymous namespace)::", "")) for r in rows)
starts = np.array([e[0] for e in ev])
ends = np.array([e[1] for e in ev])
# running maximum of the ends of all earlier-starting launches
prev_end = np.maximum.accumulate(np.concatenate([[0], ends[:-1]]))
alone = np.ones(len(ev), bool)
alone &= prev_end <= starts                       # nothing earlier still running
nxt = np.concatenate([starts[1:], [np.iinfo(np.int64).max]])
alone &= nxt >= ends                              # nothing later starting before it ends
out = {}
for name in sorted({e[2] for e in ev}):
    idx = [i for i, e in enumerate(ev) if e[2] == name]
    d = (ends[idx] - starts[idx]) / 1e3
    a = np.array(alone)[idx]
    rec = {"calls": len(idx), "mean_us_all": round(float(d.mean()), 3)}
    if a.any():
        rec.update(alone_calls=int(a.sum()), alone_mean_us=round(float(d[a].mean()), 3),
                   alone_median_us=round(float(np.median(d[a])), 3))
    if (~a).any():
        rec.update(overlapped_calls=int((~a).sum()), overlapped_mean_us=round(float(d[~a].mean()), 3))
    out[name] = rec
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
for k in ("k_fg_count", "k_compact", "k_hyp_gen", "k_vote_mfma", "k_vote_count", "k_refine_solve", "k_vote_bytes"):
    if k in out:
        print(k, out[k])
