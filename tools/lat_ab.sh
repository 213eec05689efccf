#!/bin/bash
# A/B of library variants (variants/*.so) on the sequential latency graph and
# the compaction's per-call events (bench --skip-cpu ...); each run time-limited.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    PVVOTE_LIB=variants/$v.so timeout -k 10 120 python3 tools/lat_trace.py 20 > gpurun_out/lab_$v.$rep.log 2>&1 || exit $?
    PVVOTE_LIB=variants/$v.so timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --skip-cpu --skip-e2e --skip-u1 --skip-config3 > gpurun_out/labb_$v.$rep.log 2>&1 || exit $?
    python3 - "$v" "$rep" <<'PY'
import json, sys
v, rep = sys.argv[1:]
lat = [x for x in open(f"gpurun_out/lab_{v}.{rep}.log") if x.startswith("latency")][-1].split()[-1]
d = json.loads([x for x in open(f"gpurun_out/labb_{v}.{rep}.log") if x.startswith("{")][-1])
print(v, rep, "seq_lat_us", lat, "img/s", d["value"], "compact_us", round(d["roofline_compaction"]["avg_kernel_ms"] * 1000, 2),
      "u3", d["roofline_compaction"]["frac"], "vote_us", round(d["roofline_vote_count"]["avg_kernel_ms"] * 1000, 2))
PY
  done
done
