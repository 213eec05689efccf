#!/bin/bash
# A/B of library variants (variants/*.so) on the vote bench; each run time-limited.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    PVVOTE_LIB=variants/$v.so timeout -k 10 200 python bench.py --steps 50 --warmup 10 --skip-cpu --skip-e2e --skip-u1 --skip-config3 --skip-u4 --skip-batched > gpurun_out/ab_$v.$rep.log 2>&1 || exit $?
    python - "$v" "$rep" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/ab_{sys.argv[1]}.{sys.argv[2]}.log") if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[1], sys.argv[2], "img/s", d["value"], "vote_us", round(d["roofline_vote_count"]["avg_kernel_ms"] * 1000, 2), "lat_us", round(d["latency_ms_per_image"] * 1000, 1))
PY
  done
done
