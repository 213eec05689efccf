#!/bin/bash
# k_vote_count variants: per-wave trace (tools/vote_trace.py) and the quick
# bench (vote kernel us, images/s) per library in variants/.  VARIANTS="a b"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in $VARIANTS; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 120 python tools/vote_trace.py > gpurun_out/vtrace_$v.log 2>&1 || exit $?
  echo "== $v"; grep -v amdgpu.ids gpurun_out/vtrace_$v.log | head -5
  for rep in 1 2; do
    PVVOTE_LIB=variants/$v.so timeout -k 10 200 python bench.py --steps 200 --warmup 10 --skip-cpu --skip-e2e --skip-u1 > gpurun_out/vcb_$v.$rep.log 2>&1 || exit $?
    python3 - $v $rep <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/vcb_{sys.argv[1]}.{sys.argv[2]}.log") if x.startswith("{")][-1]
d = json.loads(l)
k = d["roofline_vote_count"]
print(sys.argv[1], sys.argv[2], "img/s", d["value"], "vote_us", round(k["avg_kernel_ms"] * 1000, 2), "lat_us", round(d["latency_ms_per_image"] * 1000, 1))
PY
  done
done
