#!/bin/bash
# A/B of environment switches on the vote bench: tools/ab_env.sh "NAME=VAL" "" ...  ("" = defaults)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
i=0
for rep in 1 2; do
  for e in "$@"; do
    i=$((i+1))
    env $e PVVOTE_BENCH_NOCHECK=1 timeout -k 10 200 python bench.py --steps ${STEPS:-50} --warmup 10 --inflight ${INFLIGHT:-2} --skip-cpu --skip-e2e --skip-u1 > gpurun_out/abenv_$i.log 2>&1 || exit $?
    python - "$e" "gpurun_out/abenv_$i.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][-1]
d = json.loads(l)
print(repr(sys.argv[1]), "img/s", d["value"], "vote_us", round(d["roofline_vote_count"]["avg_kernel_ms"] * 1000, 2), "lat_us", round(d["latency_ms_per_image"] * 1000, 1))
PY
  done
done
