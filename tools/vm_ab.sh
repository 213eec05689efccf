#!/bin/bash
# A/B of the pipeline's vote variants by environment: GPU parity tests, then
# the quick bench twice per "name:ENV=VAL+ENV=VAL" spec
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for spec in $SPECS; do
  name=${spec%%:*}; envs=""; [ "$spec" != "$name" ] && envs=$(echo ${spec#*:} | tr '+' ' ')
  if [ -z "$NOTEST" ]; then
    env $envs timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/ab_tests_$name.log 2>&1 || { echo "tests failed: $spec"; tail -30 gpurun_out/ab_tests_$name.log; exit 1; }
    echo "$name: $(tail -1 gpurun_out/ab_tests_$name.log)"
  fi
  for rep in 1 2; do
    env $envs timeout -k 10 200 python bench.py --steps 40 --warmup 5 --skip-cpu --skip-e2e --skip-u1 $BENCH_ARGS > gpurun_out/ab_$name.$rep.log 2>&1 || exit $?
    python3 - gpurun_out/ab_$name.$rep.log "$name" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(sys.argv[2], "img/s", d["value"], "vote_us", round(d["roofline_vote_count"]["avg_kernel_ms"] * 1000, 2), "lat_us", round(d["latency_ms_per_image"] * 1000, 1))
PY
  done
done
