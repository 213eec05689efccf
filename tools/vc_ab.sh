#!/bin/bash
# k_vote_count A/B: GPU tests per variant, then the quick bench twice per
# "variant[:ENV=VAL]" spec (images/s, vote kernel us, latency).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for spec in $VARIANTS; do
  v=${spec%%:*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*:}
  tag=$(echo "$spec" | tr ':=' '__')
  env $envs PVVOTE_LIB=variants/$v.so timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/vcab_tests_$tag.log 2>&1 || { echo "tests failed: $spec"; tail -30 gpurun_out/vcab_tests_$tag.log; exit 1; }
  echo "$spec: $(tail -1 gpurun_out/vcab_tests_$tag.log)"
  for rep in 1 2; do
    env $envs PVVOTE_LIB=variants/$v.so timeout -k 10 200 python bench.py --steps 200 --warmup 10 --skip-cpu --skip-e2e --skip-u1 > gpurun_out/vcab_$tag.$rep.log 2>&1 || exit $?
    python3 - gpurun_out/vcab_$tag.$rep.log "$spec" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(sys.argv[2], "img/s", d["value"], "vote_us", round(d["roofline_vote_count"]["avg_kernel_ms"] * 1000, 2), "lat_us", round(d["latency_ms_per_image"] * 1000, 1))
PY
  done
done
