#!/bin/bash
# U1 variants: GPU parity tests on each variant library, then rocprof kernel
# times of k_vote_bytes (tools/u1_probe.py).  VARIANTS="name[:ENV=VAL] ..."
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for spec in $VARIANTS; do
  v=${spec%%:*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*:}
  tag=$(echo "$spec" | tr ':=' '__')
  env $envs PVVOTE_LIB=variants/$v.so timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/var_tests_$tag.log 2>&1 || { echo "tests failed: $spec"; tail -30 gpurun_out/var_tests_$tag.log; exit 1; }
  echo "$spec: $(tail -1 gpurun_out/var_tests_$tag.log)"
  env $envs PVVOTE_LIB=variants/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/var_$tag" -o u1 -- python3 tools/u1_probe.py > gpurun_out/var_$tag.log 2>&1 || exit $?
  python3 - $tag <<'PY'
import csv, sys
for r in csv.DictReader(open(f"gpurun_out/var_{sys.argv[1]}/u1_kernel_stats.csv")):
    if "vote_bytes" in r["Name"]:
        print(sys.argv[1], r["Name"][:30], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), "us avg", round(float(r["MinNs"]) / 1000, 2), "min")
PY
done
