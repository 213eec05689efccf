#!/bin/bash
# U1 A/B: parity tests of the byte kernel, then per-wave traces and rocprof
# kernel times of k_vote_bytes under each PVVOTE_BYTES_XCD setting.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/u1ab_tests.log 2>&1 || { tail -30 gpurun_out/u1ab_tests.log; exit 1; }
tail -1 gpurun_out/u1ab_tests.log
for x in ${XCDS:-0 1}; do
  PVVOTE_BYTES_XCD=$x PVVOTE_LIB=variants/u1trace.so timeout -k 10 120 python tools/bytes_trace.py > gpurun_out/btrace_$x.log 2>&1 || exit $?
  echo "== trace xcd=$x"; grep -v amdgpu.ids gpurun_out/btrace_$x.log | head -8
  PVVOTE_BYTES_XCD=$x timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/u1ab_$x" -o u1 -- python3 tools/u1_probe.py > gpurun_out/u1ab_$x.log 2>&1 || exit $?
  python3 - $x <<'PY'
import csv, sys
for r in csv.DictReader(open(f"gpurun_out/u1ab_{sys.argv[1]}/u1_kernel_stats.csv")):
    if "vote_bytes" in r["Name"]:
        print("xcd", sys.argv[1], r["Name"][:30], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), "us avg", round(float(r["MinNs"]) / 1000, 2), "min")
PY
done
