#!/bin/bash
# U1 check on the GPU box: voting parity tests, rocprof kernel time of
# k_vote_bytes (tools/u1_probe.py), a per-wave trace (variants/u1trace.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
[ -n "$LIB" ] && export PVVOTE_LIB=$LIB
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/u1c${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/u1c${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/u1c${TAG}_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/u1c${TAG}" -o u1 -- python3 tools/u1_probe.py > gpurun_out/u1c${TAG}_probe.log 2>&1 || exit $?
python3 - <<'PY'
import csv, os
for r in csv.DictReader(open(f"gpurun_out/u1c{os.environ.get('TAG', '')}/u1_kernel_stats.csv")):
    if "vote_bytes" in r["Name"] or "fill" in r["Name"].lower():
        print(r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), "us avg", round(float(r["MinNs"]) / 1000, 2), "min")
PY
PVVOTE_LIB=${TRACELIB:-variants/u1trace.so} timeout -k 10 120 python tools/bytes_trace.py > gpurun_out/u1c${TAG}_trace.log 2>&1 || exit $?
cat gpurun_out/u1c${TAG}_trace.log | grep -v "^wave "
