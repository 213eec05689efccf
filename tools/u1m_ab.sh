#!/bin/bash
# U1 matrix-core kernel: its GPU parity tests, then rocprof kernel times of
# k_vote_bytes_mfma vs the VALU k_vote_bytes (PVVOTE_BYTES_MFMA=1/0) on the
# U1 probe shapes.  Each GPU step under its own limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "${TESTK:-vote_bytes or guard_band or band_pairs or kernels_bit_exact}" > gpurun_out/u1m_tests.log 2>&1 || { tail -40 gpurun_out/u1m_tests.log; exit 1; }
tail -2 gpurun_out/u1m_tests.log
for m in ${MODES:-1 0}; do
  PVVOTE_BYTES_MFMA=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/u1m_$m" -o u1 -- python3 tools/u1_probe.py > gpurun_out/u1m_$m.log 2>&1 || { tail -20 gpurun_out/u1m_$m.log; exit 1; }
  grep "^tn=" gpurun_out/u1m_$m.log
  python3 - $m <<'PY'
import csv, sys
for r in csv.DictReader(open(f"gpurun_out/u1m_{sys.argv[1]}/u1_kernel_stats.csv")):
    if "vote_bytes" in r["Name"] or "elementwise" in r["Name"]:
        print("mfma", sys.argv[1], r["Name"][:34], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), "us avg", round(float(r["MinNs"]) / 1000, 2), "min")
PY
done
