#!/bin/bash
# round 4 checkpoint A: GPU tests, smoke, PMC traffic passes (the bench line's `traffic` fields)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r04_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r04_gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 || { tail -5 gpurun_out/r04_smoke.log; exit 1; }
tail -1 gpurun_out/r04_smoke.log
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --kernel-include-regex "k_vote|k_compact|k_fg_count|k_refine|k_hyp_gen|k_front" --pmc $c -T --output-format csv \
    -d "$PWD/gpurun_out/pmc_$c" -o b -- python3 bench.py --steps 5 --warmup 2 --skip-cpu --skip-e2e --skip-config3 --skip-u4 > gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-include-regex "k_vote_mfma|k_evd" --pmc $c -T --output-format csv \
    -d "$PWD/gpurun_out/pmcu4_$c" -o b -- python3 tools/u4_probe.py 10 > gpurun_out/pmcu4_$c.log 2>&1 || { echo "pmc u4 $c failed"; exit 1; }
done
python3 tools/pmc_traffic_json.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/r04_pmc_traffic.json \
  gpurun_out/pmcu4_FETCH_SIZE gpurun_out/pmcu4_WRITE_SIZE
bash tools/lat_ab.sh rf0 rf1 || exit $?
echo done
