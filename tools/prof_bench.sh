#!/bin/bash
# The driver's exact bench command, plain and under rocprofv3 --kernel-trace
# --stats (the summary behind the JSON line's kernel durations), then one
# FETCH_SIZE and one WRITE_SIZE pass (tools/pmc_traffic_json.py folds them).
# Every GPU step under its own time limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
CMD="bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 400 python3 $CMD > gpurun_out/bench_plain.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_plain.log; exit 1; }
grep '^{' gpurun_out/bench_plain.log | tail -1 > gpurun_out/bench_plain.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/prof_bench" -o bench -- python3 $CMD > gpurun_out/bench_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/bench_prof.log; exit 1; }
grep '^{' gpurun_out/bench_prof.log | tail -1 > gpurun_out/bench_prof.json
python3 tools/u1_trace_summary.py gpurun_out/prof_bench/bench_kernel_trace.csv gpurun_out/bench_prof.json gpurun_out/u1_timed_launches.json
python3 tools/u4_trace_summary.py gpurun_out/prof_bench/bench_kernel_trace.csv gpurun_out/bench_prof.json gpurun_out/u4_timed_launches.json
python3 tools/kernel_phases.py gpurun_out/prof_bench/bench_kernel_trace.csv gpurun_out/kernel_phases.json > /dev/null 2>&1 || true
# the full trace (~1M rows at 1,024 frames per step) stays on the box: its summaries above are what is kept
rm -f gpurun_out/prof_bench/bench_kernel_trace.csv
if [ -n "$PMC" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --kernel-include-regex "k_vote|k_compact|k_fg_count|k_refine|k_hyp_gen|k_front" --pmc $c -T --output-format csv \
      -d "$PWD/gpurun_out/pmc_$c" -o b -- python3 bench.py --steps 5 --warmup 2 --skip-cpu --skip-e2e --skip-config3 --skip-u4 > gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
    timeout -k 10 300 rocprofv3 --kernel-include-regex "k_vote_mfma|k_evd" --pmc $c -T --output-format csv \
      -d "$PWD/gpurun_out/pmcu4_$c" -o b -- python3 tools/u4_probe.py 10 > gpurun_out/pmcu4_$c.log 2>&1 || { echo "pmc u4 $c failed"; exit 1; }
  done
  python3 tools/pmc_traffic_json.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE gpurun_out/pmc_traffic.json \
    gpurun_out/pmcu4_FETCH_SIZE gpurun_out/pmcu4_WRITE_SIZE > /dev/null
fi
echo ok
