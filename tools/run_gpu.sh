#!/bin/bash
# GPU-box driver: each GPU step under its own time limit; stop at the first
# fault/abort/timeout (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    threads) step gpu_threads 300 python -u -m pytest tests/test_gpu_threads.py -x -v --timeout 200 --timeout-method thread ;;
    rtp) step rtp 300 python3 tools/replay_threads_probe.py ;;
    tests) step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    testsall) step gpu_tests 900 python -m pytest tests -m gpu -q ;;
    lat) step lat 120 python3 tools/lat_trace.py 20 &&
         step latprof 200 rocprofv3 --kernel-trace -T --output-format csv -d "$PWD/gpurun_out/prof_lat" -o lat -- python3 tools/lat_trace.py 10 &&
         python3 tools/lat_trace.py --gaps gpurun_out/prof_lat/lat_kernel_trace.csv > gpurun_out/lat_gaps.log 2>&1; cat gpurun_out/lat_gaps.log ;;
    ctrace) step ctrace 120 python3 tools/compact_trace.py ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    benchfull) step bench 600 python bench.py && cp gpurun_out/bench.log gpurun_out/bench_full.log ;;
    benchquick) step bench 400 python bench.py --steps 20 --warmup 5 --skip-cpu ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/prof" -o bench -- python3 bench.py --skip-cpu --skip-e2e ;;
    pmcfetch) step pmcfetch 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$PWD/gpurun_out/pmc_fetch" -o bench -- python3 bench.py --skip-cpu --skip-e2e --steps 20 ;;
    pmcwrite) step pmcwrite 600 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$PWD/gpurun_out/pmc_write" -o bench -- python3 bench.py --skip-cpu --skip-e2e --steps 20 ;;
    pmchbm) step pmchbm1 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$PWD/gpurun_out/pmc_fetch" -o bench -- python3 bench.py --skip-cpu --skip-e2e --steps 20 &&
            step pmchbm2 600 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$PWD/gpurun_out/pmc_write" -o bench -- python3 bench.py --skip-cpu --skip-e2e --steps 20 ;;
    pmcvalu) step pmcvalu 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T --output-format csv -d "$PWD/gpurun_out/pmc_valu" -o bench -- python3 bench.py --skip-cpu --skip-e2e --steps 20 ;;
    pmcu1v) for v in u1base u1nostore; do PVVOTE_LIB=variants/$v.so step pmcu1_$v 300 rocprofv3 --kernel-include-regex k_vote_bytes --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -T --output-format csv -d "$PWD/gpurun_out/pmcu1_$v" -o v -- python3 tools/u1_probe.py; done ;;
    profu1v) for v in ${VARIANTS:-u1base u1nostore u1nocomp}; do PVVOTE_LIB=variants/$v.so step profu1_$v 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/profu1_$v" -o u1 -- python3 tools/u1_probe.py; done ;;
    profu1x) PVVOTE_DEBUG_BYTES=3 step profu1x 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/profu1x" -o u1 -- python3 tools/u1_probe.py ;;
    profu1) step profu1 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/profu1" -o u1 -- python3 tools/u1_probe.py ;;
    profdriver) step profdriver 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/profdriver" -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    benchdriver) step benchdriver 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    listpmc) step listpmc 300 rocprofv3 -L ;;
    pmcvote) step pmcvote1 600 rocprofv3 --kernel-include-regex k_vote_count --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_SALU -T --output-format csv -d "$PWD/gpurun_out/pmc_vote1" -o v -- python3 bench.py --skip-cpu --skip-e2e --skip-u1 --steps 10 &&
             step pmcvote2 600 rocprofv3 --kernel-include-regex k_vote_count --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVES SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE SQ_INSTS_VALU_TRANS_F32 -T --output-format csv -d "$PWD/gpurun_out/pmc_vote2" -o v -- python3 bench.py --skip-cpu --skip-e2e --skip-u1 --steps 10 &&
             step pmcvote3 600 rocprofv3 --kernel-include-regex k_vote_count --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_ACCUM_PREV_HIRES -T --output-format csv -d "$PWD/gpurun_out/pmc_vote3" -o v -- python3 bench.py --skip-cpu --skip-e2e --skip-u1 --steps 10 ;;
    pmcbytes) step pmcbytes1 300 rocprofv3 --kernel-include-regex k_vote_bytes --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_SALU -T --output-format csv -d "$PWD/gpurun_out/pmc_bytes1" -o v -- python3 tools/u1_probe.py &&
              step pmcbytes2 300 rocprofv3 --kernel-include-regex k_vote_bytes --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_LDS -T --output-format csv -d "$PWD/gpurun_out/pmc_bytes2" -o v -- python3 tools/u1_probe.py ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
