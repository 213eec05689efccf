#!/bin/bash
# round 4, final code: GPU tests, smoke, the driver's bench command
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04_gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04_gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r04_gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 || { tail -5 gpurun_out/r04_smoke.log; exit 1; }
tail -1 gpurun_out/r04_smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04_final_bench.log 2>&1 || { grep -v amdgpu.ids gpurun_out/r04_final_bench.log | tail -20; exit 1; }
grep '^{' gpurun_out/r04_final_bench.log | tail -1 > gpurun_out/r04_final_bench.json
python3 -c "
import json;d=json.load(open('gpurun_out/r04_final_bench.json'))
print('value', d['value'], 'U1', d['roofline']['frac'], 'lat', d['latency_ms_per_image'], 'c3', d['stream_config3']['images_per_s'], 'e2e2', d['e2e_config2_fp16_batch32']['images_per_s'], 'cpu', d['cpu_baseline']['value'])"
echo done
