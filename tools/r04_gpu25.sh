#!/bin/bash
# the driver's bench command at the new default (1,024 frames per step): plain, timed
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
start=$(date +%s)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b25.log 2>&1 || { tail -20 gpurun_out/b25.log; exit 1; }
echo "wall $(( $(date +%s) - start )) s"
python3 -c "
import json;d=json.loads([x for x in open('gpurun_out/b25.log') if x.startswith('{')][-1])
print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'U1', d['roofline']['frac'], 'lat', d['latency_ms_per_image'], 'order', d['stream_order_ok'])
print('c3', d['stream_config3']['images_per_s'], 'c4', d['stream_config4']['images_per_s'], 'e2e2', d['e2e_config2_fp16_batch32']['images_per_s'], 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 400 python3 -u -m pytest tests/test_bench_launcher.py tests/test_gpu_stream.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/t25.log 2>&1 || { tail -20 gpurun_out/t25.log; exit 1; }
tail -1 gpurun_out/t25.log
echo done
