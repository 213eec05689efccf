#!/bin/bash
# streams kept alive: the many-graph probe twice and the driver's bench command
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -X faulthandler tools/extra_kernel_probe.py 2 > gpurun_out/xk3.log 2>&1 || { grep -v amdgpu.ids gpurun_out/xk3.log | tail -30; exit 1; }
grep "^round" gpurun_out/xk3.log
timeout -k 10 600 python3 -X faulthandler bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b29.log 2>&1 || { grep -v amdgpu.ids gpurun_out/b29.log | tail -30; exit 1; }
python3 -c "
import json;d=json.loads([x for x in open('gpurun_out/b29.log') if x.startswith('{')][-1])
print('value', d['value'], 'U1', d['roofline']['frac'], 'lat', d['latency_ms_per_image'], 'c3', d['stream_config3']['images_per_s'], 'e2e2', d['e2e_config2_fp16_batch32']['images_per_s'])"
echo done
