#!/bin/bash
# HIP runtime graph-launch knob A/B on the host cost of a 1,024-frame stream replay
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for e in "PVQ=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
  env $e timeout -k 10 300 python3 tools/replay_host_probe.py 1024 20 > gpurun_out/rh_$e.log 2>&1 || { echo "$e failed rc=$?"; tail -5 "gpurun_out/rh_$e.log"; exit 1; }
  echo "$e"; grep -v amdgpu.ids "gpurun_out/rh_$e.log" | tail -2
done
echo done
