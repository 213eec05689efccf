#!/bin/bash
# Per-variant HBM traffic of the pipeline's kernels: one FETCH_SIZE and one
# WRITE_SIZE pass per variant library (VARIANTS="name ..." -> variants/<name>.so,
# "cur" = pvnet_amd/libpvvote.so), folded by tools/pmc_traffic_json.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in $VARIANTS; do
  lib=variants/$v.so; [ "$v" = cur ] && lib=pvnet_amd/libpvvote.so
  for c in FETCH_SIZE WRITE_SIZE; do
    PVVOTE_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-include-regex "k_vote|k_compact|k_fg_count|k_refine|k_hyp_gen|k_front" \
      --pmc $c -T --output-format csv -d "$PWD/gpurun_out/abt_${v}_$c" -o b -- python3 bench.py --skip-cpu --skip-e2e --skip-u1 --steps 20 \
      > gpurun_out/abt_${v}_$c.log 2>&1 || { echo "failed: $v $c"; tail -5 gpurun_out/abt_${v}_$c.log; exit 1; }
  done
  echo "== $v"
  python3 tools/pmc_traffic_json.py gpurun_out/abt_${v}_FETCH_SIZE gpurun_out/abt_${v}_WRITE_SIZE gpurun_out/abt_$v.json | tr -d '\n ' ; echo
done
