#!/bin/bash
# PMC passes over the fp16 batch-32 backbone (tools/bb_kernels.py), the HIP
# convolution kernels only, one counter group per pass (MI355X_MICROARCH.md
# HBM / rocprofv3 sections); then tools/bb_pmc_summary.py folds them.
#   tools/bb_pmc.sh [tag]   (PVVOTE_LIB selects a variant library)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tag=${1:-cur}
RE="k_conv3x3|k_conv64|k_dec_conv|k_stem|k_decoder_tail|k_relu_pool"
i=0
dirs=""
for c in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-include-regex "$RE" --pmc $c -T --output-format csv \
    -d "$PWD/gpurun_out/bbpmc_${tag}_$i" -o p -- python3 tools/bb_kernels.py > gpurun_out/bbpmc_${tag}_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  dirs="$dirs gpurun_out/bbpmc_${tag}_$i"
done
python3 tools/bb_pmc_summary.py $dirs gpurun_out/bbpmc_${tag}.json > /dev/null && echo "pmc $tag ok"
