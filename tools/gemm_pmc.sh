#!/bin/bash
# MFMA-busy and clock counters of hipBLASLt's fp16 GEMM of layer4's
# implicit-GEMM size and of k_conv3x3 on the same shapes (tools/conv_ab.py),
# one counter pass each (MI355X_MICROARCH.md rocprofv3 section): the matrix
# pipe's busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
# GRBM_GUI_ACTIVE / 8).  Not part of the product.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES -T --output-format csv \
  -d "$PWD/gpurun_out/gemm_pmc" -o p -- python3 tools/conv_ab.py --gemm > gpurun_out/gemm_pmc.log 2>&1 || { echo "gemm pmc failed"; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-include-regex k_conv3x3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES -T --output-format csv \
  -d "$PWD/gpurun_out/conv_pmc" -o p -- python3 tools/conv_ab.py --one pvnet_amd/libpvvote.so > gpurun_out/conv_pmc.log 2>&1 || { echo "conv pmc failed"; exit 1; }
python3 - <<'PY'
import collections, csv
for d in ("gpurun_out/gemm_pmc", "gpurun_out/conv_pmc"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{d}/p_counter_collection.csv")):
        key = (r["Kernel_Name"].split("(")[0][:70], r.get("Grid_Size", ""))
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (name, grid), cs in acc.items():
        g = sum(cs["GRBM_GUI_ACTIVE"]) / len(cs["GRBM_GUI_ACTIVE"])
        m = sum(cs["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(cs["SQ_VALU_MFMA_BUSY_CYCLES"])
        if g < 1e6:
            continue
        print(f"{d.split('/')[-1]:9s} {name[:60]:60s} grid={grid:>9s} dispatches={len(cs['GRBM_GUI_ACTIVE']):3d} "
              f"GRBM_GUI_ACTIVE/8={g / 8:10.0f} MFMA busy={m / (1024 * g / 8):.3f}")
PY
