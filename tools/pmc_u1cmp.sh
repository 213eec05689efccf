cd $GRAFT_REPO_ROOT
C1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_SMEM"
C2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_BUSY_CU_CYCLES"
timeout -k 10 200 rocprofv3 --kernel-include-regex k_vote_bytes --pmc $C1 -T --output-format csv -d $PWD/gpurun_out/u1c1 -o p -- python3 tools/u1_probe.py > /dev/null 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-include-regex k_vote_bytes --pmc $C2 -T --output-format csv -d $PWD/gpurun_out/u1c2 -o p -- python3 tools/u1_probe.py > /dev/null 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-include-regex k_loop --pmc $C1 -T --output-format csv -d $PWD/gpurun_out/lb1 -o p -- ./tools/loop_bench2 > /dev/null 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-include-regex k_loop --pmc $C2 -T --output-format csv -d $PWD/gpurun_out/lb2 -o p -- ./tools/loop_bench2 > /dev/null 2>&1
