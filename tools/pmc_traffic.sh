cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-include-regex "k_vote|k_compact|k_fg_count|k_refine|k_prep|k_hyp_gen" --pmc FETCH_SIZE -T --output-format csv -d $PWD/gpurun_out/tr_fetch -o b -- python3 bench.py --skip-cpu --skip-e2e --steps 20 > /dev/null 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-include-regex "k_vote|k_compact|k_fg_count|k_refine|k_prep|k_hyp_gen" --pmc WRITE_SIZE -T --output-format csv -d $PWD/gpurun_out/tr_write -o b -- python3 bench.py --skip-cpu --skip-e2e --steps 20 > /dev/null 2>&1
