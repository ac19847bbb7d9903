cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py -q -p no:cacheprovider --timeout 200 --timeout-method thread -x > gpurun_out/gpu_r2k.log 2>&1
echo EXIT $? >> gpurun_out/gpu_r2k.log
timeout -k 10 200 python bench.py --steps 64 --warmup 8 --skip-cpu --seq-reps 3 --abi-steps 0 > gpurun_out/bench_r2k.json 2> gpurun_out/bench_r2k.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmcg_g2_2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --skip-cpu --seq-reps 1 --abi-steps 0 --timing-steps 1 > $GRAFT_REPO_ROOT/gpurun_out/pmcg_g2_2.log 2>&1
