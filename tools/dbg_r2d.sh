cd $GRAFT_REPO_ROOT
timeout -k 10 60 tools/bin/f16_probe gpurun_out/f16_probe.bin > gpurun_out/dbg_r2d.log 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider --timeout 100 --timeout-method thread >> gpurun_out/dbg_r2d.log 2>&1
echo EXIT $? >> gpurun_out/dbg_r2d.log
