cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/debug_stage.py tests/golden/tiny-rwkv-6v0-3m-FP32-to-Q4_1.bin 10 23 > gpurun_out/dbg_r2e.log 2>&1
