#!/bin/bash
# v7: parity tests, then decode / sequence A/B of the fused LoRA + attention launch
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_batch.py tests/test_gpu_pipeline_abi.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "7 or v7" > gpurun_out/v7_tests.log 2>&1
rc=$?; tail -5 gpurun_out/v7_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in RWKV_MI355X_ATT7_LORA=0 RWKV_MI355X_ATT7_LORA=1; do
  env $v timeout -k 10 300 python3 bench.py --config v7-2b9-q5_1 --steps 64 --warmup 8 --skip-cpu --seq-reps 1 --abi-steps 0 --batch "" --timing-steps 2 --pipe-stages 0 2>&1 | grep -E "decode:|k_att7|k_mv |k_mva" | sed "s/^/[$v] /"
done
