#!/bin/bash
# Whole GPU suite with the fused-Wo knobs on, then decode A/B: v6 (RWKV_MI355X_WO_FUSED),
# v4 (RWKV_MI355X_WO4_FUSED), v7 (RWKV_MI355X_ATT7_LORA)
cd $GRAFT_REPO_ROOT
RWKV_MI355X_WO_FUSED=1 RWKV_MI355X_WO4_FUSED=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/dec_tests.log 2>&1
rc=$?; tail -4 gpurun_out/dec_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in RWKV_MI355X_WO_FUSED=0 RWKV_MI355X_WO_FUSED=1; do
  env $v timeout -k 10 300 python3 bench.py --steps 256 --warmup 16 --skip-cpu --seq-reps 0 --abi-steps 32 --batch "" --timing-steps 4 --pipe-stages 0 2>&1 | grep -E "decode:|ABI|k_v6_att|k_mva |k_mv " | sed "s/^/[$v] /"
done
for v in RWKV_MI355X_WO4_FUSED=0 RWKV_MI355X_WO4_FUSED=1; do
  env $v timeout -k 10 300 python3 bench.py --config v4-169m-q8_0 --steps 256 --warmup 16 --skip-cpu --seq-reps 0 --abi-steps 0 --batch "" --timing-steps 4 --pipe-stages 0 2>&1 | grep -E "decode:|k_v4" | sed "s/^/[$v] /"
done
for v in RWKV_MI355X_ATT7_LORA=0 RWKV_MI355X_ATT7_LORA=1; do
  env $v timeout -k 10 300 python3 bench.py --config v7-2b9-q5_1 --steps 64 --warmup 8 --skip-cpu --seq-reps 0 --abi-steps 0 --batch "" --timing-steps 2 --pipe-stages 0 2>&1 | grep -E "decode:|k_att7" | sed "s/^/[$v] /"
done
