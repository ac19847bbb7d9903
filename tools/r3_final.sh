#!/bin/bash
# End-of-round-3 cycle at the final HEAD: GPU tests, smoke, bench line, rocprof stats (r3_cycle.sh),
# then the other BASELINE configurations' bench lines (decode, seq-eval, B = 8 / 64 batched).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${1:-r3d}
bash tools/r3_cycle.sh $TAG tests || exit 1
grep -E "decode|seq-eval" gpurun_out/${TAG}_bench.log | cut -c1-160
for c in v4-169m-q8_0 v7-2b9-q5_1 v5-7b-q4_1; do
  timeout -k 10 400 python3 bench.py --config $c --steps 64 --warmup 8 --batch "8,64" --seq-reps 2 --abi-steps 8 --skip-cpu > gpurun_out/${TAG}_$c.log 2>&1 || { tail -5 gpurun_out/${TAG}_$c.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_$c.log > gpurun_out/${TAG}_$c.json
  grep -E "decode|seq-eval" gpurun_out/${TAG}_$c.log | sed "s/^/[$c] /" | cut -c1-160
done
echo done
