#!/bin/bash
# Decode roofline reproducibility: the bench line (per-dispatch event roofline), then a rocprofv3
# kernel trace of `bench.py --decode-only` (graph-replayed decode only), then the recompute of the
# line's roofline from that trace.  Usage: tools/r4_prof.sh TAG
TAG=${1:-p}
ROOT=$GRAFT_REPO_ROOT
cd $ROOT && mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --skip-cpu --batch "" --seq-reps 1 --abi-steps 4 > gpurun_out/${TAG}_line.log 2>&1 || { tail -5 gpurun_out/${TAG}_line.log; exit 1; }
grep -E "decode:" gpurun_out/${TAG}_line.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_${TAG} -o run --output-format csv -- \
  python3 $ROOT/bench.py --decode-only --steps 256 > $ROOT/gpurun_out/prof_${TAG}.log 2>&1 || { tail -5 $ROOT/gpurun_out/prof_${TAG}.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/profr_${TAG} -o run --output-format csv -- \
  python3 $ROOT/bench.py --roofline-only --timing-steps 32 --warmup 0 > $ROOT/gpurun_out/profr_${TAG}.log 2>&1 || { tail -5 $ROOT/gpurun_out/profr_${TAG}.log; exit 1; }
cd $ROOT
CSV=$(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1)
echo "stats: $CSV"
python3 tools/roofline_from_csv.py $CSV gpurun_out/${TAG}_line.log | tee gpurun_out/${TAG}_roofline_check.json

CSV2=$(find gpurun_out/profr_${TAG} -name "*kernel_stats.csv" | head -1)
echo "roofline-pass stats: $CSV2"
python3 tools/roofline_from_csv.py $CSV2 gpurun_out/profr_${TAG}.log | tee gpurun_out/${TAG}_roofline_check_eager.json
echo done
