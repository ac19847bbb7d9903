#!/bin/bash
# One round-6 GPU cycle on the box, every step under its own time limit, chained so that a fault,
# abort or timeout ends the call (exit codes other than 0/1 from pytest stop everything):
#   tests  : pytest -m gpu
#   bench  : bench.py (default N = 1 line)
#   prof   : rocprofv3 kernel trace of the same build's roofline pass (bench.py --roofline-only),
#            recomputed against the bench line (tools/roofline_from_csv.py)
#   pmc    : FETCH_SIZE / WRITE_SIZE passes of the decode (separate runs), pooled per launch
# Usage: tools/r5_cycle.sh TAG [steps...]   (default steps: tests bench prof pmc)
TAG=${1:-x}
shift
STEPS=${*:-tests bench prof pmc}
ROOT=$GRAFT_REPO_ROOT
cd $ROOT && mkdir -p gpurun_out
O=$ROOT/gpurun_out
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
        --timeout-method thread > $O/r6_${TAG}_tests.log 2>&1
      rc=$?
      tail -3 $O/r6_${TAG}_tests.log
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc $rc"; exit $rc; fi
      ;;
    bench)
      timeout -k 10 500 python bench.py > $O/r6_${TAG}_bench.json 2> $O/r6_${TAG}_bench.err || { tail -5 $O/r6_${TAG}_bench.err; exit 1; }
      grep -E "decode:|seq-eval|pipeline|seq GEMM|ABI" $O/r6_${TAG}_bench.err
      ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r6_${TAG}_profr -o run --output-format csv -- \
        python3 $ROOT/bench.py --roofline-only --timing-steps 32 --warmup 0 --pipe-stages 0 > $O/r6_${TAG}_profr.log 2>&1 \
        || { tail -5 $O/r6_${TAG}_profr.log; exit 1; }
      cd $ROOT
      CSV=$(find $O/r6_${TAG}_profr -name "*kernel_stats.csv" | head -1)
      LINE=$O/r6_${TAG}_bench.json
      [ -s $LINE ] || LINE=$O/r6_${TAG}_profr.log
      python3 tools/roofline_from_csv.py $CSV $LINE > $O/r6_${TAG}_roofline_check.json
      cat $O/r6_${TAG}_roofline_check.json | head -30
      ;;
    pmc)
      cd /tmp && export TMPDIR=/tmp
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d $O/r6_${TAG}_pmc_$c -o run --output-format csv -- \
          python3 $ROOT/bench.py --decode-only --steps 16 --warmup 4 > $O/r6_${TAG}_pmc_$c.log 2>&1 \
          || { tail -5 $O/r6_${TAG}_pmc_$c.log; exit 1; }
      done
      cd $ROOT
      python3 tools/pmc_stream.py $O/r6_${TAG}_pmc_FETCH_SIZE $O/r6_${TAG}_pmc_WRITE_SIZE > $O/r6_${TAG}_pmc.json
      cat $O/r6_${TAG}_pmc.json | head -40
      ;;
    configs)
      # the other BASELINE configurations' lines (decode, seq-eval, batched B = 8 / 64, ABI decode)
      for c in ${CONFIGS:-v4-169m-q8_0 v7-2b9-q5_1 v5-7b-q4_1}; do
        timeout -k 10 400 python3 bench.py --config $c --steps 64 --warmup 8 --batch "8,64" --seq-reps 2 --abi-steps 8 \
          --skip-cpu --pipe-stages 0 > $O/r6_${TAG}_$c.log 2>&1 || { tail -5 $O/r6_${TAG}_$c.log; exit 1; }
        grep '^{' $O/r6_${TAG}_$c.log > $O/r6_${TAG}_$c.json
        grep -E "decode:|seq-eval" $O/r6_${TAG}_$c.log | sed "s/^/[$c] /" | cut -c1-160
      done
      ;;
    pipe8)
      # BASELINE config 5's pipeline: v5-7B, 8 stages on this box's one GPU, 4096 tokens
      timeout -k 10 400 python3 bench.py --config v5-7b-q4_1 --steps 8 --warmup 2 --batch "" --seq-len 4096 --seq-reps 1 \
        --abi-steps 0 --skip-cpu --timing-steps 1 --pipe-stages 8 > $O/r6_${TAG}_pipe8.log 2>&1 || { tail -5 $O/r6_${TAG}_pipe8.log; exit 1; }
      grep -E "pipeline|seq-eval" $O/r6_${TAG}_pipe8.log | cut -c1-200
      ;;
  esac
done
echo "cycle $TAG done"
