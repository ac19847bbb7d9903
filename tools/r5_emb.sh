#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/emb_tests.log 2>&1
rc=$?; tail -2 $O/emb_tests.log; grep FAILED $O/emb_tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
for c in v6-1b6-q4_0 v4-169m-q8_0; do
  timeout -k 10 200 python3 bench.py --config $c --decode-only --steps 256 --warmup 16 --skip-cpu --pipe-stages 0 > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
  echo "$c $(grep -E 'decode:' $O/ab.err) $(grep -o 'k_embed_ln[^}]*}' $O/ab.json)"
done
