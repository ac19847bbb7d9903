#!/bin/bash
# rocprofv3 kernel traces of decode (eager timing pass: bench.py --roofline-only) for the given configs
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_$c -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config $c --roofline-only --timing-steps 4 --warmup 0 --pipe-stages 0 --skip-cpu \
    > $O/trace_$c.log 2>&1 || { tail -5 $O/trace_$c.log; exit 1; }
done
echo done
