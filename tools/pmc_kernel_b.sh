#!/bin/bash
# One PMC pass (SQ counters) over the kernels matching REGEX in a short sequence-eval bench run.
# Usage: tools/pmc_kernel.sh TAG REGEX
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS \
  --kernel-include-regex "$2" -d $ROOT/gpurun_out/pmc_$1 -o run --output-format csv -- \
  python3 $ROOT/bench.py --steps 4 --warmup 1 --skip-cpu --seq-reps 1 --batch "" --abi-steps 0 --timing-steps 0 > $ROOT/gpurun_out/pmc_$1.log 2>&1 || exit 6
python3 - $ROOT/gpurun_out/pmc_$1 <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for path in f:
    for r in csv.DictReader(open(path)):
        k = r['Kernel_Name'][:60]
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        if r['Counter_Name'] == 'SQ_WAVES': n[k] += 1
for k, d in agg.items():
    print(k, 'dispatches', n[k], {c: round(v / max(n[k], 1)) for c, v in sorted(d.items())})
PY
