#!/bin/bash
# SQ counters of k_fmm per dispatch (tools/fmm_probe shapes): where a small-K workgroup's time goes.
ROOT=$GRAFT_REPO_ROOT
mkdir -p $ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD \
  --kernel-include-regex "k_fmm" -d $ROOT/gpurun_out/pmc_fmm -o run --output-format csv -- $ROOT/tools/pbin/fmm_probe > $ROOT/gpurun_out/pmc_fmm.log 2>&1 || exit 6
python3 - $ROOT/gpurun_out/pmc_fmm <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for path in f:
    for r in csv.DictReader(open(path)):
        k = (r['Kernel_Name'][:24], r.get('Grid_Size', r.get('Grid_Size_X', '')))
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        if r['Counter_Name'] == 'SQ_WAVES': n[k] += 1
for k, d in agg.items():
    w = d['SQ_WAVES'] or 1
    print(k, 'disp', n[k], 'per wave:', {c: round(v / w) for c, v in sorted(d.items()) if c != 'SQ_WAVES'}, 'waves/disp', round(w / max(n[k], 1)))
PY
