#!/bin/bash
# Decode front-end probe: the counter list of this rocprofv3, then SQ issue/stall counters and (when
# listed) instruction-cache counters over the decode kernels of a short bench run.  One PMC pass per
# rocprofv3 run; every pass under its own time limit.  Usage: tools/r3_icache.sh TAG
TAG=${1:-ic}
ROOT=$GRAFT_REPO_ROOT
mkdir -p $ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $ROOT/gpurun_out/${TAG}_counters.txt 2>&1 || true
grep -o -E '\b(SQC?_[A-Z0-9_]+|TCP_[A-Z0-9_]+)\b' $ROOT/gpurun_out/${TAG}_counters.txt | sort -u > $ROOT/gpurun_out/${TAG}_names.txt || true
pass() {  # pass NAME COUNTERS...
  local name=$1; shift
  local have=""
  for c in "$@"; do grep -qx "$c" $ROOT/gpurun_out/${TAG}_names.txt && have="$have $c"; done
  [ -z "$have" ] && { echo "pass $name: no counters listed"; return 0; }
  echo "pass $name:$have"
  timeout -s KILL 90 rocprofv3 --pmc $have --kernel-include-regex 'k_mv|k_mva|att6|maa|k_embed' \
    -d $ROOT/gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 32 --warmup 2 --skip-cpu --seq-reps 1 --seq-len 64 --batch "" --abi-steps 0 --timing-steps 0 \
    > $ROOT/gpurun_out/pmc_${TAG}_$name.log 2>&1 || { echo "pass $name failed"; tail -3 $ROOT/gpurun_out/pmc_${TAG}_$name.log; return 1; }
  python3 $ROOT/tools/pmc_agg.py $ROOT/gpurun_out/pmc_${TAG}_$name > $ROOT/gpurun_out/pmc_${TAG}_$name.txt 2>&1 || true
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU && \
pass sqc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVES SQ_IFETCH_LEVEL && \
pass sq2 SQ_WAVES SQ_WAVE_CYCLES SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM
echo done
