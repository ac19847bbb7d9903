mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wkv_chunk.py -k wkv7 > gpurun_out/r6_wkv7c_tests.txt 2>&1
rc=$?; grep -E "T=|v7|passed|failed|Error|assert" gpurun_out/r6_wkv7c_tests.txt | head -30; [ $rc = 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r6_wkv7c_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/wkv7_chunk_time.py > $GRAFT_REPO_ROOT/gpurun_out/r6_wkv7c_prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
cat gpurun_out/r6_wkv7c_prof.log | tail -3
grep -h -E "wkv7" $(find gpurun_out/r6_wkv7c_prof -name "*kernel_stats.csv") | cut -d, -f1-8
timeout -k 10 400 python tools/ab_seq.py --config v7-2b9-q5_1 --reps 3 --arm "" --arm "wkv_chunk=1" > gpurun_out/r6_ab_wkv7c_seq.txt 2>&1 || exit 1
tail -3 gpurun_out/r6_ab_wkv7c_seq.txt
