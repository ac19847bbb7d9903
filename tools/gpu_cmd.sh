mkdir -p gpurun_out
tools/ab_lib.sh v6-1b6-q4_0 3 sigmaa=this off=this@RWKV_MI355X_DECODE_FUSION=63 > gpurun_out/r6_ab_sigmaa.txt 2>&1 || exit 1
cat gpurun_out/r6_ab_sigmaa.txt
