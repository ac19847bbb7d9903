cd $GRAFT_REPO_ROOT
for m in tests/golden/tiny-rwkv-6v0-3m-Q5_1.bin tests/golden/tiny-rwkv-6v0-3m-FP32-to-Q4_1.bin; do
  timeout -k 10 120 python tools/debug_bitexact.py $m 70 >> gpurun_out/dbg_r2c.log 2>&1 || exit 1
done
python - <<'PY' >> gpurun_out/dbg_r2c.log 2>&1
import ctypes,sys
sys.path.insert(0,'tests')
from rwkv_lib import library
L=library().library
p=b'/tmp/v5cfg.bin'
assert L.rwkv_mi355x_write_synthetic_model(p,5,4096,4096,2,14336,b'Q4_1',21)
PY
timeout -k 10 200 python tools/debug_bitexact.py /tmp/v5cfg.bin 6 >> gpurun_out/dbg_r2c.log 2>&1
