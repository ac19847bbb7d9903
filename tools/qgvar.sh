#!/bin/bash
# Fast variant builds of the library that differ only in qgemm.hip's -D flags: the other objects
# come from rwkv.cppy_amd/build/.  Usage (CPU host): tools/qgvar.sh NAME "-DFLAG=1 -DX=2" [NAME FLAGS]...
cd ${GRAFT_REPO_ROOT:-/root/repo}/rwkv.cppy_amd || exit 1
make -s -j8 >/dev/null || exit 1
CXX="/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fvisibility=hidden -DRWKV_BUILD -DRWKV_SHARED -Wall -Wno-unused-result -mllvm -amdgpu-kernarg-preload-count=16 -mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize"
pids=""
while [ $# -ge 2 ]; do
  n=$1; f=$2; shift 2
  mkdir -p build_$n
  ( $CXX $f -x hip -c csrc/qgemm.hip -o build_$n/qgemm.hip.o && \
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build_$n/librwkv.so $(ls build/*.o | grep -v qgemm) build_$n/qgemm.hip.o -lpthread ) &
  pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=1; done
exit $rc
