#!/bin/sh
# Copies the data fixtures this repo's tests use from the reference's own test
# directory (/root/reference/tests).  These are data files (tiny model checkpoints
# in rwkv.cpp format and expected logits), MIT-licensed (reference LICENSE:1-3).
# Run once in the build container; the copies are committed so the GPU box (which
# has no /root/reference) can run the parity tests.
set -e
SRC=${1:-/root/reference/tests}
DST=$(dirname "$0")
for v in 4v0-660K 5v1-730K 5v2-730K 6v0-3m 7v0-834K; do
  cp "$SRC/expected-logits-$v.bin" "$DST/"
done
for v in 4v0-660K 5v1-730K 5v2-730K 7v0-834K; do
  cp "$SRC/tiny-rwkv-$v-FP32.bin" "$SRC/tiny-rwkv-$v-FP16.bin" "$DST/"
done
# RWKV v6: the FP32/FP16 tiny checkpoints are missing from the reference
# (.MISSING_LARGE_BLOBS); only pre-quantized files exist.
cp "$SRC/tiny-rwkv-6v0-3m-Q5_0.bin" "$SRC/tiny-rwkv-6v0-3m-Q5_1.bin" "$SRC/tiny-rwkv-6v0-3m-FP16-to-Q4_0.bin" "$DST/"
