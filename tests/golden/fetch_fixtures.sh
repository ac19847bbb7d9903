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
# The other pre-quantized v6 files; FP32-to-Q5_0 / FP32-to-Q5_1 are byte-identical to -Q5_0 / -Q5_1
# (same sha256) and are not copied (tests/test_gpu_parity.py DUP_V6 maps them).
for q in FP16-to-Q4_1 FP16-to-Q5_0 FP16-to-Q5_1 FP32-to-Q4_0 FP32-to-Q4_1; do
  cp "$SRC/tiny-rwkv-6v0-3m-$q.bin" "$DST/"
done
# The World tokenizer's vocabulary (a data file the reference's tokenizer test reads,
# python/rwkv_cpp/rwkv_world_tokenizer.test.py), so the harness tests run on the GPU box too.
cp "$SRC/../python/rwkv_cpp/rwkv_vocab_v20230424.txt" "$DST/"
