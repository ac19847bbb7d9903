"""Records sha256 digests of the reference's own quantized tiny-model files
(/root/reference/tests/tiny-rwkv-*-{FP32,FP16}-to-Q*.bin).  These files are the
byte-exact outputs of the reference quantizer (rwkv_quantize.inc:16-171 +
ggml quantize_row_*_ref).  The digests are committed as a known-answer fixture so
the quantizer tests run without /root/reference and without committing 40 files.
"""
import hashlib, json, os, sys

SRC = sys.argv[1] if len(sys.argv) > 1 else '/root/reference/tests'
out = {}
for v in ['4v0-660K', '5v1-730K', '5v2-730K', '6v0-3m', '7v0-834K']:
    for src in ['FP32', 'FP16']:
        for q in ['Q4_0', 'Q4_1', 'Q5_0', 'Q5_1', 'Q8_0']:
            name = f'tiny-rwkv-{v}-{src}-to-{q}.bin'
            p = os.path.join(SRC, name)
            if os.path.isfile(p):
                out[name] = hashlib.sha256(open(p, 'rb').read()).hexdigest()
json.dump(out, open(os.path.join(os.path.dirname(__file__), 'quantizer_kat_sha256.json'), 'w'), indent=1, sort_keys=True)
print(len(out), 'digests')
