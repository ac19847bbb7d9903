#!/usr/bin/env python3
"""Benchmark of the RWKV eval hot path on MI355X (BASELINE.json metric).

A "step" is one single-token decode (rwkv_eval semantics: the whole model incl. the head,
logits produced) of RWKV-v6-World-1B6 Q4_0 with the recurrent state resident in HBM
(rwkv_mi355x_eval_device).  Steps are enqueued back to back on the context's stream.
value = tokens decoded by all ranks / max-over-ranks wall time of the K timed steps.
Multi-GPU: decode does not shard -- each rank runs an independent replica
("scaling": "weak").  Sequence evaluation is reported both ways: independent replicas, and one
sequence through the in-library layer pipeline over all N GPUs (rwkv_mi355x_init_pipeline, driven by
rank 0; peer copies over xGMI).  At N = 1 the same pipeline runs with every stage on GPU 0.

Also reported (same run): 1024-token rwkv_eval_sequence throughput, ABI-level decode
(13 MB of host state in and out per token, the reference's contract), the dominant kernel's
roofline (HIP events on the context stream, algorithmic bytes), and the CPU restatement of
the reference arithmetic (oracle/) timed on this host's cores.

Synthetic weights (no checkpoint can be downloaded): rwkv_mi355x_write_synthetic_model
writes an rwkv.cpp file with the exact tensor shapes of the real checkpoint.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'rwkv.cppy_amd', 'python'))
sys.path.insert(0, os.path.join(REPO, 'tests'))

METRIC = 'tokens/sec RWKV-v6-World-1B6 Q4_0 decode + seq-eval @1/2/4/8 GPU; HBM GB/s vs peak'
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
INT8_MFMA_PEAK_TOPS = 5000.0  # dense int8 MFMA: 2x the ~2.5 PF dense bf16 rate (MI355X_MICROARCH.md, Matrix cores)
# decode kernels that stream layer / head weights (the roofline's pooled kernel class)
STREAM_KERNELS = ('k_mv', 'k_mva', 'k_v6_maa_dec', 'k_v6_maa_dec4', 'k_v6_att_fused', 'k_v6_att_co', 'k_mvsig', 'k_sig_maa',
                  'k_v4_att_fused', 'k_ffn_fused', 'k_att7_lora')

CONFIGS = {
    # name: arch, n_vocab, n_embed, n_layer, ffn (0 = arch default), format, label
    'v6-1b6-q4_0': (6, 65536, 2048, 24, 0, 'Q4_0', 'RWKV-v6-World-1B6 Q4_0'),
    'v4-169m-q8_0': (4, 50277, 768, 12, 0, 'Q8_0', 'RWKV-v4-Pile-169M Q8_0'),
    'v7-2b9-q5_1': (7, 65536, 2560, 32, 0, 'Q5_1', 'RWKV-v7-World-2.9B Q5_1'),
    'v5-7b-q4_1': (5, 65536, 4096, 32, 14336, 'Q4_1', 'RWKV-v5-World-7B Q4_1'),
}


def log(*a):
    print('[bench]', *a, file=sys.stderr, flush=True)


def physical_cores():
    """Physical cores of this host: distinct (physical id, core id) pairs in /proc/cpuinfo."""
    try:
        cores, phys = set(), '0'
        with open('/proc/cpuinfo') as f:
            for line in f:
                k, _, v = line.partition(':')
                k = k.strip()
                if k == 'physical id':
                    phys = v.strip()
                elif k == 'core id':
                    cores.add((phys, v.strip()))
        return len(cores) or None
    except OSError:
        return None


def decode_parity(L, ctx, om, tokens, olg0, ost0, n_vocab, state_len, tok_arr, P_F):
    """Parity of this run's model over every CPU-sampled token (after the timed regions).

    Gate: the GPU decode of `tokens` from a fresh state must equal the oracle's GPU-association
    variant (oracle.c OV_GPU: ggml semantics in the kernels' documented association) bit for bit,
    state and last logits.  Beside it: the distance to the ggml-order oracle (variant 0) and the
    oracle's own noise band -- variant 1 (reversed accumulation order, otherwise identical) against
    variant 0 on the same tokens.  Every matmul re-quantizes its input to Q8, so one last-bit
    difference can flip a rounding step; over many tokens a random-weight model amplifies such
    flips, and the noise band shows how far two valid restatements of the reference drift apart."""
    from oracle_ctypes import VARIANT_GPU, set_variant
    ntok = len(tokens)

    def oracle_run(variant):
        set_variant(variant)
        try:
            return om.eval_serial(tokens)
        finally:
            set_variant(0)

    # the distance to the ggml-order oracle after 1, 2, 4, ... tokens: at token 1 nothing has been
    # amplified yet, so it shows the association's own error; later tokens show the Q8 flips growing
    checks = sorted({n for n in (1, 2, 4, 8, 16, 32, 64, 128) if n < ntok} | {ntok})
    assert L.rwkv_mi355x_state_upload(ctx.ptr, None)
    glg = np.zeros(n_vocab, np.float32)
    glg_at = {}
    for i in range(ntok):
        _, p_ = tok_arr([tokens[i]])
        want = (i + 1) in checks
        assert L.rwkv_mi355x_eval_device(ctx.ptr, p_, 1, want, glg.ctypes.data_as(P_F) if want else None, want)
        if want:
            glg_at[i + 1] = glg.copy()
    gst = np.zeros(state_len, np.float32)
    assert L.rwkv_mi355x_state_download(ctx.ptr, gst.ctypes.data_as(P_F))
    t = time.time()
    set_variant(0)
    growth = []
    try:
        st = None
        for i in range(ntok):
            lg, st = om.eval_sequence([tokens[i]], st)
            if (i + 1) in checks:
                growth.append({'tokens': i + 1, 'max_abs_dlogit': float(np.abs(glg_at[i + 1] - lg).max()),
                               'max_abs_logit': float(np.abs(lg).max())})
    finally:
        set_variant(0)
    blg, bst = oracle_run(VARIANT_GPU)
    lg_ne = int(np.count_nonzero(glg.view(np.uint32) != blg.view(np.uint32)))
    st_ne = int(np.count_nonzero(gst.view(np.uint32) != bst.view(np.uint32)))
    # the noise band: the largest distance any re-associated oracle variant (1..7: reversed
    # accumulation order, scalar ggml dot, fp32 accumulators -- tests/oracle_ctypes.py noise_band)
    # keeps from variant 0 on the same tokens
    band_lg, band_st, worst = 0.0, 0.0, 0
    for v in range(1, 8):
        nlg, nst = oracle_run(v)
        dl = float(np.abs(nlg - olg0).max())
        if dl > band_lg:
            band_lg, worst = dl, v
        band_st = max(band_st, float(np.abs(nst - ost0).max()))
    log(f'parity oracle runs (GPU association + variants 1..7, {ntok} tokens each): {time.time() - t:.1f}s')
    parity = {
        'bit_exact_vs_gpu_association_oracle': lg_ne == 0 and st_ne == 0, 'bit_exact_tokens': ntok,
        'logits_differing': lg_ne, 'state_values_differing': st_ne, 'tokens': ntok,
        'vs': 'oracle variant 0 (ggml CPU numerics, ggml summation order)',
        'max_abs_dlogit': float(np.abs(glg - olg0).max()),
        'max_abs_dstate': float(np.abs(gst - ost0).max()),
        'max_abs_logit': float(np.abs(olg0).max()),
        'noise_band': {'what': 'largest distance of oracle variants 1..7 (re-associated restatements: reversed '
                               'order, scalar ggml dot, fp32 accumulators) from variant 0, same tokens',
                       'max_abs_dlogit': band_lg, 'max_abs_dstate': band_st, 'widest_variant': worst},
        'within_1p5x_band': float(np.abs(glg - olg0).max()) <= 1.5 * max(band_lg, 1e-3),
        'dlogit_vs_ggml_order_by_tokens': growth,
        'tolerance_note': 'north-star 1e-3 logit bound applies to the FP32 fixtures (tests/test_gpu_parity.py); '
                          'on quantized weights two valid restatements differ by the noise band',
    }
    log(f"parity: bit-exact vs GPU-association oracle over {ntok} tokens: {parity['bit_exact_vs_gpu_association_oracle']}"
        f" (logits differing {lg_ne}, state values differing {st_ne}); vs ggml-order oracle: max|dlogit| "
        f"{parity['max_abs_dlogit']:.3g}, oracle noise band {parity['noise_band']['max_abs_dlogit']:.3g}; by tokens "
        + ' '.join(f"{g['tokens']}:{g['max_abs_dlogit']:.2g}" for g in growth))
    return parity


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=256)
    ap.add_argument('--warmup', type=int, default=16)
    ap.add_argument('--config', default='v6-1b6-q4_0', choices=sorted(CONFIGS))
    ap.add_argument('--seq-len', type=int, default=1024)
    ap.add_argument('--seq-reps', type=int, default=3)
    ap.add_argument('--abi-steps', type=int, default=32)
    ap.add_argument('--pipe-stages', type=int, default=-1,
                    help='N = 1: stages of the one-GPU pipeline run (-1: 4; 0: skip the pipeline leg); N > 1: N')
    ap.add_argument('--timing-steps', type=int, default=8)
    ap.add_argument('--cpu-seconds', type=float, default=12.0)
    ap.add_argument('--skip-cpu', action='store_true')
    ap.add_argument('--batch', default='8,32,64,128', help='batched decode sizes (contexts per step; "" = none)')
    ap.add_argument('--batch-steps', type=int, default=32)
    ap.add_argument('--model-dir', default=os.environ.get('RWKV_BENCH_DIR', '/tmp/rwkv_bench'))
    ap.add_argument('--roofline-only', action='store_true',
                    help='only the roofline timing pass (eager decode steps, per-dispatch events): the run whose '
                         'rocprofv3 trace must reproduce the line\'s roofline (profiles/)')
    ap.add_argument('--decode-only', action='store_true',
                    help='only the timed device-resident decode (warmup + steps, graph replays): the run a '
                         'rocprofv3 kernel trace of the decode chain is taken from (profiles/)')
    args = ap.parse_args()
    errors = []  # any entry makes the run exit non-zero after the JSON line

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    # RWKV_BENCH_BACKEND=gloo: rehearsal of the multi-rank code on fewer GPUs (ranks share GPUs,
    # messages go through host memory); the real runs use nccl (RCCL), one GPU per rank
    backend = os.environ.get('RWKV_BENCH_BACKEND', 'nccl')
    import torch
    import torch.distributed as dist
    gpu = local_rank % max(1, torch.cuda.device_count()) if backend == 'gloo' else local_rank
    os.environ.setdefault('RWKV_MI355X_DEVICE', str(gpu))
    if world > 1:
        torch.cuda.set_device(gpu)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', gpu))
        else:
            dist.init_process_group(backend)
    wire = torch.device('cuda', gpu) if backend == 'nccl' else torch.device('cpu')

    def barrier():
        if world > 1:
            dist.barrier()

    def allmax(v):
        t = torch.tensor([v], device=wire)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    import rwkv_cpp
    # RWKV_MI355X_BENCH_LIB: an alternative build of the same library for A/B runs (tools/r4_quick.sh)
    lib = rwkv_cpp.RWKVSharedLibrary(os.environ.get('RWKV_MI355X_BENCH_LIB')
                                     or os.path.join(REPO, 'rwkv.cppy_amd', 'build', 'librwkv.so'))
    L = lib.library
    arch, V, C, NL, F, fmt, label = CONFIGS[args.config]
    os.makedirs(args.model_dir, exist_ok=True)
    path = os.path.join(args.model_dir, f'{args.config}-seed1.bin')
    if rank == 0 and not os.path.isfile(path):
        t = time.time()
        tmp = path + '.tmp'
        assert L.rwkv_mi355x_write_synthetic_model(tmp.encode(), arch, V, C, NL, F, fmt.encode(), 1)
        os.replace(tmp, path)
        log(f'wrote synthetic {label} ({os.path.getsize(path) / 1e9:.2f} GB) in {time.time() - t:.1f}s')
    barrier()

    t = time.time()
    ctx = lib.rwkv_init_from_file(path, 1, NL + 1)
    log(f'rank {rank}: loaded {label} in {time.time() - t:.1f}s  [{lib.rwkv_get_system_info_string()}]')
    n_vocab = L.rwkv_get_n_vocab(ctx.ptr)
    state_len = L.rwkv_get_state_len(ctx.ptr)
    rng = np.random.default_rng(1234 + rank)
    P_INT = ctypes.POINTER(ctypes.c_int32)
    P_F = ctypes.POINTER(ctypes.c_float)

    def tok_arr(toks):
        a = np.ascontiguousarray(np.asarray(toks, dtype=np.int32))
        return a, a.ctypes.data_as(P_INT)

    # ---------------- self-check (every config, before any timing) ----------------
    # serial decode (the matvec kernels) and one sequence evaluation (the GEMM / sequence kernels) must
    # give the same bits on the same tokens -- the library's invariant; a fast kernel that drops work
    # breaks it, so no speed is reported from a build that fails it
    # (skipped in the roofline-only profiling pass, whose kernel trace must hold the timed launches only)
    sc_toks = [int(t) for t in np.random.default_rng(99).integers(0, n_vocab, 0 if args.roofline_only else 12)]
    sc_st, sc_st2 = np.zeros(state_len, np.float32), np.zeros(state_len, np.float32)
    sc_lg, sc_lg2 = np.zeros(n_vocab, np.float32), np.zeros(n_vocab, np.float32)
    L.rwkv_init_state(ctx.ptr, sc_st.ctypes.data_as(P_F))
    for t in sc_toks:
        assert L.rwkv_eval(ctx.ptr, t, sc_st.ctypes.data_as(P_F), sc_st.ctypes.data_as(P_F), sc_lg.ctypes.data_as(P_F))
    sca, scp = tok_arr(sc_toks)
    if sc_toks:
        assert L.rwkv_eval_sequence(ctx.ptr, scp, len(sc_toks), None, sc_st2.ctypes.data_as(P_F),
                                    sc_lg2.ctypes.data_as(P_F))
    self_check = {'decode_equals_sequence_bits': bool(np.array_equal(sc_lg.view(np.uint32), sc_lg2.view(np.uint32)) and
                                                      np.array_equal(sc_st.view(np.uint32), sc_st2.view(np.uint32))),
                  'tokens': len(sc_toks)}
    log(f"self-check: serial decode == sequence eval bit for bit over {len(sc_toks)} tokens: "
        f"{self_check['decode_equals_sequence_bits']}")

    assert L.rwkv_mi355x_state_upload(ctx.ptr, None)

    # ---------------- decode (device-resident state) ----------------
    dec_tokens = rng.integers(0, n_vocab, size=args.warmup + args.steps)
    arrs = [tok_arr([int(t)]) for t in dec_tokens]

    def step(i):
        if not L.rwkv_mi355x_eval_device(ctx.ptr, arrs[i][1], 1, True, None, False):
            raise RuntimeError('eval_device failed')

    for i in range(args.warmup):
        step(i)
    L.rwkv_mi355x_sync(ctx.ptr)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + (0 if args.roofline_only else args.steps)):
        step(i)
    L.rwkv_mi355x_sync(ctx.ptr)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = allmax(elapsed)
    if args.roofline_only:
        # no timed decode steps ran: this line carries the roofline pass only (profiles/), never a rate
        ms_per_step, value = None, None
    else:
        ms_per_step = elapsed * 1e3 / args.steps
        value = world * args.steps / elapsed
        log(f'decode: {ms_per_step * 1e3:.1f} us/token, {value:.1f} tok/s aggregate over {world} GPU(s)')
    if args.decode_only or args.roofline_only:
        args.batch, args.seq_reps, args.abi_steps, args.skip_cpu = '', 0, 0, True

    # ---------------- batched multi-context decode ----------------
    # B independent contexts advance one token each per step (rwkv_mi355x_eval_batch_device: states
    # and logits in HBM, two state buffers alternating); tokens/s = B * steps / time
    batch = []
    for B in [int(b) for b in args.batch.split(',') if b.strip()]:
        try:
            dev = torch.device('cuda', gpu)
            sbuf = [torch.zeros((B, state_len), dtype=torch.float32, device=dev) for _ in range(2)]
            lbuf = torch.zeros((B, n_vocab), dtype=torch.float32, device=dev)
            btoks = rng.integers(0, n_vocab, size=(args.batch_steps + 4, B)).astype(np.uint32)

            def bstep(i, fresh=False):
                sin = None if fresh else sbuf[i & 1].data_ptr()
                if not L.rwkv_mi355x_eval_batch_device(ctx.ptr, btoks[i].ctypes.data, B, sin,
                                                       sbuf[(i & 1) ^ 1].data_ptr(), lbuf.data_ptr()):
                    raise RuntimeError('eval_batch_device failed')

            torch.cuda.synchronize()
            bstep(0, fresh=True)
            for i in range(1, 4):
                bstep(i)
            L.rwkv_mi355x_sync(ctx.ptr)
            barrier()
            tb = time.perf_counter()
            for i in range(4, 4 + args.batch_steps):
                bstep(i)
            L.rwkv_mi355x_sync(ctx.ptr)
            barrier()
            eb = time.perf_counter() - tb
            if world > 1:
                eb = allmax(eb)
            batch.append({'contexts': B, 'tokens_per_s': round(world * B * args.batch_steps / eb, 1),
                          'ms_per_step': round(eb * 1e3 / args.batch_steps, 4),
                          'tokens_per_s_per_context': round(args.batch_steps / eb, 1)})
            log(f'batched decode B={B}: {eb * 1e3 / args.batch_steps:.3f} ms/step, '
                f'{world * B * args.batch_steps / eb:.0f} tok/s aggregate')
            del sbuf, lbuf
        except Exception as e:
            log(f'batched decode B={B} failed: {e!r}')
            errors.append(f'batched decode B={B}: {e!r}')
            batch.append({'contexts': B, 'error': repr(e)})

    # ---------------- sequence eval ----------------
    seq = rng.integers(0, n_vocab, size=args.seq_len)
    sa, sp = tok_arr(seq)
    assert L.rwkv_mi355x_state_upload(ctx.ptr, None)
    assert L.rwkv_mi355x_eval_device(ctx.ptr, sp, len(seq), True, None, True)  # warm-up / workspace
    ts = []
    for _ in range(max(args.seq_reps, 0)):
        assert L.rwkv_mi355x_state_upload(ctx.ptr, None)
        L.rwkv_mi355x_sync(ctx.ptr)
        t1 = time.perf_counter()
        assert L.rwkv_mi355x_eval_device(ctx.ptr, sp, len(seq), True, None, True)
        ts.append(time.perf_counter() - t1)
    seq_s = min(ts) if ts else float('nan')
    seq_tps = args.seq_len / seq_s if ts else 0.0
    log(f'seq-eval T={args.seq_len}: {seq_s * 1e3:.1f} ms, {seq_tps:.0f} tok/s')

    # ---------------- sequence eval with the chunk-parallel wkv6 (v5/v6; off by default) ----------------
    # csrc/wkv_chunk.hip re-associates the recurrence (not bit-exact), so it is a separate, labelled
    # number; the headline seq_eval above is the serial, bit-exact path
    wkvc = None
    if args.seq_reps > 0 and arch in (5, 6):
        try:
            slg0 = np.zeros(n_vocab, np.float32)
            clg = np.zeros(n_vocab, np.float32)
            assert L.rwkv_eval_sequence(ctx.ptr, sp, len(seq), None, None, slg0.ctypes.data_as(P_F))
            assert L.rwkv_mi355x_debug_set(ctx.ptr, b'wkv_chunk', 1)
            assert L.rwkv_eval_sequence(ctx.ptr, sp, len(seq), None, None, clg.ctypes.data_as(P_F))
            cts = []
            for _ in range(args.seq_reps):
                assert L.rwkv_mi355x_state_upload(ctx.ptr, None)
                L.rwkv_mi355x_sync(ctx.ptr)
                t1 = time.perf_counter()
                assert L.rwkv_mi355x_eval_device(ctx.ptr, sp, len(seq), True, None, True)
                cts.append(time.perf_counter() - t1)
            assert L.rwkv_mi355x_debug_set(ctx.ptr, b'wkv_chunk', 0)
            wkvc = {'tokens_per_s': round(args.seq_len / min(cts) * world, 1), 'ms_per_sequence': round(min(cts) * 1e3, 3),
                    'what': 'seq_eval with RWKV_MI355X_WKV_CHUNK=1 (chunk-parallel wkv6, 16-token chunks, '
                            're-associated: not bit-exact, off by default)',
                    'max_abs_dlogit_vs_serial': float(np.abs(clg - slg0).max()),
                    'max_abs_logit': float(np.abs(slg0).max())}
            log(f"seq-eval, chunk-parallel wkv6: {min(cts) * 1e3:.1f} ms, {args.seq_len / min(cts):.0f} tok/s, "
                f"max|dlogit| vs serial {wkvc['max_abs_dlogit_vs_serial']:.3g}")
        except Exception as e:
            log(f'chunked wkv seq-eval failed: {e!r}')
            errors.append(f'chunked wkv seq-eval: {e!r}')

    # ---------------- sequence eval through the in-library layer pipeline ----------------
    # rwkv_mi355x_init_pipeline: ONE process drives P stage contexts (stage s on GPU devices[s], layers
    # [s*L/P, (s+1)*L/P)); rwkv_eval_sequence on it cuts the tokens into chunks of >= 256 and forwards
    # each chunk's residual stream stage to stage by a peer copy over xGMI (csrc/pipeline.cpp) -- the
    # path rwkv_eval_sequence ships.  N > 1: rank 0 drives all N GPUs while the other ranks wait at a
    # barrier (strong scaling of one sequence).  N = 1: the same schedule with every stage on GPU 0,
    # so its own overhead against one context is a number.
    pipe = None
    if args.seq_reps > 0 and args.pipe_stages != 0:
        P = world if world > 1 else (args.pipe_stages if args.pipe_stages > 0 else 4)
        P = max(2, min(P, NL))
        if rank == 0:
            try:
                ndev = torch.cuda.device_count()
                devices = [d % max(1, ndev) for d in range(P)] if world > 1 else [gpu] * P
                devs = (ctypes.c_int * P)(*devices)
                t = time.time()
                pctx = L.rwkv_mi355x_init_pipeline(path.encode(), 1, P, devs)
                if not pctx:
                    raise RuntimeError('rwkv_mi355x_init_pipeline failed')
                log(f'pipeline: {P} stages on devices {devices} loaded in {time.time() - t:.1f}s')
                pseq = np.random.default_rng(4321).integers(0, n_vocab, size=args.seq_len)
                pa, pp_ = tok_arr(pseq)
                plg = np.zeros(n_vocab, np.float32)

                def run_pipe():
                    if not L.rwkv_eval_sequence(pctx, pp_, len(pseq), None, None, plg.ctypes.data_as(P_F)):
                        raise RuntimeError('pipeline rwkv_eval_sequence failed')

                run_pipe()  # warm-up: workspaces, staging buffers
                pts = []
                for _ in range(args.seq_reps):
                    t1 = time.perf_counter()
                    run_pipe()
                    pts.append(time.perf_counter() - t1)
                # the same sequence through one context: pipeline logits must be bit-identical
                slg = np.zeros(n_vocab, np.float32)
                assert L.rwkv_eval_sequence(ctx.ptr, pp_, len(pseq), None, None, slg.ctypes.data_as(P_F))
                chunk = -(-args.seq_len // (2 * P))  # LayerPipeline::pick_chunk: ceil(T / 2P) in whole 64-token
                chunk = min(args.seq_len, max(256, -(-chunk // 64) * 64))  # tiles, at least 256, at most T
                pairs = L.rwkv_mi355x_pipeline_peer_pairs(pctx)
                pipe = {'tokens_per_s': round(args.seq_len / min(pts), 1), 'ms_per_sequence': round(min(pts) * 1e3, 3),
                        'stages': P, 'devices': devices, 'peer_pairs': pairs, 'chunk': chunk, 'T': args.seq_len,
                        'parallelism': f'layer pipeline x{P} (one process, rwkv_mi355x_init_pipeline)',
                        'scaling': 'strong',
                        'transport': ('hipMemcpyPeerAsync over xGMI, peer access enabled' if pairs else
                                      'device-local copies (every stage on one GPU)'),
                        'bit_exact_vs_single_context': bool(np.array_equal(plg.view(np.uint32), slg.view(np.uint32))),
                        'single_context_ms_per_sequence': round(seq_s * 1e3, 3),
                        'overhead_vs_single_context': round(min(pts) / seq_s, 4) if world == 1 else None,
                        'stage_weight_gb': round(L.rwkv_mi355x_weight_bytes(ctx.ptr, True) / 1e9 / P, 4)}
                L.rwkv_free(pctx)
                log(f'pipeline seq-eval, {P} stages on {devices}: {min(pts) * 1e3:.1f} ms ({args.seq_len / min(pts):.0f} '
                    f'tok/s, chunk {chunk}, peer pairs {pairs}); one context {seq_s * 1e3:.1f} ms; bit-exact '
                    f'{pipe["bit_exact_vs_single_context"]}')
                if not pipe['bit_exact_vs_single_context']:
                    errors.append('pipeline: logits differ from one context')
            except Exception as e:  # the decode line is still printed; the run exits non-zero
                errors.append(f'pipeline: {e!r}')
                log(f'pipeline seq-eval failed: {e!r}')
        barrier()

    # ---------------- ABI-level decode (host state, reference contract) ----------------
    state = np.zeros(state_len, np.float32)
    logits = np.zeros(n_vocab, np.float32)
    L.rwkv_init_state(ctx.ptr, state.ctypes.data_as(P_F))
    L.rwkv_eval(ctx.ptr, int(dec_tokens[0]), state.ctypes.data_as(P_F), state.ctypes.data_as(P_F),
                logits.ctypes.data_as(P_F))
    t2 = time.perf_counter()
    for i in range(args.abi_steps):
        assert L.rwkv_eval(ctx.ptr, int(dec_tokens[i % len(dec_tokens)]), state.ctypes.data_as(P_F), state.ctypes.data_as(P_F),
                           logits.ctypes.data_as(P_F))
    abi_tps = args.abi_steps / (time.perf_counter() - t2) if args.abi_steps > 0 else 0.0
    log(f'ABI decode (host state {state_len * 4 / 1e6:.1f} MB each way): {abi_tps:.1f} tok/s')
    # the same calls with page-locked state / logits buffers (torch pin_memory); both kinds of
    # caller buffer take engine.hip eval_host_chunked
    abi_pinned_tps = 0.0
    if args.abi_steps > 0:
        try:
            pst = torch.zeros(state_len, dtype=torch.float32).pin_memory()
            plg = torch.zeros(n_vocab, dtype=torch.float32).pin_memory()
            pp, pl = ctypes.cast(pst.data_ptr(), P_F), ctypes.cast(plg.data_ptr(), P_F)
            L.rwkv_init_state(ctx.ptr, pp)
            for i in range(2):
                assert L.rwkv_eval(ctx.ptr, int(dec_tokens[i]), pp, pp, pl)
            t2 = time.perf_counter()
            for i in range(args.abi_steps):
                assert L.rwkv_eval(ctx.ptr, int(dec_tokens[i % len(dec_tokens)]), pp, pp, pl)
            abi_pinned_tps = args.abi_steps / (time.perf_counter() - t2)
            log(f'ABI decode, page-locked host state: {abi_pinned_tps:.1f} tok/s')
        except Exception as e:
            log(f'ABI decode (page-locked) failed: {e!r}')

    # ---------------- kernel timing (HIP events on the context stream) ----------------
    def read_stats():
        n = L.rwkv_mi355x_kernel_stats(ctx.ptr, -1, None, 0, None, None, None, None)
        out = []
        for i in range(n):
            name = ctypes.create_string_buffer(128)
            la, ms, by, fl = ctypes.c_longlong(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
            L.rwkv_mi355x_kernel_stats(ctx.ptr, i, name, 128, ctypes.byref(la), ctypes.byref(ms), ctypes.byref(by),
                                       ctypes.byref(fl))
            if la.value > 0:
                out.append(dict(name=name.value.decode(), launches=la.value, ms=ms.value, bytes=by.value,
                                flops=fl.value))
        return sorted(out, key=lambda k: -k['ms'])

    roofline = None
    timing_steps = max(1, args.timing_steps)
    try:
        if args.decode_only:
            raise StopIteration
        assert L.rwkv_mi355x_state_upload(ctx.ptr, None)
        L.rwkv_mi355x_set_kernel_timing(ctx.ptr, True)
        for i in range(timing_steps):
            # a lead kernel per step: the step's launches queue up behind it and then run back to
            # back -- the same conditions with and without a profiler attached (profiles/)
            assert L.rwkv_mi355x_debug_set(ctx.ptr, b'delay_us', 4000)
            step(i % len(arrs))
            L.rwkv_mi355x_sync(ctx.ptr)
        kstats = read_stats()
        L.rwkv_mi355x_set_kernel_timing(ctx.ptr, False)
        for k in kstats:
            log(f"  {k['name']:<18} launches {k['launches']:5d} avg {k['ms'] / k['launches'] * 1e3:8.2f} us "
                f"{k['bytes'] / k['launches'] / 1e6:8.3f} MB/launch -> {k['bytes'] / k['ms'] / 1e6:8.1f} GB/s")
        # the dominant kernel class: the decode kernels that stream the weights -- every k_mv
        # (LayerNorm-prologue groups, head) / k_mva (activation-input groups) launch, the fused v6
        # maa launch and the fused v6 r,k,v,g + attention launch -- pooled; each launch timed by an
        # event pair bound to its own dispatch (hipExtLaunchKernelGGL: the begin / end timestamps a
        # rocprofv3 kernel trace reports), on the engine's stream, over timing_steps eager decode steps
        pool = [k for k in kstats if k['name'] in STREAM_KERNELS and k['bytes'] > 0]
        if not pool:
            raise RuntimeError('no decode kernel timings recorded')
        p_ms = sum(k['ms'] for k in pool)
        p_launches = sum(k['launches'] for k in pool)
        p_bytes = sum(k['bytes'] for k in pool)
        avg_us = p_ms / p_launches * 1e3
        bytes_per_launch = p_bytes / p_launches
        achieved = bytes_per_launch / (avg_us * 1e-6) / 1e9
        traffic = None
        pmc = os.path.join(REPO, 'profiles', 'pmc_traffic.json')
        if os.path.isfile(pmc):
            t = json.load(open(pmc)).get(args.config, {}).get('decode_stream')
            if t:
                traffic = t['traffic_bytes_per_launch']
        dbytes = L.rwkv_mi355x_decode_bytes(ctx.ptr, True)
        all_ms = sum(k['ms'] for k in kstats)
        roofline = {
            'kernel': 'decode weight-streaming kernels (' + ', '.join(sorted(k['name'] for k in pool)) + '), pooled',
            'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': traffic,
            'avg_launch_us': round(avg_us, 3), 'algorithmic_bytes_per_launch': round(bytes_per_launch),
            'launches_per_token': round(p_launches / timing_steps, 1),
            'method': 'per-dispatch HIP events (hipExtLaunchKernelGGL start/stop: the dispatch timestamps '
                      'rocprofv3 reports) on the engine stream over '
                      f'{timing_steps} eager decode steps, each queued behind a 4 ms lead kernel so its launches '
                      'run back to back; profiles/ holds the rocprofv3 kernel trace of this pass '
                      '(bench.py --roofline-only, reproduces these averages) and of the graph-replayed decode '
                      '(bench.py --decode-only, which the profiler itself slows down)',
            'per_kernel': {k['name']: {'launches_per_token': round(k['launches'] / timing_steps, 1),
                                       'avg_us': round(k['ms'] / k['launches'] * 1e3, 3),
                                       'GBps': round(k['bytes'] / (k['ms'] * 1e-3) / 1e9, 1) if k['bytes'] else None}
                           for k in kstats},
            'kernel_time_us_per_token': round(all_ms / timing_steps * 1e3, 1),
            'decode_bytes_per_token': round(dbytes),
            'decode_GBps_end_to_end': round(dbytes / (ms_per_step * 1e-3) / 1e9, 1) if ms_per_step else None,
            'decode_frac_end_to_end': (round(dbytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                       if ms_per_step else None),
        }
    except StopIteration:
        pass
    except Exception as e:
        errors.append(f'roofline: {e!r}')
        log(f'roofline failed: {e!r}')
        L.rwkv_mi355x_set_kernel_timing(ctx.ptr, False)

    # ---------------- sequence GEMM MFMA utilisation (same run, HIP events) ----------------
    seq_roofline = None
    if args.seq_reps > 0:
        try:
            assert L.rwkv_mi355x_state_upload(ctx.ptr, None)
            L.rwkv_mi355x_set_kernel_timing(ctx.ptr, True)
            assert L.rwkv_mi355x_eval_device(ctx.ptr, sp, len(seq), True, None, True)
            sstats = read_stats()
            L.rwkv_mi355x_set_kernel_timing(ctx.ptr, False)
            g = [k for k in sstats if k['name'].startswith('k_qgemm')]
            if not g:
                raise RuntimeError('no k_qgemm timings recorded')
            ms = sum(k['ms'] for k in g)
            flops = sum(k['flops'] for k in g)
            tops = flops / (ms * 1e-3) / 1e12
            other = [k for k in sstats if not k['name'].startswith('k_qgemm')]
            seq_roofline = {
                'kernel': 'k_qgemm (all int8-MFMA sequence GEMM launches)', 'bound': 'mfma',
                'achieved': round(tops, 1), 'peak': INT8_MFMA_PEAK_TOPS, 'unit': 'TOP/s',
                'frac': round(tops / INT8_MFMA_PEAK_TOPS, 4), 'launches': sum(k['launches'] for k in g),
                'ms_per_sequence': round(ms, 3), 'algorithmic_ops': flops,
                'share_of_seq_eval': round(ms / (seq_s * 1e3), 3) if ts else None,
                'other_matmul_ms': round(sum(k['ms'] for k in other), 3),
            }
            log(f"seq GEMM: {ms:.2f} ms per sequence, {tops:.1f} TOP/s = {100 * tops / INT8_MFMA_PEAK_TOPS:.1f}% "
                f"of the int8 MFMA peak")
        except Exception as e:
            errors.append(f'seq_roofline: {e!r}')
            log(f'seq roofline failed: {e!r}')
            L.rwkv_mi355x_set_kernel_timing(ctx.ptr, False)

    # ---------------- CPU baseline + parity of this run's model (oracle = CPU restatement) ----------------
    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.skip_cpu:
        try:
            from oracle_ctypes import OracleModel, lib as olib
            threads = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or min(16, os.cpu_count() or 1)
            olib().oracle_set_threads(threads)
            t3 = time.time()
            om = OracleModel(path)
            load_s = time.time() - t3
            cpu_tokens = [int(t) for t in np.random.default_rng(99).integers(0, n_vocab, size=256)]
            st = None
            olg = None
            ntok = 0
            t4 = time.perf_counter()
            while ntok < len(cpu_tokens):
                olg, st = om.eval_sequence([cpu_tokens[ntok]], st)
                ntok += 1
                if time.perf_counter() - t4 >= args.cpu_seconds:
                    break
            cpu_s = time.perf_counter() - t4
            cpu = {'value': round(ntok / cpu_s, 3), 'unit': 'tokens/s', 'cores': olib().oracle_get_threads(),
                   'threads': olib().oracle_get_threads(), 'host_cpus': os.cpu_count(),
                   'host_physical_cores': physical_cores(),
                   'kind': 'port',
                   'sample': f'{label} single-token decode (logits on), {ntok} tokens from a fresh state, '
                             f'{cpu_s:.1f}s; oracle/ C restatement of the reference CPU arithmetic '
                             f'(ggml Q8 activation quantization + int8 block dots), OpenMP over rows; cores = OpenMP '
                             f'threads used (OMP_NUM_THREADS, else min(16, host CPUs)), host_cpus = os.cpu_count() '
                             f'(logical), host_physical_cores = distinct (package, core) pairs in /proc/cpuinfo'}
            log(f'cpu baseline: {cpu["value"]} tok/s on {cpu["cores"]} threads (load {load_s:.1f}s)')
        except Exception as e:
            errors.append(f'cpu_baseline: {e!r}')
            log(f'cpu baseline failed: {e!r}')
        if cpu is not None:
            try:
                parity = decode_parity(L, ctx, om, cpu_tokens[:ntok], olg, st, n_vocab, state_len, tok_arr, P_F)
            except Exception as e:
                errors.append(f'parity: {e!r}')
                log(f'parity failed: {e!r}')
            om.close()

    L.rwkv_free(ctx.ptr)
    if rank == 0:
        out = {
            'metric': METRIC, 'value': round(value, 2) if value is not None else None, 'unit': 'tokens/s',
            'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 5) if ms_per_step is not None else None,
            'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': f'i8 ({fmt[:2].lower()} x q8 int8 dot) + f32', 'data': 'synthetic',
            'config': {'workload': f'{label} single-token decode (rwkv_eval semantics, logits on), '
                                   f'state resident in HBM', 'n_embed': C, 'n_layer': NL, 'n_vocab': V,
                       'weights': fmt, 'parallelism': f'replicas x{world}'},
            'seq_eval': {'tokens_per_s': round(seq_tps * world, 1), 'T': args.seq_len,
                         'ms_per_sequence': round(seq_s * 1e3, 3), 'parallelism': f'replicas x{world}',
                         'pipeline': pipe, 'wkv_chunked': wkvc},
            'abi_decode_tokens_per_s': round(abi_tps * world, 2),
            'abi_decode_pinned_tokens_per_s': round(abi_pinned_tps * world, 2),
            'batched_decode': {'what': 'B independent contexts, one token each per step, weights read once per '
                                       'step (rwkv_mi355x_eval_batch_device; bit-exact to per-context rwkv_eval)',
                               'parallelism': f'replicas x{world}', 'runs': batch},
            'roofline': roofline,
            'seq_roofline': seq_roofline,
            'cpu_baseline': cpu,
            'parity': parity,
            'self_check': self_check,
        }
        # every requested field must be present: a missing one fails the run (after the line)
        if world == 1 and not args.skip_cpu:
            if cpu is None:
                errors.append('cpu_baseline missing')
            if parity is None:
                errors.append('parity missing')
            elif not parity['bit_exact_vs_gpu_association_oracle']:
                errors.append('parity: GPU decode not bit-exact to the GPU-association oracle')
        if sc_toks and not self_check['decode_equals_sequence_bits']:
            errors.append('self-check: serial decode and sequence evaluation differ')
        if roofline is None and not args.decode_only:
            errors.append('roofline missing')
        if args.seq_reps > 0 and seq_roofline is None:
            errors.append('seq_roofline missing')
        if args.seq_reps > 0 and args.pipe_stages != 0 and pipe is None:
            errors.append('seq_eval.pipeline missing')
        if args.roofline_only:
            out['not_a_measurement'] = 'roofline-only pass: no timed decode steps; value / ms_per_step are null'
        if errors:
            out['errors'] = errors
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if errors:
        log(f'FAILED: {errors}')
        sys.exit(1)


if __name__ == '__main__':
    main()
