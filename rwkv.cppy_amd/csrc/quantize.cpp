// quantize.cpp -- model-file tooling on the host: rwkv_quantize_model_file (reference
// rwkv_quantize.inc:1-171, the ggml quantize_row_*_ref block formats it calls) and the
// synthetic-model writer used by bench.py (exact tensor shapes of real checkpoints, as written
// by the reference's python/convert_pytorch_to_ggml.py:28-161).
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <exception>
#include <sys/stat.h>

#include <algorithm>
#include <cfloat>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rwkv_mi355x.h"
#include "common.hpp"
#include "model_file.hpp"

namespace rwkvmi {

static inline void put_f16(uint8_t * p, float f) {
    const uint16_t h = f32_to_f16(f);
    memcpy(p, &h, 2);
}

// One row of k floats -> k/32 blocks of `type` (ggml reference quantizers).
void quantize_row(uint32_t type, const float * x, uint8_t * y, int64_t k) {
    const int64_t nb = k / 32;
    for (int64_t i = 0; i < nb; i++) {
        const float * xb = x + i * 32;
        if (type == W_Q4_0 || type == W_Q5_0) {
            float amax = 0.0f, max = 0.0f;
            for (int j = 0; j < 32; j++)
                if (amax < fabsf(xb[j])) {
                    amax = fabsf(xb[j]);
                    max = xb[j];
                }
            if (type == W_Q4_0) {
                uint8_t * b = y + i * 18;
                const float d = max / -8, id = d ? 1.0f / d : 0.0f;
                put_f16(b, d);
                for (int j = 0; j < 16; j++) {
                    const int a0 = std::min(15, (int)(int8_t)(xb[j] * id + 8.5f));
                    const int a1 = std::min(15, (int)(int8_t)(xb[16 + j] * id + 8.5f));
                    b[2 + j] = (uint8_t)(a0 | (a1 << 4));
                }
            } else {
                uint8_t * b = y + i * 22;
                const float d = max / -16, id = d ? 1.0f / d : 0.0f;
                put_f16(b, d);
                uint32_t qh = 0;
                for (int j = 0; j < 16; j++) {
                    const int a0 = std::min(31, (int)(int8_t)(xb[j] * id + 16.5f));
                    const int a1 = std::min(31, (int)(int8_t)(xb[16 + j] * id + 16.5f));
                    b[6 + j] = (uint8_t)((a0 & 0x0f) | ((a1 & 0x0f) << 4));
                    qh |= (uint32_t)((a0 & 0x10) >> 4) << j;
                    qh |= (uint32_t)((a1 & 0x10) >> 4) << (j + 16);
                }
                memcpy(b + 2, &qh, 4);
            }
        } else if (type == W_Q4_1 || type == W_Q5_1) {
            float mn = FLT_MAX, mx = -FLT_MAX;
            for (int j = 0; j < 32; j++) {
                mn = std::min(mn, xb[j]);
                mx = std::max(mx, xb[j]);
            }
            if (type == W_Q4_1) {
                uint8_t * b = y + i * 20;
                const float d = (mx - mn) / 15, id = d ? 1.0f / d : 0.0f;
                put_f16(b, d);
                put_f16(b + 2, mn);
                for (int j = 0; j < 16; j++) {
                    const int a0 = std::min(15, (int)(int8_t)((xb[j] - mn) * id + 0.5f));
                    const int a1 = std::min(15, (int)(int8_t)((xb[16 + j] - mn) * id + 0.5f));
                    b[4 + j] = (uint8_t)(a0 | (a1 << 4));
                }
            } else {
                uint8_t * b = y + i * 24;
                const float d = (mx - mn) / 31, id = d ? 1.0f / d : 0.0f;
                put_f16(b, d);
                put_f16(b + 2, mn);
                uint32_t qh = 0;
                for (int j = 0; j < 16; j++) {
                    const uint8_t a0 = (uint8_t)((xb[j] - mn) * id + 0.5f);
                    const uint8_t a1 = (uint8_t)((xb[16 + j] - mn) * id + 0.5f);
                    b[8 + j] = (uint8_t)((a0 & 0x0f) | ((a1 & 0x0f) << 4));
                    qh |= (uint32_t)((a0 & 0x10) >> 4) << j;
                    qh |= (uint32_t)((a1 & 0x10) >> 4) << (j + 16);
                }
                memcpy(b + 4, &qh, 4);
            }
        } else if (type == W_Q8_0) {
            uint8_t * b = y + i * 34;
            float amax = 0.0f;
            for (int j = 0; j < 32; j++) amax = std::max(amax, fabsf(xb[j]));
            const float d = amax / 127, id = d ? 1.0f / d : 0.0f;
            put_f16(b, d);
            for (int j = 0; j < 32; j++) b[2 + j] = (uint8_t)(int8_t)roundf(xb[j] * id);
        }
    }
}

// Quantize an [rows][k] fp32 matrix with a few host threads (rows are independent).
static void quantize_matrix(uint32_t type, const float * x, uint8_t * y, int64_t rows, int64_t k) {
    const size_t row_bytes = (size_t)(k / 32) * type_block_bytes(type);
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (rows * k < (1 << 20)) nt = 1;
    std::vector<std::thread> th;
    for (unsigned w = 0; w < nt; w++) {
        th.emplace_back([=]() {
            for (int64_t r = w; r < rows; r += nt) quantize_row(type, x + r * k, y + r * row_bytes, k);
        });
    }
    for (auto & t : th) t.join();
}

// rwkv_quantize.inc:1-13
static bool tensor_needs_quant(const std::string & name) {
    static const char * skip[] = {"att.v1", "att.v2", "att.g1", "att.g2", "att.a1", "att.a2", "att.w1", "att.w2", "att.r_k"};
    if (name == "emb.weight" || name == "head.weight") return false;
    for (const char * s : skip)
        if (name.find(s) != std::string::npos) return false;
    return true;
}

bool quantize_model_file(const char * in_path, const char * out_path, const char * format) {
    g_last_error = RWKV_ERROR_NONE;
    const int out_type = type_from_name(format ? format : "");
    RWKV_CHECK(RWKV_ERROR_ARGS | RWKV_ERROR_DATA_TYPE, false, out_type >= 0 && type_quantized((uint32_t)out_type),
               "Unsupported output data type (%s)", format ? format : "(null)");
    FILE * in = fopen(in_path, "rb");
    RWKV_CHECK(RWKV_ERROR_FILE | RWKV_ERROR_FILE_OPEN, false, in != nullptr, "Failed to open %s for reading", in_path);
    struct stat st;
    if (fstat(fileno(in), &st) != 0) {
        fclose(in);
        RWKV_CHECK(RWKV_ERROR_FILE | RWKV_ERROR_FILE_STAT, false, false, "failed to stat file %s", in_path);
    }
    FILE * out = fopen(out_path, "wb");
    if (!out) {
        fclose(in);
        RWKV_CHECK(RWKV_ERROR_FILE | RWKV_ERROR_FILE_OPEN, false, false, "Failed to open %s for writing", out_path);
    }
    auto fail = [&](enum rwkv_error_flags fl, const char * msg) {
        fclose(in);
        fclose(out);
        add_error(fl);
        if (g_print_errors) fprintf(stderr, "%s\n", msg);
        return false;
    };
    FileHeader h;
    if (!read_file_header(in, h)) return fail(RWKV_ERROR_FILE, "Invalid file header");
    if (h.data_type != 0 && h.data_type != 1) return fail(RWKV_ERROR_FILE, "Unsupported input data type; needs to be FP32 or FP16");
    FileHeader oh = h;
    oh.version = RWKV_FILE_VERSION;
    oh.data_type = (uint32_t)out_type;
    if (fwrite(&oh, sizeof(oh), 1, out) != 1) return fail(RWKV_ERROR_FILE_WRITE, "Failed to write file header");
    std::vector<uint8_t> data, qbuf;
    std::vector<float> fbuf;
    while (ftello(in) < (off_t)st.st_size) {
        uint32_t th[3], ne[3] = {1, 1, 1};
        if (fread(th, 4, 3, in) != 3 || th[0] < 1 || th[0] > 3 || fread(ne, 4, th[0], in) != th[0] || !type_supported(th[2]))
            return fail(RWKV_ERROR_MODEL_PARAMS, "Failed to read tensor header");
        std::string name(th[1], '\0');
        if (th[1] && fread(&name[0], 1, th[1], in) != th[1]) return fail(RWKV_ERROR_MODEL_PARAMS, "Failed to read tensor name");
        const uint64_t n = (uint64_t)ne[0] * ne[1] * ne[2];
        const size_t nb = type_nbytes(th[2], n);
        data.resize(nb);
        if (nb && fread(data.data(), 1, nb, in) != nb) return fail(RWKV_ERROR_MODEL_PARAMS, "Failed to read tensor data");
        const uint8_t * payload = data.data();
        size_t payload_bytes = nb;
        if ((th[2] == 0 || th[2] == 1) && th[0] == 2 && tensor_needs_quant(name)) {
            fbuf.resize(n);
            if (th[2] == 1) {
                for (uint64_t i = 0; i < n; i++) {
                    uint16_t v;
                    memcpy(&v, data.data() + 2 * i, 2);
                    fbuf[i] = f16_to_f32(v);
                }
            } else {
                memcpy(fbuf.data(), data.data(), n * 4);
            }
            qbuf.resize(type_nbytes((uint32_t)out_type, n));
            quantize_matrix((uint32_t)out_type, fbuf.data(), qbuf.data(), ne[1], ne[0]);
            th[2] = (uint32_t)out_type;
            payload = qbuf.data();
            payload_bytes = qbuf.size();
        }
        if (fwrite(th, 4, 3, out) != 3 || fwrite(ne, 4, th[0], out) != th[0] ||
            (th[1] && fwrite(name.data(), 1, th[1], out) != th[1]) ||
            (payload_bytes && fwrite(payload, 1, payload_bytes, out) != payload_bytes))
            return fail(RWKV_ERROR_FILE_WRITE, "Failed to write tensor");
    }
    fclose(in);
    if (fclose(out) != 0) {
        add_error(RWKV_ERROR_FILE_WRITE);
        return false;
    }
    return true;
}

// ------------------------------------------------------------------ synthetic checkpoints

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0xD1B54A32D192ED03ull) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    float uniform() { return (float)((next() >> 40) * (1.0 / 16777216.0)); }  // [0,1)
    float normal() {  // Irwin-Hall(4) approximation, unit variance
        float s4 = uniform() + uniform() + uniform() + uniform();
        return (s4 - 2.0f) * 1.7320508f;
    }
};

struct SynthTensor {
    std::string name;
    std::vector<uint32_t> ne;  // ggml order
    enum Kind { MAT, ONES, ZEROS, UNIF, CUSTOM } kind;
    float lo = 0, hi = 1;      // UNIF range
    int custom = 0;            // 1: v4 decay  2: v5.2 decay
};

static uint64_t nel(const std::vector<uint32_t> & ne) {
    uint64_t n = 1;
    for (auto v : ne) n *= v;
    return n;
}

static void fill_tensor(const SynthTensor & t, float * x, uint64_t seed) {
    const uint64_t n = nel(t.ne);
    if (t.kind == SynthTensor::MAT) {
        const int64_t K = t.ne[0], rows = (int64_t)(n / K);
        const float sd = 1.0f / sqrtf((float)K);
        unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        if (n < (1u << 20)) nt = 1;
        std::vector<std::thread> th;
        for (unsigned w = 0; w < nt; w++)
            th.emplace_back([=]() {
                for (int64_t r = w; r < rows; r += nt) {
                    Rng g(seed * 1000003ull + (uint64_t)r);
                    for (int64_t k = 0; k < K; k++) x[r * K + k] = g.normal() * sd;
                }
            });
        for (auto & h : th) h.join();
        return;
    }
    Rng g(seed);
    for (uint64_t i = 0; i < n; i++) {
        switch (t.kind) {
            case SynthTensor::ONES: x[i] = 1.0f; break;
            case SynthTensor::ZEROS: x[i] = 0.0f; break;
            case SynthTensor::UNIF: x[i] = t.lo + (t.hi - t.lo) * g.uniform(); break;
            default: {
                const float u = g.uniform();
                if (t.custom == 1) x[i] = -expf(-1.0f + 2.0f * u);               // v4: -exp(w)
                else x[i] = expf(-expf(-6.0f + 5.0f * u));                       // v5.2: exp(-exp(w))
            }
        }
    }
}

static bool write_synthetic(const char * path, int arch, uint32_t V, uint32_t C, uint32_t L, uint32_t F,
                            const char * fmt, uint64_t seed) {
    const int ftype = type_from_name(fmt);
    if (ftype < 0 || !type_supported((uint32_t)ftype) || C % 64 || arch < 4 || arch > 7) return false;
    const uint32_t S = 64, H = arch >= 5 ? C / S : 0;
    if (F == 0) F = (arch == 4 || arch == 7) ? 4 * C : (C * 7) / 2;
    F = (F + 31) / 32 * 32;
    std::vector<SynthTensor> ts;
    auto mat = [&](const std::string & n, uint32_t K, uint32_t M) { ts.push_back({n, {K, M}, SynthTensor::MAT}); };
    auto vec = [&](const std::string & n, std::vector<uint32_t> ne, SynthTensor::Kind k, float lo = 0, float hi = 1, int cu = 0) {
        SynthTensor t{n, ne, k};
        t.lo = lo;
        t.hi = hi;
        t.custom = cu;
        ts.push_back(t);
    };
    mat("emb.weight", C, V);
    vec("blocks.0.ln0.weight", {C}, SynthTensor::ONES);
    vec("blocks.0.ln0.bias", {C}, SynthTensor::ZEROS);
    const uint32_t DW7 = C >= 4096 ? 128 : 96, DA7 = DW7, DV7 = 64, DG7 = C >= 4096 ? 480 : 320;
    for (uint32_t i = 0; i < L; i++) {
        const std::string p = "blocks." + std::to_string(i) + ".";
        vec(p + "ln1.weight", {C}, SynthTensor::ONES);
        vec(p + "ln1.bias", {C}, SynthTensor::ZEROS);
        vec(p + "ln2.weight", {C}, SynthTensor::ONES);
        vec(p + "ln2.bias", {C}, SynthTensor::ZEROS);
        if (arch == 4 || arch == 5) {
            vec(p + "att.time_mix_k", {C}, SynthTensor::UNIF);
            vec(p + "att.time_mix_v", {C}, SynthTensor::UNIF);
            vec(p + "att.time_mix_r", {C}, SynthTensor::UNIF);
            if (arch == 4) {
                vec(p + "att.time_first", {C}, SynthTensor::UNIF, -1, 1);
                vec(p + "att.time_decay", {C}, SynthTensor::CUSTOM, 0, 0, 1);
            } else {
                vec(p + "att.time_mix_g", {C}, SynthTensor::UNIF);
                vec(p + "att.time_decay", {1, S, H}, SynthTensor::CUSTOM, 0, 0, 2);
                vec(p + "att.time_faaaa", {1, S, H}, SynthTensor::UNIF, -1, 1);
            }
            mat(p + "att.key.weight", C, C);
            mat(p + "att.value.weight", C, C);
            mat(p + "att.receptance.weight", C, C);
            mat(p + "att.output.weight", C, C);
            if (arch == 5) {
                mat(p + "att.gate.weight", C, C);
                vec(p + "att.ln_x.weight", {C}, SynthTensor::ONES);
                vec(p + "att.ln_x.bias", {C}, SynthTensor::ZEROS);
            }
            vec(p + "ffn.time_mix_k", {C}, SynthTensor::UNIF);
            vec(p + "ffn.time_mix_r", {C}, SynthTensor::UNIF);
            mat(p + "ffn.key.weight", C, F);
            mat(p + "ffn.value.weight", F, C);
            mat(p + "ffn.receptance.weight", C, C);
        } else if (arch == 6) {
            for (const char * s : {"x", "w", "k", "v", "r", "g"}) vec(p + "att.time_maa_" + s, {C}, SynthTensor::UNIF);
            mat(p + "att.time_maa_w1", C, 160);
            vec(p + "att.time_maa_w2", {32, C, 5}, SynthTensor::UNIF, -0.1f, 0.1f);
            vec(p + "att.time_decay", {1, S, H}, SynthTensor::UNIF, -6, -1);
            mat(p + "att.time_decay_w1", C, 64);
            mat(p + "att.time_decay_w2", 64, C);
            vec(p + "att.time_faaaa", {1, S, H}, SynthTensor::UNIF, -1, 1);
            mat(p + "att.receptance.weight", C, C);
            mat(p + "att.key.weight", C, C);
            mat(p + "att.value.weight", C, C);
            mat(p + "att.output.weight", C, C);
            mat(p + "att.gate.weight", C, C);
            vec(p + "att.ln_x.weight", {C}, SynthTensor::ONES);
            vec(p + "att.ln_x.bias", {C}, SynthTensor::ZEROS);
            vec(p + "ffn.time_maa_k", {C}, SynthTensor::UNIF);
            vec(p + "ffn.time_maa_r", {C}, SynthTensor::UNIF);
            mat(p + "ffn.key.weight", C, F);
            mat(p + "ffn.receptance.weight", C, C);
            mat(p + "ffn.value.weight", F, C);
        } else {
            vec(p + "att.x_rwkvag", {C, 1, 6}, SynthTensor::UNIF);
            vec(p + "att.w0", {C, 1, 1}, SynthTensor::UNIF, -6, -1);
            mat(p + "att.w1", C, DW7);
            mat(p + "att.w2", DW7, C);
            vec(p + "att.a0", {C, 1, 1}, SynthTensor::UNIF, -1, 1);
            mat(p + "att.a1", C, DA7);
            mat(p + "att.a2", DA7, C);
            if (i != 0) {
                vec(p + "att.v0", {C, 1, 1}, SynthTensor::UNIF, -1, 1);
                mat(p + "att.v1", C, DV7);
                mat(p + "att.v2", DV7, C);
            }
            mat(p + "att.g1", C, DG7);
            mat(p + "att.g2", DG7, C);
            vec(p + "att.k_k", {C, 1, 1}, SynthTensor::UNIF, 0, 1);
            vec(p + "att.k_a", {C, 1, 1}, SynthTensor::UNIF, 0, 1);
            vec(p + "att.r_k", {S, H}, SynthTensor::UNIF, -0.1f, 0.1f);
            mat(p + "att.receptance.weight", C, C);
            mat(p + "att.key.weight", C, C);
            mat(p + "att.value.weight", C, C);
            mat(p + "att.output.weight", C, C);
            vec(p + "att.ln_x.weight", {C}, SynthTensor::ONES);
            vec(p + "att.ln_x.bias", {C}, SynthTensor::ZEROS);
            vec(p + "ffn.x_k", {C, 1, 1}, SynthTensor::UNIF);
            mat(p + "ffn.key.weight", C, F);
            mat(p + "ffn.value.weight", F, C);
        }
    }
    vec("ln_out.weight", {C}, SynthTensor::ONES);
    vec("ln_out.bias", {C}, SynthTensor::ZEROS);
    mat("head.weight", C, V);

    FILE * f = fopen(path, "wb");
    if (!f) return false;
    FileHeader h{RWKV_FILE_MAGIC, RWKV_FILE_VERSION, V, C, L, (uint32_t)ftype};
    bool ok = fwrite(&h, sizeof(h), 1, f) == 1;
    std::vector<float> x;
    std::vector<uint8_t> buf;
    uint64_t idx = 0;
    for (const auto & t : ts) {
        if (!ok) break;
        const uint64_t n = nel(t.ne);
        x.resize(n);
        fill_tensor(t, x.data(), seed * 7919ull + (idx++));
        // dtype policy of convert_pytorch_to_ggml.py:125-137 + rwkv_quantize.inc:133-140
        uint32_t ty = 0;
        const bool is2d = t.ne.size() == 2;
        const bool keep_f32 = t.name.find(".time_") != std::string::npos || t.name.find(".r_k") != std::string::npos;
        if (ftype == 0) {
            ty = 0;
        } else if (ftype == 1) {
            ty = (is2d && !keep_f32) ? 1 : 0;
        } else {
            if (is2d && tensor_needs_quant(t.name)) ty = (uint32_t)ftype;
            else ty = (is2d && !keep_f32) ? 1 : 0;
        }
        buf.resize(type_nbytes(ty, n));
        if (ty == 0) {
            memcpy(buf.data(), x.data(), n * 4);
        } else if (ty == 1) {
            for (uint64_t i = 0; i < n; i++) {
                const uint16_t v = f32_to_f16(x[i]);
                memcpy(buf.data() + 2 * i, &v, 2);
            }
        } else {
            quantize_matrix(ty, x.data(), buf.data(), (int64_t)(n / t.ne[0]), t.ne[0]);
        }
        uint32_t th[3] = {(uint32_t)t.ne.size(), (uint32_t)t.name.size(), ty};
        ok = fwrite(th, 4, 3, f) == 3 && fwrite(t.ne.data(), 4, t.ne.size(), f) == t.ne.size() &&
             fwrite(t.name.data(), 1, t.name.size(), f) == t.name.size() &&
             fwrite(buf.data(), 1, buf.size(), f) == buf.size();
    }
    ok = (fclose(f) == 0) && ok;
    return ok;
}

}  // namespace rwkvmi

extern "C" RWKV_API bool rwkv_quantize_model_file(const char * in, const char * out, const char * fmt) {
    try {
        return rwkvmi::quantize_model_file(in, out, fmt);
    } catch (const std::exception &) {
        rwkvmi::add_error(RWKV_ERROR_ALLOC);
        return false;
    }
}

extern "C" RWKV_API bool rwkv_mi355x_write_synthetic_model(const char * path, int arch, uint32_t n_vocab,
                                                           uint32_t n_embed, uint32_t n_layer, uint32_t ffn,
                                                           const char * fmt, uint64_t seed) {
    return rwkvmi::write_synthetic(path, arch, n_vocab, n_embed, n_layer, ffn, fmt, seed);
}
