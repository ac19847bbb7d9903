// model_file.cpp -- rwkv.cpp model file reader.
// Reference: rwkv_file_format.inc:100-316, rwkv_model_loading.inc:128-419, docs/FILE_FORMAT.md.
#include "model_file.hpp"

#include <inttypes.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

namespace rwkvmi {

thread_local enum rwkv_error_flags g_last_error = RWKV_ERROR_NONE;
thread_local bool g_print_errors = true;

static const char * kTypeNames[] = {"FP32", "FP16", "Q4_0", "Q4_1", "Q4_1_O", "Q4_2", "Q4_3", "Q5_0",
                                    "Q5_1", "Q8_0", "Q8_1", "Q2_K", "Q3_K", "Q4_K", "Q5_K", "Q6_K", "Q8_K"};
static const int kTypeCount = 17;

const char * type_name(uint32_t type) { return type < (uint32_t)kTypeCount ? kTypeNames[type] : "unknown"; }

int type_from_name(const char * name) {
    for (int i = 0; i < kTypeCount; i++)
        if (strcmp(name, kTypeNames[i]) == 0) return i;
    return -1;
}

bool type_supported(uint32_t t) { return t == 0 || t == 1 || t == 2 || t == 3 || t == 7 || t == 8 || t == 9; }
bool type_quantized(uint32_t t) { return t == 2 || t == 3 || t == 7 || t == 8 || t == 9; }

size_t type_block_bytes(uint32_t t) {
    switch (t) {
        case 2: return 18;
        case 3: return 20;
        case 7: return 22;
        case 8: return 24;
        case 9: return 34;
        default: return 0;
    }
}

size_t type_nbytes(uint32_t type, uint64_t nel) {
    if (type == 0) return nel * 4;
    if (type == 1) return nel * 2;
    if (type_quantized(type)) return (nel / 32) * type_block_bytes(type);
    return 0;
}

uint16_t f32_to_f16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u, exp = (x >> 23) & 0xffu, mant = x & 0x7fffffu;
    if (exp == 0xff) return (uint16_t)(sign | 0x7c00u | (mant ? (0x200u | (mant >> 13)) : 0u));
    int e = (int)exp - 127 + 15;
    if (e >= 0x1f) return (uint16_t)(sign | 0x7c00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        mant |= 0x800000u;
        int shift = 14 - e;
        uint32_t h = mant >> shift, rem = mant & ((1u << shift) - 1u), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1u))) h++;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)e << 10) | (mant >> 13), rem = mant & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t)(sign | h);
}

float f16_to_f32(uint16_t h) {
    uint32_t sign = ((uint32_t)h & 0x8000u) << 16, exp = ((uint32_t)h >> 10) & 0x1fu, mant = (uint32_t)h & 0x3ffu, x;
    if (exp == 0) {
        if (mant == 0) {
            x = sign;
        } else {
            int e = -1;
            do {
                e++;
                mant <<= 1;
            } while (!(mant & 0x400u));
            x = sign | ((uint32_t)(127 - 15 - e) << 23) | ((mant & 0x3ffu) << 13);
        }
    } else if (exp == 0x1f) {
        x = sign | 0x7f800000u | (mant << 13);
    } else {
        x = sign | ((exp - 15 + 127) << 23) | (mant << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

bool read_file_header(FILE * f, FileHeader & h) {
    RWKV_CHECK(RWKV_ERROR_FILE_READ, false, fread(&h, sizeof(h), 1, f) == 1, "Failed to read file header");
    RWKV_CHECK(RWKV_ERROR_FILE_MAGIC, false, h.magic == RWKV_FILE_MAGIC, "Invalid file magic");
    RWKV_CHECK(RWKV_ERROR_FILE_VERSION, false, h.version >= RWKV_FILE_VERSION_MIN && h.version <= RWKV_FILE_VERSION_MAX,
               "Unsupported file version %" PRIu32, h.version);
    RWKV_CHECK(RWKV_ERROR_DATA_TYPE, false, h.data_type < (uint32_t)kTypeCount,
               "Model data type out of range (%" PRIu32 " > %d)", h.data_type, kTypeCount - 1);
    RWKV_CHECK(RWKV_ERROR_DATA_TYPE, false, type_supported(h.data_type),
               "Models in %s format are not supported by this library", type_name(h.data_type));
    RWKV_CHECK(RWKV_ERROR_DATA_TYPE, false, !type_quantized(h.data_type) || h.version == RWKV_FILE_VERSION_1,
               "The quantized model file in %s format was created with an old version of rwkv.cpp", type_name(h.data_type));
    return true;
}

// rwkv_fread_tensor_header (rwkv_file_format.inc:167-197)
static constexpr uint32_t kMaxKeyLen = 4096;

static bool read_tensor_header(FILE * f, HostTensor & t, uint32_t & key_len) {
    uint32_t h[3];
    RWKV_CHECK(RWKV_ERROR_FILE_READ, false, fread(h, 4, 3, f) == 3, "Failed to read tensor header");
    t.ndim = h[0];
    key_len = h[1];
    t.type = h[2];
    RWKV_CHECK(RWKV_ERROR_SHAPE, false, t.ndim >= 1 && t.ndim <= 3, "Tensor has an invalid shape (%" PRIu32 " dimensions)", t.ndim);
    RWKV_CHECK(RWKV_ERROR_DATA_TYPE, false, t.type < (uint32_t)kTypeCount, "Tensor data type out of range (%" PRIu32 ")", t.type);
    RWKV_CHECK(RWKV_ERROR_DATA_TYPE, false, type_supported(t.type), "Tensor data type (%s) is not supported", type_name(t.type));
    t.ne[0] = t.ne[1] = t.ne[2] = 1;
    RWKV_CHECK(RWKV_ERROR_FILE_READ, false, fread(t.ne, 4, t.ndim, f) == t.ndim, "Failed to read tensor shape");
    RWKV_CHECK(RWKV_ERROR_FILE_READ, false, key_len <= kMaxKeyLen, "Tensor name too long (%" PRIu32 " bytes)", key_len);
    for (uint32_t i = 0; i < t.ndim; i++)
        RWKV_CHECK(RWKV_ERROR_SHAPE, false, t.ne[i] >= 1 && t.ne[i] <= (1u << 30), "Tensor dimension %u out of range", t.ne[i]);
    RWKV_CHECK(RWKV_ERROR_SHAPE, false, !type_quantized(t.type) || t.ne[0] % 32 == 0,
               "Quantized tensor row length %" PRIu32 " is not a multiple of 32", t.ne[0]);
    return true;
}

static const char * kV7Layer[] = {"att.x_rwkvag", "att.w0", "att.w1", "att.w2", "att.a0", "att.a1", "att.a2",
                                  "att.g1", "att.g2", "att.r_k", "att.k_k", "att.k_a", "att.key.weight",
                                  "att.value.weight", "att.receptance.weight", "att.output.weight",
                                  "att.ln_x.weight", "att.ln_x.bias", "ln2.weight", "ln2.bias", "ffn.x_k",
                                  "ffn.key.weight", "ffn.value.weight"};
static const char * kV6Layer[] = {"att.time_maa_x", "att.time_maa_w", "att.time_maa_k", "att.time_maa_v",
                                  "att.time_maa_r", "att.time_maa_g", "att.time_maa_w1", "att.time_maa_w2",
                                  "att.time_faaaa", "att.time_decay", "att.time_decay_w1", "att.time_decay_w2",
                                  "att.key.weight", "att.value.weight", "att.receptance.weight", "att.gate.weight",
                                  "att.output.weight", "att.ln_x.weight", "att.ln_x.bias", "ln2.weight", "ln2.bias",
                                  "ffn.time_maa_k", "ffn.time_maa_r", "ffn.key.weight", "ffn.value.weight",
                                  "ffn.receptance.weight"};
static const char * kV5Layer[] = {"att.time_mix_k", "att.time_mix_v", "att.time_mix_r", "att.time_decay",
                                  "att.key.weight", "att.value.weight", "att.receptance.weight", "att.output.weight",
                                  "att.ln_x.weight", "att.ln_x.bias", "ln2.weight", "ln2.bias", "ffn.time_mix_k",
                                  "ffn.time_mix_r", "ffn.key.weight", "ffn.value.weight", "ffn.receptance.weight"};
static const char * kV4Layer[] = {"att.time_mix_k", "att.time_mix_v", "att.time_mix_r", "att.time_first",
                                  "att.time_decay", "att.key.weight", "att.value.weight", "att.receptance.weight",
                                  "att.output.weight", "ln2.weight", "ln2.bias", "ffn.time_mix_k", "ffn.time_mix_r",
                                  "ffn.key.weight", "ffn.value.weight", "ffn.receptance.weight"};

static bool need(const ModelFile & mf, const std::string & key) {
    RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS | RWKV_ERROR_PARAM_MISSING, false, mf.find(key) != nullptr,
               "Model parameter %s not found", key.c_str());
    return true;
}

// The parameter table of rwkv_set_params (rwkv_model_loading.inc:128-285).
static bool check_params(const ModelFile & mf) {
    if (!need(mf, "emb.weight") || !need(mf, "blocks.0.ln0.weight") || !need(mf, "blocks.0.ln0.bias")) return false;
    for (uint32_t i = 0; i < mf.header.n_layer; i++) {
        const std::string p = "blocks." + std::to_string(i) + ".";
        if (!need(mf, p + "ln1.weight") || !need(mf, p + "ln1.bias")) return false;
        const char ** keys;
        size_t n;
        switch (mf.arch_major) {
            case 7: keys = kV7Layer; n = sizeof(kV7Layer) / sizeof(*kV7Layer); break;
            case 6: keys = kV6Layer; n = sizeof(kV6Layer) / sizeof(*kV6Layer); break;
            case 5: keys = kV5Layer; n = sizeof(kV5Layer) / sizeof(*kV5Layer); break;
            default: keys = kV4Layer; n = sizeof(kV4Layer) / sizeof(*kV4Layer); break;
        }
        for (size_t k = 0; k < n; k++)
            if (!need(mf, p + keys[k])) return false;
        if (mf.arch_major == 5) {
            if (mf.arch_minor >= 2) {
                if (!need(mf, p + "att.time_faaaa") || !need(mf, p + "att.time_mix_g") || !need(mf, p + "att.gate.weight"))
                    return false;
            } else if (!need(mf, p + "att.time_first")) {
                return false;
            }
        }
        if (mf.arch_major == 7 && i != 0) {
            if (!need(mf, p + "att.v0") || !need(mf, p + "att.v1") || !need(mf, p + "att.v2")) return false;
        }
    }
    return need(mf, "ln_out.weight") && need(mf, "ln_out.bias") && need(mf, "head.weight");
}

// Every tensor against the dimensions the kernels derive from the header and the layer-0 tensors
// (the checks ggml's op asserts make in the reference when the graph is built): C = n_embed,
// V = n_vocab, H/S (rwkv_model_loading.inc:403-409), FFN width F, LoRA widths.  Vectors must be
// FP32/FP16; matrices [K, M] any supported type (quantized K % 32 == 0, checked at read).
static bool shape_is(const ModelFile & mf, const std::string & key, std::initializer_list<uint32_t> ne, bool vec) {
    const HostTensor * t = mf.find(key);
    if (!t) return true;  // optional (absent where the version has no such tensor); need() checks presence
    uint64_t n = 1;
    for (uint32_t v : ne) n *= v;
    bool ok = t->nel() == n;
    if (ok && !vec) {  // matrices: exactly [ne0, ne1]
        const uint32_t * e = ne.begin();
        ok = t->ndim == 2 && t->ne[0] == e[0] && t->ne[1] == e[1];
    }
    RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS | RWKV_ERROR_SHAPE, false, ok, "Parameter %s has an unexpected shape (%u x %u x %u)",
               key.c_str(), t->ne[0], t->ne[1], t->ne[2]);
    RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS | RWKV_ERROR_DATA_TYPE, false, !vec || t->type <= 1,
               "Parameter %s must be FP32 or FP16", key.c_str());
    return true;
}

static bool check_shapes(const ModelFile & mf) {
    const uint32_t C = mf.header.n_embed, V = mf.header.n_vocab;
    const uint32_t H = (uint32_t)mf.head_count, S = (uint32_t)mf.head_size;
    RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS | RWKV_ERROR_DIMENSION, false, C >= 1 && V >= 1 && mf.header.n_layer >= 1,
               "Model dimensions out of range");
    RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS | RWKV_ERROR_DIMENSION, false, mf.arch_major < 5 || (H >= 1 && (uint64_t)H * S == C),
               "n_embed %u is not head_count %u x head_size %u", C, H, S);
    // the v7 per-head prep kernels (k_v7_prep) cover channels in whole 64-lane waves
    RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS | RWKV_ERROR_UNSUPPORTED, false, mf.arch_major != 7 || C % 64 == 0,
               "v7 models need n_embed %% 64 == 0 (n_embed %u)", C);
    const HostTensor * fk = mf.find("blocks.0.ffn.key.weight");
    const uint32_t F = fk->ne[1];
    bool ok = shape_is(mf, "blocks.0.ln0.weight", {C}, true) && shape_is(mf, "blocks.0.ln0.bias", {C}, true) &&
              shape_is(mf, "ln_out.weight", {C}, true) && shape_is(mf, "ln_out.bias", {C}, true) &&
              shape_is(mf, "head.weight", {C, V}, false);
    uint32_t D5 = 0, DW = 0, DW7 = 0, DA7 = 0, DG7 = 0, DV7 = 0;
    if (mf.arch_major == 6) {
        D5 = mf.find("blocks.0.att.time_maa_w1")->ne[1];
        DW = mf.find("blocks.0.att.time_decay_w1")->ne[1];
        RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS | RWKV_ERROR_SHAPE, false, D5 % 5 == 0 && D5 / 5 <= 64 && DW >= 1,
                   "Unsupported v6 LoRA widths (maa %u, decay %u)", D5, DW);
    }
    if (mf.arch_major == 7) {
        DW7 = mf.find("blocks.0.att.w1")->ne[1];
        DA7 = mf.find("blocks.0.att.a1")->ne[1];
        DG7 = mf.find("blocks.0.att.g1")->ne[1];
        const HostTensor * v1 = mf.header.n_layer > 1 ? mf.find("blocks.1.att.v1") : nullptr;
        DV7 = v1 ? v1->ne[1] : 0;
    }
    for (uint32_t i = 0; ok && i < mf.header.n_layer; i++) {
        const std::string p = "blocks." + std::to_string(i) + ".";
        auto V1 = [&](const char * k) { return shape_is(mf, p + k, {C}, true); };
        auto M2 = [&](const char * k, uint32_t K, uint32_t M) { return shape_is(mf, p + k, {K, M}, false); };
        ok = V1("ln1.weight") && V1("ln1.bias") && V1("ln2.weight") && V1("ln2.bias") &&
             M2("att.key.weight", C, C) && M2("att.value.weight", C, C) && M2("att.receptance.weight", C, C) &&
             M2("att.output.weight", C, C) && M2("ffn.key.weight", C, F) && M2("ffn.value.weight", F, C);
        if (ok && mf.arch_major != 7) ok = M2("ffn.receptance.weight", C, C);
        if (ok && (mf.arch_major == 4 || mf.arch_major == 5))
            ok = V1("att.time_mix_k") && V1("att.time_mix_v") && V1("att.time_mix_r") && V1("ffn.time_mix_k") &&
                 V1("ffn.time_mix_r");
        if (ok && mf.arch_major == 4) ok = V1("att.time_first") && V1("att.time_decay");
        if (ok && mf.arch_major >= 5) ok = V1("att.ln_x.weight") && V1("att.ln_x.bias");
        if (ok && mf.arch_major == 5) {
            if (mf.arch_minor >= 2)
                ok = shape_is(mf, p + "att.time_decay", {C}, true) && V1("att.time_faaaa") && V1("att.time_mix_g") &&
                     M2("att.gate.weight", C, C);
            else
                ok = shape_is(mf, p + "att.time_decay", {H}, true) && shape_is(mf, p + "att.time_first", {H}, true);
            for (const char * k : {"att.time_decay", "att.time_faaaa", "att.time_first"}) {
                const HostTensor * t = mf.find(p + k);
                RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS | RWKV_ERROR_DATA_TYPE, false, !t || t->type == 0,
                           "Parameter %s%s must be FP32", p.c_str(), k);
            }
        }
        if (ok && mf.arch_major == 6) {
            ok = V1("att.time_maa_x") && V1("att.time_maa_w") && V1("att.time_maa_k") && V1("att.time_maa_v") &&
                 V1("att.time_maa_r") && V1("att.time_maa_g") && V1("att.time_faaaa") && V1("att.time_decay") &&
                 V1("ffn.time_maa_k") && V1("ffn.time_maa_r") && M2("att.time_maa_w1", C, D5) &&
                 shape_is(mf, p + "att.time_maa_w2", {D5 / 5, C, 5}, true) && M2("att.time_decay_w1", C, DW) &&
                 M2("att.time_decay_w2", DW, C) && M2("att.gate.weight", C, C);
            const HostTensor * w2 = mf.find(p + "att.time_maa_w2");
            RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS | RWKV_ERROR_SHAPE, false, !ok || (w2->type == 0 && w2->ndim == 3),
                       "Parameter %satt.time_maa_w2 must be an FP32 [D, C, 5] tensor", p.c_str());
        }
        if (ok && mf.arch_major == 7) {
            ok = shape_is(mf, p + "att.x_rwkvag", {C, 1, 6}, true) && V1("att.w0") && V1("att.a0") && V1("att.k_k") &&
                 V1("att.k_a") && shape_is(mf, p + "att.r_k", {S, H}, true) && V1("ffn.x_k") &&
                 M2("att.w1", C, DW7) && M2("att.w2", DW7, C) && M2("att.a1", C, DA7) && M2("att.a2", DA7, C) &&
                 M2("att.g1", C, DG7) && M2("att.g2", DG7, C);
            if (ok && i != 0) ok = V1("att.v0") && M2("att.v1", C, DV7) && M2("att.v2", DV7, C);
        }
    }
    return ok;
}

// Is tensor `name`'s data needed by a context owning layers [l0, l1) of an n_layer model?
static bool tensor_wanted(const std::string & name, uint32_t l0, uint32_t l1, uint32_t n_layer) {
    if (name.rfind("blocks.", 0) == 0) {
        const uint32_t i = (uint32_t)strtoul(name.c_str() + 7, nullptr, 10);
        if (name.find(".ln0.") != std::string::npos) return l0 == 0;
        return i >= l0 && i < l1;
    }
    if (name == "emb.weight") return l0 == 0;
    if (name == "head.weight" || name.rfind("ln_out.", 0) == 0) return l1 >= n_layer;
    return true;
}

bool load_model_file(const char * path, ModelFile & mf, uint32_t layer_begin, uint32_t layer_end) {
    FILE * f = fopen(path, "rb");
    RWKV_CHECK(RWKV_ERROR_FILE | RWKV_ERROR_FILE_OPEN, false, f != nullptr, "Failed to open file %s", path);
    struct stat st;
    if (fstat(fileno(f), &st) != 0) {
        fclose(f);
        RWKV_CHECK(RWKV_ERROR_FILE | RWKV_ERROR_FILE_STAT, false, false, "Failed to stat file %s", path);
    }
    if (!read_file_header(f, mf.header)) {
        fclose(f);
        RWKV_CHECK(RWKV_ERROR_FILE, false, false, "Invalid file header");
    }
    while (ftello(f) < (off_t)st.st_size) {
        HostTensor t;
        uint32_t key_len = 0;
        bool ok = read_tensor_header(f, t, key_len);
        const off_t left = (off_t)st.st_size - ftello(f);
        if (ok) {
            ok = (off_t)key_len <= left;
            if (!ok) add_error(RWKV_ERROR_FILE_READ);
        }
        if (ok) {
            t.name.resize(key_len);
            ok = key_len == 0 || fread(&t.name[0], 1, key_len, f) == key_len;
            if (!ok) add_error(RWKV_ERROR_FILE_READ);
        }
        if (ok) {
            const size_t nb = type_nbytes(t.type, t.nel());
            ok = (off_t)nb <= (off_t)st.st_size - ftello(f);
            if (!ok) add_error(RWKV_ERROR_FILE_READ);
        }
        if (ok) {
            const size_t nb = type_nbytes(t.type, t.nel());
            if (tensor_wanted(t.name, layer_begin, layer_end, mf.header.n_layer)) {
                t.data.resize(nb);
                ok = nb == 0 || fread(t.data.data(), 1, nb, f) == nb;
            } else {
                ok = fseeko(f, (off_t)nb, SEEK_CUR) == 0;  // another stage's tensor: shape only
            }
            if (!ok) add_error(RWKV_ERROR_FILE_READ);
        }
        if (!ok) {
            fclose(f);
            RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS, false, false, "Failed to read a model parameter");
        }
        mf.index[t.name] = mf.tensors.size();
        mf.tensors.push_back(std::move(t));
    }
    fclose(f);

    // rwkv_model_loading.inc:319-340
    mf.arch_major = 4;
    mf.arch_minor = 0;
    if (mf.find("blocks.0.att.ln_x.weight")) {
        mf.arch_major = 5;
        mf.arch_minor = mf.find("blocks.0.att.gate.weight") ? 2 : 1;
    }
    if (mf.find("blocks.0.att.time_maa_x")) {
        mf.arch_major = 6;
        mf.arch_minor = 0;
    }
    if (mf.find("blocks.0.att.r_k")) {
        mf.arch_major = 7;
        mf.arch_minor = 0;
    }
    if (!check_params(mf)) return false;

    // rwkv_model_loading.inc:403-409
    if (mf.arch_major == 7) {
        mf.head_count = mf.find("blocks.0.att.r_k")->ne[1];
    } else if (mf.arch_major >= 5) {
        mf.head_count = mf.find("blocks.0.att.time_decay")->ne[2];
    }
    if (mf.head_count) mf.head_size = (int64_t)mf.find("blocks.0.ln1.weight")->ne[0] / mf.head_count;
    if (!check_shapes(mf)) return false;

    const HostTensor * emb = mf.find("emb.weight");
    RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS | RWKV_ERROR_SHAPE, false, emb->ndim == 2, "Unexpected dimension count of embedding matrix %u", emb->ndim);
    RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS | RWKV_ERROR_DIMENSION, false, emb->ne[0] == mf.header.n_embed, "Unexpected dimension of embedding matrix %u", emb->ne[0]);
    RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS | RWKV_ERROR_DIMENSION, false, emb->ne[1] == mf.header.n_vocab, "Unexpected dimension of embedding matrix %u", emb->ne[1]);
    RWKV_CHECK(RWKV_ERROR_MODEL_PARAMS | RWKV_ERROR_DATA_TYPE, false, emb->type <= 1, "Embedding matrix must be FP32 or FP16");
    return true;
}

}  // namespace rwkvmi
