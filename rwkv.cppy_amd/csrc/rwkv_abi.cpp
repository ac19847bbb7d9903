// rwkv_abi.cpp -- the rwkv.h C ABI (reference rwkv.h:70-224, rwkv.cpp:70-258, rwkv_eval.inc:37-241)
// on top of the MI355X engine.  Error, ownership and NULL-argument semantics follow the
// reference; evaluation always runs on the GPU (see include/rwkv.h notes).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <inttypes.h>
#include <exception>
#include <map>
#include <mutex>
#include <string>
#include <vector>
#include <tuple>

#include "../../include/rwkv.h"
#include "../../include/rwkv_mi355x.h"
#include "engine.hpp"
#include "model_file.hpp"
#include "pipeline.hpp"

using namespace rwkvmi;

struct SharedModel {
    DeviceModel dm;
    std::atomic<int> refcount{0};
    // what was uploaded: a replica on another GPU (rwkv_mi355x_clone_context_on) re-reads it
    std::string path;
    uint32_t layer_begin = 0, layer_end = UINT32_MAX;
};

// One upload per (file, layer range, device): contexts cloned onto a GPU that already holds the
// model share that copy (the reference's clones share one model, rwkv.cpp:123-139).  Guarded by
// g_model_mutex.
typedef std::tuple<std::string, uint32_t, uint32_t, int> ReplicaKey;
static std::map<ReplicaKey, SharedModel *> g_replicas;
static ReplicaKey replica_key(const SharedModel * sm, int device) {
    return ReplicaKey(sm->path, sm->layer_begin, sm->layer_end, device);
}

struct rwkv_context {
    SharedModel * model = nullptr;
    Engine * engine = nullptr;
    uint32_t n_threads = 1;
    enum rwkv_error_flags last_error = RWKV_ERROR_NONE;
    bool print_errors = true;
    // layer pipeline (RWKV_MI355X_PIPELINE / rwkv_mi355x_init_pipeline): this context is stage 0;
    // stages[i] (i >= 1) are owned stage contexts on their own GPUs
    LayerPipeline * pipe = nullptr;
    std::vector<rwkv_context *> stages;
};

static std::mutex g_model_mutex;

#define CTX_CHECK(ctx, FLAGS, RET, cond, ...)                                        \
    do {                                                                             \
        if (!(cond)) {                                                               \
            (ctx)->last_error = (ctx)->last_error | (FLAGS);                         \
            if ((ctx)->print_errors) {                                               \
                fprintf(stderr, __VA_ARGS__);                                        \
                fprintf(stderr, "\n%s:%d: %s\n", __FILE__, __LINE__, #cond);         \
            }                                                                        \
            return RET;                                                              \
        }                                                                            \
    } while (0)

static int pick_device() {
    const char * e = getenv("RWKV_MI355X_DEVICE");
    if (e && *e) return atoi(e);
    const char * lr = getenv("LOCAL_RANK");
    int n = 0;
    if (lr && *lr && hipGetDeviceCount(&n) == hipSuccess && n > 0) return atoi(lr) % n;
    return 0;
}

extern "C" {

RWKV_API void rwkv_set_print_errors(struct rwkv_context * ctx, const bool print_errors) {
    if (ctx) ctx->print_errors = print_errors; else g_print_errors = print_errors;
}

RWKV_API bool rwkv_get_print_errors(const struct rwkv_context * ctx) { return ctx ? ctx->print_errors : g_print_errors; }

RWKV_API enum rwkv_error_flags rwkv_get_last_error(struct rwkv_context * ctx) {
    enum rwkv_error_flags * p = ctx ? &ctx->last_error : &g_last_error;
    const enum rwkv_error_flags v = *p;
    *p = RWKV_ERROR_NONE;
    return v;
}

static struct rwkv_context * new_context(SharedModel * sm, uint32_t n_threads) {
    rwkv_context * ctx = new (std::nothrow) rwkv_context();
    RWKV_CHECK(RWKV_ERROR_CTX | RWKV_ERROR_ALLOC, nullptr, ctx != nullptr, "Failed to allocate rwkv_context");
    ctx->model = sm;
    ctx->n_threads = n_threads;
    ctx->print_errors = g_print_errors;
    ctx->engine = new (std::nothrow) Engine(&sm->dm);
    if (!ctx->engine || !ctx->engine->init()) {
        delete ctx->engine;
        delete ctx;
        RWKV_CHECK(RWKV_ERROR_CTX | RWKV_ERROR_ALLOC, nullptr, false, "Failed to allocate device workspace");
    }
    sm->refcount++;
    return ctx;
}

static struct rwkv_context * init_from_file(const char * path, const uint32_t n_threads, uint32_t layer_begin = 0,
                                            uint32_t layer_end = UINT32_MAX, int device = -1) {
    int ndev = 0;
    const hipError_t de = hipGetDeviceCount(&ndev);
    RWKV_CHECK(RWKV_ERROR_CTX | RWKV_ERROR_UNSUPPORTED, nullptr, de == hipSuccess && ndev > 0,
               "No HIP device available: this library evaluates RWKV on an AMD Instinct MI355X (gfx950) only");
    ModelFile mf;
    if (!load_model_file(path, mf, layer_begin, layer_end)) return nullptr;
    RWKV_CHECK(RWKV_ERROR_ARGS, nullptr, layer_begin < layer_end && layer_begin < mf.header.n_layer,
               "Bad layer range [%u, %u) for %u layers", layer_begin, layer_end, mf.header.n_layer);
    SharedModel * sm = new (std::nothrow) SharedModel();
    RWKV_CHECK(RWKV_ERROR_CTX | RWKV_ERROR_ALLOC, nullptr, sm != nullptr, "Failed to allocate model");
    sm->dm.device = device >= 0 ? device : pick_device();
    if (sm->dm.device >= ndev) sm->dm.device = 0;
    if (hipSetDevice(sm->dm.device) != hipSuccess || !upload_model(mf, sm->dm, layer_begin, layer_end)) {
        free_model(sm->dm);
        delete sm;
        RWKV_CHECK(RWKV_ERROR_MODEL | RWKV_ERROR_ALLOC, nullptr, false, "Failed to upload the model to the GPU");
    }
    mf.tensors.clear();
    sm->path = path;
    sm->layer_begin = layer_begin;
    sm->layer_end = layer_end;
    rwkv_context * ctx = new_context(sm, n_threads);
    if (!ctx) {
        free_model(sm->dm);
        delete sm;
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_model_mutex);
    g_replicas.emplace(replica_key(sm, sm->dm.device), sm);  // first upload of this key wins
    return ctx;
}

// Every entry point that enqueues device work runs on the context's GPU (contexts of one process
// may sit on different GPUs: rwkv_mi355x_clone_context_on).
static void use_device(const rwkv_context * ctx) { (void)hipSetDevice(ctx->model->dm.device); }

static void free_context(struct rwkv_context * ctx);

// The layer pipeline behind the reference entry points: P stage contexts, stage i
// on devices[i] holding layers stage_layers(n_layer, P, i) (earlier stages take the extra layers,
// as rwkv_cpp/pipeline.py stage_layers), driven from this process by LayerPipeline.  The returned
// context is stage 0; it reports the whole model's dimensions and accepts rwkv_eval /
// rwkv_eval_sequence[_in_chunks] with host buffers, bit-identical to a single-GPU context.
static struct rwkv_context * init_pipeline(const char * path, uint32_t n_threads, int P, const int * devices) {
    int ndev = 0;
    RWKV_CHECK(RWKV_ERROR_CTX | RWKV_ERROR_UNSUPPORTED, nullptr, hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0,
               "No HIP device available");
    FileHeader h{};
    {
        FILE * f = fopen(path, "rb");
        RWKV_CHECK(RWKV_ERROR_FILE | RWKV_ERROR_FILE_OPEN, nullptr, f != nullptr, "Failed to open %s", path);
        const bool ok = read_file_header(f, h);
        fclose(f);
        if (!ok) return nullptr;
    }
    RWKV_CHECK(RWKV_ERROR_ARGS, nullptr, P >= 2 && (uint32_t)P <= h.n_layer, "Pipeline of %d stages for %u layers", P,
               h.n_layer);
    std::vector<rwkv_context *> st;
    std::vector<LayerPipeline::StageSpec> specs;
    const uint32_t base = h.n_layer / (uint32_t)P, extra = h.n_layer % (uint32_t)P;
    for (int i = 0; i < P; i++) {
        const uint32_t l0 = (uint32_t)i * base + std::min<uint32_t>((uint32_t)i, extra);
        const uint32_t l1 = l0 + base + ((uint32_t)i < extra ? 1u : 0u);
        const int dev = devices ? devices[i] : i % ndev;
        rwkv_context * c = (dev >= 0 && dev < ndev) ? init_from_file(path, n_threads, l0, l1, dev) : nullptr;
        if (!c) {
            for (rwkv_context * q : st) free_context(q);
            RWKV_CHECK(RWKV_ERROR_CTX | RWKV_ERROR_ALLOC, nullptr, false, "Failed to create pipeline stage %d on device %d",
                       i, dev);
        }
        st.push_back(c);
        specs.push_back(LayerPipeline::StageSpec{c->engine, c->model->dm.device, l0, l1});
    }
    LayerPipeline * p = new (std::nothrow) LayerPipeline();
    if (!p || !p->init(specs, h.n_embed, st[0]->model->dm.major == 7)) {
        delete p;
        for (rwkv_context * q : st) free_context(q);
        RWKV_CHECK(RWKV_ERROR_CTX | RWKV_ERROR_ALLOC, nullptr, false, "Failed to set up the layer pipeline");
    }
    rwkv_context * head = st[0];
    head->pipe = p;
    head->stages.assign(st.begin() + 1, st.end());
    return head;
}

static int env_pipeline_stages() {
    const char * e = getenv("RWKV_MI355X_PIPELINE");
    return e && *e ? atoi(e) : 0;
}

static std::vector<int> env_pipeline_devices(int P) {
    std::vector<int> d;
    const char * e = getenv("RWKV_MI355X_PIPELINE_DEVICES");  // "0,1,2,3"; default i % device count
    if (!e || !*e) return d;
    std::string v(e);
    size_t pos = 0;
    while ((int)d.size() < P && pos <= v.size()) {
        const size_t q = v.find(',', pos);
        d.push_back(atoi(v.substr(pos, q == std::string::npos ? std::string::npos : q - pos).c_str()));
        if (q == std::string::npos) break;
        pos = q + 1;
    }
    if ((int)d.size() != P) d.clear();
    return d;
}

// No C++ exception crosses the C ABI: a failed host allocation (std::bad_alloc from a corrupt
// file's sizes, say) becomes RWKV_ERROR_ALLOC and a NULL context.
// n_gpu_layers is accepted and ignored: the whole model always runs on the GPU(s).  With the
// additive setting RWKV_MI355X_PIPELINE=P (P >= 2) the context is a P-stage layer pipeline
// (devices RWKV_MI355X_PIPELINE_DEVICES="d0,d1,..." or 0..P-1 modulo the device count).
RWKV_API struct rwkv_context * rwkv_init_from_file(const char * path, const uint32_t n_threads, const uint32_t n_gpu_layers) {
    (void)n_gpu_layers;
    g_last_error = RWKV_ERROR_NONE;
    try {
        const int P = env_pipeline_stages();
        if (P >= 2) {
            const std::vector<int> devs = env_pipeline_devices(P);
            return init_pipeline(path, n_threads, P, devs.empty() ? nullptr : devs.data());
        }
        return init_from_file(path, n_threads);
    } catch (const std::exception & e) {
        RWKV_CHECK(RWKV_ERROR_CTX | RWKV_ERROR_ALLOC, nullptr, false, "Failed to load %s: %s", path, e.what());
    }
}

RWKV_API struct rwkv_context * rwkv_mi355x_init_pipeline(const char * path, const uint32_t n_threads, const int n_stages,
                                                         const int * devices) {
    g_last_error = RWKV_ERROR_NONE;
    try {
        return init_pipeline(path, n_threads, n_stages, devices);
    } catch (const std::exception & e) {
        RWKV_CHECK(RWKV_ERROR_CTX | RWKV_ERROR_ALLOC, nullptr, false, "Failed to load %s: %s", path, e.what());
    }
}

RWKV_API int rwkv_mi355x_pipeline_stages(const struct rwkv_context * ctx) {
    return ctx && ctx->pipe ? (int)ctx->pipe->stages() : (ctx ? 1 : 0);
}

RWKV_API int rwkv_mi355x_pipeline_peer_pairs(const struct rwkv_context * ctx) {
    return ctx && ctx->pipe ? ctx->pipe->peer_pairs() : 0;
}

RWKV_API struct rwkv_context * rwkv_mi355x_init_from_file_layers(const char * path, const uint32_t n_threads,
                                                                 const uint32_t layer_begin, const uint32_t layer_end) {
    g_last_error = RWKV_ERROR_NONE;
    try {
        return init_from_file(path, n_threads, layer_begin, layer_end);
    } catch (const std::exception & e) {
        RWKV_CHECK(RWKV_ERROR_CTX | RWKV_ERROR_ALLOC, nullptr, false, "Failed to load %s: %s", path, e.what());
    }
}

RWKV_API struct rwkv_context * rwkv_clone_context(struct rwkv_context * ctx, const uint32_t n_threads) {
    if (!ctx) return nullptr;
    if (ctx->pipe) {
        // a pipeline clone: the same stages on the same GPUs, each with its own engine (fresh
        // state) sharing the stage's uploaded weights
        std::vector<rwkv_context *> st;
        std::vector<LayerPipeline::StageSpec> specs;
        std::vector<rwkv_context *> src = {ctx};
        src.insert(src.end(), ctx->stages.begin(), ctx->stages.end());
        for (rwkv_context * s : src) {
            rwkv_context * c = nullptr;
            {
                std::lock_guard<std::mutex> lk(g_model_mutex);
                c = new_context(s->model, n_threads);
            }
            if (!c) {
                for (rwkv_context * q : st) free_context(q);
                return nullptr;
            }
            c->print_errors = ctx->print_errors;
            st.push_back(c);
            specs.push_back(LayerPipeline::StageSpec{c->engine, c->model->dm.device, s->model->dm.layer_lo,
                                                     s->model->dm.layer_hi});
        }
        LayerPipeline * p = new (std::nothrow) LayerPipeline();
        if (!p || !p->init(specs, ctx->model->dm.n_embed, ctx->model->dm.major == 7)) {
            delete p;
            for (rwkv_context * q : st) free_context(q);
            return nullptr;
        }
        st[0]->pipe = p;
        st[0]->stages.assign(st.begin() + 1, st.end());
        return st[0];
    }
    std::lock_guard<std::mutex> lk(g_model_mutex);
    rwkv_context * c = new_context(ctx->model, n_threads);
    if (c) c->print_errors = ctx->print_errors;
    return c;
}

RWKV_API struct rwkv_context * rwkv_mi355x_clone_context_on(struct rwkv_context * ctx, const uint32_t n_threads,
                                                            const int device) {
    if (!ctx) return nullptr;
    ctx->last_error = RWKV_ERROR_NONE;
    CTX_CHECK(ctx, RWKV_ERROR_CTX | RWKV_ERROR_UNSUPPORTED, nullptr, ctx->pipe == nullptr,
              "A layer pipeline context cannot be replicated onto one device (use rwkv_clone_context)");
    int ndev = 0;
    (void)hipGetDeviceCount(&ndev);
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, nullptr, device >= 0 && device < ndev, "Device %d out of range (0 .. %d)", device,
              ndev - 1);
    SharedModel * src = ctx->model;
    if (device == src->dm.device) return rwkv_clone_context(ctx, n_threads);
    std::lock_guard<std::mutex> lk(g_model_mutex);
    SharedModel * sm = nullptr;
    auto it = g_replicas.find(replica_key(src, device));
    if (it != g_replicas.end()) {
        sm = it->second;
    } else {
        // first context on this GPU: upload the same file and layer range there
        try {
            ModelFile mf;
            CTX_CHECK(ctx, RWKV_ERROR_MODEL | RWKV_ERROR_FILE, nullptr,
                      load_model_file(src->path.c_str(), mf, src->layer_begin, src->layer_end),
                      "Failed to re-read %s for device %d", src->path.c_str(), device);
            sm = new (std::nothrow) SharedModel();
            CTX_CHECK(ctx, RWKV_ERROR_CTX | RWKV_ERROR_ALLOC, nullptr, sm != nullptr, "Failed to allocate model");
            sm->dm.device = device;
            sm->path = src->path;
            sm->layer_begin = src->layer_begin;
            sm->layer_end = src->layer_end;
            if (hipSetDevice(device) != hipSuccess || !upload_model(mf, sm->dm, src->layer_begin, src->layer_end)) {
                free_model(sm->dm);
                delete sm;
                (void)hipSetDevice(src->dm.device);
                CTX_CHECK(ctx, RWKV_ERROR_MODEL | RWKV_ERROR_ALLOC, nullptr, false, "Failed to upload the model to GPU %d",
                          device);
            }
        } catch (const std::exception & e) {
            if (sm) free_model(sm->dm);
            delete sm;
            CTX_CHECK(ctx, RWKV_ERROR_CTX | RWKV_ERROR_ALLOC, nullptr, false, "Failed to replicate %s: %s",
                      src->path.c_str(), e.what());
        }
    }
    rwkv_context * c = new_context(sm, n_threads);
    (void)hipSetDevice(src->dm.device);
    if (!c) {
        if (it == g_replicas.end()) {
            free_model(sm->dm);
            delete sm;
        }
        ctx->last_error = ctx->last_error | RWKV_ERROR_CTX | RWKV_ERROR_ALLOC;
        return nullptr;
    }
    c->print_errors = ctx->print_errors;
    if (it == g_replicas.end()) g_replicas.emplace(replica_key(sm, device), sm);
    return c;
}

RWKV_API int rwkv_mi355x_context_device(const struct rwkv_context * ctx) { return ctx ? ctx->model->dm.device : -1; }

static bool pipe_eval(struct rwkv_context * ctx, const uint32_t * tokens, size_t T, const float * state_in,
                      float * state_out, float * logits_out, size_t chunk = 0) {
    CTX_CHECK(ctx, RWKV_ERROR_CTX, false,
              ctx->pipe->eval(tokens, T, state_in, state_out, logits_out, ctx->engine->layer_state_len(), chunk),
              "GPU evaluation failed (layer pipeline)");
    return true;
}

RWKV_API bool rwkv_eval(struct rwkv_context * ctx, const uint32_t token, const float * state_in, float * state_out,
                        float * logits_out) {
    ctx->last_error = RWKV_ERROR_NONE;
    const size_t n_vocab = ctx->model->dm.n_vocab;
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, token < n_vocab, "Token (%" PRIu32 ") is out of range (0 .. %zu)", token, n_vocab - 1);
    if (ctx->pipe) return pipe_eval(ctx, &token, 1, state_in, state_out, logits_out);
    CTX_CHECK(ctx, RWKV_ERROR_CTX | RWKV_ERROR_UNSUPPORTED, false, !ctx->model->dm.partial(),
              "This context holds layers [%u, %u) only (a pipeline stage): use rwkv_mi355x_eval_layers",
              ctx->model->dm.layer_lo, ctx->model->dm.layer_hi);
    use_device(ctx);
    CTX_CHECK(ctx, RWKV_ERROR_CTX, false, ctx->engine->eval(&token, 1, state_in, state_out, logits_out), "GPU evaluation failed");
    return true;
}

static bool eval_sequence(struct rwkv_context * ctx, const uint32_t * tokens, const size_t T, const float * state_in,
                          float * state_out, float * logits_out, size_t pipe_chunk);

RWKV_API bool rwkv_eval_sequence(struct rwkv_context * ctx, const uint32_t * tokens, const size_t T, const float * state_in,
                                 float * state_out, float * logits_out) {
    return eval_sequence(ctx, tokens, T, state_in, state_out, logits_out, 0);
}

static bool eval_sequence(struct rwkv_context * ctx, const uint32_t * tokens, const size_t T, const float * state_in,
                          float * state_out, float * logits_out, size_t pipe_chunk) {
    ctx->last_error = RWKV_ERROR_NONE;
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, T > 0, "Sequence length is 0");
    if (!tokens) return true;  // build/cache only (rwkv_eval_inc:102,122): workspace is allocated lazily
    if (T == 1) return rwkv_eval(ctx, tokens[0], state_in, state_out, logits_out);
    if (ctx->pipe) {
        const size_t nv = ctx->model->dm.n_vocab;
        for (size_t i = 0; i < T; i++)
            CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, tokens[i] < nv, "Token at index %zu (%" PRIu32 ") is out of range (0 .. %zu)",
                      i, tokens[i], nv - 1);
        return pipe_eval(ctx, tokens, T, state_in, state_out, logits_out, pipe_chunk);
    }
    CTX_CHECK(ctx, RWKV_ERROR_CTX | RWKV_ERROR_UNSUPPORTED, false, !ctx->model->dm.partial(),
              "This context holds layers [%u, %u) only (a pipeline stage): use rwkv_mi355x_eval_layers",
              ctx->model->dm.layer_lo, ctx->model->dm.layer_hi);
    const size_t n_vocab = ctx->model->dm.n_vocab;
    for (size_t i = 0; i < T; i++) {
        CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, tokens[i] < n_vocab, "Token at index %zu (%" PRIu32 ") is out of range (0 .. %zu)",
                  i, tokens[i], n_vocab - 1);
    }
    use_device(ctx);
    CTX_CHECK(ctx, RWKV_ERROR_CTX, false, ctx->engine->eval(tokens, T, state_in, state_out, logits_out), "GPU evaluation failed");
    return true;
}

RWKV_API bool rwkv_eval_sequence_in_chunks(struct rwkv_context * ctx, const uint32_t * tokens, const size_t T,
                                           const size_t chunk_size, const float * state_in, float * state_out,
                                           float * logits_out) {
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, T > 0, "Sequence length is 0");
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, chunk_size > 0, "Chunk size is 0");
    // The per-token arithmetic of this engine does not depend on how a sequence is cut, so the
    // chunked call is one device-resident pass (state never returns to the host in between);
    // results are bit-identical to the reference's chunk loop (rwkv_eval.inc:158-221).  A layer
    // pipeline context takes chunk_size as its chunk (the unit that moves between stages).
    return eval_sequence(ctx, tokens, T, state_in, state_out, logits_out, chunk_size);
}

RWKV_API size_t rwkv_get_n_vocab(const struct rwkv_context * ctx) { return ctx->model->dm.n_vocab; }
RWKV_API size_t rwkv_get_n_embed(const struct rwkv_context * ctx) { return ctx->model->dm.n_embed; }
RWKV_API size_t rwkv_get_n_layer(const struct rwkv_context * ctx) { return ctx->model->dm.n_layer; }
RWKV_API size_t rwkv_get_state_len(const struct rwkv_context * ctx) { return ctx->model->dm.state_len; }
RWKV_API size_t rwkv_get_logits_len(const struct rwkv_context * ctx) { return ctx->model->dm.n_vocab; }

RWKV_API uint32_t rwkv_get_state_buffer_element_count(const struct rwkv_context * ctx) { return (uint32_t)rwkv_get_state_len(ctx); }
RWKV_API uint32_t rwkv_get_logits_buffer_element_count(const struct rwkv_context * ctx) { return (uint32_t)rwkv_get_logits_len(ctx); }

RWKV_API void rwkv_init_state(const struct rwkv_context * ctx, float * state) {
    const DeviceModel & dm = ctx->model->dm;
    memset(state, 0, dm.state_len * sizeof(float));
    if (dm.major >= 5) return;
    const size_t C = dm.n_embed;
    for (size_t l = 0; l < dm.n_layer; l++)
        for (size_t i = 4 * C; i < 5 * C; i++) state[l * 5 * C + i] = -1e30f;
}

RWKV_API void rwkv_free(struct rwkv_context * ctx) { free_context(ctx); }

static void free_context(struct rwkv_context * ctx) {
    if (!ctx) return;
    delete ctx->pipe;  // before the stage engines it drives
    ctx->pipe = nullptr;
    for (rwkv_context * s : ctx->stages) free_context(s);
    ctx->stages.clear();
    delete ctx->engine;
    SharedModel * sm = ctx->model;
    delete ctx;
    std::lock_guard<std::mutex> lk(g_model_mutex);
    if (--sm->refcount == 0) {
        auto it = g_replicas.find(replica_key(sm, sm->dm.device));
        if (it != g_replicas.end() && it->second == sm) g_replicas.erase(it);
        (void)hipSetDevice(sm->dm.device);
        free_model(sm->dm);
        delete sm;
    }
}

RWKV_API const char * rwkv_get_system_info_string(void) {
    static std::string s;
    static std::once_flag once;
    std::call_once(once, []() {
        int n = 0, rt = 0;
        (void)hipGetDeviceCount(&n);
        (void)hipRuntimeGetVersion(&rt);
        s = "HIP=1 HIP_RUNTIME=" + std::to_string(rt) + " DEVICES=" + std::to_string(n);
        if (n > 0) {
            hipDeviceProp_t p;
            if (hipGetDeviceProperties(&p, 0) == hipSuccess) {
                s += std::string(" GFX=") + p.gcnArchName + " CUS=" + std::to_string(p.multiProcessorCount) +
                     " HBM_GB=" + std::to_string((unsigned long long)(p.totalGlobalMem >> 30));
            }
        }
        s += " CPU_PATH=0";
    });
    return s.c_str();
}

// ------------------------------------------------------------------ additive extensions

// Every stage of a pipeline context holds its own layers' slice: the whole-state calls move each
// stage's slice (state + l0 * layer_len) on that stage's GPU.
static std::vector<rwkv_context *> all_stages(rwkv_context * ctx) {
    std::vector<rwkv_context *> v = {ctx};
    v.insert(v.end(), ctx->stages.begin(), ctx->stages.end());
    return v;
}

RWKV_API bool rwkv_mi355x_state_upload(struct rwkv_context * ctx, const float * state) {
    if (!ctx || !ctx->engine) return false;
    if (ctx->pipe) {
        const size_t per = ctx->engine->layer_state_len();
        for (rwkv_context * s : all_stages(ctx)) {
            use_device(s);
            const DeviceModel & dm = s->model->dm;
            CTX_CHECK(ctx, RWKV_ERROR_CTX, false,
                      s->engine->state_upload_layers(state ? state + (size_t)dm.layer_lo * per : nullptr, dm.layer_lo,
                                                     dm.layer_hi),
                      "State upload failed (pipeline stage on device %d)", dm.device);
        }
        use_device(ctx);
        return true;
    }
    use_device(ctx);
    return ctx->engine->state_upload(state);
}
RWKV_API bool rwkv_mi355x_state_download(struct rwkv_context * ctx, float * state) {
    if (!ctx || !ctx->engine || !state) return false;
    if (ctx->pipe) {
        const size_t per = ctx->engine->layer_state_len();
        for (rwkv_context * s : all_stages(ctx)) {
            use_device(s);
            const DeviceModel & dm = s->model->dm;
            CTX_CHECK(ctx, RWKV_ERROR_CTX, false,
                      s->engine->state_download_layers(state + (size_t)dm.layer_lo * per, dm.layer_lo, dm.layer_hi),
                      "State download failed (pipeline stage on device %d)", dm.device);
        }
        use_device(ctx);
        return true;
    }
    use_device(ctx);
    return ctx->engine->state_download(state);
}

RWKV_API size_t rwkv_mi355x_layer_state_len(const struct rwkv_context * ctx) {
    return ctx && ctx->engine ? ctx->engine->layer_state_len() : 0;
}

static bool layer_range_ok(rwkv_context * ctx, uint32_t l0, uint32_t l1) {
    if (!ctx || !ctx->engine) return false;
    const uint32_t n = ctx->model->dm.n_layer;
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, l0 < l1 && l1 <= n, "Bad layer range [%u, %u) for %u layers", l0, l1, n);
    return true;
}

RWKV_API bool rwkv_mi355x_state_upload_layers(struct rwkv_context * ctx, const float * slice, uint32_t layer_begin,
                                              uint32_t layer_end) {
    ctx->last_error = RWKV_ERROR_NONE;
    if (!layer_range_ok(ctx, layer_begin, layer_end)) return false;
    use_device(ctx);
    CTX_CHECK(ctx, RWKV_ERROR_CTX, false, ctx->engine->state_upload_layers(slice, layer_begin, layer_end),
              "State upload failed");
    return true;
}

RWKV_API bool rwkv_mi355x_state_download_layers(struct rwkv_context * ctx, float * slice, uint32_t layer_begin,
                                                uint32_t layer_end) {
    ctx->last_error = RWKV_ERROR_NONE;
    if (!layer_range_ok(ctx, layer_begin, layer_end)) return false;
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, slice != nullptr, "NULL state slice");
    use_device(ctx);
    CTX_CHECK(ctx, RWKV_ERROR_CTX, false, ctx->engine->state_download_layers(slice, layer_begin, layer_end),
              "State download failed");
    return true;
}

RWKV_API void rwkv_mi355x_state_io_bytes(const struct rwkv_context * ctx, double out[2]) {
    if (!out) return;
    out[0] = ctx && ctx->engine ? ctx->engine->io_bytes_h2d() : 0.0;
    out[1] = ctx && ctx->engine ? ctx->engine->io_bytes_d2h() : 0.0;
}

RWKV_API bool rwkv_mi355x_eval_device(struct rwkv_context * ctx, const uint32_t * tokens, size_t T, bool compute_logits,
                                      float * logits_out, bool sync) {
    if (!ctx || !ctx->engine) return false;
    ctx->last_error = RWKV_ERROR_NONE;
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, T > 0 && tokens != nullptr, "Sequence length is 0");
    CTX_CHECK(ctx, RWKV_ERROR_CTX | RWKV_ERROR_UNSUPPORTED, false, !ctx->model->dm.partial(),
              "This context holds layers [%u, %u) only (a pipeline stage)", ctx->model->dm.layer_lo, ctx->model->dm.layer_hi);
    for (size_t i = 0; i < T; i++)
        CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, tokens[i] < ctx->model->dm.n_vocab, "Token out of range");
    use_device(ctx);
    CTX_CHECK(ctx, RWKV_ERROR_CTX, false, ctx->engine->eval_device(tokens, T, compute_logits || logits_out, logits_out, sync), "GPU evaluation failed");
    return true;
}

static bool eval_layers(struct rwkv_context * ctx, const uint32_t * tokens, size_t T, uint32_t layer_begin,
                        uint32_t layer_end, float * x_dev, float * vfirst_dev, bool compute_logits, float * logits_out,
                        bool sync) {
    if (!ctx || !ctx->engine) return false;
    ctx->last_error = RWKV_ERROR_NONE;
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, sync || logits_out == nullptr, "Asynchronous stage: logits stay on the device");
    const DeviceModel & dm = ctx->model->dm;
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, T > 0, "Sequence length is 0");
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, layer_begin < layer_end && layer_end <= dm.n_layer, "Bad layer range");
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, layer_begin >= dm.layer_lo && layer_end <= dm.layer_hi,
              "Layers [%u, %u) are not resident in this context (it holds [%u, %u))", layer_begin, layer_end, dm.layer_lo,
              dm.layer_hi);
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, layer_begin == 0 || x_dev != nullptr, "x_dev required after layer 0");
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, layer_begin == 0 || dm.major != 7 || vfirst_dev != nullptr,
              "vfirst_dev required after layer 0 (v7)");
    if (layer_begin == 0) {
        CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, tokens != nullptr, "Tokens required at layer 0");
        for (size_t i = 0; i < T; i++) CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, tokens[i] < dm.n_vocab, "Token out of range");
    }
    use_device(ctx);
    CTX_CHECK(ctx, RWKV_ERROR_CTX, false,
              ctx->engine->eval_layers(tokens, T, layer_begin, layer_end, x_dev, vfirst_dev, compute_logits, logits_out,
                                       sync),
              "GPU evaluation failed");
    return true;
}

RWKV_API bool rwkv_mi355x_eval_layers(struct rwkv_context * ctx, const uint32_t * tokens, size_t T,
                                      uint32_t layer_begin, uint32_t layer_end, float * x_dev, float * vfirst_dev,
                                      bool compute_logits, float * logits_out) {
    return eval_layers(ctx, tokens, T, layer_begin, layer_end, x_dev, vfirst_dev, compute_logits, logits_out, true);
}

RWKV_API bool rwkv_mi355x_eval_layers_async(struct rwkv_context * ctx, const uint32_t * tokens, size_t T,
                                            uint32_t layer_begin, uint32_t layer_end, float * x_dev, float * vfirst_dev,
                                            bool compute_logits) {
    return eval_layers(ctx, tokens, T, layer_begin, layer_end, x_dev, vfirst_dev, compute_logits, nullptr, false);
}

RWKV_API float * rwkv_mi355x_logits_device(struct rwkv_context * ctx) {
    return ctx && ctx->engine ? ctx->engine->device_logits() : nullptr;
}

static bool eval_batch(struct rwkv_context * ctx, const uint32_t * tokens, size_t n, const float * state_in,
                       float * state_out, float * logits_out, bool dev) {
    if (!ctx || !ctx->engine) return false;
    ctx->last_error = RWKV_ERROR_NONE;
    const DeviceModel & dm = ctx->model->dm;
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, n > 0 && tokens != nullptr, "Batch is empty");
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, n <= (size_t)Engine::kBatchMax, "Batch of %zu contexts (at most %d)", n,
              Engine::kBatchMax);
    CTX_CHECK(ctx, RWKV_ERROR_CTX | RWKV_ERROR_UNSUPPORTED, false, !dm.partial(),
              "This context holds layers [%u, %u) only (a pipeline stage)", dm.layer_lo, dm.layer_hi);
    CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, !dev || state_in == nullptr || state_in != state_out,
              "Device batch: state_in and state_out must be different buffers");
    for (size_t i = 0; i < n; i++)
        CTX_CHECK(ctx, RWKV_ERROR_ARGS, false, tokens[i] < dm.n_vocab, "Token at index %zu (%" PRIu32 ") is out of range",
                  i, tokens[i]);
    use_device(ctx);
    CTX_CHECK(ctx, RWKV_ERROR_CTX, false, ctx->engine->eval_batch(tokens, n, state_in, state_out, logits_out, dev),
              "GPU evaluation failed");
    return true;
}

RWKV_API bool rwkv_mi355x_eval_batch(struct rwkv_context * ctx, const uint32_t * tokens, size_t n_contexts,
                                     const float * state_in, float * state_out, float * logits_out) {
    return eval_batch(ctx, tokens, n_contexts, state_in, state_out, logits_out, false);
}

RWKV_API bool rwkv_mi355x_eval_batch_device(struct rwkv_context * ctx, const uint32_t * tokens, size_t n_contexts,
                                            const float * state_in, float * state_out, float * logits_out) {
    return eval_batch(ctx, tokens, n_contexts, state_in, state_out, logits_out, true);
}


RWKV_API bool rwkv_mi355x_sync(struct rwkv_context * ctx) {
    if (!ctx || !ctx->engine) return false;
    bool ok = true;
    for (rwkv_context * s : all_stages(ctx)) {
        use_device(s);
        ok = s->engine->sync() && ok;
    }
    use_device(ctx);
    CTX_CHECK(ctx, RWKV_ERROR_CTX, false, ok, "GPU evaluation failed (reported at synchronisation)");
    return true;
}
RWKV_API long long rwkv_mi355x_debug_buffer(struct rwkv_context * ctx, const char * name, void * out, size_t bytes) {
    return ctx && ctx->engine ? ctx->engine->debug_copy(name, out, bytes) : -1;
}
RWKV_API bool rwkv_mi355x_debug_set(struct rwkv_context * ctx, const char * name, long long value) {
    if (!ctx || !ctx->engine) return false;
    bool ok = true;
    for (rwkv_context * s : all_stages(ctx)) {
        use_device(s);
        ok = s->engine->debug_set(name, value) && ok;
    }
    use_device(ctx);
    return ok;
}
RWKV_API void * rwkv_mi355x_stream(struct rwkv_context * ctx) {
    if (!ctx || !ctx->engine) return nullptr;
    CTX_CHECK(ctx, RWKV_ERROR_CTX | RWKV_ERROR_UNSUPPORTED, nullptr, ctx->pipe == nullptr,
              "A layer pipeline context has one stream per stage");
    return (void *)ctx->engine->stream();
}
RWKV_API float * rwkv_mi355x_device_state(struct rwkv_context * ctx) {
    if (!ctx || !ctx->engine) return nullptr;
    CTX_CHECK(ctx, RWKV_ERROR_CTX | RWKV_ERROR_UNSUPPORTED, nullptr, ctx->pipe == nullptr,
              "A layer pipeline context's state is split over its stages");
    return ctx->engine->device_state();
}

RWKV_API double rwkv_mi355x_weight_bytes(const struct rwkv_context * ctx, bool with_head) {
    if (!ctx) return 0.0;
    const DeviceModel & dm = ctx->model->dm;
    return dm.layer_weight_bytes + (with_head ? dm.head_weight_bytes : 0.0);
}

RWKV_API double rwkv_mi355x_decode_bytes(const struct rwkv_context * ctx, bool with_logits) {
    if (!ctx) return 0.0;
    const DeviceModel & dm = ctx->model->dm;
    // weights + per-token small parameters + state read and written + embedding row
    double b = dm.layer_weight_bytes + dm.small_param_bytes + 2.0 * (double)dm.state_len * 4.0;
    b += (double)dm.n_embed * (dm.emb.type == W_F16 ? 2.0 : 4.0);
    if (with_logits) b += dm.head_weight_bytes + (double)dm.n_vocab * 4.0;
    return b;
}

RWKV_API double rwkv_mi355x_matmul_flops_per_token(const struct rwkv_context * ctx, bool with_head) {
    if (!ctx) return 0.0;
    const DeviceModel & dm = ctx->model->dm;
    return dm.layer_flops + (with_head ? dm.head_flops : 0.0);
}

RWKV_API void rwkv_mi355x_arch(const struct rwkv_context * ctx, int64_t out[4]) {
    if (!out) return;
    if (!ctx) {
        out[0] = out[1] = out[2] = out[3] = 0;
        return;
    }
    const DeviceModel & dm = ctx->model->dm;
    out[0] = dm.major;
    out[1] = dm.minor;
    out[2] = dm.H;
    out[3] = dm.S;
}

RWKV_API void rwkv_mi355x_set_kernel_timing(struct rwkv_context * ctx, bool on) {
    if (ctx && ctx->engine) ctx->engine->set_timing(on);
}

RWKV_API int rwkv_mi355x_kernel_stats(struct rwkv_context * ctx, int index, char * name, size_t name_len,
                                      long long * launches, double * total_ms, double * total_bytes,
                                      double * total_flops) {
    if (!ctx || !ctx->engine) return 0;
    const auto & st = ctx->engine->stats();
    if (index < 0 || index >= (int)st.size()) return (int)st.size();
    const KernelStat & k = st[index];
    if (name && name_len) {
        strncpy(name, k.name.c_str(), name_len - 1);
        name[name_len - 1] = 0;
    }
    if (launches) *launches = k.launches;
    if (total_ms) *total_ms = k.total_ms;
    if (total_bytes) *total_bytes = k.total_bytes;
    if (total_flops) *total_flops = k.total_flops;
    return (int)st.size();
}

}  // extern "C"
