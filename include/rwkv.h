/*
 * rwkv.h -- the drop-in C ABI of the MI355X RWKV eval library (librwkv.so).
 *
 * Every declaration here keeps the exact signature, value and meaning of the
 * reference's public header (cogpy/rwkv.cppy rwkv.h) so the reference's
 * python/rwkv_cpp ctypes wrapper and native callers (esn.cpp) bind unchanged.
 * Citations are reference file:line of the declaration each entry replaces.
 *
 * Behavioural notes specific to this implementation:
 *   - evaluation always runs on the MI355X (HIP device 0 unless RWKV_MI355X_DEVICE is set);
 *     n_gpu_layers is accepted for ABI compatibility and does not select a CPU path --
 *     there is no CPU compute path in this library.  Without a usable GPU,
 *     rwkv_init_from_file fails with RWKV_ERROR_CTX | RWKV_ERROR_UNSUPPORTED.
 *   - n_threads is accepted and ignored (no CPU thread pool).
 */
#ifndef RWKV_H
#define RWKV_H

#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>

#if defined(RWKV_SHARED) || defined(RWKV_BUILD)
#    define RWKV_API __attribute__ ((visibility ("default")))
#else
#    define RWKV_API
#endif

/* reference rwkv.h:23-30 */
#define RWKV_FILE_MAGIC 0x67676d66
#define RWKV_FILE_VERSION_0 100
#define RWKV_FILE_VERSION_1 101
#define RWKV_FILE_VERSION_MIN RWKV_FILE_VERSION_0
#define RWKV_FILE_VERSION_MAX RWKV_FILE_VERSION_1
#define RWKV_FILE_VERSION RWKV_FILE_VERSION_MAX

#if defined(__cplusplus)
extern "C" {
#endif

/* reference rwkv.h:38-62: flags = category | code */
enum rwkv_error_flags {
    RWKV_ERROR_NONE = 0,

    RWKV_ERROR_ARGS = 1 << 8,
    RWKV_ERROR_FILE = 2 << 8,
    RWKV_ERROR_MODEL = 3 << 8,
    RWKV_ERROR_MODEL_PARAMS = 4 << 8,
    RWKV_ERROR_GRAPH = 5 << 8,
    RWKV_ERROR_CTX = 6 << 8,

    RWKV_ERROR_ALLOC = 1,
    RWKV_ERROR_FILE_OPEN = 2,
    RWKV_ERROR_FILE_STAT = 3,
    RWKV_ERROR_FILE_READ = 4,
    RWKV_ERROR_FILE_WRITE = 5,
    RWKV_ERROR_FILE_MAGIC = 6,
    RWKV_ERROR_FILE_VERSION = 7,
    RWKV_ERROR_DATA_TYPE = 8,
    RWKV_ERROR_UNSUPPORTED = 9,
    RWKV_ERROR_SHAPE = 10,
    RWKV_ERROR_DIMENSION = 11,
    RWKV_ERROR_KEY = 12,
    RWKV_ERROR_DATA = 13,
    RWKV_ERROR_PARAM_MISSING = 14
};

/* Opaque inference context; one eval at a time per context (reference rwkv.h:64-68). */
struct rwkv_context;

/* reference rwkv.h:70-76 */
RWKV_API void rwkv_set_print_errors(struct rwkv_context * ctx, const bool print_errors);
/* reference rwkv.h:78-80 */
RWKV_API bool rwkv_get_print_errors(const struct rwkv_context * ctx);
/* reference rwkv.h:82-84: reads AND clears the flags (NULL ctx: thread-local global flags) */
RWKV_API enum rwkv_error_flags rwkv_get_last_error(struct rwkv_context * ctx);

/* reference rwkv.h:86-91 */
RWKV_API struct rwkv_context * rwkv_init_from_file(const char * model_file_path, const uint32_t n_threads, const uint32_t n_gpu_layers);
/* reference rwkv.h:93-99: shares the loaded model (reference-counted) */
RWKV_API struct rwkv_context * rwkv_clone_context(struct rwkv_context * ctx, const uint32_t n_threads);

/* reference rwkv.h:101-116: state_in NULL => fresh state; NULL outputs are skipped;
 * state_in may alias state_out. */
RWKV_API bool rwkv_eval(
    struct rwkv_context * ctx,
    const uint32_t token,
    const float * state_in,
    float * state_out,
    float * logits_out
);

/* reference rwkv.h:118-147: tokens NULL => prepare only (returns true). */
RWKV_API bool rwkv_eval_sequence(
    struct rwkv_context * ctx,
    const uint32_t * tokens,
    const size_t sequence_len,
    const float * state_in,
    float * state_out,
    float * logits_out
);

/* reference rwkv.h:149-173 */
RWKV_API bool rwkv_eval_sequence_in_chunks(
    struct rwkv_context * ctx,
    const uint32_t * tokens,
    const size_t sequence_len,
    const size_t chunk_size,
    const float * state_in,
    float * state_out,
    float * logits_out
);

/* reference rwkv.h:175-198 */
RWKV_API size_t rwkv_get_n_vocab(const struct rwkv_context * ctx);
RWKV_API size_t rwkv_get_n_embed(const struct rwkv_context * ctx);
RWKV_API size_t rwkv_get_n_layer(const struct rwkv_context * ctx);
RWKV_API size_t rwkv_get_state_len(const struct rwkv_context * ctx);
RWKV_API size_t rwkv_get_logits_len(const struct rwkv_context * ctx);

/* reference rwkv.h:200-204 */
RWKV_API void rwkv_init_state(const struct rwkv_context * ctx, float * state);

/* reference rwkv.h:206-208 */
RWKV_API void rwkv_free(struct rwkv_context * ctx);

/* reference rwkv.h:210-221: format_name one of Q4_0 Q4_1 Q5_0 Q5_1 Q8_0 */
RWKV_API bool rwkv_quantize_model_file(const char * model_file_path_in, const char * model_file_path_out, const char * format_name);

/* reference rwkv.h:223-224 */
RWKV_API const char * rwkv_get_system_info_string(void);

/* Legacy exports bound by the Python wrapper (reference rwkv.cpp:145-153,
 * rwkv_cpp_shared_library.py:91-95). */
RWKV_API uint32_t rwkv_get_state_buffer_element_count(const struct rwkv_context * ctx);
RWKV_API uint32_t rwkv_get_logits_buffer_element_count(const struct rwkv_context * ctx);

#if defined(__cplusplus)
}
#endif

#endif
