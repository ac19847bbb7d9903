// errors.hpp -- the rwkv.h error-flag convention (reference rwkv_error_handling.inc:1-95):
// flags are OR-ed into a thread-local global (init / quantize) or a per-context field (eval),
// read-and-cleared by rwkv_get_last_error, printed to stderr unless printing is disabled.
#pragma once

#include <stdio.h>

#include "../../include/rwkv.h"

namespace rwkvmi {

extern thread_local enum rwkv_error_flags g_last_error;
extern thread_local bool g_print_errors;

inline enum rwkv_error_flags operator|(enum rwkv_error_flags a, enum rwkv_error_flags b) {
    return static_cast<enum rwkv_error_flags>(static_cast<int>(a) | static_cast<int>(b));
}

inline void add_error(enum rwkv_error_flags f) { g_last_error = g_last_error | f; }

}  // namespace rwkvmi

// global-error assertion: on failure OR flags into the thread-local error, print, return RET
#define RWKV_CHECK(FLAGS, RET, cond, ...)                                 \
    do {                                                                  \
        if (!(cond)) {                                                    \
            ::rwkvmi::add_error(FLAGS);                                   \
            if (::rwkvmi::g_print_errors) {                               \
                fprintf(stderr, __VA_ARGS__);                             \
                fprintf(stderr, "\n%s:%d: %s\n", __FILE__, __LINE__, #cond); \
            }                                                             \
            return RET;                                                   \
        }                                                                 \
    } while (0)
