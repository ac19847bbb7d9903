// stamp.hpp -- in-kernel phase timestamps for the decode chain (diagnostic builds only).
//
// Compiled in only with -DRWKV_STAMP (make stamp -> build_stamp/librwkv.so); the product build
// expands every macro to nothing.  Each instrumented workgroup takes a slot in a per-CU ring
// (one atomic on its CU's own counter at kernel start, so WGs never contend across CUs) and
// thread 0 writes {start, mid, end, tag} with s_memrealtime (100 MHz, one clock for the whole
// chip) plus, in the tag word's top 20 bits, the shader-clock cycles (s_memtime) from start to
// end, so tools/stamp_run.py reports the clock the chain runs at.  mid = the kernel's "inputs ready" point (after its first dependent wait).  The
// engine dumps the rings to $RWKV_STAMP_OUT when the context is freed; tools/stamp_summary.py
// splits them into launches by time order.
#pragma once
#include <hip/hip_runtime.h>

namespace rwkvmi {

constexpr int kStampCUs = 2048;   // (xcc, se, sh, cu) slots
constexpr int kStampRing = 4096;  // records per CU

struct StampCtl {
    unsigned long long * buf;  // [kStampCUs][kStampRing][8]
    unsigned * ctr;            // [kStampCUs]
};

#ifdef RWKV_STAMP
// one copy per translation unit; the engine sets every copy (stamp_register below)
static __device__ StampCtl g_stampctl;

int stamp_register(void (*setter)(const StampCtl &));
static void stamp_set_tu_(const StampCtl & c) { (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stampctl), &c, sizeof c); }
static int stamp_reg_tu_ = stamp_register(stamp_set_tu_);

__device__ __forceinline__ unsigned stamp_cu() {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID
    const unsigned cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    return (((xcc & 7) * 8 + se) * 2 + sh) * 16 + cu;
}

// extra phase points of another wave (STAMP_X(i)), carried to thread 0 through LDS
#define STAMP_BEGIN()                                                            \
    __shared__ unsigned long long stamp_x_[4];                                    \
    if (threadIdx.x < 4) stamp_x_[threadIdx.x] = 0;                               \
    unsigned long long stamp_t0_ = __builtin_amdgcn_s_memrealtime();              \
    const unsigned long long stamp_c0_ = __builtin_amdgcn_s_memtime();            \
    unsigned long long stamp_t1_ = 0;                                             \
    unsigned stamp_slot_ = 0, stamp_cu_ = 0;                                      \
    if (threadIdx.x == 0 && g_stampctl.ctr) {                                     \
        stamp_cu_ = stamp_cu();                                                   \
        stamp_slot_ = atomicAdd(&g_stampctl.ctr[stamp_cu_], 1u) % kStampRing;     \
    }
#define STAMP_X(i)                                                    \
    do {                                                              \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   \
        if ((threadIdx.x & 63) == 0) stamp_x_[i] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
// STAMP_XN: the time this wave got here, without waiting for its outstanding loads
#define STAMP_XN(i)                                                                  \
    do {                                                                             \
        if ((threadIdx.x & 63) == 0) stamp_x_[i] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define STAMP_MID()                                          \
    do {                                                     \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
        stamp_t1_ = __builtin_amdgcn_s_memrealtime();        \
    } while (0)
#define STAMP_END(kid)   \
    do {                  \
        __syncthreads();  \
        STAMP_END_NS(kid); \
    } while (0)
#define STAMP_END_NS(kid)                                                                                \
    do {                                                                                                 \
        if (threadIdx.x == 0 && g_stampctl.buf) {                                                        \
            unsigned long long * r_ = g_stampctl.buf + ((size_t)stamp_cu_ * kStampRing + stamp_slot_) * 8; \
            r_[0] = stamp_t0_;                                                                           \
            r_[1] = stamp_t1_;                                                                           \
            r_[2] = __builtin_amdgcn_s_memrealtime();                                                    \
            const unsigned long long cyc_ = (__builtin_amdgcn_s_memtime() - stamp_c0_) & 0xFFFFFull;    \
            r_[3] = (cyc_ << 44) | ((unsigned long long)(kid) << 32) | blockIdx.x;                      \
            for (int q_ = 0; q_ < 4; q_++) r_[4 + q_] = stamp_x_[q_];                                    \
        }                                                                                                \
    } while (0)
#else
#define STAMP_X(i) \
    do {           \
    } while (0)
#define STAMP_XN(i) \
    do {            \
    } while (0)
#define STAMP_BEGIN()
#define STAMP_MID() \
    do {            \
    } while (0)
#define STAMP_END(kid) \
    do {               \
    } while (0)
#define STAMP_END_NS(kid) \
    do {                  \
    } while (0)
#endif

}  // namespace rwkvmi
