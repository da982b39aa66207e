// Shared helpers for the pcseg HIP library (gfx950 / CDNA4, wave64).
//
// Conventions of the C ABI (include/pcseg.h):
//   * every entry point takes caller-owned device pointers, plain sizes and a
//     hipStream_t passed as void*; no allocation, no host sync inside;
//   * returns 0 on success, otherwise a hipError_t-compatible code, with a
//     thread-local message readable through pcs_last_error().
#pragma once

#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <functional>

#include "../../include/pcseg.h"   // the ABI this library implements (prototype check)

#define PCS_API extern "C" __attribute__((visibility("default")))

// Device-side bounds checks of the debug library (`make debug` -> libpcseg_debug.so, built with
// -DPCS_DEBUG_BOUNDS): every clamped operand access of the row GEMM, row / wide weight gradients,
// LDS-DMA data gradient and EdgeConv is checked against its operand's rows and LOGICAL channel
// span (rounded to a quad), and a violation prints the site and traps.  Compiled out otherwise.
#ifdef PCS_DEBUG_BOUNDS
#define PCS_DCHECK(cond, fmt, ...)                                                                  \
    do {                                                                                            \
        if (!(cond)) {                                                                              \
            printf("pcs bounds: %s:%d: " fmt "\n", __FILE__, __LINE__, ##__VA_ARGS__);             \
            __builtin_trap();                                                                       \
        }                                                                                           \
    } while (0)
#else
#define PCS_DCHECK(cond, fmt, ...) \
    do {                           \
    } while (0)
#endif

// debug: the 16-B access at p lies in the first `rows` rows of the row-major operand at base (row
// stride ld floats) and inside its first `width` channels rounded up to a quad
#define PCS_DCHECK_QUAD(p, base, rows, ld, width, what)                                                  \
    do {                                                                                                 \
        const long long o_ = (long long)((p) - (base));                                                  \
        const long long r_ = o_ / (ld), c_ = o_ - r_ * (ld);                                             \
        PCS_DCHECK(o_ >= 0 && r_ < (long long)(rows) && c_ + 4 <= (long long)(((width) + 3) & ~3),       \
                   "%s: row %lld col %lld outside %lld x %d (ld %d)", what, r_, c_, (long long)(rows),   \
                   (int)(width), (int)(ld));                                                             \
    } while (0)

namespace pcs {

// ------------------------------------------------------------ launch probe (probe.cpp)
// While enabled (pcs_probe_begin .. pcs_probe_end), a launch bracketed by probe_start /
// probe_stop is timed by two HIP events on its own stream and recorded with the kernel
// name as rocprofv3 reports it and its algorithmic flops / bytes (bench.py's roofline).
bool probe_enabled();
int probe_start(const char* name, double flops, double bytes, hipStream_t s, std::function<void()> relaunch);
void probe_stop(int idx, hipStream_t s);

// scoped form for single-launch entry points: the name is formatted only while probing
struct ProbeScope {
    int idx = -1;
    hipStream_t s;
    ProbeScope(hipStream_t st, double flops, double bytes, const char* fmt, ...) : s(st) {
        if (!probe_enabled()) return;
        char nm[128];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(nm, sizeof nm, fmt, ap);
        va_end(ap);
        idx = probe_start(nm, flops, bytes, st, {});
    }
    ~ProbeScope() { probe_stop(idx, s); }
    ProbeScope(const ProbeScope&) = delete;
    ProbeScope& operator=(const ProbeScope&) = delete;
};

// ------------------------------------------------------------ error plumbing
void set_error(const char* fmt, ...);
int launch_status(const char* what);   // reads hipGetLastError after a launch

#define PCS_CHECK_ARG(cond, ...)                                   \
    do {                                                           \
        if (!(cond)) {                                             \
            ::pcs::set_error(__VA_ARGS__);                         \
            return (int)hipErrorInvalidValue;                      \
        }                                                          \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------ device helpers
constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }

// lanes strictly below this one
__device__ __forceinline__ unsigned long long lanemask_lt() {
    const int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

__device__ __forceinline__ int popc64(unsigned long long m) { return __popcll(m); }

__device__ __forceinline__ int ffs64(unsigned long long m) { return __ffsll((long long)m) - 1; }

// wave-uniform read of lane `l` (l must be wave-uniform)
__device__ __forceinline__ unsigned readlane_u(unsigned v, int l) {
    return (unsigned)__builtin_amdgcn_readlane((int)v, l);
}
// lane `l` (wave-uniform) takes v: one v_cmp + v_cndmask, visible to the compiler
__device__ __forceinline__ unsigned writelane_u(unsigned old, unsigned v, int l) {
    return lane_id() == l ? v : old;
}
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// IEEE correctly rounded single-precision sqrt of x >= 0 (the CPU's sqrtf).  On gfx950
// __fsqrt_rn / sqrtf lower to v_sqrt_f32, which is only faithful (1 ulp): the hardware
// value t is fixed up against the exact midpoints to its float neighbours -- t and a
// neighbour average to a 25-bit value and its square to 50 bits, both exact in double.
__device__ __forceinline__ float sqrt_cr(float x) {
    float t = __builtin_sqrtf(x);
    if (!(t < __builtin_inff())) return t;            // inf / NaN pass through
    const double xd = (double)x;
    const float tu = __uint_as_float(__float_as_uint(t) + 1u);          // next float up (t >= 0)
    const double mu = 0.5 * ((double)t + (double)tu);
    if (mu * mu < xd) t = tu;
    const float td = t > 0.f ? __uint_as_float(__float_as_uint(t) - 1u) : 0.f;   // next float down
    const double md = 0.5 * ((double)t + (double)td);
    if (md * md > xd) t = td;
    return t;
}

// bit pattern of a non-negative float (incl. +inf) orders like the float
__device__ __forceinline__ unsigned fbits(float x) { return __float_as_uint(x); }

// un-fused squared distance, evaluated exactly like the reference's
// ((p - c) ** 2).sum(-1) on the CPU: ((dx*dx + dy*dy) + dz*dz), no FMA.
__device__ __forceinline__ float sqdist_unfused(float px, float py, float pz, float cx, float cy, float cz) {
    const float dx = __fsub_rn(px, cx);
    const float dy = __fsub_rn(py, cy);
    const float dz = __fsub_rn(pz, cz);
    return __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
}

}  // namespace pcs
