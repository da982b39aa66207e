// Farthest point sampling, bit-exact with the reference's CPU `sample`
// (models/utils/common.py:6-34).
//
// Reference semantics per step i:
//   dist  = vector_norm(p - p_far) == sqrtf(fmaf(dz,dz, fmaf(dy,dy, dx*dx)))  (CPU ATen)
//   best  = dist where dist < best                                           (:29-30)
//   far   = first index of max(best)                                         (:31)
//
// MI355X design: one workgroup per cloud (clouds are independent; the chain of
// C steps is inherently serial), every point's coordinates and running minimum
// live in registers (PPT points per thread), so a step touches no memory except
// one 16-B LDS slot per wave.  The running minimum is kept SQUARED (sqrt is
// monotone, so min commutes with it); each thread takes its local maximum M,
// and the wave reduces them with DPP row ops + v_readlane; only the wave-level
// maximum is square-rooted (correctly rounded), and the lowest index whose
// sqrt ties it is found by a threshold compare -- so the pick reproduces the
// reference's argmax over sqrt'ed distances, ties included.  Waves combine
// through a double-buffered LDS slot array (one barrier per step).
#include "pcs_common.hpp"

#include <stdlib.h>

namespace pcs {

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int CTRL>
__device__ __forceinline__ unsigned dpp_u(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}

// wave-wide max / min of an unsigned value, result wave-uniform: DPP inside 16-lane
// rows (quad xor1, quad xor2, half-row mirror, row mirror) + v_readlane of the four
// row results.  No LDS round trips.
__device__ __forceinline__ unsigned wave_umax(unsigned v) {
    v = max(v, dpp_u<0xB1>(v));
    v = max(v, dpp_u<0x4E>(v));
    v = max(v, dpp_u<0x141>(v));
    v = max(v, dpp_u<0x140>(v));
    return max(max(readlane_u(v, 0), readlane_u(v, 16)), max(readlane_u(v, 32), readlane_u(v, 48)));
}
__device__ __forceinline__ unsigned wave_umin(unsigned v) {
    v = min(v, dpp_u<0xB1>(v));
    v = min(v, dpp_u<0x4E>(v));
    v = min(v, dpp_u<0x141>(v));
    v = min(v, dpp_u<0x140>(v));
    return min(min(readlane_u(v, 0), readlane_u(v, 16)), min(readlane_u(v, 32), readlane_u(v, 48)));
}

constexpr int kFpsLdsOut = 2048;   // centroids buffered in LDS (written once at the end)

#ifdef PCS_FPS_STAMPS
// diagnostic build only (scripts/fps_stamps.py): per-segment s_memtime cycles of wave 0, block 0
__device__ unsigned long long g_fps_stamps[8];
#define FPS_STAMP(k)                                                                      \
    do {                                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                                \
        unsigned long long tn_;                                                           \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tn_)::"memory");       \
        __builtin_amdgcn_sched_barrier(0);                                                \
        st_acc[k] += tn_ - st_prev;                                                       \
        st_prev = tn_;                                                                    \
    } while (0)
#else
#define FPS_STAMP(k) \
    do {             \
    } while (0)
#endif

constexpr int kFpsLdsCloud = 8192;   // clouds up to this size keep a coordinate copy in LDS

// One step per loop iteration:
//  1. each thread folds the new distances into its squared running minima and takes
//     its local max (squared);
//  2. wave max M* (exact, as float bits) -> S = sqrtf(M*) and lo = the smallest
//     float whose sqrt rounds to S (wave-uniform, sqrts in parallel);
//  3. the wave's candidate = lowest point index with best >= lo, i.e. the lowest
//     index among ALL its points whose reference distance sqrt(best) equals S;
//  4. lane 0 of every wave publishes (S, index) in one LDS slot; after the barrier
//     lane l of every wave reads slot l and the waves redo the (max S, min index)
//     reduction with DPP -- no serial compare chain -- and fetch the winner's
//     coordinates from the LDS copy of the cloud.
// This is exactly the reference's "first index of max(sqrt distances)".
template <int BLOCK, int PPT>
__global__ __launch_bounds__(BLOCK) void fps_kernel(const float* __restrict__ xyz, int N, int C,
                                                    const int* __restrict__ start, int* __restrict__ out_idx,
                                                    float* __restrict__ out_xyz) {
    constexpr int NW = BLOCK / kWave;
    static_assert(NW <= 64, "one slot per lane");
    __shared__ __attribute__((aligned(16))) uint2 s_key[2][NW];   // (sqrt bits + 1, index); 0 = empty
    // Per-step global stores would make every __syncthreads wait for them (the
    // barrier's fence drains vmcnt): keep the picked centroids in LDS instead.
    __shared__ float4 s_out[kFpsLdsOut];
    __shared__ float s_cloud[3 * kFpsLdsCloud];
    const bool lds_out = C <= kFpsLdsOut;
    const bool lds_cloud = N <= kFpsLdsCloud;

    const int b = blockIdx.x;
    const int t = threadIdx.x;
    const int w = t >> 6, lane = t & 63;
    const float* P = xyz + (size_t)b * N * 3;

    if (lds_cloud)
        for (int e = t; e < 3 * N; e += BLOCK) s_cloud[e] = P[e];

    // running minima as float BITS: the squared distances are >= +0 (never -0 or NaN), so
    // unsigned min/max order them exactly like fminf/fmaxf, with no canonicalising op.
    // Padding slots hold 0: never above a real point's value, and a pad's index (>= N)
    // always loses the lowest-index tie break to a real point.
    float px[PPT], py[PPT], pz[PPT];
    unsigned best[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const int p = j * BLOCK + t;
        if (p < N) {
            px[j] = P[3 * p + 0];
            py[j] = P[3 * p + 1];
            pz[j] = P[3 * p + 2];
            best[j] = 0x7f800000u;
        } else {
            px[j] = py[j] = pz[j] = 0.f;
            best[j] = 0u;
        }
    }

    int far = start[b];
    far = far < 0 ? 0 : (far >= N ? N - 1 : far);
    float cx = P[3 * far + 0], cy = P[3 * far + 1], cz = P[3 * far + 2];
    if (lds_cloud) __syncthreads();

#ifdef PCS_FPS_STAMPS
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_prev = __builtin_amdgcn_s_memtime();
#endif
    for (int i = 0; i < C; ++i) {
        FPS_STAMP(0);
        if (t == 0) {
            if (lds_out) {
                s_out[i] = make_float4(cx, cy, cz, __int_as_float(far));
            } else {
                out_idx[(size_t)b * C + i] = far;
                float* o = out_xyz + ((size_t)b * C + i) * 3;
                o[0] = cx;
                o[1] = cy;
                o[2] = cz;
            }
        }
        if (i == C - 1) break;

        unsigned M = 0u;
#ifndef PCS_FPS_SCALAR
        if constexpr (PPT % 2 == 0) {
            // two points per packed op (v_pk_add/mul/fma_f32: per-component IEEE fp32, the
            // same roundings as the scalar chain) -- half the VALU issues of the distances
            const f32x2 c2x = {cx, cx}, c2y = {cy, cy}, c2z = {cz, cz};
#pragma unroll
            for (int j = 0; j < PPT; j += 2) {
                const f32x2 dx = f32x2{px[j], px[j + 1]} - c2x;
                const f32x2 dy = f32x2{py[j], py[j + 1]} - c2y;
                const f32x2 dz = f32x2{pz[j], pz[j + 1]} - c2z;
                const f32x2 d = __builtin_elementwise_fma(dz, dz, __builtin_elementwise_fma(dy, dy, dx * dx));
                best[j] = min(__float_as_uint(d.x), best[j]);
                best[j + 1] = min(__float_as_uint(d.y), best[j + 1]);
                M = max(M, max(best[j], best[j + 1]));
            }
        } else
#endif
        {
#pragma unroll
            for (int j = 0; j < PPT; ++j) {
                const float dx = px[j] - cx, dy = py[j] - cy, dz = pz[j] - cz;
                const float d = __fmaf_rn(dz, dz, __fmaf_rn(dy, dy, __fmul_rn(dx, dx)));
                best[j] = min(__float_as_uint(d), best[j]);   // == (d < best ? d : best)
                M = max(M, best[j]);
            }
        }
        FPS_STAMP(1);
        const unsigned wk = wave_umax(M + 1u);
        FPS_STAMP(2);
        const int buf = i & 1;
        if (wk != 0) {
            const unsigned mb = wk - 1u;
            const float Mw = __uint_as_float(mb);
            const float S = sqrt_cr(Mw);
            // lo = the smallest float whose correctly rounded sqrt is S: the first float above
            // the square of the midpoint between S and its lower neighbour (exact in double;
            // a float's sqrt is never exactly a midpoint)
            float lo = 0.f;
            if (S > 0.f) {
                const double mid = 0.5 * ((double)S + (double)__uint_as_float(__float_as_uint(S) - 1u));
                const double m2 = mid * mid;
                float f = (float)m2;
                if ((double)f <= m2) f = __uint_as_float(__float_as_uint(f) + 1u);
                lo = f;
            }
            unsigned cand = 0xFFFFFFFFu;
#pragma unroll
            for (int j = PPT - 1; j >= 0; --j)
                cand = best[j] >= __float_as_uint(lo) ? (unsigned)(j * BLOCK + t) : cand;
            FPS_STAMP(3);
            const unsigned widx = wave_umin(cand);
            FPS_STAMP(4);
            if (lane == 0) s_key[buf][w] = make_uint2(__float_as_uint(S) + 1u, widx);
        } else if (lane == 0) {
            s_key[buf][w] = make_uint2(0u, 0xFFFFFFFFu);
        }
        FPS_STAMP(5);
        __syncthreads();
        FPS_STAMP(6);
        const uint2 k2 = lane < NW ? s_key[buf][lane] : make_uint2(0u, 0xFFFFFFFFu);
        const unsigned bs = wave_umax(k2.x);
        far = (int)wave_umin(k2.x == bs ? k2.y : 0xFFFFFFFFu);
        if (lds_cloud) {
            cx = s_cloud[3 * far + 0];
            cy = s_cloud[3 * far + 1];
            cz = s_cloud[3 * far + 2];
        } else {
            cx = P[3 * far + 0];
            cy = P[3 * far + 1];
            cz = P[3 * far + 2];
        }
#ifdef PCS_FPS_STAMPS
        asm volatile("" ::"v"(cx), "v"(cy), "v"(cz));
        FPS_STAMP(7);
#endif
    }
#ifdef PCS_FPS_STAMPS
    if (blockIdx.x == 0 && t == 0)
        for (int k = 0; k < 8; ++k) g_fps_stamps[k] = st_acc[k];
#endif
    if (lds_out) {
        __syncthreads();
        for (int i = t; i < C; i += BLOCK) {
            const float4 q = s_out[i];
            out_idx[(size_t)b * C + i] = __float_as_int(q.w);
            float* o = out_xyz + ((size_t)b * C + i) * 3;
            o[0] = q.x;
            o[1] = q.y;
            o[2] = q.z;
        }
    }
}

template <int BLOCK, int PPT>
static void launch_fps(const float* xyz, int B, int N, int C, const int* start, int* out_idx, float* out_xyz,
                       hipStream_t s) {
    hipLaunchKernelGGL((fps_kernel<BLOCK, PPT>), dim3(B), dim3(BLOCK), 0, s, xyz, N, C, start, out_idx, out_xyz);
}

}  // namespace pcs

// Reference: models/utils/common.py:6-34 (`sample`).  Returns indices and the
// gathered centroid coordinates (the reference returns only the coordinates).
PCS_API int pcs_fps(const float* xyz, int B, int N, int C, const int32_t* start, int32_t* out_idx,
                    float* out_xyz, void* stream) {
    using namespace pcs;
    PCS_CHECK_ARG(B >= 0 && N >= 1 && C >= 1, "pcs_fps: bad sizes B=%d N=%d C=%d", B, N, C);
    PCS_CHECK_ARG(xyz && start && out_idx && out_xyz, "pcs_fps: null pointer");
    if (B == 0) return 0;
    hipStream_t s = as_stream(stream);
    // threads per cloud by size (round-1 sweep)
    const int blk = N <= 256 ? 64 : (N <= 2048 ? 256 : (N <= 8192 ? 512 : 1024));
    const int ppt = (N + blk - 1) / blk;
    // algorithmic: C serial steps over N points per cloud (8 fp32 flops per distance + update);
    // the cloud read once, C (index, xyz) written.  A latency-bound chain: see DESIGN.md 3.1
    const double flops = 8.0 * B * (double)N * C, bytes = (double)B * (12.0 * N + 16.0 * C);
#define PCS_FPS_CASE(BL, PP)                                                                    \
    if (blk == BL && ppt <= PP) {                                                               \
        ProbeScope pr(s, flops, bytes, "pcs::fps_kernel<%d, %d>", BL, PP);                     \
        launch_fps<BL, PP>(xyz, B, N, C, start, out_idx, out_xyz, s);                           \
    } else
    PCS_FPS_CASE(64, 1) PCS_FPS_CASE(64, 2) PCS_FPS_CASE(64, 4) PCS_FPS_CASE(64, 8)
    PCS_FPS_CASE(256, 1) PCS_FPS_CASE(256, 2) PCS_FPS_CASE(256, 4) PCS_FPS_CASE(256, 8) PCS_FPS_CASE(256, 16)
    PCS_FPS_CASE(512, 2) PCS_FPS_CASE(512, 4) PCS_FPS_CASE(512, 8) PCS_FPS_CASE(512, 16)
    PCS_FPS_CASE(1024, 1) PCS_FPS_CASE(1024, 2) PCS_FPS_CASE(1024, 4) PCS_FPS_CASE(1024, 8)
    PCS_FPS_CASE(1024, 16) PCS_FPS_CASE(1024, 24) PCS_FPS_CASE(1024, 32)
    {
        set_error("pcs_fps: N=%d not supported with %d threads per cloud (max 32768 points)", N, blk);
        return (int)hipErrorInvalidValue;
    }
#undef PCS_FPS_CASE
    return launch_status("pcs_fps");
}

#ifdef PCS_FPS_STAMPS
PCS_API int pcs_debug_fps_stamps(unsigned long long* host_out) {
    return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(pcs::g_fps_stamps), sizeof(unsigned long long) * 8, 0,
                                    hipMemcpyDeviceToHost);
}
#endif
