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
// rows (quad xor1, quad xor2, half-row mirror, row mirror), then row_bcast:15 / row_bcast:31
// fold the four row results into lane 63, read with one v_readlane.  No LDS round trips.
template <int CTRL, int ROWS>
__device__ __forceinline__ unsigned dpp_old(unsigned old, unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWS, 0xF, false);
}
__device__ __forceinline__ unsigned wave_umax(unsigned v) {
    v = max(v, dpp_u<0xB1>(v));
    v = max(v, dpp_u<0x4E>(v));
    v = max(v, dpp_u<0x141>(v));
    v = max(v, dpp_u<0x140>(v));
    v = max(v, dpp_old<0x142, 0xA>(0u, v));       // row_bcast:15 -> rows 1, 3
    v = max(v, dpp_old<0x143, 0xC>(0u, v));       // row_bcast:31 -> rows 2, 3
    return readlane_u(v, 63);
}
__device__ __forceinline__ unsigned wave_umin(unsigned v) {
    v = min(v, dpp_old<0xB1, 0xF>(~0u, v));
    v = min(v, dpp_old<0x4E, 0xF>(~0u, v));
    v = min(v, dpp_old<0x141, 0xF>(~0u, v));
    v = min(v, dpp_old<0x140, 0xF>(~0u, v));
    v = min(v, dpp_old<0x142, 0xA>(~0u, v));
    v = min(v, dpp_old<0x143, 0xC>(~0u, v));
    return readlane_u(v, 63);
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
// Width (in float bit steps) of the near-tie window below a maximum.  Every float whose
// correctly rounded sqrt equals sqrt_cr(M) lies within 6 bit steps below M (a sqrt bucket
// spans at most 4 ulps of its binade, twice that in the binade below), so the window is a
// superset of the reference's tie class; 16 leaves margin.
constexpr unsigned kFpsWin = 16u;

// Per step (one loop iteration):
//  1. each thread folds the new distances into its squared running minima (float bits) and
//     takes its local max;
//  2. wave max mw (DPP chain), then the lowest index whose value lies in the window
//     [mw - kFpsWin, mw] together with a flag "its value is not mw" -- one key (idx<<1 | flag),
//     one wave-min chain; lane 0 publishes (mw + 1, key) in one 8-B LDS slot (per-slot ballots
//     with scalar selects instead measured 21 % slower, round 4: the CU's one scalar unit is
//     shared by the 8 waves);
//  3. after the barrier, lanes 0..NW-1 hold the slots: the block max M*, and the FAST PATH holds
//     when every slot in M*'s window has exactly M* and a clear flag.  Then no point other than
//     those with value M* lies in the window, all points of the reference's tie class (same
//     sqrt_cr as M*) have value exactly M*, and the winner -- the reference's first index of the
//     max sqrt distance -- is the lowest published index among the M* slots (one short DPP
//     chain over NW lanes).  No sqrt and no double arithmetic on that path.
//  4. otherwise (a near-tie somewhere in the window: rare) every wave recomputes its exact key
//     -- (sqrt_cr(mw), lowest index with a value whose sqrt_cr is that) -- and the block takes the
//     (max sqrt, min index) slot after a second barrier.  All waves see the same slots, so all
//     take the same path.
// The winner's coordinates come from the LDS copy of the cloud (SoA, ds_read) when it fits.
template <int NW>
__device__ __forceinline__ unsigned slot_umax(unsigned v) {
    // lanes 0..NW-1 (NW = 4, 8 or 16) end with the max over them
    v = max(v, dpp_u<0xB1>(v));
    v = max(v, dpp_u<0x4E>(v));
    if constexpr (NW >= 8) v = max(v, dpp_u<0x141>(v));
    if constexpr (NW >= 16) v = max(v, dpp_u<0x140>(v));
    return readlane_u(v, 0);
}
template <int NW>
__device__ __forceinline__ unsigned slot_umin(unsigned v) {
    v = min(v, dpp_u<0xB1>(v));
    v = min(v, dpp_u<0x4E>(v));
    if constexpr (NW >= 8) v = min(v, dpp_u<0x141>(v));
    if constexpr (NW >= 16) v = min(v, dpp_u<0x140>(v));
    return readlane_u(v, 0);
}

// the smallest float whose correctly rounded sqrt is S (S > 0): the first float above the exact
// (double) square of the midpoint between S and its lower neighbour (a float's sqrt is never
// exactly a midpoint)
__device__ __forceinline__ unsigned sqrt_class_lo(float S) {
    if (!(S > 0.f)) return 0u;
    const double mid = 0.5 * ((double)S + (double)__uint_as_float(__float_as_uint(S) - 1u));
    const double m2 = mid * mid;
    float f = (float)m2;
    if ((double)f <= m2) f = __uint_as_float(__float_as_uint(f) + 1u);
    return __float_as_uint(f);
}

template <int BLOCK, int PPT, bool LDSC>
__global__ __launch_bounds__(BLOCK) void fps_kernel(const float* __restrict__ xyz, int N, int C,
                                                    const int* __restrict__ start, int* __restrict__ out_idx,
                                                    float* __restrict__ out_xyz) {
    constexpr int NW = BLOCK / kWave;
    static_assert(NW == 1 || NW == 4 || NW == 8 || NW == 16, "slot reduction width");
    __shared__ __attribute__((aligned(16))) uint2 s_slot[2][NW];   // (mw + 1, idx<<1 | flag); 0 = empty wave
    __shared__ __attribute__((aligned(16))) uint2 s_key[NW];       // slow path: (sqrt bits + 1, index)
    // Per-step global stores would make every __syncthreads wait for them (the
    // barrier's fence drains vmcnt): keep the picked centroids in LDS instead.  Dynamic LDS,
    // sized to THIS call (fps_lds_bytes): [C centroids | x | y | z of the N points] -- the
    // prefetched SA1 FPS holds its CU's LDS for the whole backward it runs under, so a
    // worst-case static size (128 KB) starved the main stream's GEMMs on those 32 CUs
    extern __shared__ float4 fps_lds[];
    const bool lds_out = C <= kFpsLdsOut;
    float4* s_out = fps_lds;
    float* s_px = reinterpret_cast<float*>(fps_lds + (lds_out ? C : 0));
    float* s_py = s_px + N;
    float* s_pz = s_py + N;

    const int b = blockIdx.x;
    const int t = threadIdx.x;
    const int w = t >> 6, lane = t & 63;
    const float* P = xyz + (size_t)b * N * 3;

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
            if constexpr (LDSC) {
                s_px[p] = px[j];
                s_py[p] = py[j];
                s_pz[p] = pz[j];
            }
        } else {
            px[j] = py[j] = pz[j] = 0.f;
            best[j] = 0u;
        }
    }

    int far = start[b];
    far = far < 0 ? 0 : (far >= N ? N - 1 : far);
    float cx = P[3 * far + 0], cy = P[3 * far + 1], cz = P[3 * far + 2];
    if constexpr (LDSC) __syncthreads();

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
        } else {
#pragma unroll
            for (int j = 0; j < PPT; ++j) {
                const float dx = px[j] - cx, dy = py[j] - cy, dz = pz[j] - cz;
                const float d = __fmaf_rn(dz, dz, __fmaf_rn(dy, dy, __fmul_rn(dx, dx)));
                best[j] = min(__float_as_uint(d), best[j]);   // == (d < best ? d : best)
                M = max(M, best[j]);
            }
        }
        FPS_STAMP(1);
        // M + 1 never wraps (M <= +inf bits); 0 marks a wave with only padding slots
        const unsigned wk = wave_umax(M + 1u);
        const unsigned mw = wk - 1u;
        FPS_STAMP(2);
        // window [mw - kFpsWin, mw]; an all-padding wave (wk == 0) matches nothing (best <= +inf bits)
        const unsigned wlo = wk == 0u ? 0xFFFFFFFFu : (mw > kFpsWin ? mw - kFpsWin : 0u);
        unsigned ci = 0xFFFFFFFFu, cv = 0u;   // lowest window index of this thread and its value
#pragma unroll
        for (int j = PPT - 1; j >= 0; --j) {
            const bool in = best[j] >= wlo;
            ci = in ? (unsigned)(j * BLOCK + t) : ci;
            cv = in ? best[j] : cv;
        }
        // no candidate: 0xFFFFFFFE / 0xFFFFFFFF, above every real key
        const unsigned key = (ci << 1) | (cv != mw ? 1u : 0u);
        FPS_STAMP(3);
        const unsigned wkey = wave_umin(key);
        FPS_STAMP(4);
        const int buf = i & 1;
        if (lane == 0) s_slot[buf][w] = make_uint2(wk, wkey);
        FPS_STAMP(5);
        __syncthreads();
        FPS_STAMP(6);
        const uint2 sl = lane < NW ? s_slot[buf][lane] : make_uint2(0u, 0xFFFFFFFFu);
        const unsigned Ms = NW == 1 ? readlane_u(sl.x, 0) : slot_umax<NW>(sl.x);
        const unsigned slo = Ms > kFpsWin + 1u ? Ms - kFpsWin : 1u;
        const bool near = sl.x >= slo && (sl.x != Ms || (sl.y & 1u));
        const unsigned fk = NW == 1 ? readlane_u(sl.y, 0) : slot_umin<NW>(sl.x == Ms ? sl.y : 0xFFFFFFFFu);
        if (__builtin_expect(ballot(near) == 0ull, 1)) {
            far = (int)(fk >> 1);
        } else {
            // exact keys: the wave's max sqrt S and the lowest index whose value has that sqrt
            unsigned kx = 0u, ky = 0xFFFFFFFFu;
            if (wk != 0u) {
                const float S = sqrt_cr(__uint_as_float(mw));
                const unsigned lo = sqrt_class_lo(S);
                unsigned cand = 0xFFFFFFFFu;
#pragma unroll
                for (int j = PPT - 1; j >= 0; --j) cand = best[j] >= lo ? (unsigned)(j * BLOCK + t) : cand;
                kx = __float_as_uint(S) + 1u;
                ky = wave_umin(cand);
            }
            if (lane == 0) s_key[w] = make_uint2(kx, ky);
            __syncthreads();
            const uint2 k2 = lane < NW ? s_key[lane] : make_uint2(0u, 0xFFFFFFFFu);
            const unsigned bs = NW == 1 ? readlane_u(k2.x, 0) : slot_umax<NW>(k2.x);
            far = (int)(NW == 1 ? readlane_u(k2.y, 0) : slot_umin<NW>(k2.x == bs ? k2.y : 0xFFFFFFFFu));
        }
        if constexpr (LDSC) {
            cx = s_px[far];
            cy = s_py[far];
            cz = s_pz[far];
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

// ------------------------------------------------------------------ FPS with spatial culling
// The same selection as fps_kernel (squared running minima as float bits, the window / flag fast
// path, the exact sqrt slow path) with the points of a cloud REORDERED spatially: a counting sort
// by a 16 x 16 x 16 Morton-ordered cell grid over the cloud's box gives each thread PPT consecutive
// points of that order, i.e. a compact region, and its bounding box.  A step's new centroid can
// lower a point's minimum only if its distance is below that minimum, so a thread whose box lies
// farther from the centroid than its largest minimum skips the update (a wave whose threads all
// skip issues nothing): after the first few dozen steps most of the cloud is far from each new
// centroid.  The skip test keeps a 2^-18 relative margin over the box distance, which covers the
// fp32 rounding of both the box distance and the point distance, so a skipped point's minimum is
// exactly what the update would have left.  Ties and the window test use the points' ORIGINAL
// indices (looked up in the sorted-index table), so the pick -- the reference's first index of
// the largest sqrt distance -- does not depend on the storage order, and the in-cell order of the
// (atomic) counting sort does not matter.
constexpr int kCullCells = 4096;              // 16^3 Morton cells
constexpr float kCullMargin = 0.999996f;      // 1 - 2^-18
constexpr size_t kCullLdsMax = 160 * 1024 - 1024;   // dynamic LDS cap (the static slots take < 1 KB)

__device__ __forceinline__ unsigned morton16(unsigned x, unsigned y, unsigned z) {
    auto spread = [](unsigned v) {             // 4 bits -> every third bit
        v = (v | (v << 4)) & 0x0C3u;
        v = (v | (v << 2)) & 0x249u;
        return v;
    };
    return spread(x) | (spread(y) << 1) | (spread(z) << 2);
}

template <int BLOCK, int PPT, bool LDSC>
__global__ __launch_bounds__(BLOCK) void fps_cull_kernel(const float* __restrict__ xyz, int N, int C,
                                                         const int* __restrict__ start, int* __restrict__ out_idx,
                                                         float* __restrict__ out_xyz) {
    constexpr int NW = BLOCK / kWave;
    static_assert(NW == 4 || NW == 8 || NW == 16, "slot reduction width");
    __shared__ __attribute__((aligned(16))) uint2 s_slot[2][NW];
    __shared__ __attribute__((aligned(16))) uint2 s_key[NW];
    __shared__ float s_box[NW][6];
    // dynamic LDS: [C centroids (16 B) | sorted original index per position (u16, N) | cell counts
    // (kCullCells ints) | x | y | z of the N points (LDSC)]
    extern __shared__ float4 fps_lds[];
    const bool lds_out = C <= kFpsLdsOut;
    float4* s_out = fps_lds;
    unsigned short* s_ord = reinterpret_cast<unsigned short*>(fps_lds + (lds_out ? C : 0));
    int* s_cnt = reinterpret_cast<int*>(s_ord + ((N + 7) & ~7));
    float* s_px = reinterpret_cast<float*>(s_cnt + kCullCells);
    float* s_py = s_px + N;
    float* s_pz = s_py + N;

    const int b = blockIdx.x;
    const int t = threadIdx.x;
    const int w = t >> 6, lane = t & 63;
    const float* P = xyz + (size_t)b * N * 3;

    // ---- the cloud's box and the cell of every point (16 cells per axis over the box)
    float bx[6] = {__builtin_inff(), __builtin_inff(), __builtin_inff(), -__builtin_inff(), -__builtin_inff(),
                   -__builtin_inff()};
    for (int p = t; p < N; p += BLOCK) {
        const float x = P[3 * p], y = P[3 * p + 1], z = P[3 * p + 2];
        if (LDSC) { s_px[p] = x; s_py[p] = y; s_pz[p] = z; }
        bx[0] = fminf(bx[0], x); bx[1] = fminf(bx[1], y); bx[2] = fminf(bx[2], z);
        bx[3] = fmaxf(bx[3], x); bx[4] = fmaxf(bx[4], y); bx[5] = fmaxf(bx[5], z);
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1)
#pragma unroll
        for (int k = 0; k < 6; ++k) bx[k] = k < 3 ? fminf(bx[k], __shfl_xor(bx[k], m)) : fmaxf(bx[k], __shfl_xor(bx[k], m));
    if (lane == 0)
        for (int k = 0; k < 6; ++k) s_box[w][k] = bx[k];
    for (int c = t; c < kCullCells; c += BLOCK) s_cnt[c] = 0;
    __syncthreads();
    float lo[3], sc[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float a = s_box[0][k], e = s_box[0][k + 3];
        for (int v = 1; v < NW; ++v) { a = fminf(a, s_box[v][k]); e = fmaxf(e, s_box[v][k + 3]); }
        lo[k] = a;
        const float ext = e - a;
        sc[k] = ext > 0.f && ext < 3.0e38f ? 16.f / ext : 0.f;   // degenerate / non-finite: one cell
    }
    auto cell_of = [&](float x, float y, float z) {
        const float u[3] = {(x - lo[0]) * sc[0], (y - lo[1]) * sc[1], (z - lo[2]) * sc[2]};
        unsigned c[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) c[k] = u[k] >= 1.f ? (unsigned)fminf(u[k], 15.f) : 0u;
        return morton16(c[0], c[1], c[2]);
    };
    for (int p = t; p < N; p += BLOCK) atomicAdd(&s_cnt[cell_of(P[3 * p], P[3 * p + 1], P[3 * p + 2])], 1);
    __syncthreads();
    if (w == 0) {
        // exclusive scan of the 4096 counts by one wave: 64 runs of 64
        int sum = 0;
        for (int c = 64 * lane; c < 64 * lane + 64; ++c) sum += s_cnt[c];
        int inc = sum;
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) {
            const int o = __shfl_up(inc, m);
            inc += lane >= m ? o : 0;
        }
        int run = inc - sum;
        for (int c = 64 * lane; c < 64 * lane + 64; ++c) {
            const int n = s_cnt[c];
            s_cnt[c] = run;
            run += n;
        }
    }
    __syncthreads();
    for (int p = t; p < N; p += BLOCK)
        s_ord[atomicAdd(&s_cnt[cell_of(P[3 * p], P[3 * p + 1], P[3 * p + 2])], 1)] = (unsigned short)p;
    __syncthreads();

    // ---- this thread's PPT consecutive points of the spatial order, their box
    float px[PPT], py[PPT], pz[PPT];
    unsigned best[PPT];
    float tb[6] = {__builtin_inff(), __builtin_inff(), __builtin_inff(), -__builtin_inff(), -__builtin_inff(),
                   -__builtin_inff()};
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const int q = t * PPT + j;
        if (q < N) {
            const int p = s_ord[q];
            px[j] = LDSC ? s_px[p] : P[3 * p];
            py[j] = LDSC ? s_py[p] : P[3 * p + 1];
            pz[j] = LDSC ? s_pz[p] : P[3 * p + 2];
            best[j] = 0x7f800000u;
            tb[0] = fminf(tb[0], px[j]); tb[1] = fminf(tb[1], py[j]); tb[2] = fminf(tb[2], pz[j]);
            tb[3] = fmaxf(tb[3], px[j]); tb[4] = fmaxf(tb[4], py[j]); tb[5] = fmaxf(tb[5], pz[j]);
        } else {
            px[j] = py[j] = pz[j] = 0.f;
            best[j] = 0u;                      // padding: never above a real point, never a candidate
        }
    }
    // NaN coordinates make the box test fail (never skip) -- the update then runs as fps_kernel's
    unsigned Mt = 0x7f800000u;                // this thread's largest minimum (bits)

    int far = start[b];
    far = far < 0 ? 0 : (far >= N ? N - 1 : far);
    float cx = LDSC ? s_px[far] : P[3 * far], cy = LDSC ? s_py[far] : P[3 * far + 1],
          cz = LDSC ? s_pz[far] : P[3 * far + 2];
    const int q0 = t * PPT;

    for (int i = 0; i < C; ++i) {
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

        // ---- update (skipped when the box is provably farther than every minimum of the thread)
        const float ex = fmaxf(fmaxf(tb[0] - cx, cx - tb[3]), 0.f);
        const float ey = fmaxf(fmaxf(tb[1] - cy, cy - tb[4]), 0.f);
        const float ez = fmaxf(fmaxf(tb[2] - cz, cz - tb[5]), 0.f);
        const float d2b = (ex * ex + ey * ey + ez * ez) * kCullMargin;
        if (!(d2b > __uint_as_float(Mt))) {
            unsigned M = 0u;
            if constexpr (PPT % 2 == 0) {
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
            } else {
#pragma unroll
                for (int j = 0; j < PPT; ++j) {
                    const float dx = px[j] - cx, dy = py[j] - cy, dz = pz[j] - cz;
                    const float d = __fmaf_rn(dz, dz, __fmaf_rn(dy, dy, __fmul_rn(dx, dx)));
                    best[j] = min(__float_as_uint(d), best[j]);
                    M = max(M, best[j]);
                }
            }
            Mt = M;
        }
        const unsigned wk = wave_umax(q0 < N ? Mt + 1u : 0u);
        const unsigned mw = wk - 1u;
        const unsigned wlo = wk == 0u ? 0xFFFFFFFFu : (mw > kFpsWin ? mw - kFpsWin : 0u);
        // lowest ORIGINAL index of this thread whose value lies in the window, and that value
        unsigned ci = 0xFFFFFFFFu, cv = 0u;
        if (Mt >= wlo && q0 < N) {
#pragma unroll
            for (int j = 0; j < PPT; ++j) {
                if (best[j] >= wlo) {
                    const unsigned id = s_ord[q0 + j];
                    cv = id < ci ? best[j] : cv;
                    ci = id < ci ? id : ci;
                }
            }
        }
        const unsigned key = (ci << 1) | (cv != mw ? 1u : 0u);
        const unsigned wkey = wave_umin(key);
        const int buf = i & 1;
        if (lane == 0) s_slot[buf][w] = make_uint2(wk, wkey);
        __syncthreads();
        const uint2 sl = lane < NW ? s_slot[buf][lane] : make_uint2(0u, 0xFFFFFFFFu);
        const unsigned Ms = slot_umax<NW>(sl.x);
        const unsigned slo = Ms > kFpsWin + 1u ? Ms - kFpsWin : 1u;
        const bool near = sl.x >= slo && (sl.x != Ms || (sl.y & 1u));
        const unsigned fk = slot_umin<NW>(sl.x == Ms ? sl.y : 0xFFFFFFFFu);
        if (__builtin_expect(ballot(near) == 0ull, 1)) {
            far = (int)(fk >> 1);
        } else {
            unsigned kx = 0u, ky = 0xFFFFFFFFu;
            if (wk != 0u) {
                const float S = sqrt_cr(__uint_as_float(mw));
                const unsigned lo2 = sqrt_class_lo(S);
                unsigned cand = 0xFFFFFFFFu;
                if (Mt >= lo2 && q0 < N) {
#pragma unroll
                    for (int j = 0; j < PPT; ++j)
                        if (best[j] >= lo2) cand = min(cand, (unsigned)s_ord[q0 + j]);
                }
                kx = __float_as_uint(S) + 1u;
                ky = wave_umin(cand);
            }
            if (lane == 0) s_key[w] = make_uint2(kx, ky);
            __syncthreads();
            const uint2 k2 = lane < NW ? s_key[lane] : make_uint2(0u, 0xFFFFFFFFu);
            const unsigned bs = slot_umax<NW>(k2.x);
            far = (int)slot_umin<NW>(k2.x == bs ? k2.y : 0xFFFFFFFFu);
        }
        if constexpr (LDSC) {
            cx = s_px[far];
            cy = s_py[far];
            cz = s_pz[far];
        } else {
            cx = P[3 * far + 0];
            cy = P[3 * far + 1];
            cz = P[3 * far + 2];
        }
    }
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

static size_t fps_cull_lds_bytes(int N, int C, bool ldsc) {
    return (C <= kFpsLdsOut ? (size_t)C * 16 : 0) + (size_t)((N + 7) & ~7) * 2 + (size_t)kCullCells * 4 +
           (ldsc ? (size_t)N * 12 : 0);
}

template <int BLOCK, int PPT, bool LDSC>
static void launch_fps_cull(const float* xyz, int B, int N, int C, const int* start, int* out_idx, float* out_xyz,
                            hipStream_t s) {
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&fps_cull_kernel<BLOCK, PPT, LDSC>), hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)kCullLdsMax);
    (void)attr;
    hipLaunchKernelGGL((fps_cull_kernel<BLOCK, PPT, LDSC>), dim3(B), dim3(BLOCK), fps_cull_lds_bytes(N, C, LDSC), s,
                       xyz, N, C, start, out_idx, out_xyz);
}

// dynamic LDS of one FPS launch (fps_kernel's layout)
static size_t fps_lds_bytes(int N, int C) {
    return (C <= kFpsLdsOut ? (size_t)C * 16 : 0) + (N <= kFpsLdsCloud ? (size_t)N * 12 : 0);
}

template <int BLOCK, int PPT, bool LDSC>
static void launch_fps_lds(const float* xyz, int B, int N, int C, const int* start, int* out_idx, float* out_xyz,
                           hipStream_t s) {
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&fps_kernel<BLOCK, PPT, LDSC>), hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)(kFpsLdsOut * 16 + (LDSC ? kFpsLdsCloud * 12 : 0)));
    (void)attr;
    hipLaunchKernelGGL((fps_kernel<BLOCK, PPT, LDSC>), dim3(B), dim3(BLOCK), fps_lds_bytes(N, C), s, xyz, N, C, start,
                       out_idx, out_xyz);
}

// the culled kernel for clouds past the LDS copy (N > 8192; PointNeXt's 24 576: 1.91 -> 1.57 ms at
// B = 16, C = 1024); at 4 096 points its sort and box tests cost more than the culling saves
// (0.82 vs 0.69 ms at B = 32), so smaller clouds keep fps_kernel
constexpr int kCullMinPoints = kFpsLdsCloud + 1;

template <int BLOCK, int PPT>
static void launch_fps(const float* xyz, int B, int N, int C, const int* start, int* out_idx, float* out_xyz,
                       hipStream_t s) {
    if constexpr (BLOCK >= 256) {
        if (N >= kCullMinPoints && fps_cull_lds_bytes(N, C, N <= kFpsLdsCloud) <= kCullLdsMax) {
            if (N <= kFpsLdsCloud) launch_fps_cull<BLOCK, PPT, true>(xyz, B, N, C, start, out_idx, out_xyz, s);
            else launch_fps_cull<BLOCK, PPT, false>(xyz, B, N, C, start, out_idx, out_xyz, s);
            return;
        }
    }
    if (N <= kFpsLdsCloud) launch_fps_lds<BLOCK, PPT, true>(xyz, B, N, C, start, out_idx, out_xyz, s);
    else launch_fps_lds<BLOCK, PPT, false>(xyz, B, N, C, start, out_idx, out_xyz, s);
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
    // threads per cloud by size (round-1 sweep; round 3: 256 threads at 4096 points measured equal)
    const int blk = N <= 256 ? 64 : (N <= 2048 ? 256 : (N <= 8192 ? 512 : 1024));
    const int ppt = (N + blk - 1) / blk;
    // algorithmic: C serial steps over N points per cloud (8 fp32 flops per distance + update);
    // the cloud read once, C (index, xyz) written.  A latency-bound chain: see DESIGN.md 3.1
    const double flops = 8.0 * B * (double)N * C, bytes = (double)B * (12.0 * N + 16.0 * C);
#define PCS_FPS_CASE(BL, PP)                                                                    \
    if (blk == BL && ppt <= PP) {                                                               \
        ProbeScope pr(s, flops, bytes, "pcs::%s<%d, %d, %s>",                                    \
                      BL >= 256 && N >= kCullMinPoints && fps_cull_lds_bytes(N, C, N <= kFpsLdsCloud) <= \
                      kCullLdsMax ? "fps_cull_kernel" : "fps_kernel", BL, PP,                    \
                      N <= kFpsLdsCloud ? "true" : "false");                                    \
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
