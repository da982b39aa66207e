// DGCNN dynamic-graph kNN (reference `knn`, models/dgcnn/dgcnn.py:7-21):
//   pd[i,j] = -|x_i|^2 - (-2 x_i.x_j) - |x_j|^2 ,  idx = topk(pd, k, largest)
//
// The reference evaluates x^T x with an MKL GEMM, so its rounding (and thus
// near-tie neighbour choices, ~0.05 % of rows) is not reproducible on any other
// device; parity for DGCNN uses neighbour-index replay and this
// kernel is checked by set agreement + distance-margin tests.
//
// knn_wave_kernel (k <= 20): each wave owns 32 query rows and streams the cloud in 32-point
// candidate tiles straight into its MFMA operands.  It computes its 32 x 32 block of inner
// products with v_mfma_f32_32x32x2_f32 (the k-slice of lane half h is features
// h*F/2 .. h*F/2+F/2-1, so every lane reads one contiguous run; F = 3 is padded to
// (x, y, z, 0)), then filters it against each row's running threshold (the current k-th
// best) into per-lane LDS survivor segments (about k ln(N/k) survivors per row).  A row
// whose segments fill is merged by a ballot quickselect (no sort); the final merge ranks
// the survivors (larger pd first, ties to the lower index).  The scan starts at the wave's
// own tile, so spatially ordered clouds tighten the thresholds early.
// Seeded threshold (pcs_knn_seeded): DGCNN's graphs 2-4 are built on features of the previous
// EdgeConv, whose neighbour lists are mostly still near in the new space (15-17 of 20 shared
// on the synthetic blocks).  The k-th best distance among any k candidates is a lower bound of
// the row's true k-th best, so each row starts its scan with the threshold of its previous
// neighbours (minus a rounding margin): about 30-45 survivors per row instead of ~180, and
// the running merges almost vanish.  The lists are the same as unseeded: every true top-k
// candidate still passes the (lower) threshold.
// knn_kernel (k = 40): one thread per query row with a sorted register list.
#include "pcs_common.hpp"
#include <algorithm>

namespace pcs {

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int F, int K>
__global__ __launch_bounds__(256) void knn_kernel(const float* __restrict__ x, int N, int* __restrict__ out_idx) {
    constexpr int T = 64;
    __shared__ __attribute__((aligned(16))) float s_x[T * F];
    __shared__ float s_xx[T];
    const int b = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const float* X = x + (size_t)b * N * F;
    float q[F];
    float xxi = 0.f;
    if (i < N) {
#pragma unroll
        for (int f = 0; f < F; ++f) q[f] = X[(size_t)i * F + f];
    } else {
#pragma unroll
        for (int f = 0; f < F; ++f) q[f] = 0.f;
    }
#pragma unroll
    for (int f = 0; f < F; ++f) xxi = __fadd_rn(xxi, __fmul_rn(q[f], q[f]));
    float L[K];
    int I[K];
#pragma unroll
    for (int s = 0; s < K; ++s) { L[s] = -__int_as_float(0x7f800000); I[s] = 0; }

    for (int base = 0; base < N; base += T) {
        __syncthreads();
        const int nt = (N - base) < T ? (N - base) : T;
        for (int t = threadIdx.x; t < nt * F; t += blockDim.x) s_x[t] = X[(size_t)base * F + t];
        __syncthreads();
        if (threadIdx.x < nt) {
            float xx = 0.f;
            for (int f = 0; f < F; ++f) {
                const float v = s_x[threadIdx.x * F + f];
                xx = __fadd_rn(xx, __fmul_rn(v, v));
            }
            s_xx[threadIdx.x] = xx;
        }
        __syncthreads();
        auto insert = [&](float dot, int j) {
            const float inner = -2.f * dot;
            const float pd = __fsub_rn(__fsub_rn(-xxi, inner), s_xx[j]);
            if (pd > L[K - 1]) {
                float cv = pd;
                int ci = base + j;
#pragma unroll
                for (int s = 0; s < K; ++s) {
                    const bool sw = cv > L[s];
                    const float tv = sw ? L[s] : cv;
                    const int ti = sw ? I[s] : ci;
                    L[s] = sw ? cv : L[s];
                    I[s] = sw ? ci : I[s];
                    cv = tv;
                    ci = ti;
                }
            }
        };
        int jj = 0;
        if (F % 4 == 0) {
            // 2 candidates per packed-FMA chain (v_pk_fma_f32): twice the fp32 rate of the
            // scalar chain; each candidate's dot is still the same sequential fma over f
            for (; jj + 2 <= nt; jj += 2) {
                f32x2 d = {0.f, 0.f};
#pragma unroll
                for (int f = 0; f < F; f += 4) {
                    const float4 x0 = *reinterpret_cast<const float4*>(&s_x[(jj + 0) * F + f]);
                    const float4 x1 = *reinterpret_cast<const float4*>(&s_x[(jj + 1) * F + f]);
                    d = __builtin_elementwise_fma(f32x2{q[f + 0], q[f + 0]}, f32x2{x0.x, x1.x}, d);
                    d = __builtin_elementwise_fma(f32x2{q[f + 1], q[f + 1]}, f32x2{x0.y, x1.y}, d);
                    d = __builtin_elementwise_fma(f32x2{q[f + 2], q[f + 2]}, f32x2{x0.z, x1.z}, d);
                    d = __builtin_elementwise_fma(f32x2{q[f + 3], q[f + 3]}, f32x2{x0.w, x1.w}, d);
                }
                insert(d.x, jj);
                insert(d.y, jj + 1);
            }
        }
        for (; jj < nt; ++jj) {
            float dot = 0.f;
#pragma unroll
            for (int f = 0; f < F; ++f) dot = __fmaf_rn(q[f], s_x[jj * F + f], dot);
            insert(dot, jj);
        }
    }
    if (i < N) {
        int* o = out_idx + ((size_t)b * N + i) * K;
#pragma unroll
        for (int s = 0; s < K; ++s) o[s] = I[s];
    }
}


// ----------------------------------------------------------------------------- tiled kNN
constexpr int KNN_TC = 32;      // candidates per tile
constexpr int KNN_WAVES = 4;
constexpr int KNN_QROWS = 32 * KNN_WAVES;
constexpr int KNN_NMAX = 64;    // LDS items per row: top-k list + one survivor segment per lane half (<= 64: one per lane in a merge)
// row stride in items: one item (2 banks) past the capacity.  At 64 items (512 B) every lane's
// survivor write of a tile hit the same bank pair (SQ_LDS_BANK_CONFLICT 3.3x the LDS-active
// cycles, round 4; the padding measured neutral on its own)
constexpr int KNN_RS = KNN_NMAX + 1;

// accumulator register i of lane half h holds candidate acc_row(i, h) of the tile
// (v_mfma_f32_32x32x2_f32 C/D layout: row = (i & 3) + 8 (i >> 2) + 4 h, column = lane & 31)
__device__ __forceinline__ constexpr int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }


// Merge row r of this wave (r uniform): its top-k list (nl items) and the two lane-half
// survivor segments (c0, c1 items) -- n <= 64 items, one per lane.  rank = number of items
// that beat it (larger pd; ties to the lower index); ranks < k are written back to the list
// in order (and to `out` if non-null).  Returns the new threshold: the k-th best value, or
// -inf while the row has fewer than k candidates.
template <int K, int SEG>
__device__ __forceinline__ float knn_merge_row(float2* L, int nl, int c0, int c1, int l, int* out) {
    const int n = nl + c0 + c1;
    const bool have = l < n;
    int src = l < nl ? l : (l < nl + c0 ? K + (l - nl) : K + SEG + (l - nl - c0));
    src = have ? src : 0;
    const float2 it = L[src];
    const float v = have ? it.x : -INFINITY;
    const int id = have ? __float_as_int(it.y) : 0x7fffffff;
    int rank = 0;
    for (int j = 0; j < n; ++j) {
        const float vj = readlane_f(v, j);
        const int ij = (int)readlane_u((unsigned)id, j);
        rank += (vj > v || (vj == v && ij < id)) ? 1 : 0;
    }
    if (have && rank < K) {
        L[rank] = make_float2(v, __int_as_float(id));
        if (out) out[rank] = id;
    }
    if (n < K) return -INFINITY;
    return readlane_f(v, ffs64(ballot(have && rank == K - 1)));
}


// order-preserving uint key of a float (-0 folded into +0, so key ties == float ties)
__device__ __forceinline__ unsigned knn_key(float v) {
    const unsigned u = __float_as_uint(v + 0.f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float knn_unkey(unsigned k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// popcount of a ballot mask as two 32-bit SALU counts: a 64-bit ctpop is compared on the
// VALU (v_cmp_gt_u64 -> one more VALU->SALU hop per search step, ~5 % of the kernel)
__device__ __forceinline__ int knn_popc(unsigned long long m) {
    return __builtin_popcount((unsigned)m) + __builtin_popcount((unsigned)(m >> 32));
}

// Running merge of row r (r uniform): keep the k best of its list and both survivor
// segments (n <= 64 items, one per lane) WITHOUT sorting them: the k-th best key T is
// found by a ballot quickselect (pivot = a lane's key, counts of keys above / at it by
// ballot + SALU popcount; ~log n rounds instead of the 32 steps of a bitwise search, and a
// radix-4 search measured slower still: its VALU->SALU hops serialise on VCC), items above
// T are kept, items equal to T by lowest index, and the kept ones are compacted into the
// list.  Returns the new threshold (-inf while fewer than k).
template <int K, int SEG>
__device__ __forceinline__ float knn_select_row(float2* L, int nl, int c0, int c1, int l) {
    const int n = nl + c0 + c1;
    const bool have = l < n;
    int src = l < nl ? l : (l < nl + c0 ? K + (l - nl) : K + SEG + (l - nl - c0));
    src = have ? src : 0;
    const float2 it = L[src];
    const unsigned long long hm = ballot(have);
    unsigned long long keep = hm;
    float tnew = -INFINITY;
    if (n > K) {
        const unsigned key = have ? knn_key(it.x) : 0u;
        unsigned T;
        // quickselect over the lanes: T is the rem-th largest key of `mask`; the pivot is
        // the mask's lowest lane (items sit in arrival order), each round drops the pivot
        unsigned long long mask = hm;
        int rem = K;
        while (true) {
            const unsigned pv = readlane_u(key, ffs64(mask));
            const unsigned long long gt = ballot(key > pv) & mask;
            const int cg = knn_popc(gt);
            if (cg >= rem) { mask = gt; continue; }
            const unsigned long long ge = ballot(key >= pv) & mask;
            const int ce = knn_popc(ge);
            if (ce >= rem) { T = pv; break; }
            rem -= ce;
            mask &= ~ge;
        }
        keep = ballot(key > T) & hm;
        unsigned long long eq = ballot(key == T) & hm;
        int need = K - knn_popc(keep);
        if (knn_popc(eq) == need) {
            keep |= eq;
        } else {               // ties on the k-th value: the lowest indices
            const int id = __float_as_int(it.y);
            for (; need > 0; --need) {
                int best = -1, bid = 0x7fffffff;
                for (unsigned long long r2 = eq; r2; r2 &= r2 - 1) {
                    const int ln = ffs64(r2);
                    const int il = (int)readlane_u((unsigned)id, ln);
                    if (il < bid) { bid = il; best = ln; }
                }
                keep |= 1ull << best;
                eq &= ~(1ull << best);
            }
        }
        tnew = knn_unkey(T);
    } else if (n == K) {
        unsigned mn = 0xffffffffu;
        const unsigned key = have ? knn_key(it.x) : 0xffffffffu;
        for (int j = 0; j < n; ++j) mn = min(mn, readlane_u(key, j));
        tnew = knn_unkey(mn);
    }
    if ((keep >> l) & 1ull) L[popc64(keep & lanemask_lt())] = it;
    return tnew;
}

// One workgroup = 4 independent waves x 32 query rows (row = lane & 31 of both lane halves).
// Every wave streams the candidate tiles straight from global memory (L2-resident: one cloud
// is N*F*4 bytes) into its MFMA operand registers, one tile ahead; no block barrier, so one
// wave's running merge overlaps the others' MFMA / filter work (round 2: -23 % at F = 3,
// -14 % at F = 64 against an LDS-staged tile ring with a barrier per tile, bitwise-equal
// neighbour lists; 2- and 1-wave blocks measured slower).  The MFMA computes the transposed
// block (candidates x queries), so each lane holds 16 candidates of ONE row: filtering is per
// lane, branch-free: every candidate is written to the lane's LDS segment at its fill count
// (a rejected one is overwritten by the next), and the count advances only for survivors.
// A full segment flags the survivor as dropped; after the wave merges the flagged rows the
// dropped survivors are re-appended.  Blocks of one cloud are mapped onto one XCD
// (blockIdx round-robins over the 8 XCDs), so each XCD's L2 holds the clouds it works on.
// xx_pre (PRE): the squared norm of every point, precomputed by knn_sqnorm_kernel with the
// same partial sums and the same final add as below, so the lists are bitwise the same; it
// removes F multiply-adds per lane and tile (the candidate side recomputed every norm in every
// wave that streams it)
// seeds (SEEDED, nullable): (B, N, ks) candidate lists whose k-th best bounds each row's
// threshold from the start (rows with out-of-range or repeated seeds, or ks < K, start at -inf)
template <int F, int K, int WPB, bool PRE, bool SEEDED>
__global__ __launch_bounds__(64 * WPB, 2) void knn_wave_kernel(const float* __restrict__ x, int B, int N, int rblocks,
                                                            int* __restrict__ out_idx,
                                                            const float* __restrict__ xx_pre,
                                                            const int* __restrict__ seeds, int ks) {
    constexpr bool MF = (F % 4 == 0);
    static_assert(MF || F == 3, "F must be 3 or a multiple of 4");
    constexpr int FH = MF ? F / 2 : 2;
    constexpr int NQ = MF ? FH / 4 : 1;      // float4 per lane per tile
    constexpr int SEG = (KNN_NMAX - K) / 2;
    constexpr int CAP = SEG - 1;
    static_assert(CAP >= 16, "a segment must take one tile's 16 candidates after a merge");
    __shared__ float s_cxx[WPB][KNN_TC];
    __shared__ float2 s_it[32 * WPB * KNN_RS];

    // XCD-aware block -> (cloud, row block): linear block L runs on XCD L % 8; give each XCD
    // whole clouds when the grid tiles evenly, else the plain row-major order
    const int L = blockIdx.x;
    const int total = B * rblocks;
    int b, rb;
    if (total % 8 == 0 && (total / 8) % rblocks == 0) {
        const int per = total / 8;                   // blocks per XCD (whole clouds)
        const int j = (L % 8) * per + L / 8;
        b = j / rblocks;
        rb = j - b * rblocks;
    } else {
        b = L / rblocks;
        rb = L - b * rblocks;
    }
    const int q0 = rb * 32 * WPB;
    const int tid = threadIdx.x;
    const int w = tid >> 6, l = tid & 63, h = l >> 5, l32 = l & 31;
    const float* X = x + (size_t)b * N * F;
    const int wrow0 = w * 32;
    const int qr = min(q0 + wrow0 + l32, N - 1);
    float2* const wl = s_it + wrow0 * KNN_RS;
    float2* const sg = wl + l32 * KNN_RS + K + h * SEG;

    float a[FH];
    float xxq;
    if constexpr (MF) {
        const float* xr = X + (size_t)qr * F + h * FH;
#pragma unroll
        for (int s = 0; s < FH; s += 4) {
            const float4 v = *reinterpret_cast<const float4*>(xr + s);
            a[s] = v.x; a[s + 1] = v.y; a[s + 2] = v.z; a[s + 3] = v.w;
        }
        float part = 0.f;
#pragma unroll
        for (int s = 0; s < FH; ++s) part = __fadd_rn(part, __fmul_rn(a[s], a[s]));
        const float other = __shfl_xor(part, 32);
        xxq = h ? __fadd_rn(other, part) : __fadd_rn(part, other);
    } else {
        const float* xr = X + (size_t)qr * 3;
        a[0] = h ? xr[2] : xr[0];
        a[1] = h ? 0.f : xr[1];
        const float part = __fadd_rn(__fmul_rn(a[0], a[0]), __fmul_rn(a[1], a[1]));
        const float other = __shfl_xor(part, 32);
        xxq = h ? __fadd_rn(other, part) : __fadd_rn(part, other);
    }
    if constexpr (PRE) xxq = xx_pre[(size_t)b * N + qr];
    float tau = -INFINITY;
    if constexpr (SEEDED) {
        static_assert(PRE, "seeded threshold: precomputed norms");
        // the k-th best pd among the row's seeds (here: the minimum over k of them).  The scan's
        // pd comes from an MFMA dot in another summation order: the margin 2^-14 (|x_q|^2 + |x_s|^2)
        // covers that (|dot error| <= ~F u sum|x_q x_s| <= 64 u (|x_q|^2 + |x_s|^2) / 2)
        const int* sr = seeds + ((size_t)b * N + qr) * ks;
        float t0 = INFINITY;
        bool ok = ks >= K;
        int prev[K];
        const int nsd = ks < K ? 0 : K;
        for (int j = 0; j < nsd; ++j) {
            const int sj = sr[j];
            ok = ok && sj >= 0 && sj < N;
            const int sc = (sj >= 0 && sj < N) ? sj : 0;
#pragma unroll
            for (int u = 0; u < K; ++u) ok = ok && !(u < j && prev[u] == sc);
#pragma unroll
            for (int u = 0; u < K; ++u) prev[u] = u == j ? sc : prev[u];
            float part = 0.f;
            if constexpr (MF) {
                const float4* src = reinterpret_cast<const float4*>(X + (size_t)sc * F + h * FH);
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const float4 v = src[q];
                    part = __fmaf_rn(a[4 * q], v.x, part);
                    part = __fmaf_rn(a[4 * q + 1], v.y, part);
                    part = __fmaf_rn(a[4 * q + 2], v.z, part);
                    part = __fmaf_rn(a[4 * q + 3], v.w, part);
                }
            } else {            // F = 3: lane half 0 holds (x, y), half 1 (z, 0), as the query's a[]
                const float* sp = X + (size_t)sc * 3;
                part = __fmaf_rn(a[1], h ? 0.f : sp[1], __fmul_rn(a[0], h ? sp[2] : sp[0]));
            }
            const float dot = __fadd_rn(part, __shfl_xor(part, 32));
            const float cx = xx_pre[(size_t)b * N + sc];
            const float pd = __fsub_rn(__fsub_rn(-xxq, -2.f * dot), cx);
            t0 = fminf(t0, __fsub_rn(pd, ldexpf(__fadd_rn(xxq, cx), -14)));
        }
        tau = ok ? t0 : -INFINITY;
    }
    int cnt = 0, nl = 0;

    const int ntile = (N + KNN_TC - 1) / KNN_TC;
    const int t0 = (q0 + wrow0) / KNN_TC;                 // start at the wave's own rows
    auto tile_c0 = [&](int tt) {
        const int t = t0 + tt;
        return (t >= ntile ? t - ntile : t) * KNN_TC;
    };
    // this lane's candidate (l32) of tile tt: features h*FH .. (F = 3: (x, y) | (z, 0))
    float4 cur[NQ], nxt[NQ];
    float cxx_cur = 0.f, cxx_nxt = 0.f;          // PRE: this lane's candidate's squared norm
    auto fetch = [&](int tt, float4* dst, float& cxx) __attribute__((always_inline)) {
        const int c0 = tile_c0(tt);
        const int n = c0 + min(l32, N - c0 - 1);
        if constexpr (PRE) cxx = xx_pre[(size_t)b * N + n];
        if constexpr (MF) {
            const float4* src = reinterpret_cast<const float4*>(X + (size_t)n * F + h * FH);
#pragma unroll
            for (int q = 0; q < NQ; ++q) dst[q] = src[q];
        } else {
            const float* xr = X + (size_t)n * 3;
            dst[0] = h ? make_float4(xr[2], 0.f, 0.f, 0.f) : make_float4(xr[0], xr[1], 0.f, 0.f);
        }
    };
    fetch(0, cur, cxx_cur);
    // the first tile lands BEFORE the loop (a use of every loaded register here): with its loads
    // still pending at the loop header, hipcc's wait insertion merged that state into the loop
    // body and waited (vmcnt(1) before the MFMAs, vmcnt(0) in the filter) on every iteration for
    // the NEXT tile's prefetch.  (Measured neutral, round 4: the L2-resident tile lands under the
    // other wave's work anyway; kept so the prefetch is what the source says.)
#pragma unroll
    for (int q = 0; q < NQ; ++q) asm volatile("" ::"v"(cur[q].x), "v"(cur[q].y), "v"(cur[q].z), "v"(cur[q].w));
    asm volatile("" ::"v"(cxx_cur));
    for (int tt = 0; tt < ntile; ++tt) {
        const int c0 = tile_c0(tt);
        const int nc = min(KNN_TC, N - c0);
        if (tt + 1 < ntile) fetch(tt + 1, nxt, cxx_nxt);
        float pd[16];
        {
            typedef float f32x16 __attribute__((ext_vector_type(16)));
            f32x16 acc = {};
            float part = 0.f;
            if constexpr (!MF) {
                const float vx = cur[0].x, vy = cur[0].y;
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx, a[0], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vy, a[1], acc, 0, 0, 0);
                if constexpr (!PRE) part = __fadd_rn(__fmul_rn(vx, vx), __fmul_rn(vy, vy));
            } else {
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const float4 v = cur[q];
                    const int s = 4 * q;
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v.x, a[s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v.y, a[s + 1], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v.z, a[s + 2], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v.w, a[s + 3], acc, 0, 0, 0);
                    if constexpr (!PRE) {
                        part = __fadd_rn(part, __fmul_rn(v.x, v.x));
                        part = __fadd_rn(part, __fmul_rn(v.y, v.y));
                        part = __fadd_rn(part, __fmul_rn(v.z, v.z));
                        part = __fadd_rn(part, __fmul_rn(v.w, v.w));
                    }
                }
            }
            if constexpr (PRE) {
                if (h == 0) s_cxx[w][l32] = cxx_cur;
            } else {
                const float other = __shfl_xor(part, 32);
                if (h == 0) s_cxx[w][l32] = __fadd_rn(part, other);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float inner = -2.f * acc[i];
                pd[i] = __fsub_rn(__fsub_rn(-xxq, inner), s_cxx[w][acc_row(i, h)]);
            }
        }
        // survivors of this tile (one bit per candidate slot); when no lane's segment can fill
        // (the common case) they are appended without the overflow bookkeeping -- the same
        // writes and counts as the general loop below, which handles a filling segment
        unsigned pm = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) pm |= (acc_row(i, h) < nc && pd[i] >= tau) ? (1u << i) : 0u;
        unsigned dropped = 0;
        if (!ballot(cnt + __builtin_popcount(pm) > CAP)) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                sg[cnt] = make_float2(pd[i], __int_as_float(c0 + acc_row(i, h)));
                cnt += (pm >> i) & 1u;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const bool p = (pm >> i) & 1u;
                sg[min(cnt, CAP)] = make_float2(pd[i], __int_as_float(c0 + acc_row(i, h)));
                dropped |= (p && cnt >= CAP) ? (1u << i) : 0u;
                cnt += (p && cnt < CAP) ? 1 : 0;
            }
        }
        // merge only on overflow (merging at 6 free slots measured 6 % slower: more merges)
        const unsigned long long nm = ballot(dropped != 0 || cnt > CAP);
        if (nm) {
            unsigned rows = (unsigned)nm | (unsigned)(nm >> 32);
            while (rows) {
                const int r = __ffs(rows) - 1;
                rows &= rows - 1;
                const int c0n = (int)readlane_u((unsigned)cnt, r);
                const int c1n = (int)readlane_u((unsigned)cnt, r + 32);
                const int nlr = (int)readlane_u((unsigned)nl, r);
                const float nt = knn_select_row<K, SEG>(wl + r * KNN_RS, nlr, c0n, c1n, l);
                const bool mine = l32 == r;
                tau = mine ? nt : tau;
                cnt = mine ? 0 : cnt;
                nl = mine ? min(nlr + c0n + c1n, K) : nl;
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const bool p = ((dropped >> i) & 1u) && pd[i] >= tau;
                sg[min(cnt, CAP)] = make_float2(pd[i], __int_as_float(c0 + acc_row(i, h)));
                cnt += p ? 1 : 0;
            }
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) cur[q] = nxt[q];
        cxx_cur = cxx_nxt;
    }
    for (int r = 0; r < 32; ++r) {
        const int c0n = (int)readlane_u((unsigned)cnt, r);
        const int c1n = (int)readlane_u((unsigned)cnt, r + 32);
        const int nlr = (int)readlane_u((unsigned)nl, r);
        const int q = q0 + wrow0 + r;
        int* o = q < N ? out_idx + ((size_t)b * N + q) * K : nullptr;
        if (!o) continue;
        if (nlr + c0n + c1n > K) {
            knn_select_row<K, SEG>(wl + r * KNN_RS, nlr, c0n, c1n, l);
            knn_merge_row<K, SEG>(wl + r * KNN_RS, K, 0, 0, l, o);
            continue;
        }
        knn_merge_row<K, SEG>(wl + r * KNN_RS, nlr, c0n, c1n, l, o);
    }
}

// xx[b][n] = |x_n|^2 exactly as knn_wave_kernel forms it: two half-feature partial sums
// (sequential fp32 multiply-adds, un-fused) added once (F = 3: (x^2 + y^2) + z^2)
template <int F>
__global__ __launch_bounds__(256) void knn_sqnorm_kernel(const float* __restrict__ x, long long P,
                                                       float* __restrict__ xx) {
    const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
    if (p >= P) return;
    const float* r = x + (size_t)p * F;
    if constexpr (F % 4 == 0) {
        constexpr int FH = F / 2;
        float p0 = 0.f, p1 = 0.f;
#pragma unroll
        for (int s = 0; s < FH; ++s) p0 = __fadd_rn(p0, __fmul_rn(r[s], r[s]));
#pragma unroll
        for (int s = 0; s < FH; ++s) p1 = __fadd_rn(p1, __fmul_rn(r[FH + s], r[FH + s]));
        xx[p] = __fadd_rn(p0, p1);
    } else {
        const float p0 = __fadd_rn(__fmul_rn(r[0], r[0]), __fmul_rn(r[1], r[1]));
        const float p1 = __fadd_rn(__fmul_rn(r[2], r[2]), __fmul_rn(0.f, 0.f));
        xx[p] = __fadd_rn(p0, p1);
    }
}

// ----------------------------------------------------------------------------- pruned kNN
// The same lists as knn_wave_kernel from a fraction of its tiles.  pcs_knn_order sorts each
// cloud's points by the Morton code of their xyz; in that order 32 consecutive points form a
// compact tile in coordinate space, and -- DGCNN's EdgeConv features being functions of the local
// geometry -- mostly in feature space too.  knn_tiles_kernel summarises every tile in feature space
// (centroid, bounding radius, axis-aligned box, largest squared norm); knn_pruned_kernel gives each
// wave one tile of query rows, sorts the candidate tiles by a lower bound of the squared distance
// between the two tiles (sphere and box bounds), and scans them nearest first until a tile's bound
// exceeds the loosest row's threshold: every later tile is then provably worse than each row's
// current k-th best.  Skipping is exact: the bound is deflated for its own fp32 rounding and for
// the rounding of the scan's pd (2^-13 (|x_q|^2 + |x_c|^2) covers it, cf. the seeded margin), a
// skipped candidate's pd is strictly below the row's running threshold (so it could not even tie
// the final k-th), and the survivors that remain are ranked by the same (pd, original index) order.
// Any order is correct (a permutation of the cloud); a good one makes the scan short.
constexpr int KO_MAX = 8192;                 // points per cloud the LDS Morton sort takes
constexpr int KP_NT = KO_MAX / KNN_TC;       // candidate tiles per cloud of the pruned kernel

__host__ __device__ constexpr int knn_tile_stride(int F) { return ((3 * F + 2) + 3) & ~3; }

__device__ __forceinline__ void knn_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ unsigned knn_spread3(unsigned v) {
    v &= 1023u;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

// one cloud per block: 10-bit-per-axis Morton keys of the first three features over the cloud's
// bounding cube, bitonic-sorted in LDS as (key, index) pairs (ties: lower index first); P = the
// padded power of two.  Non-finite coordinates quantise to cell 0.
__global__ __launch_bounds__(1024) void knn_order_kernel(const float* __restrict__ x, int N, int F, int P,
                                                         int* __restrict__ order) {
    extern __shared__ unsigned long long s_key[];
    __shared__ float s_red[16][6];
    const int b = blockIdx.x, tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    const float* X = x + (size_t)b * N * F;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = tid; i < N; i += 1024) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float v = X[(size_t)i * F + a];
            if (fabsf(v) <= 3.4e38f) {
                lo[a] = fminf(lo[a], v);
                hi[a] = fmaxf(hi[a], v);
            }
        }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(lo[a], __shfl_xor(lo[a], m));
            hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], m));
        }
    }
    if (l == 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            s_red[w][a] = lo[a];
            s_red[w][3 + a] = hi[a];
        }
    }
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float mn = s_red[0][a], mx = s_red[0][3 + a];
        for (int j = 1; j < 16; ++j) {
            mn = fminf(mn, s_red[j][a]);
            mx = fmaxf(mx, s_red[j][3 + a]);
        }
        lo[a] = mn;
        hi[a] = mx;
    }
    const float ext = fmaxf(fmaxf(hi[0] - lo[0], hi[1] - lo[1]), hi[2] - lo[2]);
    const float scale = ext > 0.f && ext <= 3.4e38f ? 1023.f / ext : 0.f;
    for (int i = tid; i < P; i += 1024) {
        unsigned long long key = ~0ull;
        if (i < N) {
            unsigned m = 0;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                float t = (X[(size_t)i * F + a] - lo[a]) * scale;
                t = t == t ? fminf(fmaxf(t, 0.f), 1023.f) : 0.f;
                m |= knn_spread3((unsigned)t) << a;
            }
            key = ((unsigned long long)m << 32) | (unsigned)i;
        }
        s_key[i] = key;
    }
    __syncthreads();
    // bitonic network.  Thread t handles pairs i = t + 1024 m, so for j < 64 a wave only touches its
    // own 128-key blocks: stages between two such stages need no block barrier (a wave's LDS
    // accesses complete in order), only a wave-level fence; a barrier follows every stage whose
    // successor may be j >= 64 (j >= 64 itself, and j = 1, the last stage of a merge)
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < (P >> 1); i += 1024) {
                const int a = ((i & ~(j - 1)) << 1) | (i & (j - 1)), c = a + j;
                const unsigned long long u = s_key[a], v = s_key[c];
                if ((u > v) == ((a & k) == 0)) {
                    s_key[a] = v;
                    s_key[c] = u;
                }
            }
            if (j >= 64 || j == 1) __syncthreads();
            else knn_wave_sync();
        }
    }
    for (int i = tid; i < N; i += 1024) order[(size_t)b * N + i] = (int)(unsigned)(s_key[i] & 0xffffffffull);
}

__global__ __launch_bounds__(256) void knn_identity_order_kernel(long long P, int N, int* __restrict__ order) {
    const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
    if (p < P) order[p] = (int)(p % N);
}

// one wave per (tile, cloud): lane d < F owns feature d.  Per cloud, field-major (element [f][t] at
// f * nt + t, so a wave reading one field of 64 tiles reads 256 contiguous bytes): centroid rows
// [0, F), box low [F, 2F), box high [2F, 3F), radius (3F), largest |x|^2 (3F + 1); a cloud spans
// knn_tile_stride(F) * nt floats.  A tile with a non-finite feature gets a NaN radius (its bounds
// are never used to skip).
template <int F>
__global__ __launch_bounds__(64) void knn_tiles_kernel(const float* __restrict__ x, int N, const int* __restrict__ order,
                                                       const float* __restrict__ xx, float* __restrict__ tinfo) {
    static_assert(F <= 64, "one lane per feature");
    constexpr int TS = knn_tile_stride(F);
    __shared__ float s_t[KNN_TC][F + 1];           // the tile minus its centroid, point-major
    const int t = blockIdx.x, b = blockIdx.y, l = threadIdx.x;
    const int nt = (N + KNN_TC - 1) / KNN_TC;
    const int p0 = t * KNN_TC, np = min(KNN_TC, N - p0);
    const float* X = x + (size_t)b * N * F;
    const int* O = order + (size_t)b * N;
    // lane j < np holds point j's index; the feature loads then need no dependent index load
    const int myo = l < np ? min(max(O[p0 + l], 0), N - 1) : 0;
    float v[KNN_TC];
#pragma unroll
    for (int j = 0; j < KNN_TC; ++j) {
        const int oi = (int)readlane_u((unsigned)myo, j);
        v[j] = (j < np && l < F) ? X[(size_t)oi * F + l] : 0.f;
    }
    float lo = INFINITY, hi = -INFINITY, sum = 0.f;
    bool bad = false;
#pragma unroll
    for (int j = 0; j < KNN_TC; ++j) {
        if (j < np) {
            bad = bad || !(fabsf(v[j]) <= 3.4e38f);
            lo = fminf(lo, v[j]);
            hi = fmaxf(hi, v[j]);
            sum += v[j];
        }
    }
    const float cen = sum / (float)np;
    if (l < F) {
#pragma unroll
        for (int j = 0; j < KNN_TC; ++j) s_t[j][l] = v[j] - cen;
    }
    __syncthreads();
    float r2 = 0.f;                                  // lane j: point j's squared distance to the centroid
    if (l < np) {
#pragma unroll 8
        for (int d = 0; d < F; ++d) r2 = fmaf(s_t[l][d], s_t[l][d], r2);
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) r2 = fmaxf(r2, __shfl_xor(r2, m));
    float mxx = l < np ? xx[(size_t)b * N + myo] : 0.f;
    bad = bad || !(fabsf(mxx) <= 3.4e38f);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) mxx = fmaxf(mxx, __shfl_xor(mxx, m));
    bad = ballot(bad) != 0ull;
    float* rec = tinfo + (size_t)b * nt * TS + t;
    if (l < F) {
        rec[(size_t)l * nt] = cen;
        rec[(size_t)(F + l) * nt] = lo;
        rec[(size_t)(2 * F + l) * nt] = hi;
    }
    if (l == 0) {
        rec[(size_t)(3 * F) * nt] = bad ? NAN : sqrtf(r2) * (1.f + 0x1p-10f);
        rec[(size_t)(3 * F + 1) * nt] = mxx;
    }
}

// The tile-pair bound (knn_pairs_kernel): a lower bound of the squared feature distance between any
// row of query tile q and any candidate of tile c -- the larger of the sphere bound
// (|cen_q - cen_c| - r_q - r_c)^2 and the box-gap bound sum_d max(lo_q - hi_c, lo_c - hi_q, 0)^2,
// deflated by 2^-10 for its own fp32 rounding and by 2^-13 (max|x_q|^2 + max|x_c|^2) for the
// rounding of the pd the scan computes; -inf when unusable (NaN / overflow).

// The k-th largest of a row's values over one or two tiles: M = 16 or 32 per lane half (-inf for
// invalid slots).  Each half sorts its M (bitonic network, descending), takes the partner half's
// sorted M by shuffles, and k-th(A u B) = max over splits i of min(A[i-1], B[k-i-1]).  All
// indices compile-time.
template <int K, int M>
__device__ __forceinline__ float knn_tile_kth(const float (&pd)[M]) {
    static_assert(K <= 2 * M, "k-th of 2M");
    float v[M];
#pragma unroll
    for (int r = 0; r < M; ++r) v[r] = pd[r];
#pragma unroll
    for (int k = 2; k <= M; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < M; ++i) {
                const int p = i ^ j;
                if (p > i) {
                    const bool desc = (i & k) == 0;
                    const float x = v[i], y = v[p];
                    v[i] = desc ? fmaxf(x, y) : fminf(x, y);
                    v[p] = desc ? fminf(x, y) : fmaxf(x, y);
                }
            }
    float best = -INFINITY;
#pragma unroll
    for (int i = 0; i <= K; ++i) {
        const int j = K - i;                               // taken from the partner's list
        if (i > M || j > M) continue;
        const float av = i == 0 ? INFINITY : v[i - 1];
        const float bv = j == 0 ? INFINITY : __shfl_xor(v[j - 1], 32);
        best = fmaxf(best, fminf(av, bv));
    }
    return best;
}

// Per cloud and query tile: every candidate tile's bound (the tile-pair bound above), sorted
// ascending (ties by tile) -> the scan order of the pruned kernel, (B, nt, nt) tile ids and their
// bounds.  One block of 4 waves per (KP_PQ query tiles, cloud): thread t computes candidate tile t's
// bounds against all KP_PQ query tiles (its fields read once, coalesced, dimension-outer; the query
// tiles' fields are block-uniform), as (order-preserving bound bits, tile) 64-bit keys in LDS; then
// each wave bitonic-sorts KP_PQ / 4 rows of keys (one compare-exchange pair per lane and stage, wave
// fences only).
constexpr int KP_PQ = 8;
template <int F>
__global__ __launch_bounds__(256) void knn_pairs_kernel(const float* __restrict__ tinfo, int N, int* __restrict__ sorted_t,
                                                     float* __restrict__ sorted_lb) {
    constexpr int TS = knn_tile_stride(F);
    __shared__ unsigned long long s_k[KP_PQ][KP_NT];
    __shared__ __attribute__((aligned(16))) float s_q[3][F][KP_PQ];     // the query tiles' fields, row-minor
    const int b = blockIdx.y, tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    const int nt = (N + KNN_TC - 1) / KNN_TC;
    int P = 64;                                    // keys per row: nt padded to a power of two
    while (P < nt) P <<= 1;
    const int tq0 = blockIdx.x * KP_PQ;
    const float* TI = tinfo + (size_t)b * nt * TS;
    float* const sq = &s_q[0][0][0];
    for (int e = tid; e < 3 * F * KP_PQ; e += 256) {
        const int r = e % KP_PQ, fd = e / KP_PQ;                       // fd = field * F + d
        sq[e] = TI[fd * nt + min(tq0 + r, nt - 1)];
    }
    __syncthreads();
    for (int t = tid; t < P; t += 256) {
        if (t >= nt) {
#pragma unroll
            for (int r = 0; r < KP_PQ; ++r) s_k[r][t] = ~0ull;
            continue;
        }
        int tqr[KP_PQ];
#pragma unroll
        for (int r = 0; r < KP_PQ; ++r) tqr[r] = min(tq0 + r, nt - 1);
        float cd[KP_PQ], gap[KP_PQ];
#pragma unroll
        for (int r = 0; r < KP_PQ; ++r) cd[r] = gap[r] = 0.f;
#pragma unroll 4
        for (int d = 0; d < F; ++d) {
            const float ct = TI[d * nt + t], lt = TI[(F + d) * nt + t], ht = TI[(2 * F + d) * nt + t];
#pragma unroll
            for (int r = 0; r < KP_PQ; ++r) {
                const float cq = s_q[0][d][r], lq = s_q[1][d][r], hq = s_q[2][d][r];
                const float df = cq - ct;
                cd[r] = fmaf(df, df, cd[r]);
                const float g = fmaxf(fmaxf(lq - ht, lt - hq), 0.f);
                gap[r] = fmaf(g, g, gap[r]);
            }
        }
        const float rt = TI[3 * F * nt + t], mt = TI[(3 * F + 1) * nt + t];
#pragma unroll
        for (int r = 0; r < KP_PQ; ++r) {
            const float rs = TI[3 * F * nt + tqr[r]] + rt;
            float sph = fmaxf(sqrtf(cd[r]) * (1.f - 0x1p-10f) - rs, 0.f);
            sph *= sph;
            float lb = fmaxf(sph, gap[r]) * (1.f - 0x1p-10f) - 0x1p-13f * (TI[(3 * F + 1) * nt + tqr[r]] + mt);
            lb = (lb == lb && rs == rs && cd[r] == cd[r]) ? lb : -INFINITY;
            s_k[r][t] = ((unsigned long long)knn_key(lb) << 32) | (unsigned)t;     // ascending bound, then tile
        }
    }
    __syncthreads();
    for (int r = w; r < KP_PQ; r += 4) {
        const int tq = tq0 + r;
        if (tq >= nt) break;
        unsigned long long* K = s_k[r];
        for (int k = 2; k <= P; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = l; i < (P >> 1); i += 64) {
                    const int a = ((i & ~(j - 1)) << 1) | (i & (j - 1)), c = a + j;
                    const unsigned long long u = K[a], v = K[c];
                    if ((u > v) == ((a & k) == 0)) {
                        K[a] = v;
                        K[c] = u;
                    }
                }
                knn_wave_sync();
            }
        }
        const size_t row = ((size_t)b * nt + tq) * nt;
        for (int i = l; i < nt; i += 64) {
            const unsigned long long key = K[i];
            sorted_t[row + i] = (int)(unsigned)(key & 0xffffffffull);
            sorted_lb[row + i] = knn_unkey((unsigned)(key >> 32));
        }
    }
}

#ifdef PCS_KNN_DIAG
// diagnostic build: per wave (b, tile) 8 ints: tiles scanned, running merges, then the cycles of
// setup (seeds, bounds, sort), scan and final merge
__device__ int g_knn_diag[8 << 13];
#define KNN_STAMP(v) do { asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory"); } while (0)
#else
#define KNN_STAMP(v) do { (void)(v); } while (0)
#endif

// knn_wave_kernel's scan (PRE norms) over the candidate tiles of a Morton-ordered cloud, nearest
// first, stopping at the first tile whose bound exceeds every row's threshold.  Rows and
// candidates are addressed through `order`; survivors carry original indices.
template <int F, int K, int WPB, bool SEEDED>
__global__ __launch_bounds__(64 * WPB, 2) void knn_pruned_kernel(const float* __restrict__ x, int B, int N, int rblocks,
                                                              int* __restrict__ out_idx, const float* __restrict__ xx_pre,
                                                              const int* __restrict__ order,
                                                              const int* __restrict__ sorted_t,
                                                              const float* __restrict__ sorted_lb,
                                                              const int* __restrict__ seeds, int ks) {
    constexpr bool MF = (F % 4 == 0);
    static_assert(MF || F == 3, "F must be 3 or a multiple of 4");
    constexpr int FH = MF ? F / 2 : 2;
    constexpr int NQ = MF ? FH / 4 : 1;
    constexpr int SEG = (KNN_NMAX - K) / 2;
    constexpr int CAP = SEG - 1;
    static_assert(CAP >= 16, "a segment must take one tile's 16 candidates after a merge");
    __shared__ float2 s_cc[WPB][KNN_TC];          // (|x_c|^2, original index) of the tile in the MFMA
    __shared__ float2 s_it[32 * WPB * KNN_RS];
    __shared__ float s_lb[WPB][KP_NT];            // this wave's scan order (knn_pairs_kernel): bounds
    __shared__ int s_tl[WPB][KP_NT];              // and candidate tiles, ascending

    const int L = blockIdx.x;
    const int total = B * rblocks;
    int b, rb;
    if (total % 8 == 0 && (total / 8) % rblocks == 0) {
        const int per = total / 8;
        const int j = (L % 8) * per + L / 8;
        b = j / rblocks;
        rb = j - b * rblocks;
    } else {
        b = L / rblocks;
        rb = L - b * rblocks;
    }
    const int tid = threadIdx.x;
    const int w = tid >> 6, l = tid & 63, h = l >> 5, l32 = l & 31;
    const int tq = rb * WPB + w;                                  // this wave's query tile
    const int nt = (N + KNN_TC - 1) / KNN_TC;
    if (tq >= nt) return;                                         // (no barriers below)
    unsigned long long st0 = 0, st1 = 0, st2 = 0, st3 = 0, sta = 0, stb = 0;
    int merges = 0;
    KNN_STAMP(st0);
    const float* X = x + (size_t)b * N * F;
    const int* O = order + (size_t)b * N;
    const int pq = tq * KNN_TC + l32;
    // order entries are clamped into the cloud (memory safety; a non-permutation gives wrong lists)
    const int qi = min(max(O[min(pq, N - 1)], 0), N - 1);
    PCS_DCHECK(O[min(pq, N - 1)] == qi, "knn order entry %d outside the cloud (N %d)", O[min(pq, N - 1)], N);
    float2* const wl = s_it + (w * 32) * KNN_RS;
    float2* const sg = wl + l32 * KNN_RS + K + h * SEG;

    float a[FH];
    if constexpr (MF) {
        const float* xr = X + (size_t)qi * F + h * FH;
#pragma unroll
        for (int s = 0; s < FH; s += 4) {
            const float4 v = *reinterpret_cast<const float4*>(xr + s);
            a[s] = v.x; a[s + 1] = v.y; a[s + 2] = v.z; a[s + 3] = v.w;
        }
    } else {
        const float* xr = X + (size_t)qi * 3;
        a[0] = h ? xr[2] : xr[0];
        a[1] = h ? 0.f : xr[1];
    }
    const float xxq = xx_pre[(size_t)b * N + qi];
    float tau = -INFINITY;
    if constexpr (SEEDED) {
        const int* sr = seeds + ((size_t)b * N + qi) * ks;
        float t0 = INFINITY;
        bool ok = ks >= K;
        int prev[K];
        const int nsd = ks < K ? 0 : K;
        for (int j = 0; j < nsd; ++j) {
            const int sj = sr[j];
            ok = ok && sj >= 0 && sj < N;
            const int sc = (sj >= 0 && sj < N) ? sj : 0;
#pragma unroll
            for (int u = 0; u < K; ++u) ok = ok && !(u < j && prev[u] == sc);
#pragma unroll
            for (int u = 0; u < K; ++u) prev[u] = u == j ? sc : prev[u];
            float part = 0.f;
            if constexpr (MF) {
                const float4* src = reinterpret_cast<const float4*>(X + (size_t)sc * F + h * FH);
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const float4 v = src[q];
                    part = __fmaf_rn(a[4 * q], v.x, part);
                    part = __fmaf_rn(a[4 * q + 1], v.y, part);
                    part = __fmaf_rn(a[4 * q + 2], v.z, part);
                    part = __fmaf_rn(a[4 * q + 3], v.w, part);
                }
            } else {
                const float* sp = X + (size_t)sc * 3;
                part = __fmaf_rn(a[1], h ? 0.f : sp[1], __fmul_rn(a[0], h ? sp[2] : sp[0]));
            }
            const float dot = __fadd_rn(part, __shfl_xor(part, 32));
            const float cx = xx_pre[(size_t)b * N + sc];
            const float pd = __fsub_rn(__fsub_rn(-xxq, -2.f * dot), cx);
            t0 = fminf(t0, __fsub_rn(pd, ldexpf(__fadd_rn(xxq, cx), -14)));
        }
        tau = ok ? t0 : -INFINITY;
    }
    // the loosest row's threshold as a squared distance: -min over rows of tau (+inf while any
    // row has fewer than k candidates)
    auto loosest = [&]() {
        float m = tau;
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) m = fminf(m, __shfl_xor(m, s));
        return -m;
    };

    // this wave's scan order: the candidate tiles by ascending bound (knn_pairs_kernel)
    KNN_STAMP(sta);
    {
        const size_t row = ((size_t)b * nt + tq) * nt;
        for (int i = l; i < nt; i += 64) {
            s_tl[w][i] = sorted_t[row + i];
            s_lb[w][i] = sorted_lb[row + i];
        }
    }
    KNN_STAMP(stb);
    knn_wave_sync();

    int cnt = 0, nl = 0;
    float thr = loosest();
    float4 cur[NQ], nxt[NQ];
    int ci_cur = 0, ci_nxt = 0;                  // this lane's candidate (original index)
    float cxx_cur = 0.f, cxx_nxt = 0.f;
    auto fetch = [&](int t, float4* dst, int& ci, float& cxx) __attribute__((always_inline)) {
        const int c0 = t * KNN_TC;
        ci = min(max(O[c0 + min(l32, N - c0 - 1)], 0), N - 1);
        cxx = xx_pre[(size_t)b * N + ci];
        if constexpr (MF) {
            const float4* src = reinterpret_cast<const float4*>(X + (size_t)ci * F + h * FH);
#pragma unroll
            for (int q = 0; q < NQ; ++q) dst[q] = src[q];
        } else {
            const float* xr = X + (size_t)ci * 3;
            dst[0] = h ? make_float4(xr[2], 0.f, 0.f, 0.f) : make_float4(xr[0], xr[1], 0.f, 0.f);
        }
    };
    int tcur = s_tl[w][0];
    constexpr int KTILES = MF ? 1 : 2;
    float v2[16 * KTILES];                       // the first tiles' pd (threshold start)
    KNN_STAMP(st1);
    fetch(tcur, cur, ci_cur, cxx_cur);
    int scanned = 0;
    for (int i = 0; i < nt; ++i) {
        if (s_lb[w][i] > thr) break;             // sorted: every remaining tile is farther
        ++scanned;
        const int c0 = tcur * KNN_TC;
        const int nc = min(KNN_TC, N - c0);
        const int tnext = i + 1 < nt ? s_tl[w][i + 1] : tcur;
        if (i + 1 < nt) fetch(tnext, nxt, ci_nxt, cxx_nxt);
        float pd[16];
        {
            typedef float f32x16 __attribute__((ext_vector_type(16)));
            f32x16 acc = {};
            if constexpr (!MF) {
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[0].x, a[0], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[0].y, a[1], acc, 0, 0, 0);
            } else {
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const float4 v = cur[q];
                    const int s = 4 * q;
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v.x, a[s], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v.y, a[s + 1], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v.z, a[s + 2], acc, 0, 0, 0);
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v.w, a[s + 3], acc, 0, 0, 0);
                }
            }
            if (h == 0) s_cc[w][l32] = make_float2(cxx_cur, __int_as_float(ci_cur));
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float inner = -2.f * acc[r];
                pd[r] = __fsub_rn(__fsub_rn(-xxq, inner), s_cc[w][acc_row(r, h)].x);
            }
        }
        if (i < KTILES) {
            // the first (nearest) tile's k-th best pd of each row, then (F = 3) the first two tiles':
            // lower bounds of the row's final k-th best -- the same pd values the scan compares, so
            // no margin -- that start the threshold tight (no running merges to establish it).  F =
            // 64 stops at one tile: the second tile's 16 registers cost more than its tighter start
            // (637 vs 620 us seeded, graph 2)
            if (i == 0) {
#pragma unroll
                for (int r = 0; r < 16; ++r) v2[r] = (acc_row(r, h) < nc && pd[r] == pd[r]) ? pd[r] : -INFINITY;
                float v1[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) v1[r] = v2[r];
                tau = fmaxf(tau, knn_tile_kth<K, 16>(v1));
            } else if constexpr (KTILES == 2) {
#pragma unroll
                for (int r = 0; r < 16; ++r) v2[16 + r] = (acc_row(r, h) < nc && pd[r] == pd[r]) ? pd[r] : -INFINITY;
                tau = fmaxf(tau, knn_tile_kth<K, 16 * KTILES>(v2));
            }
            thr = loosest();
        }
        unsigned pm = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) pm |= (acc_row(r, h) < nc && pd[r] >= tau) ? (1u << r) : 0u;
        unsigned dropped = 0;
        if (!ballot(cnt + __builtin_popcount(pm) > CAP)) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                sg[cnt] = make_float2(pd[r], s_cc[w][acc_row(r, h)].y);
                cnt += (pm >> r) & 1u;
            }
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const bool p = (pm >> r) & 1u;
                sg[min(cnt, CAP)] = make_float2(pd[r], s_cc[w][acc_row(r, h)].y);
                dropped |= (p && cnt >= CAP) ? (1u << r) : 0u;
                cnt += (p && cnt < CAP) ? 1 : 0;
            }
        }
        const unsigned long long nm = ballot(dropped != 0 || cnt > CAP);
        if (nm) {
            unsigned rows = (unsigned)nm | (unsigned)(nm >> 32);
            while (rows) {
                const int r = __ffs(rows) - 1;
                rows &= rows - 1;
                const int c0n = (int)readlane_u((unsigned)cnt, r);
                const int c1n = (int)readlane_u((unsigned)cnt, r + 32);
                const int nlr = (int)readlane_u((unsigned)nl, r);
                const float ntau = knn_select_row<K, SEG>(wl + r * KNN_RS, nlr, c0n, c1n, l);
                ++merges;
                const bool mine = l32 == r;
                tau = mine ? ntau : tau;
                cnt = mine ? 0 : cnt;
                nl = mine ? min(nlr + c0n + c1n, K) : nl;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const bool p = ((dropped >> r) & 1u) && pd[r] >= tau;
                sg[min(cnt, CAP)] = make_float2(pd[r], s_cc[w][acc_row(r, h)].y);
                cnt += p ? 1 : 0;
            }
            thr = loosest();
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) cur[q] = nxt[q];
        ci_cur = ci_nxt;
        cxx_cur = cxx_nxt;
        tcur = tnext;
    }
    KNN_STAMP(st2);
    for (int r = 0; r < 32; ++r) {
        const int c0n = (int)readlane_u((unsigned)cnt, r);
        const int c1n = (int)readlane_u((unsigned)cnt, r + 32);
        const int nlr = (int)readlane_u((unsigned)nl, r);
        const int p = tq * KNN_TC + r;
        if (p >= N) continue;
        const int q = (int)readlane_u((unsigned)qi, r);
        int* o = out_idx + ((size_t)b * N + q) * K;
        if (nlr + c0n + c1n > K) {
            knn_select_row<K, SEG>(wl + r * KNN_RS, nlr, c0n, c1n, l);
            knn_merge_row<K, SEG>(wl + r * KNN_RS, K, 0, 0, l, o);
            continue;
        }
        knn_merge_row<K, SEG>(wl + r * KNN_RS, nlr, c0n, c1n, l, o);
    }
    KNN_STAMP(st3);
#ifdef PCS_KNN_DIAG
    if (l == 0) {
        int* dg = g_knn_diag + 8 * ((b * nt + tq) & ((1 << 13) - 1));
        dg[0] = scanned;
        dg[1] = merges;
        dg[2] = (int)(st1 - st0);
        dg[3] = (int)(st2 - st1);
        dg[4] = (int)(st3 - st2);
        dg[5] = (int)(sta - st0);
        dg[6] = (int)(stb - sta);
    }
#else
    (void)scanned;
    (void)merges;
    (void)sta;
    (void)stb;
#endif
}

template <int K>
constexpr bool knn_tiled() { return (KNN_NMAX - K) / 2 - 1 >= 16; }

template <int F, int K>
static void launch_knn(const float* x, int B, int N, int* out, float* xx, const int* seeds, int ks, hipStream_t s) {
    if constexpr (knn_tiled<K>()) {
        const int rb = (N + KNN_QROWS - 1) / KNN_QROWS;
        if (xx) {
            const long long P = (long long)B * N;
            hipLaunchKernelGGL((knn_sqnorm_kernel<F>), dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, x, P, xx);
            // algorithmic: the N x N inner-product tile per cloud (2F flops per pair, the
            // reference's bmm), x read + the k-lists written
            {
                if (seeds) {
                    ProbeScope pr(s, 2.0 * F * (double)N * N * B, 4.0 * (double)B * N * (F + K),
                                  "pcs::knn_wave_kernel<%d, %d, %d, true, seeded>", F, K, KNN_WAVES);
                    hipLaunchKernelGGL((knn_wave_kernel<F, K, KNN_WAVES, true, true>), dim3(rb * B),
                                       dim3(64 * KNN_WAVES), 0, s, x, B, N, rb, out, (const float*)xx, seeds, ks);
                    return;
                }
            }
            ProbeScope pr(s, 2.0 * F * (double)N * N * B, 4.0 * (double)B * N * (F + K), "pcs::knn_wave_kernel<%d, %d, %d, true>",
                          F, K, KNN_WAVES);
            hipLaunchKernelGGL((knn_wave_kernel<F, K, KNN_WAVES, true, false>), dim3(rb * B), dim3(64 * KNN_WAVES), 0, s,
                               x, B, N, rb, out, (const float*)xx, (const int*)nullptr, 0);
        } else {
            hipLaunchKernelGGL((knn_wave_kernel<F, K, KNN_WAVES, false, false>), dim3(rb * B), dim3(64 * KNN_WAVES), 0,
                               s, x, B, N, rb, out, (const float*)nullptr, (const int*)nullptr, 0);
        }
        return;
    }
    hipLaunchKernelGGL((knn_kernel<F, K>), dim3((N + 255) / 256, B), dim3(256), 0, s, x, N, out);
}

template <int F, int K>
static void launch_knn_pruned(const float* x, int B, int N, int* out, float* xx, const int* order, float* tinfo,
                              const int* seeds, int ks, hipStream_t s) {
    if constexpr (knn_tiled<K>()) {
        if (N <= KO_MAX) {
            const long long P = (long long)B * N;
            const int nt = (N + KNN_TC - 1) / KNN_TC;
            const int rb = (nt + KNN_WAVES - 1) / KNN_WAVES;
            hipLaunchKernelGGL((knn_sqnorm_kernel<F>), dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, x, P, xx);
            hipLaunchKernelGGL((knn_tiles_kernel<F>), dim3(nt, B), dim3(64), 0, s, x, N, order, (const float*)xx, tinfo);
            int* sorted_t = reinterpret_cast<int*>(tinfo + (size_t)B * nt * knn_tile_stride(F));
            float* sorted_lb = reinterpret_cast<float*>(sorted_t + (size_t)B * nt * nt);
            hipLaunchKernelGGL((knn_pairs_kernel<F>), dim3((nt + KP_PQ - 1) / KP_PQ, B), dim3(256), 0, s,
                               (const float*)tinfo, N, sorted_t, sorted_lb);
            ProbeScope pr(s, 2.0 * F * (double)N * N * B, 4.0 * (double)B * N * (F + K), "pcs::knn_pruned_kernel<%d, %d, %d, %s>",
                          F, K, KNN_WAVES, seeds ? "true" : "false");
            if (seeds)
                hipLaunchKernelGGL((knn_pruned_kernel<F, K, KNN_WAVES, true>), dim3(rb * B), dim3(64 * KNN_WAVES), 0, s, x, B,
                                   N, rb, out, (const float*)xx, order, (const int*)sorted_t, (const float*)sorted_lb,
                                   seeds, ks);
            else
                hipLaunchKernelGGL((knn_pruned_kernel<F, K, KNN_WAVES, false>), dim3(rb * B), dim3(64 * KNN_WAVES), 0, s, x,
                                   B, N, rb, out, (const float*)xx, order, (const int*)sorted_t, (const float*)sorted_lb,
                                   (const int*)nullptr, 0);
            return;
        }
    }
    launch_knn<F, K>(x, B, N, out, xx, seeds, ks, s);
}

template <int F>
static int dispatch_pruned(const float* x, int B, int N, int k, int* out, float* xx, const int* order, float* tinfo,
                           const int* seeds, int ks, hipStream_t s) {
    switch (k) {
        case 16: launch_knn_pruned<F, 16>(x, B, N, out, xx, order, tinfo, seeds, ks, s); return 0;
        case 20: launch_knn_pruned<F, 20>(x, B, N, out, xx, order, tinfo, seeds, ks, s); return 0;
        case 32: launch_knn<F, 32>(x, B, N, out, xx, seeds, ks, s); return 0;
        case 40: launch_knn<F, 40>(x, B, N, out, xx, seeds, ks, s); return 0;
        default:
            set_error("pcs_knn_pruned: k=%d not instantiated (16, 20, 32, 40)", k);
            return (int)hipErrorInvalidValue;
    }
}

template <int F>
static int dispatch_k(const float* x, int B, int N, int k, int* out, float* xx, const int* seeds, int ks,
                      hipStream_t s) {
    switch (k) {
        case 16: launch_knn<F, 16>(x, B, N, out, xx, seeds, ks, s); return 0;
        case 20: launch_knn<F, 20>(x, B, N, out, xx, seeds, ks, s); return 0;
        case 32: launch_knn<F, 32>(x, B, N, out, xx, seeds, ks, s); return 0;
        case 40: launch_knn<F, 40>(x, B, N, out, xx, seeds, ks, s); return 0;
        default:
            set_error("pcs_knn: k=%d not instantiated (16, 20, 32, 40)", k);
            return (int)hipErrorInvalidValue;
    }
}

}  // namespace pcs

static int knn_run(const float* x, int B, int N, int F, int k, int32_t* out_idx, float* xx, const int32_t* seeds,
                   int ks, void* stream) {
    using namespace pcs;
    PCS_CHECK_ARG(B >= 0 && N >= 1 && k >= 1 && k <= N, "pcs_knn: bad sizes B=%d N=%d k=%d", B, N, k);
    PCS_CHECK_ARG(x && out_idx, "pcs_knn: null pointer");
    if (B == 0) return 0;
    hipStream_t s = as_stream(stream);
    int rc;
    switch (F) {
        case 3: rc = dispatch_k<3>(x, B, N, k, out_idx, xx, xx ? seeds : nullptr, ks, s); break;
        case 64: rc = dispatch_k<64>(x, B, N, k, out_idx, xx, seeds, ks, s); break;
        default:
            set_error("pcs_knn: F=%d not instantiated (3, 64)", F);
            return (int)hipErrorInvalidValue;
    }
    if (rc) return rc;
    return launch_status("pcs_knn");
}

// Reference: models/dgcnn/dgcnn.py:7-21.  x point-major (B, N, F) fp32; out (B, N, k) int32,
// best first.  F in {3, 64}; k in {16, 20, 32, 40}.
PCS_API int pcs_knn(const float* x, int B, int N, int F, int k, int32_t* out_idx, void* stream) {
    return knn_run(x, B, N, F, k, out_idx, nullptr, nullptr, 0, stream);
}

PCS_API int pcs_knn_workspace(int B, int N, size_t* bytes) {
    PCS_CHECK_ARG(bytes && B >= 0 && N >= 0, "pcs_knn_workspace: bad arguments");
    *bytes = (size_t)B * N * sizeof(float) + 256;
    return 0;
}

// pcs_knn with a caller workspace (pcs_knn_workspace bytes): the squared norms are computed
// once per point instead of once per point and streaming wave (same lists, fewer VALU ops)
PCS_API int pcs_knn_ws(const float* x, int B, int N, int F, int k, int32_t* out_idx, void* ws, size_t ws_bytes,
                       void* stream) {
    PCS_CHECK_ARG(ws && ws_bytes >= (size_t)B * N * sizeof(float) + 256, "pcs_knn_ws: workspace too small");
    float* xx = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
    return knn_run(x, B, N, F, k, out_idx, xx, nullptr, 0, stream);
}

// pcs_knn_ws whose rows start from the threshold of a previous neighbour list (seeds (B, N, ks)
// int32, e.g. the previous EdgeConv's graph): the same lists, fewer survivors to merge.  Any
// seeds are safe -- a row whose seeds are out of range, repeated or fewer than k is searched
// unseeded.
PCS_API int pcs_knn_seeded(const float* x, int B, int N, int F, int k, const int32_t* seeds, int ks, int32_t* out_idx,
                           void* ws, size_t ws_bytes, void* stream) {
    PCS_CHECK_ARG(ws && ws_bytes >= (size_t)B * N * sizeof(float) + 256, "pcs_knn_seeded: workspace too small");
    PCS_CHECK_ARG(seeds && ks >= 1, "pcs_knn_seeded: null seeds or ks < 1");
    float* xx = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
    return knn_run(x, B, N, F, k, out_idx, xx, seeds, ks, stream);
}

// ----------------------------------------------------------------------------- pruned kNN API
static size_t knn_align256(size_t n) { return (n + 255) & ~size_t(255); }

// Morton order of each cloud's points by their first three features (DGCNN: the xyz graph's
// input), (B, N) int32 -- the order pcs_knn_pruned scans in.  Clouds past 8192 points get the
// identity order (correct, unpruned in effect).
PCS_API int pcs_knn_order(const float* x, int B, int N, int F, int32_t* order, void* stream) {
    using namespace pcs;
    PCS_CHECK_ARG(B >= 0 && N >= 1 && F >= 3, "pcs_knn_order: bad sizes B=%d N=%d F=%d", B, N, F);
    PCS_CHECK_ARG(x && order, "pcs_knn_order: null pointer");
    if (B == 0) return 0;
    hipStream_t s = as_stream(stream);
    if (N > KO_MAX) {
        const long long P = (long long)B * N;
        hipLaunchKernelGGL(knn_identity_order_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, P, N, order);
        return launch_status("pcs_knn_order");
    }
    int P = 64;
    while (P < N) P <<= 1;
    const size_t lds = (size_t)P * sizeof(unsigned long long);
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&knn_order_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)(KO_MAX * sizeof(unsigned long long)));
    (void)attr;
    hipLaunchKernelGGL(knn_order_kernel, dim3(B), dim3(1024), lds, s, x, N, F, P, order);
    return launch_status("pcs_knn_order");
}

PCS_API int pcs_knn_pruned_workspace(int B, int N, int F, size_t* bytes) {
    using namespace pcs;
    PCS_CHECK_ARG(bytes && B >= 0 && N >= 0 && F >= 1, "pcs_knn_pruned_workspace: bad arguments");
    const size_t nt = ((size_t)N + KNN_TC - 1) / KNN_TC;
    // squared norms | tile fields (B, TS, nt) | scan orders (B, nt, nt) tile ids | their bounds
    *bytes = knn_align256((size_t)B * N * sizeof(float)) + 256;
    if (N <= KO_MAX)    // (larger clouds take the unpruned kernel: norms only)
        *bytes += (size_t)B * nt * knn_tile_stride(F) * sizeof(float) + 2 * (size_t)B * nt * nt * sizeof(float);
    return 0;
}

// pcs_knn_seeded (seeds nullable) scanning each cloud in `order` (pcs_knn_order's output, a
// permutation of 0..N-1 per cloud) with tile pruning: the same lists from a fraction of the
// candidate tiles.  Workspace: pcs_knn_pruned_workspace(B, N, F) bytes.
PCS_API int pcs_knn_pruned(const float* x, int B, int N, int F, int k, const int32_t* order, const int32_t* seeds,
                           int ks, int32_t* out_idx, void* ws, size_t ws_bytes, void* stream) {
    using namespace pcs;
    PCS_CHECK_ARG(B >= 0 && N >= 1 && k >= 1 && k <= N, "pcs_knn_pruned: bad sizes B=%d N=%d k=%d", B, N, k);
    PCS_CHECK_ARG(x && out_idx && order, "pcs_knn_pruned: null pointer");
    PCS_CHECK_ARG(!seeds || ks >= 1, "pcs_knn_pruned: ks < 1");
    size_t need = 0;
    pcs_knn_pruned_workspace(B, N, F, &need);
    PCS_CHECK_ARG(ws && ws_bytes >= need, "pcs_knn_pruned: workspace too small (%zu < %zu)", ws_bytes, need);
    if (B == 0) return 0;
    hipStream_t s = as_stream(stream);
    const uintptr_t base = (reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255);
    float* xx = reinterpret_cast<float*>(base);
    float* tinfo = reinterpret_cast<float*>(base + knn_align256((size_t)B * N * sizeof(float)));
    int rc;
    switch (F) {
        case 3: rc = dispatch_pruned<3>(x, B, N, k, out_idx, xx, order, tinfo, seeds, ks, s); break;
        case 64: rc = dispatch_pruned<64>(x, B, N, k, out_idx, xx, order, tinfo, seeds, ks, s); break;
        default:
            set_error("pcs_knn_pruned: F=%d not instantiated (3, 64)", F);
            return (int)hipErrorInvalidValue;
    }
    if (rc) return rc;
    return launch_status("pcs_knn_pruned");
}

#ifdef PCS_KNN_DIAG
// diagnostic build only: the per-wave scanned-tile counts of the last pruned launch ((b, tile) order)
PCS_API int pcs_knn_diag(int* out, int n) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pcs::g_knn_diag), sizeof(int) * (size_t)std::min(n, 8 << 13));
}
#endif
