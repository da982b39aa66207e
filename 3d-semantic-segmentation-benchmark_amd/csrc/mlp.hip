// Shared-MLP engine: 1x1 conv + training-mode BatchNorm + ReLU/LeakyReLU (+ max over K)
// on point-major rows, fp32 on the MFMA cores (v_mfma_f32_32x32x2_f32).
//
// Reference semantics: MiniPointNet / UnitPointNet (models/utils/common.py:125-178),
// EdgeConv's conv->BN->LeakyReLU->max (models/dgcnn/dgcnn.py:67-76), DGCNN's
// conv5..conv7 (dgcnn.py:188-207): z = W x + b ; y = BN_train(z) ; a = act(y) ; [max over K].
//
// Design:
//  * GEMM over rows, Z[M x N] = T(A)[M x K] . W^T, where T is identity or the
//    PREVIOUS layer's BN+activation applied while the A tile is loaded -- so a
//    BN-applied activation is never written to HBM; only pre-BN Z is stored;
//  * the epilogue adds the conv bias and emits per-block fp64 partial sums
//    (sum z, sum z^2) per channel; `bn_finalize` turns them into scale/shift
//    (s = gamma/sqrt(var+eps), t = beta - mean*s) and updates the running stats
//    exactly like nn.BatchNorm (momentum, unbiased running_var);
//  * pooling reads Z once: max_k act(z*s+t) with the first argmax;
//  * backward: dgrad GEMM (dA_prev = dZ . W) whose epilogue already reduces the
//    previous layer's BN-backward sums (sum dy, sum dy*xhat); wgrad GEMM
//    (dW = dZ^T . T(A_prev)) split over rows, each split's partial tile stored and
//    summed in a fixed order by a second kernel (deterministic: no float atomics).
// Statistics are accumulated in fp64 (as ATen's CPU batch norm does).
#include "mlp_common.hpp"

#include <type_traits>

#include <stdlib.h>

namespace pcs {

// ------------------------------------------------------------------ row GEMM
// C[M x N] = T(A)[M x K] . B[K x N],  B[k][n] = W[n*ldw + k]  (W row-major N x K).
//
// WM x WN waves (4 or 8: 256 or 512 threads); each wave owns TM x TN 32x32 MFMA tiles.
// K is consumed in 32-deep slabs staged through a double-buffered LDS ring with the
// next slab's global loads in flight (registers) while the current slab is computed.
// Inside a slab the k order is permuted so that lane half h takes k = 16h + s
// (s = 0..15): each lane's A/B fragments are then 16 CONSECUTIVE floats of one LDS
// row, read with ds_read_b128; the 144-B row stride (BK + 4 floats) makes those
// reads bank-conflict free.  The MFMA sums over k, so the permutation only
// reorders the fp32 accumulation.
constexpr int GBK = 32;
constexpr int GLDK = GBK + 4;

// row swizzle of channel c's LDS row (multiples of 4: keeps 4-row groups 16-B contiguous)
__device__ __forceinline__ int lds_swz(int c) { return ((c >> 3) & 7) << 2; }

//
// BT: B is stored k-major, B[k][n] = W[k*ldw + n] (the data-gradient GEMM reads the layer's
// own weight matrix, no transpose): quads are loaded along n and written transposed into
// Bs with the lds_swz row swizzle (the fragment reads apply the same swizzle).
// EPI: what the epilogue computes besides storing C, fixed at compile time so the per-element
// epilogue is straight-line code: EPI_STATS (BN partials of C), EPI_BWD (BN-backward partials
// of the previous layer), EPI_POOL (fused max/min over K rows), or EPI_GENERIC (decided from
// the arguments at run time: the combinations the engine never issues).
constexpr int EPI_STATS = 1, EPI_BWD = 2, EPI_POOL = 4, EPI_GENERIC = 8;


template <int BM, int BN, int WM, int WN, int AM, bool BT, int EPI>
__global__ __launch_bounds__(WM * WN * 64, 2) void gemm_rows_kernel(GemmArgs g) {
    constexpr int NT = WM * WN * 64;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int AV = BM * GBK / 4 / NT;
    constexpr int BV = (BN * GBK / 4 + NT - 1) / NT;
    constexpr bool kBFull = (BN * GBK / 4) % NT == 0;     // every thread owns BV whole B quads
    static_assert((WM * WN == 4 || WM * WN == 8) && TM >= 1 && TN >= 1 && AV >= 1, "tile");
    __shared__ __attribute__((aligned(16))) float As[2][BM][GLDK];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN][GLDK];
    __shared__ double red[2][WM][BN];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (scalar) index
    const int wm = wave / WN, wn = wave % WN;
    const int n0 = blockIdx.y * BN;
    const int h = lane >> 5, l32 = lane & 31;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    float4 ra[AV], rz[AV], rb[BV];
    unsigned rg[AV];
    // every A float4 of this thread sits at the same k offset 4*(tid&7) of a slab, so one
    // coefficient quad per slab serves all of them
    Quad q;
    // clamps keep every load inside the operand's own K (N) channels, rounded up to a quad: a
    // column-block alias (W + C of an EdgeConv, a row-stride view of a wider buffer) must not
    // read past its last row's end
    const int lda_last = ((g.K + 3) & ~3) - 4;
    const int ldw_last = BT ? ((g.N + 3) & ~3) - 4 : ((g.K + 3) & ~3) - 4;
    const bool bt_scalar = BT && ((g.ldw & 3) || (reinterpret_cast<uintptr_t>(g.W) & 15));
    auto gload = [&](int m0, int k0) {
        const int gk = k0 + 4 * (tid & 7);
        const int gkc = min(gk, lda_last);
        load_quad<AM>(g.a, gk, g.K, q);
#pragma unroll
        for (int it = 0; it < AV; ++it) {
            const int gr = min(m0 + ((it * NT + tid) >> 3), g.M - 1);
            load_raw<AM>(g.a, gr, gkc, ra[it], rz[it], rg[it]);
        }
#pragma unroll
        for (int it = 0; it < BV; ++it) {
            const int e = it * NT + tid;
            if constexpr (BT) {
                const int gk = min(k0 + e / (BN / 4), g.K - 1);
                if (bt_scalar) {      // k-major rows that are not 16-B aligned (a first layer's W from
                                      // column dx_col0 on, rows of 3 + D): scalar loads
                    const float* wr = g.W + (size_t)gk * g.ldw;
                    const int gn = n0 + 4 * (e % (BN / 4)), nl = g.N - 1;
                    PCS_DCHECK(gk >= 0 && gk < g.K, "row GEMM k-major W row %d of %d", gk, g.K);
                    if (kBFull || e < BN * GBK / 4)
                        rb[it] = make_float4(wr[min(gn, nl)], wr[min(gn + 1, nl)], wr[min(gn + 2, nl)],
                                             wr[min(gn + 3, nl)]);
                } else {
                    const int gn = min(n0 + 4 * (e % (BN / 4)), ldw_last);
                    PCS_DCHECK(gk >= 0 && gk < g.K && gn >= 0 && gn + 4 <= ((g.N + 3) & ~3),
                               "row GEMM k-major W (%d, %d) outside %d x %d", gk, gn, g.K, g.N);
                    if (kBFull || e < BN * GBK / 4)
                        rb[it] = *reinterpret_cast<const float4*>(g.W + (size_t)gk * g.ldw + gn);
                }
            } else {
                const int gn = min(n0 + (e >> 3), g.N - 1);
                if (g.ldw & 3) {      // unpadded weight rows (a stack's first layer, K = 3 + D): scalar loads
                    const float* wr = g.W + (size_t)gn * g.ldw;
                    const int gk = k0 + 4 * (e & 7), kl = g.K - 1;
                    PCS_DCHECK(gn >= 0 && gn < g.N, "row GEMM W row %d of %d", gn, g.N);
                    if (kBFull || e < BN * GBK / 4)
                        rb[it] = make_float4(wr[min(gk, kl)], wr[min(gk + 1, kl)], wr[min(gk + 2, kl)],
                                             wr[min(gk + 3, kl)]);
                } else {
                    const int gk2 = min(k0 + 4 * (e & 7), ldw_last);
                    PCS_DCHECK(gn >= 0 && gn < g.N && gk2 >= 0 && gk2 + 4 <= ((g.K + 3) & ~3),
                               "row GEMM W (%d, %d) outside %d x %d", gn, gk2, g.N, g.K);
                    if (kBFull || e < BN * GBK / 4)
                        rb[it] = *reinterpret_cast<const float4*>(g.W + (size_t)gn * g.ldw + gk2);
                }
            }
        }
    };
    auto sstore = [&](int buf, int m0, int k0) {
        const int gk = k0 + 4 * (tid & 7);
#pragma unroll
        for (int it = 0; it < AV; ++it) {
            const int r = (it * NT + tid) >> 3;
            *reinterpret_cast<float4*>(&As[buf][r][4 * (tid & 7)]) =
                xform4<AM>(g.a, ra[it], rz[it], rg[it], min(m0 + r, g.M - 1), q, gk, g.K);
        }
#pragma unroll
        for (int it = 0; it < BV; ++it) {
            const int e = it * NT + tid;
            if constexpr (BT) {
                const int kk = e / (BN / 4), n = 4 * (e % (BN / 4));
                const float4 v = k0 + kk < g.K ? rb[it] : make_float4(0.f, 0.f, 0.f, 0.f);
                if (kBFull || e < BN * GBK / 4) {
                    Bs[buf][n + 0][kk ^ lds_swz(n + 0)] = v.x;
                    Bs[buf][n + 1][kk ^ lds_swz(n + 1)] = v.y;
                    Bs[buf][n + 2][kk ^ lds_swz(n + 2)] = v.z;
                    Bs[buf][n + 3][kk ^ lds_swz(n + 3)] = v.w;
                }
            } else {
                const int gk2 = k0 + 4 * (e & 7);
                float4 v = rb[it];
                v.x = gk2 + 0 < g.K ? v.x : 0.f;
                v.y = gk2 + 1 < g.K ? v.y : 0.f;
                v.z = gk2 + 2 < g.K ? v.z : 0.f;
                v.w = gk2 + 3 < g.K ? v.w : 0.f;
                if (kBFull || e < BN * GBK / 4) *reinterpret_cast<float4*>(&Bs[buf][e >> 3][4 * (e & 7)]) = v;
            }
        }
    };

    // ---- persistent loop: this block owns row tiles blockIdx.x + t*gridDim.x; the (tile, slab)
    // iterations are flattened so the NEXT tile's first slab is loading while this tile's
    // epilogue stores C (no exposed prologue per tile)
    constexpr bool GEN = (EPI & EPI_GENERIC) != 0;
    const bool want_stats = GEN ? g.stats != nullptr : (EPI & EPI_STATS) != 0;
    const bool want_b = GEN ? g.bstats != nullptr : (EPI & EPI_BWD) != 0;
    const bool do_pool = GEN ? g.pool_k != 0 : (EPI & EPI_POOL) != 0;
    double s1[TN], s2[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) { s1[j] = 0.0; s2[j] = 0.0; }
    const int nk = (g.K + GBK - 1) / GBK;
    const int mtiles = (g.M + BM - 1) / BM;
    const int my_tiles = blockIdx.x < mtiles ? (mtiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
    const int total = my_tiles * nk;
    if (total > 0) {
        gload(blockIdx.x * BM, 0);
        sstore(0, blockIdx.x * BM, 0);
    }
    __syncthreads();
    for (int it = 0; it < total; ++it) {
        const int buf = it & 1;
        const int ti = it / nk, ks = it - ti * nk;
        const int m0 = (blockIdx.x + ti * gridDim.x) * BM;
        const int tn = (it + 1) / nk, kn = (it + 1) - tn * nk;
        const int m0n = (blockIdx.x + tn * gridDim.x) * BM;      // past the end: clamped loads, unused
        gload(m0n, kn * GBK);     // unconditional: no phi copies of in-flight registers
        // keep the next slab's loads in flight: nothing that consumes them may be
        // scheduled above the MFMAs of this slab
        __builtin_amdgcn_sched_barrier(0);
        // two-level fp32 accumulation (tiles with <= 2 MFMA blocks per wave, whose second set of
        // accumulators fits the register budget; the 4-block 128 x 128 tile would spill): the
        // slab's 16 MFMA steps (32 k) go into a fresh accumulator that is then added to the
        // tile's running sum, so an output element sees 16 + K/32 roundings instead of K/2 (one
        // per MFMA step).  Over K = 512 .. 2048 (the data gradients of the wide layers) that is
        // 2-3x less rounding error in dX, the CPU reference's sgemm level
        // (scripts/diag/stack_grad_error.py); the cost is 16 VALU adds per 16 MFMAs.
        constexpr bool TWO = TM * TN <= 2;
        f32x16 sacc[TWO ? TM : 1][TWO ? TN : 1];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            float4 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                a[i] = *reinterpret_cast<const float4*>(&As[buf][wm * WTM + i * 32 + l32][16 * h + 4 * qq]);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = wn * WTN + j * 32 + l32;
                b[j] = *reinterpret_cast<const float4*>(&Bs[buf][n][(16 * h + 4 * qq) ^ (BT ? lds_swz(n) : 0)]);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    f32x16& d = TWO ? sacc[TWO ? i : 0][TWO ? j : 0] : acc[i][j];
                    const f32x16 c0 = {};
                    d = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, (TWO && qq == 0) ? c0 : d, 0, 0, 0);
                    d = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, d, 0, 0, 0);
                    d = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, d, 0, 0, 0);
                    d = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, d, 0, 0, 0);
                }
        }
        if constexpr (TWO) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] += sacc[TWO ? i : 0][TWO ? j : 0];
        }
        __builtin_amdgcn_sched_barrier(0);
        if (ks == nk - 1) {
            // ---- tile epilogue: bias, store, per-channel partial reductions.  The fused
            // BN-backward epilogue's Z loads are issued for a whole column strip first
            // (clamped addresses, no branches) so their latency is paid once, not per element.
            // A tile whose rows and columns are all in range (every tile but a ragged last
            // one) takes the FULL path: no per-element bounds checks, and C / Z addressed as a
            // wave-uniform 64-bit row base + a 32-bit per-lane offset (saddr loads / stores)
            // instead of a 64-bit multiply-add per element.
            auto epilogue = [&](auto full_t) __attribute__((always_inline)) {
                constexpr bool FULL = decltype(full_t)::value;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int col = n0 + wn * WTN + j * 32 + l32;
                    const bool cok = FULL || col < g.N;
                    const int colc = cok ? col : g.N - 1;
                    const float bv = (g.bias && cok) ? g.bias[col] : 0.f;
                    float sp = 0.f, tp = 0.f, mp = 0.f, ip = 0.f;
                    // pooling keeps one extreme per column: the max of C where the consumer's BN scale
                    // (sign of gamma) is >= 0, else the min -- tracked as the max of -C (sign flip)
                    const unsigned pflip = (do_pool && g.psign && g.psign[colc] < 0.f) ? 0x80000000u : 0u;
                    if (want_b) { sp = g.e.s[colc]; tp = g.e.t[colc]; mp = g.e.mean[colc]; ip = g.e.inv[colc]; }
#pragma unroll
                    for (int i = 0; i < TM; ++i) {
                    const int rb = __builtin_amdgcn_readfirstlane(m0 + wm * WTM + i * 32);   // wave-uniform
                    float* const Cb = g.C + (size_t)rb * g.ldc;
                    const float* const Zb = g.e.z + (size_t)rb * g.e.ldz;
                    // fused pooling state of this lane's rows of the 32-row block (a group of 32, or
                    // one group of 16 per hb): running max/min of C and the first row reaching it
                    float pmx = -INFINITY;
                    int imx = 4 * h;
#pragma unroll
                    for (int hb = 0; hb < 2; ++hb) {     // Z loads batched 8 at a time (register budget)
                        if (do_pool && g.pool_k == 16 && hb == 1) { pmx = -INFINITY; imx = 16 + 4 * h; }
                        float zt[8];
                        if (want_b) {
#pragma unroll
                            for (int rr = 0; rr < 8; ++rr) {
                                const int r = 8 * hb + rr;
                                const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
                                if constexpr (FULL) {
                                    const unsigned bo = 4u * (unsigned)(rl * g.e.ldz + col);   // 32-bit byte offset
                                    zt[rr] = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(Zb) + bo);
                                } else {
                                    const int row = min(rb + rl, g.M - 1);
                                    zt[rr] = g.e.z[(size_t)row * g.e.ldz + colc];
                                }
                            }
                        }
#pragma unroll
                        for (int rr = 0; rr < 8; ++rr) {
                            const int r = 8 * hb + rr;
                            const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
                            const bool ok = FULL || (rb + rl < g.M && cok);
                            const float v = acc[i][j][r] + bv;
                            if constexpr (FULL) {
                                const unsigned bo = 4u * (unsigned)(rl * g.ldc + col);
                                *reinterpret_cast<float*>(reinterpret_cast<char*>(Cb) + bo) = v;
                            } else {
                                if (ok) g.C[(size_t)(rb + rl) * g.ldc + col] = v;
                            }
                            if (do_pool) {
                                const int rib = rl;                          // increasing in r: first wins
                                const float pv = __uint_as_float(__float_as_uint(v) ^ pflip);
                                if (pv > pmx) { pmx = pv; imx = rib; }
                            }
                            if (want_stats) {
                                const double d = ok ? (double)v : 0.0;
                                s1[j] += d;
                                s2[j] += d * d;
                            }
                            if (want_b) {
                                const float z = zt[rr];
                                const float dy = v * dact_f(z * sp + tp, g.e.act, g.e.slope);
                                const float xh = (z - mp) * ip;
                                const double dd = ok ? (double)dy : 0.0;
                                s1[j] += dd;
                                s2[j] += dd * (double)xh;
                            }
                            acc[i][j][r] = 0.f;
                        }
                        if (do_pool && (g.pool_k == 16 || hb == 1)) {
                            // merge with the other lane half (same column, the other rows), first row on ties
                            const float ox = __shfl_xor(pmx, 32);
                            const int oix = __shfl_xor(imx, 32);
                            if (ox > pmx || (ox == pmx && oix < imx)) { pmx = ox; imx = oix; }
                            const int r0 = rb + (g.pool_k == 16 ? 16 * hb : 0);
                            if (h == 0 && cok && r0 < g.M) {
                                const size_t gi = (size_t)(r0 / g.pool_k);
                                const int base = g.pool_k == 16 ? 16 * hb : 0;
                                const size_t o = gi * g.N + col;
                                g.pz[o] = __uint_as_float(__float_as_uint(pmx) ^ pflip);
                                g.pa[o] = (unsigned char)(imx - base);
                            }
                        }
                    }
                    }
                }
            };
            if (m0 + BM <= g.M && n0 + BN <= g.N) epilogue(std::true_type{});
            else epilogue(std::false_type{});
        }
        if (it + 1 < total) sstore(buf ^ 1, m0n, kn * GBK);
        __syncthreads();
    }

    if (want_stats || want_b) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int lc = wn * WTN + j * 32 + l32;
            double a = s1[j] + __shfl_xor(s1[j], 32);
            double b = s2[j] + __shfl_xor(s2[j], 32);
            if (lane < 32) {
                red[0][wm][lc] = a;
                red[1][wm][lc] = b;
            }
        }
        __syncthreads();
        double* out = want_stats ? g.stats : g.bstats;
        for (int c = tid; c < BN; c += NT) {
            const int col = n0 + c;
            if (col < g.N) {
                double a = 0.0, b = 0.0;
#pragma unroll
                for (int w = 0; w < WM; ++w) { a += red[0][w][c]; b += red[1][w][c]; }
                out[(size_t)col * gridDim.x + blockIdx.x] = a;
                out[((size_t)g.N + col) * gridDim.x + blockIdx.x] = b;
            }
        }
    }
}

// ------------------------------------------------------------------ weight gradient
// part[split][n][k] = sum_{r in split} X[r][n] * Y[r][k] ; pdb[split][n] = sum_{r in split} X[r][n]
// (rows split over gridDim.x; wgrad_reduce_kernel adds the splits into dW / db in split order)
// X = the layer's dZ (through its BNBWD/POOLBWD transform: rebuilt from the output
// gradient and Z on load), Y = the layer's input (through the previous layer's BNACT).
// Same LDS/fragment scheme as the row GEMM with the ROW index as the reduction
// axis: X and Y slabs of 32 rows are stored transposed ([channel][row], 144-B
// stride) so each lane's fragment is 16 consecutive rows.  Each block accumulates its
// row range in the MFMA's fp32 accumulators and stores its partial tile: every element of
// part[split] is written by exactly one block, and the reduce sums the splits in order, so
// two identical backward passes give bitwise-identical gradients.

//
// Wave grid: WGO x WGI waves split the BO x BI tile and WR = 4 / (WGO * WGI) waves split
// each slab's 32 rows (thin tiles: a 32-wide side has one wave, the spare waves take
// disjoint row quarters/halves of the slab and add their partial tiles separately).
template <int BO, int BI, int XM, int YM, int NS>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(Operand xo, int N, Operand yo, int K, int M,
                                                       int rows_per_block, float* __restrict__ part,
                                                       float* __restrict__ pdb) {
    constexpr int BR = 32, LDR = BR + 4;
    constexpr int WGO = BO >= 64 ? 2 : 1, WGI = BI >= 64 ? 2 : 1, WR = 4 / (WGO * WGI);
    constexpr int QPW = 4 / WR;                       // 4-row fragment groups (q) per wave per half-slab
    constexpr int TM = BO / WGO / 32, TN = BI / WGI / 32;
    constexpr int XV = BR * BO / 4 / 256, YV = BR * BI / 4 / 256;
    static_assert(TM >= 1 && TN >= 1 && XV >= 1 && YV >= 1, "wgrad tile");
    static_assert(WR == 1, "one wave per output fragment: the partial tile is stored, not accumulated");
    __shared__ __attribute__((aligned(16))) float Xs[2][BO][LDR];
    __shared__ __attribute__((aligned(16))) float Ys[2][BI][LDR];
    __shared__ float dbs[256 / (BO / 4)][BO];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wi = wave % WGI, wo = (wave / WGI) % WGO, wr = wave / (WGI * WGO);
    const int h = lane >> 5, l32 = lane & 31;
    const int tiles_i = (K + BI - 1) / BI;
    // XCD-aware order (a bijective remap of the (split, tile) grid, speed only): workgroups are
    // dispatched round-robin over the 8 XCDs in linear-id order, so XCD x takes a contiguous run
    // of remapped ids, tile-fastest -- the tiles of one row split (the same X / Y rows) run
    // together on one XCD and share its L2 instead of each fetching the rows from HBM
    const int lin = blockIdx.x + blockIdx.y * gridDim.x;
    const int nwg = gridDim.x * gridDim.y, q8 = nwg / 8, r8 = nwg % 8, xcd = lin % 8;
    const int rt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + lin / 8;
    const int sp = rt / gridDim.y, ti = rt - sp * gridDim.y;
    const int n0 = (ti / tiles_i) * BO;
    const int k0 = (ti % tiles_i) * BI;
    const int rb = sp * rows_per_block;
    const int re = min(M, rb + rows_per_block);
    const bool do_db = (pdb != nullptr) && (k0 == 0);
    float* __restrict__ tile_part = part + (size_t)sp * N * K;

    // Transposed LDS stores without bank conflicts: each 32-lane half stores 4 rows x 8
    // channel quads, and the row index is XOR-swizzled in 4-row groups by the channel
    // (lds_swz), so the 32 ds_write_b32 of a half hit 32 distinct banks; the fragment reads
    // apply the same swizzle (4-row groups stay intact, so they remain ds_read_b128).
    // this thread's fixed channel quads (and their transform coefficients) and rows
    const int half = tid >> 5;
    const int xc4 = (half % (BO / 32)) * 8 + ((tid >> 2) & 7), yc4 = (half % (BI / 32)) * 8 + ((tid >> 2) & 7);
    const int xr = (half / (BO / 32)) * 4 + (tid & 3), yr = (half / (BI / 32)) * 4 + (tid & 3);
    constexpr int XRPI = 1024 / BO, YRPI = 1024 / BI;     // rows per load iteration
    const int gn = n0 + 4 * xc4, gk = k0 + 4 * yc4;
    Quad qx, qy;
    load_quad<XM>(xo, gn, N, qx);
    load_quad<YM>(yo, gk, K, qy);
    float dbv[4] = {0.f, 0.f, 0.f, 0.f};

    // the MFMA accumulates the block's rows (<= a few thousand) directly in fp32: a second
    // flush accumulator would cost TM*TN*16 more VGPRs and push the wide tiles into scratch
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // NS register stages: each slab's loads are issued NS slabs ahead of their LDS store
    // (thin tiles, where one slab of MFMAs is too short to cover HBM latency)
    static_assert(NS >= 1 && NS <= 4, "stages");
    float4 rx[NS][XV], rxz[NS][XV], ry[NS][YV], ryz[NS][YV];
    unsigned rxa[NS][XV], rya[NS][YV];
    const int gnc = min(gn, ((N + 3) & ~3) - 4), gkc = min(gk, ((K + 3) & ~3) - 4);   // inside the operands' channels
    auto gload = [&](int st, int r0) {
#pragma unroll
        for (int it = 0; it < XV; ++it) {
            const int gr = min(r0 + it * XRPI + xr, M - 1);
            load_raw<XM>(xo, gr, gnc, rx[st][it], rxz[st][it], rxa[st][it]);
        }
#pragma unroll
        for (int it = 0; it < YV; ++it) {
            const int gr = min(r0 + it * YRPI + yr, M - 1);
            load_raw<YM>(yo, gr, gkc, ry[st][it], ryz[st][it], rya[st][it]);
        }
    };
    auto sstore = [&](int st, int buf, int r0) {
#pragma unroll
        for (int it = 0; it < XV; ++it) {
            const int r = it * XRPI + xr;
            float4 v = xform4<XM>(xo, rx[st][it], rxz[st][it], rxa[st][it], r0 + r, qx, gn, N);
            if (r0 + r >= re) v = make_float4(0.f, 0.f, 0.f, 0.f);
            const int rs = r ^ lds_swz(4 * xc4);      // the 4 channels of a quad share the swizzle
            Xs[buf][4 * xc4 + 0][rs] = v.x;
            Xs[buf][4 * xc4 + 1][rs] = v.y;
            Xs[buf][4 * xc4 + 2][rs] = v.z;
            Xs[buf][4 * xc4 + 3][rs] = v.w;
            if (do_db) { dbv[0] += v.x; dbv[1] += v.y; dbv[2] += v.z; dbv[3] += v.w; }
        }
#pragma unroll
        for (int it = 0; it < YV; ++it) {
            const int r = it * YRPI + yr;
            float4 v = xform4<YM>(yo, ry[st][it], ryz[st][it], rya[st][it], r0 + r, qy, gk, K);
            if (r0 + r >= re) v = make_float4(0.f, 0.f, 0.f, 0.f);
            const int rs = r ^ lds_swz(4 * yc4);
            Ys[buf][4 * yc4 + 0][rs] = v.x;
            Ys[buf][4 * yc4 + 1][rs] = v.y;
            Ys[buf][4 * yc4 + 2][rs] = v.z;
            Ys[buf][4 * yc4 + 3][rs] = v.w;
        }
    };

    const int nslab = (re - rb + BR - 1) / BR;
    if (nslab > 0) {
#pragma unroll
        for (int u = 0; u < NS; ++u) gload(u, rb + u * BR);
        sstore(0, 0, rb);
    }
    __syncthreads();
    // one slab: issue the loads of slab sl+NS into stage `lst` (unconditional, clamped past the
    // end), MFMAs on LDS buffer sl&1, then slab sl+1 from stage `sst` into the other buffer
    auto body = [&](int sl, int lst, int sst) {
        const int buf = sl & 1;
        gload(lst, rb + (sl + NS) * BR);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int qi = 0; qi < QPW; ++qi) {
            const int q = wr * QPW + qi;
            float4 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                a[i] = *reinterpret_cast<const float4*>(
                    &Xs[buf][wo * (BO / WGO) + i * 32 + l32][(16 * h + 4 * q) ^ lds_swz(wo * (BO / WGO) + i * 32 + l32)]);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                b[j] = *reinterpret_cast<const float4*>(
                    &Ys[buf][wi * (BI / WGI) + j * 32 + l32][(16 * h + 4 * q) ^ lds_swz(wi * (BI / WGI) + j * 32 + l32)]);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
                }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (sl + 1 < nslab) sstore(sst, buf ^ 1, rb + (sl + 1) * BR);
        __syncthreads();
    };
    // slab sl's registers live in stage sl % NS: freed once stored, refilled with slab sl + NS
    for (int sl = 0; sl < nslab; sl += NS) {
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            if (sl + u >= nslab) break;
            body(sl + u, u, (u + 1) % NS);
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int kcol = k0 + wi * (BI / WGI) + j * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = n0 + wo * (BO / WGO) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (n < N && kcol < K) tile_part[(size_t)n * K + kcol] = acc[i][j][r];
            }
        }
    if (do_db) {
        dbs[xr][4 * xc4 + 0] = dbv[0];
        dbs[xr][4 * xc4 + 1] = dbv[1];
        dbs[xr][4 * xc4 + 2] = dbv[2];
        dbs[xr][4 * xc4 + 3] = dbv[3];
        __syncthreads();
        if (tid < BO && n0 + tid < N) {
            float a = 0.f;
#pragma unroll
            for (int gi = 0; gi < 256 / (BO / 4); ++gi) a += dbs[gi][tid];
            pdb[(size_t)sp * N + n0 + tid] = a;
        }
    }
}

// dW[e] += sum_{s < splits} part[s][e] (e < nk) and db[e] += sum_s pdb[s][e] (e < N, the
// blocks past dW's): the weight and bias gradients from the wgrad's per-split partials.
// 64 elements per block as 16 lanes x float4, so one wave instruction reads four 256-B runs
// (splits g .. g+3 of the same 64 elements); the block's 16 lane groups take splits g, g + 16,
// ... (fp64, two interleaved accumulators), then the 16 group sums are added in group order
// through LDS -- a fixed summation tree, so the result is reproducible bit for bit.
// (Round 2's 16-element blocks read 64-B runs: ~18 us per FP1-sized reduce, ~1.8 TB/s.)
constexpr int kRedElems = 64, kRedGroups = 16;
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int splits, long long nk,
                                                           float* __restrict__ dW, const float* __restrict__ pdb,
                                                           int N, float* __restrict__ db) {
    __shared__ double red[kRedGroups][kRedElems];
    const int q = threadIdx.x & 15, g = threadIdx.x >> 4;
    const long long wblocks = (nk + kRedElems - 1) / kRedElems;
    const bool bias = blockIdx.x >= wblocks;
    const float* src = bias ? pdb : part;
    float* out = bias ? db : dW;
    const long long n = bias ? N : nk;
    const long long eb = (bias ? blockIdx.x - wblocks : (long long)blockIdx.x) * kRedElems;
    const long long e0 = eb + 4 * q;
    double a[4] = {0.0, 0.0, 0.0, 0.0}, b[4] = {0.0, 0.0, 0.0, 0.0};
    if (n % 4 == 0 && e0 + 3 < n) {          // rows of n floats: 16-B aligned float4 runs
        int sp = g;
        for (; sp + kRedGroups < splits; sp += 2 * kRedGroups) {
            const float4 v = *reinterpret_cast<const float4*>(src + (size_t)sp * n + e0);
            const float4 w = *reinterpret_cast<const float4*>(src + (size_t)(sp + kRedGroups) * n + e0);
            a[0] += (double)v.x; a[1] += (double)v.y; a[2] += (double)v.z; a[3] += (double)v.w;
            b[0] += (double)w.x; b[1] += (double)w.y; b[2] += (double)w.z; b[3] += (double)w.w;
        }
        if (sp < splits) {
            const float4 v = *reinterpret_cast<const float4*>(src + (size_t)sp * n + e0);
            a[0] += (double)v.x; a[1] += (double)v.y; a[2] += (double)v.z; a[3] += (double)v.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (e0 + j < n)
                for (int sp = g; sp < splits; sp += kRedGroups) a[j] += (double)src[(size_t)sp * n + e0 + j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) red[g][4 * q + j] = a[j] + b[j];
    __syncthreads();
    if (threadIdx.x < kRedElems && eb + threadIdx.x < n) {
        double sum = red[0][threadIdx.x];
#pragma unroll
        for (int i = 1; i < kRedGroups; ++i) sum += red[i][threadIdx.x];
        const long long e = eb + threadIdx.x;
        out[e] = (float)((double)out[e] + sum);
    }
}

// ------------------------------------------------------------------ BN finalize (forward)
// One WAVE per channel (4 channels per 256-thread block): each lane sums a strided share of the
// channel's nb fp64 partials, then a fixed xor-butterfly over the 64 lanes -- no LDS tree and no
// block barriers (round 3's block-per-channel LDS tree took 5-9 us per launch, ~44 launches per
// PointNet++ step).  The summation order is fixed: bitwise reproducible.
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// The two fp64 partial sums of channel n over nb row blocks.  TPC threads per channel (the block's
// 256 threads cover 256 / TPC channels), sized so a thread holds <= 4 partials per array, all issued
// before the first add: the partials come from the producing kernel's blocks on every XCD and are
// read back from HBM / MALL, so each dependent round of loads costs a full memory latency -- one
// round instead of nb / 128 (round 5: the 1024-partial data-gradient finalizes took ~10 us).  Then
// a wave reduce and, for TPC > 64, an LDS reduce over the channel's waves.  Fixed order.
template <int TPC>
__device__ __forceinline__ void channel_sums(const double* __restrict__ part, int nb, int N, int n, double& S1,
                                             double& S2) {
    constexpr int WPC = TPC / 64;                     // waves per channel (TPC = 64, 128, 256)
    __shared__ double red[2][4];
    const int r = threadIdx.x % TPC, w = (threadIdx.x / 64) % WPC;
    const bool ok = n < N;
    const double* p1 = part + (size_t)(ok ? n : 0) * nb;
    const double* p2 = part + ((size_t)N + (ok ? n : 0)) * nb;
    double a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = r + u * TPC;
        a[u] = ok && i < nb ? p1[i] : 0.0;
        b[u] = ok && i < nb ? p2[i] : 0.0;
    }
    for (int i = r + 4 * TPC; ok && i < nb; i += TPC) {
        a[0] += p1[i];
        b[0] += p2[i];
    }
    double x = wave_sum_f64((a[0] + a[1]) + (a[2] + a[3]));
    double y = wave_sum_f64((b[0] + b[1]) + (b[2] + b[3]));
    if constexpr (WPC > 1) {
        const int cb = (threadIdx.x / TPC) * WPC;     // this channel's wave slots
        if ((threadIdx.x & 63) == 0) {
            red[0][cb + w] = x;
            red[1][cb + w] = y;
        }
        __syncthreads();
        x = red[0][cb];
        y = red[1][cb];
#pragma unroll
        for (int k = 1; k < WPC; ++k) {
            x += red[0][cb + k];
            y += red[1][cb + k];
        }
    }
    S1 = x;
    S2 = y;
}

// threads per channel of a finalize over nb partials (<= 4 loads per array and thread up to 1024)
static int finalize_tpc(int nb) { return nb <= 256 ? 64 : (nb <= 512 ? 128 : 256); }

template <int TPC>
__global__ __launch_bounds__(256) void bn_finalize_kernel(const double* __restrict__ part, int nb, int N, long long M,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps, float momentum,
                                                          float* __restrict__ run_mean, float* __restrict__ run_var,
                                                          float* __restrict__ s, float* __restrict__ t,
                                                          float* __restrict__ mean_out, float* __restrict__ inv_out,
                                                          long long* __restrict__ nbt) {
    const int n = blockIdx.x * (256 / TPC) + threadIdx.x / TPC;
    double S1, S2;
    channel_sums<TPC>(part, nb, N, n, S1, S2);
    if (n < N && threadIdx.x % TPC == 0) {
        if (nbt && n == 0) nbt[0] += 1;         // BatchNorm.num_batches_tracked
        const double mean = S1 / (double)M;
        double var = S2 / (double)M - mean * mean;
        if (var < 0.0) var = 0.0;
        const float invstd = (float)(1.0 / sqrt(var + (double)eps));
        const float g = gamma ? gamma[n] : 1.f;
        const float bb = beta ? beta[n] : 0.f;
        const float sc = g * invstd;
        s[n] = sc;
        t[n] = bb - (float)mean * sc;
        mean_out[n] = (float)mean;
        inv_out[n] = invstd;
        if (run_mean) {
            const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
            run_mean[n] = (float)((1.0 - momentum) * run_mean[n] + momentum * mean);
            run_var[n] = (float)((1.0 - momentum) * run_var[n] + momentum * unbiased);
        }
    }
}

// ------------------------------------------------------------------ BN finalize (backward)
// sums (sum dy, sum dy*xhat) -> dgamma, dbeta (added when `accum`) and the dZ coefficients
// kB = s*sum_dy/M, kC = s*sum_dyx/M; TPC threads per channel as above
template <int TPC>
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const double* __restrict__ part, int nb, int N,
                                                              long long M, const float* __restrict__ s,
                                                              const float* __restrict__ inv,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              float* __restrict__ kB, float* __restrict__ kC,
                                                              int accum) {
    const int n = blockIdx.x * (256 / TPC) + threadIdx.x / TPC;
    double S1, S2;
    channel_sums<TPC>(part, nb, N, n, S1, S2);
    if (n < N && threadIdx.x % TPC == 0) {
        if (dbeta) dbeta[n] = accum ? dbeta[n] + (float)S1 : (float)S1;
        if (dgamma) dgamma[n] = accum ? dgamma[n] + (float)S2 : (float)S2;
        kB[n] = (float)((double)s[n] * S1 / (double)M);
        kC[n] = (float)((double)s[n] * S2 / (double)M * (inv ? (double)inv[n] : 1.0));
    }
}

// ------------------------------------------------------------------ elementwise helpers (float4 over channels)
// All engine tensors have N % 4 == 0, row stride == N (dense) unless stated; one
// thread owns one float4 of channels (c4) in one row.
struct F4 {
    float v[4];
};
__device__ __forceinline__ F4 ld4(const float* p) {
    const float4 q = *reinterpret_cast<const float4*>(p);
    return F4{{q.x, q.y, q.z, q.w}};
}
__device__ __forceinline__ void st4(float* p, const F4& a) {
    *reinterpret_cast<float4*>(p) = make_float4(a.v[0], a.v[1], a.v[2], a.v[3]);
}

// ------------------------------------------------------------------ column reduce of (dy, dy*xhat)
// standalone BN-backward reduce when dA comes from outside the engine.  Block =
// 256 threads = (N/4 channel quads) x (rows in flight); partial [blockIdx.x][2][N].
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const float* __restrict__ dA, int ldd,
                                                            const float* __restrict__ Z, int ldz, int M, int N,
                                                            const float* __restrict__ s, const float* __restrict__ t,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ inv, int act, float slope,
                                                            int rows_per_block, double* __restrict__ part,
                                                            DropMask dm) {
    extern __shared__ double red_dyn[];   // [2][256][4]
    const int nq = N / 4;                 // channel quads; blockIdx.y walks 256-quad column tiles
    const int q0 = blockIdx.y * 256;
    const int tq = threadIdx.x % min(nq - q0, 256);
    const int rstep = 256 / min(nq - q0, 256);
    const int rlane = threadIdx.x / min(nq - q0, 256);
    const int c = 4 * (q0 + tq);
    double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
    const int rb = blockIdx.x * rows_per_block;
    const int re = min(M, rb + rows_per_block);
    if (rlane < rstep) {
        float sc[4], tc[4], mc[4], ic[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) { sc[j] = s[c + j]; tc[j] = t[c + j]; mc[j] = mean[c + j]; ic[j] = inv[c + j]; }
        // U rows per trip, all their loads issued before the first add (one row per trip kept
        // ~1 row of loads in flight per wave: ~3.2 TB/s on DGCNN's M x 512 reduces); the sums
        // still run row by row in the same order, so the partials are unchanged
        constexpr int U = 4;
        auto row = [&](int r, const F4& z, F4 g) {
            if (dm.on) {
#pragma unroll
                for (int j = 0; j < 4; ++j) g.v[j] = dm.apply(g.v[j], (unsigned long long)r * N + c + j);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float dy = g.v[j] * dact_f(z.v[j] * sc[j] + tc[j], act, slope);
                a[j] += (double)dy;
                b[j] += (double)dy * (double)((z.v[j] - mc[j]) * ic[j]);
            }
        };
        int r = rb + rlane;
        for (; r + (U - 1) * rstep < re; r += U * rstep) {
            F4 z[U], g[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                z[u] = ld4(Z + (size_t)(r + u * rstep) * ldz + c);
                g[u] = ld4(dA + (size_t)(r + u * rstep) * ldd + c);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) row(r + u * rstep, z[u], g[u]);
        }
        for (; r < re; r += rstep) row(r, ld4(Z + (size_t)r * ldz + c), ld4(dA + (size_t)r * ldd + c));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        red_dyn[(0 * 256 + threadIdx.x) * 4 + j] = a[j];
        red_dyn[(1 * 256 + threadIdx.x) * 4 + j] = b[j];
    }
    __syncthreads();
    if (rlane == 0) {
        for (int rr = 1; rr < rstep; ++rr) {
            const int o = rr * min(nq - q0, 256) + tq;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                a[j] += red_dyn[(0 * 256 + o) * 4 + j];
                b[j] += red_dyn[(1 * 256 + o) * 4 + j];
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            part[(size_t)(c + j) * gridDim.x + blockIdx.x] = a[j];
            part[((size_t)N + c + j) * gridDim.x + blockIdx.x] = b[j];
        }
    }
}

// ------------------------------------------------------------------ pooling over K with BN + act
// pooled[g][c] = max_k act(z*s+t) (first max), argmax u8, from the one extreme per channel the
// producer kept (the max of z where gamma >= 0, the min where gamma < 0: sign(s) = sign(gamma))
__global__ __launch_bounds__(256) void pool_finalize_kernel(const float* __restrict__ pz,
                                                            const unsigned char* __restrict__ pa, long long GN, int N,
                                                            const float* __restrict__ s, const float* __restrict__ t,
                                                            float slope, float* __restrict__ out,
                                                            unsigned char* __restrict__ arg, float* __restrict__ out2,
                                                            int ld2) {
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < GN; e += (long long)gridDim.x * 256) {
        const int c = (int)(e % N);
        const float sc = s[c], tc = t[c];
        const float v = act_f(pz[e] * sc + tc, 0, slope);
        out[e] = v;
        if (out2) out2[(e / N) * ld2 + c] = v;
        arg[e] = sc == 0.f ? (unsigned char)0 : pa[e];
    }
}

// the same, one channel quad per thread (N % 4 == 0, 16-B aligned pz / out, 4-B aligned pa / arg):
// 16-B loads and stores and 32-bit quad indexing instead of a 64-bit modulo per element
__global__ __launch_bounds__(256) void pool_finalize_q_kernel(const float4* __restrict__ pz,
                                                              const uchar4* __restrict__ pa, int GN4, int nq,
                                                              const float* __restrict__ s, const float* __restrict__ t,
                                                              float slope, float4* __restrict__ out,
                                                              uchar4* __restrict__ arg, float* __restrict__ out2,
                                                              int ld2) {
    for (int e = blockIdx.x * 256 + threadIdx.x; e < GN4; e += gridDim.x * 256) {
        const int g = e / nq, c = 4 * (e - g * nq);
        const float4 sc = *reinterpret_cast<const float4*>(s + c), tc = *reinterpret_cast<const float4*>(t + c);
        const float4 z = pz[e];
        const uchar4 a = pa[e];
        const float4 v = make_float4(act_f(z.x * sc.x + tc.x, 0, slope), act_f(z.y * sc.y + tc.y, 0, slope),
                                     act_f(z.z * sc.z + tc.z, 0, slope), act_f(z.w * sc.w + tc.w, 0, slope));
        out[e] = v;
        if (out2) *reinterpret_cast<float4*>(out2 + (size_t)g * ld2 + c) = v;
        arg[e] = make_uchar4(sc.x == 0.f ? 0 : a.x, sc.y == 0.f ? 0 : a.y, sc.z == 0.f ? 0 : a.z,
                             sc.w == 0.f ? 0 : a.w);
    }
}

__global__ __launch_bounds__(256) void pool_fwd_kernel(const float* __restrict__ Z, int nq, int G, int K,
                                                       const float* __restrict__ s, const float* __restrict__ t,
                                                       int act, float slope, float* __restrict__ out,
                                                       unsigned char* __restrict__ arg) {
    const int N = 4 * nq;
    const int total4 = G * nq;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < total4; e += gridDim.x * 256) {
        const int g = e / nq;
        const int c = 4 * (e - g * nq);
        float sc[4], tc[4], m[4];
        int a[4] = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 4; ++j) { sc[j] = s[c + j]; tc[j] = t[c + j]; }
        const float* z = Z + (size_t)g * K * N + c;
        {
            const F4 v = ld4(z);
#pragma unroll
            for (int j = 0; j < 4; ++j) m[j] = act_f(v.v[j] * sc[j] + tc[j], act, slope);
        }
        for (int k = 1; k < K; ++k) {
            const F4 v = ld4(z + (size_t)k * N);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float y = act_f(v.v[j] * sc[j] + tc[j], act, slope);
                if (y > m[j]) { m[j] = y; a[j] = k; }
            }
        }
        st4(out + (size_t)g * N + c, F4{{m[0], m[1], m[2], m[3]}});
        *reinterpret_cast<uchar4*>(arg + (size_t)g * N + c) =
            make_uchar4((unsigned char)a[0], (unsigned char)a[1], (unsigned char)a[2], (unsigned char)a[3]);
    }
}

// BN-backward sums for a pooled layer: only the argmax row of each (g, c) carries dy
__global__ __launch_bounds__(256) void pool_bwd_reduce_kernel(const float* __restrict__ dpool,
                                                              const unsigned char* __restrict__ arg,
                                                              const float* __restrict__ Z, int N, int G, int K,
                                                              const float* __restrict__ s,
                                                              const float* __restrict__ t,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ inv, int act, float slope,
                                                              int groups_per_block, double* __restrict__ part) {
    __shared__ double r1[4][64], r2[4][64];
    const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
    const int col = blockIdx.y * 64 + lane;
    const int gb = blockIdx.x * groups_per_block;
    const int ge = min(G, gb + groups_per_block);
    double a = 0.0, b = 0.0;
    if (col < N) {
        const float sc = s[col], tc = t[col], mc = mean[col], ic = inv[col];
#pragma unroll 4
        for (int g = gb + ph; g < ge; g += 4) {
            const int k = arg[(size_t)g * N + col];
            const float z = Z[((size_t)g * K + k) * N + col];
            const float dy = dpool[(size_t)g * N + col] * dact_f(z * sc + tc, act, slope);
            a += (double)dy;
            b += (double)dy * (double)((z - mc) * ic);
        }
    }
    r1[ph][lane] = a;
    r2[ph][lane] = b;
    __syncthreads();
    if (ph == 0 && col < N) {
        part[(size_t)col * gridDim.x + blockIdx.x] = r1[0][lane] + r1[1][lane] + r1[2][lane] + r1[3][lane];
        part[((size_t)N + col) * gridDim.x + blockIdx.x] = r2[0][lane] + r2[1][lane] + r2[2][lane] + r2[3][lane];
    }
}

// a = act(z*s + t) materialised (outputs consumed outside the engine)
__global__ __launch_bounds__(256) void bn_act_kernel(const float* __restrict__ Z, int ldz, int total4, int nq,
                                                     const float* __restrict__ s, const float* __restrict__ t,
                                                     int act, float slope, float* __restrict__ out, int ldo) {
    for (int e = blockIdx.x * 256 + threadIdx.x; e < total4; e += gridDim.x * 256) {
        const int r = e / nq;
        const int c = 4 * (e - r * nq);
        const F4 z = ld4(Z + (size_t)r * ldz + c);
        const F4 sv = ld4(s + c), tv = ld4(t + c);          // one quad load each (c % 4 == 0)
        F4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o.v[j] = act_f(z.v[j] * sv.v[j] + tv.v[j], act, slope);
        st4(out + (size_t)r * ldo + c, o);
    }
}


// bn_act with the training-mode dropout that follows it fused in (no mask stored)
__global__ __launch_bounds__(256) void bn_act_drop_kernel(const float* __restrict__ Z, int ldz, int total4, int nq,
                                                          const float* __restrict__ s, const float* __restrict__ t,
                                                          int act, float slope, float* __restrict__ out, int ldo,
                                                          unsigned long long seed, unsigned thr, float scale) {
    for (int e = blockIdx.x * 256 + threadIdx.x; e < total4; e += gridDim.x * 256) {
        const int r = e / nq;
        const int c = 4 * (e - r * nq);
        const F4 z = ld4(Z + (size_t)r * ldz + c);
        const F4 sv = ld4(s + c), tv = ld4(t + c);
        const unsigned long long i0 = (unsigned long long)r * (4ull * nq) + c;
        F4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float a = act_f(z.v[j] * sv.v[j] + tv.v[j], act, slope);
            o.v[j] = dropout_keep(seed, i0 + j, thr) ? a * scale : 0.f;
        }
        st4(out + (size_t)r * ldo + c, o);
    }
}

__global__ __launch_bounds__(256) void dropout_bwd_kernel(const float* __restrict__ g, int ldg, int total4, int nq,
                                                          float* __restrict__ gi, int ldi, unsigned long long seed,
                                                          unsigned thr, float scale) {
    for (int e = blockIdx.x * 256 + threadIdx.x; e < total4; e += gridDim.x * 256) {
        const int r = e / nq;
        const int c = 4 * (e - r * nq);
        const F4 v = ld4(g + (size_t)r * ldg + c);
        const unsigned long long i0 = (unsigned long long)r * (4ull * nq) + c;
        F4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o.v[j] = dropout_keep(seed, i0 + j, thr) ? v.v[j] * scale : 0.f;
        st4(gi + (size_t)r * ldi + c, o);
    }
}

static unsigned dropout_thr(double p) {
    const double v = p * 4294967296.0;
    return v >= 4294967295.0 ? 4294967295u : (unsigned)v;
}

DropMask drop_mask(double p, long long seed) {
    DropMask d{};
    d.seed = (unsigned long long)seed;
    d.thr = dropout_thr(p);
    d.scale = (float)(1.0 / (1.0 - p));
    d.on = 1;
    return d;
}

void bn_finalize_launch(const double* part, int nb, int N, long long M, const float* gamma, const float* beta,
                        float eps, float momentum, float* run_mean, float* run_var, float* s, float* t, float* mean,
                        float* invstd, long long* nbt, hipStream_t st) {
    const int tpc = finalize_tpc(nb);
    const dim3 grid((N + 256 / tpc - 1) / (256 / tpc));
#define PCS_FIN(T) hipLaunchKernelGGL(bn_finalize_kernel<T>, grid, dim3(256), 0, st, part, nb, N, M, gamma, beta, eps, \
                                      momentum, run_mean, run_var, s, t, mean, invstd, nbt)
    if (tpc == 64) PCS_FIN(64);
    else if (tpc == 128) PCS_FIN(128);
    else PCS_FIN(256);
#undef PCS_FIN
}

void bn_bwd_finalize_launch(const double* part, int nb, int N, long long M, const float* s, const float* inv,
                            float* dgamma, float* dbeta, float* kB, float* kC, int accum, hipStream_t st) {
    const int tpc = finalize_tpc(nb);
    const dim3 grid((N + 256 / tpc - 1) / (256 / tpc));
#define PCS_FIN(T) hipLaunchKernelGGL(bn_bwd_finalize_kernel<T>, grid, dim3(256), 0, st, part, nb, N, M, s, inv, dgamma, \
                                      dbeta, kB, kC, accum)
    if (tpc == 64) PCS_FIN(64);
    else if (tpc == 128) PCS_FIN(128);
    else PCS_FIN(256);
#undef PCS_FIN
}

static inline unsigned ew_grid(long long total) {
    long long g = (total + 255) / 256;
    if (g > 8192) g = 8192;
    return (unsigned)(g < 1 ? 1 : g);
}

template <int BM, int BN, int WM, int WN>
static void launch_gemm(const GemmArgs& g, int gx, bool bt, hipStream_t s) {
    const dim3 grid(gx, (g.N + BN - 1) / BN);
    const int e = (g.stats ? EPI_STATS : 0) | (g.bstats ? EPI_BWD : 0) | (g.pool_k ? EPI_POOL : 0);
#define PCS_GEMM(AMODE, BTV, EPIV) \
    hipLaunchKernelGGL((gemm_rows_kernel<BM, BN, WM, WN, AMODE, BTV, EPIV>), grid, dim3(WM * WN * 64), 0, s, g)
    if (bt) {   // data-gradient GEMMs: dZ operand (rebuilt on load) or a plain / materialised one
        switch (g.a.mode) {
#define PCS_BT(AMODE) \
    if (e == 0) PCS_GEMM(AMODE, true, 0); \
    else if (e == EPI_BWD) PCS_GEMM(AMODE, true, EPI_BWD); \
    else PCS_GEMM(AMODE, true, EPI_GENERIC);
        case OP_PLAIN: PCS_BT(OP_PLAIN) break;
        case OP_BNBWD: PCS_BT(OP_BNBWD) break;
        default: PCS_BT(OP_POOLBWD) break;
#undef PCS_BT
        }
        return;
    }
#define PCS_FWD(AMODE) \
    if (e == 0) PCS_GEMM(AMODE, false, 0); \
    else if (e == EPI_STATS) PCS_GEMM(AMODE, false, EPI_STATS); \
    else if (e == (EPI_STATS | EPI_POOL)) PCS_GEMM(AMODE, false, EPI_STATS | EPI_POOL); \
    else PCS_GEMM(AMODE, false, EPI_GENERIC);
    switch (g.a.mode) {
    case OP_PLAIN: PCS_FWD(OP_PLAIN) break;
    case OP_BNACT: PCS_FWD(OP_BNACT) break;
    case OP_BNBWD:
        if (e == 0) PCS_GEMM(OP_BNBWD, false, 0);
        else PCS_GEMM(OP_BNBWD, false, EPI_GENERIC);
        break;
    default:
        if (e == 0) PCS_GEMM(OP_POOLBWD, false, 0);
        else PCS_GEMM(OP_POOLBWD, false, EPI_GENERIC);
        break;
    }
#undef PCS_FWD
#undef PCS_GEMM
}

// the EPI template argument launch_gemm picks for these arguments (mirrors it)
static int gemm_epi(int mode, bool bt, bool stats, bool bstats, bool pool) {
    const int e = (stats ? EPI_STATS : 0) | (bstats ? EPI_BWD : 0) | (pool ? EPI_POOL : 0);
    if (bt) return (e == 0 || e == EPI_BWD) ? e : EPI_GENERIC;
    if (mode == OP_PLAIN || mode == OP_BNACT)
        return (e == 0 || e == EPI_STATS || e == (EPI_STATS | EPI_POOL)) ? e : EPI_GENERIC;
    return e == 0 ? 0 : EPI_GENERIC;
}

template <int BO, int BI, int XM>
static void launch_wgrad_y(dim3 grid, hipStream_t st, const Operand& x, int N, const Operand& y, int K, int M,
                           int rows, float* part, float* pdb) {
    // thin tiles keep two slabs of loads in flight, wide tiles one
    constexpr int NS = BO <= 64 && BI <= 64 ? 2 : 1;
    if (y.mode == OP_BNACT)
        hipLaunchKernelGGL((wgrad_kernel<BO, BI, XM, OP_BNACT, NS>), grid, dim3(256), 0, st, x, N, y, K, M, rows, part,
                           pdb);
    else
        hipLaunchKernelGGL((wgrad_kernel<BO, BI, XM, OP_PLAIN, NS>), grid, dim3(256), 0, st, x, N, y, K, M, rows, part,
                           pdb);
}

template <int BO, int BI>
static void launch_wgrad(dim3 grid, hipStream_t st, const Operand& x, int N, const Operand& y, int K, int M, int rows,
                         float* part, float* pdb) {
    switch (x.mode) {
    case OP_PLAIN: launch_wgrad_y<BO, BI, OP_PLAIN>(grid, st, x, N, y, K, M, rows, part, pdb); break;
    case OP_BNBWD: launch_wgrad_y<BO, BI, OP_BNBWD>(grid, st, x, N, y, K, M, rows, part, pdb); break;
    default: launch_wgrad_y<BO, BI, OP_POOLBWD>(grid, st, x, N, y, K, M, rows, part, pdb); break;
    }
}

}  // namespace pcs

using namespace pcs;

// row-GEMM tile (BM x BN) for M rows and N outputs: the largest tile that still
// gives >= 2 blocks per CU (256 CUs), else the one with the most blocks
// bwd: the data-gradient GEMM (k-major W, or an A rebuilt from dZ: BNBWD / POOLBWD), with a
// heavier operand transform and BN-backward epilogue; its tile policy is below
static void gemm_tile(int M, int N, bool bwd, int* bm, int* bn, int* nt = nullptr) {
    struct T { int bm, bn; };
    static const T big[] = {{128, 128}, {64, 128}, {64, 64}, {32, 128}};
    static const T mid[] = {{128, 64}, {64, 64}};
    static const T mid64[] = {{64, 64}, {128, 64}};
    // Data-gradient tiles by regime (same-box A/B, round 1; round 2 re-check: 64 x 128 on the
    // 128-wide PointNet++ layers, one A read instead of two, made the step 8 % slower): the thin, HBM-latency-bound
    // layers (PointNet++, EdgeConv) run best on 64 x 64 tiles (4 blocks per CU, more loads in
    // flight: PointNet++ step -1 %); the big MFMA-bound ones (DGCNN conv5-7: N >= 256 over
    // >= 64K rows) on the wide list despite its register pressure (DGCNN step -2 %).
    // Round 3 re-check: a 64 x 128 tile on EIGHT waves (512 threads, each wave the 32 x 32 block
    // of the 64 x 64 tile; the rebuilt dZ slab loaded and transformed once per 128 output columns
    // instead of once per 64) made the PointNet++ step 1-2 % slower (same-box A/B, 2 rounds).
    // Round 4: 32 x 128 tiles for the 128-wide data gradients (dZ read once, 4 waves across the
    // columns): 5.24 vs 5.07 ms.  Compiling the 64 x 64 tiles for 3 / 4 blocks per CU (168 / 128
    // VGPRs) spills: 5.31 / 5.61 vs 5.05 ms.  The BN-backward 64 x 64 data gradient now runs on
    // the LDS-DMA kernel of dgrad.hip (bitwise the same results).
    if (nt) *nt = 256;
    bool wide;
    const T* c;
    // (64 x 64 tiles first for the thin forward layers measured 4.62 vs 4.58 ms,
    // profiles/r05_ab_fwd_thin_tiles.txt)
    if (!bwd) {
        wide = N > 64;
        c = wide ? big : mid;
    } else {
        wide = N > 64 && N >= 256 && M >= 65536;
        c = wide ? big : mid64;
    }
    const int nc = wide ? 4 : 2;
    if (N <= 32) { *bm = 128; *bn = 32; return; }
    long long best = -1;
    for (int i = 0; i < nc; ++i) {
        const long long blocks = (long long)((M + c[i].bm - 1) / c[i].bm) * ((N + c[i].bn - 1) / c[i].bn);
        if (blocks >= 512) { *bm = c[i].bm; *bn = c[i].bn; return; }
        if (blocks > best) { best = blocks; *bm = c[i].bm; *bn = c[i].bn; }
    }
}

// Persistent grid of the row GEMM: as many row blocks per column tile as fit on the chip
// at once (LDS-limited blocks per CU x 256 CUs), each walking its row tiles with the next
// tile's first slab prefetched under the current tile's epilogue.
static int gemm_grid_x(int M, int N, int bm, int bn, int nt = 256) {
    const int mtiles = (M + bm - 1) / bm;
    const int lds = 4 * (bm + bn) * 2 * GLDK + 16 * bn;         // As + Bs + red (bytes)
    int per_cu = (160 * 1024) / lds;
    const int cap = 4;
    (void)nt;
    per_cu = per_cu < 1 ? 1 : (per_cu > cap ? cap : per_cu);
    const int ntiles = (N + bn - 1) / bn;
    const int slots = (256 * per_cu + ntiles - 1) / ntiles;
    if (mtiles <= slots) return mtiles;
    const int tpb = (mtiles + slots - 1) / slots;
    return (mtiles + tpb - 1) / tpb;
}

// wave grid of a row-GEMM tile (mirrors the launch table in pcs_gemm_rows)
static void gemm_waves(int bm, int bn, int nt, int* wm, int* wn) {
    (void)nt;
    if (bn == 32 || (bm == 128 && bn == 64)) { *wm = 4; *wn = 1; }
    else if (bm == 32) { *wm = 1; *wn = 4; }
    else { *wm = 2; *wn = 2; }
}

// algorithmic HBM bytes of reading operand o over M rows x K channels (SURVEY.md 8(d) model)
static double operand_bytes(const pcs_operand& o, int M, int K) {
    if (o.mode == PCS_OP_POOLBWD) return 4.0 * M * K + 5.0 * (double)(M / o.pool_k) * K;   // z + dpool + argmax
    return 4.0 * M * K * (o.mode == PCS_OP_BNBWD ? 2 : 1);
}

// number of row blocks the row GEMM uses for M rows and N outputs (sizes the stats workspace)
// Forward GEMMs in the wide regime (gemm_nt_regime) write one BN partial per 256-row tile,
// whichever kernel runs them (gemm_nt, or the row GEMM with that many persistent blocks when
// the operand needs an on-load transform), so the partial count depends on (M, N) only.
static int row_blocks(int M, int N, bool bwd) {
    if (!bwd && gemm_nt_regime(M, N)) return gemm_nt_row_tiles(M);
    int bm, bn, nt;
    gemm_tile(M, N, bwd, &bm, &bn, &nt);
    return gemm_grid_x(M, N, bm, bn, nt);
}

PCS_API int pcs_gemm_row_blocks(int M, int N) { return row_blocks(M, N, false); }

PCS_API int pcs_gemm_row_blocks_dgrad(int M, int N) { return row_blocks(M, N, true); }

static int check_operand(const pcs_operand* o, int K, const char* who, const char* which) {
    PCS_CHECK_ARG(o && o->data, "%s: %s operand missing", who, which);
    PCS_CHECK_ARG(o->mode >= PCS_OP_PLAIN && o->mode <= PCS_OP_POOLBWD, "%s: %s mode %d", who, which, o->mode);
    PCS_CHECK_ARG(o->ld % 4 == 0 && o->ld >= K, "%s: %s ld=%d must be a multiple of 4 and >= %d", who, which, o->ld,
                  K);
    PCS_CHECK_ARG(o->mode < PCS_OP_BNACT || (o->s && o->t && K % 4 == 0),
                  "%s: %s needs s/t and K %% 4 == 0 (K=%d)", who, which, K);
    PCS_CHECK_ARG(o->mode < PCS_OP_BNBWD || (o->z && o->ldz % 4 == 0 && o->ldz >= K && o->mean && o->alpha && o->kb),
                  "%s: %s needs z/ldz/mean/alpha/kb", who, which);
    PCS_CHECK_ARG(o->mode != PCS_OP_POOLBWD || (o->arg && o->pool_k >= 1 && o->pool_k <= 256),
                  "%s: %s needs arg and 1 <= pool_k <= 256", who, which);
    return 0;
}

Operand pcs::to_dev_operand(const pcs_operand* o, int rows, int cols) {
    Operand r{};
    if (!o) return r;
    r.rows = rows; r.cols = cols;
    r.data = o->data; r.ld = o->ld; r.mode = o->mode;
    r.s = o->s; r.t = o->t; r.act = o->act; r.slope = eff_slope(o->act, o->slope);
    r.z = o->z; r.ldz = o->ldz;
    r.mean = o->mean; r.inv = o->inv; r.alpha = o->alpha; r.kb = o->kb;
    r.arg = o->arg; r.pool_k = o->pool_k;
    return r;
}

static Operand to_dev(const pcs_operand* o, int rows, int cols) { return to_dev_operand(o, rows, cols); }

void pcs::wgrad_reduce_launch(const float* part, int splits, long long nk, float* dW, const float* pdb, int N,
                              float* db, hipStream_t st) {
    const long long blocks = (nk + kRedElems - 1) / kRedElems + (db ? (N + kRedElems - 1) / kRedElems : 0);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, part, splits, nk, dW, pdb, N, db);
}

// dZ (M x C, row stride ldo) = the BNBWD / POOLBWD transform of operand o, materialised: the
// same load_quad / load_raw / xform4 the GEMM loaders apply, so the values are bitwise those
// the GEMMs would rebuild on load.  Wide layers read dZ once per column tile of their data /
// weight gradient; for ceil(Cin / 128) >= 3 one pass here is cheaper than rebuilding it in
// every tile (DGCNN conv5-7: -2.1 ms of GEMM time for +0.5 ms here, scripts/dgcnn_head_ab.py).
template <int MODE>
__global__ __launch_bounds__(256) void dz_kernel(Operand o, int total4, int nq, float* __restrict__ out, int ldo,
                                                 DropMask dm) {
    const int C = 4 * nq;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < total4; e += gridDim.x * 256) {
        const int r = e / nq;
        const int c = 4 * (e - r * nq);
        Quad q;
        load_quad<MODE>(o, c, C, q);
        float4 v, z;
        unsigned a = 0;
        load_raw<MODE>(o, r, c, v, z, a);
        if (dm.on) {                 // the stack's fused dropout, on the top layer's output gradient
            const unsigned long long i0 = (unsigned long long)r * C + c;
            v.x = dm.apply(v.x, i0);
            v.y = dm.apply(v.y, i0 + 1);
            v.z = dm.apply(v.z, i0 + 2);
            v.w = dm.apply(v.w, i0 + 3);
        }
        *reinterpret_cast<float4*>(out + (size_t)r * ldo + c) = xform4<MODE>(o, v, z, a, r, q, c, C);
    }
}

int pcs::materialize_dz(const pcs_operand* x, int M, int C, float* out, int ldo, hipStream_t st, double drop_p,
                        long long drop_seed) {
    PCS_CHECK_ARG(x && (x->mode == PCS_OP_BNBWD || x->mode == PCS_OP_POOLBWD) && C % 4 == 0 && ldo % 4 == 0 &&
                      ldo >= C && out,
                  "materialize_dz: needs a BNBWD/POOLBWD operand, C %% 4 == 0, ldo >= C");
    const long long total4 = (long long)M * (C / 4);
    PCS_CHECK_ARG(total4 < (1ll << 31), "materialize_dz: too many elements");
    if (total4 == 0) return 0;
    const Operand o = to_dev(x, M, C);
    if (x->mode == PCS_OP_BNBWD)
        hipLaunchKernelGGL(dz_kernel<OP_BNBWD>, dim3(ew_grid(total4)), dim3(256), 0, st, o, (int)total4, C / 4, out,
                           ldo, drop_p > 0.0 ? drop_mask(drop_p, drop_seed) : DropMask{});
    else
        hipLaunchKernelGGL(dz_kernel<OP_POOLBWD>, dim3(ew_grid(total4)), dim3(256), 0, st, o, (int)total4, C / 4, out,
                           ldo, DropMask{});
    return launch_status("materialize_dz");
}

// C = T(A) . W^T (+bias), W row-major N x K (row stride ldw).
// stats (nullable): [2][N][row_blocks] fp64 partial (sum, sumsq) of C.
// bstats (nullable): fused BN-backward partials of the layer whose pre-BN output is epi->z (same shape as C):
//   [2][N][row_blocks] of (sum dy, sum dy*xhat), dy = C * act'(z*s+t), xhat = (z-mean)*inv.
// bt = 0: W row-major N x K (B[k][n] = W[n*ldw + k]); bt = 1: W row-major K x N
// (B[k][n] = W[k*ldw + n], ldw >= N) -- the data-gradient GEMM on the layer's own weights.
int pcs::gemm_rows_ex(const pcs_operand* a, int M, int K, const float* W, int ldw, int bt, const float* bias, float* C,
                 int ldc, int N, double* stats, const pcs_operand* epi, double* bstats, void* stream, float* pz,
                 unsigned char* pa, int pool_k, const float* psign) {
    PCS_CHECK_ARG(pool_k == 0 || ((pool_k == 16 || pool_k == 32) && M % pool_k == 0 && pz && pa && !bt),
                  "pcs_gemm_rows: fused pooling needs pool_k 16|32 dividing M and pz/pa");
    PCS_CHECK_ARG(M >= 0 && K >= 1 && N >= 1, "pcs_gemm_rows: bad sizes M=%d K=%d N=%d", M, K, N);
    if (int e = check_operand(a, K, "pcs_gemm_rows", "A")) return e;
    PCS_CHECK_ARG(W && C, "pcs_gemm_rows: null pointer");
    PCS_CHECK_ARG(!(stats && bstats), "pcs_gemm_rows: stats and bstats are exclusive");
    PCS_CHECK_ARG(!bstats || (epi && epi->z && epi->s && epi->t && epi->mean && epi->inv),
                  "pcs_gemm_rows: bstats needs epi z/s/t/mean/inv");
    PCS_CHECK_ARG(ldw >= (bt ? N : K), "pcs_gemm_rows: ldw=%d must be >= %d", ldw, bt ? N : K);
    PCS_CHECK_ARG(!bt || a->mode != PCS_OP_BNACT, "pcs_gemm_rows: k-major W needs a PLAIN/BNBWD/POOLBWD A");
    // the epilogue addresses a 32-row block of C / epi Z with 32-bit offsets
    PCS_CHECK_ARG((long long)ldc * 32 + N < (1ll << 31) && (!epi || (long long)epi->ldz * 32 + N < (1ll << 31)),
                  "pcs_gemm_rows: row stride too large (ldc=%d)", ldc);
    if (M == 0) return 0;
    hipStream_t s = as_stream(stream);
    // plain operands of a wide layer, no fused epilogue but BN statistics: the LDS-DMA wide GEMM
    if (!bt && a->mode == PCS_OP_PLAIN && !pool_k && !bstats && gemm_nt_ok(a->data, a->ld, W, ldw, M, N, K)) {
        int probe = -1;
        if (probe_enabled()) {
            char nm[96];
            const bool b256 = gemm_nt_bn(N) == 256;
            snprintf(nm, sizeof nm, "pcs::gemm_nt_kernel<%d, %d, %d, %s>", b256 ? 256 : 128, b256 ? 2 : 4,
                     b256 ? 4 : 2, stats ? "true" : "false");
            const pcs_operand ac = *a;
            probe = probe_start(nm, 2.0 * M * K * N, 4.0 * M * K + 4.0 * M * N, s, [=]() {
                gemm_rows_ex(&ac, M, K, W, ldw, 0, bias, C, ldc, N, stats, nullptr, nullptr, stream);
            });
        }
        const int e = gemm_nt(a->data, a->ld, W, ldw, M, N, K, bias, C, ldc, stats, s);
        probe_stop(probe, s);
        return e;
    }
    // the forward GEMM of an inner layer (K % 32 == 0, PLAIN or BNACT A) over > 64 outputs and
    // >= 8192 rows: LDS-DMA ring kernel (fwd_dma.hip) with the row GEMM's epilogue, one BN partial
    // per row_blocks() block.  Measured in-step on PointNet++ (round 5): 64 -> 128 pooled 114 -> 77 us,
    // 128 -> 128 35 -> 31, 128 -> 256 pooled 80 -> 61, 256 -> 512 pooled 67 -> 55, FP1-3 -5..-8 us
    // per layer; the thin ones stay on the row GEMM (32 -> 32 over 1 M rows: 54 vs 117 us, 32 -> 64
    // pooled 102 vs 128, 64 -> 64 38 vs 42: one slab per 64-row tile, two barriers and an in-place
    // transform pass per slab are not hidden), as do small M (FP4, 2048 rows: 34 vs 37 us).
    // Variant 1 (pcs_gemm_rows_variant) takes the DMA kernel wherever it is legal (tests).
    const int fv = dgrad_forced_variant();
    if (!bt && !bstats && fv >= 0 && (fv >= 1 || (N > 64 && M >= 8192)) &&
        fwd_dma_ok(a, M, K, W, ldw, N, pool_k, bias)) {
        const int gx = row_blocks(M, N, false);
        int probe = -1;
        if (probe_enabled()) {
            const pcs_operand ac = *a;
            probe = probe_start(fwd_dma_name(a->mode == PCS_OP_BNACT, stats != nullptr, pool_k != 0, N),
                                2.0 * M * K * N, operand_bytes(*a, M, K) + 4.0 * M * N * (pool_k ? 0 : 1) +
                                (pool_k ? 5.0 * (double)(M / pool_k) * N + 4.0 * M * N : 0.0), s, [=]() {
                                    gemm_rows_ex(&ac, M, K, W, ldw, 0, bias, C, ldc, N, stats, nullptr, nullptr,
                                                 stream, pz, pa, pool_k, psign);
                                });
        }
        const int e = fwd_dma(a, M, K, W, ldw, bias, C, ldc, N, stats, gx, pz, pa, pool_k, psign, s);
        probe_stop(probe, s);
        if (e) return e;
        return launch_status("pcs_gemm_rows");
    }
    // the 64 x 64 data gradient (BN-backward, pooled BN-backward or plain dZ operand): LDS-DMA ring
    // kernel (dgrad.hip), bitwise the same (pcs_gemm_rows_kmajor_variant(-1) forces the row GEMM)
    if (bt && a->mode != PCS_OP_BNACT && !stats && !pool_k && !bias && dgrad_forced_variant() >= 0 &&
        dgrad_dma_ok(a, M, K, W, ldw, N)) {
        int bm, bn;
        gemm_tile(M, N, true, &bm, &bn);
        if (bm == 64 && bn == 64) {
            const int gx = bstats ? row_blocks(M, N, true) : gemm_grid_x(M, N, 64, 64);
            int probe = -1;
            if (probe_enabled()) {
                const double bytes = operand_bytes(*a, M, K) + 4.0 * M * N * (bstats ? 2 : 1);
                const pcs_operand ac = *a, ec = epi ? *epi : pcs_operand{};
                const bool he = epi != nullptr;
                probe = probe_start(dgrad_dma_name(bstats != nullptr, a->mode, N), 2.0 * M * K * N,
                                    bytes, s, [=]() {
                                        gemm_rows_ex(&ac, M, K, W, ldw, bt, bias, C, ldc, N, stats, he ? &ec : nullptr,
                                                     bstats, stream);
                                    });
            }
            const int e = dgrad_dma(a, M, K, W, ldw, C, ldc, N, epi, bstats, gx, s);
            probe_stop(probe, s);
            if (e) return e;
            return launch_status("pcs_gemm_rows");
        }
    }
    GemmArgs g{to_dev(a, M, K), M, K, W, ldw, bias, C, ldc, N, stats, to_dev(epi, M, N), bstats, pz, pa, pool_k, psign};
    int probe = -1;
    if (probe_enabled()) {
        char nm[96];
        int bm, bn, nt, wm, wn;
        gemm_tile(M, N, a->mode >= PCS_OP_BNBWD || bt, &bm, &bn, &nt);
        gemm_waves(bm, bn, nt, &wm, &wn);
        snprintf(nm, sizeof nm, "pcs::gemm_rows_kernel<%d, %d, %d, %d, %d, %s, %d>", bm, bn, wm, wn, a->mode,
                 bt ? "true" : "false", gemm_epi(a->mode, bt != 0, stats != nullptr, bstats != nullptr, pool_k != 0));
        const double bytes = operand_bytes(*a, M, K) + 4.0 * M * N * (bstats ? 2 : 1);
        const pcs_operand ac = *a, ec = epi ? *epi : pcs_operand{};
        const bool he = epi != nullptr;
        probe = probe_start(nm, 2.0 * M * K * N, bytes, s, [=]() {
            gemm_rows_ex(&ac, M, K, W, ldw, bt, bias, C, ldc, N, stats, he ? &ec : nullptr, bstats, stream);
        });
    }
    int bm, bn, nt;
    const bool bwd = a->mode >= PCS_OP_BNBWD || bt;
    gemm_tile(M, N, bwd, &bm, &bn, &nt);
    // stats partials: one per row block as row_blocks() counts them (<= the row tiles: persistent)
    const int gx = (stats || bstats) ? row_blocks(M, N, bwd) : gemm_grid_x(M, N, bm, bn, nt);
    const bool b = bt != 0;
    if (bn == 32) launch_gemm<128, 32, 4, 1>(g, gx, b, s);
    else if (bm == 128 && bn == 64) launch_gemm<128, 64, 4, 1>(g, gx, b, s);
    else if (bm == 128) launch_gemm<128, 128, 2, 2>(g, gx, b, s);
    else if (bm == 64 && bn == 128) launch_gemm<64, 128, 2, 2>(g, gx, b, s);
    else if (bm == 64) launch_gemm<64, 64, 2, 2>(g, gx, b, s);
    else launch_gemm<32, 128, 1, 4>(g, gx, b, s);
    probe_stop(probe, s);
    return launch_status("pcs_gemm_rows");
}

PCS_API int pcs_gemm_rows(const pcs_operand* a, int M, int K, const float* W, int ldw, const float* bias, float* C,
                          int ldc, int N, double* stats, const pcs_operand* epi, double* bstats, void* stream) {
    return gemm_rows_ex(a, M, K, W, ldw, 0, bias, C, ldc, N, stats, epi, bstats, stream);
}

PCS_API int pcs_gemm_rows_kmajor(const pcs_operand* a, int M, int K, const float* W, int ldw, float* C, int ldc,
                                 int N, const pcs_operand* epi, double* bstats, void* stream) {
    return gemm_rows_ex(a, M, K, W, ldw, 1, nullptr, C, ldc, N, nullptr, epi, bstats, stream);
}

PCS_API int pcs_gemm_rows_variant(const pcs_operand* a, int M, int K, const float* W, int ldw, const float* bias,
                                  float* C, int ldc, int N, double* stats, int variant, void* stream) {
    PCS_CHECK_ARG(variant >= -1 && variant <= 1, "pcs_gemm_rows_variant: variant=%d", variant);
    const int prev = dgrad_forced_variant();     // restored, not reset (an earlier pcs_set_kernel_variant holds)
    dgrad_force_variant(variant);
    const int e = gemm_rows_ex(a, M, K, W, ldw, 0, bias, C, ldc, N, stats, nullptr, nullptr, stream);
    dgrad_force_variant(prev);
    return e;
}

PCS_API int pcs_set_kernel_variant(int variant) {
    PCS_CHECK_ARG(variant == -1 || variant == 0, "pcs_set_kernel_variant: variant=%d", variant);
    dgrad_force_variant(variant);
    return 0;
}

PCS_API int pcs_gemm_rows_kmajor_variant(const pcs_operand* a, int M, int K, const float* W, int ldw, float* C,
                                         int ldc, int N, const pcs_operand* epi, double* bstats, int variant,
                                         void* stream) {
    PCS_CHECK_ARG(variant >= -1 && variant <= 3, "pcs_gemm_rows_kmajor_variant: variant=%d", variant);
    const int prev = dgrad_forced_variant();
    dgrad_force_variant(variant);
    const int e = gemm_rows_ex(a, M, K, W, ldw, 1, nullptr, C, ldc, N, nullptr, epi, bstats, stream);
    dgrad_force_variant(prev);
    return e;
}

// wgrad tile (BO x BI) and its row split for N x K over M rows: ~1024 blocks, 2048 for the big
// MFMA-bound contractions (>= 16 GFLOP, e.g. DGCNN conv5-7: step -1 %, round 1).  Round 2
// re-checked 256 / 512 / 1024 blocks with the partial-tile reduce: within +-8 % per shape,
// no consistent winner (scripts/gemm_bench.py).
static void wgrad_plan(int N, int K, int M, int* BO, int* BI, int* splits, int* rows) {
    *BO = N > 64 ? 128 : 64;
    *BI = K > 64 ? 128 : 64;
    const int tiles = ((N + *BO - 1) / *BO) * ((K + *BI - 1) / *BI);
    // (512 / 256 blocks for the smaller ones measured +0.3 / +0.8 % on DGCNN, round 3)
    // (round 4, in-step: 512 / 2048 blocks for the smaller ones were within noise of 1024 on both
    // models -- shorter lane blocks did not free CUs for the critical path's small kernels sooner)
    const int target = 2.0 * M * N * K >= 1.6e10 ? 2048 : 1024;
    int sp = (target + tiles - 1) / tiles;
    // the partial tiles (sp x N x K floats, written once and read once by the reduce) stay
    // below half the operands' bytes M x (N + K), as long as >= 512 blocks remain
    const long long cap = std::max<long long>((512 + tiles - 1) / tiles, (long long)M * (N + K) / (2LL * N * K));
    if (sp > cap) sp = (int)cap;
    int r = (M + sp - 1) / sp;
    r = ((r + 255) / 256) * 256;
    if (r < 256) r = 256;
    *rows = r;
    *splits = (M + r - 1) / r;
}

// Column passes over a layer's dZ (M x C rows; cin = its input width) by its backward
// GEMMs: the data gradient (M x cin output) re-reads dZ once per column tile, the weight
// gradient (C x cin) once per cin tile.
int pcs::dz_passes(int M, int C, int cin, bool dgrad, bool wgrad) {
    int n = 0;
    if (dgrad) {
        int bm, bn, nt;
        gemm_tile(M, cin, true, &bm, &bn, &nt);
        n += (cin + bn - 1) / bn;
    }
    if (wgrad) {
        int BO, BI, sp, rows;
        wgrad_plan(C, cin, M, &BO, &BI, &sp, &rows);
        n += (cin + BI - 1) / BI;
    }
    return n;
}

size_t pcs::wgrad_ws_bytes(int N, int K, int M) {
    if (M <= 0) return 0;
    int BO, BI, sp, rows;
    wgrad_plan(N, K, M, &BO, &BI, &sp, &rows);
    const size_t b = (size_t)sp * ((size_t)N * K + N) * sizeof(float) + 256;
    // the wide kernel (plain operands) may take the launch: size for either
    return std::max(b, wgrad_nt_ws_bytes(N, K, M));
}

// dW (N x K) += T(X)^T . T(Y) over M rows; db (N) += column sums of T(X) (nullable).  Each row
// split's partial goes to the workspace, then one reduce per output adds the splits in order.
int pcs::wgrad_launch(const pcs_operand* x, int N, const pcs_operand* y, int K, int M, float* dW, float* db, void* ws,
                      size_t ws_bytes, void* stream) {
    PCS_CHECK_ARG(M >= 0 && N >= 1 && K >= 1, "pcs_wgrad: bad sizes");
    if (int e = check_operand(x, N, "pcs_wgrad", "X")) return e;
    if (int e = check_operand(y, K, "pcs_wgrad", "Y")) return e;
    PCS_CHECK_ARG(x->mode != PCS_OP_BNACT, "pcs_wgrad: X operand cannot be BNACT");
    PCS_CHECK_ARG(y->mode <= PCS_OP_BNACT, "pcs_wgrad: Y operand must be PLAIN or BNACT");
    PCS_CHECK_ARG(dW && N % 4 == 0, "pcs_wgrad: dW null or N not a multiple of 4");
    if (M == 0) return 0;
    const size_t need = wgrad_ws_bytes(N, K, M);
    PCS_CHECK_ARG(ws && ws_bytes >= need, "pcs_wgrad: workspace too small (%zu < %zu)", ws_bytes, need);
    float* part = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
    hipStream_t st = as_stream(stream);
    if (x->mode == PCS_OP_PLAIN && y->mode == PCS_OP_PLAIN && !db && wgrad_nt_ok(x->data, x->ld, y->data, y->ld, M, N, K)) {
        // a wide layer's materialised dZ and plain input: the LDS-DMA wide weight gradient
        int probe = -1;
        if (probe_enabled()) {
            const float *xd = x->data, *yd = y->data;
            const int lx = x->ld, ly = y->ld;
            probe = probe_start(wgrad_nt_name(N, K, M), 2.0 * M * N * K, 4.0 * M * (N + K), st,
                                [=]() { wgrad_nt(xd, lx, yd, ly, M, N, K, part, st); });
        }
        const int sp = wgrad_nt(x->data, x->ld, y->data, y->ld, M, N, K, part, st);
        probe_stop(probe, st);
        const long long nk = (long long)N * K;
        hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((nk + kRedElems - 1) / kRedElems)), dim3(256), 0, st,
                           part, sp, nk, dW, (const float*)nullptr, N, (float*)nullptr);
        return launch_status("pcs_wgrad");
    }
    int BO, BI, splits, rows;
    wgrad_plan(N, K, M, &BO, &BI, &splits, &rows);
    float* pdb = db ? part + (size_t)splits * N * K : nullptr;
    const int tiles = ((N + BO - 1) / BO) * ((K + BI - 1) / BI);
    const dim3 grid(splits, tiles);
    const Operand xd = to_dev(x, M, N), yd = to_dev(y, M, K);
    // the partial-tile launch alone (the probe's replay rewrites only the workspace)
    auto tiles_launch = [=]() {
        if (BO == 128 && BI == 128) launch_wgrad<128, 128>(grid, st, xd, N, yd, K, M, rows, part, pdb);
        else if (BO == 128) launch_wgrad<128, 64>(grid, st, xd, N, yd, K, M, rows, part, pdb);
        else if (BI == 128) launch_wgrad<64, 128>(grid, st, xd, N, yd, K, M, rows, part, pdb);
        else launch_wgrad<64, 64>(grid, st, xd, N, yd, K, M, rows, part, pdb);
    };
    int probe = -1;
    if (probe_enabled()) {
        char nm[96];
        snprintf(nm, sizeof nm, "pcs::wgrad_kernel<%d, %d, %d, %d, %d>", BO, BI, x->mode, y->mode,
                 BO <= 64 && BI <= 64 ? 2 : 1);
        probe = probe_start(nm, 2.0 * M * N * K, operand_bytes(*x, M, N) + operand_bytes(*y, M, K), st,
                            tiles_launch);
    }
    tiles_launch();
    probe_stop(probe, st);
    const long long nk = (long long)N * K;
    const long long blocks = (nk + kRedElems - 1) / kRedElems + (db ? (N + kRedElems - 1) / kRedElems : 0);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, part, splits, nk, dW, pdb, N, db);
    return launch_status("pcs_wgrad");
}

PCS_API int pcs_wgrad_workspace(int N, int K, int M, size_t* bytes) {
    PCS_CHECK_ARG(bytes && N >= 1 && K >= 1 && M >= 0, "pcs_wgrad_workspace: bad arguments");
    *bytes = wgrad_ws_bytes(N, K, M);
    return 0;
}

PCS_API int pcs_wgrad(const pcs_operand* x, int N, const pcs_operand* y, int K, int M, float* dW, float* db,
                      void* workspace, size_t ws_bytes, void* stream) {
    return wgrad_launch(x, N, y, K, M, dW, db, workspace, ws_bytes, stream);
}

// BN forward finalize: part [2][N][nb] -> s, t, mean, invstd; running stats updated in place (nullable).
PCS_API int pcs_bn_finalize(const double* part, int nb, int N, long long M, const float* gamma, const float* beta,
                            float eps, float momentum, float* run_mean, float* run_var, float* s, float* t,
                            float* mean, float* invstd, void* stream) {
    PCS_CHECK_ARG(nb >= 1 && N >= 1 && M >= 1, "pcs_bn_finalize: bad sizes");
    bn_finalize_launch(part, nb, N, M, gamma, beta, eps, momentum, run_mean, run_var, s, t, mean, invstd, nullptr,
                       as_stream(stream));
    return launch_status("pcs_bn_finalize");
}

// BN backward finalize: part [2][N][nb] of (sum dy, sum dy*xhat) -> dgamma, dbeta (+= when accum), kB, kC.
PCS_API int pcs_bn_bwd_finalize(const double* part, int nb, int N, long long M, const float* s, const float* invstd,
                                float* dgamma, float* dbeta, float* kB, float* kC, int accum, void* stream) {
    PCS_CHECK_ARG(nb >= 1 && N >= 1 && M >= 1, "pcs_bn_bwd_finalize: bad sizes");
    bn_bwd_finalize_launch(part, nb, N, M, s, invstd, dgamma, dbeta, kB, kC, accum, as_stream(stream));
    return launch_status("pcs_bn_bwd_finalize");
}

static const int kRedRows = 256;

PCS_API int pcs_bn_bwd_reduce_blocks(int M) { return (M + kRedRows - 1) / kRedRows; }

PCS_API int pcs_bn_bwd_reduce(const float* dA, int ldd, const float* Z, int ldz, int M, int N, const float* s,
                              const float* t, const float* mean, const float* inv, int act, float slope, double* part,
                              void* stream) {
    PCS_CHECK_ARG(M >= 1 && N >= 4 && N % 4 == 0 && ldd % 4 == 0 && ldz % 4 == 0,
                  "pcs_bn_bwd_reduce: bad sizes (N, strides must be multiples of 4)");
    const int nq = N / 4;
    const dim3 grid((M + kRedRows - 1) / kRedRows, (nq + 255) / 256);
    hipLaunchKernelGGL(bn_bwd_reduce_kernel, grid, dim3(256), 2 * 256 * 4 * sizeof(double), as_stream(stream), dA, ldd,
                       Z, ldz, M, N, s, t, mean, inv, act, eff_slope(act, slope), kRedRows, part, DropMask{});
    return launch_status("pcs_bn_bwd_reduce");
}

// the same with the stack's fused dropout applied to dA on load (its mask recomputed from the seed)
int pcs::bn_bwd_reduce_dropout(const float* dA, int ldd, const float* Z, int ldz, int M, int N, const float* s,
                               const float* t, const float* mean, const float* inv, int act, float slope,
                               double* part, double p, long long seed, hipStream_t st) {
    PCS_CHECK_ARG(M >= 1 && N >= 4 && N % 4 == 0 && ldd % 4 == 0 && ldz % 4 == 0 && p > 0.0 && p < 1.0,
                  "bn_bwd_reduce_dropout: bad sizes or p");
    const dim3 grid((M + kRedRows - 1) / kRedRows, (N / 4 + 255) / 256);
    hipLaunchKernelGGL(bn_bwd_reduce_kernel, grid, dim3(256), 2 * 256 * 4 * sizeof(double), st, dA, ldd, Z, ldz, M, N,
                       s, t, mean, inv, act, eff_slope(act, slope), kRedRows, part, drop_mask(p, seed));
    return launch_status("bn_bwd_reduce_dropout");
}

PCS_API int pcs_pool_fwd(const float* Z, int N, long long G, int K, const float* s, const float* t, int act,
                         float slope, float* out, uint8_t* arg, void* stream) {
    PCS_CHECK_ARG(G >= 0 && K >= 1 && K <= 256 && N >= 4 && N % 4 == 0, "pcs_pool_fwd: bad sizes");
    const long long total = G * N / 4;
    PCS_CHECK_ARG(G * K * (long long)N < (1ll << 40) && total < (1ll << 31), "pcs_pool_fwd: too many elements");
    if (total == 0) return 0;
    hipLaunchKernelGGL(pool_fwd_kernel, dim3(ew_grid(total)), dim3(256), 0, as_stream(stream), Z, N / 4, (int)G, K, s,
                       t, act, eff_slope(act, slope), out, arg);
    return launch_status("pcs_pool_fwd");
}

int pcs::pool_finalize(const float* pz, const unsigned char* pa, long long G, int N, const float* s, const float* t,
                       int act, float slope, float* out, unsigned char* arg, hipStream_t st, float* out2,
                       int ld2) {
    const long long GN = G * N;
    if (GN == 0) return 0;
    PCS_CHECK_ARG(!out2 || ld2 >= N, "pool_finalize: second output stride %d < %d channels", ld2, N);
    auto al = [](const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; };
    if (N % 4 == 0 && GN / 4 < (1ll << 31) && al(pz, 16) && al(out, 16) && al(pa, 4) && al(arg, 4) && al(s, 16) &&
        al(t, 16) && (!out2 || (al(out2, 16) && ld2 % 4 == 0))) {
        const long long GN4 = GN / 4;
        const unsigned blocks = (unsigned)std::min<long long>((GN4 + 255) / 256, 8192);
        hipLaunchKernelGGL(pool_finalize_q_kernel, dim3(blocks), dim3(256), 0, st, reinterpret_cast<const float4*>(pz),
                           reinterpret_cast<const uchar4*>(pa), (int)GN4, N / 4, s, t, eff_slope(act, slope),
                           reinterpret_cast<float4*>(out), reinterpret_cast<uchar4*>(arg), out2, ld2);
        return launch_status("pool_finalize");
    }
    long long blocks = (GN + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(pool_finalize_kernel, dim3((unsigned)blocks), dim3(256), 0, st, pz, pa, GN, N, s, t,
                       eff_slope(act, slope), out, arg, out2, ld2);
    return launch_status("pool_finalize");
}

PCS_API int pcs_pool_bwd_reduce_blocks(long long G) { return (int)((G + 63) / 64); }

PCS_API int pcs_pool_bwd_reduce(const float* dpool, const uint8_t* arg, const float* Z, int N, long long G, int K,
                                const float* s, const float* t, const float* mean, const float* inv, int act,
                                float slope, double* part, void* stream) {
    PCS_CHECK_ARG(G >= 1 && G < (1ll << 31) && K >= 1 && N >= 1, "pcs_pool_bwd_reduce: bad sizes");
    const int gpb = 64;
    const dim3 grid((unsigned)((G + gpb - 1) / gpb), (N + 63) / 64);
    hipLaunchKernelGGL(pool_bwd_reduce_kernel, grid, dim3(256), 0, as_stream(stream), dpool, arg, Z, N, (int)G, K, s,
                       t, mean, inv, act, eff_slope(act, slope), gpb, part);
    return launch_status("pcs_pool_bwd_reduce");
}

int pcs::bn_act_dropout(const float* Z, int ldz, int M, int N, const float* s, const float* t, int act, float slope,
                        float* out, int ldo, double p, long long seed, hipStream_t st) {
    PCS_CHECK_ARG(M >= 0 && N >= 4 && N % 4 == 0 && ldz % 4 == 0 && ldo % 4 == 0 && p > 0.0 && p < 1.0,
                  "bn_act_dropout: bad sizes or p=%g", p);
    const long long total = (long long)M * N / 4;
    PCS_CHECK_ARG(total < (1ll << 31), "bn_act_dropout: too many elements");
    if (total == 0) return 0;
    hipLaunchKernelGGL(bn_act_drop_kernel, dim3(ew_grid(total)), dim3(256), 0, st, Z, ldz, (int)total, N / 4, s, t, act,
                       eff_slope(act, slope), out, ldo, (unsigned long long)seed, dropout_thr(p),
                       (float)(1.0 / (1.0 - p)));
    return launch_status("bn_act_dropout");
}

PCS_API int pcs_dropout_bwd(const float* gout, int ldg, int M, int N, double p, int64_t seed, float* gin, int ldi,
                            void* stream) {
    PCS_CHECK_ARG(M >= 0 && N >= 4 && N % 4 == 0 && ldg % 4 == 0 && ldi % 4 == 0 && p > 0.0 && p < 1.0,
                  "pcs_dropout_bwd: bad sizes or p=%g", p);
    PCS_CHECK_ARG(gout && gin, "pcs_dropout_bwd: null pointer");
    const long long total = (long long)M * N / 4;
    PCS_CHECK_ARG(total < (1ll << 31), "pcs_dropout_bwd: too many elements");
    if (total == 0) return 0;
    hipLaunchKernelGGL(dropout_bwd_kernel, dim3(ew_grid(total)), dim3(256), 0, as_stream(stream), gout, ldg, (int)total,
                       N / 4, gin, ldi, (unsigned long long)seed, dropout_thr(p), (float)(1.0 / (1.0 - p)));
    return launch_status("pcs_dropout_bwd");
}

__global__ __launch_bounds__(256) void copy_cols_kernel(const float* __restrict__ src, int lds, int total4, int nq,
                                                       float* __restrict__ dst, int ldd) {
    for (int e = blockIdx.x * 256 + threadIdx.x; e < total4; e += gridDim.x * 256) {
        const int r = e / nq;
        const int c = 4 * (e - r * nq);
        st4(dst + (size_t)r * ldd + c, ld4(src + (size_t)r * lds + c));
    }
}

PCS_API int pcs_copy_cols(const float* src, int lds, int M, int C, float* dst, int ldd, void* stream) {
    PCS_CHECK_ARG(M >= 0 && C >= 4 && C % 4 == 0 && lds % 4 == 0 && ldd % 4 == 0 && lds >= C && ldd >= C,
                  "pcs_copy_cols: bad sizes M=%d C=%d lds=%d ldd=%d", M, C, lds, ldd);
    PCS_CHECK_ARG(src && dst && (reinterpret_cast<uintptr_t>(src) & 15) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0,
                  "pcs_copy_cols: null or unaligned pointer");
    const long long total = (long long)M * C / 4;
    PCS_CHECK_ARG(total < (1ll << 31), "pcs_copy_cols: too many elements");
    if (total == 0) return 0;
    hipLaunchKernelGGL(copy_cols_kernel, dim3(ew_grid(total)), dim3(256), 0, as_stream(stream), src, lds, (int)total,
                       C / 4, dst, ldd);
    return launch_status("pcs_copy_cols");
}

PCS_API int pcs_bn_act(const float* Z, int ldz, int M, int N, const float* s, const float* t, int act, float slope,
                       float* out, int ldo, void* stream) {
    PCS_CHECK_ARG(M >= 0 && N >= 4 && N % 4 == 0 && ldz % 4 == 0 && ldo % 4 == 0, "pcs_bn_act: bad sizes");
    const long long total = (long long)M * N / 4;
    PCS_CHECK_ARG(total < (1ll << 31), "pcs_bn_act: too many elements");
    if (total == 0) return 0;
    hipLaunchKernelGGL(bn_act_kernel, dim3(ew_grid(total)), dim3(256), 0, as_stream(stream), Z, ldz, (int)total, N / 4,
                       s, t, act, eff_slope(act, slope), out, ldo);
    return launch_status("pcs_bn_act");
}
