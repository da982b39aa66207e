// LDS-free engine GEMMs for fp32 MFMA (v_mfma_f32_32x32x2_f32) on gfx950.
//
// Why LDS-free: one f32 MFMA takes 64 cycles and consumes ONE A and ONE B value per
// lane, so the operand bandwidth a wave needs is tiny and every fragment can come
// straight from global memory (L1/L2) into VGPRs.  Dropping the LDS staging removes
// the LDS round trip, every __syncthreads of the main loop and the LDS-imposed
// occupancy limit; latency is hidden by a 2-stage register pipeline (the next slab's
// loads are in flight under the current slab's MFMAs) and by 2 waves per SIMD.
//
//  * gemm_direct_kernel  (row GEMM, forward and data-gradient, same contract as
//    gemm_rows_kernel in mlp.hip): each wave owns a (32*TM) x (32*TN) tile of C.  A
//    slab is 16 k deep and lane half h holds k = k0 + 8h + e (e = 0..7) -- two
//    float4 per fragment row, read as 32 contiguous bytes of one row of A (or W).
//    MFMA step e pairs k0+e (h=0) with k0+8+e (h=1); the MFMA sums over that pair,
//    so the permutation only reorders the fp32 accumulation.  The per-channel
//    transform coefficients (BN scale/shift, BN-backward terms) are staged once per
//    block in LDS (read-only afterwards).
//  * wgrad_direct_kernel (dW += T(X)^T . T(Y) over rows, same contract as
//    wgrad_kernel): the reduction axis is the row index, so lane l32 reads ONE
//    channel of two consecutive rows (h) per MFMA -- 2 x 128 contiguous bytes per
//    load instruction, no transpose needed.  Each wave walks its own 16-row slabs;
//    partial tiles are flushed every 256 rows into an LDS fp32 tile (ds_add_f32)
//    and blocks combine with fp32 global atomics.
#include "mlp_common.hpp"

#include <stdlib.h>

namespace pcs {

__device__ __forceinline__ float f4e(const float4& v, int e) {
    return e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w));
}

constexpr int DBK = 16;

template <int TM, int TN, int WN, int AM>
__global__ __launch_bounds__(256, 2) void gemm_direct_kernel(GemmArgs g) {
    constexpr int WM = 4 / WN;
    constexpr int BM = WM * 32 * TM, BN = WN * 32 * TN;
    constexpr int NCO = AM == OP_PLAIN ? 0 : (AM == OP_BNACT ? 2 : 5);
    extern __shared__ float4 coef[];             // [NCO][kq]
    __shared__ double red[2][WM][BN];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int h = lane >> 5, l32 = lane & 31;
    const int mw = blockIdx.x * BM + wm * 32 * TM;
    const int nw = blockIdx.y * BN + wn * 32 * TN;
    const int K = g.K;
    const int kq = (K + 3) >> 2;

    if (NCO) {
        for (int e = tid; e < kq; e += 256) {
            coef[e] = reinterpret_cast<const float4*>(g.a.s)[e];
            coef[kq + e] = reinterpret_cast<const float4*>(g.a.t)[e];
            if (NCO == 5) {
                coef[2 * kq + e] = reinterpret_cast<const float4*>(g.a.mean)[e];
                coef[3 * kq + e] = reinterpret_cast<const float4*>(g.a.alpha)[e];
                coef[4 * kq + e] = reinterpret_cast<const float4*>(g.a.kb)[e];
            }
        }
        __syncthreads();
    }

    int rc[TM], nc[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) rc[i] = min(mw + 32 * i + l32, g.M - 1);
#pragma unroll
    for (int j = 0; j < TN; ++j) nc[j] = min(nw + 32 * j + l32, g.N - 1);
    const int lda_last = g.a.ld - 4, ldw_last = g.ldw - 4;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    float4 ra[2][TM][2], rz[2][TM][2], rb[2][TN][2];
    unsigned rg[2][TM][2];

    auto gload = [&](int st, int k0) {
#pragma unroll
        for (int hq = 0; hq < 2; ++hq) {
            const int c = k0 + 8 * h + 4 * hq;
            const int ca = min(c, lda_last), cw = min(c, ldw_last);
#pragma unroll
            for (int i = 0; i < TM; ++i) load_raw<AM>(g.a, rc[i], ca, ra[st][i][hq], rz[st][i][hq], rg[st][i][hq]);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                rb[st][j][hq] = *reinterpret_cast<const float4*>(g.W + (size_t)nc[j] * g.ldw + cw);
        }
    };
    auto compute = [&](int st, int k0) {
        float4 a[TM][2], b[TN][2];
#pragma unroll
        for (int hq = 0; hq < 2; ++hq) {
            const int c = k0 + 8 * h + 4 * hq;
            Quad q;
            if (NCO) {
                const int qi = min(c >> 2, kq - 1);
                q.s = coef[qi];
                q.t = coef[kq + qi];
                if (NCO == 5) {
                    q.mean = coef[2 * kq + qi];
                    q.alpha = coef[3 * kq + qi];
                    q.kb = coef[4 * kq + qi];
                }
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
                a[i][hq] = xform4<AM>(g.a, ra[st][i][hq], rz[st][i][hq], rg[st][i][hq], rc[i], q, c, K);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                float4 v = rb[st][j][hq];
                v.x = c + 0 < K ? v.x : 0.f;
                v.y = c + 1 < K ? v.y : 0.f;
                v.z = c + 2 < K ? v.z : 0.f;
                v.w = c + 3 < K ? v.w : 0.f;
                b[j][hq] = v;
            }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4e(a[i][e >> 2], e & 3), f4e(b[j][e >> 2], e & 3),
                                                                     acc[i][j], 0, 0, 0);
    };

    const int nk = (K + DBK - 1) / DBK;
    gload(0, 0);
    for (int ks = 0; ks < nk; ks += 2) {
        gload(1, (ks + 1) * DBK);      // clamped past the end: unconditional, no phi copies
        __builtin_amdgcn_sched_barrier(0);
        compute(0, ks * DBK);
        if (ks + 1 >= nk) break;
        __builtin_amdgcn_sched_barrier(0);
        gload(0, (ks + 2) * DBK);
        __builtin_amdgcn_sched_barrier(0);
        compute(1, (ks + 1) * DBK);
        __builtin_amdgcn_sched_barrier(0);
    }

    // ---- epilogue: bias, store, per-channel partial reductions (as gemm_rows_kernel)
    const bool want_stats = g.stats != nullptr;
    const bool want_b = g.bstats != nullptr;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int lc = wn * 32 * TN + j * 32 + l32;
        const int col = nw + j * 32 + l32;
        const bool cok = col < g.N;
        const float bv = (g.bias && cok) ? g.bias[col] : 0.f;
        float sp = 0.f, tp = 0.f, mp = 0.f, ip = 0.f;
        if (want_b && cok) { sp = g.e.s[col]; tp = g.e.t[col]; mp = g.e.mean[col]; ip = g.e.inv[col]; }
        double s1 = 0.0, s2 = 0.0;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = mw + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (row < g.M && cok) {
                    const float v = acc[i][j][r] + bv;
                    g.C[(size_t)row * g.ldc + col] = v;
                    if (want_stats) {
                        s1 += (double)v;
                        s2 += (double)v * (double)v;
                    }
                    if (want_b) {
                        const float z = g.e.z[(size_t)row * g.e.ldz + col];
                        const float dy = v * dact_f(z * sp + tp, g.e.act, g.e.slope);
                        const float xh = (z - mp) * ip;
                        s1 += (double)dy;
                        s2 += (double)dy * (double)xh;
                    }
                }
            }
        }
        if (want_stats || want_b) {
            s1 += __shfl_xor(s1, 32);
            s2 += __shfl_xor(s2, 32);
            if (lane < 32) {
                red[0][wm][lc] = s1;
                red[1][wm][lc] = s2;
            }
        }
    }
    if (want_stats || want_b) {
        __syncthreads();
        double* out = want_stats ? g.stats : g.bstats;
        for (int c = tid; c < BN; c += 256) {
            const int col = blockIdx.y * BN + c;
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
constexpr int WSLAB = 16;          // rows per slab (8 MFMA steps of 2 rows)
constexpr int WFLUSH = 16;         // slabs between flushes of the wave accumulators (256 rows)

template <int TM, int TN, int XM, int YM>
__global__ __launch_bounds__(256, 2) void wgrad_direct_kernel(Operand xo, int N, Operand yo, int K, int M,
                                                              int rows_per_block, float* __restrict__ dW,
                                                              float* __restrict__ db) {
    constexpr int BO = 32 * TM, BI = 32 * TN;
    __shared__ float tile[BO][BI + 1];
    __shared__ float dbs[4][2][BO];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    const int tiles_i = (K + BI - 1) / BI;
    const int n0 = (blockIdx.y / tiles_i) * BO;
    const int k0 = (blockIdx.y % tiles_i) * BI;
    const int rb = blockIdx.x * rows_per_block;
    const int re = min(M, rb + rows_per_block);
    const bool do_db = (db != nullptr) && (k0 == 0);

    for (int e = tid; e < BO * (BI + 1); e += 256) (&tile[0][0])[e] = 0.f;

    // this lane's fixed channels and their transform coefficients
    int xn[TM], yk[TN];
    bool xok[TM];
    float xs[TM], xt[TM], xm[TM], xa[TM], xk[TM], ys[TN], yt[TN], dbv[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int n = n0 + 32 * i + l32;
        xok[i] = n < N;
        xn[i] = min(n, N - 1);
        xs[i] = xt[i] = xm[i] = xa[i] = xk[i] = 0.f;
        if (XM >= OP_BNBWD) {
            xs[i] = xo.s[xn[i]]; xt[i] = xo.t[xn[i]]; xm[i] = xo.mean[xn[i]];
            xa[i] = xo.alpha[xn[i]]; xk[i] = xo.kb[xn[i]];
        }
        dbv[i] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        yk[j] = min(k0 + 32 * j + l32, K - 1);
        ys[j] = yt[j] = 0.f;
        if (YM == OP_BNACT) { ys[j] = yo.s[yk[j]]; yt[j] = yo.t[yk[j]]; }
    }

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    float rx[2][TM][8], rxz[2][TM][8], ry[2][TN][8];
    unsigned rxa[2][TM][8];
    auto gload = [&](int st, int r0) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int r = min(r0 + 2 * s + h, M - 1);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                if (XM == OP_POOLBWD) {
                    const int gg = r / xo.pool_k;
                    rx[st][i][s] = xo.data[(size_t)gg * xo.ld + xn[i]];
                    rxa[st][i][s] = xo.arg[(size_t)gg * xo.ld + xn[i]];
                } else {
                    rx[st][i][s] = xo.data[(size_t)r * xo.ld + xn[i]];
                }
                if (XM >= OP_BNBWD) rxz[st][i][s] = xo.z[(size_t)r * xo.ldz + xn[i]];
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) ry[st][j][s] = yo.data[(size_t)r * yo.ld + yk[j]];
        }
    };
    auto compute = [&](int st, int r0) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int r = r0 + 2 * s + h;
            const bool rok = r < re;
            float x[TM], y[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                float v = rx[st][i][s];
                if (XM == OP_POOLBWD) {
                    const int rr = min(r, M - 1);
                    const unsigned kk = (unsigned)(rr - (rr / xo.pool_k) * xo.pool_k);
                    v = rxa[st][i][s] == kk ? v : 0.f;
                }
                if (XM >= OP_BNBWD) {
                    const float z = rxz[st][i][s];
                    const float dy = v * dact_f(z * xs[i] + xt[i], xo.act, xo.slope);
                    v = xs[i] * dy - xk[i] - xa[i] * (z - xm[i]);
                }
                v = (rok && xok[i]) ? v : 0.f;
                x[i] = v;
                dbv[i] += v;
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const float v = ry[st][j][s];
                y[j] = YM == OP_BNACT ? act_f(v * ys[j] + yt[j], yo.act, yo.slope) : v;
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[i], y[j], acc[i][j], 0, 0, 0);
        }
    };
    auto flush = [&]() {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    atomicAdd(&tile[i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h][j * 32 + l32], acc[i][j][r]);
                    acc[i][j][r] = 0.f;
                }
    };
    __syncthreads();

    const int nslab = (re - rb + WSLAB - 1) / WSLAB;
    int done = 0;
    int sl = wave;
    if (sl < nslab) gload(0, rb + sl * WSLAB);
    for (; sl < nslab; sl += 8) {
        gload(1, rb + (sl + 4) * WSLAB);
        __builtin_amdgcn_sched_barrier(0);
        compute(0, rb + sl * WSLAB);
        if (++done == WFLUSH) { flush(); done = 0; }
        if (sl + 4 >= nslab) break;
        __builtin_amdgcn_sched_barrier(0);
        gload(0, rb + (sl + 8) * WSLAB);
        __builtin_amdgcn_sched_barrier(0);
        compute(1, rb + (sl + 4) * WSLAB);
        if (++done == WFLUSH) { flush(); done = 0; }
        __builtin_amdgcn_sched_barrier(0);
    }
    if (done) flush();
    if (do_db) {
#pragma unroll
        for (int i = 0; i < TM; ++i) dbs[wave][h][i * 32 + l32] = dbv[i];
    }
    __syncthreads();
    for (int e = tid; e < BO * BI; e += 256) {
        const int o = e / BI, c = e - o * BI;
        const int n = n0 + o, k = k0 + c;
        if (n < N && k < K) atomicAdd(&dW[(size_t)n * K + k], tile[o][c]);
    }
    if (do_db && tid < BO && n0 + tid < N) {
        float a = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) a += dbs[w][0][tid] + dbs[w][1][tid];
        atomicAdd(&db[n0 + tid], a);
    }
}

// ------------------------------------------------------------------ dispatch
struct DirectTile { int tm, tn, wn; };

// tile of the row GEMM for N outputs / M rows: the widest block (<= 256 columns, so A
// is read once for N <= 256) whose wave count still fills the chip twice over
static DirectTile direct_tile(int M, int N) {
    const int tn = N <= 32 ? 1 : 2;
    const int wn = N <= 64 ? 1 : (N <= 128 ? 2 : 4);
    const int bn = wn * 32 * tn;
    const long long ntile = (N + bn - 1) / bn;
    const long long waves2 = (long long)((M + (4 / wn) * 64 - 1) / ((4 / wn) * 64)) * ntile * 4;
    const int tm = waves2 >= 2048 ? 2 : 1;
    return DirectTile{tm, tn, wn};
}

void direct_gemm_name(int M, int N, int mode, char* buf, int cap) {
    const DirectTile t = direct_tile(M, N);
    snprintf(buf, cap, "pcs::gemm_direct_kernel<%d, %d, %d, %d>", t.tm, t.tn, t.wn, mode);
}

void direct_wgrad_name(int N, int K, int xm, int ym, char* buf, int cap) {
    snprintf(buf, cap, "pcs::wgrad_direct_kernel<%d, %d, %d, %d>", N <= 32 ? 1 : 2, K <= 32 ? 1 : 2, xm, ym);
}

int direct_row_blocks(int M, int N) {
    const DirectTile t = direct_tile(M, N);
    const int bm = (4 / t.wn) * 32 * t.tm;
    return (M + bm - 1) / bm;
}

template <int TM, int TN, int WN>
static void launch_direct(const GemmArgs& g, hipStream_t s) {
    constexpr int BM = (4 / WN) * 32 * TM, BN = WN * 32 * TN;
    const dim3 grid((g.M + BM - 1) / BM, (g.N + BN - 1) / BN);
    const int kq = (g.K + 3) / 4;
    switch (g.a.mode) {
    case OP_PLAIN: hipLaunchKernelGGL((gemm_direct_kernel<TM, TN, WN, OP_PLAIN>), grid, dim3(256), 0, s, g); break;
    case OP_BNACT:
        hipLaunchKernelGGL((gemm_direct_kernel<TM, TN, WN, OP_BNACT>), grid, dim3(256), 2 * kq * 16, s, g);
        break;
    case OP_BNBWD:
        hipLaunchKernelGGL((gemm_direct_kernel<TM, TN, WN, OP_BNBWD>), grid, dim3(256), 5 * kq * 16, s, g);
        break;
    default:
        hipLaunchKernelGGL((gemm_direct_kernel<TM, TN, WN, OP_POOLBWD>), grid, dim3(256), 5 * kq * 16, s, g);
        break;
    }
}

bool launch_gemm_direct(const GemmArgs& g, hipStream_t s) {
    if (g.a.mode != OP_PLAIN && g.K > 4096) return false;     // coefficient staging limit (80 KB)
    const DirectTile t = direct_tile(g.M, g.N);
#define PCS_DT(A, B, C) if (t.tm == A && t.tn == B && t.wn == C) { launch_direct<A, B, C>(g, s); return true; }
    PCS_DT(2, 1, 1) PCS_DT(1, 1, 1)
    PCS_DT(2, 2, 1) PCS_DT(1, 2, 1)
    PCS_DT(2, 2, 2) PCS_DT(1, 2, 2)
    PCS_DT(2, 2, 4) PCS_DT(1, 2, 4)
#undef PCS_DT
    return false;
}

template <int TM, int TN, int XM>
static void launch_wd_y(dim3 grid, hipStream_t st, const Operand& x, int N, const Operand& y, int K, int M, int rows,
                        float* dW, float* db) {
    if (y.mode == OP_BNACT)
        hipLaunchKernelGGL((wgrad_direct_kernel<TM, TN, XM, OP_BNACT>), grid, dim3(256), 0, st, x, N, y, K, M, rows, dW,
                           db);
    else
        hipLaunchKernelGGL((wgrad_direct_kernel<TM, TN, XM, OP_PLAIN>), grid, dim3(256), 0, st, x, N, y, K, M, rows, dW,
                           db);
}

template <int TM, int TN>
static void launch_wd(hipStream_t st, const Operand& x, int N, const Operand& y, int K, int M, float* dW, float* db) {
    const int tiles = ((N + 32 * TM - 1) / (32 * TM)) * ((K + 32 * TN - 1) / (32 * TN));
    int splits = (2048 + tiles - 1) / tiles;
    int rows = (M + splits - 1) / splits;
    rows = ((rows + 4 * WSLAB - 1) / (4 * WSLAB)) * (4 * WSLAB);
    if (rows < 4 * WSLAB) rows = 4 * WSLAB;
    splits = (M + rows - 1) / rows;
    const dim3 grid(splits, tiles);
    switch (x.mode) {
    case OP_PLAIN: launch_wd_y<TM, TN, OP_PLAIN>(grid, st, x, N, y, K, M, rows, dW, db); break;
    case OP_BNBWD: launch_wd_y<TM, TN, OP_BNBWD>(grid, st, x, N, y, K, M, rows, dW, db); break;
    default: launch_wd_y<TM, TN, OP_POOLBWD>(grid, st, x, N, y, K, M, rows, dW, db); break;
    }
}

bool launch_wgrad_direct(const Operand& x, int N, const Operand& y, int K, int M, float* dW, float* db,
                         hipStream_t s) {
    const int tm = N <= 32 ? 1 : 2, tn = K <= 32 ? 1 : 2;
    if (tm == 1 && tn == 1) launch_wd<1, 1>(s, x, N, y, K, M, dW, db);
    else if (tm == 1) launch_wd<1, 2>(s, x, N, y, K, M, dW, db);
    else if (tn == 1) launch_wd<2, 1>(s, x, N, y, K, M, dW, db);
    else launch_wd<2, 2>(s, x, N, y, K, M, dW, db);
    return true;
}

static int g_engine_impl = [] {
    const char* e = getenv("PCS_GEMM_IMPL");
    return (e && e[0] == '1') ? 1 : 0;
}();

int engine_impl() { return g_engine_impl; }

}  // namespace pcs

// Engine GEMM implementation: 0 = LDS-staged kernels (mlp.hip, default), 1 = LDS-free
// kernels.  Process-wide; set it only while no engine work is being enqueued.
PCS_API int pcs_engine_select(int impl) {
    using namespace pcs;
    PCS_CHECK_ARG(impl == 0 || impl == 1, "pcs_engine_select: impl must be 0 or 1");
    g_engine_impl = impl;
    return 0;
}
