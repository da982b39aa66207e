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
//    (dW = dZ^T . T(A_prev)) split over rows with fp32 atomics; dZ is
//    materialised once per layer by an elementwise kernel.
// Statistics are accumulated in fp64 (as ATen's CPU batch norm does).
#include "pcs_common.hpp"

namespace pcs {

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { ACT_RELU = 0, ACT_LRELU = 1, ACT_NONE = 2 };

__device__ __forceinline__ float act_f(float y, int act, float slope) {
    if (act == ACT_RELU) return y > 0.f ? y : 0.f;
    if (act == ACT_LRELU) return y > 0.f ? y : y * slope;
    return y;
}
// derivative as autograd computes it: relu -> (result > 0); leaky_relu -> (input > 0 ? 1 : slope)
__device__ __forceinline__ float dact_f(float y, int act, float slope) {
    if (act == ACT_RELU) return y > 0.f ? 1.f : 0.f;
    if (act == ACT_LRELU) return y > 0.f ? 1.f : slope;
    return 1.f;
}

struct GemmArgs {
    const float* A; int lda; int M; int K;     // A rows (M x K), row stride lda
    const float* s_in; const float* t_in;      // A transform: act(a*s+t) per K channel (or null)
    int act_in; float slope_in;
    const float* W; int ldw;                   // B[k][n] = W[n*ldw + k]
    const float* bias;                         // per n (or null)
    float* C; int ldc; int N;                  // output rows (M x N)
    double* stats;                             // [gridDim.x][2][N]: sum, sum of squares of C (or null)
    // fused backward reduce for the layer that produced A's *output* space (dgrad epilogue):
    const float* zp; int ldzp;                 // that layer's pre-BN Z (M x N)
    const float* sp; const float* tp; const float* meanp; const float* invp;
    int actp; float slopep;
    double* bstats;                            // [gridDim.x][2][N]: sum dy, sum dy*xhat (or null)
};

// ------------------------------------------------------------------ row GEMM
// C[M x N] = T(A)[M x K] . B[K x N],  B[k][n] = W[n*ldw + k]  (W row-major N x K).
//
// 256 threads = 4 waves in a WM x WN grid; each wave owns TM x TN 32x32 MFMA tiles.
// K is consumed in 32-deep slabs staged through a double-buffered LDS ring with the
// next slab's global loads in flight (registers) while the current slab is computed.
// Inside a slab the k order is permuted so that lane half h takes k = 16h + s
// (s = 0..15): each lane's A/B fragments are then 16 CONSECUTIVE floats of one LDS
// row, read with ds_read_b128; the 144-B row stride (BK + 4 floats) makes those
// reads bank-conflict free.  The MFMA sums over k, so the permutation only
// reorders the fp32 accumulation.
constexpr int GBK = 32;
constexpr int GLDK = GBK + 4;

template <int BM, int BN, int WM, int WN, bool AXF>
__global__ __launch_bounds__(256, 2) void gemm_rows_kernel(GemmArgs g) {
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int AV = BM * GBK / 4 / 256;
    constexpr int BV = (BN * GBK / 4 + 255) / 256;
    static_assert(WM * WN == 4 && TM >= 1 && TN >= 1, "tile");
    __shared__ __attribute__((aligned(16))) float As[2][BM][GLDK];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN][GLDK];
    __shared__ double red[2][WM][BN];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    const int h = lane >> 5, l32 = lane & 31;
    const bool wvec = (g.ldw & 3) == 0;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    float4 ra[AV], rb[BV];
    // every A float4 of this thread sits at the same k offset 4*(tid&7) of a slab, so one
    // (scale, shift) quad per slab serves all of them
    float4 rs = make_float4(0.f, 0.f, 0.f, 0.f), rt = rs;
    auto gload = [&](int k0) {
        if (AXF) {
            const int gk = k0 + 4 * (tid & 7);
            rs.x = gk + 0 < g.K ? g.s_in[gk + 0] : 0.f;
            rs.y = gk + 1 < g.K ? g.s_in[gk + 1] : 0.f;
            rs.z = gk + 2 < g.K ? g.s_in[gk + 2] : 0.f;
            rs.w = gk + 3 < g.K ? g.s_in[gk + 3] : 0.f;
            rt.x = gk + 0 < g.K ? g.t_in[gk + 0] : 0.f;
            rt.y = gk + 1 < g.K ? g.t_in[gk + 1] : 0.f;
            rt.z = gk + 2 < g.K ? g.t_in[gk + 2] : 0.f;
            rt.w = gk + 3 < g.K ? g.t_in[gk + 3] : 0.f;
        }
#pragma unroll
        for (int it = 0; it < AV; ++it) {
            const int e = it * 256 + tid;
            const int r = e >> 3, c4 = e & 7;
            const int gr = m0 + r, gk = k0 + 4 * c4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (gr < g.M && gk < g.K) v = *reinterpret_cast<const float4*>(g.A + (size_t)gr * g.lda + gk);
            ra[it] = v;
        }
#pragma unroll
        for (int it = 0; it < BV; ++it) {
            const int e = it * 256 + tid;
            const int n = e >> 3, c4 = e & 7;
            const int gn = n0 + n, gk = k0 + 4 * c4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (e < BN * GBK / 4 && gn < g.N && gk < g.K) {
                const float* w = g.W + (size_t)gn * g.ldw + gk;
                if (wvec && gk + 3 < g.K) v = *reinterpret_cast<const float4*>(w);
                else {
                    v.x = w[0];
                    v.y = gk + 1 < g.K ? w[1] : 0.f;
                    v.z = gk + 2 < g.K ? w[2] : 0.f;
                    v.w = gk + 3 < g.K ? w[3] : 0.f;
                }
            }
            rb[it] = v;
        }
    };
    auto sstore = [&](int buf, int k0) {
#pragma unroll
        for (int it = 0; it < AV; ++it) {
            const int e = it * 256 + tid;
            const int r = e >> 3, c4 = e & 7;
            const int gk = k0 + 4 * c4;
            float4 v = ra[it];
            if (AXF) {
                v.x = gk + 0 < g.K ? act_f(v.x * rs.x + rt.x, g.act_in, g.slope_in) : 0.f;
                v.y = gk + 1 < g.K ? act_f(v.y * rs.y + rt.y, g.act_in, g.slope_in) : 0.f;
                v.z = gk + 2 < g.K ? act_f(v.z * rs.z + rt.z, g.act_in, g.slope_in) : 0.f;
                v.w = gk + 3 < g.K ? act_f(v.w * rs.w + rt.w, g.act_in, g.slope_in) : 0.f;
            } else {
                v.y = gk + 1 < g.K ? v.y : 0.f;
                v.z = gk + 2 < g.K ? v.z : 0.f;
                v.w = gk + 3 < g.K ? v.w : 0.f;
            }
            *reinterpret_cast<float4*>(&As[buf][r][4 * c4]) = v;
        }
#pragma unroll
        for (int it = 0; it < BV; ++it) {
            const int e = it * 256 + tid;
            if (e < BN * GBK / 4) *reinterpret_cast<float4*>(&Bs[buf][e >> 3][4 * (e & 7)]) = rb[it];
        }
    };

    const int nk = (g.K + GBK - 1) / GBK;
    gload(0);
    sstore(0, 0);
    __syncthreads();
    for (int ks = 0; ks < nk; ++ks) {
        const int buf = ks & 1;
        if (ks + 1 < nk) gload((ks + 1) * GBK);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float4 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                a[i] = *reinterpret_cast<const float4*>(&As[buf][wm * WTM + i * 32 + l32][16 * h + 4 * q]);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                b[j] = *reinterpret_cast<const float4*>(&Bs[buf][wn * WTN + j * 32 + l32][16 * h + 4 * q]);
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
        if (ks + 1 < nk) sstore(buf ^ 1, (ks + 1) * GBK);
        __syncthreads();
    }

    // ---- epilogue: bias, store, per-channel partial reductions
    const bool want_stats = g.stats != nullptr;
    const bool want_b = g.bstats != nullptr;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int lc = wn * WTN + j * 32 + l32;
        const int col = n0 + lc;
        const bool cok = col < g.N;
        const float bv = (g.bias && cok) ? g.bias[col] : 0.f;
        float sp = 0.f, tp = 0.f, mp = 0.f, ip = 0.f;
        if (want_b && cok) { sp = g.sp[col]; tp = g.tp[col]; mp = g.meanp[col]; ip = g.invp[col]; }
        double s1 = 0.0, s2 = 0.0;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (row < g.M && cok) {
                    const float v = acc[i][j][r] + bv;
                    g.C[(size_t)row * g.ldc + col] = v;
                    if (want_stats) {
                        s1 += (double)v;
                        s2 += (double)v * (double)v;
                    }
                    if (want_b) {
                        const float z = g.zp[(size_t)row * g.ldzp + col];
                        const float dy = v * dact_f(z * sp + tp, g.actp, g.slopep);
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
            const int col = n0 + c;
            if (col < g.N) {
                double a = 0.0, b = 0.0;
#pragma unroll
                for (int w = 0; w < WM; ++w) { a += red[0][w][c]; b += red[1][w][c]; }
                out[((size_t)blockIdx.x * 2 + 0) * g.N + col] = a;
                out[((size_t)blockIdx.x * 2 + 1) * g.N + col] = b;
            }
        }
    }
}

// ------------------------------------------------------------------ weight gradient
// dW[n][k] += sum_r X[r][n] * T(Y)[r][k] ; db[n] += sum_r X[r][n]   (rows split over gridDim.x)
// Same LDS/fragment scheme as the row GEMM with the ROW index as the reduction
// axis: X and T(Y) slabs of 32 rows are stored transposed ([channel][row], 144-B
// stride) so each lane's fragment is 16 consecutive rows.  fp32 partial sums are
// flushed every 8 slabs (256 rows) into a second accumulator to bound the
// accumulation error, and blocks combine with fp32 atomics.
template <int BO, int BI, bool YXF>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(const float* __restrict__ X, int ldx, int N,
                                                       const float* __restrict__ Y, int ldy, int K,
                                                       const float* __restrict__ s, const float* __restrict__ t,
                                                       int act, float slope, int M, int rows_per_block,
                                                       float* __restrict__ dW, float* __restrict__ db) {
    constexpr int BR = 32, LDR = BR + 4;
    constexpr int TM = BO / 64, TN = BI / 64;
    constexpr int XV = BR * BO / 4 / 256, YV = BR * BI / 4 / 256;
    __shared__ __attribute__((aligned(16))) float Xs[2][BO][LDR];
    __shared__ __attribute__((aligned(16))) float Ys[2][BI][LDR];
    __shared__ float dbs[256 / (BO / 4)][BO];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wo = wave >> 1, wi = wave & 1;
    const int h = lane >> 5, l32 = lane & 31;
    const int tiles_i = (K + BI - 1) / BI;
    const int n0 = (blockIdx.y / tiles_i) * BO;
    const int k0 = (blockIdx.y % tiles_i) * BI;
    const int rb = blockIdx.x * rows_per_block;
    const int re = min(M, rb + rows_per_block);
    const bool do_db = (db != nullptr) && (k0 == 0);

    // this thread's fixed channel quads
    const int xc4 = tid % (BO / 4), yc4 = tid % (BI / 4);
    float ys[4] = {1.f, 1.f, 1.f, 1.f}, yt[4] = {0.f, 0.f, 0.f, 0.f};
    if (YXF) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int gk = k0 + 4 * yc4 + j;
            if (gk < K) { ys[j] = s[gk]; yt[j] = t[gk]; }
        }
    }
    float dbv[4] = {0.f, 0.f, 0.f, 0.f};

    f32x16 acc[TM][TN], tot[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) { acc[i][j][r] = 0.f; tot[i][j][r] = 0.f; }

    float4 rx[XV], ry[YV];
    auto gload = [&](int r0) {
#pragma unroll
        for (int it = 0; it < XV; ++it) {
            const int e = it * 256 + tid;
            const int r = e / (BO / 4);
            const int gr = r0 + r, gn = n0 + 4 * xc4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (gr < re && gn < N) v = *reinterpret_cast<const float4*>(X + (size_t)gr * ldx + gn);
            rx[it] = v;
        }
#pragma unroll
        for (int it = 0; it < YV; ++it) {
            const int e = it * 256 + tid;
            const int r = e / (BI / 4);
            const int gr = r0 + r, gk = k0 + 4 * yc4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (gr < re && gk < K) v = *reinterpret_cast<const float4*>(Y + (size_t)gr * ldy + gk);
            ry[it] = v;
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int it = 0; it < XV; ++it) {
            const int e = it * 256 + tid;
            const int r = e / (BO / 4);
            const float4 v = rx[it];
            Xs[buf][4 * xc4 + 0][r] = v.x;
            Xs[buf][4 * xc4 + 1][r] = v.y;
            Xs[buf][4 * xc4 + 2][r] = v.z;
            Xs[buf][4 * xc4 + 3][r] = v.w;
            if (do_db) { dbv[0] += v.x; dbv[1] += v.y; dbv[2] += v.z; dbv[3] += v.w; }
        }
#pragma unroll
        for (int it = 0; it < YV; ++it) {
            const int e = it * 256 + tid;
            const int r = e / (BI / 4);
            float4 v = ry[it];
            if (YXF) {
                const int gk = k0 + 4 * yc4;
                v.x = gk + 0 < K ? act_f(v.x * ys[0] + yt[0], act, slope) : 0.f;
                v.y = gk + 1 < K ? act_f(v.y * ys[1] + yt[1], act, slope) : 0.f;
                v.z = gk + 2 < K ? act_f(v.z * ys[2] + yt[2], act, slope) : 0.f;
                v.w = gk + 3 < K ? act_f(v.w * ys[3] + yt[3], act, slope) : 0.f;
            }
            Ys[buf][4 * yc4 + 0][r] = v.x;
            Ys[buf][4 * yc4 + 1][r] = v.y;
            Ys[buf][4 * yc4 + 2][r] = v.z;
            Ys[buf][4 * yc4 + 3][r] = v.w;
        }
    };

    const int nslab = (re - rb + BR - 1) / BR;
    if (nslab > 0) {
        gload(rb);
        sstore(0);
    }
    __syncthreads();
    for (int sl = 0; sl < nslab; ++sl) {
        const int buf = sl & 1;
        if (sl + 1 < nslab) gload(rb + (sl + 1) * BR);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float4 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                a[i] = *reinterpret_cast<const float4*>(&Xs[buf][wo * (BO / 2) + i * 32 + l32][16 * h + 4 * q]);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                b[j] = *reinterpret_cast<const float4*>(&Ys[buf][wi * (BI / 2) + j * 32 + l32][16 * h + 4 * q]);
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
        if ((sl & 7) == 7) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) { tot[i][j][r] += acc[i][j][r]; acc[i][j][r] = 0.f; }
        }
        if (sl + 1 < nslab) sstore(buf ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int kcol = k0 + wi * (BI / 2) + j * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = n0 + wo * (BO / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (n < N && kcol < K) atomicAdd(&dW[(size_t)n * K + kcol], tot[i][j][r] + acc[i][j][r]);
            }
        }
    if (do_db) {
        const int grp = tid / (BO / 4);
        dbs[grp][4 * xc4 + 0] = dbv[0];
        dbs[grp][4 * xc4 + 1] = dbv[1];
        dbs[grp][4 * xc4 + 2] = dbv[2];
        dbs[grp][4 * xc4 + 3] = dbv[3];
        __syncthreads();
        if (tid < BO && n0 + tid < N) {
            float a = 0.f;
#pragma unroll
            for (int gi = 0; gi < 256 / (BO / 4); ++gi) a += dbs[gi][tid];
            atomicAdd(&db[n0 + tid], a);
        }
    }
}

// ------------------------------------------------------------------ BN finalize (forward)
// one block per channel: reduce nb partials -> mean/var -> s,t ; running-stat update
__global__ __launch_bounds__(256) void bn_finalize_kernel(const double* __restrict__ part, int nb, int N, long long M,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps, float momentum,
                                                          float* __restrict__ run_mean, float* __restrict__ run_var,
                                                          float* __restrict__ s, float* __restrict__ t,
                                                          float* __restrict__ mean_out, float* __restrict__ inv_out) {
    __shared__ double r1[256], r2[256];
    const int n = blockIdx.x;
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < nb; i += 256) {
        a += part[((size_t)i * 2 + 0) * N + n];
        b += part[((size_t)i * 2 + 1) * N + n];
    }
    r1[threadIdx.x] = a;
    r2[threadIdx.x] = b;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            r1[threadIdx.x] += r1[threadIdx.x + o];
            r2[threadIdx.x] += r2[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double mean = r1[0] / (double)M;
        double var = r2[0] / (double)M - mean * mean;
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
// kB = s*sum_dy/M, kC = s*sum_dyx/M
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const double* __restrict__ part, int nb, int N,
                                                              long long M, const float* __restrict__ s,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              float* __restrict__ kB, float* __restrict__ kC,
                                                              int accum) {
    __shared__ double r1[256], r2[256];
    const int n = blockIdx.x;
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < nb; i += 256) {
        a += part[((size_t)i * 2 + 0) * N + n];
        b += part[((size_t)i * 2 + 1) * N + n];
    }
    r1[threadIdx.x] = a;
    r2[threadIdx.x] = b;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            r1[threadIdx.x] += r1[threadIdx.x + o];
            r2[threadIdx.x] += r2[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double S1 = r1[0], S2 = r2[0];
        if (dbeta) dbeta[n] = accum ? dbeta[n] + (float)S1 : (float)S1;
        if (dgamma) dgamma[n] = accum ? dgamma[n] + (float)S2 : (float)S2;
        kB[n] = (float)((double)s[n] * S1 / (double)M);
        kC[n] = (float)((double)s[n] * S2 / (double)M);
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
                                                            int rows_per_block, double* __restrict__ part) {
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
        for (int r = rb + rlane; r < re; r += rstep) {
            const F4 z = ld4(Z + (size_t)r * ldz + c);
            const F4 g = ld4(dA + (size_t)r * ldd + c);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float dy = g.v[j] * dact_f(z.v[j] * sc[j] + tc[j], act, slope);
                a[j] += (double)dy;
                b[j] += (double)dy * (double)((z.v[j] - mc[j]) * ic[j]);
            }
        }
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
            part[((size_t)blockIdx.x * 2 + 0) * N + c + j] = a[j];
            part[((size_t)blockIdx.x * 2 + 1) * N + c + j] = b[j];
        }
    }
}

// dZ = s*dy - kB - kC*xhat   (dy = dA * act'(z*s+t), xhat = (z-mean)*inv), dense rows
__global__ __launch_bounds__(256) void bn_bwd_dz_kernel(const float* __restrict__ dA, int ldd,
                                                        const float* __restrict__ Z, int ldz, int total4, int nq,
                                                        const float* __restrict__ s, const float* __restrict__ t,
                                                        const float* __restrict__ mean, const float* __restrict__ inv,
                                                        const float* __restrict__ kB, const float* __restrict__ kC,
                                                        int act, float slope, float* __restrict__ dZ) {
    for (int e = blockIdx.x * 256 + threadIdx.x; e < total4; e += gridDim.x * 256) {
        const int r = e / nq;
        const int c = 4 * (e - r * nq);
        const F4 z = ld4(Z + (size_t)r * ldz + c);
        const F4 g = ld4(dA + (size_t)r * ldd + c);
        F4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float dy = g.v[j] * dact_f(z.v[j] * s[c + j] + t[c + j], act, slope);
            const float xh = (z.v[j] - mean[c + j]) * inv[c + j];
            o.v[j] = s[c + j] * dy - kB[c + j] - kC[c + j] * xh;
        }
        st4(dZ + (size_t)r * 4 * nq + c, o);
    }
}

// ------------------------------------------------------------------ pooling over K with BN + act
// pooled[g][c] = max_k act(z*s+t) (first max), argmax u8
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
        part[((size_t)blockIdx.x * 2 + 0) * N + col] = r1[0][lane] + r1[1][lane] + r1[2][lane] + r1[3][lane];
        part[((size_t)blockIdx.x * 2 + 1) * N + col] = r2[0][lane] + r2[1][lane] + r2[2][lane] + r2[3][lane];
    }
}

// dZ of a pooled layer: dy is dpool at the argmax row, 0 elsewhere
__global__ __launch_bounds__(256) void pool_bwd_dz_kernel(const float* __restrict__ dpool,
                                                          const unsigned char* __restrict__ arg,
                                                          const float* __restrict__ Z, int nq, int G, int K,
                                                          const float* __restrict__ s, const float* __restrict__ t,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ inv,
                                                          const float* __restrict__ kB, const float* __restrict__ kC,
                                                          int act, float slope, float* __restrict__ dZ) {
    const int N = 4 * nq;
    const long long total4 = (long long)G * K * nq;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total4; e += (long long)gridDim.x * 256) {
        const int r = (int)(e / nq);
        const int c = 4 * (int)(e - (long long)r * nq);
        const int g = r / K;
        const int k = r - g * K;
        const F4 z = ld4(Z + (size_t)r * N + c);
        const uchar4 aq = *reinterpret_cast<const uchar4*>(arg + (size_t)g * N + c);
        const F4 dp = ld4(dpool + (size_t)g * N + c);
        const unsigned char av[4] = {aq.x, aq.y, aq.z, aq.w};
        F4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float dy = av[j] == k ? dp.v[j] * dact_f(z.v[j] * s[c + j] + t[c + j], act, slope) : 0.f;
            const float xh = (z.v[j] - mean[c + j]) * inv[c + j];
            o.v[j] = s[c + j] * dy - kB[c + j] - kC[c + j] * xh;
        }
        st4(dZ + (size_t)r * N + c, o);
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
        F4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o.v[j] = act_f(z.v[j] * s[c + j] + t[c + j], act, slope);
        st4(out + (size_t)r * ldo + c, o);
    }
}

static inline unsigned ew_grid(long long total) {
    long long g = (total + 255) / 256;
    if (g > 8192) g = 8192;
    return (unsigned)(g < 1 ? 1 : g);
}

template <int BM, int BN, int WM, int WN>
static void launch_gemm(const GemmArgs& g, hipStream_t s) {
    const dim3 grid((g.M + BM - 1) / BM, (g.N + BN - 1) / BN);
    if (g.s_in) hipLaunchKernelGGL((gemm_rows_kernel<BM, BN, WM, WN, true>), grid, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((gemm_rows_kernel<BM, BN, WM, WN, false>), grid, dim3(256), 0, s, g);
}

template <int BO, int BI>
static void launch_wgrad(dim3 grid, hipStream_t st, const float* X, int ldx, int N, const float* Y, int ldy, int K,
                         const float* s, const float* t, int act, float slope, int M, int rows, float* dW, float* db) {
    if (s) hipLaunchKernelGGL((wgrad_kernel<BO, BI, true>), grid, dim3(256), 0, st, X, ldx, N, Y, ldy, K, s, t, act,
                              slope, M, rows, dW, db);
    else hipLaunchKernelGGL((wgrad_kernel<BO, BI, false>), grid, dim3(256), 0, st, X, ldx, N, Y, ldy, K, s, t, act,
                            slope, M, rows, dW, db);
}

}  // namespace pcs

using namespace pcs;

// number of row blocks the row GEMM uses for M rows and N outputs (sizes the stats workspace)
PCS_API int pcs_gemm_row_blocks(int M, int N) {
    (void)N;
    return (M + 127) / 128;
}

// C = act_in(A*s_in+t_in) . W^T (+bias), W row-major N x K (row stride ldw).
// stats (nullable): [row_blocks][2][N] fp64 partial (sum, sumsq) of C.
// bstats (nullable): fused BN-backward partials of the layer whose pre-BN output is zp (same shape as C):
//   [row_blocks][2][N] of (sum dy, sum dy*xhat), dy = C * act'(zp*sp+tp), xhat = (zp-meanp)*invp.
PCS_API int pcs_gemm_rows(const float* A, int lda, int M, int K, const float* s_in, const float* t_in, int act_in,
                          float slope_in, const float* W, int ldw, const float* bias, float* C, int ldc,
                          int N, double* stats, const float* zp, int ldzp, const float* sp, const float* tp,
                          const float* meanp, const float* invp, int actp, float slopep, double* bstats,
                          void* stream) {
    PCS_CHECK_ARG(M >= 0 && K >= 1 && N >= 1, "pcs_gemm_rows: bad sizes M=%d K=%d N=%d", M, K, N);
    PCS_CHECK_ARG(lda % 4 == 0 && lda >= K, "pcs_gemm_rows: lda=%d must be a multiple of 4 and >= K=%d", lda, K);
    PCS_CHECK_ARG(A && W && C, "pcs_gemm_rows: null pointer");
    PCS_CHECK_ARG(!(stats && bstats), "pcs_gemm_rows: stats and bstats are exclusive");
    PCS_CHECK_ARG(!bstats || (zp && sp && tp && meanp && invp), "pcs_gemm_rows: bstats needs zp/sp/tp/meanp/invp");
    PCS_CHECK_ARG((s_in == nullptr) == (t_in == nullptr), "pcs_gemm_rows: s_in/t_in must both be set or null");
    PCS_CHECK_ARG(ldw >= K, "pcs_gemm_rows: ldw=%d < K=%d", ldw, K);
    if (M == 0) return 0;
    GemmArgs g{A, lda, M, K, s_in, t_in, act_in, slope_in, W, ldw, bias, C, ldc, N, stats,
               zp, ldzp, sp, tp, meanp, invp, actp, slopep, bstats};
    hipStream_t s = as_stream(stream);
    if (N <= 32) launch_gemm<128, 32, 4, 1>(g, s);
    else if (N <= 64) launch_gemm<128, 64, 4, 1>(g, s);
    else launch_gemm<128, 128, 2, 2>(g, s);
    return launch_status("pcs_gemm_rows");
}

// dW (N x K) += X^T . act(Y*s+t) over M rows; db (N) += column sums of X. dW/db zeroed by caller.
PCS_API int pcs_wgrad(const float* X, int ldx, int N, const float* Y, int ldy, int K, const float* s, const float* t,
                      int act, float slope, int M, float* dW, float* db, void* stream) {
    PCS_CHECK_ARG(M >= 0 && N >= 1 && K >= 1, "pcs_wgrad: bad sizes");
    PCS_CHECK_ARG(X && Y && dW, "pcs_wgrad: null pointer");
    PCS_CHECK_ARG(ldx % 4 == 0 && ldy % 4 == 0 && N % 4 == 0, "pcs_wgrad: ldx/ldy/N must be multiples of 4");
    if (M == 0) return 0;
    const int BO = N > 64 ? 128 : 64, BI = K > 64 ? 128 : 64;
    const int tiles = ((N + BO - 1) / BO) * ((K + BI - 1) / BI);
    int splits = (1024 + tiles - 1) / tiles;
    int rows = (M + splits - 1) / splits;
    rows = ((rows + 255) / 256) * 256;
    if (rows < 256) rows = 256;
    splits = (M + rows - 1) / rows;
    const dim3 grid(splits, tiles);
    hipStream_t st = as_stream(stream);
    if (BO == 128 && BI == 128) launch_wgrad<128, 128>(grid, st, X, ldx, N, Y, ldy, K, s, t, act, slope, M, rows, dW, db);
    else if (BO == 128) launch_wgrad<128, 64>(grid, st, X, ldx, N, Y, ldy, K, s, t, act, slope, M, rows, dW, db);
    else if (BI == 128) launch_wgrad<64, 128>(grid, st, X, ldx, N, Y, ldy, K, s, t, act, slope, M, rows, dW, db);
    else launch_wgrad<64, 64>(grid, st, X, ldx, N, Y, ldy, K, s, t, act, slope, M, rows, dW, db);
    return launch_status("pcs_wgrad");
}

// BN forward finalize: part [nb][2][N] -> s, t, mean, invstd; running stats updated in place (nullable).
PCS_API int pcs_bn_finalize(const double* part, int nb, int N, long long M, const float* gamma, const float* beta,
                            float eps, float momentum, float* run_mean, float* run_var, float* s, float* t,
                            float* mean, float* invstd, void* stream) {
    PCS_CHECK_ARG(nb >= 1 && N >= 1 && M >= 1, "pcs_bn_finalize: bad sizes");
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(N), dim3(256), 0, as_stream(stream), part, nb, N, M, gamma, beta, eps,
                       momentum, run_mean, run_var, s, t, mean, invstd);
    return launch_status("pcs_bn_finalize");
}

// BN backward finalize: part [nb][2][N] of (sum dy, sum dy*xhat) -> dgamma, dbeta (+= when accum), kB, kC.
PCS_API int pcs_bn_bwd_finalize(const double* part, int nb, int N, long long M, const float* s, float* dgamma,
                                float* dbeta, float* kB, float* kC, int accum, void* stream) {
    PCS_CHECK_ARG(nb >= 1 && N >= 1 && M >= 1, "pcs_bn_bwd_finalize: bad sizes");
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(N), dim3(256), 0, as_stream(stream), part, nb, N, M, s, dgamma,
                       dbeta, kB, kC, accum);
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
                       Z, ldz, M, N, s, t, mean, inv, act, slope, kRedRows, part);
    return launch_status("pcs_bn_bwd_reduce");
}

PCS_API int pcs_bn_bwd_dz(const float* dA, int ldd, const float* Z, int ldz, int M, int N, const float* s,
                          const float* t, const float* mean, const float* inv, const float* kB, const float* kC,
                          int act, float slope, float* dZ, void* stream) {
    PCS_CHECK_ARG(M >= 0 && N >= 4 && N % 4 == 0 && ldd % 4 == 0 && ldz % 4 == 0, "pcs_bn_bwd_dz: bad sizes");
    const long long total = (long long)M * N / 4;
    PCS_CHECK_ARG(total < (1ll << 31), "pcs_bn_bwd_dz: too many elements");
    if (total == 0) return 0;
    hipLaunchKernelGGL(bn_bwd_dz_kernel, dim3(ew_grid(total)), dim3(256), 0, as_stream(stream), dA, ldd, Z, ldz,
                       (int)total, N / 4, s, t, mean, inv, kB, kC, act, slope, dZ);
    return launch_status("pcs_bn_bwd_dz");
}

PCS_API int pcs_pool_fwd(const float* Z, int N, long long G, int K, const float* s, const float* t, int act,
                         float slope, float* out, uint8_t* arg, void* stream) {
    PCS_CHECK_ARG(G >= 0 && K >= 1 && K <= 256 && N >= 4 && N % 4 == 0, "pcs_pool_fwd: bad sizes");
    const long long total = G * N / 4;
    PCS_CHECK_ARG(G * K * (long long)N < (1ll << 40) && total < (1ll << 31), "pcs_pool_fwd: too many elements");
    if (total == 0) return 0;
    hipLaunchKernelGGL(pool_fwd_kernel, dim3(ew_grid(total)), dim3(256), 0, as_stream(stream), Z, N / 4, (int)G, K, s,
                       t, act, slope, out, arg);
    return launch_status("pcs_pool_fwd");
}

PCS_API int pcs_pool_bwd_reduce_blocks(long long G) { return (int)((G + 63) / 64); }

PCS_API int pcs_pool_bwd_reduce(const float* dpool, const uint8_t* arg, const float* Z, int N, long long G, int K,
                                const float* s, const float* t, const float* mean, const float* inv, int act,
                                float slope, double* part, void* stream) {
    PCS_CHECK_ARG(G >= 1 && G < (1ll << 31) && K >= 1 && N >= 1, "pcs_pool_bwd_reduce: bad sizes");
    const int gpb = 64;
    const dim3 grid((unsigned)((G + gpb - 1) / gpb), (N + 63) / 64);
    hipLaunchKernelGGL(pool_bwd_reduce_kernel, grid, dim3(256), 0, as_stream(stream), dpool, arg, Z, N, (int)G, K, s,
                       t, mean, inv, act, slope, gpb, part);
    return launch_status("pcs_pool_bwd_reduce");
}

PCS_API int pcs_pool_bwd_dz(const float* dpool, const uint8_t* arg, const float* Z, int N, long long G, int K,
                            const float* s, const float* t, const float* mean, const float* inv, const float* kB,
                            const float* kC, int act, float slope, float* dZ, void* stream) {
    PCS_CHECK_ARG(G >= 0 && G < (1ll << 31) && K >= 1 && K <= 256 && N >= 4 && N % 4 == 0,
                  "pcs_pool_bwd_dz: bad sizes");
    const long long total = G * K * N / 4;
    if (total == 0) return 0;
    hipLaunchKernelGGL(pool_bwd_dz_kernel, dim3(ew_grid(total)), dim3(256), 0, as_stream(stream), dpool, arg, Z, N / 4,
                       (int)G, K, s, t, mean, inv, kB, kC, act, slope, dZ);
    return launch_status("pcs_pool_bwd_dz");
}

PCS_API int pcs_bn_act(const float* Z, int ldz, int M, int N, const float* s, const float* t, int act, float slope,
                       float* out, int ldo, void* stream) {
    PCS_CHECK_ARG(M >= 0 && N >= 4 && N % 4 == 0 && ldz % 4 == 0 && ldo % 4 == 0, "pcs_bn_act: bad sizes");
    const long long total = (long long)M * N / 4;
    PCS_CHECK_ARG(total < (1ll << 31), "pcs_bn_act: too many elements");
    if (total == 0) return 0;
    hipLaunchKernelGGL(bn_act_kernel, dim3(ew_grid(total)), dim3(256), 0, as_stream(stream), Z, ldz, (int)total, N / 4,
                       s, t, act, slope, out, ldo);
    return launch_status("pcs_bn_act");
}
