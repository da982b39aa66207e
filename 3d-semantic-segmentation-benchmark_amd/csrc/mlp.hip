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
    const float* W; int ldw;                   // BT: B[k][n] = W[n*ldw+k]; else B[k][n] = W[k*ldw+n]
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
template <int BM, int BN, int WM, int WN, bool BT, bool AXF>
__global__ __launch_bounds__(256) void gemm_rows_kernel(GemmArgs g) {
    constexpr int BK = 32;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    static_assert(WM * WN == 4, "4 waves");
    static_assert(TM >= 1 && TN >= 1, "tile");
    __shared__ float As[BM][BK + 1];
    __shared__ float Bs[BK][BN + 1];
    __shared__ double red[2][WM][BN];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    for (int k0 = 0; k0 < g.K; k0 += BK) {
        // ---- A tile (BM x BK), float4 loads along K (lda % 4 == 0)
#pragma unroll
        for (int it = 0; it < BM * BK / 4 / 256; ++it) {
            const int e = it * 256 + tid;
            const int r = e / (BK / 4), c4 = e % (BK / 4);
            const int gr = m0 + r, gk = k0 + c4 * 4;
            float v[4] = {0.f, 0.f, 0.f, 0.f};
            if (gr < g.M && gk < g.K) {
                const float4 q = *reinterpret_cast<const float4*>(g.A + (size_t)gr * g.lda + gk);
                v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (gk + i >= g.K) v[i] = 0.f;
                    else if (AXF) v[i] = act_f(v[i] * g.s_in[gk + i] + g.t_in[gk + i], g.act_in, g.slope_in);
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) As[r][c4 * 4 + i] = v[i];
        }
        // ---- B tile (BK x BN)
        if (BT) {
#pragma unroll
            for (int it = 0; it < (BK * BN + 255) / 256; ++it) {
                const int e = it * 256 + tid;
                if (e < BK * BN) {
                    const int n = e / BK, kk = e % BK;
                    const int gn = n0 + n, gk = k0 + kk;
                    Bs[kk][n] = (gn < g.N && gk < g.K) ? g.W[(size_t)gn * g.ldw + gk] : 0.f;
                }
            }
        } else {
#pragma unroll
            for (int it = 0; it < (BK * BN + 255) / 256; ++it) {
                const int e = it * 256 + tid;
                if (e < BK * BN) {
                    const int kk = e / BN, n = e % BN;
                    const int gn = n0 + n, gk = k0 + kk;
                    Bs[kk][n] = (gn < g.N && gk < g.K) ? g.W[(size_t)gk * g.ldw + gn] : 0.f;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < BK; kk += 2) {
            float a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) a[i] = As[wm * WTM + i * 32 + (lane & 31)][kk + (lane >> 5)];
#pragma unroll
            for (int j = 0; j < TN; ++j) b[j] = Bs[kk + (lane >> 5)][wn * WTN + j * 32 + (lane & 31)];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }

    // ---- epilogue: bias, store, per-channel partial reductions
    const bool want_stats = g.stats != nullptr;
    const bool want_b = g.bstats != nullptr;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int lc = wn * WTN + j * 32 + (lane & 31);
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
                const int row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
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
template <bool YXF>
__global__ __launch_bounds__(256) void wgrad_kernel(const float* __restrict__ X, int ldx, int N,
                                                    const float* __restrict__ Y, int ldy, int K,
                                                    const float* __restrict__ s, const float* __restrict__ t,
                                                    int act, float slope, int M, int rows_per_block,
                                                    float* __restrict__ dW, float* __restrict__ db) {
    constexpr int BR = 32, BO = 64, BI = 64;
    __shared__ float Xs[BR][BO + 1];
    __shared__ float Ys[BR][BI + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wo = wave >> 1, wi = wave & 1;
    const int tiles_i = (K + BI - 1) / BI;
    const int n0 = (blockIdx.y / tiles_i) * BO;
    const int k0 = (blockIdx.y % tiles_i) * BI;
    const int rb = blockIdx.x * rows_per_block;
    const int re = min(M, rb + rows_per_block);
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    float dbacc = 0.f;
    const bool do_db = (db != nullptr) && (k0 == 0);
    for (int r0 = rb; r0 < re; r0 += BR) {
#pragma unroll
        for (int it = 0; it < BR * BO / 256; ++it) {
            const int e = it * 256 + tid;
            const int rr = e / BO, c = e % BO;
            const int gr = r0 + rr, gn = n0 + c;
            Xs[rr][c] = (gr < re && gn < N) ? X[(size_t)gr * ldx + gn] : 0.f;
            const int gk = k0 + c;
            float y = 0.f;
            if (gr < re && gk < K) {
                y = Y[(size_t)gr * ldy + gk];
                if (YXF) y = act_f(y * s[gk] + t[gk], act, slope);
            }
            Ys[rr][c] = y;
        }
        __syncthreads();
        if (do_db && tid < BO) {
#pragma unroll 8
            for (int rr = 0; rr < BR; ++rr) dbacc += Xs[rr][tid];
        }
#pragma unroll
        for (int kk = 0; kk < BR; kk += 2) {
            const float a = Xs[kk + (lane >> 5)][wo * 32 + (lane & 31)];
            const float b = Ys[kk + (lane >> 5)][wi * 32 + (lane & 31)];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
        }
        __syncthreads();
    }
    const int kcol = k0 + wi * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int n = n0 + wo * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (n < N && kcol < K) atomicAdd(&dW[(size_t)n * K + kcol], acc[r]);
    }
    if (do_db && tid < BO && n0 + tid < N) atomicAdd(&db[n0 + tid], dbacc);
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
// sums (sum dy, sum dy*xhat) -> dgamma, dbeta and dZ coefficients kB = s*sum_dy/M, kC = s*sum_dyx/M
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const double* __restrict__ part, int nb, int N,
                                                              long long M, const float* __restrict__ s,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              float* __restrict__ kB, float* __restrict__ kC,
                                                              const float* __restrict__ inv) {
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
        if (dbeta) dbeta[n] = (float)r1[0];
        if (dgamma) dgamma[n] = (float)r2[0];
        kB[n] = (float)((double)s[n] * r1[0] / (double)M);
        kC[n] = (float)((double)s[n] * r2[0] / (double)M);
        (void)inv;
    }
}

// ------------------------------------------------------------------ column reduce of (dy, dy*xhat)
// standalone BN-backward reduce when dA comes from outside the engine
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const float* __restrict__ dA, int ldd,
                                                            const float* __restrict__ Z, int ldz, int M, int N,
                                                            const float* __restrict__ s, const float* __restrict__ t,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ inv, int act, float slope,
                                                            int rows_per_block, double* __restrict__ part) {
    __shared__ double r1[4][64], r2[4][64];
    const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
    const int col = blockIdx.y * 64 + lane;
    const int rb = blockIdx.x * rows_per_block;
    const int re = min(M, rb + rows_per_block);
    double a = 0.0, b = 0.0;
    if (col < N) {
        const float sc = s[col], tc = t[col], mc = mean[col], ic = inv[col];
        for (int r = rb + ph; r < re; r += 4) {
            const float z = Z[(size_t)r * ldz + col];
            const float dy = dA[(size_t)r * ldd + col] * dact_f(z * sc + tc, act, slope);
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

// dZ = s*dy - kB - kC*xhat   (dy = dA * act'(z*s+t), xhat = (z-mean)*inv)
__global__ __launch_bounds__(256) void bn_bwd_dz_kernel(const float* __restrict__ dA, int ldd,
                                                        const float* __restrict__ Z, int ldz, long long total, int N,
                                                        const float* __restrict__ s, const float* __restrict__ t,
                                                        const float* __restrict__ mean, const float* __restrict__ inv,
                                                        const float* __restrict__ kB, const float* __restrict__ kC,
                                                        int act, float slope, float* __restrict__ dZ) {
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long r = e / N;
        const int c = (int)(e - r * N);
        const float z = Z[r * ldz + c];
        const float dy = dA[r * ldd + c] * dact_f(z * s[c] + t[c], act, slope);
        const float xh = (z - mean[c]) * inv[c];
        dZ[e] = s[c] * dy - kB[c] - kC[c] * xh;
    }
}

// ------------------------------------------------------------------ pooling over K with BN + act
// pooled[g][c] = max_k act(z*s+t) (first max), argmax u8
__global__ __launch_bounds__(256) void pool_fwd_kernel(const float* __restrict__ Z, int N, long long G, int K,
                                                       const float* __restrict__ s, const float* __restrict__ t,
                                                       int act, float slope, float* __restrict__ out,
                                                       unsigned char* __restrict__ arg) {
    const long long total = G * N;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long g = e / N;
        const int c = (int)(e - g * N);
        const float sc = s[c], tc = t[c];
        const float* z = Z + g * K * N + c;
        float m = act_f(z[0] * sc + tc, act, slope);
        int a = 0;
        for (int k = 1; k < K; ++k) {
            const float v = act_f(z[(long long)k * N] * sc + tc, act, slope);
            if (v > m) { m = v; a = k; }
        }
        out[e] = m;
        arg[e] = (unsigned char)a;
    }
}

// BN-backward sums for a pooled layer: only the argmax row of each (g, c) carries dy
__global__ __launch_bounds__(256) void pool_bwd_reduce_kernel(const float* __restrict__ dpool,
                                                              const unsigned char* __restrict__ arg,
                                                              const float* __restrict__ Z, int N, long long G, int K,
                                                              const float* __restrict__ s,
                                                              const float* __restrict__ t,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ inv, int act, float slope,
                                                              int groups_per_block, double* __restrict__ part) {
    __shared__ double r1[4][64], r2[4][64];
    const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
    const int col = blockIdx.y * 64 + lane;
    const long long gb = (long long)blockIdx.x * groups_per_block;
    const long long ge = min(G, gb + groups_per_block);
    double a = 0.0, b = 0.0;
    if (col < N) {
        const float sc = s[col], tc = t[col], mc = mean[col], ic = inv[col];
        for (long long g = gb + ph; g < ge; g += 4) {
            const int k = arg[g * N + col];
            const float z = Z[(g * K + k) * N + col];
            const float dy = dpool[g * N + col] * dact_f(z * sc + tc, act, slope);
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
                                                          const float* __restrict__ Z, int N, long long G, int K,
                                                          const float* __restrict__ s, const float* __restrict__ t,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ inv,
                                                          const float* __restrict__ kB, const float* __restrict__ kC,
                                                          int act, float slope, float* __restrict__ dZ) {
    const long long total = G * K * N;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long r = e / N;
        const int c = (int)(e - r * N);
        const long long g = r / K;
        const int k = (int)(r - g * K);
        const float z = Z[e];
        float dy = 0.f;
        if (arg[g * N + c] == k) dy = dpool[g * N + c] * dact_f(z * s[c] + t[c], act, slope);
        const float xh = (z - mean[c]) * inv[c];
        dZ[e] = s[c] * dy - kB[c] - kC[c] * xh;
    }
}

// a = act(z*s + t) materialised (outputs consumed outside the engine)
__global__ __launch_bounds__(256) void bn_act_kernel(const float* __restrict__ Z, int ldz, long long total, int N,
                                                     const float* __restrict__ s, const float* __restrict__ t,
                                                     int act, float slope, float* __restrict__ out, int ldo) {
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long r = e / N;
        const int c = (int)(e - r * N);
        out[r * ldo + c] = act_f(Z[r * ldz + c] * s[c] + t[c], act, slope);
    }
}

static inline unsigned ew_grid(long long total) {
    long long g = (total + 255) / 256;
    if (g > 16384) g = 16384;
    return (unsigned)(g < 1 ? 1 : g);
}

template <int BM, int BN, int WM, int WN, bool BT>
static void launch_gemm(const GemmArgs& g, hipStream_t s) {
    const dim3 grid((g.M + BM - 1) / BM, (g.N + BN - 1) / BN);
    if (g.s_in) hipLaunchKernelGGL((gemm_rows_kernel<BM, BN, WM, WN, BT, true>), grid, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((gemm_rows_kernel<BM, BN, WM, WN, BT, false>), grid, dim3(256), 0, s, g);
}

}  // namespace pcs

using namespace pcs;

// number of row blocks the row GEMM uses for M rows and N outputs (sizes the stats workspace)
PCS_API int pcs_gemm_row_blocks(int M, int N) {
    (void)N;
    return (M + 127) / 128;
}

// C = act_in(A*s_in+t_in) . B (+bias), B = W^T (trans_w=1, W is N x K) or W (trans_w=0, W is K x N).
// stats (nullable): [row_blocks][2][N] fp64 partial (sum, sumsq) of C.
// bstats (nullable): fused BN-backward partials of the layer whose pre-BN output is zp (same shape as C):
//   [row_blocks][2][N] of (sum dy, sum dy*xhat), dy = C * act'(zp*sp+tp), xhat = (zp-meanp)*invp.
PCS_API int pcs_gemm_rows(const float* A, int lda, int M, int K, const float* s_in, const float* t_in, int act_in,
                          float slope_in, const float* W, int ldw, int trans_w, const float* bias, float* C, int ldc,
                          int N, double* stats, const float* zp, int ldzp, const float* sp, const float* tp,
                          const float* meanp, const float* invp, int actp, float slopep, double* bstats,
                          void* stream) {
    PCS_CHECK_ARG(M >= 0 && K >= 1 && N >= 1, "pcs_gemm_rows: bad sizes M=%d K=%d N=%d", M, K, N);
    PCS_CHECK_ARG(lda % 4 == 0 && lda >= K, "pcs_gemm_rows: lda=%d must be a multiple of 4 and >= K=%d", lda, K);
    PCS_CHECK_ARG(A && W && C, "pcs_gemm_rows: null pointer");
    PCS_CHECK_ARG(!(stats && bstats), "pcs_gemm_rows: stats and bstats are exclusive");
    PCS_CHECK_ARG(!bstats || (zp && sp && tp && meanp && invp), "pcs_gemm_rows: bstats needs zp/sp/tp/meanp/invp");
    PCS_CHECK_ARG((s_in == nullptr) == (t_in == nullptr), "pcs_gemm_rows: s_in/t_in must both be set or null");
    if (M == 0) return 0;
    GemmArgs g{A, lda, M, K, s_in, t_in, act_in, slope_in, W, ldw, bias, C, ldc, N, stats,
               zp, ldzp, sp, tp, meanp, invp, actp, slopep, bstats};
    hipStream_t s = as_stream(stream);
    if (trans_w) {
        if (N <= 32) launch_gemm<128, 32, 4, 1, true>(g, s);
        else if (N <= 64) launch_gemm<128, 64, 4, 1, true>(g, s);
        else launch_gemm<128, 128, 2, 2, true>(g, s);
    } else {
        if (N <= 32) launch_gemm<128, 32, 4, 1, false>(g, s);
        else if (N <= 64) launch_gemm<128, 64, 4, 1, false>(g, s);
        else launch_gemm<128, 128, 2, 2, false>(g, s);
    }
    return launch_status("pcs_gemm_rows");
}

// dW (N x K) += X^T . act(Y*s+t) over M rows; db (N) += column sums of X. dW/db zeroed by caller.
PCS_API int pcs_wgrad(const float* X, int ldx, int N, const float* Y, int ldy, int K, const float* s, const float* t,
                      int act, float slope, int M, float* dW, float* db, void* stream) {
    PCS_CHECK_ARG(M >= 0 && N >= 1 && K >= 1, "pcs_wgrad: bad sizes");
    PCS_CHECK_ARG(X && Y && dW, "pcs_wgrad: null pointer");
    if (M == 0) return 0;
    const int tiles = ((N + 63) / 64) * ((K + 63) / 64);
    int splits = (2048 + tiles - 1) / tiles;
    int rows = (M + splits - 1) / splits;
    rows = ((rows + 31) / 32) * 32;
    if (rows < 256) rows = 256;
    splits = (M + rows - 1) / rows;
    const dim3 grid(splits, tiles);
    if (s) hipLaunchKernelGGL(wgrad_kernel<true>, grid, dim3(256), 0, as_stream(stream), X, ldx, N, Y, ldy, K, s, t,
                              act, slope, M, rows, dW, db);
    else hipLaunchKernelGGL(wgrad_kernel<false>, grid, dim3(256), 0, as_stream(stream), X, ldx, N, Y, ldy, K, s, t,
                            act, slope, M, rows, dW, db);
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

// BN backward finalize: part [nb][2][N] of (sum dy, sum dy*xhat) -> dgamma, dbeta, kB, kC.
PCS_API int pcs_bn_bwd_finalize(const double* part, int nb, int N, long long M, const float* s, float* dgamma,
                                float* dbeta, float* kB, float* kC, void* stream) {
    PCS_CHECK_ARG(nb >= 1 && N >= 1 && M >= 1, "pcs_bn_bwd_finalize: bad sizes");
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(N), dim3(256), 0, as_stream(stream), part, nb, N, M, s, dgamma,
                       dbeta, kB, kC, (const float*)nullptr);
    return launch_status("pcs_bn_bwd_finalize");
}

PCS_API int pcs_bn_bwd_reduce_blocks(int M) { return (M + 1023) / 1024; }

PCS_API int pcs_bn_bwd_reduce(const float* dA, int ldd, const float* Z, int ldz, int M, int N, const float* s,
                              const float* t, const float* mean, const float* inv, int act, float slope, double* part,
                              void* stream) {
    PCS_CHECK_ARG(M >= 1 && N >= 1, "pcs_bn_bwd_reduce: bad sizes");
    const int rows = 1024;
    const dim3 grid((M + rows - 1) / rows, (N + 63) / 64);
    hipLaunchKernelGGL(bn_bwd_reduce_kernel, grid, dim3(256), 0, as_stream(stream), dA, ldd, Z, ldz, M, N, s, t, mean,
                       inv, act, slope, rows, part);
    return launch_status("pcs_bn_bwd_reduce");
}

PCS_API int pcs_bn_bwd_dz(const float* dA, int ldd, const float* Z, int ldz, int M, int N, const float* s,
                          const float* t, const float* mean, const float* inv, const float* kB, const float* kC,
                          int act, float slope, float* dZ, void* stream) {
    PCS_CHECK_ARG(M >= 0 && N >= 1, "pcs_bn_bwd_dz: bad sizes");
    const long long total = (long long)M * N;
    if (total == 0) return 0;
    hipLaunchKernelGGL(bn_bwd_dz_kernel, dim3(ew_grid(total)), dim3(256), 0, as_stream(stream), dA, ldd, Z, ldz, total,
                       N, s, t, mean, inv, kB, kC, act, slope, dZ);
    return launch_status("pcs_bn_bwd_dz");
}

PCS_API int pcs_pool_fwd(const float* Z, int N, long long G, int K, const float* s, const float* t, int act,
                         float slope, float* out, uint8_t* arg, void* stream) {
    PCS_CHECK_ARG(G >= 0 && K >= 1 && K <= 256 && N >= 1, "pcs_pool_fwd: bad sizes");
    const long long total = G * N;
    if (total == 0) return 0;
    hipLaunchKernelGGL(pool_fwd_kernel, dim3(ew_grid(total)), dim3(256), 0, as_stream(stream), Z, N, G, K, s, t, act,
                       slope, out, arg);
    return launch_status("pcs_pool_fwd");
}

PCS_API int pcs_pool_bwd_reduce_blocks(long long G) { return (int)((G + 255) / 256); }

PCS_API int pcs_pool_bwd_reduce(const float* dpool, const uint8_t* arg, const float* Z, int N, long long G, int K,
                                const float* s, const float* t, const float* mean, const float* inv, int act,
                                float slope, double* part, void* stream) {
    PCS_CHECK_ARG(G >= 1 && K >= 1 && N >= 1, "pcs_pool_bwd_reduce: bad sizes");
    const int gpb = 256;
    const dim3 grid((unsigned)((G + gpb - 1) / gpb), (N + 63) / 64);
    hipLaunchKernelGGL(pool_bwd_reduce_kernel, grid, dim3(256), 0, as_stream(stream), dpool, arg, Z, N, G, K, s, t,
                       mean, inv, act, slope, gpb, part);
    return launch_status("pcs_pool_bwd_reduce");
}

PCS_API int pcs_pool_bwd_dz(const float* dpool, const uint8_t* arg, const float* Z, int N, long long G, int K,
                            const float* s, const float* t, const float* mean, const float* inv, const float* kB,
                            const float* kC, int act, float slope, float* dZ, void* stream) {
    PCS_CHECK_ARG(G >= 0 && K >= 1 && N >= 1, "pcs_pool_bwd_dz: bad sizes");
    const long long total = G * K * N;
    if (total == 0) return 0;
    hipLaunchKernelGGL(pool_bwd_dz_kernel, dim3(ew_grid(total)), dim3(256), 0, as_stream(stream), dpool, arg, Z, N, G,
                       K, s, t, mean, inv, kB, kC, act, slope, dZ);
    return launch_status("pcs_pool_bwd_dz");
}

PCS_API int pcs_bn_act(const float* Z, int ldz, int M, int N, const float* s, const float* t, int act, float slope,
                       float* out, int ldo, void* stream) {
    PCS_CHECK_ARG(M >= 0 && N >= 1, "pcs_bn_act: bad sizes");
    const long long total = (long long)M * N;
    if (total == 0) return 0;
    hipLaunchKernelGGL(bn_act_kernel, dim3(ew_grid(total)), dim3(256), 0, as_stream(stream), Z, ldz, total, N, s, t,
                       act, slope, out, ldo);
    return launch_status("pcs_bn_act");
}
