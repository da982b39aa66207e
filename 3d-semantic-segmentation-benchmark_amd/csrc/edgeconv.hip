// Fused EdgeConv (reference `EdgeConv`, models/dgcnn/dgcnn.py:60-77, with
// `get_graph_feature`, dgcnn.py:24-57): per point i with neighbours j_1..j_k
//   z_(i,j) = W [x_j - x_i ; x_i]      (Conv2d 1x1, bias=False, over the (B, 2C, N, k) edge tensor)
//   out_i   = max_k LeakyReLU(BN_train(z_(i,j)))
//
// The edge tensor is never formed.  With W = [W1 | W2] (Cout x 2C):
//   z_(i,j) = W1 x_j - W1 x_i + W2 x_i = (Y_j - Y_i) + P_i ,   Y = X W1^T,  P = X W2^T
// so the 1x1 convolution runs over the N points (two row GEMMs on the engine, k = 20x fewer
// flops than over the N k edges) and one gather pass (edgeconv_fwd_kernel) forms every edge
// value once in registers: BatchNorm statistics (fp64 partials over all B N k edges, as the
// reference's BatchNorm2d), the running max over k (gamma >= 0) or min (gamma < 0) with its
// first index (the pooled output is act(s z + t), s = gamma invstd: monotone in z), and
// the per-point sum over k that the backward needs.
//
// Backward (training-mode BN): with dy nonzero only at each (i, c)'s argmax edge,
//   dZ_e = s dy_e - kB - kC (z_e - mean)                        (BN backward, per channel)
//   dP_i = sum_k dZ_(i,k) = D_i - k kB - kC (S_i - k mean)      (D = s dy at the argmax, S = sum_k z)
//   dY_m = sum_{e: j_e = m} dZ_e - dP_m                         (CSR inverse of the kNN graph)
//   dW   = [dY | dP]^T X ,  dX = dY W1 + dP W2                  (one wgrad, one data-gradient GEMM)
// The gradients are written interleaved, G[:, 2c] = dY_c and G[:, 2c+1] = dP_c, so that W
// read as a (2 Cout) x C matrix (row 2c = W1 row c, row 2c+1 = W2 row c) is W's own memory:
// dW = G^T X lands in W's layout and dX = G W_int needs no weight copy.
#include "mlp_common.hpp"

namespace pcs {

// neighbours per batch of the forward gather (one at a time, round 4, measured slower:
// profiles/r05_ab_edgeconv_gathers.txt)
constexpr int EC_FB = 8;

constexpr int kEdgeFwdBlocks = 1024;

// one thread = one point x 4 channels; 256 / (Cout/4) points per block, grid-stride over points
__global__ __launch_bounds__(256) void edgeconv_fwd_kernel(const float* __restrict__ Y, float* __restrict__ PQ,
                                                           const int32_t* __restrict__ idx, int N, int k, int Cout,
                                                           long long G, const float* __restrict__ sgn,
                                                           float* __restrict__ pz, unsigned char* __restrict__ pa,
                                                           float* __restrict__ S, double* __restrict__ part) {
    const int tq = Cout / 4;                       // threads per point
    const int pb = 256 / tq;                       // points per block pass
    const int slot = threadIdx.x / tq;
    const int c = 4 * (threadIdx.x - slot * tq);
    double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
    // one extreme per channel: the max of z where gamma > 0, the min (as the max of -z) where
    // gamma < 0; where gamma == 0 every edge pools to act(t) and the first (k = 0) is the argmax
    unsigned flip[4] = {0u, 0u, 0u, 0u};
    bool keep0[4] = {false, false, false, false};
    if (sgn && slot < pb) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            flip[q] = sgn[c + q] < 0.f ? 0x80000000u : 0u;
            keep0[q] = sgn[c + q] == 0.f;
        }
    }
    // XCD-aware point order: blocks b, b + 8, ... share an XCD (dispatch round-robin; speed
    // only), so XCD x takes the contiguous range [x Gx, (x+1) Gx) of points and its blocks sweep
    // it together, pb points each per pass: at any time an XCD gathers the Y rows of about one
    // cloud (1 MB at N = 4096, Cout = 64), which its 4 MB L2 holds
    const int nx = gridDim.x % 8 == 0 ? 8 : 1;
    const int xcd = blockIdx.x % nx, lb = blockIdx.x / nx, nl = gridDim.x / nx;
    const long long Gx = (G + nx - 1) / nx;
    const long long gx0 = (long long)xcd * Gx, gx1 = min(G, gx0 + Gx);
    if (slot < pb) {
        for (long long g = gx0 + (long long)lb * pb + slot; g < gx1; g += (long long)nl * pb) {
            const long long cloud = (g / N) * N;
            const float4 yi = *reinterpret_cast<const float4*>(Y + g * Cout + c);
            const float4 pi = *reinterpret_cast<const float4*>(PQ + g * Cout + c);
            const float yv[4] = {yi.x, yi.y, yi.z, yi.w}, pv[4] = {pi.x, pi.y, pi.z, pi.w};
            float mx[4], sm[4];
            int amx[4] = {0, 0, 0, 0};
            const int32_t* nb = idx + g * k;
            // EC_FB neighbours per batch: the batch's index loads, then all its Y-row gathers, are issued
            // before its arithmetic, which runs in neighbour order (the same sums and argmax as one
            // neighbour at a time); k = 20 takes three batches instead of 20 dependent index -> row rounds
            for (int k0 = 0; k0 < k; k0 += EC_FB) {
                int jb[EC_FB];
                float4 yb[EC_FB];
#pragma unroll
                for (int u = 0; u < EC_FB; ++u) jb[u] = k0 + u < k ? min(max(nb[k0 + u], 0), N - 1) : 0;
#pragma unroll
                for (int u = 0; u < EC_FB; ++u) {
                    PCS_DCHECK(cloud + jb[u] < G && c + 4 <= Cout, "edgeconv fwd Y row %lld col %d outside %lld x %d",
                               cloud + jb[u], c, G, Cout);
                    yb[u] = *reinterpret_cast<const float4*>(Y + (cloud + jb[u]) * Cout + c);
                }
#pragma unroll
                for (int u = 0; u < EC_FB; ++u) {
                    const int kk = k0 + u;
                    if (kk >= k) break;
                    const float jv[4] = {yb[u].x, yb[u].y, yb[u].z, yb[u].w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float z = __fadd_rn(__fsub_rn(jv[q], yv[q]), pv[q]);
                        const float zf = __uint_as_float(__float_as_uint(z) ^ flip[q]);
                        if (kk == 0) {
                            mx[q] = zf;
                            sm[q] = z;
                        } else {
                            if (zf > mx[q] && !keep0[q]) { mx[q] = zf; amx[q] = kk; }
                            sm[q] = __fadd_rn(sm[q], z);
                        }
                        s1[q] += (double)z;
                        s2[q] += (double)z * (double)z;
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) mx[q] = __uint_as_float(__float_as_uint(mx[q]) ^ flip[q]);
            *reinterpret_cast<float4*>(pz + g * Cout + c) = make_float4(mx[0], mx[1], mx[2], mx[3]);
            *reinterpret_cast<uchar4*>(pa + g * Cout + c) =
                make_uchar4((unsigned char)amx[0], (unsigned char)amx[1], (unsigned char)amx[2], (unsigned char)amx[3]);
            *reinterpret_cast<float4*>(S + g * Cout + c) = make_float4(sm[0], sm[1], sm[2], sm[3]);
            // P is replaced by Q = P - Y (the backward's per-source-point term)
            *reinterpret_cast<float4*>(PQ + g * Cout + c) =
                make_float4(__fsub_rn(pv[0], yv[0]), __fsub_rn(pv[1], yv[1]), __fsub_rn(pv[2], yv[2]),
                            __fsub_rn(pv[3], yv[3]));
        }
    }
    // block reduce of the BN partials over the point slots -> part[2][Cout][gridDim.x]
    __shared__ double red[2][256][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        red[0][threadIdx.x][q] = s1[q];
        red[1][threadIdx.x][q] = s2[q];
    }
    __syncthreads();
    if (threadIdx.x < tq) {
        for (int sl = 1; sl < pb; ++sl) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                s1[q] += red[0][sl * tq + threadIdx.x][q];
                s2[q] += red[1][sl * tq + threadIdx.x][q];
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            part[(size_t)(c + q) * gridDim.x + blockIdx.x] = s1[q];
            part[((size_t)Cout + c + q) * gridDim.x + blockIdx.x] = s2[q];
        }
    }
}

// BN-backward sums over the pooled edges (the only ones with dy != 0): part[2][Cout][gridDim.x]
__global__ __launch_bounds__(256) void edgeconv_bwd_reduce_kernel(const float* __restrict__ dout, int ldo,
                                                                  const float* __restrict__ pz, long long G, int Cout,
                                                                  const float* __restrict__ coef, float slope,
                                                                  int rows_per_block, double* __restrict__ part) {
    __shared__ double r1[4][64], r2[4][64];
    const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
    const int col = blockIdx.y * 64 + lane;
    const long long gb = (long long)blockIdx.x * rows_per_block;
    const long long ge = min(G, gb + rows_per_block);
    double a = 0.0, b = 0.0;
    if (col < Cout) {
        const float s = coef[col], t = coef[Cout + col], mean = coef[2 * Cout + col], inv = coef[3 * Cout + col];
#pragma unroll 4
        for (long long g = gb + ph; g < ge; g += 4) {
            const long long e = g * Cout + col;
            const float z = pz[e];              // the pooled (argmax) edge's z
            const float dy = dout[g * ldo + col] * dact_f(z * s + t, ACT_LRELU, slope);
            a += (double)dy;
            b += (double)dy * (double)((z - mean) * inv);
        }
    }
    r1[ph][lane] = a;
    r2[ph][lane] = b;
    __syncthreads();
    if (ph == 0 && col < Cout) {
        part[(size_t)col * gridDim.x + blockIdx.x] = r1[0][lane] + r1[1][lane] + r1[2][lane] + r1[3][lane];
        part[((size_t)Cout + col) * gridDim.x + blockIdx.x] = r2[0][lane] + r2[1][lane] + r2[2][lane] + r2[3][lane];
    }
}

// per (point, channel): D = s dy at the argmax edge, dP = D - k kB - kC (S - k mean) -> G[:, 2c+1]
__global__ __launch_bounds__(256) void edgeconv_bwd_center_kernel(const float* __restrict__ dout, int ldo,
                                                                  const float* __restrict__ pz,
                                                                  const float* __restrict__ S, long long G, int Cout,
                                                                  int k, const float* __restrict__ coef,
                                                                  const float* __restrict__ kBC, float slope,
                                                                  float* __restrict__ D, float* __restrict__ Gd) {
    const long long GN = G * Cout;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < GN; e += (long long)gridDim.x * 256) {
        const int c = (int)(e % Cout);
        const long long g = e / Cout;
        const float s = coef[c], t = coef[Cout + c], mean = coef[2 * Cout + c];
        const float kb = kBC[c], kc = kBC[Cout + c];
        const float z = pz[e];
        const float d = s * (dout[g * ldo + c] * dact_f(z * s + t, ACT_LRELU, slope));
        D[e] = d;
        const double dp = (double)d - (double)k * kb - (double)kc * ((double)S[e] - (double)k * mean);
        Gd[g * 2 * Cout + 2 * c + 1] = (float)dp;
    }
}

// the same, one channel quad per thread (Cout % 4 == 0, 16-B aligned rows): 16-B loads of dout /
// S / pz, a 16-B store of D and 32-bit quad indexing instead of a 64-bit division per element;
// Same per-element arithmetic.
__global__ __launch_bounds__(256) void edgeconv_bwd_center_q_kernel(const float4* __restrict__ dout, int ldo4,
                                                                    const float4* __restrict__ pz,
                                                                    const float4* __restrict__ S, int GN4, int nq,
                                                                    int k, const float* __restrict__ coef,
                                                                    const float* __restrict__ kBC, float slope,
                                                                    float4* __restrict__ D, float* __restrict__ Gd) {
    const int Cout = 4 * nq;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < GN4; e += gridDim.x * 256) {
        const int g = e / nq, c = 4 * (e - g * nq);
        const float4 sv = *reinterpret_cast<const float4*>(coef + c);
        const float4 tv = *reinterpret_cast<const float4*>(coef + Cout + c);
        const float4 mv = *reinterpret_cast<const float4*>(coef + 2 * Cout + c);
        const float4 kbv = *reinterpret_cast<const float4*>(kBC + c);
        const float4 kcv = *reinterpret_cast<const float4*>(kBC + Cout + c);
        const float4 z = pz[e];
        const float4 dv = dout[(size_t)g * ldo4 + (c >> 2)], Sv = S[e];
        const float s4[4] = {sv.x, sv.y, sv.z, sv.w}, t4[4] = {tv.x, tv.y, tv.z, tv.w};
        const float m4[4] = {mv.x, mv.y, mv.z, mv.w}, kb4[4] = {kbv.x, kbv.y, kbv.z, kbv.w};
        const float kc4[4] = {kcv.x, kcv.y, kcv.z, kcv.w}, z4[4] = {z.x, z.y, z.z, z.w};
        const float d4i[4] = {dv.x, dv.y, dv.z, dv.w}, S4[4] = {Sv.x, Sv.y, Sv.z, Sv.w};
        float d4[4];
        float* gr = Gd + (size_t)g * 2 * Cout + 2 * c + 1;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            d4[j] = s4[j] * (d4i[j] * dact_f(z4[j] * s4[j] + t4[j], ACT_LRELU, slope));
            const double dp = (double)d4[j] - (double)k * kb4[j] - (double)kc4[j] * ((double)S4[j] - (double)k * m4[j]);
            gr[2 * j] = (float)dp;
        }
        D[e] = make_float4(d4[0], d4[1], d4[2], d4[3]);
    }
}

// per target point m (one wave, lanes over channels): sum over the edges whose neighbour is m
//   G_in = sum [arg == kk] D_i  - cnt (kB + kC (Y_m - mean)) - kC sum Q_i ,  dY = G_in - dP_m -> G[:, 2c]
// (z_e = Y_m + Q_i; fp64 accumulation, so the unspecified CSR order does not change the result)
constexpr int EC_U = 4;                      // slot rows per batch (16 measured +0.11 ms on DGCNN)
__global__ __launch_bounds__(256) void edgeconv_bwd_gather_kernel(const float* __restrict__ Y,
                                                                  const float* __restrict__ Q,
                                                                  const float* __restrict__ D,
                                                                  const unsigned char* __restrict__ arg,
                                                                  const int32_t* __restrict__ off,
                                                                  const int32_t* __restrict__ ent, long long G,
                                                                  int Cout, int k, const float* __restrict__ coef,
                                                                  const float* __restrict__ kBC,
                                                                  float* __restrict__ Gd) {
    // XCD-aware order (bijective remap of the 1-D grid, speed only): XCD x takes a contiguous
    // run of target points, so the D / Q / arg rows its waves gather stay within ~one cloud
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
    const int tb = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
    const long long m = (long long)tb * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (m >= G) return;
    const int a = off[m], zend = off[m + 1];
    for (int c0 = 0; c0 < Cout; c0 += 64) {
        const int c = c0 + lane;
        const int cc = c < Cout ? c : Cout - 1;
        double accd = 0.0, accq = 0.0;
        for (int base = a; base < zend; base += 64) {
            const int n = min(64, zend - base);
            int row = 0, kk = 0;
            if (lane < n) {
                const int s = ent[base + lane];
                row = s / k;
                kk = s - row * k;
            }
            auto term = [&](int e, double& ad, double& aq) {
                const long long r = (long long)__builtin_amdgcn_readlane(row, e);
                const int kv = __builtin_amdgcn_readlane(kk, e);
                const size_t o = (size_t)r * Cout + cc;
                PCS_DCHECK(r >= 0 && r < G, "edgeconv bwd gather row %lld of %lld", r, G);
                const float dv = D[o];
                const float qv = Q[o];
                const int av = arg[o];
                ad += av == kv ? (double)dv : 0.0;
                aq += (double)qv;
            };
            int e = 0;
            // EC_U slot rows in flight per lane: all of a batch's loads are issued before its adds, which
            // then run in list order (the same fp64 sums as one slot at a time).  Lists average k entries,
            // so one or two batches cover a target instead of k / 4 dependent rounds of loads.
            for (; e + EC_U <= n; e += EC_U) {
                float dv[EC_U], qv[EC_U];
                int av[EC_U], kvs[EC_U];
#pragma unroll
                for (int u = 0; u < EC_U; ++u) {
                    const long long r = (long long)__builtin_amdgcn_readlane(row, e + u);
                    kvs[u] = __builtin_amdgcn_readlane(kk, e + u);
                    const size_t o = (size_t)r * Cout + cc;
                    PCS_DCHECK(r >= 0 && r < G, "edgeconv bwd gather row %lld of %lld", r, G);
                    dv[u] = D[o];
                    qv[u] = Q[o];
                    av[u] = arg[o];
                }
#pragma unroll
                for (int u = 0; u < EC_U; ++u) {
                    accd += av[u] == kvs[u] ? (double)dv[u] : 0.0;
                    accq += (double)qv[u];
                }
            }
            for (; e + 4 <= n; e += 4) {
                term(e, accd, accq);
                term(e + 1, accd, accq);
                term(e + 2, accd, accq);
                term(e + 3, accd, accq);
            }
            for (; e < n; ++e) term(e, accd, accq);
        }
        if (c < Cout) {
            const double cnt = (double)(zend - a);
            const double kb = kBC[c], kc = kBC[Cout + c], mean = coef[2 * Cout + c];
            const double ym = Y[m * Cout + c];
            const double gin = accd - cnt * (kb + kc * (ym - mean)) - kc * accq;
            const size_t go = (size_t)m * 2 * Cout + 2 * c;
            Gd[go] = (float)(gin - (double)Gd[go + 1]);
        }
    }
}

static pcs_operand plain(const float* p, int ld) {
    pcs_operand o{};
    o.data = p;
    o.ld = ld;
    o.mode = PCS_OP_PLAIN;
    return o;
}

static int fwd_blocks(long long G, int Cout) {
    const long long pb = 256 / (Cout / 4);
    const long long need = (G + pb - 1) / pb;
    const long long nb = std::min<long long>(kEdgeFwdBlocks, std::max<long long>(need, 1));
    return (int)(nb >= 8 ? (nb + 7) / 8 * 8 : nb);         // a multiple of 8: the XCD-aware order
}

static const int kEdgeRedRows = 512;

}  // namespace pcs

using namespace pcs;

PCS_API int pcs_edgeconv_workspace(int B, int N, int C, int Cout, int backward, size_t* bytes) {
    PCS_CHECK_ARG(bytes && B >= 1 && N >= 1 && C >= 1 && Cout >= 4, "pcs_edgeconv_workspace: bad arguments");
    const long long G = (long long)B * N;
    if (!backward) {
        *bytes = (size_t)fwd_blocks(G, Cout) * 2 * Cout * sizeof(double);
    } else {
        const long long nb = (G + kEdgeRedRows - 1) / kEdgeRedRows;
        // G (interleaved dY|dP) + D + kB/kC + reduce partials + the weight gradient's partial tiles
        *bytes = (size_t)G * 2 * Cout * 4 + (size_t)G * Cout * 4 + (size_t)2 * Cout * 4 + 256 +
                 (size_t)nb * 2 * Cout * sizeof(double) + 256 + wgrad_ws_bytes(2 * Cout, C, (int)G);
    }
    return 0;
}

// Training-mode EdgeConv forward.  X (B*N rows, stride ldx) with C channels, idx (B, N, k)
// int32 neighbour table (per-cloud indices), W (Cout, 2C) = the Conv2d weight, BN gamma/beta
// and running stats (updated in place, num_batches_tracked bumped).  Outputs (caller-owned):
// Y, PQ (B*N x Cout; PQ holds Q = P - Y on return), S (B*N x Cout), pz (B*N x Cout: the pooled
// edge's z -- max over k (gamma > 0), min (< 0), edge 0 (== 0)), pa (B*N x Cout u8: its slot), coef (4 x Cout: s, t, mean, invstd), out (B*N x Cout) pooled
// activation, arg (B*N x Cout u8) its neighbour slot.  Reference: dgcnn.py:60-77.
PCS_API int pcs_edgeconv_fwd(const float* X, int ldx, int C, const int32_t* idx, int B, int N, int k,
                             const float* W, int Cout, const float* gamma, const float* beta, float* run_mean,
                             float* run_var, long long* num_batches, float momentum, float eps, float slope,
                             float* Y, float* PQ, float* S, float* pz, unsigned char* pa, float* coef, float* out,
                             unsigned char* arg, float* out2, int ld2, void* workspace, size_t ws_bytes,
                             void* stream) {
    PCS_CHECK_ARG(B >= 1 && N >= 1 && k >= 1 && k <= 256 && C >= 1 && Cout >= 4 && Cout % 4 == 0 && Cout <= 1024,
                  "pcs_edgeconv_fwd: bad sizes B=%d N=%d k=%d C=%d Cout=%d", B, N, k, C, Cout);
    PCS_CHECK_ARG(X && idx && W && Y && PQ && S && pz && pa && coef && out && arg && workspace,
                  "pcs_edgeconv_fwd: null pointer");
    PCS_CHECK_ARG(!out2 || ld2 >= Cout, "pcs_edgeconv_fwd: out2 stride %d < Cout=%d", ld2, Cout);
    const long long G = (long long)B * N;
    PCS_CHECK_ARG(G * k < (1ll << 31), "pcs_edgeconv_fwd: too many edges");
    size_t need = 0;
    pcs_edgeconv_workspace(B, N, C, Cout, 0, &need);
    PCS_CHECK_ARG(ws_bytes >= need, "pcs_edgeconv_fwd: workspace %zu < %zu bytes", ws_bytes, need);
    hipStream_t st = as_stream(stream);
    const pcs_operand xa = plain(X, ldx);
    // Y = X W1^T, P = X W2^T: W's rows read with stride 2C (W2 starts C floats in)
    if (int e = gemm_rows_ex(&xa, (int)G, C, W, 2 * C, 0, nullptr, Y, Cout, Cout, nullptr, nullptr, nullptr, stream))
        return e;
    if (int e = gemm_rows_ex(&xa, (int)G, C, W + C, 2 * C, 0, nullptr, PQ, Cout, Cout, nullptr, nullptr, nullptr,
                             stream))
        return e;
    double* part = static_cast<double*>(workspace);
    const int nb = fwd_blocks(G, Cout);
    {
        // compulsory bytes: Y, Q and idx read once, (max z, min z, S) fp32 + 2 argmax u8 written;
        // flops: the k edge values (2 adds) and BN sums (3) per (point, channel)
        ProbeScope pr(st, 5.0 * (double)G * k * Cout, 4.0 * (double)G * (2.0 * Cout + k) + 14.0 * (double)G * Cout,
                      "pcs::edgeconv_fwd_kernel");
        hipLaunchKernelGGL(edgeconv_fwd_kernel, dim3(nb), dim3(256), 0, st, Y, PQ, idx, N, k, Cout, G, gamma, pz, pa, S, part);
    }
    bn_finalize_launch(part, nb, Cout, G * k, gamma, beta, eps, momentum, run_mean, run_var, coef, coef + Cout,
                       coef + 2 * Cout, coef + 3 * Cout, num_batches, st);
    return pool_finalize(pz, pa, G, Cout, coef, coef + Cout, ACT_LRELU, slope, out, arg, st, out2, ld2);
}

// Training-mode EdgeConv backward (the forward's saved tensors; csr_off/csr_ent = pcs_inverse_index
// of idx with targets N).  Accumulates dW (Cout x 2C), dgamma, dbeta (+=); writes dX (nullable,
// stride lddx, C % 4 == 0).  dout: gradient of the pooled output (B*N x Cout, row stride ldo >= Cout: a
// column block of a wider gradient -- DGCNN's head concatenation -- is read in place).
PCS_API int pcs_edgeconv_bwd(const float* X, int ldx, int C, const int32_t* csr_off, const int32_t* csr_ent, int B,
                             int N, int k, const float* W, int Cout, const float* Y, const float* Q, const float* S,
                             const float* pz, const unsigned char* arg, const float* coef, float slope,
                             const float* dout, int ldo, float* dX, int lddx, float* dW, float* dgamma,
                             float* dbeta, void* workspace, size_t ws_bytes, void* stream) {
    PCS_CHECK_ARG(B >= 1 && N >= 1 && k >= 1 && k <= 256 && C >= 1 && Cout >= 4 && Cout % 4 == 0 && Cout <= 1024,
                  "pcs_edgeconv_bwd: bad sizes B=%d N=%d k=%d C=%d Cout=%d", B, N, k, C, Cout);
    PCS_CHECK_ARG(X && csr_off && csr_ent && W && Y && Q && S && pz && arg && coef && dout && dW && workspace,
                  "pcs_edgeconv_bwd: null pointer");
    PCS_CHECK_ARG(!dX || (C % 4 == 0 && lddx >= C && lddx % 4 == 0), "pcs_edgeconv_bwd: dX needs C %% 4 == 0");
    PCS_CHECK_ARG(ldo >= Cout, "pcs_edgeconv_bwd: dout row stride %d < Cout=%d", ldo, Cout);
    const long long G = (long long)B * N;
    size_t need = 0;
    pcs_edgeconv_workspace(B, N, C, Cout, 1, &need);
    PCS_CHECK_ARG(ws_bytes >= need, "pcs_edgeconv_bwd: workspace %zu < %zu bytes", ws_bytes, need);
    hipStream_t st = as_stream(stream);
    char* w = static_cast<char*>(workspace);
    float* Gd = reinterpret_cast<float*>(w);
    w += (size_t)G * 2 * Cout * 4;
    float* D = reinterpret_cast<float*>(w);
    w += (size_t)G * Cout * 4;
    float* kBC = reinterpret_cast<float*>(w);
    w += (size_t)2 * Cout * 4;
    w = reinterpret_cast<char*>(((uintptr_t)w + 255) & ~(uintptr_t)255);
    double* part = reinterpret_cast<double*>(w);
    const int nb = (int)((G + kEdgeRedRows - 1) / kEdgeRedRows);
    w += (size_t)nb * 2 * Cout * sizeof(double);
    w = reinterpret_cast<char*>(((uintptr_t)w + 255) & ~(uintptr_t)255);
    const size_t wg_bytes = wgrad_ws_bytes(2 * Cout, C, (int)G);
    hipLaunchKernelGGL(edgeconv_bwd_reduce_kernel, dim3(nb, (Cout + 63) / 64), dim3(256), 0, st, dout, ldo, pz, G, Cout,
                       coef, slope, kEdgeRedRows, part);
    bn_bwd_finalize_launch(part, nb, Cout, G * k, coef, coef + 3 * Cout, dgamma, dbeta, kBC, kBC + Cout, 1, st);
    const long long GN = G * Cout;
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (Cout % 4 == 0 && ldo % 4 == 0 && GN / 4 < (1ll << 31) && al16(dout) && al16(pz) && al16(S) && al16(D) &&
        al16(coef) && al16(kBC)) {
        const long long GN4 = GN / 4;
        const unsigned eq = (unsigned)std::min<long long>((GN4 + 255) / 256, 65536);
        hipLaunchKernelGGL(edgeconv_bwd_center_q_kernel, dim3(eq), dim3(256), 0, st,
                           reinterpret_cast<const float4*>(dout), ldo / 4, reinterpret_cast<const float4*>(pz),
                           reinterpret_cast<const float4*>(S), (int)GN4, Cout / 4, k, coef, kBC, slope,
                           reinterpret_cast<float4*>(D), Gd);
    } else {
        const unsigned eg = (unsigned)std::min<long long>((GN + 255) / 256, 65536);
        hipLaunchKernelGGL(edgeconv_bwd_center_kernel, dim3(eg), dim3(256), 0, st, dout, ldo, pz, S, G, Cout, k, coef,
                           kBC, slope, D, Gd);
    }
    {
        // compulsory bytes: Y, Q, D, arg and the inverse map read once, the (dY | dP) rows written
        ProbeScope pr(st, 0.0, 4.0 * (double)G * Cout * 3 + (double)G * Cout + 4.0 * (double)G * (k + 1) +
                                   8.0 * (double)G * Cout, "pcs::edgeconv_bwd_gather_kernel");
        hipLaunchKernelGGL(edgeconv_bwd_gather_kernel, dim3((unsigned)((G + 3) / 4)), dim3(256), 0, st, Y, Q, D, arg,
                           csr_off, csr_ent, G, Cout, k, coef, kBC, Gd);
    }
    if (int e = launch_status("pcs_edgeconv_bwd")) return e;
    // dW (as 2Cout x C) += G^T X ;  dX = G W_int
    const pcs_operand ga = plain(Gd, 2 * Cout);
    const pcs_operand xa = plain(X, ldx);
    if (int e = wgrad_launch(&ga, 2 * Cout, &xa, C, (int)G, dW, nullptr, w, wg_bytes, stream)) return e;
    if (dX)
        if (int e = gemm_rows_ex(&ga, (int)G, 2 * Cout, W, C, 1, nullptr, dX, lddx, C, nullptr, nullptr, nullptr,
                                 stream))
            return e;
    return 0;
}
