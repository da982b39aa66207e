// Gather / scatter kernels around the neighbour indices (HBM-bound):
//   group fwd/bwd     reference `group` gather + centroid subtract (+ /r)      common.py:62-71
//   maxk fwd/bwd      reference `reduce(..., 'max')` over the K axis              common.py:85-86
//   interp fwd/bwd    reference `interpolate` IDW sum over the 3 neighbours       common.py:115-122
//   edge fwd/bwd      reference `get_graph_feature` cat(x_j - x_i, x_i)           dgcnn.py:41-53
//
// Layout: point-major rows, (rows, channels) row-contiguous fp32, so every
// neighbour fetch is one contiguous channel vector (coalesced across lanes).
// Backward scatters use fp32 atomics (global_atomic_add_f32); forward results
// are bit-exact with the reference's CPU arithmetic order.
#include "pcs_common.hpp"

namespace pcs {

__device__ __forceinline__ long long gtid() { return (long long)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ long long gstride() { return (long long)gridDim.x * blockDim.x; }

static inline dim3 grid_for(long long n, int block = 256) {
    long long g = (n + block - 1) / block;
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    return dim3((unsigned)g);
}

// ------------------------------------------------------------------ group
__global__ void group_fwd_kernel(const float* __restrict__ xyz, const float* __restrict__ feats,
                                 const float* __restrict__ cent, const int* __restrict__ idx, int C, int N, int K,
                                 int D, float r, int normalize, float* __restrict__ out, int ld, long long total) {
    for (long long t = gtid(); t < total; t += gstride()) {
        const long long row = t / ld;
        const int ch = (int)(t - row * ld);
        const long long g = row / K;          // centroid row b*C + c
        const int b = (int)(g / C);
        const int p = idx[row];
        float v;
        if (ch >= 3 + D) {
            v = 0.f;                          // row padding (keeps rows 16-B aligned for the GEMM)
        } else if (ch < 3) {
            v = xyz[((long long)b * N + p) * 3 + ch] - cent[g * 3 + ch];
            if (normalize) v = v / r;
        } else {
            v = feats[((long long)b * N + p) * D + (ch - 3)];
        }
        out[t] = v;
    }
}

// one thread per (row, 4 output channels): same per-element arithmetic, one 16-B store
// (ld % 4 == 0; rows are 16-B aligned).  I: the index type -- int whenever the quad count fits
// (every bench shape): three 64-bit divisions per quad were a large share of its VALU work
template <typename I>
__global__ __launch_bounds__(256) void group_fwd_q_kernel(const float* __restrict__ xyz,
                                                          const float* __restrict__ feats,
                                                          const float* __restrict__ cent, const int* __restrict__ idx,
                                                          int C, int N, int K, int D, float r, int normalize,
                                                          float* __restrict__ out, int nq, I total) {
    for (I t = (I)blockIdx.x * 256 + threadIdx.x; t < total; t += (I)gridDim.x * 256) {
        const I row = t / nq;
        const int q = (int)(t - row * nq);
        const I g = row / K;                  // centroid row b*C + c
        const int b = (int)(g / C);
        const long long pb = (long long)b * N + idx[row];
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int ch = 4 * q + e;
            float x;
            if (ch < 3) {
                x = xyz[pb * 3 + ch] - cent[g * 3 + ch];
                if (normalize) x = x / r;
            } else if (ch < 3 + D) {
                x = feats[pb * D + (ch - 3)];
            } else {
                x = 0.f;
            }
            v[e] = x;
        }
        reinterpret_cast<float4*>(out)[(long long)t] = make_float4(v[0], v[1], v[2], v[3]);
    }
}

// ------------------------------------------------------------------ max over K
__global__ void maxk_fwd_kernel(const float* __restrict__ x, int K, int Ch, float* __restrict__ out,
                                unsigned char* __restrict__ arg, long long total) {
    for (long long t = gtid(); t < total; t += gstride()) {
        const long long g = t / Ch;
        const int ch = (int)(t - g * Ch);
        const float* base = x + g * K * Ch + ch;
        float m = base[0];
        int a = 0;
        for (int k = 1; k < K; ++k) {
            const float v = base[(long long)k * Ch];
            if (v > m || (v != v && m == m)) { m = v; a = k; }   // first max; NaN propagates like torch.max
        }
        out[t] = m;
        arg[t] = (unsigned char)a;
    }
}

__global__ void maxk_bwd_kernel(const float* __restrict__ gout, const unsigned char* __restrict__ arg, int K,
                                int Ch, float* __restrict__ gx, long long total) {
    for (long long t = gtid(); t < total; t += gstride()) {
        const long long row = t / Ch;           // g*K + k
        const int ch = (int)(t - row * Ch);
        const long long g = row / K;
        const int k = (int)(row - g * K);
        const long long o = g * Ch + ch;
        gx[t] = (arg[o] == k) ? gout[o] : 0.f;
    }
}

// ------------------------------------------------------------------ 3-NN IDW interpolation
// out[b,n, col_off + ch] (row stride ld_out) = sum_k (p[idx_k] * w_k) / norm,  w_k = 1/(d_k + 1e-9)
__global__ void interp_fwd_kernel(const float* __restrict__ pts, const int* __restrict__ idx,
                                  const float* __restrict__ dist, int N, int M, int D, float* __restrict__ out,
                                  int ld_out, int col_off, long long total) {
    for (long long t = gtid(); t < total; t += gstride()) {
        const long long row = t / D;            // b*N + n
        const int ch = (int)(t - row * D);
        const int b = (int)(row / N);
        const float w0 = 1.0f / (dist[row * 3 + 0] + 1e-9f);
        const float w1 = 1.0f / (dist[row * 3 + 1] + 1e-9f);
        const float w2 = 1.0f / (dist[row * 3 + 2] + 1e-9f);
        const float nrm = (w0 + w1) + w2;
        const float* P = pts + (long long)b * M * D + ch;
        const float t0 = (P[(long long)idx[row * 3 + 0] * D] * w0) / nrm;
        const float t1 = (P[(long long)idx[row * 3 + 1] * D] * w1) / nrm;
        const float t2 = (P[(long long)idx[row * 3 + 2] * D] * w2) / nrm;
        out[row * ld_out + col_off + ch] = (t0 + t1) + t2;
    }
}

// [f1 | IDW-interpolate(pts)] rows in one pass, one thread per (row, 4 channels): the
// skip features are copied, the interpolated quad uses float4 gathers of the three
// neighbours with the scalar kernel's per-element arithmetic.  D1, D2, ld_out % 4 == 0.
template <typename I>
__global__ __launch_bounds__(256) void interp_cat_q_kernel(const float* __restrict__ f1, int D1,
                                                           const float* __restrict__ pts,
                                                           const int* __restrict__ idx,
                                                           const float* __restrict__ dist, int N, int M, int D2,
                                                           float* __restrict__ out, int ldq, I total) {
    const int q1 = D1 / 4, nq = q1 + D2 / 4;
    for (I t = (I)blockIdx.x * 256 + threadIdx.x; t < total; t += (I)gridDim.x * 256) {
        const long long row = (long long)(t / nq);           // b*N + n
        const int q = (int)(t - (I)row * nq);
        float4 o;
        if (q < q1) {
            o = reinterpret_cast<const float4*>(f1)[row * q1 + q];
        } else {
            const int b = (int)(row / N);
            const float w0 = 1.0f / (dist[row * 3 + 0] + 1e-9f);
            const float w1 = 1.0f / (dist[row * 3 + 1] + 1e-9f);
            const float w2 = 1.0f / (dist[row * 3 + 2] + 1e-9f);
            const float nrm = (w0 + w1) + w2;
            const float4* P = reinterpret_cast<const float4*>(pts + (long long)b * M * D2) + (q - q1);
            const int dq = D2 / 4;
            const float4 a = P[(long long)idx[row * 3 + 0] * dq];
            const float4 c = P[(long long)idx[row * 3 + 1] * dq];
            const float4 d = P[(long long)idx[row * 3 + 2] * dq];
            o.x = ((a.x * w0) / nrm + (c.x * w1) / nrm) + (d.x * w2) / nrm;
            o.y = ((a.y * w0) / nrm + (c.y * w1) / nrm) + (d.y * w2) / nrm;
            o.z = ((a.z * w0) / nrm + (c.z * w1) / nrm) + (d.z * w2) / nrm;
            o.w = ((a.w * w0) / nrm + (c.w * w1) / nrm) + (d.w * w2) / nrm;
        }
        reinterpret_cast<float4*>(out)[row * ldq + q] = o;
    }
}

// ------------------------------------------------------------------ EdgeConv graph feature
// out row (b,i,j) = [x[nbr] - x[i], x[i]]  (2D channels, row stride W >= 2D, pad zeroed),
// x point-major (B, N, D)
__global__ void edge_fwd_kernel(const float* __restrict__ x, const int* __restrict__ idx, int N, int k, int D,
                                int W, float* __restrict__ out, long long total) {
    for (long long t = gtid(); t < total; t += gstride()) {
        const long long row = t / W;            // (b*N + i)*k + j
        const int ch = (int)(t - row * W);
        const long long pi = row / k;           // b*N + i
        const int b = (int)(pi / N);
        if (ch >= 2 * D) { out[t] = 0.f; continue; }
        const float xi = x[pi * D + (ch < D ? ch : ch - D)];
        if (ch < D) {
            const int p = idx[row];
            out[t] = x[((long long)b * N + p) * D + ch] - xi;
        } else {
            out[t] = xi;
        }
    }
}

}  // namespace pcs

using namespace pcs;

// Reference: models/utils/common.py:62-71.  out (B*C*K, 3+D).
PCS_API int pcs_group_fwd(const float* xyz, const float* feats, const float* centroids, const int32_t* idx, int B,
                          int N, int C, int K, int D, float r, int normalize, float* out, int ld_out, void* stream) {
    PCS_CHECK_ARG(B >= 0 && N >= 1 && C >= 0 && K >= 1 && D >= 0 && ld_out >= 3 + D, "pcs_group_fwd: bad sizes");
    PCS_CHECK_ARG(xyz && centroids && idx && out && (D == 0 || feats), "pcs_group_fwd: null pointer");
    const long long total = (long long)B * C * K * ld_out;
    if (total == 0) return 0;
    if (ld_out % 4 == 0 && (uintptr_t)out % 16 == 0) {
        // algorithmic bytes (SURVEY.md 8(d) group fwd): source points + centroids + idx read once,
        // the grouped rows written
        ProbeScope pr(as_stream(stream), 0.0,
                      4.0 * ((double)B * N * (3 + D) + 3.0 * B * C + (double)B * C * K) + 4.0 * (double)total,
                      "pcs::group_fwd_q_kernel");
        if (total / 4 < (1ll << 31) - 65536 * 256)
            hipLaunchKernelGGL(group_fwd_q_kernel<int>, grid_for(total / 4), dim3(256), 0, as_stream(stream), xyz,
                               feats, centroids, idx, C, N, K, D, r, normalize, out, ld_out / 4, (int)(total / 4));
        else
            hipLaunchKernelGGL(group_fwd_q_kernel<long long>, grid_for(total / 4), dim3(256), 0, as_stream(stream), xyz,
                               feats, centroids, idx, C, N, K, D, r, normalize, out, ld_out / 4, total / 4);
        return launch_status("pcs_group_fwd");
    }
    hipLaunchKernelGGL(group_fwd_kernel, grid_for(total), dim3(256), 0, as_stream(stream), xyz, feats, centroids,
                       idx, C, N, K, D, r, normalize, out, ld_out, total);
    return launch_status("pcs_group_fwd");
}

// Reference: common.py:85-86.  x (G*K, Ch) -> out (G, Ch), argmax (G, Ch) u8 (first max).
PCS_API int pcs_maxk_fwd(const float* x, long long G, int K, int Ch, float* out, uint8_t* argmax, void* stream) {
    PCS_CHECK_ARG(G >= 0 && K >= 1 && K <= 256 && Ch >= 1, "pcs_maxk_fwd: bad sizes (K must be 1..256)");
    const long long total = G * Ch;
    if (total == 0) return 0;
    PCS_CHECK_ARG(x && out && argmax, "pcs_maxk_fwd: null pointer");
    hipLaunchKernelGGL(maxk_fwd_kernel, grid_for(total), dim3(256), 0, as_stream(stream), x, K, Ch, out, argmax,
                       total);
    return launch_status("pcs_maxk_fwd");
}

PCS_API int pcs_maxk_bwd(const float* grad_out, const uint8_t* argmax, long long G, int K, int Ch, float* grad_x,
                         void* stream) {
    PCS_CHECK_ARG(G >= 0 && K >= 1 && K <= 256 && Ch >= 1, "pcs_maxk_bwd: bad sizes");
    const long long total = G * K * Ch;
    if (total == 0) return 0;
    PCS_CHECK_ARG(grad_out && argmax && grad_x, "pcs_maxk_bwd: null pointer");
    hipLaunchKernelGGL(maxk_bwd_kernel, grid_for(total), dim3(256), 0, as_stream(stream), grad_out, argmax, K, Ch,
                       grad_x, total);
    return launch_status("pcs_maxk_bwd");
}

// Reference: common.py:115-122.  pts (B, M, D); idx/dist (B, N, 3) from pcs_knn_select;
// out[(b*N+n)*ld_out + col_off + ch].
PCS_API int pcs_interp_fwd(const float* pts, const int32_t* idx, const float* dist, int B, int N, int M, int D,
                           float* out, int ld_out, int col_off, void* stream) {
    PCS_CHECK_ARG(B >= 0 && N >= 0 && M >= 3 && D >= 1 && ld_out >= col_off + D && col_off >= 0,
                  "pcs_interp_fwd: bad sizes");
    const long long total = (long long)B * N * D;
    if (total == 0) return 0;
    PCS_CHECK_ARG(pts && idx && dist && out, "pcs_interp_fwd: null pointer");
    if (D % 4 == 0 && col_off % 4 == 0 && ld_out % 4 == 0 && ((uintptr_t)out | (uintptr_t)pts) % 16 == 0) {
        // the interpolated columns as the f1-less case of the fused kernel, shifted by col_off
        const long long rows = (long long)B * N;
        if (rows * (D / 4) < (1ll << 31) - 65536 * 256)
            hipLaunchKernelGGL(interp_cat_q_kernel<int>, grid_for(rows * (D / 4)), dim3(256), 0, as_stream(stream),
                               (const float*)nullptr, 0, pts, idx, dist, N, M, D, out + col_off, ld_out / 4,
                               (int)(rows * (D / 4)));
        else
            hipLaunchKernelGGL(interp_cat_q_kernel<long long>, grid_for(rows * (D / 4)), dim3(256), 0,
                               as_stream(stream), (const float*)nullptr, 0, pts, idx, dist, N, M, D, out + col_off,
                               ld_out / 4, rows * (D / 4));
        return launch_status("pcs_interp_fwd");
    }
    hipLaunchKernelGGL(interp_fwd_kernel, grid_for(total), dim3(256), 0, as_stream(stream), pts, idx, dist, N, M, D,
                       out, ld_out, col_off, total);
    return launch_status("pcs_interp_fwd");
}

// Reference: dgcnn.py:41-53.  x (B, N, D) point-major; idx (B, N, k); out (B*N*k, 2D).
PCS_API int pcs_edge_fwd(const float* x, const int32_t* idx, int B, int N, int k, int D, float* out, int ld_out,
                         void* stream) {
    PCS_CHECK_ARG(B >= 0 && N >= 1 && k >= 1 && D >= 1 && ld_out >= 2 * D, "pcs_edge_fwd: bad sizes");
    const long long total = (long long)B * N * k * ld_out;
    if (total == 0) return 0;
    PCS_CHECK_ARG(x && idx && out, "pcs_edge_fwd: null pointer");
    hipLaunchKernelGGL(edge_fwd_kernel, grid_for(total), dim3(256), 0, as_stream(stream), x, idx, N, k, D, ld_out, out,
                       total);
    return launch_status("pcs_edge_fwd");
}

// Reference FeaturePropagation (common.py:115-122, 238-240): rows (B*N, ld_out) =
// [f1 (B, N, D1) | interpolate(pts (B, M, D2))] in one pass; D1, D2, ld_out multiples of 4
// with ld_out >= D1 + D2 (the pad columns are not written).  f1 may be null when D1 == 0.
PCS_API int pcs_interp_cat_fwd(const float* f1, int D1, const float* pts, const int32_t* idx, const float* dist,
                               int B, int N, int M, int D2, float* out, int ld_out, void* stream) {
    PCS_CHECK_ARG(B >= 0 && N >= 0 && M >= 3 && D2 >= 4 && D1 >= 0 && ld_out >= D1 + D2, "pcs_interp_cat_fwd: bad sizes");
    PCS_CHECK_ARG(D1 % 4 == 0 && D2 % 4 == 0 && ld_out % 4 == 0, "pcs_interp_cat_fwd: D1, D2, ld_out must be multiples of 4");
    PCS_CHECK_ARG(pts && idx && dist && out && (D1 == 0 || f1), "pcs_interp_cat_fwd: null pointer");
    PCS_CHECK_ARG(((uintptr_t)out | (uintptr_t)pts | (uintptr_t)f1) % 16 == 0, "pcs_interp_cat_fwd: 16-B alignment");
    const long long total = (long long)B * N * ((D1 + D2) / 4);
    if (total == 0) return 0;
    // algorithmic bytes (SURVEY.md 8(d) interp fwd): coarse features + skip + (idx, dist) read
    // once, the concatenated rows written
    ProbeScope pr(as_stream(stream), 9.0 * (double)B * N * D2,
                  4.0 * ((double)B * M * D2 + (double)B * N * D1 + 6.0 * B * N + (double)B * N * (D1 + D2)),
                  "pcs::interp_cat_q_kernel");
    if (total < (1ll << 31) - 65536 * 256)
        hipLaunchKernelGGL(interp_cat_q_kernel<int>, grid_for(total), dim3(256), 0, as_stream(stream), f1, D1, pts, idx,
                           dist, N, M, D2, out, ld_out / 4, (int)total);
    else
        hipLaunchKernelGGL(interp_cat_q_kernel<long long>, grid_for(total), dim3(256), 0, as_stream(stream), f1, D1, pts,
                           idx, dist, N, M, D2, out, ld_out / 4, total);
    return launch_status("pcs_interp_cat_fwd");
}
