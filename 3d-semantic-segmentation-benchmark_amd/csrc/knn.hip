// DGCNN dynamic-graph kNN (reference `knn`, models/dgcnn/dgcnn.py:7-21):
//   pd[i,j] = -|x_i|^2 - (-2 x_i.x_j) - |x_j|^2 ,  idx = topk(pd, k, largest)
//
// The reference evaluates x^T x with an MKL GEMM, so its rounding (and thus
// near-tie neighbour choices, ~0.05 % of rows) is not reproducible on any other
// device; parity for DGCNN uses neighbour-index replay and this
// kernel is checked by set agreement + distance-margin tests.
//
// One thread per query row keeps its feature vector and a sorted top-K list in
// registers; candidate points stream through LDS in 64-point tiles that every
// lane reads by broadcast, so the (B, N, N) distance matrix of the reference is
// never materialised.  Ties resolve to the lower index (strict > insertion).
#include "pcs_common.hpp"

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

template <int F, int K>
static void launch_knn(const float* x, int B, int N, int* out, hipStream_t s) {
    hipLaunchKernelGGL((knn_kernel<F, K>), dim3((N + 255) / 256, B), dim3(256), 0, s, x, N, out);
}

template <int F>
static int dispatch_k(const float* x, int B, int N, int k, int* out, hipStream_t s) {
    switch (k) {
        case 16: launch_knn<F, 16>(x, B, N, out, s); return 0;
        case 20: launch_knn<F, 20>(x, B, N, out, s); return 0;
        case 32: launch_knn<F, 32>(x, B, N, out, s); return 0;
        case 40: launch_knn<F, 40>(x, B, N, out, s); return 0;
        default:
            set_error("pcs_knn: k=%d not instantiated (16, 20, 32, 40)", k);
            return (int)hipErrorInvalidValue;
    }
}

}  // namespace pcs

// Reference: models/dgcnn/dgcnn.py:7-21.  x point-major (B, N, F) fp32; out (B, N, k) int32,
// best first.  F in {3, 64}; k in {16, 20, 32, 40}.
PCS_API int pcs_knn(const float* x, int B, int N, int F, int k, int32_t* out_idx, void* stream) {
    using namespace pcs;
    PCS_CHECK_ARG(B >= 0 && N >= 1 && k >= 1 && k <= N, "pcs_knn: bad sizes B=%d N=%d k=%d", B, N, k);
    PCS_CHECK_ARG(x && out_idx, "pcs_knn: null pointer");
    if (B == 0) return 0;
    hipStream_t s = as_stream(stream);
    int rc;
    switch (F) {
        case 3: rc = dispatch_k<3>(x, B, N, k, out_idx, s); break;
        case 64: rc = dispatch_k<64>(x, B, N, k, out_idx, s); break;
        default:
            set_error("pcs_knn: F=%d not instantiated (3, 64)", F);
            return (int)hipErrorInvalidValue;
    }
    if (rc) return rc;
    return launch_status("pcs_knn");
}
