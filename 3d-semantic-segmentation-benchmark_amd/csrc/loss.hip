// Masked one-hot cross entropy, forward + gradient in one pass.
//
// Reference: Training/train_model.py:15-57 `masked_onehot_cross_entropy`:
//   lp   = log_softmax(logits, -1)                     (B, L, C)
//   tok  = -sum_c onehot[c] * lp[c]                     (B, L)
//   mask = position < length[b]
//   loss = sum(tok * mask) / sum(mask)   (0 when every position is padding)
// One thread per (b, l) row (C is the class count, 13/14 here); the same pass
// writes d loss / d logits = mask * (softmax * sum(onehot) - onehot) / count, so the
// backward is a single scale by the incoming gradient.  Block partial sums are
// fp64 and reduced by a second one-block kernel (deterministic).
#include "pcs_common.hpp"

namespace pcs {

constexpr int kCeBlock = 256;
constexpr int kCeMaxC = 64;

template <typename T>
__device__ __forceinline__ float tgt_at(const T* p) { return (float)*p; }

template <typename T>
__global__ __launch_bounds__(kCeBlock) void masked_ce_kernel(const float* __restrict__ logits, int ld,
                                                             const T* __restrict__ tgt, int ldt,
                                                             const int32_t* __restrict__ lengths, int B, int L, int C,
                                                             double* __restrict__ partial,
                                                             float* __restrict__ grad) {
    __shared__ double red[kCeBlock / 64];
    __shared__ float s_inv_count;
    if (threadIdx.x == 0) {
        long long cnt = 0;
        for (int b = 0; b < B; ++b) cnt += min(max(lengths[b], 0), L);
        s_inv_count = cnt > 0 ? 1.0f / (float)cnt : 0.f;
    }
    __syncthreads();
    const float inv_count = s_inv_count;
    const long long row = (long long)blockIdx.x * kCeBlock + threadIdx.x;
    double acc = 0.0;
    if (row < (long long)B * L) {
        const int b = (int)(row / L), l = (int)(row - (long long)b * L);
        const bool valid = l < lengths[b];
        const float* x = logits + row * ld;
        const T* y = tgt + row * ldt;
        float m = x[0];
        for (int c = 1; c < C; ++c) m = fmaxf(m, x[c]);
        float se = 0.f;
        for (int c = 0; c < C; ++c) se += expf(x[c] - m);
        const float lse = logf(se);
        float tok = 0.f, ysum = 0.f;
        for (int c = 0; c < C; ++c) {
            const float yc = tgt_at(y + c);
            tok -= yc * (x[c] - m - lse);
            ysum += yc;
        }
        if (valid) acc = (double)tok;
        if (grad) {
            float* g = grad + row * ld;
            const float w = valid ? inv_count : 0.f;
            for (int c = 0; c < C; ++c) g[c] = w * (expf(x[c] - m - lse) * ysum - tgt_at(y + c));
        }
    }
    // block reduction (fp64)
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int w = 0; w < kCeBlock / 64; ++w) s += red[w];
        partial[blockIdx.x] = s;
    }
}

__global__ __launch_bounds__(256) void masked_ce_final_kernel(const double* __restrict__ partial, int nb,
                                                              const int32_t* __restrict__ lengths, int B, int L,
                                                              float* __restrict__ loss) {
    __shared__ double red[256];
    double s = 0.0;
    for (int i = threadIdx.x; i < nb; i += 256) s += partial[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        long long cnt = 0;
        for (int b = 0; b < B; ++b) cnt += min(max(lengths[b], 0), L);
        loss[0] = cnt > 0 ? (float)(red[0] / (double)cnt) : 0.f;
    }
}

}  // namespace pcs

using namespace pcs;

PCS_API int pcs_masked_ce_blocks(int B, int L) {
    return (int)(((long long)B * L + kCeBlock - 1) / kCeBlock);
}

PCS_API int pcs_masked_ce(const float* logits, int ld, const void* targets, int target_kind, int ldt,
                          const int32_t* lengths, int B, int L, int C, double* partial, float* loss, float* grad,
                          void* stream) {
    PCS_CHECK_ARG(B >= 1 && L >= 1 && C >= 1 && C <= kCeMaxC && ld >= C && ldt >= C,
                  "pcs_masked_ce: bad sizes B=%d L=%d C=%d ld=%d ldt=%d", B, L, C, ld, ldt);
    PCS_CHECK_ARG(target_kind == 0 || target_kind == 1, "pcs_masked_ce: target_kind must be 0 (u8) or 1 (f32)");
    PCS_CHECK_ARG(logits && targets && lengths && partial && loss, "pcs_masked_ce: null pointer");
    const int nb = pcs_masked_ce_blocks(B, L);
    hipStream_t s = as_stream(stream);
    if (target_kind == 0)
        hipLaunchKernelGGL(masked_ce_kernel<uint8_t>, dim3(nb), dim3(kCeBlock), 0, s, logits, ld,
                           (const uint8_t*)targets, ldt, lengths, B, L, C, partial, grad);
    else
        hipLaunchKernelGGL(masked_ce_kernel<float>, dim3(nb), dim3(kCeBlock), 0, s, logits, ld,
                           (const float*)targets, ldt, lengths, B, L, C, partial, grad);
    hipLaunchKernelGGL(masked_ce_final_kernel, dim3(1), dim3(256), 0, s, partial, nb, lengths, B, L, loss);
    return launch_status("pcs_masked_ce");
}
