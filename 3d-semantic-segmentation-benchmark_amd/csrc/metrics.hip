// Segmentation metrics on the GPU (reference Training/metrics.py:3-142): one pass over the
// points computes what the reference gathers with per-sample / per-class Python loops and
// one `.item()` host sync per (sample, class) pair:
//   pred class  = argmax_c predictions[b, n, :]   (first maximum, as torch.argmax)
//   label class = argmax_c labels[b, n, :]
//   confusion[label][pred] += 1, correct += label == pred        (metrics.py:19-24, 66-77)
//   per class c: inter[c] += (labels[c] == 1) && pred == c,
//                union[c] += (labels[c] == 1) || pred == c        (metrics.py:97-108, 132-140)
// over the points n < lengths[b].  Counts are exact: LDS uint32 histograms per block,
// flushed with 64-bit atomics.
#include "pcs_common.hpp"

namespace pcs {

template <typename L>
__global__ __launch_bounds__(256) void seg_metrics_kernel(const float* __restrict__ pred,
                                                          const L* __restrict__ labels,
                                                          const int32_t* __restrict__ lengths, int B, int N, int C,
                                                          unsigned long long* __restrict__ conf,
                                                          unsigned long long* __restrict__ inter,
                                                          unsigned long long* __restrict__ uni,
                                                          unsigned long long* __restrict__ correct) {
    extern __shared__ unsigned int hist[];          // conf C*C | inter C | union C | correct
    const int nb = C * C + 2 * C + 1;
    for (int i = threadIdx.x; i < nb; i += 256) hist[i] = 0;
    __syncthreads();
    const long long total = (long long)B * N;
    for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
        const int b = (int)(t / N);
        const int n = (int)(t - (long long)b * N);
        if (n >= lengths[b]) continue;
        const float* pr = pred + t * C;
        const L* lr = labels + t * C;
        int p = 0, l = 0;
        float pm = pr[0];
        L lm = lr[0];
        for (int c = 1; c < C; ++c) {
            const float v = pr[c];
            if (v > pm) { pm = v; p = c; }
            const L u = lr[c];
            if (u > lm) { lm = u; l = c; }
        }
        atomicAdd(&hist[l * C + p], 1u);
        if (l == p) atomicAdd(&hist[C * C + 2 * C], 1u);
        for (int c = 0; c < C; ++c) {
            const bool lab = lr[c] == (L)1;
            const bool pc = p == c;
            if (lab && pc) atomicAdd(&hist[C * C + c], 1u);
            if (lab || pc) atomicAdd(&hist[C * C + C + c], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nb; i += 256) {
        const unsigned long long v = hist[i];
        if (!v) continue;
        if (i < C * C) atomicAdd(&conf[i], v);
        else if (i < C * C + C) atomicAdd(&inter[i - C * C], v);
        else if (i < C * C + 2 * C) atomicAdd(&uni[i - C * C - C], v);
        else atomicAdd(correct, v);
    }
}

}  // namespace pcs

// predictions (B, N, C) fp32, labels (B, N, C) fp32 (label_u8 = 0) or uint8 (1), lengths (B)
// int32; conf (C x C), inter (C), uni (C), correct (1): int64 counters, ACCUMULATED (+=).
PCS_API int pcs_seg_metrics(const float* pred, const void* labels, int label_u8, const int32_t* lengths, int B, int N,
                            int C, int64_t* conf, int64_t* inter, int64_t* uni, int64_t* correct, void* stream) {
    using namespace pcs;
    PCS_CHECK_ARG(B >= 0 && N >= 0 && C >= 1 && C <= 64, "pcs_seg_metrics: bad sizes B=%d N=%d C=%d", B, N, C);
    PCS_CHECK_ARG(pred && labels && lengths && conf && inter && uni && correct, "pcs_seg_metrics: null pointer");
    if ((long long)B * N == 0) return 0;
    long long g = ((long long)B * N + 255) / 256;
    if (g > 1024) g = 1024;
    const size_t sh = (size_t)(C * C + 2 * C + 1) * sizeof(unsigned int);
    auto* cf = reinterpret_cast<unsigned long long*>(conf);
    auto* it = reinterpret_cast<unsigned long long*>(inter);
    auto* un = reinterpret_cast<unsigned long long*>(uni);
    auto* co = reinterpret_cast<unsigned long long*>(correct);
    if (label_u8)
        hipLaunchKernelGGL(seg_metrics_kernel<uint8_t>, dim3((unsigned)g), dim3(256), sh, as_stream(stream), pred,
                           static_cast<const uint8_t*>(labels), lengths, B, N, C, cf, it, un, co);
    else
        hipLaunchKernelGGL(seg_metrics_kernel<float>, dim3((unsigned)g), dim3(256), sh, as_stream(stream), pred,
                           static_cast<const float*>(labels), lengths, B, N, C, cf, it, un, co);
    return launch_status("pcs_seg_metrics");
}
