// Sliding-window scene inference, merge step (reference predict_single_scene,
// models/dgcnn/utils.py:67-131): windows w = 0..nw-1 start at w*step and hold
// min(win, n - w*step) points; their logits are packed at rows wo[w] .. of `wl` (C per row).
// Per point p (one thread): the logits of the windows covering p are summed in window
// order (as the reference's `all_logits[start:end] += logits` loop), divided by the
// count, then argmax (first maximum) and the max softmax probability 1 / sum exp(x - max).
#include "pcs_common.hpp"

namespace pcs {

__global__ __launch_bounds__(256) void window_merge_kernel(const float* __restrict__ wl,
                                                           const long long* __restrict__ wo, int nw, long long n,
                                                           int C, long long step, long long win,
                                                           long long* __restrict__ pred, float* __restrict__ conf) {
    for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < n; p += (long long)gridDim.x * 256) {
        long long lo = p - win + 1;
        int w0 = lo <= 0 ? 0 : (int)((lo + step - 1) / step);
        int w1 = (int)min((long long)nw - 1, p / step);
        const float cnt = (float)(w1 - w0 + 1);
        // mean logit of class c over the covering windows (re-read: no per-thread arrays)
        auto mean = [&](int c) {
            float a = 0.f;
            for (int w = w0; w <= w1; ++w) a = __fadd_rn(a, wl[(wo[w] + (p - (long long)w * step)) * C + c]);
            return __fdiv_rn(a, cnt);
        };
        int am = 0;
        float mx = mean(0);
        for (int c = 1; c < C; ++c) {
            const float v = mean(c);
            if (v > mx) { mx = v; am = c; }
        }
        float s = 0.f;
        for (int c = 0; c < C; ++c) s += expf(mean(c) - mx);
        pred[p] = am;
        conf[p] = 1.f / s;
    }
}

}  // namespace pcs

using namespace pcs;

PCS_API int pcs_window_merge(const float* window_logits, const long long* window_rows, int nw, long long n, int C,
                             long long step, long long win, long long* pred, float* conf, void* stream) {
    PCS_CHECK_ARG(nw >= 1 && n >= 1 && C >= 1 && C <= 64 && step >= 1 && win >= step,
                  "pcs_window_merge: bad sizes nw=%d n=%lld C=%d step=%lld win=%lld", nw, n, C, step, win);
    PCS_CHECK_ARG((long long)(nw - 1) * step < n && (long long)nw * step >= n - win + 1 && (nw == 1 || win < n),
                  "pcs_window_merge: %d windows of %lld (step %lld) do not tile %lld points", nw, win, step, n);
    PCS_CHECK_ARG(window_logits && window_rows && pred && conf, "pcs_window_merge: null pointer");
    long long g = (n + 255) / 256;
    if (g > 65536) g = 65536;
    hipLaunchKernelGGL(window_merge_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), window_logits,
                       window_rows, nw, n, C, step, win, pred, conf);
    return launch_status("pcs_window_merge");
}
