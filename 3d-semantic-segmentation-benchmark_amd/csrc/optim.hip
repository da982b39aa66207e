// Adam over flat fp32 buffers in one launch (the parameters, gradients and both moment
// estimates of the whole model live in four contiguous arrays with identical layout).
//
// Same update, in the same fp32 operation order, as torch.optim.Adam's default
// (foreach) implementation for amsgrad=False, maximize=False, which the reference
// trains with (Training/train_model.py:263, lr 1e-3):
//   g += wd * p                       (weight_decay != 0)
//   m  = lerp(m, g, 1 - beta1)        (m + w * (g - m), w < 0.5)
//   v  = v * beta2 + (1 - beta2) * g * g
//   p += step * m / (sqrt(v) / bc2_sqrt + eps),   step = -lr / (1 - beta1^t)
// Memory bound: 16 B read + 12 B written per parameter, float4-vectorised.
#include "pcs_common.hpp"

namespace pcs {

__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, float w1, float beta2, float omb2,
                                      float step, float bc2s, float eps, float wd) {
    if (wd != 0.f) g = g + wd * p;
    m = w1 < 0.5f ? m + w1 * (g - m) : g - (g - m) * (1.f - w1);
    v = v * beta2;
    v = v + omb2 * g * g;
    const float den = sqrtf(v) / bc2s + eps;
    p = p + step * (m / den);
}

// The step-dependent scalars on the device, so that a HIP graph that captured the optimizer
// step stays correct on every replay: state[0] (int64 step count) += 1, then the bias
// corrections in double exactly as the host path computes them (torch passes Python floats):
// coef[0] = -(lr / (1 - beta1^t)), coef[1] = sqrt(1 - beta2^t), rounded to fp32.
__global__ void adam_tick_kernel(long long* __restrict__ state, double lr, double beta1, double beta2) {
    const long long t = state[0] + 1;
    state[0] = t;
    float* coef = reinterpret_cast<float*>(state + 1);
    coef[0] = (float)(-(lr / (1.0 - pow(beta1, (double)t))));
    coef[1] = (float)sqrt(1.0 - pow(beta2, (double)t));
}

// coefp (nullable): read step / bc2s from the device (written by adam_tick_kernel)
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long long n,
                                                   float w1, float beta2, float omb2, float step, float bc2s,
                                                   float eps, float wd, const float* __restrict__ coefp) {
    if (coefp) {
        step = coefp[0];
        bc2s = coefp[1];
    }
    const long long n4 = n / 4;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        float4 pp = reinterpret_cast<float4*>(p)[i];
        const float4 gg = reinterpret_cast<const float4*>(g)[i];
        float4 mm = reinterpret_cast<float4*>(m)[i];
        float4 vv = reinterpret_cast<float4*>(v)[i];
        adam1(pp.x, gg.x, mm.x, vv.x, w1, beta2, omb2, step, bc2s, eps, wd);
        adam1(pp.y, gg.y, mm.y, vv.y, w1, beta2, omb2, step, bc2s, eps, wd);
        adam1(pp.z, gg.z, mm.z, vv.z, w1, beta2, omb2, step, bc2s, eps, wd);
        adam1(pp.w, gg.w, mm.w, vv.w, w1, beta2, omb2, step, bc2s, eps, wd);
        reinterpret_cast<float4*>(p)[i] = pp;
        reinterpret_cast<float4*>(m)[i] = mm;
        reinterpret_cast<float4*>(v)[i] = vv;
    }
    if (blockIdx.x == 0 && threadIdx.x < (int)(n - n4 * 4)) {
        const long long i = n4 * 4 + threadIdx.x;
        adam1(p[i], g[i], m[i], v[i], w1, beta2, omb2, step, bc2s, eps, wd);
    }
}

}  // namespace pcs

using namespace pcs;

// one Adam step over n parameters; beta1_w = 1 - beta1 (the lerp weight), beta2_w = 1 - beta2 (both
// rounded from double, as torch passes python floats), step = -lr/(1-beta1^t),
// bc2_sqrt = sqrt(1 - beta2^t).  p, g, m, v: 16-byte aligned device arrays of n floats.
PCS_API int pcs_adam(float* p, const float* g, float* m, float* v, long long n, float beta1_w, float beta2,
                     float beta2_w, float step, float bc2_sqrt, float eps, float weight_decay, void* stream) {
    PCS_CHECK_ARG(n >= 0 && p && g && m && v, "pcs_adam: bad arguments");
    PCS_CHECK_ARG(((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0,
                  "pcs_adam: buffers must be 16-byte aligned");
    if (n == 0) return 0;
    long long blocks = (n / 4 + 255) / 256;
    blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), p, g, m, v, n, beta1_w,
                       beta2, beta2_w, step, bc2_sqrt, eps, weight_decay, (const float*)nullptr);
    return launch_status("pcs_adam");
}

// The same step with the step count kept on the device (graph-capturable): state = 16 bytes
// of device memory {int64 t; float coef[2]} zero-initialised before the first step; each call
// increments t and derives step = -lr / (1 - beta1^t), bc2_sqrt = sqrt(1 - beta2^t) there.
PCS_API int pcs_adam_dev(float* p, const float* g, float* m, float* v, long long n, float beta1_w, float beta2_f,
                         float beta2_w, double lr, double beta1, double beta2, float eps, float weight_decay,
                         long long* state, void* stream) {
    PCS_CHECK_ARG(n >= 0 && p && g && m && v && state, "pcs_adam_dev: bad arguments");
    PCS_CHECK_ARG(((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v | (uintptr_t)state) % 16 == 0,
                  "pcs_adam_dev: buffers must be 16-byte aligned");
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(adam_tick_kernel, dim3(1), dim3(1), 0, st, state, lr, beta1, beta2);
    if (n == 0) return launch_status("pcs_adam_dev");
    long long blocks = (n / 4 + 255) / 256;
    blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, st, p, g, m, v, n, beta1_w, beta2_f,
                       beta2_w, 0.f, 1.f, eps, weight_decay, reinterpret_cast<const float*>(state + 1));
    return launch_status("pcs_adam_dev");
}
