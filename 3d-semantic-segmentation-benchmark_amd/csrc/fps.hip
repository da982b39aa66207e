// Farthest point sampling, bit-exact with the reference's CPU `sample`
// (models/utils/common.py:6-34).
//
// Reference semantics per step i:
//   dist  = vector_norm(p - p_far) == sqrtf(fmaf(dz,dz, fmaf(dy,dy, dx*dx)))  (CPU ATen)
//   best  = dist where dist < best                                           (:29-30)
//   far   = first index of max(best)                                         (:31)
//
// MI355X design: one workgroup per cloud (clouds are independent; the chain of
// C steps is inherently serial), every point's coordinates and running minimum
// live in registers (PPT points per thread), so a step touches no memory except
// one 16-B LDS slot per wave.  The running minimum is kept SQUARED (sqrt is
// monotone, so min commutes with it); each thread takes its local maximum M,
// computes S = sqrtf(M) once (correctly rounded) and the lowest of its points
// whose sqrt rounds to S -- so the key (S, lowest index) reproduces the
// reference's argmax over sqrt'ed distances, ties included, with one sqrt per
// thread per step instead of one per point.  Keys are reduced wave-wide with
// shuffles, then across waves through a double-buffered LDS slot array.
#include "pcs_common.hpp"

namespace pcs {

__device__ __forceinline__ void umax64(unsigned& hi, unsigned& lo, unsigned h2, unsigned l2) {
    const bool take = (h2 > hi) || (h2 == hi && l2 > lo);
    hi = take ? h2 : hi;
    lo = take ? l2 : lo;
}

template <int BLOCK, int PPT>
__global__ __launch_bounds__(BLOCK) void fps_kernel(const float* __restrict__ xyz, int N, int C,
                                                    const int* __restrict__ start, int* __restrict__ out_idx,
                                                    float* __restrict__ out_xyz) {
    constexpr int NW = BLOCK / kWave;
    __shared__ unsigned s_khi[2][NW];
    __shared__ unsigned s_klo[2][NW];
    __shared__ float4 s_pos[2][NW];

    const int b = blockIdx.x;
    const int t = threadIdx.x;
    const int w = t >> 6;
    const float* P = xyz + (size_t)b * N * 3;

    float px[PPT], py[PPT], pz[PPT], best[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const int p = j * BLOCK + t;
        if (p < N) {
            px[j] = P[3 * p + 0];
            py[j] = P[3 * p + 1];
            pz[j] = P[3 * p + 2];
            best[j] = __int_as_float(0x7f800000);
        } else {
            px[j] = py[j] = pz[j] = 0.f;
            best[j] = -1.f;  // never a candidate
        }
    }

    int far = start[b];
    far = far < 0 ? 0 : (far >= N ? N - 1 : far);
    float cx = P[3 * far + 0], cy = P[3 * far + 1], cz = P[3 * far + 2];

    for (int i = 0; i < C; ++i) {
        if (t == 0) {
            out_idx[(size_t)b * C + i] = far;
            float* o = out_xyz + ((size_t)b * C + i) * 3;
            o[0] = cx;
            o[1] = cy;
            o[2] = cz;
        }
        if (i == C - 1) break;

        float M = -1.f;
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const float dx = px[j] - cx, dy = py[j] - cy, dz = pz[j] - cz;
            const float d = __fmaf_rn(dz, dz, __fmaf_rn(dy, dy, __fmul_rn(dx, dx)));
            if (best[j] >= 0.f) best[j] = d < best[j] ? d : best[j];
            M = fmaxf(M, best[j]);
        }

        unsigned khi = 0, klo = 0;
        int jsel = 0;
        if (M >= 0.f) {
            const float S = __fsqrt_rn(M);
            float lo = M;
            for (int it = 0; it < 4 && lo > 0.f; ++it) {
                const float pl = __uint_as_float(__float_as_uint(lo) - 1u);
                if (__fsqrt_rn(pl) == S) lo = pl; else break;
            }
            jsel = PPT;
#pragma unroll
            for (int j = PPT - 1; j >= 0; --j)
                if (best[j] >= lo) jsel = j;
            khi = __float_as_uint(S) + 1u;
            klo = 0xFFFFFFFFu - (unsigned)(jsel * BLOCK + t);
        }
        unsigned mhi = khi, mlo = klo;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const unsigned h2 = (unsigned)__shfl_xor((int)mhi, o);
            const unsigned l2 = (unsigned)__shfl_xor((int)mlo, o);
            umax64(mhi, mlo, h2, l2);
        }
        const int buf = i & 1;
        if ((t & 63) == 0) {
            s_khi[buf][w] = mhi;
            s_klo[buf][w] = mlo;
        }
        if (khi != 0 && khi == mhi && klo == mlo) {
            float x = 0.f, y = 0.f, z = 0.f;
#pragma unroll
            for (int j = 0; j < PPT; ++j)
                if (j == jsel) { x = px[j]; y = py[j]; z = pz[j]; }
            s_pos[buf][w] = make_float4(x, y, z, 0.f);
        }
        __syncthreads();
        unsigned bh = s_khi[buf][0], bl = s_klo[buf][0];
        int bw = 0;
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) {
            const unsigned h2 = s_khi[buf][ww], l2 = s_klo[buf][ww];
            if ((h2 > bh) || (h2 == bh && l2 > bl)) { bh = h2; bl = l2; bw = ww; }
        }
        far = (int)(0xFFFFFFFFu - bl);
        const float4 q = s_pos[buf][bw];
        cx = q.x;
        cy = q.y;
        cz = q.z;
    }
}

template <int BLOCK, int PPT>
static void launch_fps(const float* xyz, int B, int N, int C, const int* start, int* out_idx, float* out_xyz,
                       hipStream_t s) {
    hipLaunchKernelGGL((fps_kernel<BLOCK, PPT>), dim3(B), dim3(BLOCK), 0, s, xyz, N, C, start, out_idx, out_xyz);
}

}  // namespace pcs

// Reference: models/utils/common.py:6-34 (`sample`).  Returns indices and the
// gathered centroid coordinates (the reference returns only the coordinates).
PCS_API int pcs_fps(const float* xyz, int B, int N, int C, const int32_t* start, int32_t* out_idx,
                    float* out_xyz, void* stream) {
    using namespace pcs;
    PCS_CHECK_ARG(B >= 0 && N >= 1 && C >= 1, "pcs_fps: bad sizes B=%d N=%d C=%d", B, N, C);
    PCS_CHECK_ARG(xyz && start && out_idx && out_xyz, "pcs_fps: null pointer");
    if (B == 0) return 0;
    hipStream_t s = as_stream(stream);
    if (N <= 64) launch_fps<64, 1>(xyz, B, N, C, start, out_idx, out_xyz, s);
    else if (N <= 256) launch_fps<256, 1>(xyz, B, N, C, start, out_idx, out_xyz, s);
    else if (N <= 1024) launch_fps<256, 4>(xyz, B, N, C, start, out_idx, out_xyz, s);
    else if (N <= 4096) launch_fps<512, 8>(xyz, B, N, C, start, out_idx, out_xyz, s);
    else if (N <= 8192) launch_fps<512, 16>(xyz, B, N, C, start, out_idx, out_xyz, s);
    else if (N <= 16384) launch_fps<1024, 16>(xyz, B, N, C, start, out_idx, out_xyz, s);
    else if (N <= 32768) launch_fps<1024, 32>(xyz, B, N, C, start, out_idx, out_xyz, s);
    else {
        set_error("pcs_fps: N=%d exceeds the 32768-point limit", N);
        return (int)hipErrorInvalidValue;
    }
    return launch_status("pcs_fps");
}
