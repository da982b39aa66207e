// Block batch assembly from an HBM-resident block store.
//
// Reference: data_processing/block_datasets.py -- `__getitem__` samples rows of one
// block (:118-128) and `collate_blocks` (:5-31) zero-pads the batch to (B, N, 9)
// points / (B, N, 14) one-hot labels.  Here every block of the split lives in
// one (P, 9) f32 + (P, 14) u8 pair of device arrays, and a batch is one gather:
// out row (b, n) = store row src[b*N + n], or zeros where src < 0 (padding).
#include "pcs_common.hpp"

namespace pcs {

__global__ __launch_bounds__(256) void gather_blocks_kernel(const float* __restrict__ pts,
                                                            const uint8_t* __restrict__ lab,
                                                            const long long* __restrict__ src, long long rows,
                                                            float* __restrict__ out_pts,
                                                            uint8_t* __restrict__ out_lab) {
    // one thread per output element of the 9 point channels, then of the 14 label bytes
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    if (e < rows * 9) {
        const long long r = e / 9;
        const int c = (int)(e - r * 9);
        const long long s = src[r];
        out_pts[e] = s >= 0 ? pts[s * 9 + c] : 0.f;
    }
    if (e < rows * 14) {
        const long long r = e / 14;
        const int c = (int)(e - r * 14);
        const long long s = src[r];
        out_lab[e] = s >= 0 ? lab[s * 14 + c] : (uint8_t)0;
    }
}

// Harness-B batch (Training/train_model.py:89-171): sample i's
// rows are packed at [off[i], off[i] + len[i]) of pts (rows x D) / ids (class per row);
// out_pts (B, L, D) = rows zero-padded to L, out_lab (B, L, C) = one-hot f32 of ids.
__global__ __launch_bounds__(256) void pad_onehot_kernel(const float* __restrict__ pts, int D,
                                                         const int32_t* __restrict__ ids,
                                                         const long long* __restrict__ off,
                                                         const int32_t* __restrict__ len, int B, int L, int C,
                                                         float* __restrict__ out_pts, float* __restrict__ out_lab) {
    const long long total = (long long)B * L;
    for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
        const int b = (int)(t / L);
        const int n = (int)(t - (long long)b * L);
        const bool in = n < len[b];
        const long long r = in ? off[b] + n : 0;
        for (int d = 0; d < D; ++d) out_pts[t * D + d] = in ? pts[r * D + d] : 0.f;
        const int cls = in ? ids[r] : -1;
        for (int c = 0; c < C; ++c) out_lab[t * C + c] = c == cls ? 1.f : 0.f;
    }
}

}  // namespace pcs

using namespace pcs;

PCS_API int pcs_pad_onehot(const float* points, int D, const int32_t* ids, const long long* offsets,
                           const int32_t* lengths, int B, int L, int C, float* out_points, float* out_labels,
                           void* stream) {
    PCS_CHECK_ARG(B >= 0 && L >= 0 && D >= 1 && C >= 1, "pcs_pad_onehot: bad sizes B=%d L=%d D=%d C=%d", B, L, D, C);
    if ((long long)B * L == 0) return 0;
    PCS_CHECK_ARG(points && ids && offsets && lengths && out_points && out_labels, "pcs_pad_onehot: null pointer");
    long long g = ((long long)B * L + 255) / 256;
    if (g > 65536) g = 65536;
    hipLaunchKernelGGL(pad_onehot_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), points, D, ids, offsets,
                       lengths, B, L, C, out_points, out_labels);
    return launch_status("pcs_pad_onehot");
}

PCS_API int pcs_gather_blocks(const float* points, const uint8_t* labels, const long long* src, long long rows,
                              float* out_points, uint8_t* out_labels, void* stream) {
    PCS_CHECK_ARG(rows >= 0, "pcs_gather_blocks: bad size");
    if (rows == 0) return 0;
    PCS_CHECK_ARG(points && labels && src && out_points && out_labels, "pcs_gather_blocks: null pointer");
    const long long total = rows * 14;
    hipLaunchKernelGGL(gather_blocks_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream),
                       points, labels, src, rows, out_points, out_labels);
    return launch_status("pcs_gather_blocks");
}
