// Inverse neighbour maps and atomic-free gather backward for group / interpolate.
//
// The backward of a neighbour gather (models/utils/common.py:64-65 `group`,
// :120-122 `interpolate`) is a scatter-add into the source points.  Instead of
// fp32 atomics (one per gathered element, order-nondeterministic), the geometry
// stage -- which depends on coordinates only and runs on the side stream, off the
// critical path -- also builds the INVERSE map of each neighbour table: for every
// source point, the ascending list of gather slots that read it (CSR: offsets +
// entries, from a stable rocPRIM radix sort of (target, slot) pairs).  The
// backward then gathers: one thread per (source point, channel) sums its slots'
// gradients in ascending slot order -- deterministic, no atomics, no zero fill.
#include "pcs_common.hpp"

#include <rocprim/rocprim.hpp>

namespace pcs {

__global__ __launch_bounds__(256) void inv_keys_kernel(const int32_t* __restrict__ idx, long long n, int per_batch,
                                                       int targets, uint32_t* __restrict__ keys,
                                                       int32_t* __restrict__ vals) {
    const long long s = (long long)blockIdx.x * 256 + threadIdx.x;
    if (s < n) {
        const int b = (int)(s / per_batch);
        keys[s] = (uint32_t)b * (uint32_t)targets + (uint32_t)idx[s];
        vals[s] = (int32_t)s;
    }
}

// offsets[t] = first position of key t in the sorted keys (lower bound), t in [0, T]
__global__ __launch_bounds__(256) void inv_offsets_kernel(const uint32_t* __restrict__ sorted, long long n,
                                                          long long T, int32_t* __restrict__ offsets) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    if (t > T) return;
    long long lo = 0, hi = n;
    while (lo < hi) {
        const long long mid = (lo + hi) >> 1;
        if ((long long)sorted[mid] < t) lo = mid + 1;
        else hi = mid;
    }
    offsets[t] = (int32_t)lo;
}

// grad_feats[(b, p), c] = sum over slots s reading p (ascending) of gout[s][3 + c]
__global__ __launch_bounds__(256) void group_bwd_csr_kernel(const float* __restrict__ gout, int ld,
                                                            const int32_t* __restrict__ off,
                                                            const int32_t* __restrict__ ent, int total, int D,
                                                            float* __restrict__ gfeats) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    const int t = e / D, c = e - t * D;
    float acc = 0.f;
    const int a = off[t], z = off[t + 1];
    for (int i = a; i < z; ++i) acc += gout[(size_t)ent[i] * ld + 3 + c];
    gfeats[e] = acc;
}

// grad_pts[(b, m), c] = sum over slots s = 3*row + j reading m (ascending) of
//   (gout[row][col_off + c] / norm_row) * w_j      -- the autograd rounding of
// interpolate's (p*w)/norm (common.py:119-122), as the atomic kernel computes it
__global__ __launch_bounds__(256) void interp_bwd_csr_kernel(const float* __restrict__ gout, int ld, int col_off,
                                                             const float* __restrict__ dist,
                                                             const int32_t* __restrict__ off,
                                                             const int32_t* __restrict__ ent, int total, int D,
                                                             float* __restrict__ gpts) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    const int t = e / D, c = e - t * D;
    float acc = 0.f;
    const int a = off[t], z = off[t + 1];
    for (int i = a; i < z; ++i) {
        const int s = ent[i];
        const int row = s / 3, j = s - 3 * row;
        const float w0 = 1.0f / (dist[(size_t)row * 3 + 0] + 1e-9f);
        const float w1 = 1.0f / (dist[(size_t)row * 3 + 1] + 1e-9f);
        const float w2 = 1.0f / (dist[(size_t)row * 3 + 2] + 1e-9f);
        const float nrm = (w0 + w1) + w2;
        const float wj = j == 0 ? w0 : (j == 1 ? w1 : w2);
        acc += (gout[(size_t)row * ld + col_off + c] / nrm) * wj;
    }
    gpts[e] = acc;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static int key_bits(long long T) {
    int bits = 1;
    while (bits < 32 && (1ll << bits) < T) ++bits;
    return bits;
}

}  // namespace pcs

using namespace pcs;

// workspace bytes of pcs_inverse_index for n_slots gather slots into n_targets (= B*T) sources
PCS_API int pcs_inverse_index_workspace(long long n_slots, long long n_targets, size_t* bytes) {
    PCS_CHECK_ARG(n_slots >= 1 && n_slots < (1ll << 31) && n_targets >= 1 && n_targets < (1ll << 31) && bytes,
                  "pcs_inverse_index_workspace: bad sizes");
    size_t tmp = 0;
    const hipError_t e = rocprim::radix_sort_pairs((void*)nullptr, tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                   (const int32_t*)nullptr, (int32_t*)nullptr, (size_t)n_slots, 0,
                                                   key_bits(n_targets));
    if (e != hipSuccess) {
        set_error("pcs_inverse_index_workspace: %s", hipGetErrorString(e));
        return (int)e;
    }
    *bytes = align256(tmp) + 3 * align256((size_t)n_slots * 4);
    return 0;
}

// idx: (B * per_batch) int32 neighbour table, values in [0, targets); offsets (B*targets + 1),
// entries (B * per_batch): slots reading source (b, p) are entries[offsets[b*targets+p] ..
// offsets[b*targets+p+1]) in ascending order.
PCS_API int pcs_inverse_index(const int32_t* idx, int B, int per_batch, int targets, int32_t* offsets,
                              int32_t* entries, void* workspace, size_t ws_bytes, void* stream) {
    PCS_CHECK_ARG(B >= 1 && per_batch >= 1 && targets >= 1, "pcs_inverse_index: bad sizes");
    const long long n = (long long)B * per_batch, T = (long long)B * targets;
    PCS_CHECK_ARG(n < (1ll << 31) && T < (1ll << 31), "pcs_inverse_index: too many slots/targets");
    PCS_CHECK_ARG(idx && offsets && entries && workspace, "pcs_inverse_index: null pointer");
    size_t need = 0;
    if (int e = pcs_inverse_index_workspace(n, T, &need)) return e;
    PCS_CHECK_ARG(ws_bytes >= need, "pcs_inverse_index: workspace %zu < %zu bytes", ws_bytes, need);
    char* w = (char*)workspace;
    const size_t slot_bytes = align256((size_t)n * 4);
    uint32_t* keys_in = (uint32_t*)w;
    uint32_t* keys_out = (uint32_t*)(w + slot_bytes);
    int32_t* vals_in = (int32_t*)(w + 2 * slot_bytes);
    void* tmp = w + 3 * slot_bytes;
    size_t tmp_bytes = need - 3 * slot_bytes;
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(inv_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, idx, n, per_batch,
                       targets, keys_in, vals_in);
    const hipError_t e = rocprim::radix_sort_pairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, entries, (size_t)n, 0,
                                                   key_bits(T), s);
    if (e != hipSuccess) {
        set_error("pcs_inverse_index: radix sort: %s", hipGetErrorString(e));
        return (int)e;
    }
    hipLaunchKernelGGL(inv_offsets_kernel, dim3((unsigned)((T + 1 + 255) / 256)), dim3(256), 0, s, keys_out, n, T,
                       offsets);
    return launch_status("pcs_inverse_index");
}

// grad_feats (B, N, D) = backward of group's feature gather (overwrites; no zero fill needed).
PCS_API int pcs_group_bwd_csr(const float* grad_out, int ld_gout, const int32_t* offsets, const int32_t* entries,
                              int B, int N, int D, float* grad_feats, void* stream) {
    PCS_CHECK_ARG(B >= 1 && N >= 1 && D >= 1 && ld_gout >= 3 + D, "pcs_group_bwd_csr: bad sizes");
    const long long total = (long long)B * N * D;
    PCS_CHECK_ARG(total < (1ll << 31), "pcs_group_bwd_csr: too many elements");
    PCS_CHECK_ARG(grad_out && offsets && entries && grad_feats, "pcs_group_bwd_csr: null pointer");
    hipLaunchKernelGGL(group_bwd_csr_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream),
                       grad_out, ld_gout, offsets, entries, (int)total, D, grad_feats);
    return launch_status("pcs_group_bwd_csr");
}

// grad_pts (B, M, D) = backward of interpolate's IDW gather (overwrites).
PCS_API int pcs_interp_bwd_csr(const float* grad_out, int ld_gout, int col_off, const float* dist,
                               const int32_t* offsets, const int32_t* entries, int B, int M, int D, float* grad_pts,
                               void* stream) {
    PCS_CHECK_ARG(B >= 1 && M >= 1 && D >= 1 && ld_gout >= col_off + D && col_off >= 0, "pcs_interp_bwd_csr: bad sizes");
    const long long total = (long long)B * M * D;
    PCS_CHECK_ARG(total < (1ll << 31), "pcs_interp_bwd_csr: too many elements");
    PCS_CHECK_ARG(grad_out && dist && offsets && entries && grad_pts, "pcs_interp_bwd_csr: null pointer");
    hipLaunchKernelGGL(interp_bwd_csr_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream),
                       grad_out, ld_gout, col_off, dist, offsets, entries, (int)total, D, grad_pts);
    return launch_status("pcs_interp_bwd_csr");
}
