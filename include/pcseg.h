/*
 * pcseg -- MI355X-native (gfx950) point-cloud segmentation hot path, C ABI.
 *
 * Drop-in boundary for the reference's `models/` hot path
 * (piotr-bledowski/3D-Semantic-Segmentation-Benchmark).  The reference is pure
 * Python on PyTorch, so there is no reference FFI to mirror; each entry point
 * below replaces the reference function cited next to it, and the Python
 * package `pcseg` binds them with ctypes.
 *
 * Conventions
 *   - all pointers are caller-owned DEVICE pointers (fp32 / int32 / uint8),
 *     row-contiguous, point-major: (B, N, C) means channels innermost;
 *   - `stream` is a hipStream_t passed as void*; every call is stream-ordered,
 *     asynchronous and allocation-free (capturable into a hipGraph);
 *   - return 0 on success, else a hipError_t-compatible code; the message is
 *     available from pcs_last_error() (thread-local);
 *   - "grad_*" outputs documented as accumulating must be zeroed by the caller.
 */
#ifndef PCSEG_H_
#define PCSEG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* pcs_last_error(void);
int pcs_abi_version(void);

/* ---- neighbour search ------------------------------------------------- */

/* models/utils/common.py:6-34 `sample`: iterative farthest point sampling,
 * bit-exact with the CPU reference (vector_norm rounding, first-index argmax).
 * xyz (B,N,3); start (B) = the reference's torch.randint draw (common.py:22);
 * out_idx (B,C) int32; out_xyz (B,C,3) gathered centroids. */
int pcs_fps(const float* xyz, int B, int N, int C, const int32_t* start,
            int32_t* out_idx, float* out_xyz, void* stream);

/* models/utils/common.py:51-61 `group` neighbour choice: distances un-fused,
 * d > r2 -> inf, topk(K, smallest) with libstdc++ tie/padding semantics.
 * centroids (B,C,3), xyz (B,N,3), r2 = float32(r*r); out_idx (B,C,K). */
int pcs_ball_query(const float* centroids, const float* xyz, int B, int C,
                   int N, float r2, int K, int32_t* out_idx, void* stream);

/* models/utils/common.py:107-114 `interpolate` neighbour choice:
 * topk(k, smallest) of un-fused squared distances from each query to ref.
 * query (B,N,3), ref (B,M,3); out_idx (B,N,k), out_dist (B,N,k) or NULL. */
int pcs_knn_select(const float* query, const float* ref, int B, int N, int M,
                   int k, int32_t* out_idx, float* out_dist, void* stream);

/* models/dgcnn/dgcnn.py:7-21 `knn`: k nearest in feature space
 * (largest -|xi|^2 + 2 xi.xj - |xj|^2).  x (B,N,F) point-major,
 * F in {3,64}, k in {16,20,32,40}; out_idx (B,N,k) best first. */
int pcs_knn(const float* x, int B, int N, int F, int k, int32_t* out_idx,
            void* stream);

/* ---- gather / scatter --------------------------------------------------- */

/* models/utils/common.py:62-71: out (B*C*K, 3+D) rows
 * [ (xyz[idx]-centroid) (/ r if normalize), feats[idx] ]. */
int pcs_group_fwd(const float* xyz, const float* feats, const float* centroids,
                  const int32_t* idx, int B, int N, int C, int K, int D,
                  float r, int normalize, float* out, void* stream);
/* grad_feats (B,N,D) += scatter(grad_out[:, 3:])   (accumulating) */
int pcs_group_bwd(const float* grad_out, const int32_t* idx, int B, int N,
                  int C, int K, int D, float* grad_feats, void* stream);

/* models/utils/common.py:85-86 `reduce(x,'max')` over K:
 * x (G*K, Ch) -> out (G, Ch), argmax (G, Ch) uint8 (first max). */
int pcs_maxk_fwd(const float* x, long long G, int K, int Ch, float* out,
                 uint8_t* argmax, void* stream);
/* grad_x (G*K, Ch) = grad_out routed to argmax, 0 elsewhere (overwrites). */
int pcs_maxk_bwd(const float* grad_out, const uint8_t* argmax, long long G,
                 int K, int Ch, float* grad_x, void* stream);

/* models/utils/common.py:115-122: IDW over 3 neighbours.
 * pts (B,M,D); idx/dist (B,N,3); out[(b*N+n)*ld_out + col_off + c]. */
int pcs_interp_fwd(const float* pts, const int32_t* idx, const float* dist,
                   int B, int N, int M, int D, float* out, int ld_out,
                   int col_off, void* stream);
/* grad_pts (B,M,D) += weighted scatter   (accumulating) */
int pcs_interp_bwd(const float* grad_out, const int32_t* idx, const float* dist,
                   int B, int N, int M, int D, int ld_gout, int col_off,
                   float* grad_pts, void* stream);

/* models/dgcnn/dgcnn.py:41-53 `get_graph_feature`: x (B,N,D) point-major,
 * idx (B,N,k); out (B*N*k, 2D) rows [x_j - x_i, x_i]. */
int pcs_edge_fwd(const float* x, const int32_t* idx, int B, int N, int k,
                 int D, float* out, void* stream);
/* grad_x (B,N,D) += backward of the above   (accumulating) */
int pcs_edge_bwd(const float* grad_out, const int32_t* idx, int B, int N,
                 int k, int D, float* grad_x, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PCSEG_H_ */
