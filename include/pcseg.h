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
/* 4 since round 6 (added pcs_knn_order, pcs_knn_pruned, pcs_knn_pruned_workspace).
 * 3 since round 5 (pcs_group_bwd_csr / pcs_interp_bwd_csr take n_slots, pcs_edgeconv_fwd an
 * optional second output, pcs_edgeconv_bwd the output gradient's row stride; new:
 * pcs_geometry_stream, pcs_probe_times and the kernel-variant calls; round 4 dropped
 * pcs_knn_morton_seeds and added pcs_inverse_index_batch); bindings refuse another version */
int pcs_abi_version(void);
/* sizeof(pcs_operand), for bindings to check their struct layout */
int pcs_operand_size(void);
/* sizeof(pcs_mlp_layer) (25 eight-byte slots = 200), likewise */
int pcs_mlp_layer_size(void);

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
/* pcs_knn with a caller workspace of pcs_knn_workspace(B, N) bytes: the
 * squared norms are computed once per point (same lists as pcs_knn). */
int pcs_knn_workspace(int B, int N, size_t* bytes);
int pcs_knn_ws(const float* x, int B, int N, int F, int k, int32_t* out_idx,
               void* ws, size_t ws_bytes, void* stream);
/* pcs_knn_ws whose rows start from the threshold of a previous neighbour list
 * (seeds (B,N,ks) int32: DGCNN's previous EdgeConv graph, dgcnn.py:183-189 feeding
 * get_graph_feature at :29-56): the same lists as pcs_knn, fewer survivors to merge.
 * Rows whose seeds are out of range, repeated or fewer than k search unseeded. */
int pcs_knn_seeded(const float* x, int B, int N, int F, int k, const int32_t* seeds,
                   int ks, int32_t* out_idx, void* ws, size_t ws_bytes, void* stream);
/* Morton order (B,N) int32 of each cloud's points by their first three features (x (B,N,F),
 * F >= 3: DGCNN's xyz, dgcnn.py:183 / :228 graph input); clouds past 8192 points get the
 * identity order.  Computed once per forward and shared by its four graphs. */
int pcs_knn_order(const float* x, int B, int N, int F, int32_t* order, void* stream);
/* pcs_knn_seeded (seeds nullable) scanning each cloud in `order` (a permutation of 0..N-1 per
 * cloud, pcs_knn_order's output) nearest tiles first, skipping the candidate tiles that are
 * provably farther than every row's k-th best: the same lists as pcs_knn.  Workspace:
 * pcs_knn_pruned_workspace(B, N, F) bytes. */
int pcs_knn_pruned_workspace(int B, int N, int F, size_t* bytes);
int pcs_knn_pruned(const float* x, int B, int N, int F, int k, const int32_t* order,
                   const int32_t* seeds, int ks, int32_t* out_idx, void* ws, size_t ws_bytes,
                   void* stream);

/* ---- geometry plan of a PointNet++-family forward --------------------------
 * One call enqueues, on one stream and in this order, every neighbour structure of a
 * forward: per level l, FPS of the previous level's points (level 0: coords) down to C
 * centroids (pcs_fps, start = starts[l*B + b]), then its nq ball queries (pcs_ball_query
 * against the previous level's points, or the centroids themselves when on_self -- the
 * InvResMLP grouping, models/utils/common.py:288), then `event` is recorded (nullable);
 * after all levels, when interp: the 3-NN of each FeaturePropagation from level L-1 down to
 * 0 (pcs_knn_select of level l-1's points (coords for l = 0) among level l's centroids), then
 * every inverse map -- the ball queries' and the 3-NN's, when inverse -- in one
 * pcs_inverse_index_batch, then nn_event.  So with interp the level events cover the FPS and
 * ball queries only and nn_event covers every inverse map; without interp each level's maps
 * precede its `event`.  Same kernels and arguments as the per-op calls:
 * bitwise the same plan.  Outputs caller-owned; the inverse maps share one workspace of
 * pcs_geometry_plan_workspace bytes.  Replaces pcseg.common.GeometryPlan's ~20 calls. */
#define PCS_GEO_MAX_LEVELS 6
#define PCS_GEO_MAX_QUERIES 4
typedef struct pcs_geo_level {
    int64_t C, nq;
    double r2[PCS_GEO_MAX_QUERIES];      /* float32(r*r) of each query */
    int64_t K[PCS_GEO_MAX_QUERIES];
    int64_t on_self[PCS_GEO_MAX_QUERIES];
    int32_t* fps_idx;                     /* (B, C) */
    float* cent;                          /* (B, C, 3) */
    int32_t* ball[PCS_GEO_MAX_QUERIES];  /* (B, C, K[q]) */
    int32_t* ball_off[PCS_GEO_MAX_QUERIES];  /* (B * targets + 1) */
    int32_t* ball_ent[PCS_GEO_MAX_QUERIES];  /* (B * C * K[q]) */
    int32_t* nn_idx; float* nn_dist;      /* (B, N_{l-1}, 3): the FeaturePropagation 3-NN into level l */
    int32_t* nn_off; int32_t* nn_ent;     /* its inverse map (B * C + 1), (B * N_{l-1} * 3) */
    void* event;                          /* hipEvent_t recorded after the level's FPS + ball queries */
} pcs_geo_level;
int pcs_geometry_plan_workspace(int B, int N, const pcs_geo_level* levels, int L, int interp,
                                int inverse, size_t* bytes);
int pcs_geometry_plan(const float* coords, int B, int N, const int32_t* starts,
                      const pcs_geo_level* levels, int L, int interp, int inverse, void* nn_event,
                      void* workspace, size_t ws_bytes, void* stream);

/* ---- gather / scatter --------------------------------------------------- */

/* models/utils/common.py:62-71: out (B*C*K, 3+D) rows
 * [ (xyz[idx]-centroid) (/ r if normalize), feats[idx] ]. */
int pcs_group_fwd(const float* xyz, const float* feats, const float* centroids,
                  const int32_t* idx, int B, int N, int C, int K, int D,
                  float r, int normalize, float* out, int ld_out, void* stream);
/* (its backward is pcs_group_bwd_csr over the inverse map of idx, below) */

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
/* FeaturePropagation rows (common.py:238-240): out (B*N, ld_out) = [f1 (B,N,D1) |
 * interpolate(pts (B,M,D2))] in one pass; D1, D2, ld_out multiples of 4, 16-B aligned
 * buffers, f1 may be null when D1 == 0. */
int pcs_interp_cat_fwd(const float* f1, int D1, const float* pts, const int32_t* idx,
                       const float* dist, int B, int N, int M, int D2, float* out,
                       int ld_out, void* stream);
/* (its backward is pcs_interp_bwd_csr over the inverse map of idx, below) */

/* models/dgcnn/dgcnn.py:41-53 `get_graph_feature`: x (B,N,D) point-major,
 * idx (B,N,k); out (B*N*k, 2D) rows [x_j - x_i, x_i]. */
int pcs_edge_fwd(const float* x, const int32_t* idx, int B, int N, int k,
                 int D, float* out, int ld_out, void* stream);
/* grad_x (B,N,D) = backward of the above (overwrites), over the inverse map of
 * idx (pcs_inverse_index, targets = N): fixed-order fp64 sums, no atomics. */
int pcs_edge_bwd(const float* grad_out, int ld_gout, const int32_t* offsets,
                 const int32_t* entries, int B, int N, int k, int D, float* grad_x,
                 void* stream);

/* ---- shared-MLP engine: 1x1 conv + training-mode BN + ReLU/LeakyReLU ------
 * models/utils/common.py:125-178 (MiniPointNet/UnitPointNet), dgcnn.py:67-76,
 * dgcnn.py:188-207.  act: 0 = ReLU, 1 = LeakyReLU(slope), 2 = identity.
 * BN partial-sum workspaces are fp64 [2][N][blocks] (each channel's partials
 * contiguous, so the finalize kernels read them coalesced). */

/* Operand of the engine GEMMs: row-major rows (row stride ld, multiple of 4)
 * read through a per-channel transform applied on load, so BatchNorm-applied
 * activations and BatchNorm-backward gradients never round-trip HBM:
 *   PCS_OP_PLAIN   : data[r][c]
 *   PCS_OP_BNACT   : act(data[r][c]*s[c] + t[c])              (forward BN + act)
 *   PCS_OP_BNBWD   : s*dy - kb - alpha*(z - mean)              (BN backward, dZ)
 *                    dy = data[r][c] * act'(z*s + t), z = Z[r][c] (row stride ldz)
 *   PCS_OP_POOLBWD : as BNBWD with data[r][c] = arg[g][c] == k ? dpool[g][c] : 0,
 *                    g = r / pool_k, k = r % pool_k (data/arg are G x ld)
 * alpha = kC*invstd and kb = kB from pcs_bn_bwd_finalize; inv = invstd (epilogue). */
enum { PCS_OP_PLAIN = 0, PCS_OP_BNACT = 1, PCS_OP_BNBWD = 2, PCS_OP_POOLBWD = 3 };
typedef struct pcs_operand {
    const float* data; int ld; int mode;
    const float* s; const float* t; int act; float slope;
    const float* z; int ldz;
    const float* mean; const float* inv; const float* alpha; const float* kb;
    const uint8_t* arg; int pool_k;
} pcs_operand;

/* row blocks of pcs_gemm_rows with a PLAIN / BNACT A (sizes its stats/bstats workspace) */
int pcs_gemm_row_blocks(int M, int N);
/* row blocks of pcs_gemm_rows_kmajor, or of pcs_gemm_rows when A is BNBWD or POOLBWD
 * (the data-gradient form; sizes its bstats workspace) */
int pcs_gemm_row_blocks_dgrad(int M, int N);
/* C (M x N, ldc) = T(A) . W^T (+bias), W row-major N x K with row stride ldw.
 * stats: partial (sum, sum^2) of C per channel.  bstats: fused BN-backward
 * partials (sum dy, sum dy*xhat) of the layer whose pre-BN output is epi->z
 * (dy = C * act'(z*s+t), xhat = (z-mean)*inv; epi's s/t/mean/inv/act/slope). */
int pcs_gemm_rows(const pcs_operand* a, int M, int K, const float* W, int ldw,
                  const float* bias, float* C, int ldc, int N, double* stats,
                  const pcs_operand* epi, double* bstats, void* stream);
/* Data-gradient form of pcs_gemm_rows: W row-major K x N (B[k][n] = W[k*ldw + n],
 * ldw >= N, a multiple of 4) -- dA = dZ . W on the layer's own weight matrix, no
 * transpose.  LDS engine only; A must be PLAIN, BNBWD or POOLBWD. */
int pcs_gemm_rows_kmajor(const pcs_operand* a, int M, int K, const float* W, int ldw,
                         float* C, int ldc, int N, const pcs_operand* epi,
                         double* bstats, void* stream);
/* pcs_gemm_rows with its kernel forced for this one call (A/B and tests): variant -1 = the
 * register-staged row GEMM, 0 = the policy (the LDS-DMA forward kernel for > 64 outputs over
 * >= 8192 rows), 1 = the LDS-DMA forward kernel wherever it is legal (K % 32 == 0, PLAIN / BNACT
 * A, 16-B aligned rows). */
int pcs_gemm_rows_variant(const pcs_operand* a, int M, int K, const float* W, int ldw,
                          const float* bias, float* C, int ldc, int N, double* stats,
                          int variant, void* stream);
/* The calling thread's engine kernels for every later call (A/B and tests only; the product
 * never calls it): -1 = the register-staged row GEMMs only (no LDS-DMA forward / data-gradient
 * kernels), 0 = the policy. */
int pcs_set_kernel_variant(int variant);
/* pcs_gemm_rows_kmajor with its kernel forced for this one call (A/B measurements and the
 * bitwise tests; the product always calls the policy): variant -1 = the register-staged row
 * GEMM, 0 = the policy, 1..3 = the LDS-DMA kernel with 64 x 3 / 128 x 2 / 128 x 3 column tile x
 * ring stages.  Results are bitwise equal across variants. */
int pcs_gemm_rows_kmajor_variant(const pcs_operand* a, int M, int K, const float* W, int ldw,
                                 float* C, int ldc, int N, const pcs_operand* epi,
                                 double* bstats, int variant, void* stream);
/* Wide-layer GEMM on plain operands (DGCNN conv5..conv7 forward and data gradient,
 * models/dgcnn/dgcnn.py:188-207 -- the conv1d products the reference runs in ATen):
 * C (M x N, ldc) = A (M x R, lda) . B (N x R, ldb)^T (+ bias), both operands
 * row-major with the contraction axis contiguous.  stats (nullable): [2][N][row
 * tiles] fp64 partial (sum, sum^2) of C (pcs_gemm_nt_row_tiles(M) tiles, the
 * layout pcs_bn_finalize reads).  Needs M >= 65536, N >= 256, R % 32 == 0, lda
 * and ldb multiples of 4 (>= R), 16-B aligned A and B. */
int pcs_gemm_nt(const float* A, int lda, const float* B, int ldb, int M, int N, int R,
                const float* bias, float* C, int ldc, double* stats, void* stream);
int pcs_gemm_nt_row_tiles(int M);
/* dW (N x K) += T(X)^T . T(Y) over M rows; db (N, nullable) += column sums of
 * T(X).  X: PLAIN/BNBWD/POOLBWD (the layer's dZ), Y: PLAIN/BNACT (its input).
 * (accumulating) Deterministic: each row split's partial tile is stored in the
 * workspace (pcs_wgrad_workspace bytes) and the splits are added in a fixed order,
 * so identical calls give bitwise-identical dW/db.  The workspace is in use until
 * the call's work on `stream` completes. */
int pcs_wgrad_workspace(int N, int K, int M, size_t* bytes);
int pcs_wgrad(const pcs_operand* x, int N, const pcs_operand* y, int K, int M,
              float* dW, float* db, void* workspace, size_t ws_bytes, void* stream);
/* BN forward finalize: partials -> scale s, shift t, mean, invstd; running
 * mean/var updated with `momentum` and the unbiased variance (nullable). */
int pcs_bn_finalize(const double* part, int nb, int N, long long M,
                    const float* gamma, const float* beta, float eps,
                    float momentum, float* run_mean, float* run_var, float* s,
                    float* t, float* mean, float* invstd, void* stream);
/* BN backward finalize: partials -> dgamma, dbeta (written, or added when
 * accum != 0), kB = s*sum_dy/M, kC = s*sum(dy*xhat)/M (* invstd[c] when
 * invstd is given: the `alpha` of PCS_OP_BNBWD)
 * (dZ = s*dy - kB - kC*xhat). */
int pcs_bn_bwd_finalize(const double* part, int nb, int N, long long M,
                        const float* s, const float* invstd, float* dgamma,
                        float* dbeta, float* kB, float* kC, int accum,
                        void* stream);
int pcs_bn_bwd_reduce_blocks(int M);
int pcs_bn_bwd_reduce(const float* dA, int ldd, const float* Z, int ldz, int M,
                      int N, const float* s, const float* t, const float* mean,
                      const float* inv, int act, float slope, double* part,
                      void* stream);
/* common.py:211-212 / dgcnn.py:76: pooled (G x N) = max_k act(Z*s+t), first
 * argmax (u8); Z rows are (g*K + k). */
int pcs_pool_fwd(const float* Z, int N, long long G, int K, const float* s,
                 const float* t, int act, float slope, float* out,
                 uint8_t* arg, void* stream);
int pcs_pool_bwd_reduce_blocks(long long G);
int pcs_pool_bwd_reduce(const float* dpool, const uint8_t* arg, const float* Z,
                        int N, long long G, int K, const float* s,
                        const float* t, const float* mean, const float* inv,
                        int act, float slope, double* part, void* stream);
/* nn.Dropout(p) in training mode after a stack's activation (dgcnn.py:206-207 conv6 /
 * conv7): element (r, c) of an M x N output is kept when a counter-based hash of
 * (seed, r*N + c) clears p (same Bernoulli(1-p) keep / 1/(1-p) scale as torch's, a
 * different random stream); the forward is fused into the stack's output (drop_p /
 * drop_seed of its top layer), the mask is recomputed here, never stored:
 * gin (ldi) = gout (ldg) * keep / (1 - p). */
int pcs_dropout_bwd(const float* gout, int ldg, int M, int N, double p, int64_t seed,
                    float* gin, int ldi, void* stream);
/* dst (M x C, row stride ldd) = src (M x C, row stride lds): a row block copied into
 * columns of a wider buffer (DGCNN's cat(x1..x4, colour) into the head's (B*N, 1408)
 * buffer, dgcnn.py:200 / :245); float4 rows, 16-B aligned pointers, C, lds, ldd % 4 == 0. */
int pcs_copy_cols(const float* src, int lds, int M, int C, float* dst, int ldd, void* stream);
/* out (M x N, ldo) = act(Z*s + t) */
int pcs_bn_act(const float* Z, int ldz, int M, int N, const float* s,
               const float* t, int act, float slope, float* out, int ldo,
               void* stream);

/* ---- shared-MLP stack in one call -------------------------------------------
 * A stack of nl layers conv1x1 (W, bias) -> BatchNorm (gamma, beta; batch statistics
 * with running-stat update, or running statistics when use_batch = 0) -> act, on
 * point-major rows, optionally max-pooled over consecutive groups of pool_k rows
 * (reference: common.py:125-178 + reduce 'max' common.py:211-212, dgcnn.py:67-76,
 * dgcnn.py:188-207).  Every field is 8 bytes, so bindings can pack a record as 24
 * little-endian u64/i64/f64 slots.
 *   W (cout x ldw) row-major, columns >= cin zero;  cin of layer 0 = kin, of layer
 *   l = cout of layer l-1;  cout % 4 == 0.  num_batches (nullable) += 1 per forward
 *   that updates running statistics.  act: 0 ReLU, 1 LeakyReLU(slope), 2 identity.
 *   Z (M x cout) and coef (4 x cout: scale, shift, mean, invstd) are written by the
 *   forward and read by the backward.  dW (cout x cin), db, dgamma, dbeta: gradients,
 *   accumulating (nullable = not wanted). */
typedef struct pcs_mlp_layer {
    const float* W; int64_t ldw, cin, cout;
    const float* bias; const float* gamma; const float* beta;
    float* run_mean; float* run_var; int64_t* num_batches;
    double momentum, eps;
    int64_t use_batch, act; double slope;
    float* Z; float* coef;
    float* dW; float* db; float* dgamma; float* dbeta;
    double drop_p;        /* top layer, un-pooled: inverted dropout of the output (0 = none) */
    int64_t drop_seed;    /* its mask: pcs_dropout_keep(seed, row * cout + col) */
    int64_t bwd_fuse;     /* backward kernel choice for this layer (a per-call field, no
                           * process-global switch): PCS_BWD_FUSE_DEFAULT fuses the data +
                           * weight gradient of a thin layer into one launch only over >= 2^19
                           * rows, _OFF never, _ALL for every eligible layer (same results to
                           * fp32 rounding; tests / A-B runs) */
    int64_t dx_col0;      /* first layer, backward: the first input column whose data gradient
                           * the caller needs -- the grouped rows of a SetAbstraction start with
                           * 3 relative-coordinate columns whose gradient nobody reads
                           * (common.py:64-65 gathers only features back); dX columns
                           * [0, dx_col0) are then left unwritten and the data-gradient GEMM
                           * covers kin - dx_col0 columns (0 = all) */
} pcs_mlp_layer;

#define PCS_BWD_FUSE_DEFAULT 0
#define PCS_BWD_FUSE_OFF 1
#define PCS_BWD_FUSE_ALL 2

/* workspace bytes of pcs_mlp_forward (backward = 0) or pcs_mlp_backward (1) */
int pcs_mlp_workspace(int M, int kin, int ldx, const pcs_mlp_layer* layers, int nl,
                      int pool_k, int backward, size_t* bytes);
/* X (M x ldx rows, kin channels) -> out = pooled (M/pool_k x cout_L) + argmax u8
 * (pool_k > 0), or the activation (M x cout_L, row stride ldo; 0 = cout_L): a stack can
 * write its activation straight into a column block of a wider buffer (DGCNN's conv5
 * output inside the [x1..x4 | x5] concatenation conv6 reads, dgcnn.py:203-206). */
int pcs_mlp_forward(const float* X, int ldx, int kin, int M, pcs_mlp_layer* layers,
                    int nl, int pool_k, float* out, int ldo, uint8_t* arg, void* workspace,
                    size_t ws_bytes, void* stream);
/* gout = d loss / d out (same shape as out; row stride ldg, = cout_L when pooled);
 * accumulates every layer's dW/db/dgamma/dbeta; dX (M x lddx, nullable; lddx 0 = ldx)
 * = d loss / d X (pad columns zeroed). */
int pcs_mlp_backward(const float* X, int ldx, int kin, int M,
                     const pcs_mlp_layer* layers, int nl, int pool_k,
                     const uint8_t* arg, const float* gout, int ldg, float* dX, int lddx,
                     void* workspace, size_t ws_bytes, void* stream);
/* The same, but the weight gradients are left running on the device's wgrad lane (a side
 * stream) after return, so they overlap the caller's next work.  Until
 * pcs_wgrad_lane_join(stream) has been enqueued, dW/db are not ready and X, gout, the
 * layers' Z/coef and the workspace must stay allocated (lane stream: pcs_wgrad_lane). */
int pcs_mlp_backward_deferred(const float* X, int ldx, int kin, int M,
                              const pcs_mlp_layer* layers, int nl, int pool_k,
                              const uint8_t* arg, const float* gout, int ldg, float* dX, int lddx,
                              void* workspace, size_t ws_bytes, void* stream);
/* the current device's wgrad lane stream (null if none could be created) */
int pcs_wgrad_lane(void** side_stream);
/* `stream` waits for every weight gradient enqueued on the current device's lane so far */
int pcs_wgrad_lane_join(void* stream);
/* the current device's geometry stream (FPS, ball queries, 3-NN, inverse maps of a forward,
 * often the NEXT step's): created once per device at the lowest stream priority, so its long
 * neighbour-search blocks yield the compute units to the step stream's kernels */
int pcs_geometry_stream(void** stream);

/* ---- harness-B batch (Training/train_model.py:89-171, preprocess_batch_to_train_format)
 * sample i's rows are packed at [offsets[i], offsets[i] + lengths[i]) of points (rows x D)
 * and ids (class index per row, int32); writes out_points (B, L, D) zero-padded and
 * out_labels (B, L, C) one-hot fp32 (rows n < lengths[i], lengths[i] <= L). */
int pcs_pad_onehot(const float* points, int D, const int32_t* ids, const long long* offsets,
                   const int32_t* lengths, int B, int L, int C, float* out_points,
                   float* out_labels, void* stream);

/* ---- sliding-window scene inference, merge step (models/dgcnn/utils.py:67-131)
 * nw windows start at w*step (win points each, fewer at the end), their logits packed at
 * rows window_rows[w] .. of window_logits (C per row); per point: mean logits of the
 * covering windows (summed in window order), pred = argmax, conf = max softmax.  C <= 64. */
int pcs_window_merge(const float* window_logits, const long long* window_rows, int nw,
                     long long n, int C, long long step, long long win, long long* pred,
                     float* conf, void* stream);

/* ---- segmentation metrics (Training/metrics.py:3-142) ------------------------
 * predictions (B, N, C) fp32, labels (B, N, C) fp32 (label_u8 = 0) or uint8 (1),
 * lengths (B) int32; over points n < lengths[b]: pred = argmax predictions, label =
 * argmax labels (first maximum); conf[label][pred], correct (label == pred), per
 * class inter (labels[c] == 1 && pred == c) and uni (labels[c] == 1 || pred == c).
 * int64 counters are accumulated (+=).  C <= 64. */
int pcs_seg_metrics(const float* pred, const void* labels, int label_u8,
                    const int32_t* lengths, int B, int N, int C, int64_t* conf,
                    int64_t* inter, int64_t* uni, int64_t* correct, void* stream);

/* ---- fused EdgeConv (training-mode BN) --------------------------------------
 * Replaces get_graph_feature + Conv2d(2C->Cout, 1x1, bias=False) + BatchNorm2d +
 * LeakyReLU + max over k (models/dgcnn/dgcnn.py:24-57, 60-77) without forming the
 * (B, 2C, N, k) edge tensor: z_(i,j) = (Y_j - Y_i) + P_i with Y = X W1^T,
 * P = X W2^T (W = [W1 | W2]).  Rows are B*N points (X stride ldx, C channels);
 * idx (B, N, k) int32 per-cloud neighbour indices; Cout % 4 == 0. */
/* workspace bytes of pcs_edgeconv_fwd (backward = 0) / pcs_edgeconv_bwd (1) */
int pcs_edgeconv_workspace(int B, int N, int C, int Cout, int backward, size_t* bytes);
/* forward: Y, PQ (returns Q = P - Y), S = sum_k z (each B*N x Cout), pz / pa
 * (B*N x Cout: the pooled edge's z -- the max over k where gamma > 0, the min where
 * gamma < 0, edge 0 where gamma == 0 -- and its first slot), coef (s, t, mean,
 * invstd; 4 x Cout), pooled activation out (B*N x Cout) + argmax slot arg (u8);
 * out2 (nullable, row stride ld2 >= Cout, 16-B aligned rows for the vector path): a
 * second copy of `out` -- DGCNN's EdgeConv outputs written straight into their column
 * block of the head's concatenation (dgcnn.py:200); running stats / num_batches
 * updated in place. */
int pcs_edgeconv_fwd(const float* X, int ldx, int C, const int32_t* idx, int B, int N,
                     int k, const float* W, int Cout, const float* gamma,
                     const float* beta, float* run_mean, float* run_var,
                     long long* num_batches, float momentum, float eps, float slope,
                     float* Y, float* PQ, float* S, float* pz, uint8_t* pa,
                     float* coef, float* out, uint8_t* arg, float* out2, int ld2,
                     void* workspace, size_t ws_bytes, void* stream);
/* backward from the forward's saved tensors and the CSR inverse of idx
 * (pcs_inverse_index, targets = N): dW (Cout x 2C), dgamma, dbeta accumulate (+=);
 * dX (nullable; C % 4 == 0) is written.  dout: gradient of `out`, row stride
 * ldo >= Cout (a column block of a wider gradient is read in place). */
int pcs_edgeconv_bwd(const float* X, int ldx, int C, const int32_t* csr_off,
                     const int32_t* csr_ent, int B, int N, int k, const float* W,
                     int Cout, const float* Y, const float* Q, const float* S,
                     const float* pz, const uint8_t* arg, const float* coef,
                     float slope, const float* dout, int ldo, float* dX, int lddx,
                     float* dW, float* dgamma, float* dbeta, void* workspace,
                     size_t ws_bytes, void* stream);

/* ---- launch probe (measurement) -----------------------------------------------
 * While enabled, every engine GEMM launch (pcs_gemm_rows / pcs_wgrad, also those
 * issued inside pcs_mlp_forward/backward) is bracketed by HIP events recorded on its
 * own stream.  pcs_probe_end returns the record count; pcs_probe_get(i) returns the
 * kernel name (as rocprofv3 reports it), algorithmic flops / HBM bytes and the
 * measured milliseconds (waits for the launch). */
int pcs_probe_begin(void);
int pcs_probe_end(void);
int pcs_probe_get(int i, char* name, int cap, double* flops, double* bytes,
                  float* ms);
/* Record i's stream (the hipStream_t its launch was enqueued on): bench.py separates the
 * launches on the step's own (critical-path) stream from the side streams'. */
int pcs_probe_stream(int i, void** stream);
/* record i's start / end in ms after record 0's start (waits for its stop event) */
int pcs_probe_times(int i, double* t0_ms, double* t1_ms);
/* After pcs_probe_end: re-issue every recorded launch of kernel `name` back to back
 * `reps` times (after one untimed pass) between two events on their stream; returns
 * the average microseconds per launch -- comparable with rocprofv3's AverageNs for
 * that kernel.  The launches rewrite their outputs. */
int pcs_probe_replay(const char* name, int reps, float* us_per_launch, int* launches);
/* Occupy `stream` for about `us` microseconds (one wave sleeping on the realtime
 * clock), so the host can enqueue a whole probed step before the GPU reaches it: the
 * probe's event brackets then time the kernels back to back, as they run in a
 * GPU-bound step, without host-enqueue gaps. */
int pcs_spin(int us, void* stream);

/* ---- inverse neighbour maps (atomic-free gather backward) ------------------ */

/* For a neighbour table idx (B x per_batch, values in [0, targets)), the CSR
 * inverse: the slots reading source (b, p) are entries[offsets[b*targets+p] ..
 * offsets[b*targets+p+1]), ascending.  offsets (B*targets + 1), entries
 * (B*per_batch) int32; workspace of pcs_inverse_index_workspace bytes. */
int pcs_inverse_index_workspace(long long n_slots, long long n_targets,
                                size_t* bytes);
int pcs_inverse_index(const int32_t* idx, int B, int per_batch, int targets,
                      int32_t* offsets, int32_t* entries, void* workspace,
                      size_t ws_bytes, void* stream);
/* Several maps of B clouds each in one call: the maps of <= 8192 targets share three
 * launches (chunk counts, scan, ranked scatter; blockIdx.z = map), larger ones follow one
 * by one.  Same outputs as one pcs_inverse_index per map.  Replaces the per-table
 * index/sort loop of the reference's scatter-add backward (common.py:64-65, :120-122;
 * dgcnn.py:60-77 get_graph_feature's gather) -- there autograd's index_add. */
typedef struct pcs_inverse_map {
    const int32_t* idx;    /* (B * per_batch) neighbour table */
    int per_batch;
    int targets;
    int32_t* offsets;      /* (B * targets + 1) */
    int32_t* entries;      /* (B * per_batch) */
} pcs_inverse_map;
int pcs_inverse_index_batch_workspace(const pcs_inverse_map* maps, int nmaps, int B,
                                      size_t* bytes);
int pcs_inverse_index_batch(const pcs_inverse_map* maps, int nmaps, int B, void* workspace,
                            size_t ws_bytes, void* stream);
/* common.py:64-65 backward without atomics: grad_feats (B,N,D) = sum of
 * grad_out[slot][3 + c] over the slots reading each point (overwrites).  n_slots =
 * the grouped rows (B*C*K; sizes the launch probe's byte model only).  D <= 512.
 * (ABI 3: n_slots added.) */
int pcs_group_bwd_csr(const float* grad_out, int ld_gout, const int32_t* offsets,
                      const int32_t* entries, int B, int N, int D, long long n_slots,
                      float* grad_feats, void* stream);
/* common.py:115-122 backward without atomics: grad_pts (B,M,D) (overwrites).
 * n_slots = 3 x the fine rows.  D <= 512.  (ABI 3: n_slots added.) */
int pcs_interp_bwd_csr(const float* grad_out, int ld_gout, int col_off,
                       const float* dist, const int32_t* offsets,
                       const int32_t* entries, int B, int M, int D, long long n_slots,
                       float* grad_pts, void* stream);

/* ---- block batches --------------------------------------------------------- */

/* data_processing/block_datasets.py:5-31,118-128: a padded batch gathered from an
 * HBM-resident block store.  points (P,9) f32, labels (P,14) u8, src (rows)
 * int64 store row per output row (< 0 = zero padding); out_points (rows,9),
 * out_labels (rows,14). */
int pcs_gather_blocks(const float* points, const uint8_t* labels,
                      const long long* src, long long rows, float* out_points,
                      uint8_t* out_labels, void* stream);

/* ---- optimizer -------------------------------------------------------------- */

/* torch.optim.Adam step (amsgrad=False; the reference trains with Adam lr 1e-3,
 * Training/train_model.py:263) over flat fp32 arrays of n parameters: p, g, m
 * (exp_avg), v (exp_avg_sq); beta1_w = 1 - beta1, beta2_w = 1 - beta2 (computed in
 * double, as torch does with python floats), step = -lr / (1 - beta1^t),
 * bc2_sqrt = sqrt(1 - beta2^t).  16-byte aligned buffers. */
int pcs_adam(float* p, const float* g, float* m, float* v, long long n, float beta1_w,
             float beta2, float beta2_w, float step, float bc2_sqrt, float eps,
             float weight_decay, void* stream);
/* pcs_adam with the step count on the device (graph-capturable: a captured step replays
 * correctly): state = 16 B of zero-initialised device memory {int64 t; float coef[2]}; each
 * call does t += 1 and the bias corrections step = -lr / (1 - beta1^t), bc2_sqrt =
 * sqrt(1 - beta2^t) in double on the device (the host path's arithmetic), then the update. */
int pcs_adam_dev(float* p, const float* g, float* m, float* v, long long n, float beta1_w,
                 float beta2_f, float beta2_w, double lr, double beta1, double beta2, float eps,
                 float weight_decay, long long* state, void* stream);

/* ---- loss ---------------------------------------------------------------- */

/* Training/train_model.py:15-57 `masked_onehot_cross_entropy`: logits (B,L,C)
 * rows of stride ld, one-hot targets (u8 when target_kind = 0, f32 when 1) rows
 * of stride ldt, lengths (B) int32; loss (1 float) = mean over positions
 * l < lengths[b] of -sum_c onehot*log_softmax (0 if none).  grad (nullable,
 * rows of stride ld) = d loss / d logits.  partial: fp64 workspace of
 * pcs_masked_ce_blocks(B, L) entries.  C <= 64. */
int pcs_masked_ce_blocks(int B, int L);
int pcs_masked_ce(const float* logits, int ld, const void* targets,
                  int target_kind, int ldt, const int32_t* lengths, int B,
                  int L, int C, double* partial, float* loss, float* grad,
                  void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PCSEG_H_ */
