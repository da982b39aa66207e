// Native orchestration of a shared-MLP stack: one ABI call runs a whole
// conv1x1 -> BatchNorm -> act [-> max over K] stack forward (or backward), so the
// host pays one call per MiniPointNet / UnitPointNet / EdgeConv / DGCNN conv block
// instead of one Python round trip per kernel.
//
// Reference semantics: MiniPointNet / UnitPointNet (models/utils/common.py:125-178)
// followed by reduce(..., 'max') (common.py:211-212), EdgeConv (models/dgcnn/dgcnn.py:
// 67-76), DGCNN conv5..conv7 (dgcnn.py:188-207); nn.BatchNorm train/eval semantics
// (batch statistics + running-stat update with the unbiased variance, or running
// statistics in eval mode).
//
// The kernels are the engine's (mlp.hip / gemm_direct.hip): forward per layer = one
// row GEMM with the previous layer's BN+act applied on load and fp64 BN partials in
// its epilogue + one finalize; backward per layer = one wgrad + one dgrad whose
// epilogue already reduces the previous layer's BN-backward sums + one finalize.
// Scratch comes from a caller-provided workspace (pcs_mlp_workspace bytes).
#include "mlp_common.hpp"

#include <algorithm>
#include <mutex>
#include <vector>

namespace pcs {

// eval-mode BatchNorm: s = gamma * rsqrt(var + eps), t = beta - mean * s, from running stats
__global__ __launch_bounds__(256) void bn_eval_coef_kernel(const float* __restrict__ rm, const float* __restrict__ rv,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float eps, int N,
                                                           float* __restrict__ coef) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n >= N) return;
    const float inv = 1.0f / sqrtf(rv[n] + eps);
    const float m = rm[n];
    const float sc = (gamma ? gamma[n] : 1.f) * inv;
    coef[n] = sc;
    coef[N + n] = (beta ? beta[n] : 0.f) - m * sc;
    coef[2 * N + n] = m;
    coef[3 * N + n] = inv;
}

// out (cols x rows) = in (rows x cols, row stride ld)^T ; out row stride = rows
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ in, int rows, int cols, int ld,
                                                        float* __restrict__ out) {
    __shared__ float tile[32][33];
    const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int y = ty; y < 32; y += 8) {
        const int r = r0 + y, c = c0 + tx;
        tile[y][tx] = (r < rows && c < cols) ? in[(size_t)r * ld + c] : 0.f;
    }
    __syncthreads();
    for (int y = ty; y < 32; y += 8) {
        const int c = c0 + y, r = r0 + tx;
        if (c < cols && r < rows) out[(size_t)c * rows + r] = tile[tx][y];
    }
}

__global__ __launch_bounds__(256) void zero_kernel(float* __restrict__ p, long long n) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) p[i] = 0.f;
}

static void zero_f32(float* p, long long n, hipStream_t st) {
    if (n <= 0) return;
    long long g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(zero_kernel, dim3((unsigned)g), dim3(256), 0, st, p, n);
}

// columns [c0, ld) of M rows := 0 (the pad columns a GEMM writing c0 channels leaves untouched)
__global__ __launch_bounds__(256) void zero_cols_kernel(float* __restrict__ p, long long M, int ld, int c0) {
    const int w = ld - c0;
    const long long n = M * w;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const long long r = i / w;
        p[r * ld + c0 + (i - r * w)] = 0.f;
    }
}

static void zero_cols(float* p, long long M, int ld, int c0, hipStream_t st) {
    if (M <= 0 || c0 >= ld) return;
    long long g = (M * (ld - c0) + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(zero_cols_kernel, dim3((unsigned)g), dim3(256), 0, st, p, M, ld, c0);
}

// ---------------------------------------------------------------- workspace carving
struct Carve {
    char* base;
    size_t used, cap;
    template <typename T>
    T* take(size_t count) {
        const size_t off = (used + 255) & ~size_t(255);
        used = off + count * sizeof(T);
        return base ? reinterpret_cast<T*>(base + off) : nullptr;
    }
};

static int max_cout(const pcs_mlp_layer* L, int nl) {
    int m = 4;
    for (int l = 0; l < nl; ++l) m = (int)L[l].cout > m ? (int)L[l].cout : m;
    return m;
}

// partial-sum entries (doubles) the finalize of every stage needs, maximum over stages
static size_t max_partials(int M, int kin, const pcs_mlp_layer* L, int nl, int pool_k, bool backward) {
    size_t m = 0;
    for (int l = 0; l < nl; ++l) {
        const size_t c = (size_t)L[l].cout;
        m = std::max(m, 2 * c * (size_t)pcs_gemm_row_blocks(M, (int)c));
        if (backward) m = std::max(m, 2 * c * (size_t)pcs_gemm_row_blocks_dgrad(M, (int)c));
        // a fused inner layer writes its input's BN-backward partials, one per fused block
        if (backward && l > 0) {
            m = std::max(m, 2 * (size_t)L[l].cin * (size_t)fused_bwd_grid(M, (int)L[l].cout, (int)L[l].cin, true, -1));
            if (L[l].cout == 128 && L[l].cin % 128 == 0)
                m = std::max(m, 2 * (size_t)L[l].cin * (size_t)bwd_ring_grid(M, (int)L[l].cin));
        }
    }
    if (backward) {
        const size_t c = (size_t)L[nl - 1].cout;
        const size_t nb = pool_k ? (size_t)pcs_pool_bwd_reduce_blocks(M / pool_k) : (size_t)pcs_bn_bwd_reduce_blocks(M);
        m = std::max(m, 2 * c * nb);
    }
    (void)kin;
    return m;
}

// A layer's backward GEMMs read its dZ once per column tile (dz_passes); rebuilt on load,
// every pass reads two arrays (dy and Z), materialised once (read 2, write 1) every pass
// reads one.  From 4 passes on the materialised form moves fewer bytes (DGCNN conv5-7:
// -2.1 ms of GEMM time for +0.5 ms of materialising, scripts/dgcnn_head_ab.py).
// (lower thresholds, 2 and 3 passes, and a byte-model policy measured slower: profiles/r05_ab_dz_threshold.txt,
// profiles/r05_ab_dz_policy.txt)
constexpr int kDzPasses = 4;
static bool materialize_dz_of(const pcs_mlp_layer& P, int M, bool dgrad) {
    return dz_passes(M, (int)P.cout, (int)P.cin, dgrad, P.dW != nullptr) >= kDzPasses;
}

// the ring kernel (bwd_ring.hip) takes the eligible 128-wide BNBWD inner layers under policy 'all'
// only: isolated it runs 127 us per FP1 layer (0.43 of the fp32 MFMA peak) and the PointNet++ step
// measured 4.80 ms with it against 4.55 ms on the default dgrad + lane-wgrad pair
static bool ring_wanted(int policy) { return policy == PCS_BWD_FUSE_ALL; }

// Rotation depth of a backward's dA / kB / alpha buffers.  The dgrad of layer l reuses the buffers
// that layer l + kRot - 1's wgrad reads, so it must wait for that wgrad on the lane; with kRot = 6 no
// stack of the models (<= 5 layers) ever waits.  (Round 4 rotated over 3: the dgrads of FP1's first two
// layers waited ~90 us each for the lane's wgrads of layers 3 / 4; A/B in profiles/r05_ab_rotation.txt.)
constexpr int kRot = 6;

struct BwdScratch {
    float* dz;             // the top layer's materialised dZ (M x cout), when it is wide
    bool dz_ok(bool top) const { return !top || dz != nullptr; }
    double* part;
    float* kb[kRot];       // BN-backward coefficients and data gradients rotate over kRot buffers:
    float* alpha[kRot];    // a layer's wgrad (side stream) may still read one while the next
                           // kRot - 1 layers' dgrads run
    float* wt;
    float* dA[kRot];
    char* wg;              // wgrad partial tiles (shared by the call's wgrads: one side stream)
    size_t wg_bytes;
    char* wg0;             // the first layer's, when its wgrad runs on the caller's stream
    size_t wg0_bytes;
    char* fw;              // fused inner layers' dW partials (caller's stream only)
    size_t fw_bytes;
    float* drop;           // the top layer's output gradient through its dropout (when not materialised)
};

static size_t carve_backward(Carve& cv, int M, int kin, int ldx, const pcs_mlp_layer* L, int nl, int pool_k,
                             BwdScratch* out) {
    const int mc = std::max(max_cout(L, nl), ldx);
    BwdScratch s{};
    s.part = cv.take<double>(max_partials(M, kin, L, nl, pool_k, true));
    for (int i = 0; i < kRot; ++i) { s.kb[i] = cv.take<float>(mc); s.alpha[i] = cv.take<float>(mc); }
    size_t wt = 0, da = 0;
    for (int l = 0; l < nl; ++l) {
        wt = std::max(wt, (size_t)L[l].cout * (size_t)L[l].ldw);
        if (l > 0) da = std::max(da, (size_t)M * (size_t)L[l].cin);
    }
    s.wt = cv.take<float>(wt);
    // as many dA buffers as the stack's dgrads use (nl - 1), at most kRot
    for (int i = 0; i < kRot; ++i) s.dA[i] = i < std::max(1, std::min(nl - 1, kRot)) ? cv.take<float>(da) : nullptr;
    size_t wg = 0;
    for (int l = 0; l < nl; ++l)
        if (L[l].dW) wg = std::max(wg, wgrad_ws_bytes((int)L[l].cout, (int)L[l].cin, M));
    s.wg_bytes = wg;
    s.wg = cv.take<char>(wg);
    s.wg0_bytes = L[0].dW ? wgrad_ws_bytes((int)L[0].cout, (int)L[0].cin, M) : 0;
    s.wg0 = cv.take<char>(s.wg0_bytes);
    size_t fw = 0;
    for (int l = 1; l < nl; ++l)
        if (L[l].dW) {
            fw = std::max(fw, fused_bwd_ws_bytes(M, (int)L[l].cout, (int)L[l].cin));
            if (L[l].cout == 128 && L[l].cin % 128 == 0) fw = std::max(fw, bwd_ring_ws_bytes(M, 128, (int)L[l].cin));
        }
    if (L[0].dW && L[0].cin <= 32) fw = std::max(fw, fused_wgrad_ws_bytes(M, (int)L[0].cout, (int)L[0].cin));
    s.fw_bytes = fw;
    s.fw = cv.take<char>(fw);
    s.dz = materialize_dz_of(L[nl - 1], M, true) ? cv.take<float>((size_t)M * (size_t)L[nl - 1].cout) : nullptr;
    s.drop = L[nl - 1].drop_p > 0.0 && !s.dz ? cv.take<float>((size_t)M * (size_t)L[nl - 1].cout) : nullptr;
    if (out) *out = s;
    return cv.used;
}

// the top layer's pooling is fused into its GEMM epilogue (z-space max/min + pool_finalize)
static bool fused_pool(int pool_k) { return pool_k == 16 || pool_k == 32; }

struct FwdScratch {
    double* part;
    float* pz;
    unsigned char* pa;
};

static size_t carve_forward(Carve& cv, int M, int kin, const pcs_mlp_layer* L, int nl, int pool_k, FwdScratch* out) {
    FwdScratch s{};
    s.part = cv.take<double>(max_partials(M, kin, L, nl, pool_k, false));
    if (fused_pool(pool_k)) {
        const size_t gn = (size_t)(M / pool_k) * (size_t)L[nl - 1].cout;
        s.pz = cv.take<float>(gn);              // the one extreme per channel (gemm_rows_ex's pz / pa)
        s.pa = cv.take<unsigned char>(gn);
    }
    if (out) *out = s;
    return cv.used;
}

// ---------------------------------------------------------------- wgrad on a second stream
// In a stack's backward, layer l's weight gradient and data gradient both only READ the
// layer's rebuilt dZ; they are independent GEMMs.  The wgrad runs on a per-device side
// stream (forked from the caller's stream by an event), so it overlaps the dgrad and the
// BN-backward finalize of the same layer; the caller's stream joins it before the next
// layer's dgrad, whose outputs (the dA buffer and the BN-backward coefficients) recycle
// the buffers this wgrad reads.  A backward call holds its lane's lock from the first fork to
// the final join, so concurrent callers on one device never share the event ring; all of a
// call's wgrads run in order on the side stream and share one partial-tile workspace.
struct WgradLane {
    hipStream_t side = nullptr;
    hipEvent_t ev[16] = {};     // two per forked wgrad: a whole stack's forks before the ring wraps
    int next = 0;
    std::mutex use;
};

static WgradLane* wgrad_lane() {
    static WgradLane lanes[16];
    static std::mutex mu;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
    std::lock_guard<std::mutex> g(mu);
    WgradLane& L = lanes[dev];
    if (!L.side) {
        // normal priority (0), below a high-priority caller stream, so the critical path gets free
        // CUs first (the lane at the caller's high priority measured slower,
        // profiles/r03_ab_s14_lane_priority.txt; at the lowest priority it was neutral,
        // profiles/r05_ab_lane_priority.txt)
        if (hipStreamCreateWithPriority(&L.side, hipStreamNonBlocking, 0) != hipSuccess) {
            L.side = nullptr;
            return nullptr;
        }
        for (auto& e : L.ev)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    }
    return &L;
}

static hipEvent_t lane_event(WgradLane* L) {
    hipEvent_t e = L->ev[L->next];
    L->next = (L->next + 1) & 15;
    return e;
}

static pcs_operand plain_op(const float* data, int ld) {
    pcs_operand o{};
    o.data = data; o.ld = ld; o.mode = PCS_OP_PLAIN;
    return o;
}

static pcs_operand bnact_op(const float* data, int ld, const pcs_mlp_layer& P) {
    pcs_operand o = plain_op(data, ld);
    o.mode = PCS_OP_BNACT;
    o.s = P.coef; o.t = P.coef + P.cout; o.act = (int)P.act; o.slope = (float)P.slope;
    return o;
}

// BN-backward operand of layer P (its dZ rebuilt from output gradient `dy` and P.Z)
static pcs_operand bnbwd_op(const float* dy, int ld, const pcs_mlp_layer& P, const float* alpha, const float* kb) {
    pcs_operand o = bnact_op(dy, ld, P);
    o.mode = PCS_OP_BNBWD;
    o.z = P.Z; o.ldz = (int)P.cout;
    o.mean = P.coef + 2 * P.cout; o.inv = P.coef + 3 * P.cout;
    o.alpha = alpha; o.kb = kb;
    return o;
}

static int check_layers(int M, int kin, int ldx, const pcs_mlp_layer* L, int nl, int pool_k, const char* who) {
    PCS_CHECK_ARG(M >= 0 && kin >= 1 && ldx >= kin && ldx % 4 == 0 && L && nl >= 1,
                  "%s: bad sizes M=%d kin=%d ldx=%d nl=%d", who, M, kin, ldx, nl);
    PCS_CHECK_ARG(pool_k == 0 || (pool_k >= 1 && pool_k <= 256 && M % pool_k == 0),
                  "%s: pool_k=%d must divide M=%d and be <= 256", who, pool_k, M);
    int cin = kin;
    for (int l = 0; l < nl; ++l) {
        PCS_CHECK_ARG(L[l].W && L[l].Z && L[l].coef, "%s: layer %d: W/Z/coef missing", who, l);
        PCS_CHECK_ARG(L[l].cin == cin, "%s: layer %d: cin=%lld, expected %d", who, l, (long long)L[l].cin, cin);
        PCS_CHECK_ARG(L[l].cout >= 4 && L[l].cout % 4 == 0, "%s: layer %d: cout=%lld must be a multiple of 4", who,
                      l, (long long)L[l].cout);
        PCS_CHECK_ARG(L[l].ldw >= L[l].cin && (L[l].ldw % 4 == 0 || l == 0),
                      "%s: layer %d: ldw=%lld (a multiple of 4 except for the first layer)", who, l,
                      (long long)L[l].ldw);
        PCS_CHECK_ARG(L[l].use_batch || (L[l].run_mean && L[l].run_var),
                      "%s: layer %d: eval-mode BatchNorm needs running statistics", who, l);
        PCS_CHECK_ARG(L[l].act >= 0 && L[l].act <= 2, "%s: layer %d: act=%lld", who, l, (long long)L[l].act);
        PCS_CHECK_ARG(L[l].bwd_fuse >= PCS_BWD_FUSE_DEFAULT && L[l].bwd_fuse <= PCS_BWD_FUSE_ALL,
                      "%s: layer %d: bwd_fuse=%lld", who, l, (long long)L[l].bwd_fuse);
        cin = (int)L[l].cout;
    }
    return 0;
}

}  // namespace pcs

using namespace pcs;

PCS_API int pcs_mlp_workspace(int M, int kin, int ldx, const pcs_mlp_layer* layers, int nl, int pool_k, int backward,
                              size_t* bytes) {
    if (int e = check_layers(M, kin, ldx, layers, nl, pool_k, "pcs_mlp_workspace")) return e;
    PCS_CHECK_ARG(bytes, "pcs_mlp_workspace: null bytes");
    Carve cv{nullptr, 0, 0};
    if (backward) carve_backward(cv, M, kin, ldx, layers, nl, pool_k, nullptr);
    else carve_forward(cv, M, kin, layers, nl, pool_k, nullptr);
    *bytes = cv.used + 256;
    return 0;
}

PCS_API int pcs_mlp_forward(const float* X, int ldx, int kin, int M, pcs_mlp_layer* layers, int nl, int pool_k,
                            float* out, int ldo, uint8_t* arg, void* ws, size_t ws_bytes, void* stream) {
    if (int e = check_layers(M, kin, ldx, layers, nl, pool_k, "pcs_mlp_forward")) return e;
    PCS_CHECK_ARG(X && out && (!pool_k || arg), "pcs_mlp_forward: null pointer");
    PCS_CHECK_ARG(layers[nl - 1].drop_p == 0.0 || (!pool_k && layers[nl - 1].drop_p > 0.0 && layers[nl - 1].drop_p < 1.0),
                  "pcs_mlp_forward: drop_p=%g (un-pooled top layer only, 0 <= p < 1)", layers[nl - 1].drop_p);
    const int CT = (int)layers[nl - 1].cout;
    if (ldo == 0) ldo = CT;
    PCS_CHECK_ARG(!pool_k ? (ldo >= CT && ldo % 4 == 0) : ldo == CT,
                  "pcs_mlp_forward: ldo=%d (a multiple of 4 >= cout; pooled outputs are dense)", ldo);
    if (M == 0) return 0;
    hipStream_t st = as_stream(stream);
    Carve cv{static_cast<char*>(ws), 0, ws_bytes};
    FwdScratch S;
    carve_forward(cv, M, kin, layers, nl, pool_k, &S);
    double* part = S.part;
    PCS_CHECK_ARG(ws && cv.used <= ws_bytes, "pcs_mlp_forward: workspace too small (%zu < %zu)", ws_bytes, cv.used);
    const bool fuse = fused_pool(pool_k);

    const float* A = X;
    int lda = ldx, K = kin;
    for (int l = 0; l < nl; ++l) {
        pcs_mlp_layer& P = layers[l];
        const int C = (int)P.cout;
        const pcs_operand a = l == 0 ? plain_op(A, lda) : bnact_op(A, lda, layers[l - 1]);
        float* s = P.coef;
        const bool top_pool = fuse && l == nl - 1;
        float* pz = top_pool ? S.pz : nullptr;
        unsigned char* pa = top_pool ? S.pa : nullptr;
        const int pk = top_pool ? pool_k : 0;
        if (P.use_batch) {
            const int nb = pcs_gemm_row_blocks(M, C);
            if (int e = gemm_rows_ex(&a, M, K, P.W, (int)P.ldw, 0, P.bias, P.Z, C, C, part, nullptr, nullptr, stream,
                                     pz, pa, pk, P.gamma))
                return e;
            const bool track = P.run_mean != nullptr;
            bn_finalize_launch(part, nb, C, M, P.gamma, P.beta, (float)P.eps, track ? (float)P.momentum : 0.f,
                               P.run_mean, P.run_var, s, s + C, s + 2 * C, s + 3 * C,
                               reinterpret_cast<long long*>(P.num_batches), st);
        } else {
            if (int e = gemm_rows_ex(&a, M, K, P.W, (int)P.ldw, 0, P.bias, P.Z, C, C, nullptr, nullptr, nullptr, stream,
                                     pz, pa, pk, P.gamma))
                return e;
            hipLaunchKernelGGL(bn_eval_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, st, P.run_mean, P.run_var,
                               P.gamma, P.beta, (float)P.eps, C, s);
        }
        A = P.Z; lda = C; K = C;
    }
    const pcs_mlp_layer& T = layers[nl - 1];
    const int C = (int)T.cout;
    if (fuse)
        return pool_finalize(S.pz, S.pa, M / pool_k, C, T.coef, T.coef + C, (int)T.act,
                             (float)T.slope, out, arg, st);
    if (pool_k)
        return pcs_pool_fwd(T.Z, C, M / pool_k, pool_k, T.coef, T.coef + C, (int)T.act, (float)T.slope, out, arg,
                            stream);
    if (T.drop_p > 0.0)
        return bn_act_dropout(T.Z, C, M, C, T.coef, T.coef + C, (int)T.act, (float)T.slope, out, ldo, T.drop_p,
                              (long long)T.drop_seed, st);
    return pcs_bn_act(T.Z, C, M, C, T.coef, T.coef + C, (int)T.act, (float)T.slope, out, ldo, stream);
}

static int mlp_backward(const float* X, int ldx, int kin, int M, const pcs_mlp_layer* layers, int nl, int pool_k,
                        const uint8_t* arg, const float* gout, int ldg, float* dX, int lddx, void* ws,
                        size_t ws_bytes, void* stream, bool defer) {
    if (int e = check_layers(M, kin, ldx, layers, nl, pool_k, "pcs_mlp_backward")) return e;
    if (lddx == 0) lddx = ldx;
    PCS_CHECK_ARG(lddx >= kin && lddx % 4 == 0, "pcs_mlp_backward: lddx=%d (a multiple of 4 >= kin=%d)", lddx, kin);
    PCS_CHECK_ARG(X && gout && (!pool_k || arg), "pcs_mlp_backward: null pointer");
    PCS_CHECK_ARG(ldg >= (int)layers[nl - 1].cout && ldg % 4 == 0 && (!pool_k || ldg == (int)layers[nl - 1].cout),
                  "pcs_mlp_backward: ldg=%d (a multiple of 4 >= cout; pooled gradients are dense)", ldg);
    if (M == 0) return 0;
    hipStream_t st = as_stream(stream);
    Carve cv{static_cast<char*>(ws), 0, ws_bytes};
    BwdScratch S;
    carve_backward(cv, M, kin, ldx, layers, nl, pool_k, &S);
    PCS_CHECK_ARG(ws && cv.used <= ws_bytes, "pcs_mlp_backward: workspace too small (%zu < %zu)", ws_bytes, cv.used);

    // ---- top layer: BN-backward sums of its output gradient
    const pcs_mlp_layer& T = layers[nl - 1];
    const int CL = (int)T.cout;
    const float* sT = T.coef;
    int nb;
    if (pool_k) {
        const long long G = M / pool_k;
        nb = pcs_pool_bwd_reduce_blocks(G);
        if (int e = pcs_pool_bwd_reduce(gout, arg, T.Z, CL, G, pool_k, sT, sT + CL, sT + 2 * CL, sT + 3 * CL,
                                        (int)T.act, (float)T.slope, S.part, stream))
            return e;
    } else {
        nb = pcs_bn_bwd_reduce_blocks(M);
        // the stack's fused dropout (DGCNN conv6 / conv7, dgcnn.py:196-207; PointNet++ FP1's
        // head): where the top layer's dZ is materialised (the wide layers), the mask is applied
        // on load by this reduce and by the dZ pass -- no masked copy of the gradient; otherwise
        // the masked gradient is written once and read by both consumers
        bool drop_on_load = false;
        if (T.drop_p > 0.0) {
            const pcs_operand xt = bnbwd_op(gout, ldg, T, S.alpha[0], S.kb[0]);
            bool fused_top = false;
            if (nl > 1 && T.dW) {
                pcs_operand q = bnbwd_op(nullptr, 0, layers[nl - 2], nullptr, nullptr);
                q.data = layers[nl - 2].Z;
                q.ld = (int)T.cin;
                fused_top = ring_wanted((int)T.bwd_fuse) && bwd_ring_ok(M, CL, (int)T.cin, T.W, (int)T.ldw, &xt, &q);
                fused_top = fused_top || (fused_bwd_wanted((int)T.bwd_fuse, M) &&
                                          fused_bwd_ok(M, CL, (int)T.cin, (int)T.ldw, &xt, &q));
            }
            drop_on_load = !fused_top && materialize_dz_of(T, M, nl > 1 || dX) && S.dz;
            if (!drop_on_load) {
                float* g2 = S.drop ? S.drop : S.dz;
                PCS_CHECK_ARG(g2, "pcs_mlp_backward: no dropout scratch");
                if (int e = pcs_dropout_bwd(gout, ldg, M, CL, T.drop_p, T.drop_seed, g2, CL, stream)) return e;
                gout = g2;
                ldg = CL;
            }
        }
        if (drop_on_load) {
            if (int e = bn_bwd_reduce_dropout(gout, ldg, T.Z, CL, M, CL, sT, sT + CL, sT + 2 * CL, sT + 3 * CL,
                                              (int)T.act, (float)T.slope, S.part, T.drop_p, (long long)T.drop_seed,
                                              st))
                return e;
        } else if (int e = pcs_bn_bwd_reduce(gout, ldg, T.Z, CL, M, CL, sT, sT + CL, sT + 2 * CL, sT + 3 * CL,
                                             (int)T.act, (float)T.slope, S.part, stream)) {
            return e;
        }
    }
    int pp = 0;
    if (int e = pcs_bn_bwd_finalize(S.part, nb, CL, M, sT, sT + 3 * CL, T.dgamma, T.dbeta, S.kb[pp], S.alpha[pp], 1,
                                    stream))
        return e;
    if (!T.use_batch) { zero_f32(S.kb[pp], CL, st); zero_f32(S.alpha[pp], CL, st); }
    // the top layer's dZ is never materialised: both consumers rebuild it on load
    pcs_operand xop = bnbwd_op(gout, ldg, T, S.alpha[pp], S.kb[pp]);
    if (pool_k) { xop.mode = PCS_OP_POOLBWD; xop.arg = arg; xop.pool_k = pool_k; }

    int da = 0;
    WgradLane* lane = wgrad_lane();
    std::unique_lock<std::mutex> lane_lock;
    if (lane) lane_lock = std::unique_lock<std::mutex>(lane->use);
    hipEvent_t pending = nullptr;          // the last wgrad launched on the side stream
    // done[l]: layer l's wgrad finished.  The dgrad of layer l recycles the dA / kb / alpha
    // buffers (kRot-way rotation) that layer l + kRot - 1's wgrad read, so it waits for that one
    // only: the wgrads above keep running under this dgrad.
    std::vector<hipEvent_t> done(nl, nullptr);
    auto join = [&]() {
        if (pending) {
            (void)hipStreamWaitEvent(st, pending, 0);
            pending = nullptr;
        }
    };
    // every exit after the first fork joins the side stream (its work reads this call's buffers)
    auto fail = [&](int e) {
        join();
        return e;
    };
    for (int l = nl - 1; l >= 0; --l) {
        const pcs_mlp_layer& P = layers[l];
        const int C = (int)P.cout, Cin = (int)P.cin;
        // a thin inner layer with a weight gradient: data + weight gradient in one launch
        // (fused_bwd.hip) from one read of its rebuilt dZ, on the caller's stream
        pcs_operand qop{};
        if (l > 0) {
            qop = bnbwd_op(nullptr, 0, layers[l - 1], nullptr, nullptr);
            qop.data = layers[l - 1].Z;
            qop.ld = Cin;
        }
        // a 128-wide BNBWD inner layer: data + weight gradient on the LDS-DMA ring (bwd_ring.hip)
        const bool ring = l > 0 && P.dW && ring_wanted((int)P.bwd_fuse) &&
                          bwd_ring_ok(M, C, Cin, P.W, (int)P.ldw, &xop, &qop);
        const bool fused = ring || (l > 0 && P.dW && fused_bwd_wanted((int)P.bwd_fuse, M) &&
                                    fused_bwd_ok(M, C, Cin, (int)P.ldw, &xop, &qop));
        if (!fused && materialize_dz_of(P, M, l > 0 || dX) && S.dz_ok(l == nl - 1)) {
            // the top layer's into its own buffer (gout is the caller's), inner ones in place
            // over the dA buffer the rebuilt operand reads
            float* dst = l == nl - 1 ? S.dz : const_cast<float*>(xop.data);
            // the top layer's gradient still carries its dropout when the mask is applied on load
            const bool dm = l == nl - 1 && P.drop_p > 0.0 && xop.data != S.drop && xop.data != S.dz;
            if (int e = materialize_dz(&xop, M, C, dst, C, st, dm ? P.drop_p : 0.0, dm ? (long long)P.drop_seed : 0))
                return fail(e);
            xop = plain_op(dst, C);
        }
        // the first layer's wgrad goes to the caller's stream when no dgrad follows it (the
        // stack's input needs no gradient): it then runs beside the lane's pending wgrads
        // instead of queueing behind them at the end of the backward
        const bool wg_here = l == 0 && !dX && nl > 1;
        if (fused) {
            // its wgrad is part of the fused launch below
        } else if (P.dW && wg_here && fused_bwd_wanted((int)P.bwd_fuse, M) && fused_wgrad_ok(M, C, Cin, ldx, &xop)) {
            if (int e = fused_wgrad(&xop, C, X, ldx, Cin, M, P.dW, P.db, S.fw, S.fw_bytes, st)) return fail(e);
        } else if (P.dW && wg_here) {
            const pcs_operand y = plain_op(X, ldx);
            if (int e = pcs::wgrad_launch(&xop, C, &y, Cin, M, P.dW, P.db, S.wg0, S.wg0_bytes, stream)) return fail(e);
        } else if (P.dW) {
            void* ws_stream = stream;
            if (lane) {                    // fork: the side stream waits for dZ's inputs
                hipEvent_t ready = lane_event(lane);
                (void)hipEventRecord(ready, st);
                (void)hipStreamWaitEvent(lane->side, ready, 0);
                ws_stream = lane->side;
            }
            const pcs_mlp_layer* Q = l > 0 ? &layers[l - 1] : nullptr;
            const pcs_operand y = Q ? bnact_op(Q->Z, Cin, *Q) : plain_op(X, ldx);
            const int e = pcs::wgrad_launch(&xop, C, &y, Cin, M, P.dW, P.db, S.wg, S.wg_bytes, ws_stream);
            if (lane) {                    // recorded even on error, so the join below covers it
                pending = lane_event(lane);
                (void)hipEventRecord(pending, lane->side);
                done[l] = pending;
            }
            if (e) return fail(e);
        }
        if (l + kRot - 1 < nl && done[l + kRot - 1]) (void)hipStreamWaitEvent(st, done[l + kRot - 1], 0);
        if (l == 0 && !dX) break;
        // dgrad B operand: B[k = cout][n = cin] = W[k][n], read k-major straight from W (bt = 1);
        // a first layer whose row stride is not a multiple of 4 goes through the transpose Wt
        const bool bt = P.ldw % 4 == 0;
        const float* Bw = P.W;
        int ldb = (int)P.ldw;
        // (a first layer's dX from column dx_col0 reads W^T's rows c0..: one transpose launch, measured
        // equal to reading W k-major in place with scalar loads, profiles/r03_ab_ev3.txt)
        if (!bt) {
            const dim3 g((Cin + 31) / 32, (C + 31) / 32);
            hipLaunchKernelGGL(transpose_kernel, g, dim3(256), 0, st, P.W, C, Cin, (int)P.ldw, S.wt);
            Bw = S.wt;
            ldb = C;
        }
        if (l > 0) {
            const pcs_mlp_layer& Q = layers[l - 1];
            float* dA = S.dA[da];
            int nbg;
            if (ring) {
                nbg = bwd_ring_grid(M, Cin);
                if (int e = bwd_ring(&xop, &qop, Cin, P.W, (int)P.ldw, M, dA, Cin, S.part, P.dW, P.db, S.fw, S.fw_bytes,
                                     st))
                    return fail(e);
            } else if (fused) {
                nbg = fused_bwd_grid(M, C, Cin, true, xop.mode);
                if (int e = fused_bwd(&xop, C, &qop, Cin, P.W, (int)P.ldw, M, dA, Cin, S.part, P.dW, P.db, S.fw,
                                      S.fw_bytes, st))
                    return fail(e);
            } else {
                nbg = pcs_gemm_row_blocks_dgrad(M, Cin);
                pcs_operand epi = bnbwd_op(nullptr, 0, Q, nullptr, nullptr);
                if (int e = gemm_rows_ex(&xop, M, C, Bw, ldb, bt, nullptr, dA, Cin, Cin, nullptr, &epi, S.part, stream))
                    return fail(e);
            }
            pp = (pp + 1) % kRot;
            const float* sq = Q.coef;
            if (int e = pcs_bn_bwd_finalize(S.part, nbg, Cin, M, sq, sq + 3 * Cin, Q.dgamma, Q.dbeta, S.kb[pp],
                                            S.alpha[pp], 1, stream))
                return fail(e);
            if (!Q.use_batch) { zero_f32(S.kb[pp], Cin, st); zero_f32(S.alpha[pp], Cin, st); }
            xop = bnbwd_op(dA, Cin, Q, S.alpha[pp], S.kb[pp]);
            da = (da + 1) % kRot;
        } else {
            // dX columns [c0, kin): a caller that reads no gradient of the first c0 input columns
            // (the relative coordinates of grouped rows, pcs_mlp_layer.dx_col0) gets a GEMM of
            // kin - c0 outputs on the rows c0.. of W^T -- e.g. 64 instead of 67 (SA2), 128 instead
            // of 131 (SA3): whole column tiles instead of a nearly empty last one
            int c0 = (int)P.dx_col0;
            if (c0 < 0 || c0 >= kin) c0 = 0;
            const bool wide = xop.mode == PCS_OP_PLAIN && (c0 * C) % 4 == 0 &&
                              gemm_nt_ok(xop.data, xop.ld, S.wt + (size_t)c0 * C, C, M, kin - c0, C);
            if (c0 == 0) zero_cols(dX, M, lddx, kin, st);   // the pad columns [kin, lddx); with c0 > 0 the
                                                           // caller reads only [c0, kin): none written
            if (wide) {
                // W^T (kin x C, a few MB) from column c0 on and the wide GEMM, dX = dZ . (W^T)^T with both
                // operands contiguous along C (W^T is already there when the first layer took the
                // transpose above: unaligned rows and c0 == 0)
                if (bt || c0 > 0) {
                    const dim3 g((Cin + 31) / 32, (C + 31) / 32);
                    hipLaunchKernelGGL(transpose_kernel, g, dim3(256), 0, st, P.W, C, Cin, (int)P.ldw, S.wt);
                }
                if (int e = gemm_rows_ex(&xop, M, C, S.wt + (size_t)c0 * C, C, 0, nullptr, dX + c0, lddx, kin - c0,
                                         nullptr, nullptr, nullptr, stream))
                    return fail(e);
            } else if (c0 > 0 && (c0 * C) % 4 == 0) {
                if (bt) {
                    const dim3 g((Cin + 31) / 32, (C + 31) / 32);
                    hipLaunchKernelGGL(transpose_kernel, g, dim3(256), 0, st, P.W, C, Cin, (int)P.ldw, S.wt);
                }
                if (int e = gemm_rows_ex(&xop, M, C, S.wt + (size_t)c0 * C, C, 0, nullptr, dX + c0, lddx, kin - c0,
                                         nullptr, nullptr, nullptr, stream))
                    return fail(e);
            } else if (c0 > 0) {
                // W read k-major in place from column c0 (scalar loads where its rows are unaligned)
                if (int e = gemm_rows_ex(&xop, M, C, P.W + c0, (int)P.ldw, 1, nullptr, dX + c0, lddx, kin - c0,
                                         nullptr, nullptr, nullptr, stream))
                    return fail(e);
            } else if (int e = gemm_rows_ex(&xop, M, C, Bw, ldb, bt, nullptr, dX, lddx, kin, nullptr, nullptr, nullptr,
                                            stream)) {
                return fail(e);
            }
        }
    }
    if (!defer) join();
    return launch_status("pcs_mlp_backward");
}

PCS_API int pcs_mlp_backward(const float* X, int ldx, int kin, int M, const pcs_mlp_layer* layers, int nl,
                             int pool_k, const uint8_t* arg, const float* gout, int ldg, float* dX, int lddx,
                             void* ws, size_t ws_bytes, void* stream) {
    return mlp_backward(X, ldx, kin, M, layers, nl, pool_k, arg, gout, ldg, dX, lddx, ws, ws_bytes, stream, false);
}

PCS_API int pcs_mlp_backward_deferred(const float* X, int ldx, int kin, int M, const pcs_mlp_layer* layers, int nl,
                                      int pool_k, const uint8_t* arg, const float* gout, int ldg, float* dX,
                                      int lddx, void* ws, size_t ws_bytes, void* stream) {
    return mlp_backward(X, ldx, kin, M, layers, nl, pool_k, arg, gout, ldg, dX, lddx, ws, ws_bytes, stream, true);
}

PCS_API int pcs_wgrad_lane(void** side_stream) {
    PCS_CHECK_ARG(side_stream, "pcs_wgrad_lane: null pointer");
    WgradLane* lane = wgrad_lane();
    *side_stream = lane ? lane->side : nullptr;
    return 0;
}

PCS_API int pcs_geometry_stream(void** stream) {
    PCS_CHECK_ARG(stream, "pcs_geometry_stream: null pointer");
    static hipStream_t streams[16];
    static std::mutex mu;
    int dev = 0;
    *stream = nullptr;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return launch_status("pcs_geometry_stream");
    std::lock_guard<std::mutex> g(mu);
    if (!streams[dev]) {
        // normal priority (0, a torch.cuda.Stream's), below the bench's high-priority step stream
        // (the lowest priority measured neutral, profiles/r05_ab_geometry_blocks.txt)
        if (hipStreamCreateWithPriority(&streams[dev], hipStreamNonBlocking, 0) != hipSuccess) {
            streams[dev] = nullptr;
            return launch_status("pcs_geometry_stream");
        }
    }
    *stream = streams[dev];
    return 0;
}

PCS_API int pcs_wgrad_lane_join(void* stream) {
    WgradLane* lane = wgrad_lane();
    if (!lane) return 0;
    std::lock_guard<std::mutex> g(lane->use);
    hipEvent_t e = lane_event(lane);
    if (hipEventRecord(e, lane->side) != hipSuccess || hipStreamWaitEvent(as_stream(stream), e, 0) != hipSuccess)
        return launch_status("pcs_wgrad_lane_join");
    return 0;
}
