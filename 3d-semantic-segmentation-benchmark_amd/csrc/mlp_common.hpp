// Shared definitions of the shared-MLP engine kernels (mlp.hip, gemm_direct.hip):
// operand descriptors with their on-load transforms and the row-GEMM argument block.
#pragma once

#include <algorithm>
#include <functional>

#include "pcs_common.hpp"

namespace pcs {

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { ACT_RELU = 0, ACT_LRELU = 1, ACT_NONE = 2 };

// The activation is folded into one slope at the ABI boundary (eff_slope): ReLU = 0,
// LeakyReLU = its slope, identity = 1; both functions are branch-free selects.
// derivative as autograd computes it: relu -> (result > 0); leaky_relu -> (input > 0 ? 1 : slope)
__device__ __forceinline__ float act_f(float y, int, float slope) { return y > 0.f ? y : y * slope; }
__device__ __forceinline__ float dact_f(float y, int, float slope) { return y > 0.f ? 1.f : slope; }

static inline float eff_slope(int act, float slope) {
    return act == ACT_RELU ? 0.f : act == ACT_LRELU ? slope : 1.f;
}

// Operand descriptor (layout-identical to pcs_operand in include/pcseg.h).  The
// value fed to the MFMA for channel c of row r is
//   PLAIN   : data[r][c]
//   BNACT   : act(data[r][c]*s[c] + t[c])                  (forward: previous layer's BN + act)
//   BNBWD   : s*dy - kb - alpha*(z - mean),  dy = data[r][c]*act'(z*s+t), z = Z[r][c]
//   POOLBWD : as BNBWD with data[r][c] = (arg[g][c] == k) ? dpool[g][c] : 0, g = r / pool_k, k = r % pool_k
// i.e. BNBWD/POOLBWD rebuild the layer's dZ (BatchNorm backward) on the fly from its
// output gradient and pre-BN Z, so dZ is never written to HBM.
struct Operand {
    const float* data; int ld; int mode;
    const float* s; const float* t; int act; float slope;
    const float* z; int ldz;
    const float* mean; const float* inv; const float* alpha; const float* kb;
    const unsigned char* arg; int pool_k;
    int rows, cols;           // the operand's extent (rows x logical channels): debug bounds checks only
};
enum { OP_PLAIN = 0, OP_BNACT = 1, OP_BNBWD = 2, OP_POOLBWD = 3 };

// per-channel coefficients of a transform, for 4 consecutive channels
struct Quad {
    float4 s, t, mean, alpha, kb;
};

// transform modes require K % 4 == 0 (checked at the ABI), so a channel quad is all in or all
// out.  Loads use clamped (always in-bounds) addresses and selects instead of branches, so
// the compiler keeps the next slab's loads in flight under the current slab's MFMAs.
template <int MODE>
__device__ __forceinline__ void load_quad(const Operand& o, int c, int K, Quad& q) {
    const int cc = c < K ? c : 0;          // the out-of-range quad is zeroed in xform4
    if (MODE >= OP_BNACT) {
        q.s = *reinterpret_cast<const float4*>(o.s + cc);
        q.t = *reinterpret_cast<const float4*>(o.t + cc);
    }
    if (MODE >= OP_BNBWD) {
        q.mean = *reinterpret_cast<const float4*>(o.mean + cc);
        q.alpha = *reinterpret_cast<const float4*>(o.alpha + cc);
        q.kb = *reinterpret_cast<const float4*>(o.kb + cc);
    }
}

// r / pool_k and r % pool_k of a POOLBWD operand: shifts when pool_k is a power of two (every
// PointNet++-family pool: K = 16, 32, 64), a division otherwise -- the engine's group sizes made the
// per-element 32-bit divisions a large share of the operand loaders' VALU work
__device__ __forceinline__ int pool_group(const Operand& o, int r) {
    const int k = o.pool_k;
    return (k & (k - 1)) == 0 ? r >> (31 - __clz(k)) : r / k;
}
__device__ __forceinline__ unsigned pool_slot(const Operand& o, int r) {
    const int k = o.pool_k;
    return (unsigned)((k & (k - 1)) == 0 ? (r & (k - 1)) : r - (r / k) * k);
}

// raw global loads of one float4 at (row r, channels c..c+3); r and c must be in bounds
// (callers clamp).  POOLBWD: v = dpool[g][c..], a = the 4 argmax bytes; z only for BNBWD/POOLBWD.
template <int MODE>
__device__ __forceinline__ void load_raw(const Operand& o, int r, int c, float4& v, float4& z, unsigned& a) {
    PCS_DCHECK(o.rows <= 0 || (r >= 0 && r < o.rows && c >= 0 && c + 4 <= ((o.cols + 3) & ~3)),
               "operand load row %d col %d outside %d x %d (mode %d)", r, c, o.rows, o.cols, MODE);
    if (MODE == OP_POOLBWD) {
        const int g = pool_group(o, r);
        v = *reinterpret_cast<const float4*>(o.data + (size_t)g * o.ld + c);
        a = *reinterpret_cast<const unsigned*>(o.arg + (size_t)g * o.ld + c);
    } else {
        v = *reinterpret_cast<const float4*>(o.data + (size_t)r * o.ld + c);
    }
    if (MODE >= OP_BNBWD) z = *reinterpret_cast<const float4*>(o.z + (size_t)r * o.ldz + c);
}

template <int MODE>
__device__ __forceinline__ float xform1(const Operand& o, float v, float z, float s, float t, float mean, float alpha,
                                        float kb) {
    if (MODE == OP_BNACT) return act_f(v * s + t, o.act, o.slope);
    if (MODE >= OP_BNBWD) {
        const float dy = v * dact_f(z * s + t, o.act, o.slope);
        return s * dy - kb - alpha * (z - mean);
    }
    return v;
}

// transformed float4 of row r: channels at or beyond K give 0 (per element for PLAIN,
// whose K need not be a multiple of 4); POOLBWD keeps dpool only where argmax == r % pool_k
template <int MODE>
__device__ __forceinline__ float4 xform4(const Operand& o, float4 v, float4 z, unsigned a, int r, const Quad& q,
                                         int c, int K) {
    if (MODE == OP_PLAIN) {
        v.x = c + 0 < K ? v.x : 0.f;
        v.y = c + 1 < K ? v.y : 0.f;
        v.z = c + 2 < K ? v.z : 0.f;
        v.w = c + 3 < K ? v.w : 0.f;
        return v;
    }
    if (MODE == OP_POOLBWD) {
        const unsigned k = pool_slot(o, r);
        v.x = (a & 0xffu) == k ? v.x : 0.f;
        v.y = ((a >> 8) & 0xffu) == k ? v.y : 0.f;
        v.z = ((a >> 16) & 0xffu) == k ? v.z : 0.f;
        v.w = (a >> 24) == k ? v.w : 0.f;
    }
    float4 out;
    out.x = xform1<MODE>(o, v.x, z.x, q.s.x, q.t.x, q.mean.x, q.alpha.x, q.kb.x);
    out.y = xform1<MODE>(o, v.y, z.y, q.s.y, q.t.y, q.mean.y, q.alpha.y, q.kb.y);
    out.z = xform1<MODE>(o, v.z, z.z, q.s.z, q.t.z, q.mean.z, q.alpha.z, q.kb.z);
    out.w = xform1<MODE>(o, v.w, z.w, q.s.w, q.t.w, q.mean.w, q.alpha.w, q.kb.w);
    const bool in = c < K;
    return in ? out : make_float4(0.f, 0.f, 0.f, 0.f);
}

// inverted-dropout keep test of element i, counter-based: the lowbias32 integer hash (C. Wellons)
// of a Weyl step of the 32-bit element index, mixed with the 64-bit seed -- 32-bit multiplies only.
// (Round 4 used the splitmix64 finaliser, whose 64-bit multiplies made the dropout-masked DGCNN
// conv6 / conv7 reduce and dZ passes VALU-bound: 299 vs ~150 us for conv6's reduce in-step.)  Same
// Bernoulli(1 - p) keep as torch's nn.Dropout, a different random stream.
__device__ __forceinline__ bool dropout_keep(unsigned long long seed, unsigned long long i, unsigned thr) {
    unsigned x = (unsigned)i * 0x9E3779B9u + (unsigned)seed;
    x ^= (unsigned)(i >> 32) * 0x85EBCA6Bu ^ (unsigned)(seed >> 32);
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x >= thr;
}

// a stack's fused inverted dropout, applied to its output gradient where that is read
// (seed, keep threshold, 1 / (1 - p)); on = 0: off
struct DropMask {
    unsigned long long seed;
    unsigned thr;
    float scale;
    int on;
    __device__ __forceinline__ float apply(float g, unsigned long long i) const {
        return dropout_keep(seed, i, thr) ? g * scale : 0.f;
    }
};
DropMask drop_mask(double p, long long seed);
// pcs_bn_bwd_reduce with the stack's dropout applied to dA on load (mlp.hip)
int bn_bwd_reduce_dropout(const float* dA, int ldd, const float* Z, int ldz, int M, int N, const float* s,
                          const float* t, const float* mean, const float* inv, int act, float slope, double* part,
                          double p, long long seed, hipStream_t st);

struct GemmArgs {
    Operand a; int M; int K;                   // A rows (M x K) through its transform
    const float* W; int ldw;                   // B[k][n] = W[n*ldw + k]
    const float* bias;                         // per n (or null)
    float* C; int ldc; int N;                  // output rows (M x N)
    double* stats;                             // [2][N][gridDim.x]: sum, sum of squares of C (or null)
    // fused BN-backward reduce of the layer whose OUTPUT space C lives in (dgrad epilogue):
    // uses e.z (its pre-BN Z, M x N), e.s, e.t, e.mean, e.inv, e.act, e.slope
    Operand e;
    double* bstats;                            // [2][N][gridDim.x]: sum dy, sum dy*xhat (or null)
    // fused max-or-min pooling of C over groups of pool_k consecutive rows (pool_k = 16 or 32; 0 =
    // off): pz [M/pool_k][N] = the max of C for columns with psign[n] >= 0 (or psign null), the min
    // for psign[n] < 0 -- the one extreme a monotone consumer act(s*z+t) with sign(s) = sign(psign)
    // needs -- and pa [M/pool_k][N] its first row within the group (pool_finalize)
    float* pz; unsigned char* pa; int pool_k; const float* psign;
};

// bn_finalize_kernel launch that also bumps BatchNorm.num_batches_tracked (nbt, nullable)
void bn_finalize_launch(const double* part, int nb, int N, long long M, const float* gamma, const float* beta,
                        float eps, float momentum, float* run_mean, float* run_var, float* s, float* t, float* mean,
                        float* invstd, long long* nbt, hipStream_t st);
// bn_bwd_finalize_kernel launch: (sum dy, sum dy*xhat) partials -> dgamma/dbeta (+= when accum), kB, kC
void bn_bwd_finalize_launch(const double* part, int nb, int N, long long M, const float* s, const float* inv,
                            float* dgamma, float* dbeta, float* kB, float* kC, int accum, hipStream_t st);
// column passes of a layer's backward GEMMs over its dZ (M x C; cin = the layer's input width)
int dz_passes(int M, int C, int cin, bool dgrad, bool wgrad);
// out (M x C, stride ldo) = the BNBWD / POOLBWD operand x materialised (bitwise the on-load values)
// (drop_p > 0: the BNBWD operand's gradient through the stack's dropout mask, drop_seed)
int materialize_dz(const pcs_operand* x, int M, int C, float* out, int ldo, hipStream_t st, double drop_p = 0.0,
                   long long drop_seed = 0);
// row GEMM with W row-major N x K (bt = 0, = pcs_gemm_rows) or K x N (bt = 1)
int gemm_rows_ex(const pcs_operand* a, int M, int K, const float* W, int ldw, int bt, const float* bias, float* C,
                 int ldc, int N, double* stats, const pcs_operand* epi, double* bstats, void* stream,
                 float* pz = nullptr, unsigned char* pa = nullptr, int pool_k = 0, const float* psign = nullptr);
// the 64 x 64 data gradient through an LDS-DMA ring (dgrad.hip): bitwise
// gemm_rows_kernel<64, 64, 2, 2, PLAIN | BNBWD | POOLBWD, true, 0 | EPI_BWD> for the shapes dgrad_dma_ok accepts;
// gx = the row blocks (= BN-backward partials per column)
bool dgrad_dma_ok(const pcs_operand* a, int M, int K, const float* W, int ldw, int N);
const char* dgrad_dma_name(bool bwd, int mode, int N);  // the kernel dgrad_dma launches (probe / profile name)
// force a column tile x ring variant for the calling thread's next launches (0 = the policy; 1: 64 x 3,
// 2: 128 x 2, 3: 128 x 3); -1 = the register-staged row GEMM instead of the DMA kernel
void dgrad_force_variant(int v);
int dgrad_forced_variant();
int dgrad_dma(const pcs_operand* a, int M, int K, const float* W, int ldw, float* C, int ldc, int N,
              const pcs_operand* epi, double* bstats, int gx, hipStream_t st);
// the forward row GEMM through an LDS-DMA ring (fwd_dma.hip): C = T(A) . W^T + bias with A PLAIN or
// BNACT, K % 32 == 0, optional fp64 BN partials (stats, gx row blocks) and fused pooling (pz / pa /
// pool_k 16 | 32 / psign) -- gemm_rows_kernel's epilogue
bool fwd_dma_ok(const pcs_operand* a, int M, int K, const float* W, int ldw, int N, int pool_k, const float* bias);
const char* fwd_dma_name(bool xf, bool stats, bool pool, int N);
int fwd_dma(const pcs_operand* a, int M, int K, const float* W, int ldw, const float* bias, float* C, int ldc, int N,
            double* stats, int gx, float* pz, unsigned char* pa, int pool_k, const float* psign, hipStream_t st);
// wide-layer GEMM on plain operands (gemm_big.hip): C = A . B^T, A (M x R), B (N x R) row-major
bool gemm_nt_regime(int M, int N);                 // (M, N) the wide path is built for
int gemm_nt_row_tiles(int M);                      // its BN-partial row blocks
int gemm_nt_bn(int N);                             // its column tile (128 or 256)
bool gemm_nt_ok(const float* A, int lda, const float* B, int ldb, int M, int N, int R);
int gemm_nt(const float* A, int lda, const float* B, int ldb, int M, int N, int R, const float* bias, float* C, int ldc,
            double* stats, hipStream_t st);
// wide weight gradient on plain operands (gemm_big.hip): partial tiles per row split
bool wgrad_nt_ok(const float* X, int ldx, const float* Y, int ldy, int M, int N, int K);
size_t wgrad_nt_ws_bytes(int N, int K, int M);
int wgrad_nt(const float* X, int ldx, const float* Y, int ldy, int M, int N, int K, float* part, hipStream_t st);
const char* wgrad_nt_name(int N, int K, int M);
// pooled output of a stack from the GEMM's fused z-space extreme (pz/pa of gemm_rows_ex): out =
// act(s*z + t) with z = the max of the group where gamma >= 0, its min where gamma < 0 (the one
// extreme the producer kept per channel; s = gamma * invstd with invstd > 0, so the signs agree)
// and arg 0 where s == 0 -- act(s*z+t) is monotone in z, so this is max_k act(s*z_k + t) with its
// first argmax.  pz / pa: (G, N).  out2 (nullable, row stride ld2): a second copy of the pooled
// rows (the DGCNN EdgeConvs' outputs land in their column block of the head's concatenation too)
int pool_finalize(const float* pz, const unsigned char* pa, long long G, int N, const float* s, const float* t,
                  int act, float slope, float* out, unsigned char* arg, hipStream_t st, float* out2 = nullptr,
                  int ld2 = 0);
// engine launch probe: probe_enabled / probe_start / probe_stop (pcs_common.hpp, probe.cpp)
// weight gradient with deterministic partials: workspace bytes for (N, K, M), and the launch
size_t wgrad_ws_bytes(int N, int K, int M);
int wgrad_launch(const pcs_operand* x, int N, const pcs_operand* y, int K, int M, float* dW, float* db, void* ws,
                 size_t ws_bytes, void* stream);

// device-side operand of an ABI operand (the activation folded into one slope) over rows x cols
// (its extent, for the debug library's bounds checks)
Operand to_dev_operand(const pcs_operand* o, int rows, int cols);
// dW[e] += sum_s part[s][e] (e < nk), db[e] += sum_s pdb[s][e] (e < N; pdb/db nullable): fixed order
void wgrad_reduce_launch(const float* part, int splits, long long nk, float* dW, const float* pdb, int N, float* db,
                         hipStream_t st);
// out = dropout_p(act(Z*s + t)) (pcs_mlp_layer.drop_p / drop_seed of a stack's top layer)
int bn_act_dropout(const float* Z, int ldz, int M, int N, const float* s, const float* t, int act, float slope,
                   float* out, int ldo, double p, long long seed, hipStream_t st);
// fused data + weight gradient of one thin inner layer (fused_bwd.hip): C = its width, CI = its
// input width; q = the previous layer's pre-BN Z with its BN coefficients (s, t, mean, inv, act)
// policy = pcs_mlp_layer.bwd_fuse of the layer: PCS_BWD_FUSE_DEFAULT (only layers over >= 2^19
// rows), PCS_BWD_FUSE_OFF, PCS_BWD_FUSE_ALL (every eligible layer)
bool fused_bwd_wanted(int policy, int M);
bool fused_bwd_ok(int M, int C, int CI, int ldw, const pcs_operand* x, const pcs_operand* q);
int fused_bwd_grid(int M, int C, int CI, bool da, int xm);   // blocks = BN-backward partials (xm < 0: max)
size_t fused_bwd_ws_bytes(int M, int C, int CI);
int fused_bwd(const pcs_operand* x, int C, const pcs_operand* q, int CI, const float* W, int ldw, int M, float* dA,
              int ldd, double* bstats, float* dW, float* db, void* ws, size_t ws_bytes, hipStream_t st);
// the same kernel, weight gradient only, for a stack's first layer over raw rows X (M x kin,
// stride ldx; kin <= 32): dW (C x kin) and db += ...
bool fused_wgrad_ok(int M, int C, int kin, int ldx, const pcs_operand* x);
size_t fused_wgrad_ws_bytes(int M, int C, int kin);
int fused_wgrad(const pcs_operand* x, int C, const float* X, int ldx, int kin, int M, float* dW, float* db, void* ws,
                size_t ws_bytes, hipStream_t st);

// fused data + weight gradient of a 128-wide BNBWD inner layer over an LDS-DMA ring (bwd_ring.hip):
// C = 128, CI = its input width (a multiple of 128); q as fused_bwd's; gx = bwd_ring_grid row blocks
// (= BN-backward partials per column)
bool bwd_ring_ok(int M, int C, int CI, const float* W, int ldw, const pcs_operand* x, const pcs_operand* q);
int bwd_ring_grid(int M, int CI);
size_t bwd_ring_ws_bytes(int M, int C, int CI);
int bwd_ring(const pcs_operand* x, const pcs_operand* q, int CI, const float* W, int ldw, int M, float* dA, int ldd,
             double* bstats, float* dW, float* db, void* ws, size_t ws_bytes, hipStream_t st);

}  // namespace pcs
