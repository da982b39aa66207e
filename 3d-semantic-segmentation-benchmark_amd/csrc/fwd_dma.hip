// Forward GEMM of a shared-MLP layer, LDS-DMA staged (round 5):
//   Z[M x N] = T(A)[M x K] . W^T + bias,  W the layer's conv weight, row-major N x K (ldw),
//   T = identity (XF = false: a stack's first layer) or the previous layer's BN + activation
//   (XF: PCS_OP_BNACT, xform4<OP_BNACT>) applied once per element in a pass over the landed slab;
//   epilogue (gemm_rows_kernel's): bias, the Z store, fp64 BN partials of Z (sum, sum of squares)
//   per row block (STATS) and, for a pooled top layer, each group's extreme of Z and its first
//   row (POOL: pool_k 16 / 32; the max where the consumer's gamma >= 0, else the min).
// Reference: the forward of models/utils/common.py:125-178 (MiniPointNet / UnitPointNet: conv ->
// BN -> ReLU [-> max over K], common.py:211-212), models/dgcnn/dgcnn.py:188-207.
//
// Why (DESIGN.md 3.3, round-4 "next"): the register-staged row GEMM holds ONE slab of A and W in
// VGPRs while computing the previous one, at 2 blocks per CU; on the thin inner layers (K = 32 ..
// 256 over 16 K - 1 M rows) a tile is one to eight slabs, so each tile's load latency is barely
// covered and the forward ran at 1.3 - 2.5 TB/s.  Here A and W slabs go global -> LDS by LDS-DMA
// through an NS-stage ring that flattens (row tile, slab) iterations, so the loads of the next
// one or two TILES are in flight under the current tile's MFMAs and epilogue.  A block covers 64
// rows x BN columns (BN = 128 when N > 64: a row block's A is read once for up to 128 outputs).
// LDS images: A rows (32 floats) and W rows (32 k of one output channel) have their 16-B chunks
// XOR-swizzled by (row >> 1) & 7 on the source address, so both fragment reads are ds_read_b128
// of 16 consecutive rows, conflict free.  Every wave issues the same D DMA instructions per stage
// and the stage is retired by a counted s_waitcnt vmcnt + a raw s_barrier (dma_ring.hpp).
// Slab k order and the two-level fp32 accumulation are dgrad.hip's.
#include "dma_ring.hpp"
#include "mlp_common.hpp"

#include <cstdio>

namespace pcs {

constexpr int FW_BM = 64, FW_BK = 32;
constexpr int FW_A = FW_BM * FW_BK;                  // floats of one A slab: 8 KB
constexpr int FW_C = 256;                            // coefficients: s | t x 32, one 64-float slot per wave

struct FwdArgs {
    Operand a;                 // PLAIN or BNACT (s, t, act/slope): M x K, row stride ld
    int M, K;
    const float* W;            // N x K, row stride ldw
    int ldw;
    const float* bias;         // N or null
    float* C;                  // M x N, row stride ldc
    int ldc, N;
    double* stats;             // [2][N][gx] or null
    float* pz;                 // pooled extreme [M / pool_k][N] (POOL)
    unsigned char* pa;         // its row within the group
    int pool_k;
    const float* psign;        // per column: the consumer's gamma (the extreme's sign), nullable
    int gx, ntn;               // row blocks, column tiles
};

constexpr int fw_stage(int BN, bool XF) { return FW_A + FW_BK * BN + (XF ? FW_C : 0); }
constexpr int fw_blocks(int BN, int NS, bool XF) { return NS * fw_stage(BN, XF) * 4 + 4096 <= 80 * 1024 ? 2 : 1; }

template <int BN, int NS, bool XF, bool STATS, bool POOL>
__global__ __launch_bounds__(256, fw_blocks(BN, NS, XF)) void fwd_dma_kernel(const FwdArgs g) {
    constexpr int TN = BN / 64;
    constexpr int DB = FW_BK * BN;                      // the W slab: BN rows of 32 k
    constexpr int WO = FW_A, CO = FW_A + DB;            // W slab, coefficients
    constexpr int STAGE = fw_stage(BN, XF);
    constexpr int BI = BN / 32;                         // W-slab DMA instructions per wave (BN / 8 per block)
    constexpr int D = 2 + BI + (XF ? 1 : 0);            // DMA instructions per wave and stage
    constexpr int EC = 16 * TN;                         // full-tile C stores per lane
    __shared__ __attribute__((aligned(16))) float lds[NS * STAGE];
    __shared__ double red[2][2][STATS ? BN : 1];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int h = lane >> 5, l32 = lane & 31;

    // XCD-aware (row block, column tile): consecutive remapped ids share an XCD, and the column
    // tiles of one row block (the same A rows) are consecutive
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
    const int rb = t / g.ntn, ct = t - rb * g.ntn;
    const int n0 = ct * BN;

    const int nk = g.K / FW_BK;
    const int mtiles = (g.M + FW_BM - 1) / FW_BM;
    const int my_tiles = rb < mtiles ? (mtiles - 1 - rb) / g.gx + 1 : 0;
    const int total = my_tiles * nk;
    const unsigned lbase = dg_lds_addr(lds);
    // full-tile stores of the pooled extreme per lane: pz + pa per group, one or two groups per
    // 32-row block (every lane stores: the two lane halves hold the same merged extreme)
    const int EP = POOL ? TN * 2 * (g.pool_k == 16 ? 2 : 1) : 0;

    // ---- DMA of flattened iteration it (row tile it / nk, slab it % nk) into stage it % NS
    auto issue = [&](int it) {
        const int ti = it / nk, ks = it - ti * nk;
        const int m0 = (rb + ti * g.gx) * FW_BM, k0 = ks * FW_BK;
        const unsigned sb = lbase + 4u * (unsigned)((it % NS) * STAGE);
#pragma unroll
        for (int j = 0; j < 2; ++j) {                  // A: 8 rows x 8 chunks per instruction
            const int r = 8 * (2 * wave + j) + (lane >> 3);
            const int row = min(m0 + r, g.M - 1);
            const float* src = g.a.data + (size_t)row * g.a.ld + k0 + 4 * ((lane & 7) ^ dg_swz(r));
            PCS_DCHECK_QUAD(src, g.a.data, g.M, g.a.ld, g.K, "fwd A");
            dg_glds16(src, __builtin_amdgcn_readfirstlane(sb + 4u * (unsigned)((2 * wave + j) * 256)));
        }
#pragma unroll
        for (int j = 0; j < BI; ++j) {                 // W: rows n0 .. n0 + BN - 1 (clamped), k0 .. k0 + 31
            const int r = 8 * (wave * BI + j) + (lane >> 3);
            const int n = min(n0 + r, g.N - 1);
            const float* src = g.W + (size_t)n * g.ldw + k0 + 4 * ((lane & 7) ^ dg_swz(r));
            PCS_DCHECK_QUAD(src, g.W, g.N, g.ldw, g.K, "fwd W");
            dg_glds16(src, __builtin_amdgcn_readfirstlane(sb + 4u * (unsigned)(WO + (wave * BI + j) * 256)));
        }
        if (XF && lane < 16) {                         // s | t of k0 .. k0 + 31, one slot per wave
            const float* src = (lane < 8 ? g.a.s : g.a.t) + k0 + 4 * (lane & 7);
            dg_glds16(src, __builtin_amdgcn_readfirstlane(sb + 4u * (unsigned)(CO + wave * 64)));
        }
    };

    f32x16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = f32x16{};
    double s1[TN], s2[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) { s1[j] = 0.0; s2[j] = 0.0; }
    int col[TN];
    bool cok[TN];
    float bv[TN];
    unsigned pflip[TN];
    // per-column epilogue constants, before any DMA (a load issued later would make the compiler's
    // wait for it drain the ring)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        col[j] = n0 + wn * (BN / 2) + 32 * j + l32;
        cok[j] = col[j] < g.N;
        const int cc = cok[j] ? col[j] : g.N - 1;
        bv[j] = (g.bias && cok[j]) ? g.bias[cc] : 0.f;
        pflip[j] = (POOL && g.psign && g.psign[cc] < 0.f) ? 0x80000000u : 0u;
    }
    bool stores_full = false;                          // the last epilogue's stores were unconditional
    for (int s = 0; s < NS - 1; ++s)
        if (s < total) issue(s);

    for (int it = 0; it < total; ++it) {
        const int ti = it / nk, ks = it - ti * nk;
        const int m0 = (rb + ti * g.gx) * FW_BM;
        float* st = lds + (it % NS) * STAGE;
        // stage it landed (this wave's DMAs), then everyone's.  May stay in flight: the next
        // stage's D DMAs (NS = 3) and, at a tile's first slab, the previous full tile's stores
        // (issued after the DMA of stage it + NS - 2)
        {
            const bool nxt = min(total - 1, it + NS - 2) > it;
            const bool ex = ks == 0 && it > 0 && stores_full;
            if (ex && POOL && EP == TN * 4) {
                if (nxt) __builtin_amdgcn_s_waitcnt(dg_vmcnt(D + EC + TN * 4));
                else __builtin_amdgcn_s_waitcnt(dg_vmcnt(EC + TN * 4));
            } else if (ex && POOL) {
                if (nxt) __builtin_amdgcn_s_waitcnt(dg_vmcnt(D + EC + TN * 2));
                else __builtin_amdgcn_s_waitcnt(dg_vmcnt(EC + TN * 2));
            } else if (ex) {
                if (nxt) __builtin_amdgcn_s_waitcnt(dg_vmcnt(D + EC));
                else __builtin_amdgcn_s_waitcnt(dg_vmcnt(EC));
            } else if (nxt) {
                __builtin_amdgcn_s_waitcnt(dg_vmcnt(D));
            } else {
                __builtin_amdgcn_s_waitcnt(dg_vmcnt(0));
            }
            asm volatile("" ::: "memory");
        }
        dg_barrier();
        // ---- the previous layer's BN + activation, in place: thread = (k quad kq, rows r, r + 32)
        if constexpr (XF) {
            const int kq = tid & 7;
            Quad q;
            q.s = *reinterpret_cast<const float4*>(st + CO + 4 * kq);
            q.t = *reinterpret_cast<const float4*>(st + CO + 32 + 4 * kq);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int r = (tid >> 3) + 32 * i;
                float* p = st + r * FW_BK + 4 * (kq ^ dg_swz(r));
                const float4 v = *reinterpret_cast<const float4*>(p);
                *reinterpret_cast<float4*>(p) =
                    xform4<OP_BNACT>(g.a, v, v, 0u, m0 + r, q, ks * FW_BK + 4 * kq, g.K);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            dg_barrier();
        }
        const bool last = ks == nk - 1;
        // the next DMA (into the stage every wave finished reading one iteration ago); after the
        // epilogue's math on a tile's last slab
        if (!last && it + NS - 1 < total) issue(it + NS - 1);
        // ---- MFMAs: the slab into a fresh accumulator, then added (two-level)
        {
            const float* As = st;
            const float* Ws = st + WO;
            const int ar = wm * 32 + l32;
            f32x16 sacc[TN];
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const float4 a = *reinterpret_cast<const float4*>(As + ar * FW_BK + 4 * ((4 * h + qq) ^ dg_swz(ar)));
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int br = wn * (BN / 2) + 32 * j + l32;
                    const float4 b = *reinterpret_cast<const float4*>(Ws + br * FW_BK + 4 * ((4 * h + qq) ^ dg_swz(br)));
                    const f32x16 c0 = {};
                    sacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, qq == 0 ? c0 : sacc[j], 0, 0, 0);
                    sacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, sacc[j], 0, 0, 0);
                    sacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, sacc[j], 0, 0, 0);
                    sacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, sacc[j], 0, 0, 0);
                }
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[j] += sacc[j];
        }
        if (last) {
            // ---- tile epilogue: bias, BN partials and the pooled extreme first, then the next DMA,
            // then the stores -- unconditional on a full tile, so the next wait can count them
            const int rb0 = m0 + wm * 32;
            const bool full = m0 + FW_BM <= g.M && n0 + BN <= g.N;
            float v[TN][16];
            float pmx[TN][2];
            int imx[TN][2];
#pragma unroll
            for (int j = 0; j < TN; ++j) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    v[j][r] = acc[j][r] + bv[j];
                    acc[j][r] = 0.f;
                }
                if constexpr (STATS) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int row = rb0 + (r & 3) + 8 * (r >> 2) + 4 * h;
                        const double d = (full || (row < g.M && cok[j])) ? (double)v[j][r] : 0.0;
                        s1[j] += d;
                        s2[j] += d * d;
                    }
                }
                if constexpr (POOL) {
                    // per lane half: running extreme of its rows of each group (a group of 32 rows,
                    // or one group of 16 per half-block), first row on ties; then the two halves merge
#pragma unroll
                    for (int hb = 0; hb < 2; ++hb) {
                        pmx[j][hb] = -INFINITY;
                        imx[j][hb] = 16 * hb + 4 * h;
                    }
#pragma unroll
                    for (int r = 0; r < 16; ++r) {          // rows increasing in r: the first wins ties
                        const int hb = g.pool_k == 16 ? r >> 3 : 0;
                        const int rl = (r & 3) + 8 * (r >> 2) + 4 * h;
                        const float pv = __uint_as_float(__float_as_uint(v[j][r]) ^ pflip[j]);
                        if (pv > pmx[j][hb]) {
                            pmx[j][hb] = pv;
                            imx[j][hb] = rl;
                        }
                    }
#pragma unroll
                    for (int hb = 0; hb < 2; ++hb) {
                        const float ox = __shfl_xor(pmx[j][hb], 32);
                        const int oix = __shfl_xor(imx[j][hb], 32);
                        if (ox > pmx[j][hb] || (ox == pmx[j][hb] && oix < imx[j][hb])) {
                            pmx[j][hb] = ox;
                            imx[j][hb] = oix;
                        }
                    }
                }
            }
            if (it + NS - 1 < total) issue(it + NS - 1);
            stores_full = full;
            if (full) {
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    float* cb = g.C + (size_t)rb0 * g.ldc + col[j];
#pragma unroll
                    for (int r = 0; r < 16; ++r) cb[(size_t)((r & 3) + 8 * (r >> 2) + 4 * h) * g.ldc] = v[j][r];
                    if constexpr (POOL) {
#pragma unroll
                        for (int hb = 0; hb < 2; ++hb) {
                            if (hb == 1 && g.pool_k != 16) break;
                            const size_t o = (size_t)((rb0 + 16 * hb) / g.pool_k) * g.N + col[j];
                            g.pz[o] = __uint_as_float(__float_as_uint(pmx[j][hb]) ^ pflip[j]);
                            g.pa[o] = (unsigned char)(imx[j][hb] - 16 * hb);
                        }
                    }
                }
            } else {
#pragma unroll
                for (int j = 0; j < TN; ++j) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int row = rb0 + (r & 3) + 8 * (r >> 2) + 4 * h;
                        if (row < g.M && cok[j]) g.C[(size_t)row * g.ldc + col[j]] = v[j][r];
                    }
                    if constexpr (POOL) {
#pragma unroll
                        for (int hb = 0; hb < 2; ++hb) {
                            if (hb == 1 && g.pool_k != 16) break;
                            const int r0 = rb0 + 16 * hb;
                            if (h == 0 && cok[j] && r0 < g.M) {
                                const size_t o = (size_t)(r0 / g.pool_k) * g.N + col[j];
                                g.pz[o] = __uint_as_float(__float_as_uint(pmx[j][hb]) ^ pflip[j]);
                                g.pa[o] = (unsigned char)(imx[j][hb] - 16 * hb);
                            }
                        }
                    }
                }
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(dg_vmcnt(0));
    (void)EP;

    if constexpr (STATS) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int lc = wn * (BN / 2) + 32 * j + l32;
            const double a = s1[j] + __shfl_xor(s1[j], 32);
            const double b = s2[j] + __shfl_xor(s2[j], 32);
            if (lane < 32) {
                red[0][wm][lc] = a;
                red[1][wm][lc] = b;
            }
        }
        __syncthreads();
        for (int c = tid; c < BN; c += 256) {
            const int cl = n0 + c;
            if (cl < g.N) {
                g.stats[(size_t)cl * g.gx + rb] = red[0][0][c] + red[0][1][c];
                g.stats[((size_t)g.N + cl) * g.gx + rb] = red[1][0][c] + red[1][1][c];
            }
        }
    }
}

// The shapes the kernel takes: K a multiple of 32 (whole slabs), 16-B aligned rows of A and W,
// N % 4 == 0 (BN-partial layout), a pooled layer's groups aligned to the 32-row MFMA blocks
bool fwd_dma_ok(const pcs_operand* a, int M, int K, const float* W, int ldw, int N, int pool_k, const float* bias) {
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (!a || (a->mode != PCS_OP_PLAIN && a->mode != PCS_OP_BNACT)) return false;
    const bool base = M >= 1 && K >= FW_BK && K % FW_BK == 0 && N >= 4 && N % 4 == 0 && ldw % 4 == 0 && ldw >= K &&
                      al16(W) && a->ld % 4 == 0 && a->ld >= K && al16(a->data) && (pool_k == 0 || pool_k == 16 ||
                      pool_k == 32) && (pool_k == 0 || M % pool_k == 0);
    (void)bias;
    if (a->mode == PCS_OP_PLAIN) return base;
    return base && al16(a->s) && al16(a->t);
}

// column tile: 128 outputs when N > 64 (a row block's A read once for them), else 64
// (a 3-stage ring for the 128-column tiles measured 4.60 vs 4.58 ms, profiles/r05_ab_fwd_dma_stages.txt)
constexpr int kFwdNs128 = 2;
static void fwd_shape(int N, int* bn, int* ns) {
    *bn = N > 64 ? 128 : 64;
    *ns = *bn == 64 ? 3 : kFwdNs128;
}

const char* fwd_dma_name(bool xf, bool stats, bool pool, int N) {
    int bn, ns;
    fwd_shape(N, &bn, &ns);
    static char names[2][2][2][2][64];
    char* nm = names[bn == 128][xf][stats][pool];
    snprintf(nm, 64, "pcs::fwd_dma_kernel<%d, %d, %s, %s, %s>", bn, ns, xf ? "true" : "false", stats ? "true" : "false",
             pool ? "true" : "false");
    return nm;
}

template <int BN, int NS, bool XF>
static void launch_fwd(const FwdArgs& g, hipStream_t st) {
    const unsigned blocks = (unsigned)((long long)g.gx * g.ntn);
    const bool S = g.stats != nullptr, P = g.pool_k != 0;
    if (S && P) hipLaunchKernelGGL((fwd_dma_kernel<BN, NS, XF, true, true>), dim3(blocks), dim3(256), 0, st, g);
    else if (S) hipLaunchKernelGGL((fwd_dma_kernel<BN, NS, XF, true, false>), dim3(blocks), dim3(256), 0, st, g);
    else if (P) hipLaunchKernelGGL((fwd_dma_kernel<BN, NS, XF, false, true>), dim3(blocks), dim3(256), 0, st, g);
    else hipLaunchKernelGGL((fwd_dma_kernel<BN, NS, XF, false, false>), dim3(blocks), dim3(256), 0, st, g);
}

int fwd_dma(const pcs_operand* a, int M, int K, const float* W, int ldw, const float* bias, float* C, int ldc, int N,
            double* stats, int gx, float* pz, unsigned char* pa, int pool_k, const float* psign, hipStream_t st) {
    FwdArgs g{};
    g.a = to_dev_operand(a, M, K);
    g.M = M;
    g.K = K;
    g.W = W;
    g.ldw = ldw;
    g.bias = bias;
    g.C = C;
    g.ldc = ldc;
    g.N = N;
    g.stats = stats;
    g.pz = pz;
    g.pa = pa;
    g.pool_k = pool_k;
    g.psign = psign;
    g.gx = gx;
    int bn, ns;
    fwd_shape(N, &bn, &ns);
    g.ntn = (N + bn - 1) / bn;
    const long long blocks = (long long)gx * g.ntn;
    PCS_CHECK_ARG(gx >= 1 && blocks < (1ll << 31), "fwd_dma: bad grid");
    const bool xf = a->mode == PCS_OP_BNACT;
    if (bn == 64) {
        if (xf) launch_fwd<64, 3, true>(g, st);
        else launch_fwd<64, 3, false>(g, st);
    } else {
        if (xf) launch_fwd<128, kFwdNs128, true>(g, st);
        else launch_fwd<128, kFwdNs128, false>(g, st);
    }
    return 0;
}

}  // namespace pcs
