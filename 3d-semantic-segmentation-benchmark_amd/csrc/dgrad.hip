// Data-gradient GEMM of a shared-MLP layer, LDS-DMA staged:
//   dA[M x N] = dZ[M x K] . W[K x N],  W the layer's weights read k-major (N = its input width),
//   dZ either rebuilt from the layer's (dy, z) by its BN+activation backward (XM = 1: A operand
//   PCS_OP_BNBWD, xform4<OP_BNBWD>), rebuilt from a pooled top layer's gradient (XM = 2:
//   PCS_OP_POOLBWD -- dy non-zero only at each group's argmax row, xform4<OP_POOLBWD>) or read
//   as it lies (XM = 0: a materialised dZ, PCS_OP_PLAIN);
//   optional epilogue: the previous layer's BN-backward partial sums (sum dy', sum dy'*xhat')
//   over this block's rows -- exactly gemm_rows_kernel<64, 64, 2, 2, BNBWD | PLAIN, true, EPI> of
//   mlp.hip (same k order inside a slab, same two-level fp32 accumulation, same epilogue), so the
//   outputs are bitwise those of that kernel (tests/test_gpu_dgrad_dma.py).
// Reference: the backward of models/utils/common.py:125-178 (MiniPointNet / UnitPointNet:
// conv -> BN -> ReLU) as autograd runs it.
//
// Why a second kernel (VERDICT r3 #1b): the register-staged row GEMM holds one slab of (dy, z, W)
// in VGPRs while computing the previous one and needs 240 VGPRs with its epilogue -- 2 waves per
// SIMD, one slab in flight per block, and over 64-column tiles it reads every row block's
// operand once per column tile.  Here the raw slabs go global -> LDS by LDS-DMA
// (global_load_lds_dwordx4, no VGPR destination) through an NS-stage ring; the BN-backward
// transform (XM > 0) is applied once per element in a pass over the landed slab (LDS -> VGPR ->
// LDS, in place), then the MFMAs read the slab.  POOLBWD (round 5) lands only the z slab, the
// <= 4 pooled-gradient rows and argmax bytes of the groups the 64-row tile spans (wave w: group
// w) and the coefficients; its transform expands the argmax-routed gradient in place over z.  A block covers 64 rows x BN columns (BN = 128 when
// N > 64: the row block's operand is read once).  Every wave issues the same D DMA instructions
// per stage, so a stage is retired by a counted `s_waitcnt vmcnt` + a raw s_barrier -- never
// __syncthreads(), whose fence would drain the ring (cdna_hip_programming.md, glds rules).
// LDS images are lane-linear (an LDS-DMA writes base + 16 * lane); the dy / z rows (32 floats)
// have their 16-B chunks XOR-swizzled by (row >> 1) & 7 on the SOURCE address and on every read,
// so the fragment reads (ds_read_b128 of 16 rows) are bank-conflict free.  The W slab is stored
// [k][n] as it lies in memory; a lane's B fragment is 4 ds_read_b32 down a column.
// Grid: (row blocks) x (column tiles), persistent over row tiles like the row GEMM, XCD-remapped.
#include "dma_ring.hpp"
#include "mlp_common.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace pcs {

constexpr int DG_BM = 64, DG_BK = 32;
constexpr int DG_A = DG_BM * DG_BK;                  // floats of one dy (or z) slab: 8 KB
constexpr int DG_C = 256;                            // coefficients: s, t, mean, alpha, kb x 32 (+ pad)
constexpr int DG_P = 4 * 32 + 4 * 8;                 // POOLBWD: 4 pooled-gradient rows + their argmax bytes

struct DgradArgs {
    Operand a;                 // BNBWD: data = dy (ld), z (ldz), s, t, mean, alpha, kb, act/slope
    int M, K;
    const float* W;            // k-major: B[k][n] = W[k * ldw + n]
    int ldw;
    float* C;                  // M x N, row stride ldc
    int ldc, N;
    Operand e;                 // epilogue: the previous layer's z (ldz), s, t, mean, inv, act/slope
    double* bstats;            // [2][N][gx] or null
    int gx, ntn;               // row blocks, column tiles
};

// LDS floats of one ring stage: A slab (+ z slab + coefficients when XM = 1; coefficients + pooled
// rows when XM = 2, whose A is rebuilt in place over its z slab) + the W slab
constexpr int dg_stage(int BN, int XM) {
    return (XM == 1 ? 2 * DG_A + DG_C : XM == 2 ? DG_A + DG_C + DG_P : DG_A) + DG_BK * BN;
}
// blocks per CU the ring allows (160 KB of LDS)
constexpr int dg_blocks(int BN, int NS, int XM) { return NS * dg_stage(BN, XM) * 4 + 4096 <= 80 * 1024 ? 2 : 1; }

// BN = 64 or 128 output columns per block (4 waves as 2 x 2: a wave owns 32 rows x BN/2
// columns, TN = BN / 64 MFMA blocks), NS ring stages; XM: A as it lies (0), rebuilt by the BN
// backward from (dy, z) (1) or from (pooled dy, argmax, z) (2)
template <bool BWD, int BN, int NS, int XM>
__global__ __launch_bounds__(256, dg_blocks(BN, NS, XM)) void dgrad_kernel(const DgradArgs g) {
    constexpr bool XF = XM > 0;
    constexpr int TN = BN / 64;
    constexpr int DB = DG_BK * BN;                      // the W slab
    constexpr int AW = XM == 1 ? 2 * DG_A : DG_A;       // the A (+ z) slabs
    constexpr int ZO = XM == 1 ? DG_A : 0;              // the z slab (XM = 2: in place of A)
    constexpr int CO = AW + DB;                         // the coefficients
    constexpr int PO = CO + DG_C;                       // XM = 2: pooled rows [4][32], argmax [4][32 B]
    constexpr int STAGE = dg_stage(BN, XM);             // floats per stage
    constexpr int BI = BN / 32;                         // W-slab DMA instructions per wave (BN/16 per block)
    constexpr int D = (XF ? 5 : 2) + BI;                // DMA instructions per wave and stage
                                                        // (XM = 2: z x 2, coefficients, pooled row, argmax)
    constexpr int E = 16 * TN;                          // prefetched Z loads / full-tile stores per lane
    __shared__ __attribute__((aligned(16))) float lds[NS * STAGE];
    __shared__ double red[2][2][BN];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int h = lane >> 5, l32 = lane & 31;

    // XCD-aware (row block, column tile): consecutive remapped ids share an XCD, and the column
    // tiles of one row block are consecutive
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
    const int rb = t / g.ntn, ct = t - rb * g.ntn;
    const int n0 = ct * BN;

    const int nk = g.K / DG_BK;
    const int mtiles = (g.M + DG_BM - 1) / DG_BM;
    const int my_tiles = rb < mtiles ? (mtiles - 1 - rb) / g.gx + 1 : 0;
    const int total = my_tiles * nk;
    const unsigned lbase = dg_lds_addr(lds);
    const int nlast = ((g.N + 3) & ~3) - 4;                // last in-range column quad
    // POOLBWD: the group of row r is r >> psh (pool_k a power of two) or r / pool_k; a 64-row tile
    // spans <= 4 groups (pool_k 16 / 32, or a multiple of 64: one)
    const int pk = XM == 2 ? g.a.pool_k : 1;
    const int G = XM == 2 ? g.M / pk : 1;
    // ---- DMA of flattened iteration it (row tile it / nk, slab it % nk) into stage it % NS
    auto issue = [&](int it) {
        const int ti = it / nk, ks = it - ti * nk;
        const int m0 = (rb + ti * g.gx) * DG_BM, k0 = ks * DG_BK;
        const unsigned sb = lbase + 4u * (unsigned)((it % NS) * STAGE);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int r = 8 * (2 * wave + j) + (lane >> 3);
            const int row = min(m0 + r, g.M - 1);
            const int ch = 4 * ((lane & 7) ^ dg_swz(r));
            const unsigned d = __builtin_amdgcn_readfirstlane(sb + 4u * (unsigned)((2 * wave + j) * 256));
            if (XM != 2) {
                PCS_DCHECK_QUAD(g.a.data + (size_t)row * g.a.ld + k0 + ch, g.a.data, g.M, g.a.ld, g.K, "dgrad dZ/dy");
                dg_glds16(g.a.data + (size_t)row * g.a.ld + k0 + ch, d);
            }
            if (XF) {
                PCS_DCHECK_QUAD(g.a.z + (size_t)row * g.a.ldz + k0 + ch, g.a.z, g.M, g.a.ldz, g.K, "dgrad z");
                dg_glds16(g.a.z + (size_t)row * g.a.ldz + k0 + ch, d + 4u * ZO);
            }
        }
        // POOLBWD: wave w lands group (first group of the tile) + w, clamped to the last group:
        // its 32 pooled-gradient floats (lanes 0-7) and its 32 argmax bytes (lanes 0-1)
        if (XM == 2) {
            const int gw = min(pool_group(g.a, m0) + wave, G - 1);
            const unsigned dp = __builtin_amdgcn_readfirstlane(sb + 4u * (unsigned)(PO + 32 * wave));
            const unsigned da = __builtin_amdgcn_readfirstlane(sb + 4u * (unsigned)(PO + 128 + 8 * wave));
            if (lane < 8) {
                PCS_DCHECK_QUAD(g.a.data + (size_t)gw * g.a.ld + k0 + 4 * lane, g.a.data, G, g.a.ld, g.K, "dgrad dpool");
                dg_glds16(g.a.data + (size_t)gw * g.a.ld + k0 + 4 * lane, dp);
            }
            if (lane < 2) {
                PCS_DCHECK(gw < G && k0 + 16 * lane + 16 <= g.K, "dgrad argmax group %d of %d col %d", gw, G,
                           k0 + 16 * lane);
                dg_glds16(reinterpret_cast<const float*>(g.a.arg + (size_t)gw * g.a.ld + k0 + 16 * lane), da);
            }
        }
        // W slab rows k0 .. k0+31, columns n0 .. n0+BN-1: 64 lanes x 16 B = 256 / BN * 4 rows per
        // instruction, BI instructions per wave
#pragma unroll
        for (int j = 0; j < BI; ++j) {
            const int e = (wave * BI + j) * 64 + lane;        // 16-B chunk of the slab
            const int kr = e / (BN / 4), cq = e - kr * (BN / 4);
            const int col = min(n0 + 4 * cq, nlast);
            const unsigned d = __builtin_amdgcn_readfirstlane(sb + 4u * (unsigned)(AW + (wave * BI + j) * 256));
            PCS_DCHECK_QUAD(g.W + (size_t)(k0 + kr) * g.ldw + col, g.W, g.K, g.ldw, g.N, "dgrad W");
            dg_glds16(g.W + (size_t)(k0 + kr) * g.ldw + col, d);
        }
        // coefficients: wave 0 s | t, wave 1 mean | alpha, wave 2 kb | kb, wave 3 kb | kb (pad)
        if (XF && lane < 16) {
            const float* src = wave == 0 ? (lane < 8 ? g.a.s : g.a.t)
                             : wave == 1 ? (lane < 8 ? g.a.mean : g.a.alpha) : g.a.kb;
            const unsigned d = __builtin_amdgcn_readfirstlane(sb + 4u * (unsigned)(CO + wave * 64));
            dg_glds16(src + k0 + 4 * (lane & 7), d);
        }
    };

    f32x16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = f32x16{};
    double s1[TN], s2[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) { s1[j] = 0.0; s2[j] = 0.0; }
    // the epilogue's Z values of this lane (previous layer's pre-BN output), loaded PF slabs
    // before the tile's last one so their HBM latency hides under those slabs' work
    const int PF = nk >= 3 ? 2 : nk - 1;
    int col[TN], colc[TN];
    bool cok[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        col[j] = n0 + wn * (BN / 2) + 32 * j + l32;
        cok[j] = col[j] < g.N;
        colc[j] = cok[j] ? col[j] : g.N - 1;
    }
    float zt[TN][16];
    bool stores_full = false;                  // the last epilogue's stores were unconditional
    // the epilogue's per-column coefficients, before any DMA (a load issued later would make the
    // compiler's wait for it drain the ring)
    float sp[TN], tp[TN], mp[TN], ip[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        sp[j] = tp[j] = mp[j] = ip[j] = 0.f;
        if (BWD) { sp[j] = g.e.s[colc[j]]; tp[j] = g.e.t[colc[j]]; mp[j] = g.e.mean[colc[j]]; ip[j] = g.e.inv[colc[j]]; }
    }
    for (int s = 0; s < NS - 1; ++s)
        if (s < total) issue(s);

    for (int it = 0; it < total; ++it) {
        const int ti = it / nk, ks = it - ti * nk;
        const int m0 = (rb + ti * g.gx) * DG_BM;
        float* st = lds + (it % NS) * STAGE;
        // stage it landed (this wave's DMAs), then everyone's.  Issued after this wave's stage-it
        // DMAs and allowed to stay in flight: the next stage's D DMAs (NS = 3), the Z prefetch's
        // loads between its issue and the epilogue, a full tile's stores right before the last DMA
        {
            const bool nxt = min(total - 1, it + NS - 2) > it;
            // (the Z loads count when issued after stage it's DMAs: at most NS - 1 slabs ago)
            const bool ex = (BWD && ks > nk - 1 - PF && ks <= nk - 2 - PF + NS) || (ks == 0 && it > 0 && stores_full);
            if (nxt && ex) __builtin_amdgcn_s_waitcnt(dg_vmcnt(D + E));
            else if (ex) __builtin_amdgcn_s_waitcnt(dg_vmcnt(E));
            else if (nxt) __builtin_amdgcn_s_waitcnt(dg_vmcnt(D));
            else __builtin_amdgcn_s_waitcnt(dg_vmcnt(0));
            asm volatile("" ::: "memory");
        }
        dg_barrier();
        // ---- BN-backward transform of the dy slab, in place: thread = (k quad kq, rows r, r + 32)
        if constexpr (XF) {
            const int kq = tid & 7;
            const float* cf = st + CO;
            Quad q;
            q.s = *reinterpret_cast<const float4*>(cf + 4 * kq);
            q.t = *reinterpret_cast<const float4*>(cf + 32 + 4 * kq);
            q.mean = *reinterpret_cast<const float4*>(cf + 64 + 4 * kq);
            q.alpha = *reinterpret_cast<const float4*>(cf + 96 + 4 * kq);
            q.kb = *reinterpret_cast<const float4*>(cf + 128 + 4 * kq);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int r = (tid >> 3) + 32 * i;
                float* p = st + r * DG_BK + 4 * (kq ^ dg_swz(r));
                const float4 z = *reinterpret_cast<const float4*>(p + ZO);
                if constexpr (XM == 2) {
                    // the group's landed slot: rows past the last group read its (clamped) copy
                    const int gl = min(pool_group(g.a, m0 + r) - pool_group(g.a, m0), 3);
                    const float4 v = *reinterpret_cast<const float4*>(st + PO + 32 * gl + 4 * kq);
                    const unsigned a = *reinterpret_cast<const unsigned*>(st + PO + 128 + 8 * gl + kq);
                    *reinterpret_cast<float4*>(p) =
                        xform4<OP_POOLBWD>(g.a, v, z, a, m0 + r, q, ks * DG_BK + 4 * kq, g.K);
                } else {
                    const float4 v = *reinterpret_cast<const float4*>(p);
                    *reinterpret_cast<float4*>(p) =
                        xform4<OP_BNBWD>(g.a, v, z, 0u, m0 + r, q, ks * DG_BK + 4 * kq, g.K);
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            dg_barrier();
        }
        const bool last = ks == nk - 1;
        // the next DMA (into the stage every wave finished reading one iteration ago); after the
        // epilogue's sums instead on a tile's last slab
        if (!last && it + NS - 1 < total) issue(it + NS - 1);
        if (BWD && ks == nk - 1 - PF) {
            const int rb0 = m0 + wm * 32;
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = min(rb0 + (r & 3) + 8 * (r >> 2) + 4 * h, g.M - 1);
                    zt[j][r] = g.e.z[(size_t)row * g.e.ldz + colc[j]];
                }
        }
        // ---- MFMAs: slab into a fresh accumulator, then added (two-level, as the row GEMM)
        {
            const float* As = st;
            const float* Bs = st + AW;
            const int ar = wm * 32 + l32;
            f32x16 sacc[TN];
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const float4 a = *reinterpret_cast<const float4*>(As + ar * DG_BK + 4 * ((4 * h + qq) ^ dg_swz(ar)));
                const int kb = 16 * h + 4 * qq;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int bc = wn * (BN / 2) + 32 * j + l32;
                    const float b0 = Bs[(kb + 0) * BN + bc], b1 = Bs[(kb + 1) * BN + bc];
                    const float b2 = Bs[(kb + 2) * BN + bc], b3 = Bs[(kb + 3) * BN + bc];
                    const f32x16 c0 = {};
                    sacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b0, qq == 0 ? c0 : sacc[j], 0, 0, 0);
                    sacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b1, sacc[j], 0, 0, 0);
                    sacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b2, sacc[j], 0, 0, 0);
                    sacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b3, sacc[j], 0, 0, 0);
                }
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[j] += sacc[j];
        }
        if (last) {
            // ---- tile epilogue (gemm_rows_kernel's): the BN-backward sums first (they wait for the
            // prefetched Z), then the next DMA, then the stores -- unconditional on a full tile, so
            // the next wait can count them
            const int rb0 = m0 + wm * 32;
            const bool full = m0 + DG_BM <= g.M && n0 + BN <= g.N;
            float v[TN][16];
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    v[j][r] = acc[j][r] + 0.f;           // (the row GEMM's "+ bias" with bias 0: -0 -> +0)
                    acc[j][r] = 0.f;
                }
            if (BWD) {
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int row = rb0 + (r & 3) + 8 * (r >> 2) + 4 * h;
                        const bool ok = full || (row < g.M && cok[j]);
                        const float z = zt[j][r];
                        const float dy = v[j][r] * dact_f(z * sp[j] + tp[j], g.e.act, g.e.slope);
                        const float xh = (z - mp[j]) * ip[j];
                        const double dd = ok ? (double)dy : 0.0;
                        s1[j] += dd;
                        s2[j] += dd * (double)xh;
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
                }
            } else {
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int row = rb0 + (r & 3) + 8 * (r >> 2) + 4 * h;
                        if (row < g.M && cok[j]) g.C[(size_t)row * g.ldc + col[j]] = v[j][r];
                    }
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(dg_vmcnt(0));

    if (BWD) {
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
                g.bstats[(size_t)cl * g.gx + rb] = red[0][0][c] + red[0][1][c];
                g.bstats[((size_t)g.N + cl) * g.gx + rb] = red[1][0][c] + red[1][1][c];
            }
        }
    }
}

bool dgrad_dma_ok(const pcs_operand* a, int M, int K, const float* W, int ldw, int N) {
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (!a || (a->mode != PCS_OP_BNBWD && a->mode != PCS_OP_PLAIN && a->mode != PCS_OP_POOLBWD)) return false;
    const bool base = M >= 1 && K >= DG_BK && K % DG_BK == 0 && N >= 4 && N % 4 == 0 && ldw % 4 == 0 && ldw >= N &&
                      al16(W) && a->ld % 4 == 0 && al16(a->data);
    if (a->mode == PCS_OP_PLAIN) return base;
    const bool bn = base && a->ldz % 4 == 0 && al16(a->z) && al16(a->s) && al16(a->t) && al16(a->mean) &&
                    al16(a->alpha) && al16(a->kb);
    if (a->mode == PCS_OP_BNBWD) return bn;
    // POOLBWD: a 64-row tile spans <= 4 groups (pool_k 16 or 32) or lies in one (a multiple of 64);
    // the argmax rows (stride ld bytes) land 16 B at a time
    const int pk = a->pool_k;
    return bn && a->arg && (pk == 16 || pk == 32 || (pk % 64 == 0 && pk <= 256)) && M % pk == 0 && a->ld % 16 == 0 &&
           al16(a->arg);
}

// Variant (column tile x ring stages): 128 x 2 when N > 64 (one column tile reads the row block's
// operand once; two stages fit two blocks per CU), else 64 x 3.  Measured: the PointNet++
// 131072 x 128 x 128 dgrad 95.5 -> 80.2 us isolated, step 5.05 -> 5.01 ms; 128 x 3 (one block per
// CU) 105.8 us (profiles/r04_ab_dgrad_variants.txt).  pcs_gemm_rows_kmajor_variant forces one
// variant for a single call (A/B and the bitwise tests; no process-wide switch).  The switch is
// per HOST THREAD: pcs_set_kernel_variant covers the launches the calling thread makes (forward
// passes), not those of PyTorch's autograd device thread (the backward of loss.backward()).
static thread_local int t_variant = 0;            // 0: policy; 1: 64 x 3; 2: 128 x 2; 3: 128 x 3

void dgrad_force_variant(int v) { t_variant = v; }
int dgrad_forced_variant() { return t_variant; }

static void dgrad_shape(int N, int* bn, int* ns) {
    switch (t_variant) {
        case 1: *bn = 64; *ns = 3; return;
        case 2: *bn = N > 64 ? 128 : 64; *ns = *bn == 64 ? 3 : 2; return;
        case 3: *bn = N > 64 ? 128 : 64; *ns = 3; return;
        default: *bn = N > 64 ? 128 : 64; *ns = *bn == 64 ? 3 : 2; return;
    }
}

const char* dgrad_dma_name(bool bwd, int mode, int N) {
    int bn, ns;
    dgrad_shape(N, &bn, &ns);
    const int xm = mode == PCS_OP_BNBWD ? 1 : mode == PCS_OP_POOLBWD ? 2 : 0;
    static char names[2][3][3][48];
    static bool init = false;
    if (!init) {
        const int shapes[3][2] = {{64, 3}, {128, 2}, {128, 3}};
        for (int b = 0; b < 2; ++b)
            for (int x = 0; x < 3; ++x)
                for (int v = 0; v < 3; ++v)
                    snprintf(names[b][x][v], sizeof names[b][x][v], "pcs::dgrad_kernel<%s, %d, %d, %d>",
                             b ? "true" : "false", shapes[v][0], shapes[v][1], x);
        init = true;
    }
    return names[bwd][xm][bn == 64 ? 0 : (ns == 2 ? 1 : 2)];
}

template <int BN, int NS, int XM>
static void launch_dgrad(const DgradArgs& g, bool bwd, hipStream_t st) {
    const unsigned blocks = (unsigned)((long long)g.gx * g.ntn);
    if (bwd) hipLaunchKernelGGL((dgrad_kernel<true, BN, NS, XM>), dim3(blocks), dim3(256), 0, st, g);
    else hipLaunchKernelGGL((dgrad_kernel<false, BN, NS, XM>), dim3(blocks), dim3(256), 0, st, g);
}

template <int XM>
static void launch_dgrad_xm(const DgradArgs& g, int bn, int ns, bool bwd, hipStream_t st) {
    if (bn == 64) launch_dgrad<64, 3, XM>(g, bwd, st);
    else if (ns == 2) launch_dgrad<128, 2, XM>(g, bwd, st);
    else launch_dgrad<128, 3, XM>(g, bwd, st);
}

int dgrad_dma(const pcs_operand* a, int M, int K, const float* W, int ldw, float* C, int ldc, int N,
              const pcs_operand* epi, double* bstats, int gx, hipStream_t st) {
    DgradArgs g{};
    g.a = to_dev_operand(a, M, K);
    g.M = M;
    g.K = K;
    g.W = W;
    g.ldw = ldw;
    g.C = C;
    g.ldc = ldc;
    g.N = N;
    if (epi) g.e = to_dev_operand(epi, M, N);
    g.bstats = bstats;
    g.gx = gx;
    int bn, ns;
    dgrad_shape(N, &bn, &ns);
    g.ntn = (N + bn - 1) / bn;
    const long long blocks = (long long)gx * g.ntn;
    PCS_CHECK_ARG(gx >= 1 && blocks < (1ll << 31), "dgrad_dma: bad grid");
    const bool bw = bstats != nullptr;
    if (a->mode == PCS_OP_BNBWD) launch_dgrad_xm<1>(g, bn, ns, bw, st);
    else if (a->mode == PCS_OP_POOLBWD) launch_dgrad_xm<2>(g, bn, ns, bw, st);
    else launch_dgrad_xm<0>(g, bn, ns, bw, st);
    return 0;
}

}  // namespace pcs
