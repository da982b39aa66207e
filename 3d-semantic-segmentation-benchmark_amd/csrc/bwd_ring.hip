// Fused data + weight gradient of a 128-wide BN layer over an LDS-DMA ring.
//
// Reference semantics: the autograd backward of conv1x1 -> BatchNorm(train) -> act for an inner
// layer l of a MiniPointNet / UnitPointNet stack (models/utils/common.py:125-178; PointNet++ FP1's
// 128 -> 128 layers, FP2's 256 -> 128 layer, PointNeXt's 128-wide decoder layers):
//   dZ_l      = BN-backward of (dy_l, Z_l)                     (M x 128, rebuilt on load)
//   dA_{l-1}  = dZ_l . W_l                                     (M x CI; then layer l-1's BN-backward sums)
//   dW_l     += dZ_l^T . act(BN(Z_{l-1})),   db_l += column sums of dZ_l
// The separate path runs the data gradient (dgrad.hip, caller's stream) and the weight gradient
// (mlp.hip wgrad, side lane) as two GEMMs that both stream dy_l, Z_l and Z_{l-1} from HBM and
// share the CUs; round 5 measured the pair at 0.31 of the fp32 MFMA peak together.  Here ONE
// workgroup per CU reads each operand once:
//   * W_l's 128 x 128 column tile (64 KB) and the 5 x 128 BN-backward coefficients are resident
//     in LDS for the whole launch;
//   * dy_l / Z_l arrive in 64-row x 32-column slabs through a 3-stage global_load_lds_dwordx4 ring
//     (no VGPR destination; counted `s_waitcnt vmcnt` + raw s_barrier retire a stage), and are
//     turned into dZ in place by one pass (one float4 per thread);
//   * Z_{l-1}'s 64 x 128 tile arrives by the same DMA once per row tile, a full tile ahead.
// Eight waves, two per SIMD: waves 0-3 own the data gradient (2 x 2: 32 rows x 64 columns each,
// the layer l-1 BN-backward epilogue of dgrad_kernel), waves 4-7 own the weight gradient (wave
// 4 + v: dW columns n0 + 32v .. +31, all 128 rows, one accumulator per slab) -- each SIMD
// interleaves one data-gradient and one weight-gradient wave, 32 + 32 MFMAs per slab.
// Every MFMA is v_mfma_f32_32x32x2_f32 (fp32 in and accumulate); the weight gradient is one
// partial tile per workgroup, summed in workgroup order by wgrad_reduce_kernel (deterministic:
// no float atomics).  Rows past M are zeroed in dZ, so they add nothing to dW / db.
#include "dma_ring.hpp"
#include "mlp_common.hpp"

#include <cstdio>

namespace pcs {

constexpr int BR_C = 128;                      // the layer's width: dZ columns, the data gradient's K
constexpr int BR_BM = 64, BR_BK = 32;          // rows per tile, dZ columns per slab
constexpr int BR_NK = BR_C / BR_BK;            // slabs per tile
constexpr int BR_NS = 3;                       // ring stages
constexpr int BR_SLAB = BR_BM * BR_BK;         // floats of one dy (or z) slab: 8 KB
constexpr int BR_STAGE = 2 * BR_SLAB;          // dy + z
constexpr int BR_X = BR_BM * 128;              // the input tile (64 rows x the 128-column tile): 32 KB
constexpr int BR_W = BR_C * 128;               // W's column tile: 64 KB
constexpr int BR_THREADS = 512;

struct BwdRingArgs {
    Operand a;            // layer l's dZ operand, BNBWD: dy (data, ld), z (ldz), s, t, mean, alpha, kb
    Operand q;            // layer l-1: data = its pre-BN Z (M x CI, stride ld), s, t, mean, inv, slope
    const float* W;       // layer l's weight, row-major 128 x CI (W[c * ldw + i])
    int ldw;
    int M, CI;
    float* dA;            // M x CI, row stride ldd
    int ldd;
    double* bstats;       // [2][CI][gx]: layer l-1's (sum dy, sum dy*xhat) per row block
    float* part;          // [gx][128][CI]: dW partial of row block rb (its column tiles side by side)
    float* pdb;           // [gx][128]: db partial (column tile 0's workgroups) or null
    int gx, ntn;          // row blocks, 128-column tiles
};

// 16-B chunk swizzle of a 128-float input-tile row: rows 2p / 2p + 1 (the weight-gradient B
// fragments) and R / R + 4 (the epilogue's Z reads) land in opposite bank halves
__device__ __forceinline__ int br_xswz(int r) { return ((r ^ (r >> 2)) & 1) << 3; }
__device__ __forceinline__ int br_acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// s_waitcnt vmcnt(n) for the few counts the ring uses (the immediate must be a constant)
__device__ __forceinline__ void br_vm_wait(int n) {
    switch (n) {
    case 2: __builtin_amdgcn_s_waitcnt(dg_vmcnt(2)); break;
    case 4: __builtin_amdgcn_s_waitcnt(dg_vmcnt(4)); break;
    case 6: __builtin_amdgcn_s_waitcnt(dg_vmcnt(6)); break;
    case 32: __builtin_amdgcn_s_waitcnt(dg_vmcnt(32)); break;
    case 34: __builtin_amdgcn_s_waitcnt(dg_vmcnt(34)); break;
    case 36: __builtin_amdgcn_s_waitcnt(dg_vmcnt(36)); break;
    case 38: __builtin_amdgcn_s_waitcnt(dg_vmcnt(38)); break;
    default: __builtin_amdgcn_s_waitcnt(dg_vmcnt(0)); break;
    }
    asm volatile("" ::: "memory");
}

// CI: the input width (128 or 256), also the row stride of dA and of the previous layer's Z
template <int CI>
__global__ __launch_bounds__(BR_THREADS, 1) void bwd_ring_kernel(const BwdRingArgs g) {
    __shared__ __attribute__((aligned(16))) float Wl[BR_W];
    __shared__ __attribute__((aligned(16))) float ring[BR_NS * BR_STAGE];
    __shared__ __attribute__((aligned(16))) float Xl[BR_X];
    __shared__ __attribute__((aligned(16))) float cf[5 * BR_C];     // s | t | mean | alpha | kb
    __shared__ float qc[4][128];                   // layer l-1's s | t | mean | inv over the column tile
    __shared__ double red[2][2][128];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool awave = wave < 4;                   // data gradient (else weight gradient)
    const int wm = (wave >> 1) & 1, wn = wave & 1;
    const int v = wave & 3;
    const int h = lane >> 5, l32 = lane & 31;

    // XCD-aware (row block, column tile) as dgrad_kernel
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
    const int rb = t / g.ntn, ct = t - rb * g.ntn;
    const int n0 = ct * 128;
    const int M = g.M;
    const int tiles = (M + BR_BM - 1) / BR_BM;
    const int my_tiles = rb < tiles ? (tiles - 1 - rb) / g.gx + 1 : 0;
    const int total = my_tiles * BR_NK;

    // ---- resident operands and per-lane coefficients, all loaded before the first DMA (a plain
    // load issued later would make the compiler's wait for it drain the ring)
    for (int e = tid; e < BR_C * 32; e += BR_THREADS) {
        const int k = e >> 5, n = 4 * (e & 31);
        PCS_DCHECK_QUAD(g.W + (size_t)k * g.ldw + n0 + n, g.W, BR_C, g.ldw, g.CI, "bwd_ring W");
        const float4 w = *reinterpret_cast<const float4*>(g.W + (size_t)k * g.ldw + n0 + n);
        *reinterpret_cast<float4*>(&Wl[k * 128 + (n ^ (((k >> 4) & 1) << 5))]) = w;
    }
    for (int e = tid; e < 5 * BR_C; e += BR_THREADS) {
        const int c = e & (BR_C - 1), f = e >> 7;
        const float* src = f == 0 ? g.a.s : f == 1 ? g.a.t : f == 2 ? g.a.mean : f == 3 ? g.a.alpha : g.a.kb;
        cf[e] = src[c];
    }
    // (read from LDS where used: registers kept across the loop would spill, and a spill reload is a
    // vector-memory load whose compiler-inserted wait drains the ring)
    for (int e = tid; e < 4 * 128; e += BR_THREADS) {
        const int c = e & 127, f = e >> 7;
        const float* src = f == 0 ? g.q.s : f == 1 ? g.q.t : f == 2 ? g.q.mean : g.q.inv;
        qc[f][c] = src[n0 + c];
    }
    const float qslope = g.q.slope;
    __builtin_amdgcn_s_waitcnt(dg_vmcnt(0));
    __syncthreads();

    const unsigned rbase = dg_lds_addr(ring), xbase = dg_lds_addr(Xl);
    // per-lane float offsets of the input-tile reads (row part + swizzled chunk; the two variants are
    // the two values of the row's swizzle bit, br_xswz):
    //   data gradient, row wm*32 + acc_row(r, h), column wn*64 + 32j + l32: swizzle bit (r & 1) ^ h,
    //     chunk bit 3 = j ^ that bit -> xa0 (j ^ r even) / xa1 (odd), + 128 * ((r & 3) + 8 * (r >> 2));
    //   weight gradient, row 2p + h, column 32v + l32: swizzle bit ((p >> 1) & 1) ^ h -> xw0 / xw1, + 256 p
    const int xa0 = wm * 4096 + 512 * h + 4 * (16 * wn + (l32 >> 2) + 8 * h) + (l32 & 3);
    const int xa1 = wm * 4096 + 512 * h + 4 * (16 * wn + (l32 >> 2) + 8 * (1 - h)) + (l32 & 3);
    const int xw0 = 128 * h + 4 * ((8 * v + (l32 >> 2)) ^ (8 * h)) + (l32 & 3);
    const int xw1 = 128 * h + 4 * ((8 * v + (l32 >> 2)) ^ (8 * (1 - h))) + (l32 & 3);
    // dy / z slabs of flattened iteration it (row tile it / 4, slab it % 4) into stage it % NS:
    // thread = (row tid >> 3, 16-B chunk tid & 7), one DMA of dy and one of z per wave
    auto issue_stage = [&](int it) __attribute__((always_inline)) {
        const int ti = it >> 2, ks = it & 3;
        const int m0 = (rb + ti * g.gx) * BR_BM, k0 = ks * BR_BK;
        const int r = tid >> 3;
        const int row = min(m0 + r, M - 1);
        const int ch = 4 * ((tid & 7) ^ dg_swz(r));
        const unsigned d = __builtin_amdgcn_readfirstlane(rbase + 4u * (unsigned)((it % BR_NS) * BR_STAGE + wave * 256));
        const unsigned oy = (unsigned)(row * g.a.ld + k0 + ch), oz = (unsigned)(row * g.a.ldz + k0 + ch);
        PCS_DCHECK_QUAD(g.a.data + oy, g.a.data, M, g.a.ld, BR_C, "bwd_ring dy");
        PCS_DCHECK_QUAD(g.a.z + oz, g.a.z, M, g.a.ldz, BR_C, "bwd_ring z");
        dg_glds16(g.a.data + oy, d);
        dg_glds16(g.a.z + oz, d + 4u * BR_SLAB);
    };
    // the input tile of row tile ti: 2048 chunks, 4 DMAs per wave (each two 128-float rows)
    auto issue_x = [&](int ti) __attribute__((always_inline)) {
        const int m0 = (rb + ti * g.gx) * BR_BM;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = (wave * 4 + j) * 64 + lane;
            const int r = e >> 5, c = e & 31;
            const int row = min(m0 + r, M - 1);
            const float* src = g.q.data + (unsigned)(row * CI + n0 + 4 * (c ^ br_xswz(r)));
            PCS_DCHECK_QUAD(src, g.q.data, M, CI, CI, "bwd_ring input");
            dg_glds16(src, __builtin_amdgcn_readfirstlane(xbase + 4u * (unsigned)((wave * 4 + j) * 256)));
        }
    };

    // role registers, shared: R[0..1] the data gradient's accumulators and R[2..3] its per-slab sums
    // (data-gradient waves) or R[ks] the weight gradient's accumulator of slab ks (weight-gradient
    // waves); F the input tile's values -- raw Z at the epilogue's rows (data gradient) or the B
    // fragments act(BN(Z)) (weight gradient).  One register set for both roles keeps the kernel
    // within the 256 registers of two waves per SIMD.
    f32x16 R[BR_NK];
#pragma unroll
    for (int j = 0; j < BR_NK; ++j) R[j] = f32x16{};
    float F[32];
    double s1[2] = {0.0, 0.0}, s2[2] = {0.0, 0.0};
    float4 dbv[BR_NK];
#pragma unroll
    for (int j = 0; j < BR_NK; ++j) dbv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    bool stores_full = false;

    if (total > 0) {
        issue_stage(0);
        issue_x(0);
    }
    if (total > 1) issue_stage(1);

    const int tr = tid >> 3, tkq = tid & 7;        // this thread's (row, k quad) of the dZ pass
    for (int ti = 0; ti < my_tiles; ++ti) {
        const int m0 = (rb + ti * g.gx) * BR_BM;
#pragma unroll
        for (int ks = 0; ks < BR_NK; ++ks) {
            const int it = ti * BR_NK + ks;
            // ---- stage it landed (with it, at a tile's first slab, the input tile issued before it).
            // A wave's vector-memory ops per tile, in order: slab 0 -> stage it + 2, the next input
            // tile (4); slabs 1, 2 -> stage it + 2; slab 3 -> stage it + 2, the data-gradient waves'
            // 32 full-tile stores.  Those issued after stage it may stay in flight:
            {
                const int s2 = it + 1 < total ? 2 : 0;
                const int x4 = ti + 1 < my_tiles ? 4 : 0;
                const int st32 = awave && ti > 0 && stores_full ? 32 : 0;
                const int n = ks == 0 ? s2 + st32 : ks == 1 ? st32 + s2 + x4 : ks == 2 ? x4 + s2 : s2;
                br_vm_wait(n);
            }
            dg_barrier();
            float* st = ring + (it % BR_NS) * BR_STAGE;
            // ---- dZ in place: BN backward of (dy, z), rows past M zeroed
            {
                float* p = st + tr * BR_BK + 4 * (tkq ^ dg_swz(tr));
                const float4 dy = *reinterpret_cast<const float4*>(p);
                const float4 z = *reinterpret_cast<const float4*>(p + BR_SLAB);
                const int k = ks * BR_BK + 4 * tkq;
                Quad qd;
                qd.s = *reinterpret_cast<const float4*>(&cf[k]);
                qd.t = *reinterpret_cast<const float4*>(&cf[BR_C + k]);
                qd.mean = *reinterpret_cast<const float4*>(&cf[2 * BR_C + k]);
                qd.alpha = *reinterpret_cast<const float4*>(&cf[3 * BR_C + k]);
                qd.kb = *reinterpret_cast<const float4*>(&cf[4 * BR_C + k]);
                float4 o = xform4<OP_BNBWD>(g.a, dy, z, 0u, m0 + tr, qd, k, BR_C);
                if (m0 + tr >= M) o = make_float4(0.f, 0.f, 0.f, 0.f);
                *reinterpret_cast<float4*>(p) = o;
                dbv[ks].x += o.x; dbv[ks].y += o.y; dbv[ks].z += o.z; dbv[ks].w += o.w;
            }
            // ---- at a tile's first slab: the input tile into registers -- the epilogue's raw Z
            // (data-gradient waves) or the weight gradient's act(BN(Z)) B fragments -- so its LDS
            // buffer can take the next tile
            if (ks == 0) {
                if (awave) {
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            F[16 * j + r] = Xl[((j ^ r) & 1 ? xa1 : xa0) + 128 * ((r & 3) + 8 * (r >> 2))];
                } else {
                    const float bs = qc[0][32 * v + l32], bt = qc[1][32 * v + l32];
#pragma unroll
                    for (int p = 0; p < 32; ++p)
                        F[p] = act_f(Xl[((p >> 1) & 1 ? xw1 : xw0) + 256 * p] * bs + bt, 0, qslope);
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            dg_barrier();
            // ---- refill: the stage every wave finished reading one iteration ago; at a tile's first
            // slab also the next input tile (every wave has its copy of this one)
            if (it + 2 < total) issue_stage(it + 2);
            if (ks == 0 && ti + 1 < my_tiles) issue_x(ti + 1);

            if (awave) {
                // ---- data gradient: 32 rows x 64 columns of dZ . W (the slab into a fresh
                // accumulator, then added: dgrad_kernel's two-level fp32 sum)
                const int ar = wm * 32 + l32;
#pragma unroll
                for (int qq = 0; qq < 4; ++qq) {
                    const float4 a = *reinterpret_cast<const float4*>(st + ar * BR_BK + 4 * ((4 * h + qq) ^ dg_swz(ar)));
                    const int kr = ks * BR_BK + 16 * h + 4 * qq;
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int bc = (wn * 64 + 32 * j + l32) ^ (h << 5);
                        const float b0 = Wl[(kr + 0) * 128 + bc], b1 = Wl[(kr + 1) * 128 + bc];
                        const float b2 = Wl[(kr + 2) * 128 + bc], b3 = Wl[(kr + 3) * 128 + bc];
                        const f32x16 c0 = {};
                        R[2 + j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b0, qq == 0 ? c0 : R[2 + j], 0, 0, 0);
                        R[2 + j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b1, R[2 + j], 0, 0, 0);
                        R[2 + j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b2, R[2 + j], 0, 0, 0);
                        R[2 + j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b3, R[2 + j], 0, 0, 0);
                    }
                }
#pragma unroll
                for (int j = 0; j < 2; ++j) R[j] += R[2 + j];
                if (ks == BR_NK - 1) {
                    // ---- tile epilogue: layer l-1's BN-backward sums, then the stores --
                    // unconditional on a full tile, so the next wait can count them
                    const int rb0 = m0 + wm * 32;
                    const bool full = m0 + BR_BM <= M;
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int c = wn * 64 + 32 * j + l32;
                        const float sp = qc[0][c], tp = qc[1][c], mp = qc[2][c], ip = qc[3][c];
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const float o = R[j][r] + 0.f;
                            R[j][r] = o;
                            const bool ok = full || rb0 + br_acc_row(r, h) < M;
                            const float z = F[16 * j + r];
                            const float dy = o * dact_f(z * sp + tp, 0, qslope);
                            const float xh = (z - mp) * ip;
                            const double dd = ok ? (double)dy : 0.0;
                            s1[j] += dd;
                            s2[j] += dd * (double)xh;
                        }
                    }
                    stores_full = full;
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        float* cb = g.dA + (size_t)(rb0 + 4 * h) * CI + n0 + wn * 64 + 32 * j + l32;
                        if (full) {
#pragma unroll
                            for (int r = 0; r < 16; ++r) cb[((r & 3) + 8 * (r >> 2)) * CI] = R[j][r];
                        } else {
#pragma unroll
                            for (int r = 0; r < 16; ++r)
                                if (rb0 + br_acc_row(r, h) < M) cb[((r & 3) + 8 * (r >> 2)) * CI] = R[j][r];
                        }
                        R[j] = f32x16{};
                    }
                }
            } else {
                // ---- weight gradient: dW[32 ks .. +31][n0 + 32 v .. +31] += dZ_slab^T . X, 2 rows per MFMA
#pragma unroll
                for (int p = 0; p < 32; ++p) {
                    const int zr = 2 * p + h;
                    const float a = st[zr * BR_BK + 4 * ((l32 >> 2) ^ dg_swz(zr)) + (l32 & 3)];
                    R[ks] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, F[p], R[ks], 0, 0, 0);
                }
            }
        }
    }
    br_vm_wait(0);
    __syncthreads();

    // ---- layer l-1's BN-backward partials of this row block (both lane halves, both row halves)
    if (awave) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const double a = s1[j] + __shfl_xor(s1[j], 32);
            const double b = s2[j] + __shfl_xor(s2[j], 32);
            if (lane < 32) {
                red[0][wm][wn * 64 + 32 * j + l32] = a;
                red[1][wm][wn * 64 + 32 * j + l32] = b;
            }
        }
    }
    // db partial: each thread's column-quad sums over its rows, added in row order through LDS
    float* dbs = ring;                             // [4][64 rows][32]
#pragma unroll
    for (int ks = 0; ks < BR_NK; ++ks)
        *reinterpret_cast<float4*>(&dbs[(ks * BR_BM + tr) * BR_BK + 4 * tkq]) = dbv[ks];
    __syncthreads();
    if (tid < 128) {
        const int cl = n0 + tid;
        g.bstats[(size_t)cl * g.gx + rb] = red[0][0][tid] + red[0][1][tid];
        g.bstats[((size_t)CI + cl) * g.gx + rb] = red[1][0][tid] + red[1][1][tid];
        if (g.pdb && ct == 0) {
            const int ks = tid >> 5, kk = tid & 31;
            float s = 0.f;
            for (int r = 0; r < BR_BM; ++r) s += dbs[(ks * BR_BM + r) * BR_BK + kk];
            g.pdb[(size_t)rb * BR_C + tid] = s;
        }
    }
    // dW partial: this workgroup's 128 x 128 column tile of its row block's slot
    if (!awave) {
        float* part = g.part + (size_t)rb * BR_C * CI + n0 + 32 * v + l32;
#pragma unroll
        for (int ks = 0; ks < BR_NK; ++ks)
#pragma unroll
            for (int r = 0; r < 16; ++r) part[(ks * 32 + br_acc_row(r, h)) * CI] = R[ks][r];
    }
}

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

bool bwd_ring_ok(int M, int C, int CI, const float* W, int ldw, const pcs_operand* x, const pcs_operand* q) {
    if (M < BR_BM || !W || !al16(W) || C != BR_C || (CI != 128 && CI != 256) || ldw % 4 != 0 || ldw < CI) return false;
    if (!x || x->mode != PCS_OP_BNBWD || x->ld % 4 != 0 || x->ld < C || x->ldz % 4 != 0 || x->ldz < C) return false;
    if (!al16(x->data) || !al16(x->z) || !x->s || !x->t || !x->mean || !x->alpha || !x->kb) return false;
    return q && q->data && al16(q->data) && q->ld == CI && q->s && q->t && q->mean && q->inv;
}

int bwd_ring_grid(int M, int CI) {
    const int tiles = (M + BR_BM - 1) / BR_BM, ntn = CI / 128;
    return std::max(1, std::min(tiles, 256 / ntn));
}

size_t bwd_ring_ws_bytes(int M, int C, int CI) {
    return (size_t)bwd_ring_grid(M, CI) * ((size_t)C * CI + C) * sizeof(float) + 256;
}

int bwd_ring(const pcs_operand* x, const pcs_operand* q, int CI, const float* W, int ldw, int M, float* dA, int ldd,
             double* bstats, float* dW, float* db, void* ws, size_t ws_bytes, hipStream_t st) {
    PCS_CHECK_ARG(bwd_ring_ok(M, BR_C, CI, W, ldw, x, q),
                  "bwd_ring: unsupported shape CI=%d M=%d", CI, M);
    PCS_CHECK_ARG(dA && ldd == CI && bstats && dW, "bwd_ring: bad output arguments");
    PCS_CHECK_ARG(ws && ws_bytes >= bwd_ring_ws_bytes(M, BR_C, CI), "bwd_ring: workspace too small");
    BwdRingArgs a{};
    a.a = to_dev_operand(x, M, BR_C);
    a.q = to_dev_operand(q, M, CI);
    a.W = W;
    a.ldw = ldw;
    a.M = M;
    a.CI = CI;
    a.dA = dA;
    a.ldd = ldd;
    a.bstats = bstats;
    a.gx = bwd_ring_grid(M, CI);
    a.ntn = CI / 128;
    a.part = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
    a.pdb = db ? a.part + (size_t)a.gx * BR_C * CI : nullptr;
    const dim3 grid((unsigned)(a.gx * a.ntn));
    auto launch = [=]() {
        if (CI == 128) hipLaunchKernelGGL(bwd_ring_kernel<128>, grid, dim3(BR_THREADS), 0, st, a);
        else hipLaunchKernelGGL(bwd_ring_kernel<256>, grid, dim3(BR_THREADS), 0, st, a);
    };
    int probe = -1;
    if (probe_enabled()) {
        // algorithmic bytes: dy and Z once per column tile, the input tile read and dA written once, W
        const double bytes = 8.0 * M * BR_C * a.ntn + 8.0 * M * CI + 4.0 * BR_C * CI;
        probe = probe_start(CI == 128 ? "pcs::bwd_ring_kernel<128>" : "pcs::bwd_ring_kernel<256>", 4.0 * M * BR_C * CI,
                            bytes, st, launch);
    }
    launch();
    probe_stop(probe, st);
    wgrad_reduce_launch(a.part, a.gx, (long long)BR_C * CI, dW, a.pdb, BR_C, db, st);
    return launch_status("bwd_ring");
}

}  // namespace pcs
