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
constexpr int BR_NS = 5;                       // ring stages (four slabs in flight)
constexpr int BR_SLAB = BR_BM * BR_BK;         // floats of one dy (or z) slab: 8 KB
constexpr int BR_STAGE = 2 * BR_SLAB;          // dy + z
constexpr int BR_X = BR_BM * 128;              // the input tile (64 rows x the 128-column tile): 32 KB
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

// s_waitcnt vmcnt(n), n even in [0, 42] (the immediate must be a constant)
__device__ __forceinline__ void br_vm_wait(int n) {
    switch (n) {
#define BR_W(k) \
    case k: __builtin_amdgcn_s_waitcnt(dg_vmcnt(k)); break;
    BR_W(2) BR_W(4) BR_W(6) BR_W(8) BR_W(10) BR_W(12) BR_W(14) BR_W(32) BR_W(34) BR_W(36) BR_W(38) BR_W(40) BR_W(42)
#undef BR_W
    default: __builtin_amdgcn_s_waitcnt(dg_vmcnt(0)); break;
    }
    asm volatile("" ::: "memory");
}

// CI: the input width (128 or 256), also the row stride of dA and of the previous layer's Z.
// Waves 0-3 (data gradient): wave v owns dA columns n0 + 32v .. +31 over all 64 rows (two 32-row
// MFMA blocks) and holds its W fragments -- W[32 ks + 16 h + 4 qq + u][n0 + 32 v + l32], 64 values
// -- in registers for the whole launch.  Waves 4-7 (weight gradient): wave 4 + v owns dW columns
// n0 + 32v .. +31, one 32 x 32 accumulator per slab.  Per slab every wave waits only for its OWN
// slab DMAs (the rows it rebuilds into dZ are the rows it loaded), rebuilds them, and one barrier
// publishes the slab.
template <int CI>
__global__ __launch_bounds__(BR_THREADS, 1) void bwd_ring_kernel(const BwdRingArgs g) {
    __shared__ __attribute__((aligned(16))) float ring[BR_NS * BR_STAGE];
    __shared__ __attribute__((aligned(16))) float Xl[2][BR_X];
    __shared__ __attribute__((aligned(16))) float cf[5 * BR_C];     // s | t | mean | alpha | kb
    __shared__ float qc[4][128];                   // layer l-1's s | t | mean | inv over the column tile

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool awave = wave < 4;                   // data gradient (else weight gradient)
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

    // ---- resident operands, all loaded before the first DMA (a plain load issued later would make
    // the compiler's wait for it drain the ring): the dZ coefficients and layer l-1's BN over the
    // column tile in LDS, the data-gradient waves' W fragments in registers
    for (int e = tid; e < 5 * BR_C; e += BR_THREADS) {
        const int c = e & (BR_C - 1), f = e >> 7;
        const float* src = f == 0 ? g.a.s : f == 1 ? g.a.t : f == 2 ? g.a.mean : f == 3 ? g.a.alpha : g.a.kb;
        cf[e] = src[c];
    }
    for (int e = tid; e < 4 * 128; e += BR_THREADS) {
        const int c = e & 127, f = e >> 7;
        const float* src = f == 0 ? g.q.s : f == 1 ? g.q.t : f == 2 ? g.q.mean : g.q.inv;
        qc[f][c] = src[n0 + c];
    }
    const float qslope = g.q.slope;
    __builtin_amdgcn_s_waitcnt(dg_vmcnt(0));
    __syncthreads();

    const unsigned rbase = dg_lds_addr(ring), xbase = dg_lds_addr(&Xl[0][0]);
    // per-lane float offsets of the input-tile reads (row part + swizzled chunk; the two variants are
    // the two values of the row's swizzle bit, br_xswz):
    //   data gradient, row 32 rb2 + acc_row(r, h), column 32v + l32: swizzle bit (r & 1) ^ h -> xa0
    //     (r even) / xa1 (r odd), + 4096 rb2 + 128 * ((r & 3) + 8 * (r >> 2));
    //   weight gradient, row 2p + h, column 32v + l32: swizzle bit ((p >> 1) & 1) ^ h -> xw0 / xw1, + 256 p
    const int xa0 = 512 * h + 4 * (8 * (v ^ h) + (l32 >> 2)) + (l32 & 3);
    const int xa1 = 512 * h + 4 * (8 * (v ^ h ^ 1) + (l32 >> 2)) + (l32 & 3);
    const int xw0 = 128 * h + 4 * (8 * (v ^ h) + (l32 >> 2)) + (l32 & 3);
    const int xw1 = 128 * h + 4 * (8 * (v ^ h ^ 1) + (l32 >> 2)) + (l32 & 3);

    // dy / z slabs of flattened iteration it (row tile it / 4, slab it % 4) into stage it % NS:
    // thread = (row tid >> 3, 16-B chunk tid & 7), one DMA of dy and one of z per wave -- a wave's
    // DMAs land exactly the rows its threads rebuild
    const int tr = tid >> 3, tkq = tid & 7;
    auto issue_stage = [&](int it) __attribute__((always_inline)) {
        const int ti = it >> 2, ks = it & 3;
        const int m0 = (rb + ti * g.gx) * BR_BM, k0 = ks * BR_BK;
        const int row = min(m0 + tr, M - 1);
        const int ch = 4 * (tkq ^ dg_swz(tr));
        const unsigned d = __builtin_amdgcn_readfirstlane(rbase + 4u * (unsigned)((it % BR_NS) * BR_STAGE + wave * 256));
        const unsigned oy = (unsigned)(row * g.a.ld + k0 + ch), oz = (unsigned)(row * g.a.ldz + k0 + ch);
        PCS_DCHECK_QUAD(g.a.data + oy, g.a.data, M, g.a.ld, BR_C, "bwd_ring dy");
        PCS_DCHECK_QUAD(g.a.z + oz, g.a.z, M, g.a.ldz, BR_C, "bwd_ring z");
        dg_glds16(g.a.data + oy, d);
        dg_glds16(g.a.z + oz, d + 4u * BR_SLAB);
    };
    // the input tile of row tile ti into buffer ti & 1: 2048 chunks, 4 DMAs per wave (each two rows)
    auto issue_x = [&](int ti) __attribute__((always_inline)) {
        const int m0 = (rb + ti * g.gx) * BR_BM;
        const unsigned xb = xbase + 4u * (unsigned)((ti & 1) * BR_X);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = (wave * 4 + j) * 64 + lane;
            const int r = e >> 5, c = e & 31;
            const int row = min(m0 + r, M - 1);
            const float* src = g.q.data + (unsigned)(row * CI + n0 + 4 * (c ^ br_xswz(r)));
            PCS_DCHECK_QUAD(src, g.q.data, M, CI, CI, "bwd_ring input");
            dg_glds16(src, __builtin_amdgcn_readfirstlane(xb + 4u * (unsigned)((wave * 4 + j) * 256)));
        }
    };
    // role registers: R[0..1] the data gradient's row-block accumulators (data-gradient waves), or
    // R[ks] and R[4 + ks] the weight gradient's two accumulators of slab ks (even / odd row pairs:
    // ONE dependent chain of v_mfma_f32_32x32x2_f32 issues at half the matrix pipe's rate, measured
    // with in-kernel stamps).  The input tile is read from its LDS buffer where used (it stays there
    // for the whole tile: the next one fills the other buffer), so the kernel fits the 256 registers
    // of two waves per SIMD.
    f32x16 R[2 * BR_NK];
#pragma unroll
    for (int j = 0; j < 2 * BR_NK; ++j) R[j] = f32x16{};
    double s1 = 0.0, s2 = 0.0;
    // db: the column sums of this wave's 8 dZ rows per slab (lane-group reduction), lane group ks
    // (lanes 8 ks .. 8 ks + 7) accumulating slab ks's column quad tkq over the tiles
    float4 dbv = make_float4(0.f, 0.f, 0.f, 0.f);
    const float bs = qc[0][32 * v + l32], bt = qc[1][32 * v + l32];     // (weight gradient's B transform)

    // refill j (after the barrier that ends iteration j; j = -5 .. -1 is the prologue): at a tile's
    // first slab that tile's input tile (its buffer was last read by the tile two before, done by
    // now), then stage j + 5 into the stage iteration j's MFMAs just finished with
    auto refill = [&](int j) __attribute__((always_inline)) {
        const int sj = j + BR_NS;
        if ((sj & 3) == 0 && (sj >> 2) < my_tiles) issue_x(sj >> 2);
        if (sj < total) issue_stage(sj);
    };
    // vector-memory ops a wave has issued after stage i's two DMAs when it waits for them (in
    // iteration i - 1): refills i - 4 .. i - 2 (4 for an input tile, 2 per stage) and the
    // data-gradient waves' full-tile stores of iterations i - 4 .. i - 1 (32)
    auto younger = [&](int i) __attribute__((always_inline)) {
        int n = 0;
#pragma unroll
        for (int j = i - 4; j <= i - 2; ++j) {
            const int sj = j + BR_NS;
            if (j >= -BR_NS) {
                if ((sj & 3) == 0 && (sj >> 2) < my_tiles) n += 4;
                if (sj < total) n += 2;
            }
        }
#pragma unroll
        for (int j = i - 4; j <= i - 1; ++j)
            if (awave && j >= 0 && (j & 3) == 3 && (rb + (j >> 2) * g.gx) * BR_BM + BR_BM <= M) n += 32;
        return n;
    };
    // this wave's rows of slab i: wait for its own DMAs (its rows are exactly the ones it loaded, so no
    // barrier is needed before the rebuild), then dZ in place: BN backward of (dy, z), rows past M zeroed
    auto rebuild = [&](int i) __attribute__((always_inline)) {
        br_vm_wait(younger(i));
        const int ti = i >> 2, ks = i & 3;
        const int m0 = (rb + ti * g.gx) * BR_BM;
        float* p = ring + (i % BR_NS) * BR_STAGE + tr * BR_BK + 4 * (tkq ^ dg_swz(tr));
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
#pragma unroll
        for (int m = 8; m < 64; m <<= 1) {
            o.x += __shfl_xor(o.x, m); o.y += __shfl_xor(o.y, m);
            o.z += __shfl_xor(o.z, m); o.w += __shfl_xor(o.w, m);
        }
        if ((lane >> 3) == ks) { dbv.x += o.x; dbv.y += o.y; dbv.z += o.z; dbv.w += o.w; }
    };
    // the end of iteration i: every wave's rows of slab i + 1 rebuilt and its MFMAs on slab i issued
    auto publish = [&](int i) __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        dg_barrier();
        refill(i);
    };

    // Software pipeline, per iteration i: MFMAs on slab i (rebuilt and published last iteration) and
    // the rebuild of slab i + 1, then one barrier.  The two waves of a SIMD take the two in opposite
    // order -- a data-gradient wave issues its MFMAs first, a weight-gradient wave rebuilds first --
    // so each one's rebuild (VALU + LDS) runs under the other's MFMAs and the matrix pipe stays busy.
    if (awave) {
        // data-gradient waves: W's fragments held in registers for the whole launch (landed before
        // the first DMA, so no later wait for them counts the ring)
        float Wr[BR_NK * 16];
#pragma unroll
        for (int j = 0; j < BR_NK * 16; ++j) {
            const int k = 32 * (j >> 4) + 16 * h + (j & 15);
            PCS_DCHECK(k < BR_C && n0 + 32 * v + l32 < g.CI, "bwd_ring W row %d col %d", k, n0 + 32 * v + l32);
            Wr[j] = g.W[(size_t)k * g.ldw + n0 + 32 * v + l32];
        }
        __builtin_amdgcn_s_waitcnt(dg_vmcnt(0));
#pragma unroll
        for (int j = -BR_NS; j < 0; ++j) refill(j);
        if (total > 0) rebuild(0);
        publish(-1);
        const int c = 32 * v + l32;
        for (int ti = 0; ti < my_tiles; ++ti) {
            const int m0 = (rb + ti * g.gx) * BR_BM;
            const float* xl = &Xl[ti & 1][0];
#pragma unroll
            for (int ks = 0; ks < BR_NK; ++ks) {
                const int i = ti * BR_NK + ks;
                const float* st = ring + (i % BR_NS) * BR_STAGE;
                // ---- data gradient: dA[64 rows][32v + l32] += dZ_slab . W_slab, both row blocks
#pragma unroll
                for (int b2 = 0; b2 < 2; ++b2) {
                    const int ar = 32 * b2 + l32;
#pragma unroll
                    for (int qq = 0; qq < 4; ++qq) {
                        const float4 a = *reinterpret_cast<const float4*>(st + ar * BR_BK + 4 * ((4 * h + qq) ^ dg_swz(ar)));
                        const float* w = &Wr[16 * ks + 4 * qq];
                        R[b2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, w[0], R[b2], 0, 0, 0);
                        R[b2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, w[1], R[b2], 0, 0, 0);
                        R[b2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, w[2], R[b2], 0, 0, 0);
                        R[b2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, w[3], R[b2], 0, 0, 0);
                    }
                }
                if (ks == BR_NK - 1) {
                    // ---- tile epilogue: layer l-1's BN-backward sums (per tile in fp32, then into the
                    // fp64 totals), then the stores -- unconditional on a full tile, so later waits
                    // can count them
                    const bool full = m0 + BR_BM <= M;
                    const float sp = qc[0][c], tp = qc[1][c], mp = qc[2][c], ip = qc[3][c];
                    float t1 = 0.f, t2 = 0.f;
#pragma unroll
                    for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const float o = R[b2][r] + 0.f;
                            R[b2][r] = o;
                            const bool ok = full || m0 + 32 * b2 + br_acc_row(r, h) < M;
                            const float z = xl[(r & 1 ? xa1 : xa0) + 4096 * b2 + 128 * ((r & 3) + 8 * (r >> 2))];
                            const float dy = ok ? o * dact_f(z * sp + tp, 0, qslope) : 0.f;
                            t1 += dy;
                            t2 += dy * ((z - mp) * ip);
                        }
                    s1 += (double)t1;
                    s2 += (double)t2;
#pragma unroll
                    for (int b2 = 0; b2 < 2; ++b2) {
                        float* cb = g.dA + (size_t)(m0 + 32 * b2 + 4 * h) * CI + n0 + c;
                        if (full) {
#pragma unroll
                            for (int r = 0; r < 16; ++r) cb[((r & 3) + 8 * (r >> 2)) * CI] = R[b2][r];
                        } else {
#pragma unroll
                            for (int r = 0; r < 16; ++r)
                                if (m0 + 32 * b2 + br_acc_row(r, h) < M) cb[((r & 3) + 8 * (r >> 2)) * CI] = R[b2][r];
                        }
                        R[b2] = f32x16{};
                    }
                }
                if (i + 1 < total) rebuild(i + 1);
                publish(i);
            }
        }
    } else {
#pragma unroll
        for (int j = -BR_NS; j < 0; ++j) refill(j);
        if (total > 0) rebuild(0);
        publish(-1);
        for (int ti = 0; ti < my_tiles; ++ti) {
            const float* xl = &Xl[ti & 1][0];
#pragma unroll
            for (int ks = 0; ks < BR_NK; ++ks) {
                const int i = ti * BR_NK + ks;
                const float* st = ring + (i % BR_NS) * BR_STAGE;
                if (i + 1 < total) rebuild(i + 1);
                // ---- weight gradient: dW[32 ks .. +31][n0 + 32 v .. +31] += dZ_slab^T . X, 2 rows per MFMA
#pragma unroll
                for (int p = 0; p < 32; ++p) {
                    const int zr = 2 * p + h;
                    const float a = st[zr * BR_BK + 4 * ((l32 >> 2) ^ dg_swz(zr)) + (l32 & 3)];
                    const float b = act_f(xl[((p >> 1) & 1 ? xw1 : xw0) + 256 * p] * bs + bt, 0, qslope);
                    R[ks + 4 * (p & 1)] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, R[ks + 4 * (p & 1)], 0, 0, 0);
                }
                publish(i);
            }
        }
    }
    br_vm_wait(0);
    __syncthreads();

    // ---- layer l-1's BN-backward partials of this row block: a data-gradient wave owns its 32 columns
    if (awave) {
        const double a = s1 + __shfl_xor(s1, 32);
        const double b = s2 + __shfl_xor(s2, 32);
        if (lane < 32) {
            const int cl = n0 + 32 * v + l32;
            g.bstats[(size_t)cl * g.gx + rb] = a;
            g.bstats[((size_t)CI + cl) * g.gx + rb] = b;
        }
    }
    // db partial: the waves' column-quad sums (lane 8 ks + tkq of each wave holds slab ks, quad
    // tkq), added in wave order
    float* dbs = ring;                             // [8 waves][4 slabs][32]
    if (lane < 32)
        *reinterpret_cast<float4*>(&dbs[(wave * BR_NK + (lane >> 3)) * BR_BK + 4 * tkq]) = dbv;
    __syncthreads();
    if (tid < 128 && g.pdb && ct == 0) {
        const int ks = tid >> 5, kk = tid & 31;
        float sum = 0.f;
        for (int w = 0; w < 8; ++w) sum += dbs[(w * BR_NK + ks) * BR_BK + kk];
        g.pdb[(size_t)rb * BR_C + tid] = sum;
    }
    // dW partial: this workgroup's 128 x 128 column tile of its row block's slot
    if (!awave) {
        float* part = g.part + (size_t)rb * BR_C * CI + n0 + 32 * v + l32;
#pragma unroll
        for (int ks = 0; ks < BR_NK; ++ks)
#pragma unroll
            for (int r = 0; r < 16; ++r) part[(ks * 32 + br_acc_row(r, h)) * CI] = R[ks][r] + R[4 + ks][r];
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
