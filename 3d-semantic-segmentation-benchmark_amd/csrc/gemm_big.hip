// Wide-layer GEMM on plain operands: C[M x N] = A[M x R] . B[N x R]^T (+ bias), fp32 on the
// MFMA cores (v_mfma_f32_32x32x2_f32), LDS filled by LDS-DMA (global_load_lds_dwordx4).
//
// Used where both operands are plain row-major matrices with the contraction axis contiguous
// and the GEMM is large enough to be MFMA-bound: DGCNN's conv5..conv7 (models/dgcnn/dgcnn.py:
// 188-207) forward (A = the layer input, B = W) and data gradient (A = the materialised dZ,
// B = W^T, transposed once per backward), M = B*N = 131072 rows.  The general row GEMM
// (mlp.hip) keeps everything that needs an on-load transform (BN+act, BN-backward rebuild),
// the fused pooling epilogue, or narrow tiles.
//
// Design (CDNA4):
//  * 256 x BN output tile (BN = 256 or 128) per 512-thread workgroup, 8 waves as WM x WN,
//    each wave 4 x 2 (or 2 x 2) 32x32 MFMA tiles; one workgroup per CU (128 / 96 KB of LDS);
//  * K in 32-deep slabs, two LDS stages: slab s+1's DMA is issued before slab s is read, so the
//    loads land under 4-8K cycles of MFMAs; one vmcnt(0) + barrier per slab;
//  * the LDS image is lane-linear (an LDS-DMA writes base + 16 * lane), rows of 32 floats whose
//    16-B chunks are XOR-swizzled by (row >> 1) & 7 -- applied to the per-lane SOURCE address
//    and to the fragment read, so the ds_read_b128 of 16 consecutive rows hit 16 distinct
//    16-B slots of the 256-B bank row (conflict-free);
//  * inside a slab lane half h takes k = 16h + 4qq + c (qq, c = 0..3): each lane's A and B
//    fragments are float4s of one LDS row (the MFMA sums over k, so the permutation only
//    reorders the fp32 accumulation, as in the row GEMM);
//  * XCD-aware tile order (bijective remap of the 1-D grid): each XCD walks a contiguous run of
//    tiles, so the column tiles of one 256-row A strip run on one L2 at the same time;
//  * epilogue: bias, store, and (STATS) per-column fp64 (sum, sum of squares) of the tile's
//    rows into the BN partial layout [2][N][row tiles] that bn_finalize reads.
#include "mlp_common.hpp"

namespace pcs {

constexpr int NT_BM = 256, NT_BK = 32;

__device__ __forceinline__ int nt_swz(int r) { return (r >> 1) & 7; }

// One LDS-DMA (16 B per lane to LDS byte address dst + 16 * lane), issued from inline asm so
// hipcc does not track it: it would otherwise drain the DMA queue (vmcnt(0)) before the first
// ds_read of every slab, serialising the next slab's loads with this slab's MFMAs.  Completion
// is waited for explicitly (vmcnt(0) + barrier at the end of each slab).  M0 is written and
// restored inside the statement (it is compiler-reserved).
__device__ __forceinline__ void glds16(const float* gsrc, unsigned dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(dst)
                 : "memory");
}

__device__ __forceinline__ unsigned lds_addr(const float* p) {
    return (unsigned)(uintptr_t)((const __attribute__((address_space(3))) float*)p);
}

template <int BN, int WM, int WN, bool STATS>
__global__ __launch_bounds__(512, 1) void gemm_nt_kernel(const float* __restrict__ A, int lda,
                                                         const float* __restrict__ B, int ldb, int M, int N, int R,
                                                         const float* __restrict__ bias, float* __restrict__ C, int ldc,
                                                         double* __restrict__ stats, int ntn, int mtiles) {
    constexpr int BM = NT_BM, BK = NT_BK;
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
    constexpr int STAGE = (BM + BN) * BK;                  // floats per LDS stage
    constexpr int AI = BM * BK / 256 / 8;                  // 1-KB DMA instructions per wave per stage (A)
    constexpr int BI = BN * BK / 256 / 8;                  // (B)
    static_assert(WM * WN == 8 && TM >= 1 && TN >= 1 && AI >= 1 && BI >= 1, "nt tile");
    // ONE shared array (a second __shared__ object can make hipcc drain the DMA queue before
    // every ds_read); the epilogue reuses it for the stats reduction
    __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int h = lane >> 5, l32 = lane & 31;

    // bijective XCD remap: blocks bid, bid + 8, ... share an XCD; give them consecutive tiles
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
    const int mt = t / ntn, nt = t - mt * ntn;
    const int m0 = mt * BM, n0 = nt * BN;

    // per-lane DMA sources (rows clamped in range: rows past M / N are computed and discarded)
    const int lrow = lane >> 3, lpos = lane & 7;
    const float* asrc[AI];
    const float* bsrc[BI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
        const int r = (wave * AI + j) * 8 + lrow;
        asrc[j] = A + (size_t)min(m0 + r, M - 1) * lda + 4 * (lpos ^ nt_swz(r));
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
        const int r = (wave * BI + j) * 8 + lrow;
        bsrc[j] = B + (size_t)min(n0 + r, N - 1) * ldb + 4 * (lpos ^ nt_swz(r));
    }
    const unsigned lbase = lds_addr(lds);
    auto stage = [&](int buf, int k0) {
        const unsigned sa = __builtin_amdgcn_readfirstlane(lbase + 4u * (unsigned)(buf * STAGE + wave * AI * 256));
        const unsigned sb = __builtin_amdgcn_readfirstlane(lbase + 4u * (unsigned)(buf * STAGE + BM * BK + wave * BI * 256));
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            PCS_DCHECK_QUAD(asrc[j] + k0, A, M, lda, R, "gemm_nt A");
            glds16(asrc[j] + k0, sa + 1024u * j);
        }
#pragma unroll
        for (int j = 0; j < BI; ++j) {
            PCS_DCHECK_QUAD(bsrc[j] + k0, B, N, ldb, R, "gemm_nt B");
            glds16(bsrc[j] + k0, sb + 1024u * j);
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // fragment offsets (floats) inside a stage, chunk 4h of row; qq XORs into the chunk index
    int aoff[TM], boff[TN], asw[TM], bsw[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int r = wm * WTM + i * 32 + l32;
        aoff[i] = r * BK;
        asw[i] = nt_swz(r);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int r = wn * WTN + j * 32 + l32;
        boff[j] = BM * BK + r * BK;
        bsw[j] = nt_swz(r);
    }

    const int ns = R / BK;
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int s = 0; s < ns; ++s) {
        const int buf = s & 1;
        if (s + 1 < ns) stage(buf ^ 1, (s + 1) * BK);
        const float* st = lds + buf * STAGE;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            float4 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                a[i] = *reinterpret_cast<const float4*>(st + aoff[i] + 4 * ((4 * h + qq) ^ asw[i]));
#pragma unroll
            for (int j = 0; j < TN; ++j)
                b[j] = *reinterpret_cast<const float4*>(st + boff[j] + 4 * ((4 * h + qq) ^ bsw[j]));
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
                }
        }
        // the MFMAs stay above the wait: they touch no memory, so hipcc would otherwise hoist the
        // wait (for the NEXT slab's DMA) and the barrier above them and expose the DMA latency
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // ---- epilogue
    double s1[TN], s2[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * WTN + j * 32 + l32;
        const bool cok = col < N;
        const float bv = (bias && cok) ? bias[col] : 0.f;
        s1[j] = 0.0;
        s2[j] = 0.0;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int rb = m0 + wm * WTM + i * 32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = rb + (r & 3) + 8 * (r >> 2) + 4 * h;
                const float v = acc[i][j][r] + bv;
                const bool ok = cok && row < M;
                if (ok) C[(size_t)row * ldc + col] = v;
                if (STATS) {
                    const double d = ok ? (double)v : 0.0;
                    s1[j] += d;
                    s2[j] += d * d;
                }
            }
        }
    }
    if (STATS) {
        double* red = reinterpret_cast<double*>(lds);        // [2][WM][BN]
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const double a = s1[j] + __shfl_xor(s1[j], 32);
            const double b = s2[j] + __shfl_xor(s2[j], 32);
            const int lc = wn * WTN + j * 32 + l32;
            if (lane < 32) {
                red[wm * BN + lc] = a;
                red[(WM + wm) * BN + lc] = b;
            }
        }
        __syncthreads();
        for (int c = tid; c < BN; c += 512) {
            const int col = n0 + c;
            if (col < N) {
                double a = 0.0, b = 0.0;
#pragma unroll
                for (int w = 0; w < WM; ++w) { a += red[w * BN + c]; b += red[(WM + w) * BN + c]; }
                stats[(size_t)col * mtiles + mt] = a;
                stats[((size_t)N + col) * mtiles + mt] = b;
            }
        }
    }
}

// the wide path's column tile for N outputs: 256 unless a 128-wide tile wastes less (round 3:
// 6 x 256 columns for conv6's 1408 measured slower than 11 x 128, profiles/r03_final_checks.txt)
// (256- or 128-column tiles throughout measured 16.52 / 16.09 vs 16.07 ms, profiles/r05_ab_nt_column_tile.txt)
int gemm_nt_bn(int N) {
    const int w256 = ((N + 255) / 256) * 256 - N, w128 = ((N + 127) / 128) * 128 - N;
    return w128 < w256 ? 128 : 256;
}
static int nt_bn(int N) { return gemm_nt_bn(N); }

bool gemm_nt_regime(int M, int N) { return M >= 65536 && N >= 256; }

int gemm_nt_row_tiles(int M) { return (M + NT_BM - 1) / NT_BM; }

bool gemm_nt_ok(const float* A, int lda, const float* B, int ldb, int M, int N, int R) {
    return gemm_nt_regime(M, N) && R % NT_BK == 0 && R >= NT_BK && lda % 4 == 0 && ldb % 4 == 0 && lda >= R &&
           ldb >= R && (reinterpret_cast<uintptr_t>(A) & 15) == 0 && (reinterpret_cast<uintptr_t>(B) & 15) == 0;
}

int gemm_nt(const float* A, int lda, const float* B, int ldb, int M, int N, int R, const float* bias, float* C, int ldc,
            double* stats, hipStream_t st) {
    const int mtiles = gemm_nt_row_tiles(M);
    const int bn = nt_bn(N);
    const int ntn = (N + bn - 1) / bn;
    const long long tiles = (long long)mtiles * ntn;
    PCS_CHECK_ARG(tiles < (1ll << 31), "gemm_nt: too many tiles");
    const dim3 grid((unsigned)tiles);
#define PCS_NT(BNV, WMV, WNV)                                                                                     \
    do {                                                                                                          \
        if (stats)                                                                                                \
            hipLaunchKernelGGL((gemm_nt_kernel<BNV, WMV, WNV, true>), grid, dim3(512), 0, st, A, lda, B, ldb, M, N, \
                               R, bias, C, ldc, stats, ntn, mtiles);                                              \
        else                                                                                                      \
            hipLaunchKernelGGL((gemm_nt_kernel<BNV, WMV, WNV, false>), grid, dim3(512), 0, st, A, lda, B, ldb, M, \
                               N, R, bias, C, ldc, stats, ntn, mtiles);                                           \
    } while (0)
    if (bn == 256) PCS_NT(256, 2, 4);
    else PCS_NT(128, 4, 2);
#undef PCS_NT
    return launch_status("gemm_nt");
}


// ------------------------------------------------------------------ weight gradient, plain operands
// part[split][n][k] = sum over the split's rows m of X[m][n] * Y[m][k]   (X = a wide layer's
// materialised dZ, M x N; Y = its input, M x K; both row-major).  The reduction axis is the
// ROW, so both LDS images are row slabs [32 rows][256 | BI channels] copied by LDS-DMA as they
// lie in memory; a lane's MFMA operand is one float (X[m][n] / Y[m][k], m = 2p + h of m-pair p),
// read with ds_read_b32.  Odd rows have their 16-B chunks XOR 8 (source address and read), so
// the two lane halves (rows 2p, 2p + 1) hit disjoint bank halves.  Splits of rows_per_split
// (a multiple of 32; M % 32 == 0) rows: every slab is full, no zero fill.  The partial tiles are
// summed in split order by wgrad_reduce_kernel (deterministic).
__device__ __forceinline__ int tn_swz(int m) { return (m & 1) << 3; }

template <int BI, int WM, int WN>
__global__ __launch_bounds__(512, 1) void wgrad_nt_kernel(const float* __restrict__ X, int ldx,
                                                          const float* __restrict__ Y, int ldy, int M, int N, int K,
                                                          int rows_per_split, int tiles_k, int tiles,
                                                          float* __restrict__ part) {
    constexpr int BO = 256, BR = 32;
    constexpr int WTO = BO / WM, WTI = BI / WN, TM = WTO / 32, TN = WTI / 32;
    constexpr int STAGE = BR * (BO + BI);
    constexpr int XCPR = BO / 4, YCPR = BI / 4;             // 16-B chunks per LDS row
    constexpr int XI = BR * BO / 256 / 8, YI = BR * BI / 256 / 8;   // 1-KB DMAs per wave per stage
    static_assert(WM * WN == 8 && TM >= 1 && TN >= 1 && XI >= 1 && YI >= 1, "tn tile");
    __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wo = wave / WN, wi = wave % WN;
    const int h = lane >> 5, l32 = lane & 31;

    // XCD remap, then tile-fastest: the tiles of one row split (same X / Y rows) share an L2
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
    const int sp = t / tiles, ti = t - sp * tiles;
    const int n0 = (ti / tiles_k) * BO, k0 = (ti % tiles_k) * BI;
    const int rb = sp * rows_per_split;
    const int ns = (min(M, rb + rows_per_split) - rb) / BR;

    // DMA sources: instruction j of this wave covers LDS rows starting at (wave*XI + j) * (64/XCPR)
    const float* xsrc[XI];
    const float* ysrc[YI];
#pragma unroll
    for (int j = 0; j < XI; ++j) {
        const int e = (wave * XI + j) * 64 + lane;          // chunk index in the slab
        const int r = e / XCPR, c = e % XCPR;
        xsrc[j] = X + (size_t)(rb + r) * ldx + min(n0 + 4 * (c ^ tn_swz(r)), ((N + 3) & ~3) - 4);
    }
#pragma unroll
    for (int j = 0; j < YI; ++j) {
        const int e = (wave * YI + j) * 64 + lane;
        const int r = e / YCPR, c = e % YCPR;
        ysrc[j] = Y + (size_t)(rb + r) * ldy + min(k0 + 4 * (c ^ tn_swz(r)), ((K + 3) & ~3) - 4);
    }
    const unsigned lbase = lds_addr(lds);
    auto stage = [&](int buf, int slab) {
        const size_t xo = (size_t)slab * BR * ldx, yo = (size_t)slab * BR * ldy;
        const unsigned sx = __builtin_amdgcn_readfirstlane(lbase + 4u * (unsigned)(buf * STAGE + wave * XI * 256));
        const unsigned sy =
            __builtin_amdgcn_readfirstlane(lbase + 4u * (unsigned)(buf * STAGE + BR * BO + wave * YI * 256));
#pragma unroll
        for (int j = 0; j < XI; ++j) {
            PCS_DCHECK_QUAD(xsrc[j] + xo, X, M, ldx, N, "wgrad_nt X");
            glds16(xsrc[j] + xo, sx + 1024u * j);
        }
#pragma unroll
        for (int j = 0; j < YI; ++j) {
            PCS_DCHECK_QUAD(ysrc[j] + yo, Y, M, ldy, K, "wgrad_nt Y");
            glds16(ysrc[j] + yo, sy + 1024u * j);
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // operand offsets (floats) within a stage for row parity h (rows 2p + h: the swizzle is fixed
    // per lane, the row advances by 2 * row length per m-pair)
    int xoff[TM], yoff[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int n = wo * WTO + i * 32 + l32;
        xoff[i] = h * BO + 4 * ((n >> 2) ^ tn_swz(h)) + (n & 3);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int k = wi * WTI + j * 32 + l32;
        yoff[j] = BR * BO + h * BI + 4 * ((k >> 2) ^ tn_swz(h)) + (k & 3);
    }

    if (ns > 0) {
        stage(0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (int s = 0; s < ns; ++s) {
        const int buf = s & 1;
        if (s + 1 < ns) stage(buf ^ 1, s + 1);
        const float* st = lds + buf * STAGE;
        // all 16 m-pairs' operands are read up front (TM + TN floats each): the ds_reads run far
        // ahead of the MFMAs that consume them instead of one MFMA ahead
        float a[16][TM], b[16][TN];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
#pragma unroll
            for (int i = 0; i < TM; ++i) a[u][i] = st[xoff[i] + 2 * u * BO];
#pragma unroll
            for (int j = 0; j < TN; ++j) b[u][j] = st[yoff[j] + 2 * u * BI];
        }
        __builtin_amdgcn_sched_barrier(0);      // keep the reads ahead (the scheduler sinks them)
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][i], b[u][j], acc[i][j], 0, 0, 0);
        // the MFMAs stay above the wait: they touch no memory, so hipcc would otherwise hoist the
        // wait (for the NEXT slab's DMA) and the barrier above them and expose the DMA latency
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    float* __restrict__ tp = part + (size_t)sp * N * K;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int k = k0 + wi * WTI + j * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = n0 + wo * WTO + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (n < N && k < K) tp[(size_t)n * K + k] = acc[i][j][r];
            }
        }
}

// plan of the wide weight gradient: column tile BI (256, or 128 when it wastes less or the
// 256-wide tiles are too few), ~512 blocks, row splits a multiple of 32 rows
static void wgrad_nt_plan(int N, int K, int M, int* bi, int* tiles_k, int* tiles, int* splits, int* rows) {
    const int tn = (N + 255) / 256;
    const int w256 = ((K + 255) / 256) * 256 - K, w128 = ((K + 127) / 128) * 128 - K;
    int b = (w128 < w256 || tn * ((K + 255) / 256) < 8) ? 128 : 256;
    *bi = b;
    *tiles_k = (K + b - 1) / b;
    *tiles = tn * *tiles_k;
    int sp = (512 + *tiles - 1) / *tiles;
    int r = (M + sp - 1) / sp;
    r = ((r + 31) / 32) * 32;
    *rows = r;
    *splits = (M + r - 1) / r;
}

// Taken only for few output tiles (<= 4, e.g. DGCNN conv7's 256 x 512): there it beats the
// row-split wgrad (mlp.hip) by 25 %, while on conv5 / conv6 (12-22 tiles, 96-180 slabs per
// split) it runs 8-13 % behind it (scripts/gemm_nt_ab.py, same-process A/B).
bool wgrad_nt_ok(const float* X, int ldx, const float* Y, int ldy, int M, int N, int K) {
    int bi, tk, tiles, sp, rows;
    wgrad_nt_plan(N, K, M, &bi, &tk, &tiles, &sp, &rows);
    return tiles <= 4 && M >= 65536 && M % 32 == 0 && N >= 256 && K >= 128 && N % 4 == 0 && K % 4 == 0 && ldx % 4 == 0 &&
           ldy % 4 == 0 && ldx >= N && ldy >= K && (reinterpret_cast<uintptr_t>(X) & 15) == 0 &&
           (reinterpret_cast<uintptr_t>(Y) & 15) == 0;
}

size_t wgrad_nt_ws_bytes(int N, int K, int M) {
    int bi, tk, tiles, sp, rows;
    wgrad_nt_plan(N, K, M, &bi, &tk, &tiles, &sp, &rows);
    return (size_t)sp * N * K * sizeof(float) + 256;
}

// launches the partial tiles; returns the number of splits (the reduce's count) or -1
int wgrad_nt(const float* X, int ldx, const float* Y, int ldy, int M, int N, int K, float* part, hipStream_t st) {
    int bi, tk, tiles, sp, rows;
    wgrad_nt_plan(N, K, M, &bi, &tk, &tiles, &sp, &rows);
    const dim3 grid((unsigned)(sp * tiles));
    if (bi == 256)
        hipLaunchKernelGGL((wgrad_nt_kernel<256, 2, 4>), grid, dim3(512), 0, st, X, ldx, Y, ldy, M, N, K, rows, tk,
                           tiles, part);
    else
        hipLaunchKernelGGL((wgrad_nt_kernel<128, 4, 2>), grid, dim3(512), 0, st, X, ldx, Y, ldy, M, N, K, rows, tk,
                           tiles, part);
    return sp;
}

const char* wgrad_nt_name(int N, int K, int M) {
    int bi, tk, tiles, sp, rows;
    wgrad_nt_plan(N, K, M, &bi, &tk, &tiles, &sp, &rows);
    return bi == 256 ? "pcs::wgrad_nt_kernel<256, 2, 4>" : "pcs::wgrad_nt_kernel<128, 4, 2>";
}
}  // namespace pcs

using namespace pcs;

// C[M x N] = A[M x R] . B[N x R]^T (+ bias); stats (nullable): [2][N][pcs_gemm_nt_row_tiles(M)]
// fp64 (sum, sum of squares) partials of C.  Both operands row-major with the contraction axis
// contiguous (lda, ldb multiples of 4, 16-B aligned), R a multiple of 32, M >= 65536, N >= 256.
PCS_API int pcs_gemm_nt(const float* A, int lda, const float* B, int ldb, int M, int N, int R, const float* bias,
                        float* C, int ldc, double* stats, void* stream) {
    PCS_CHECK_ARG(A && B && C && M >= 1 && N >= 1 && R >= 1 && ldc >= N, "pcs_gemm_nt: bad arguments");
    PCS_CHECK_ARG(gemm_nt_ok(A, lda, B, ldb, M, N, R),
                  "pcs_gemm_nt: needs M >= 65536, N >= 256, R %% 32 == 0, lda/ldb multiples of 4 >= R, 16-B aligned "
                  "operands (M=%d N=%d R=%d lda=%d ldb=%d)", M, N, R, lda, ldb);
    return gemm_nt(A, lda, B, ldb, M, N, R, bias, C, ldc, stats, as_stream(stream));
}

PCS_API int pcs_gemm_nt_row_tiles(int M) { return gemm_nt_row_tiles(M); }
