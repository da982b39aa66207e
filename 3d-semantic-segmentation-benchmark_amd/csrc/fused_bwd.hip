// Fused backward of one thin shared-MLP layer: data gradient AND weight gradient from ONE
// read of the layer's rebuilt dZ.
//
// Reference semantics: the autograd backward of conv1x1 -> BatchNorm(train) -> act
// (MiniPointNet / UnitPointNet, models/utils/common.py:125-178), for an inner layer l of a
// stack whose input is the previous layer's BN + activation:
//   dA_{l-1} = dZ_l . W_l                 (M x CI; then BN-backward sums of layer l-1)
//   dW_l    += dZ_l^T . act(BN(Z_{l-1}))  (C x CI),   db_l += column sums of dZ_l
// The separate path (mlp.hip) runs these as two GEMMs -- the dgrad on the caller's stream,
// the wgrad on the side lane -- and each rebuilds dZ (output gradient x act' and the BN
// backward) from HBM: on the thin layers (C, CI <= 128 over 10^5..10^6 rows: PointNet++
// SA1/SA2/SA3/FP1, PointNeXt) both are HBM-latency bound and the pair reads dZ's inputs
// two or three times.  Here one workgroup stages a 64-row tile once:
//   Zs = dZ tile (rebuilt on load, rows past M zeroed)     64 x C
//   Xs = the previous layer's RAW pre-BN Z tile             64 x CI
// and runs both MFMA products out of LDS:
//   * dA tile = Zs . W with W's fragments held in registers for the whole launch (each wave
//     owns one 32-wide column strip of dA), stored with the previous layer's BN-backward
//     partial sums (sum dy, sum dy*xhat, dy = dA*act'(z*s+t), z read back from Xs) -- the
//     epilogue of the dgrad GEMM;
//   * dW += Zs^T . act(Xs*s + t): the activation is applied as the B fragment is read, so
//     the raw z stays available for the epilogue; accumulators live across the block's
//     tiles (persistent grid), one partial tile per block, summed in block order by
//     wgrad_reduce_kernel (deterministic: no float atomics).
// Every MFMA is v_mfma_f32_32x32x2_f32 (fp32 in, fp32 accumulate), so the results differ
// from the two-GEMM path only in fp32 summation order.
#include "mlp_common.hpp"

namespace pcs {

constexpr int FB_BM = 64;        // rows per tile

struct FusedBwdArgs {
    Operand x;            // layer l's dZ operand: BNBWD / POOLBWD (rebuilt on load) or PLAIN, C wide
    Operand q;            // layer l-1: data = its pre-BN Z (M x CI, stride ld), s/t/mean/inv/slope
    const float* W;       // layer l's weight, row-major C x CI (W[c * ldw + i])
    int ldw;
    int M;
    float* dA;            // M x CI, row stride ldd
    int ldd;
    double* bstats;       // [2][CI][gridDim.x]: layer l-1's (sum dy, sum dy*xhat) per block
    float* part;          // [gridDim.x][C][kp]: this block's dW partial (columns < kp)
    float* pdb;           // [gridDim.x][C]: this block's db partial (or null)
    int kx;               // valid input columns (< CI: a stack's first layer, its raw input zero-padded)
    int kp;               // dW row length (= kx)
};

__device__ __forceinline__ int acc_row_of(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// 256 threads, two blocks per CU: while one block stages its next tile (all of a tile's
// loads in flight per thread chunk), the other runs its MFMAs.  (A 512-thread producer /
// consumer variant with a double-buffered LDS tile, one block per CU, measured slower:
// 145 vs 117 us isolated on the FP1 shape -- one consumer wave per SIMD does not keep the
// MFMA pipe fed through its LDS fragment reads.)
// DA = false: weight gradient only (a stack's first layer, whose input needs no gradient):
// the input is the plain raw rows (q.s == null: identity, no BN), kx <= CI columns.
// WIDE: the wide layers (C + CI > 96) at ONE block per CU (one wave per SIMD, up to 512 VGPRs):
// the next tile's raw loads are then held in registers under the current tile's MFMAs as on
// the narrow layers, instead of being staged in chunks after the barrier.
// waves per block: the 128 x 128 instance (the widest, MFMA-heaviest: 256 MFMAs per wave and tile on
// four waves) runs eight waves -- two per SIMD, so one wave's staging, epilogue and LDS reads hide
// under the other's MFMAs -- each with one dA row tile and two dW tiles (<= 256 registers;
// profiles/r05_ab_fused_wide_waves.txt).  (The engine runs its 128-wide BNBWD layers on the LDS-DMA
// ring kernel instead, bwd_ring.hip; this instance serves the PLAIN / POOLBWD operands.)
__host__ __device__ constexpr int fb_waves(int C, int CI, bool da) { return da && C == 128 && CI == 128 ? 8 : 4; }

template <int C, int CI, int XM, bool DA, bool WIDE = false>
__global__ __launch_bounds__(64 * fb_waves(C, CI, DA), WIDE ? 1 : 2) void fused_bwd_kernel(
    FusedBwdArgs f) {
    constexpr int NWV = fb_waves(C, CI, DA), NT = 64 * NWV;
    // WL: W (C x CI) staged once in LDS and its B fragments read per MFMA, instead of C / 2 registers
    // per lane for the whole launch (the eight-wave instance: 256 registers per wave)
    // (W from LDS at three blocks per CU for the narrow instances measured neutral,
    // profiles/r05_ab_fused_wlds_occupancy.txt)
    constexpr bool WL = DA && NWV == 8;
    constexpr int BM = FB_BM;
    constexpr int ZS = C + 2;                  // row stride = 2 (mod 64) banks: the dA fragment reads
                                               // (32 rows x 2 k) hit 64 distinct banks
    constexpr int XS = CI + 4;                 // float4-aligned rows (row reads only)
    constexpr int NIT = CI / 32, NCT = C / 32;
    constexpr int TW = NCT * NIT;              // 32 x 32 tiles of dW
    // SPLIT (CI = 32 with a data gradient): the dA strip has only two 32-row tiles, so waves 0, 1
    // take dA and waves 2, 3 take every dW tile -- C / 2 MFMAs per wave on every SIMD (round 4 gave
    // all four waves a share of dW, so waves 0, 1 carried dA + dW: 1.5x the MFMA time per tile on
    // two SIMDs while the other two idled)
    constexpr bool SPLIT = DA && NIT == 1;
    constexpr int DWW = SPLIT ? 2 : NWV;       // waves sharing the dW tiles
    constexpr int WPT = TW >= DWW ? TW / DWW : 1;  // dW tiles per wave
    constexpr int WR = TW >= DWW ? 1 : DWW / TW;   // waves splitting one dW tile's rows
    constexpr int NRT = NIT == 4 && NWV == 4 ? 2 : 1;   // dA row tiles per wave
    static_assert(C % 32 == 0 && CI % 32 == 0 && C <= 128 && CI <= 128, "fused backward widths");
    __shared__ __attribute__((aligned(16))) float Zs[BM * ZS];
    __shared__ __attribute__((aligned(16))) float Xs[BM * XS];
    __shared__ double red[2][NWV][32];
    __shared__ float Ws[WL ? C * CI : 1];
    __shared__ float wred[WR > 1 ? (WR - 1) * TW * 1024 : 1];   // per (row subset, tile)

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5, l32 = lane & 31;

    // ---- data-gradient assignment: column strip a_ct, row tiles a_rt0 .. a_rt0 + NRT - 1
    const int a_ct = NIT == 4 ? (w & 3) : (NIT == 2 ? (w & 1) : 0);
    const int a_rt0 = NIT == 4 ? (NWV == 8 ? (w >> 2) : 0) : (NIT == 2 ? (w >> 1) : (w & 1));
    const bool a_on = DA && (NIT >= 2 || w < 2);
    const int a_col = a_ct * 32 + l32;
    float wf[DA && !WL ? C / 2 : 1];           // wf[j] = W[2j + h][a_col]: B fragments of every k step
    float es = 0.f, et = 0.f, em = 0.f, ei = 0.f;
    if constexpr (DA) {
#pragma unroll
        for (int j = 0; j < (WL ? 0 : C / 2); ++j) wf[j] = f.W[(size_t)(2 * j + h) * f.ldw + a_col];
        if (WL)
            for (int e = tid; e < C * CI; e += NT) Ws[e] = f.W[(size_t)(e / CI) * f.ldw + e % CI];
        // previous layer's BN at this lane's dA column (BN-backward epilogue)
        es = f.q.s[a_col]; et = f.q.t[a_col]; em = f.q.mean[a_col]; ei = f.q.inv[a_col];
    }
    const float qslope = DA ? f.q.slope : 1.f;

    // ---- weight-gradient assignment over the DWW dW waves (index wd): tiles t = ct_c * NIT + ct_i.
    // TW >= DWW: wave wd takes t = wd + DWW u (all share ct_i = wd % NIT); TW < DWW: wave wd takes
    // t = wd % TW over the row pairs p = wd / TW (mod WR).  wsub < 0: no dW on this wave (SPLIT)
    const bool dw_on = !SPLIT || w >= 2;
    const int wd = SPLIT ? (w >= 2 ? w - 2 : 0) : w;
    const int t_base = TW >= DWW ? wd : (wd % TW);
    const int w_i = t_base % NIT;
    const int wsub = !dw_on ? -1 : (TW >= DWW ? 0 : wd / TW);
    const int b_col = w_i * 32 + l32;
    const float bs = DA ? f.q.s[b_col] : 1.f, bt = DA ? f.q.t[b_col] : 0.f;   // !DA: identity

    f32x16 accW[WPT];
#pragma unroll
    for (int u = 0; u < WPT; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) accW[u][r] = 0.f;
    double s1 = 0.0, s2 = 0.0;
    float dbs = 0.f;

    const int M = f.M;
    const int tiles = (M + BM - 1) / BM;
    // staging: thread = one dZ channel quad over rows r0 + j*RPP (one coefficient quad) and
    // one raw-input quad over rows s0 + j*RPI
    constexpr int CQ = C / 4, RPP = NT / CQ, NJ = BM / RPP;
    constexpr int IQ = CI / 4, RPI = NT / IQ, NJX = BM / RPI;
    // PF: the narrow layers (SA1-sized, HBM-bound) hold the NEXT tile's raw loads in registers
    // while the current tile's MFMAs run; the wide ones stage in chunks after the barrier
    constexpr bool PF = C + CI <= 96 || WIDE;
    constexpr int CH = PF ? NJ : (NJ < 4 ? NJ : 4);      // rows in flight per chunk
    const int cq = tid % CQ, r0 = tid / CQ;
    const int iq = tid % IQ, s0 = tid / IQ;
    const bool xin = DA || 4 * iq < f.kx;                // !DA: columns past the raw input are 0
    Quad qd;
    load_quad<XM>(f.x, 4 * cq, C, qd);
    float4 pv[CH], pz[CH], px[NJX];
    unsigned pa[CH];
    auto issue_dz = [&](int m0, int j0) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < CH; ++j)
            load_raw<XM>(f.x, min(m0 + r0 + (j0 + j) * RPP, M - 1), 4 * cq, pv[j], pz[j], pa[j]);
    };
    // db: this thread's column-quad sums of dZ over the rows it stages (all tiles), added over the
    // RPP threads of its quad at the end -- a fixed order, no per-tile LDS column walk
    float4 dbv = make_float4(0.f, 0.f, 0.f, 0.f);
    auto commit_dz = [&](int m0, int j0) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            const int r = r0 + (j0 + j) * RPP;
            float4 o = xform4<XM>(f.x, pv[j], pz[j], pa[j], min(m0 + r, M - 1), qd, 4 * cq, C);
            if (m0 + r >= M) o = make_float4(0.f, 0.f, 0.f, 0.f);
            float* d = &Zs[r * ZS + 4 * cq];
            d[0] = o.x; d[1] = o.y; d[2] = o.z; d[3] = o.w;
            dbv.x += o.x; dbv.y += o.y; dbv.z += o.z; dbv.w += o.w;
        }
    };
    auto issue_x = [&](int m0) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < NJX; ++j) {
            const int rc = min(m0 + s0 + j * RPI, M - 1);
            PCS_DCHECK(!xin || f.q.rows <= 0 || (rc >= 0 && rc < f.q.rows && 4 * iq + 4 <= ((f.q.cols + 3) & ~3)),
                       "fused backward input row %d quad %d outside %d x %d", rc, iq, f.q.rows, f.q.cols);
            px[j] = xin ? *reinterpret_cast<const float4*>(f.q.data + (size_t)rc * f.q.ld + 4 * iq)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto commit_x = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < NJX; ++j) *reinterpret_cast<float4*>(&Xs[(s0 + j * RPI) * XS + 4 * iq]) = px[j];
    };
    if (PF && (int)blockIdx.x < tiles) {
        issue_dz((int)blockIdx.x * BM, 0);
        issue_x((int)blockIdx.x * BM);
    }
    for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
        const int m0 = t * BM;
        __syncthreads();                       // the previous tile's reads of Zs / Xs are done
        if constexpr (PF) {
            commit_dz(m0, 0);
            commit_x();
        } else {
#pragma unroll
            for (int j0 = 0; j0 < NJ; j0 += CH) {
                issue_dz(m0, j0);
                commit_dz(m0, j0);
            }
            issue_x(m0);
            commit_x();
        }
        __syncthreads();
        if (PF && t + (int)gridDim.x < tiles) {          // next tile's loads fly under this tile's MFMAs
            issue_dz(m0 + (int)gridDim.x * BM, 0);
            issue_x(m0 + (int)gridDim.x * BM);
        }

        // ---- dA tile(s) = Zs . W
        if (DA && a_on) {
            f32x16 accA[NRT];
#pragma unroll
            for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
                for (int r = 0; r < 16; ++r) accA[rt][r] = 0.f;
            // A fragments read PD k-steps ahead of their MFMAs (a static register ring: the loop
            // is fully unrolled), so the LDS latency hides behind PD * NRT MFMAs
            constexpr int PD = 4;
            float ar[PD][NRT];
            auto afrag = [&](int j, int sl) __attribute__((always_inline)) {
#pragma unroll
                for (int rt = 0; rt < NRT; ++rt) ar[sl][rt] = Zs[((a_rt0 + rt) * 32 + l32) * ZS + 2 * j + h];
            };
#pragma unroll
            for (int j = 0; j < PD; ++j) afrag(j, j);
#pragma unroll
            for (int j = 0; j < C / 2; ++j) {
                float a[NRT];
#pragma unroll
                for (int rt = 0; rt < NRT; ++rt) a[rt] = ar[j % PD][rt];
                if (j + PD < C / 2) afrag(j + PD, j % PD);
#pragma unroll
                for (int rt = 0; rt < NRT; ++rt)
                    accA[rt] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                        a[rt], WL ? Ws[(2 * j + h) * CI + a_col] : wf[WL ? 0 : j], accA[rt], 0, 0, 0);
            }
#pragma unroll
            for (int rt = 0; rt < NRT; ++rt) {
                const int rb = (a_rt0 + rt) * 32;
                // the 16 z of this lane's rows read up front (one LDS round trip, not 16); rows
                // past M (zero dZ, clamped z) are masked out of the store and the sums, no branch
                float zz[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) zz[r] = Xs[(rb + acc_row_of(r, h)) * XS + a_col];
                const bool full = m0 + rb + 32 <= M;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = rb + acc_row_of(r, h);
                    const float v = accA[rt][r];
                    const bool ok = full || m0 + row < M;
                    if (ok) f.dA[(size_t)(m0 + row) * f.ldd + a_col] = v;
                    const float dy = v * dact_f(zz[r] * es + et, 0, qslope);
                    const float xh = (zz[r] - em) * ei;
                    s1 += ok ? (double)dy : 0.0;
                    s2 += ok ? (double)dy * (double)xh : 0.0;
                }
            }
        }
        // ---- dW += Zs^T . act(Xs*s + t): the fragments of row pair pq + 1 are read while row pair
        // pq's MFMAs run (two register slots), so no MFMA waits on its own LDS reads
        if (dw_on) {
            constexpr int NP = BM / 2 / WR;
            float xr[2], za[2][WPT];
            auto frag = [&](int pq, int sl) __attribute__((always_inline)) {
                const int r = 2 * (pq * WR + wsub) + h;
                xr[sl] = Xs[r * XS + b_col];
#pragma unroll
                for (int u = 0; u < WPT; ++u) za[sl][u] = Zs[r * ZS + ((t_base + DWW * u) / NIT) * 32 + l32];
            };
            frag(0, 0);
#pragma unroll
            for (int pq = 0; pq < NP; ++pq) {
                const int sl = pq & 1;
                if (pq + 1 < NP) frag(pq + 1, sl ^ 1);
                const float b = act_f(xr[sl] * bs + bt, 0, qslope);
#pragma unroll
                for (int u = 0; u < WPT; ++u)
                    accW[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(za[sl][u], b, accW[u], 0, 0, 0);
            }
        }
    }
    // db partials: the RPP threads of each column quad, added in thread order (Zs is free now)
    __syncthreads();
    if (f.pdb) {
        *reinterpret_cast<float4*>(&Zs[r0 * C + 4 * cq]) = dbv;
        __syncthreads();
        if (tid < C) {
            for (int j = 0; j < RPP; ++j) dbs += Zs[j * C + tid];
        }
    }

    // ---- previous layer's BN-backward partials: both lane halves, then the waves of a strip
    s1 += __shfl_xor(s1, 32);
    s2 += __shfl_xor(s2, 32);
    if (lane < 32) {
        red[0][w][l32] = a_on ? s1 : 0.0;
        red[1][w][l32] = a_on ? s2 : 0.0;
    }
    __syncthreads();
    if (DA && tid < CI) {
        const int ct = tid / 32, lc = tid % 32;
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int v = 0; v < NWV; ++v) {
            const int vct = NIT == 4 ? (v & 3) : (NIT == 2 ? (v & 1) : 0);
            const bool von = NIT >= 2 || v < 2;
            if (von && vct == ct) { a += red[0][v][lc]; b += red[1][v][lc]; }
        }
        f.bstats[(size_t)tid * gridDim.x + blockIdx.x] = a;
        f.bstats[((size_t)CI + tid) * gridDim.x + blockIdx.x] = b;
    }
    if (f.pdb && tid < C) f.pdb[(size_t)blockIdx.x * C + tid] = dbs;
    // ---- dW partial tile(s): waves splitting one tile's rows add theirs in wave order
    float* part = f.part + (size_t)blockIdx.x * C * f.kp;
    if constexpr (WR > 1) {
        if (wsub > 0) {
#pragma unroll
            for (int r = 0; r < 16; ++r) wred[((wsub - 1) * TW + t_base) * 1024 + r * 64 + lane] = accW[0][r];
        }
        __syncthreads();
        if (wsub == 0) {
#pragma unroll
            for (int s = 1; s < WR; ++s)
#pragma unroll
                for (int r = 0; r < 16; ++r) accW[0][r] += wred[((s - 1) * TW + t_base) * 1024 + r * 64 + lane];
        }
    }
    if (wsub == 0) {
#pragma unroll
        for (int u = 0; u < WPT; ++u) {
            const int tt = t_base + DWW * u;
            const int c0 = (tt / NIT) * 32, i0 = (tt % NIT) * 32;
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (DA || i0 + l32 < f.kp) part[(size_t)(c0 + acc_row_of(r, h)) * f.kp + i0 + l32] = accW[u][r];
        }
    }
}

template <int C, int CI>
static void launch_fused(dim3 grid, hipStream_t st, const FusedBwdArgs& a) {
    constexpr bool W = C + CI > 96;
    constexpr int NT = 64 * fb_waves(C, CI, true);
    switch (a.x.mode) {
    case OP_PLAIN: hipLaunchKernelGGL((fused_bwd_kernel<C, CI, OP_PLAIN, true, W>), grid, dim3(NT), 0, st, a); break;
    case OP_BNBWD: hipLaunchKernelGGL((fused_bwd_kernel<C, CI, OP_BNBWD, true, W>), grid, dim3(NT), 0, st, a); break;
    default: hipLaunchKernelGGL((fused_bwd_kernel<C, CI, OP_POOLBWD, true, W>), grid, dim3(NT), 0, st, a); break;
    }
}

template <int C>
static void launch_fused_ci(int CI, dim3 grid, hipStream_t st, const FusedBwdArgs& a) {
    if (CI == 32) launch_fused<C, 32>(grid, st, a);
    else if (CI == 64) launch_fused<C, 64>(grid, st, a);
    else launch_fused<C, 128>(grid, st, a);
}

// weight gradient only, input width <= 32 (a stack's first layer over raw rows)
template <int C>
static void launch_wgrad_only(dim3 grid, hipStream_t st, const FusedBwdArgs& a) {
    switch (a.x.mode) {
    case OP_PLAIN: hipLaunchKernelGGL((fused_bwd_kernel<C, 32, OP_PLAIN, false>), grid, dim3(256), 0, st, a); break;
    case OP_BNBWD: hipLaunchKernelGGL((fused_bwd_kernel<C, 32, OP_BNBWD, false>), grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((fused_bwd_kernel<C, 32, OP_POOLBWD, false>), grid, dim3(256), 0, st, a); break;
    }
}

static bool fb_width(int c) { return c == 32 || c == 64 || c == 128; }

// the per-layer policy (pcs_mlp_layer.bwd_fuse): by default only layers over >= 2^19 rows (SA1:
// HBM-bound, the fused launch beats the dgrad + lane wgrad pair there); on the 128-wide layers
// the overlapped pair is faster
bool fused_bwd_wanted(int policy, int M) {
    if (policy == PCS_BWD_FUSE_OFF) return false;
    return policy == PCS_BWD_FUSE_ALL || M >= (1 << 19);
}

// shape / operand eligibility of the fused kernel (the policy is the caller's decision)
bool fused_bwd_ok(int M, int C, int CI, int ldw, const pcs_operand* x, const pcs_operand* q) {
    if (M < 4 * FB_BM || !fb_width(C) || !fb_width(CI) || ldw % 4 != 0 || ldw < CI) return false;
    if (!x || !q || x->mode == PCS_OP_BNACT || x->ld % 4 != 0 || x->ld < C) return false;
    if (x->mode == PCS_OP_POOLBWD && (x->pool_k < 1 || M % x->pool_k != 0)) return false;
    if (x->mode != PCS_OP_PLAIN && x->ldz % 4 != 0) return false;
    return q->data && q->ld % 4 == 0 && q->ld >= CI && q->s && q->t && q->mean && q->inv;
}

// the kernel instance for (C, CI, operand mode, da), as the launchers pick it
template <int C, int CI, bool DA>
static const void* fb_kernel_ci(int xm) {
    constexpr bool W = DA && C + CI > 96;
    if (xm == OP_PLAIN) return reinterpret_cast<const void*>(&fused_bwd_kernel<C, CI, OP_PLAIN, DA, W>);
    if (xm == OP_BNBWD) return reinterpret_cast<const void*>(&fused_bwd_kernel<C, CI, OP_BNBWD, DA, W>);
    return reinterpret_cast<const void*>(&fused_bwd_kernel<C, CI, OP_POOLBWD, DA, W>);
}
template <int C>
static const void* fb_kernel_c(int CI, int xm, bool da) {
    if (!da) return fb_kernel_ci<C, 32, false>(xm);
    if (CI == 32) return fb_kernel_ci<C, 32, true>(xm);
    if (CI == 64) return fb_kernel_ci<C, 64, true>(xm);
    return fb_kernel_ci<C, 128, true>(xm);
}
static const void* fb_kernel(int C, int CI, int xm, bool da) {
    return C == 32 ? fb_kernel_c<32>(CI, xm, da) : (C == 64 ? fb_kernel_c<64>(CI, xm, da) : fb_kernel_c<128>(CI, xm, da));
}

// persistent grid: as many blocks per CU as are resident at once (the occupancy query: VGPRs and
// LDS of the instance; the wide layers run one wave per SIMD).  xm = the operand mode of the launch;
// xm < 0 (workspace sizing): the largest grid over the modes.  The grid is the number of
// BN-backward partials, which the caller's finalize reads (engine.hip passes the launch's mode).
// (Round 4 used the smallest grid over the modes for every launch: SA1's middle layer, BNBWD at
// 164 VGPRs, ran 2 blocks per CU where 3 are resident.)
int fused_bwd_grid(int M, int C, int CI, bool da, int xm) {
    static int occ[3][3][2][3];                // [C][CI][da][mode], 0 = not queried
    const int ci = C == 32 ? 0 : (C == 64 ? 1 : 2), ii = CI == 32 ? 0 : (CI == 64 ? 1 : 2);
    const int modes[3] = {(int)OP_PLAIN, (int)OP_BNBWD, (int)OP_POOLBWD};
    int hi = 1, mine = 0;
    for (int k = 0; k < 3; ++k) {
        int& n = occ[ci][ii][da ? 1 : 0][k];
        if (n == 0) {
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fb_kernel(C, CI, modes[k], da), 64 * fb_waves(C, CI, da),
                                                             0) != hipSuccess)
                n = 1;
            n = std::min(std::max(n, 1), 4);
        }
        hi = std::max(hi, n);
        if (modes[k] == xm) mine = n;
    }
    const int per_cu = xm < 0 || mine == 0 ? hi : mine;
    const int tiles = (M + FB_BM - 1) / FB_BM;
    return std::min(tiles, 256 * per_cu);
}

size_t fused_bwd_ws_bytes(int M, int C, int CI) {
    return (size_t)fused_bwd_grid(M, C, CI, true, -1) * ((size_t)C * CI + C) * sizeof(float) + 256;
}

int fused_bwd(const pcs_operand* x, int C, const pcs_operand* q, int CI, const float* W, int ldw, int M, float* dA,
              int ldd, double* bstats, float* dW, float* db, void* ws, size_t ws_bytes, hipStream_t st) {
    PCS_CHECK_ARG(fused_bwd_ok(M, C, CI, ldw, x, q), "fused_bwd: unsupported shape C=%d CI=%d M=%d", C, CI, M);
    PCS_CHECK_ARG(dA && ldd >= CI && ldd % 4 == 0 && bstats && dW && W, "fused_bwd: bad output arguments");
    PCS_CHECK_ARG(ws && ws_bytes >= fused_bwd_ws_bytes(M, C, CI), "fused_bwd: workspace too small");
    const int G = fused_bwd_grid(M, C, CI, true, x->mode);
    float* part = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
    float* pdb = db ? part + (size_t)G * C * CI : nullptr;
    FusedBwdArgs a{to_dev_operand(x, M, C), to_dev_operand(q, M, CI), W, ldw, M, dA, ldd, bstats, part, pdb, CI, CI};
    const dim3 grid(G);
    auto launch = [=]() {
        if (C == 32) launch_fused_ci<32>(CI, grid, st, a);
        else if (C == 64) launch_fused_ci<64>(CI, grid, st, a);
        else launch_fused_ci<128>(CI, grid, st, a);
    };
    int probe = -1;
    if (probe_enabled()) {
        char nm[80];
        snprintf(nm, sizeof nm, "pcs::fused_bwd_kernel<%d, %d, %d>", C, CI, x->mode);
        const double xb = x->mode == PCS_OP_POOLBWD ? 4.0 * M * C + 5.0 * (double)(M / x->pool_k) * C
                                                   : 4.0 * M * C * (x->mode == PCS_OP_BNBWD ? 2 : 1);
        probe = probe_start(nm, 4.0 * M * C * CI, xb + 8.0 * M * CI, st, launch);
    }
    launch();
    probe_stop(probe, st);
    wgrad_reduce_launch(part, G, (long long)C * CI, dW, pdb, C, db, st);
    return launch_status("fused_bwd");
}

bool fused_wgrad_ok(int M, int C, int kin, int ldx, const pcs_operand* x) {
    if (M < 4 * FB_BM || !fb_width(C) || kin < 1 || kin > 32 || ldx % 4 != 0 || ldx < kin) return false;
    if (!x || x->mode == PCS_OP_BNACT || x->ld % 4 != 0 || x->ld < C) return false;
    if (x->mode == PCS_OP_POOLBWD && (x->pool_k < 1 || M % x->pool_k != 0)) return false;
    return x->mode == PCS_OP_PLAIN || x->ldz % 4 == 0;
}

size_t fused_wgrad_ws_bytes(int M, int C, int kin) {
    return (size_t)fused_bwd_grid(M, C, 32, false, -1) * ((size_t)C * kin + C) * sizeof(float) + 256;
}

int fused_wgrad(const pcs_operand* x, int C, const float* X, int ldx, int kin, int M, float* dW, float* db, void* ws,
                size_t ws_bytes, hipStream_t st) {
    PCS_CHECK_ARG(fused_wgrad_ok(M, C, kin, ldx, x) && X && dW, "fused_wgrad: unsupported C=%d kin=%d M=%d", C, kin, M);
    PCS_CHECK_ARG(ws && ws_bytes >= fused_wgrad_ws_bytes(M, C, kin), "fused_wgrad: workspace too small");
    const int G = fused_bwd_grid(M, C, 32, false, x->mode);
    float* part = reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(ws) + 255) & ~uintptr_t(255));
    float* pdb = db ? part + (size_t)G * C * kin : nullptr;
    Operand q{};
    q.data = X; q.ld = ldx; q.slope = 1.f;
    q.rows = M; q.cols = kin;
    FusedBwdArgs a{to_dev_operand(x, M, C), q, nullptr, 0, M, nullptr, 0, nullptr, part, pdb, kin, kin};
    const dim3 grid(G);
    auto launch = [=]() {
        if (C == 32) launch_wgrad_only<32>(grid, st, a);
        else if (C == 64) launch_wgrad_only<64>(grid, st, a);
        else launch_wgrad_only<128>(grid, st, a);
    };
    int probe = -1;
    if (probe_enabled()) {
        char nm[80];
        snprintf(nm, sizeof nm, "pcs::fused_bwd_kernel<%d, 32, %d, false>", C, x->mode);
        const double xb = x->mode == PCS_OP_POOLBWD ? 4.0 * M * C + 5.0 * (double)(M / x->pool_k) * C
                                                   : 4.0 * M * C * (x->mode == PCS_OP_BNBWD ? 2 : 1);
        probe = probe_start(nm, 2.0 * M * C * kin, xb + 4.0 * M * kin, st, launch);
    }
    launch();
    probe_stop(probe, st);
    wgrad_reduce_launch(part, G, (long long)C * kin, dW, pdb, C, db, st);
    return launch_status("fused_wgrad");
}

}  // namespace pcs
