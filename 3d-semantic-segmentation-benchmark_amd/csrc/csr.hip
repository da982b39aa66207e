// Inverse neighbour maps and atomic-free gather backward for group / interpolate.
//
// The backward of a neighbour gather (models/utils/common.py:64-65 `group`,
// :120-122 `interpolate`) is a scatter-add into the source points.  Instead of
// fp32 atomics (one per gathered element), the geometry stage -- which depends on
// coordinates only and runs on the side stream, off the critical path -- also
// builds the INVERSE map of each neighbour table: for every source point, the
// list of gather slots that read it (CSR: offsets + entries).  The backward then
// gathers: one thread per (source point, channel) sums its slots' gradients.
//
// Build (clouds of <= 8192 targets): a chunked stable counting sort over many workgroups,
// lists ascending by construction (inverse_count / inverse_scan / inverse_rank below).
// Larger clouds (PointNeXt's first ball query, 24 576 targets): one workgroup per cloud,
// one launch per map.  Every slot of cloud b
// reads a point of cloud b, so cloud b's entries are exactly positions
// [b*per_batch, (b+1)*per_batch) and the clouds are independent: LDS histogram of
// the cloud's targets -> in-LDS exclusive scan -> LDS-atomic scatter of the slots
// into scratch (arbitrary order inside a list).  A second kernel sorts every list, one
// wave per list: a slot's position is the number of the list's slots below it (lists
// average ~8 entries; the longest, ball-query padding hubs, a few hundred, take
// ceil(L/64) * L wave steps).  Every list ends up in ascending slot order whatever the
// scatter's order, and the consumers walk a list in that order (fp64 accumulation),
// so the backward is bitwise reproducible.
#include <cstdlib>

#include "pcs_common.hpp"

namespace pcs {

constexpr int kInvThreads = 1024;
constexpr int kInvLdsTargets = 32768;   // 128 KB of LDS counters; larger clouds count in global memory

// block-wide exclusive scan of cnt[0, n) in place (kInvThreads threads); returns the total
__device__ int block_exclusive_scan(int* cnt, int n, int* wsum) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int per = (n + kInvThreads - 1) / kInvThreads;
    const int a = tid * per, z = min(a + per, n);
    int local = 0;
    for (int i = a; i < z; ++i) local += cnt[i];
    int incl = local;   // inclusive wave scan
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d, 64);
        if (lane >= d) incl += v;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    if (tid < 64) {
        int w = tid < kInvThreads / 64 ? wsum[tid] : 0;
        int wi = w;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(wi, d, 64);
            if (tid >= d) wi += v;
        }
        if (tid < kInvThreads / 64) wsum[tid] = wi - w;     // exclusive wave offsets
        if (tid == kInvThreads / 64 - 1) wsum[kInvThreads / 64] = wi;
    }
    __syncthreads();
    int run = wsum[wv] + incl - local;
    for (int i = a; i < z; ++i) {
        const int c = cnt[i];
        cnt[i] = run;
        run += c;
    }
    const int total = wsum[kInvThreads / 64];
    __syncthreads();
    return total;
}

template <bool kLds>
__global__ __launch_bounds__(kInvThreads) void inverse_index_kernel(const int32_t* __restrict__ idx, int per_batch,
                                                                    int targets, int nbatch,
                                                                    int32_t* __restrict__ offsets,
                                                                    int* gcnt, int32_t* __restrict__ scratch) {
    extern __shared__ int smem[];
    int* wsum = smem;                                   // kInvThreads/64 + 1
    int* cnt = kLds ? smem + 32 : gcnt + (size_t)blockIdx.x * targets;
    const int b = blockIdx.x, tid = threadIdx.x;
    const int32_t* id = idx + (size_t)b * per_batch;
    const long long base = (long long)b * per_batch;
    for (int t = tid; t < targets; t += kInvThreads) cnt[t] = 0;
    __syncthreads();
    for (int s = tid; s < per_batch; s += kInvThreads) {
        const unsigned t = (unsigned)id[s];
        if (t < (unsigned)targets) atomicAdd(&cnt[t], 1);
    }
    __syncthreads();
    block_exclusive_scan(cnt, targets, wsum);
    int32_t* off = offsets + (size_t)b * targets;
    for (int t = tid; t < targets; t += kInvThreads) off[t] = (int32_t)(base + cnt[t]);
    if (b == nbatch - 1 && tid == 0) offsets[(size_t)nbatch * targets] = (int32_t)(base + per_batch);
    __syncthreads();
    // scatter (list order = atomic arrival order)
    int32_t* scr = scratch + base;
    for (int s = tid; s < per_batch; s += kInvThreads) {
        const unsigned t = (unsigned)id[s];
        if (t < (unsigned)targets) scr[atomicAdd(&cnt[t], 1)] = (int32_t)(base + s);
    }
}

// entries[off[T] ...] = list T's slots in ascending order, one wave per list.  Short lists
// (<= 64, nearly all of them): each lane's rank = the number of the list's slots below its
// own, counted over v_readlane broadcasts.  Longer lists (ball-query padding hubs, a few
// hundred; kNN hubs of zero-padded clouds, thousands): runs of kSortLds slots are bitonic-
// sorted in the wave's LDS slice; a single run is the answer, several runs are merged by
// rank (own index in the run + a binary search in every other run).  O(L log^2 L) per list.
constexpr int kSortLds = 1024;

__device__ inline void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// bitonic sort of v[0, P) (P a power of two >= 128) by one wave
__device__ void wave_bitonic(int* v, int P, int lane) {
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = lane; i < P / 2; i += 64) {
                const int lo = 2 * i - (i & (j - 1)), hi = lo + j;
                const int x = v[lo], y = v[hi];
                if ((x > y) == ((lo & k) == 0)) { v[lo] = y; v[hi] = x; }
            }
            wave_sync();
        }
}

__global__ __launch_bounds__(256) void inverse_sort_kernel(const int32_t* __restrict__ off, int32_t* scratch,
                                                           int n_lists, int32_t* __restrict__ entries) {
    __shared__ int lds[4][kSortLds];
    const int w = threadIdx.x >> 6;
    const int T = blockIdx.x * 4 + w;
    const int lane = threadIdx.x & 63;
    if (T >= n_lists) return;
    const int a = off[T], z = off[T + 1], L = z - a;
    if (L <= 64) {
        const int v = lane < L ? scratch[a + lane] : 0;
        int r = 0;
        for (int e = 0; e < L; ++e) r += __builtin_amdgcn_readlane(v, e) < v;
        if (lane < L) entries[a + r] = v;
        return;
    }
    int* v = lds[w];
    for (int r0 = a; r0 < z; r0 += kSortLds) {          // sort each run in LDS
        const int n = min(kSortLds, z - r0);
        int P = 128;
        while (P < n) P <<= 1;
        for (int i = lane; i < P; i += 64) v[i] = i < n ? scratch[r0 + i] : INT_MAX;
        wave_sync();
        wave_bitonic(v, P, lane);
        int32_t* dst = L <= kSortLds ? entries : scratch;
        for (int i = lane; i < n; i += 64) dst[r0 + i] = v[i];
        wave_sync();
    }
    if (L <= kSortLds) return;
    for (int i = a + lane; i < z; i += 64) {             // merge the sorted runs by rank
        const int x = scratch[i];
        const int mine = (i - a) / kSortLds;
        int rank = (i - a) - mine * kSortLds;
        for (int r0 = a, run = 0; r0 < z; r0 += kSortLds, ++run) {
            if (run == mine) continue;
            int lo = r0, hi = min(r0 + kSortLds, z);     // count of run elements < x
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (scratch[mid] < x) lo = mid + 1;
                else hi = mid;
            }
            rank += lo - r0;
        }
        entries[a + rank] = x;
    }
}

// ---------------------------------------------------------------- chunked stable counting sort
// The map of clouds with <= 8192 targets (every PointNet++ / DGCNN map and all but PointNeXt's
// first ball query) is a stable counting sort of the slots by target, spread over many
// workgroups and free of atomics on the ordering path, so every list comes out ascending with
// no sort pass.  Clouds of more than one chunk:
//   1. inverse_count_kernel (chunk c, cloud b): LDS histogram of chunk c's targets -> hist[b][c][t];
//   2. inverse_scan_kernel (cloud b, 1024 threads, one target per thread and slice of 1024):
//      offsets[b][t] = b*per + the totals of the earlier targets (block scan), and in place
//      hist[b][c][t] := offsets[b][t] + the counts of t in chunks < c (chunk c's list base).
//      Every hist access is a coalesced row of targets; each column is walked once;
//   3. inverse_rank_kernel (chunk c, cloud b): each wave owns a contiguous quarter (half) of the
//      chunk and counts it per target in LDS; per-wave bases = the chunk's base + the counts of
//      the earlier waves; then each wave walks its slots in order, 64 at a time: the lanes
//      reading the same target are found by a ballot over the target's bits (a match), a
//      slot's position is its wave base + the number of matching lanes below it, and the
//      group's last lane advances the base.
// A cloud of one chunk skips 1-2: the rank kernel scans its own LDS counts into the offsets.
// Slot order = list order: ascending, deterministic.
// BATCHED: the three kernels take up to kInvBatch maps (blockIdx.z = map), so a geometry plan's
// 8 PointNet++ maps or a DGCNN forward's 4 kNN maps cost 3 launches, not 3 per map (the small
// maps are launch-bound: 10-14 us each alone).  Each map has its own hist region.
// (Round 4 first fused the scan into the rank kernel for every cloud: each of a cloud's chunks
// then re-read all its chunks' counts -- quadratic in the chunk count, 0.98 ms per DGCNN map.)
// a chunk holds two slots per target (>= 4096): the per-target passes of a rank block (LDS
// counter init, bases) are paid once per 2 x targets slots.  Round 4, batched as the models call
// it (scripts/inverse_ab.py): PointNet++ 8 maps 90 -> 70 us, DGCNN 4 maps 227 -> 223 us; one
// slot per target, or chunks of >= 8192 / 16384 slots, measured slower
constexpr int kChunkMin = 4096, kChunkPerTarget = 2, kRankMaxTargets = 8192, kInvBatch = 24;

static int rank_chunk(int targets) { return std::max(kChunkMin, (targets + 255) / 256 * 256 * kChunkPerTarget); }

struct InvMap {
    const int32_t* idx;
    int32_t* offsets;
    int32_t* entries;
    int* hist;                 // [B][nch][targets] (nch > 1)
    int per, targets, chunk, nch, nbits;
};
struct InvBatch {
    InvMap m[kInvBatch];
};

__global__ __launch_bounds__(256) void inverse_count_kernel(const InvBatch bat, int nbatch) {
    extern __shared__ int cnt[];
    const InvMap& m = bat.m[blockIdx.z];
    const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, targets = m.targets;
    if (m.nch <= 1 || c >= m.nch) return;
    for (int t = tid; t < targets; t += 256) cnt[t] = 0;
    __syncthreads();
    const int32_t* id = m.idx + (size_t)b * m.per;
    const int s1 = min(m.per, (c + 1) * m.chunk);
    for (int s = c * m.chunk + tid; s < s1; s += 256) {
        const unsigned t = (unsigned)id[s];
        if (t < (unsigned)targets) atomicAdd(&cnt[t], 1);     // counts: order-free
    }
    __syncthreads();
    int* h = m.hist + ((size_t)b * m.nch + c) * targets;
    for (int t = tid; t < targets; t += 256) h[t] = cnt[t];
    (void)nbatch;
}

// exclusive scan of one value per thread over a 1024-thread block; *all = the block's total
__device__ __forceinline__ int block_scan_1024(int v, int* wsum, int* all) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int u = __shfl_up(incl, d, 64);
        if (lane >= d) incl += u;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
        const int x = wsum[w];
        pre += w < wv ? x : 0;
        tot += x;
    }
    __syncthreads();                                     // wsum is reused by the next call
    *all = tot;
    return pre + incl - v;
}

__global__ __launch_bounds__(1024) void inverse_scan_kernel(const InvBatch bat, int nbatch) {
    __shared__ int wsum[16];
    const InvMap& m = bat.m[blockIdx.y];
    if (m.nch <= 1) return;
    const int b = blockIdx.x, tid = threadIdx.x, targets = m.targets, nch = m.nch;
    int* h = m.hist + (size_t)b * nch * targets;
    int carry = b * m.per;
    for (int t0 = 0; t0 < targets; t0 += 1024) {
        const int t = t0 + tid;
        const bool in = t < targets;
        int tot = 0;
        if (in) {
            int c = 0;
            for (; c + 4 <= nch; c += 4)
                tot += h[(size_t)c * targets + t] + h[(size_t)(c + 1) * targets + t] +
                       h[(size_t)(c + 2) * targets + t] + h[(size_t)(c + 3) * targets + t];
            for (; c < nch; ++c) tot += h[(size_t)c * targets + t];
        }
        int all;
        int run = carry + block_scan_1024(tot, wsum, &all);
        if (in) {
            m.offsets[(size_t)b * targets + t] = run;
            for (int c = 0; c < nch; c += 8) {
                int v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = c + u < nch ? h[(size_t)(c + u) * targets + t] : 0;
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (c + u < nch) {
                        h[(size_t)(c + u) * targets + t] = run;
                        run += v[u];
                    }
            }
        }
        carry += all;
    }
    if (b == nbatch - 1 && tid == 0) m.offsets[(size_t)nbatch * targets] = nbatch * m.per;
}

template <int W>
__global__ __launch_bounds__(W * 64) void inverse_rank_kernel(const InvBatch bat, int nbatch) {
    constexpr int NT = W * 64;
    extern __shared__ int wb[];                         // [W][targets]: per-wave counts, then bases; + [W]
    const InvMap& m = bat.m[blockIdx.z];
    const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
    if (c >= m.nch) return;
    const int targets = m.targets, per = m.per, chunk = m.chunk, nch = m.nch;
    int* wsum = wb + W * targets;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int t = tid; t < W * targets; t += NT) wb[t] = 0;
    __syncthreads();
    const int32_t* id = m.idx + (size_t)b * per;
    const int sub = chunk / W;                          // chunk is a multiple of 256
    const int ws = min(per, c * chunk + wave * sub), we = min(per, c * chunk + (wave + 1) * sub);
    int* mb = wb + wave * targets;
    for (int s = ws + lane; s < we; s += 64) {
        const unsigned t = (unsigned)id[s];
        if (t < (unsigned)targets) atomicAdd(&mb[t], 1);
    }
    __syncthreads();
    if (nch > 1) {
        // the chunk's list bases (inverse_scan_kernel) -> per-wave bases
        const int* hc = m.hist + ((size_t)b * nch + c) * targets;
        for (int t = tid; t < targets; t += NT) {
            int run = hc[t];
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const int v = wb[w * targets + t];
                wb[w * targets + t] = run;
                run += v;
            }
        }
    } else {
        // one chunk: this block scans its own counts; each thread a run of consecutive targets
        const int pt = (targets + NT - 1) / NT;
        const int a = min(tid * pt, targets), z = min(a + pt, targets);
        int local = 0;
        for (int t = a; t < z; ++t)
#pragma unroll
            for (int w = 0; w < W; ++w) local += wb[w * targets + t];
        int incl = local;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(incl, d, 64);
            if (lane >= d) incl += v;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        int run = b * per + incl - local;
        for (int w = 0; w < wave; ++w) run += wsum[w];
        for (int t = a; t < z; ++t) {
            m.offsets[(size_t)b * targets + t] = run;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const int v = wb[w * targets + t];
                wb[w * targets + t] = run;
                run += v;
            }
        }
        if (b == nbatch - 1 && tid == 0) m.offsets[(size_t)nbatch * targets] = nbatch * per;
    }
    __syncthreads();
    const int gbase = b * per, nbits = m.nbits;
    int32_t* entries = m.entries;
    const unsigned long long lt = lanemask_lt();
    for (int g = ws; g < we; g += 64) {
        const int s = g + lane;
        const int t = s < we ? id[s] : -1;
        const bool ok = (unsigned)t < (unsigned)targets;
        unsigned long long peers = ballot(ok);
        for (int bit = 0; bit < nbits; ++bit) {
            const bool on = (t >> bit) & 1;
            const unsigned long long mk = ballot(on);
            peers &= on ? mk : ~mk;
        }
        const int rank = popc64(peers & lt), cnt = popc64(peers);
        if (ok) {
            const int p = mb[t];
            entries[p + rank] = gbase + s;
            if (rank == cnt - 1) mb[t] = p + cnt;      // the group's last lane advances the base
        }
    }
}

// hist bytes of one map, 256-B aligned (0 for a one-chunk cloud).  B * nch * targets <= B * (per +
// targets) ints (chunk >= targets): within the single-map workspace, inv_ws_bytes below
static size_t hist_region(int B, int per, int targets) {
    const int chunk = rank_chunk(targets), nch = (per + chunk - 1) / chunk;
    return nch > 1 ? ((size_t)B * nch * targets * 4 + 255) / 256 * 256 : 0;
}

// enqueue the counting sort of maps[0, n) (every targets <= kRankMaxTargets, n <= kInvBatch);
// hist regions carved from ws (hist_region each); returns the bytes carved
static size_t rank_batch(const pcs_inverse_map* maps, int n, int B, char* ws, hipStream_t s) {
    InvBatch bat{};
    int maxnch = 1, maxT = 1, maxT4 = 0, maxT8 = 0;
    bool any_multi = false;
    size_t off = 0;
    for (int i = 0; i < n; ++i) {
        InvMap& m = bat.m[i];
        m.idx = maps[i].idx;
        m.offsets = maps[i].offsets;
        m.entries = maps[i].entries;
        m.per = maps[i].per_batch;
        m.targets = maps[i].targets;
        m.chunk = rank_chunk(m.targets);
        m.nch = (m.per + m.chunk - 1) / m.chunk;
        m.nbits = 0;
        while ((1 << m.nbits) < m.targets) ++m.nbits;
        m.hist = reinterpret_cast<int*>(ws + off);
        off += hist_region(B, m.per, m.targets);
        maxnch = std::max(maxnch, m.nch);
        maxT = std::max(maxT, m.targets);
        if (m.targets <= 4096) maxT4 = std::max(maxT4, m.targets);
        else maxT8 = std::max(maxT8, m.targets);
        any_multi |= m.nch > 1;
    }
    if (any_multi) {
        hipLaunchKernelGGL(inverse_count_kernel, dim3(maxnch, B, n), dim3(256), maxT * sizeof(int), s, bat, B);
        hipLaunchKernelGGL(inverse_scan_kernel, dim3(B, n), dim3(1024), 0, s, bat, B);
    }
    // rank: 4 waves for <= 4096 targets (64 KB of LDS counters), 2 above; one launch per width
    // (the other width's maps get nch = 0 in its copy: their blocks exit at once)
    for (int W : {4, 2}) {
        const int mt = W == 4 ? maxT4 : maxT8;
        if (!mt) continue;
        InvBatch bw = bat;
        int nchw = 1;
        for (int i = 0; i < n; ++i) {
            if ((bw.m[i].targets <= 4096) != (W == 4)) bw.m[i].nch = 0;
            nchw = std::max(nchw, bw.m[i].nch);
        }
        const size_t lds = ((size_t)W * mt + W) * sizeof(int);
        if (W == 4) {
            // up to (4 * 4096 + 4) ints = 65552 B: above the 64 KB default cap, set like <2>'s
            static const hipError_t attr = hipFuncSetAttribute(
                reinterpret_cast<const void*>(&inverse_rank_kernel<4>), hipFuncAttributeMaxDynamicSharedMemorySize,
                (4 * 4096 + 4) * (int)sizeof(int));
            (void)attr;
            hipLaunchKernelGGL(inverse_rank_kernel<4>, dim3(nchw, B, n), dim3(256), lds, s, bw, B);
        } else {
            static const hipError_t attr = hipFuncSetAttribute(
                reinterpret_cast<const void*>(&inverse_rank_kernel<2>), hipFuncAttributeMaxDynamicSharedMemorySize,
                (2 * kRankMaxTargets + 2) * (int)sizeof(int));
            (void)attr;
            hipLaunchKernelGGL(inverse_rank_kernel<2>, dim3(nchw, B, n), dim3(128), lds, s, bw, B);
        }
    }
    return off;
}

// Gather backward over the inverse maps (round 5: streaming).  The lists of consecutive targets
// are consecutive in `entries`, so one wave walks the lists of TW consecutive targets as ONE
// contiguous entry range [off[t0], off[t0 + TW]): the entries are fetched 64 at a time, one per
// lane (with the IDW coefficients of an interpolation slot computed lane-parallel), and walked
// with v_readlane, U gradient rows in flight per lane; lanes own channels, so every row is read as
// contiguous channel runs.  A target's list ends where the running entry index reaches the next
// offset (uniform control: the offsets of the wave's targets sit one per lane), and its fp64 sum
// is written out then.  Per channel the terms are added in list order -- the same order, per-term
// rounding and fp64 accumulation as the round-4 one-wave-per-target kernels, so the outputs are
// bitwise unchanged -- but the wave no longer waits on offsets -> entries -> rows -> store for
// every target: the per-target latency chain became a stream with U x V loads in flight.
//
// V channels per lane: VEC -- V consecutive channels (one float V-vector load per row; rows and
// col_off 16-B aligned, D = 64 V), else channels lane + 64 v (scalar loads; any col_off, D <= 64 V).
// IDW: interpolation slots s = 3 * row + j with term (g / norm_row) * w_j (common.py:119-122);
// otherwise group slots s = row with term g (common.py:64-65).
template <int V, bool VEC, bool IDW, int U>
__global__ __launch_bounds__(256) void csr_bwd_stream_kernel(const float* __restrict__ gout, int ld, int col_off,
                                                             const float* __restrict__ dist,
                                                             const int32_t* __restrict__ off,
                                                             const int32_t* __restrict__ ent, int targets, int D,
                                                             int TW, float* __restrict__ out, int ldo, int n_slots) {
    typedef float fv __attribute__((ext_vector_type(V)));
    const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int t0 = wid * TW;
    if (t0 >= targets) return;
    const int nt = min(TW, targets - t0);
    const int ol = off[t0 + min(lane, nt)];             // off[t0 .. t0 + nt], one per lane
    const int E0 = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(ol, 0));
    const int E1 = __builtin_amdgcn_readlane(ol, nt);
    int cch[V];
    bool cok[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int c = VEC ? V * lane + v : lane + 64 * v;
        cok[v] = c < D;
        cch[v] = col_off + (cok[v] ? c : D - 1);
    }
    double acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.0;
    int cur = 0;                                        // the current target, relative to t0
    int nb = __builtin_amdgcn_readlane(ol, 1);          // its list's end
    auto flush = [&]() {
        float* o = out + (size_t)(t0 + cur) * ldo;
        if (VEC) {
            fv w;
#pragma unroll
            for (int v = 0; v < V; ++v) w[v] = (float)acc[v];
            *reinterpret_cast<fv*>(o + V * lane) = w;
        } else {
#pragma unroll
            for (int v = 0; v < V; ++v)
                if (cok[v]) o[lane + 64 * v] = (float)acc[v];
        }
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] = 0.0;
        ++cur;
        nb = __builtin_amdgcn_readlane(ol, min(cur + 1, nt));
    };
    for (int base = E0; base < E1; base += 64) {
        const int n = min(64, E1 - base);
        int row = 0;
        float nrm = 1.f, wj = 0.f;
        if (lane < n) {
            const int s = ent[base + lane];
            // a stale or corrupt inverse map would read outside the slot rows (debug library only)
            PCS_DCHECK(s >= 0 && s < n_slots, "csr backward: entry %d = slot %d outside %d slots", base + lane, s,
                       n_slots);
            if (IDW) {
                row = s / 3;
                const int j = s - 3 * row;
                const float w0 = 1.0f / (dist[(size_t)row * 3 + 0] + 1e-9f);
                const float w1 = 1.0f / (dist[(size_t)row * 3 + 1] + 1e-9f);
                const float w2 = 1.0f / (dist[(size_t)row * 3 + 2] + 1e-9f);
                nrm = (w0 + w1) + w2;
                wj = j == 0 ? w0 : (j == 1 ? w1 : w2);
            } else {
                row = s;
            }
        }
        for (int e = 0; e < n; e += U) {
            float val[U][V];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int eu = min(e + u, n - 1);
                const float* g = gout + (size_t)__builtin_amdgcn_readlane(row, eu) * ld;
                if (VEC) {
                    const fv gv = *reinterpret_cast<const fv*>(g + col_off + V * lane);
#pragma unroll
                    for (int v = 0; v < V; ++v) val[u][v] = gv[v];
                } else {
#pragma unroll
                    for (int v = 0; v < V; ++v) val[u][v] = g[cch[v]];
                }
                if (IDW) {
                    const float nv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(nrm), eu));
                    const float wv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wj), eu));
#pragma unroll
                    for (int v = 0; v < V; ++v) val[u][v] = (val[u][v] / nv) * wv;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (e + u < n) {
                    const int gi = base + e + u;
                    while (gi == nb) flush();           // the lists that end here (empty ones too)
#pragma unroll
                    for (int v = 0; v < V; ++v) acc[v] += (double)val[u][v];
                }
            }
        }
    }
    while (cur < nt) flush();                           // the last list and any empty ones after it
}

// get_graph_feature backward (dgcnn.py:41-53, rows [x_j - x_i, x_i] of stride ld): point t's
// gradient = sum_j (g_b[t,j] - g_a[t,j]) over its own k rows, plus g_a of every edge row
// whose neighbour is t (its inverse-map list, ascending).  One wave per point, lanes over
// channels, fp64 accumulation in a fixed order.
__global__ __launch_bounds__(256) void edge_bwd_csr_kernel(const float* __restrict__ gout, int ld, int k,
                                                           const int32_t* __restrict__ off,
                                                           const int32_t* __restrict__ ent, int targets, int D,
                                                           float* __restrict__ gx) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= targets) return;
    const int a = off[t], z = off[t + 1];
    for (int c0 = 0; c0 < D; c0 += 64) {
        const int c = c0 + lane;
        const int cc = c < D ? c : D - 1;
        double acc = 0.0;
        for (int j = 0; j < k; ++j) {
            const float* g = gout + ((size_t)t * k + j) * ld;
            acc += (double)g[D + cc];
            acc -= (double)g[cc];
        }
        for (int base = a; base < z; base += 64) {
            const int n = min(64, z - base);
            const int mine = lane < n ? ent[base + lane] : 0;
            for (int e = 0; e < n; ++e) acc += (double)gout[(size_t)__builtin_amdgcn_readlane(mine, e) * ld + cc];
        }
        if (c < D) gx[(size_t)t * D + c] = (float)acc;
    }
}

}  // namespace pcs

using namespace pcs;

// workspace bytes of one map: the legacy path's scatter scratch (one int per slot) + global
// counters, or the counting sort's chunk histogram, whichever is larger
static size_t inv_ws_bytes(long long n_slots, long long n_targets) {
    return ((size_t)n_slots * 4 + 255) / 256 * 256 + ((size_t)n_targets * 4 + 255) / 256 * 256;
}

static int check_map(const pcs_inverse_map& m, int B, const char* who) {
    PCS_CHECK_ARG(m.per_batch >= 1 && m.targets >= 1, "%s: bad sizes per_batch=%d targets=%d", who, m.per_batch,
                  m.targets);
    PCS_CHECK_ARG((long long)B * m.per_batch < (1ll << 31) && (long long)B * m.targets < (1ll << 31),
                  "%s: too many slots/targets", who);
    PCS_CHECK_ARG(m.idx && m.offsets && m.entries, "%s: null pointer", who);
    return 0;
}

// workspace of a batch: the counting-sort maps' hist regions side by side (they are live
// together), or the largest legacy map's scratch (those run one after another, after them)
static size_t batch_ws_bytes(const pcs_inverse_map* maps, int n, int B) {
    size_t rank = 0, legacy = 256;
    for (int i = 0; i < n; ++i) {
        if (maps[i].targets <= kRankMaxTargets)
            rank += hist_region(B, maps[i].per_batch, maps[i].targets);
        else
            legacy = std::max(legacy, inv_ws_bytes((long long)B * maps[i].per_batch, (long long)B * maps[i].targets));
    }
    return std::max(rank, legacy);
}

// one map of more than kRankMaxTargets targets: LDS (or global) counting scatter + list sort
static void legacy_map(const pcs_inverse_map& m, int B, void* workspace, hipStream_t s) {
    const long long n = (long long)B * m.per_batch, T = (long long)B * m.targets;
    int32_t* scratch = static_cast<int32_t*>(workspace);
    // algorithmic bytes of the map (both kernels): idx read, entries + offsets written
    ProbeScope pr(s, 0.0, 8.0 * (double)n + 4.0 * (double)(T + 1),
                  m.targets <= kInvLdsTargets ? "pcs::inverse_index+sort<true>" : "pcs::inverse_index+sort<false>");
    int* gcnt = reinterpret_cast<int*>(static_cast<char*>(workspace) + ((size_t)n * 4 + 255) / 256 * 256);
    if (m.targets <= kInvLdsTargets) {
        static const hipError_t attr = hipFuncSetAttribute(
            reinterpret_cast<const void*>(&inverse_index_kernel<true>), hipFuncAttributeMaxDynamicSharedMemorySize,
            (32 + kInvLdsTargets) * (int)sizeof(int));
        (void)attr;
        hipLaunchKernelGGL(inverse_index_kernel<true>, dim3(B), dim3(kInvThreads), (32 + m.targets) * sizeof(int), s,
                           m.idx, m.per_batch, m.targets, B, m.offsets, (int*)nullptr, scratch);
    } else {
        hipLaunchKernelGGL(inverse_index_kernel<false>, dim3(B), dim3(kInvThreads), 32 * sizeof(int), s, m.idx,
                           m.per_batch, m.targets, B, m.offsets, gcnt, scratch);
    }
    hipLaunchKernelGGL(inverse_sort_kernel, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, s, m.offsets, scratch, (int)T,
                       m.entries);
}

PCS_API int pcs_inverse_index_workspace(long long n_slots, long long n_targets, size_t* bytes) {
    PCS_CHECK_ARG(n_slots >= 1 && n_slots < (1ll << 31) && n_targets >= 1 && n_targets < (1ll << 31) && bytes,
                  "pcs_inverse_index_workspace: bad sizes");
    *bytes = inv_ws_bytes(n_slots, n_targets);
    return 0;
}

PCS_API int pcs_inverse_index_batch_workspace(const pcs_inverse_map* maps, int nmaps, int B, size_t* bytes) {
    PCS_CHECK_ARG(maps && nmaps >= 1 && B >= 1 && bytes, "pcs_inverse_index_batch_workspace: bad arguments");
    for (int i = 0; i < nmaps; ++i)
        PCS_CHECK_ARG(maps[i].per_batch >= 1 && maps[i].targets >= 1, "pcs_inverse_index_batch_workspace: map %d", i);
    *bytes = batch_ws_bytes(maps, nmaps, B);
    return 0;
}

// the inverse maps of several neighbour tables of B clouds each (see pcs_inverse_index), in as
// few launches as their shapes allow: 3 for any number of <= 8192-target maps
PCS_API int pcs_inverse_index_batch(const pcs_inverse_map* maps, int nmaps, int B, void* workspace, size_t ws_bytes,
                                    void* stream) {
    PCS_CHECK_ARG(maps && nmaps >= 1 && B >= 1, "pcs_inverse_index_batch: bad arguments");
    for (int i = 0; i < nmaps; ++i)
        if (int e = check_map(maps[i], B, "pcs_inverse_index_batch")) return e;
    const size_t need = batch_ws_bytes(maps, nmaps, B);
    PCS_CHECK_ARG(workspace && ws_bytes >= need, "pcs_inverse_index_batch: workspace %zu < %zu bytes", ws_bytes, need);
    hipStream_t s = as_stream(stream);
    pcs_inverse_map rk[kInvBatch];
    int nr = 0;
    double bytes = 0.0;
    for (int i = 0; i < nmaps; ++i)
        if (maps[i].targets <= kRankMaxTargets)
            bytes += 12.0 * B * (double)maps[i].per_batch + 4.0 * ((double)B * maps[i].targets + 1);
    {
        // chunked stable counting sort (above): idx read twice, entries + offsets written
        ProbeScope pr(s, 0.0, bytes, "pcs::inverse_index<rank>");
        char* ws = static_cast<char*>(workspace);
        for (int i = 0; i < nmaps; ++i) {
            if (maps[i].targets > kRankMaxTargets) continue;
            rk[nr++] = maps[i];
            if (nr == kInvBatch) {        // the next group's hist regions follow this group's
                ws += rank_batch(rk, nr, B, ws, s);
                nr = 0;
            }
        }
        if (nr) rank_batch(rk, nr, B, ws, s);
    }
    for (int i = 0; i < nmaps; ++i)
        if (maps[i].targets > kRankMaxTargets) legacy_map(maps[i], B, workspace, s);
    return launch_status("pcs_inverse_index_batch");
}

// idx: (B * per_batch) int32 neighbour table, values in [0, targets); offsets (B*targets + 1),
// entries (B * per_batch): slots reading source (b, p) are entries[offsets[b*targets+p] ..
// offsets[b*targets+p+1]), ascending.
PCS_API int pcs_inverse_index(const int32_t* idx, int B, int per_batch, int targets, int32_t* offsets,
                              int32_t* entries, void* workspace, size_t ws_bytes, void* stream) {
    PCS_CHECK_ARG(B >= 1 && per_batch >= 1 && targets >= 1, "pcs_inverse_index: bad sizes");
    const long long n = (long long)B * per_batch, T = (long long)B * targets;
    PCS_CHECK_ARG(n < (1ll << 31) && T < (1ll << 31), "pcs_inverse_index: too many slots/targets");
    PCS_CHECK_ARG(idx && offsets && entries, "pcs_inverse_index: null pointer");
    PCS_CHECK_ARG(workspace && ws_bytes >= inv_ws_bytes(n, T), "pcs_inverse_index: workspace %zu < %zu bytes",
                  ws_bytes, inv_ws_bytes(n, T));
    const pcs_inverse_map m{idx, per_batch, targets, offsets, entries};
    return pcs_inverse_index_batch(&m, 1, B, workspace, ws_bytes, stream);
}

// targets per wave of the streaming CSR backward: one.  Several consecutive lists per wave (up to
// 16, keeping ~16 waves per CU) measured slower in-step: PointNet++ 4.98 vs 4.82 ms with 8 per
// wave at SA2 (the group backward 174 vs ~60 us: fewer waves hide less latency), 4.93 with 4
// (profiles/r05_ab_csr_tw.txt)
static int csr_tw(long long targets) {
    (void)targets;
    return 1;
}

template <int V, bool VEC, bool IDW>
static void launch_stream(const float* gout, int ld, int col_off, const float* dist, const int32_t* off,
                          const int32_t* ent, int targets, int D, float* out, int ldo, int n_slots, hipStream_t s) {
    constexpr int U = VEC ? 16 : (16 / V > 4 ? 16 / V : 4);
    const int tw = csr_tw(targets);
    const long long waves = (targets + tw - 1) / tw;
    hipLaunchKernelGGL((csr_bwd_stream_kernel<V, VEC, IDW, U>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s,
                       gout, ld, col_off, dist, off, ent, targets, D, tw, out, ldo, n_slots);
}

template <bool IDW>
static int csr_bwd_chunk(const float* gout, int ld, int col_off, const float* dist, const int32_t* off,
                         const int32_t* ent, int targets, int D, float* out, int ldo, int n_slots, hipStream_t s) {
    const bool al = ld % 4 == 0 && col_off % 4 == 0 && ldo % 4 == 0 && ((uintptr_t)gout | (uintptr_t)out) % 16 == 0;
    if (al && D == 64) launch_stream<1, false, IDW>(gout, ld, col_off, dist, off, ent, targets, D, out, ldo, n_slots, s);
    else if (al && D == 128) launch_stream<2, true, IDW>(gout, ld, col_off, dist, off, ent, targets, D, out, ldo, n_slots, s);
    else if (al && D == 256) launch_stream<4, true, IDW>(gout, ld, col_off, dist, off, ent, targets, D, out, ldo, n_slots, s);
    else if (D <= 64) launch_stream<1, false, IDW>(gout, ld, col_off, dist, off, ent, targets, D, out, ldo, n_slots, s);
    else if (D <= 128) launch_stream<2, false, IDW>(gout, ld, col_off, dist, off, ent, targets, D, out, ldo, n_slots, s);
    else if (D <= 256) launch_stream<4, false, IDW>(gout, ld, col_off, dist, off, ent, targets, D, out, ldo, n_slots, s);
    else if (D <= 512) launch_stream<8, false, IDW>(gout, ld, col_off, dist, off, ent, targets, D, out, ldo, n_slots, s);
    else PCS_CHECK_ARG(false, "csr backward: D=%d > 512", D);
    return 0;
}

// the streaming CSR backward over channels [0, D) of rows at col_off, output rows of stride ldo: one
// launch per 512 channels, V = the channel chunks per lane
template <bool IDW>
static int csr_bwd(const float* gout, int ld, int col_off, const float* dist, const int32_t* off, const int32_t* ent,
                   int targets, int D, float* out, int n_slots, hipStream_t s) {
    for (int c0 = 0; c0 < D; c0 += 512)
        if (int e = csr_bwd_chunk<IDW>(gout, ld, col_off + c0, dist, off, ent, targets, std::min(512, D - c0), out + c0,
                                       D, n_slots, s))
            return e;
    return 0;
}

static const char* csr_bwd_name(bool idw, int ld, int col_off, const void* gout, const void* out, int D) {
    const bool al = ld % 4 == 0 && col_off % 4 == 0 && ((uintptr_t)gout | (uintptr_t)out) % 16 == 0;
    const int V = D <= 64 ? 1 : D <= 128 ? 2 : D <= 256 ? 4 : 8;
    const bool vec = al && V > 1 && D == 64 * V && V <= 4;
    const int U = vec ? 16 : (16 / V > 4 ? 16 / V : 4);
    static char names[2][4][2][64];
    const int vi = V == 1 ? 0 : V == 2 ? 1 : V == 4 ? 2 : 3;
    char* nm = names[idw][vi][vec];
    snprintf(nm, 64, "pcs::csr_bwd_stream_kernel<%d, %s, %s, %d>", V, vec ? "true" : "false", idw ? "true" : "false", U);
    return nm;
}

// grad_feats (B, N, D) = backward of group's feature gather (overwrites; no zero fill needed).
PCS_API int pcs_group_bwd_csr(const float* grad_out, int ld_gout, const int32_t* offsets, const int32_t* entries,
                              int B, int N, int D, long long n_slots, float* grad_feats, void* stream) {
    PCS_CHECK_ARG(B >= 1 && N >= 1 && D >= 1 && ld_gout >= 3 + D && n_slots >= 0, "pcs_group_bwd_csr: bad sizes");
    const long long total = (long long)B * N * D, targets = (long long)B * N;
    PCS_CHECK_ARG(total < (1ll << 31) && n_slots < (1ll << 31), "pcs_group_bwd_csr: too many elements");
    PCS_CHECK_ARG(grad_out && offsets && entries && grad_feats, "pcs_group_bwd_csr: null pointer");
    hipStream_t s = as_stream(stream);
    // algorithmic bytes (SURVEY.md 8(d) group bwd): the D gradient columns of every grouped row (one
    // per slot) and its entry read once, the source gradient written, the offsets read
    ProbeScope pr(s, 0.0, 4.0 * (double)n_slots * (D + 1) + 4.0 * (double)total + 4.0 * (double)(targets + 1), "%s",
                  probe_enabled() ? csr_bwd_name(false, ld_gout, 3, grad_out, grad_feats, D) : "");
    if (int e = csr_bwd<false>(grad_out, ld_gout, 3, nullptr, offsets, entries, (int)targets, D, grad_feats,
                               (int)n_slots, s))
        return e;
    return launch_status("pcs_group_bwd_csr");
}

// grad_pts (B, M, D) = backward of interpolate's IDW gather (overwrites).
PCS_API int pcs_interp_bwd_csr(const float* grad_out, int ld_gout, int col_off, const float* dist,
                               const int32_t* offsets, const int32_t* entries, int B, int M, int D,
                               long long n_slots, float* grad_pts, void* stream) {
    PCS_CHECK_ARG(B >= 1 && M >= 1 && D >= 1 && ld_gout >= col_off + D && col_off >= 0 && n_slots >= 0,
                  "pcs_interp_bwd_csr: bad sizes");
    const long long total = (long long)B * M * D, targets = (long long)B * M;
    PCS_CHECK_ARG(total < (1ll << 31) && n_slots < (1ll << 31), "pcs_interp_bwd_csr: too many elements");
    PCS_CHECK_ARG(grad_out && dist && offsets && entries && grad_pts, "pcs_interp_bwd_csr: null pointer");
    hipStream_t s = as_stream(stream);
    // algorithmic bytes: per slot its row's D gradient columns, its entry and its row's 3 distances
    // (read once per slot), the coarse gradient written, the offsets read
    ProbeScope pr(s, 0.0, 4.0 * (double)n_slots * (D + 4) + 4.0 * (double)total + 4.0 * (double)(targets + 1), "%s",
                  probe_enabled() ? csr_bwd_name(true, ld_gout, col_off, grad_out, grad_pts, D) : "");
    if (int e = csr_bwd<true>(grad_out, ld_gout, col_off, dist, offsets, entries, (int)targets, D, grad_pts,
                              (int)n_slots, s))
        return e;
    return launch_status("pcs_interp_bwd_csr");
}

// grad_x (B, N, D) = backward of get_graph_feature over the inverse map of idx (targets N)
// (overwrites).  Reference: dgcnn.py:41-53.
PCS_API int pcs_edge_bwd(const float* grad_out, int ld_gout, const int32_t* offsets, const int32_t* entries, int B,
                         int N, int k, int D, float* grad_x, void* stream) {
    PCS_CHECK_ARG(B >= 1 && N >= 1 && k >= 1 && D >= 1 && ld_gout >= 2 * D, "pcs_edge_bwd: bad sizes");
    const long long targets = (long long)B * N;
    PCS_CHECK_ARG(targets * k < (1ll << 31) && targets * D < (1ll << 31), "pcs_edge_bwd: too many elements");
    PCS_CHECK_ARG(grad_out && offsets && entries && grad_x, "pcs_edge_bwd: null pointer");
    hipLaunchKernelGGL(edge_bwd_csr_kernel, dim3((unsigned)((targets + 3) / 4)), dim3(256), 0, as_stream(stream),
                       grad_out, ld_gout, k, offsets, entries, (int)targets, D, grad_x);
    return launch_status("pcs_edge_bwd");
}
