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
// no sort pass:
//   1. inverse_count_kernel (chunk c, cloud b; clouds of more than one chunk only): LDS
//      histogram of chunk c's targets -> hist[b][c][t];
//   2. inverse_rank_kernel (chunk c, cloud b): each wave owns a contiguous quarter (half) of the
//      chunk and counts it per target in LDS; each thread then takes a run of targets, adds up
//      their totals over the chunks (the LDS counts when the cloud is one chunk) and the counts
//      of the chunks before c, and one block scan turns them into the targets' list offsets
//      (written by chunk 0) and this chunk's per-wave list bases; finally each wave walks its
//      slots in order, 64 at a time: the lanes reading the same target are found by a ballot
//      over the target's bits (a match), a slot's position is its wave base + the number of
//      matching lanes below it, and the group's last lane advances the base.
// Slot order = list order: ascending, deterministic.  Chunks hold >= max(4096, targets) slots, so
// the hist workspace (B * chunks * targets ints) fits in the B*per + B*targets ints the
// workspace already provides.  One launch for a one-chunk cloud, two otherwise.
constexpr int kChunkMin = 4096, kRankMaxTargets = 8192;

static int rank_chunk(int targets) { return std::max(kChunkMin, (targets + 255) / 256 * 256); }

__global__ __launch_bounds__(256) void inverse_count_kernel(const int32_t* __restrict__ idx, int per, int targets,
                                                            int chunk, int nch, int* __restrict__ hist) {
    extern __shared__ int cnt[];
    const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    for (int t = tid; t < targets; t += 256) cnt[t] = 0;
    __syncthreads();
    const int32_t* id = idx + (size_t)b * per;
    const int s1 = min(per, (c + 1) * chunk);
    for (int s = c * chunk + tid; s < s1; s += 256) {
        const unsigned t = (unsigned)id[s];
        if (t < (unsigned)targets) atomicAdd(&cnt[t], 1);     // counts: order-free
    }
    __syncthreads();
    int* h = hist + ((size_t)b * nch + c) * targets;
    for (int t = tid; t < targets; t += 256) h[t] = cnt[t];
}

template <int W>
__global__ __launch_bounds__(W * 64) void inverse_rank_kernel(const int32_t* __restrict__ idx, int per, int targets,
                                                              int chunk, int nch, int nbatch, int nbits,
                                                              const int* __restrict__ hist,
                                                              int32_t* __restrict__ offsets,
                                                              int32_t* __restrict__ entries) {
    constexpr int NT = W * 64;
    extern __shared__ int wb[];                         // [W][targets]: per-wave counts, then bases; + [W]
    int* wsum = wb + W * targets;
    const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int t = tid; t < W * targets; t += NT) wb[t] = 0;
    __syncthreads();
    const int32_t* id = idx + (size_t)b * per;
    const int sub = chunk / W;                          // chunk is a multiple of 256
    const int ws = min(per, c * chunk + wave * sub), we = min(per, c * chunk + (wave + 1) * sub);
    int* mb = wb + wave * targets;
    for (int s = ws + lane; s < we; s += 64) {
        const unsigned t = (unsigned)id[s];
        if (t < (unsigned)targets) atomicAdd(&mb[t], 1);
    }
    __syncthreads();
    // this thread's run of targets: totals over the cloud's chunks and the counts before chunk c
    const int pt = (targets + NT - 1) / NT;
    const int a = min(tid * pt, targets), z = min(a + pt, targets);
    const int* hb = hist + (size_t)b * nch * targets;
    auto totals = [&](int t, int& pre) {
        int tot = 0;
        pre = 0;
        if (nch == 1) {
#pragma unroll
            for (int w = 0; w < W; ++w) tot += wb[w * targets + t];
        } else {
            for (int cc = 0; cc < nch; ++cc) {
                const int v = hb[(size_t)cc * targets + t];
                pre += cc < c ? v : 0;
                tot += v;
            }
        }
        return tot;
    };
    int local = 0;
    for (int t = a; t < z; ++t) {
        int pre;
        local += totals(t, pre);
    }
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
        int pre;
        const int tot = totals(t, pre);
        if (c == 0) offsets[(size_t)b * targets + t] = run;
        int base = run + pre;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const int v = wb[w * targets + t];
            wb[w * targets + t] = base;
            base += v;
        }
        run += tot;
    }
    if (b == nbatch - 1 && c == 0 && tid == 0) offsets[(size_t)nbatch * targets] = nbatch * per;
    __syncthreads();
    const int gbase = b * per;
    const unsigned long long lt = lanemask_lt();
    for (int g = ws; g < we; g += 64) {
        const int s = g + lane;
        const int t = s < we ? id[s] : -1;
        const bool ok = (unsigned)t < (unsigned)targets;
        unsigned long long peers = ballot(ok);
        for (int bit = 0; bit < nbits; ++bit) {
            const bool on = (t >> bit) & 1;
            const unsigned long long m = ballot(on);
            peers &= on ? m : ~m;
        }
        const int rank = popc64(peers & lt), cnt = popc64(peers);
        if (ok) {
            const int p = mb[t];
            entries[p + rank] = gbase + s;
            if (rank == cnt - 1) mb[t] = p + cnt;      // the group's last lane advances the base
        }
    }
}

// Gather backward over the inverse maps: ONE WAVE PER SOURCE POINT, lanes over channels,
// so every slot's gradient row is read as contiguous channel runs (coalesced).  The slot
// list is fetched 64 entries at a time, one per lane (with the entry's per-slot
// coefficients computed once, lane-parallel), then walked with v_readlane, 4 row loads
// in flight per lane.

// grad_feats[(b, p), c] = sum over slots s reading p of gout[s][3 + c]  (fp64 accumulation)
__global__ __launch_bounds__(256) void group_bwd_csr_kernel(const float* __restrict__ gout, int ld,
                                                            const int32_t* __restrict__ off,
                                                            const int32_t* __restrict__ ent, int targets, int D,
                                                            float* __restrict__ gfeats) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= targets) return;
    const int a = off[t], z = off[t + 1];
    for (int c0 = 0; c0 < D; c0 += 64) {
        const int c = c0 + lane;
        const int cc = 3 + (c < D ? c : D - 1);
        double acc = 0.0;
        for (int base = a; base < z; base += 64) {
            const int n = min(64, z - base);
            const int mine = lane < n ? ent[base + lane] : 0;
            int e = 0;
            for (; e + 4 <= n; e += 4) {
                const float v0 = gout[(size_t)__builtin_amdgcn_readlane(mine, e) * ld + cc];
                const float v1 = gout[(size_t)__builtin_amdgcn_readlane(mine, e + 1) * ld + cc];
                const float v2 = gout[(size_t)__builtin_amdgcn_readlane(mine, e + 2) * ld + cc];
                const float v3 = gout[(size_t)__builtin_amdgcn_readlane(mine, e + 3) * ld + cc];
                acc += (double)v0;
                acc += (double)v1;
                acc += (double)v2;
                acc += (double)v3;
            }
            for (; e < n; ++e) acc += (double)gout[(size_t)__builtin_amdgcn_readlane(mine, e) * ld + cc];
        }
        if (c < D) gfeats[(size_t)t * D + c] = (float)acc;
    }
}

// grad_pts[(b, m), c] = sum over slots s = 3*row + j reading m (fp64 accumulation) of
//   (gout[row][col_off + c] / norm_row) * w_j      -- the autograd rounding of
// interpolate's (p*w)/norm (common.py:119-122), as the atomic kernel computes it
__global__ __launch_bounds__(256) void interp_bwd_csr_kernel(const float* __restrict__ gout, int ld, int col_off,
                                                             const float* __restrict__ dist,
                                                             const int32_t* __restrict__ off,
                                                             const int32_t* __restrict__ ent, int targets, int D,
                                                             float* __restrict__ gpts) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= targets) return;
    const int a = off[t], z = off[t + 1];
    for (int c0 = 0; c0 < D; c0 += 64) {
        const int c = c0 + lane;
        const int cc = col_off + (c < D ? c : D - 1);
        double acc = 0.0;
        for (int base = a; base < z; base += 64) {
            const int n = min(64, z - base);
            // this lane's entry: its row and IDW coefficients (nrm, w_j)
            int row = 0;
            float nrm = 1.f, wj = 0.f;
            if (lane < n) {
                const int s = ent[base + lane];
                row = s / 3;
                const int j = s - 3 * row;
                const float w0 = 1.0f / (dist[(size_t)row * 3 + 0] + 1e-9f);
                const float w1 = 1.0f / (dist[(size_t)row * 3 + 1] + 1e-9f);
                const float w2 = 1.0f / (dist[(size_t)row * 3 + 2] + 1e-9f);
                nrm = (w0 + w1) + w2;
                wj = j == 0 ? w0 : (j == 1 ? w1 : w2);
            }
            auto term = [&](int e) {
                const int r = __builtin_amdgcn_readlane(row, e);
                const float nv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(nrm), e));
                const float wv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wj), e));
                return (gout[(size_t)r * ld + cc] / nv) * wv;
            };
            int e = 0;
            for (; e + 4 <= n; e += 4) {
                const float v0 = term(e), v1 = term(e + 1), v2 = term(e + 2), v3 = term(e + 3);
                acc += (double)v0;
                acc += (double)v1;
                acc += (double)v2;
                acc += (double)v3;
            }
            for (; e < n; ++e) acc += (double)term(e);
        }
        if (c < D) gpts[(size_t)t * D + c] = (float)acc;
    }
}

// The same for D = 64 V (V = 2, 4: FP1 / FP2-4 of PointNet++): one pass over the slot list,
// each lane owning V consecutive channels (float2 / float4 loads of a 16-B aligned row run), so
// the list, the distances and the IDW coefficients are read once instead of D / 64 times.
// Same per-term rounding and per-channel fp64 summation order as the kernel above.
template <int V>
__global__ __launch_bounds__(256) void interp_bwd_csr_vec_kernel(const float* __restrict__ gout, int ld, int col_off,
                                                                 const float* __restrict__ dist,
                                                                 const int32_t* __restrict__ off,
                                                                 const int32_t* __restrict__ ent, int targets,
                                                                 float* __restrict__ gpts) {
    typedef float fv __attribute__((ext_vector_type(V)));
    constexpr int D = 64 * V;
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= targets) return;
    const int a = off[t], z = off[t + 1];
    double acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.0;
    const float* g0 = gout + col_off + V * lane;
    for (int base = a; base < z; base += 64) {
        const int n = min(64, z - base);
        int row = 0;
        float nrm = 1.f, wj = 0.f;
        if (lane < n) {
            const int s = ent[base + lane];
            row = s / 3;
            const int j = s - 3 * row;
            const float w0 = 1.0f / (dist[(size_t)row * 3 + 0] + 1e-9f);
            const float w1 = 1.0f / (dist[(size_t)row * 3 + 1] + 1e-9f);
            const float w2 = 1.0f / (dist[(size_t)row * 3 + 2] + 1e-9f);
            nrm = (w0 + w1) + w2;
            wj = j == 0 ? w0 : (j == 1 ? w1 : w2);
        }
        auto term = [&](int e, fv& out) {
            const int r = __builtin_amdgcn_readlane(row, e);
            const float nv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(nrm), e));
            const float wv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wj), e));
            const fv gv = *reinterpret_cast<const fv*>(g0 + (size_t)r * ld);
#pragma unroll
            for (int v = 0; v < V; ++v) out[v] = (gv[v] / nv) * wv;
        };
        int e = 0;
        for (; e + 4 <= n; e += 4) {
            fv t0, t1, t2, t3;
            term(e, t0);
            term(e + 1, t1);
            term(e + 2, t2);
            term(e + 3, t3);
#pragma unroll
            for (int v = 0; v < V; ++v) {
                acc[v] += (double)t0[v];
                acc[v] += (double)t1[v];
                acc[v] += (double)t2[v];
                acc[v] += (double)t3[v];
            }
        }
        for (; e < n; ++e) {
            fv t0;
            term(e, t0);
#pragma unroll
            for (int v = 0; v < V; ++v) acc[v] += (double)t0[v];
        }
    }
    fv o;
#pragma unroll
    for (int v = 0; v < V; ++v) o[v] = (float)acc[v];
    *reinterpret_cast<fv*>(gpts + (size_t)t * D + V * lane) = o;
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

// workspace bytes of pcs_inverse_index: the scatter's scratch lists (one int per slot) and,
// when one cloud's targets overflow the LDS counters, the global counters
static size_t inv_ws_bytes(long long n_slots, long long n_targets) {
    return ((size_t)n_slots * 4 + 255) / 256 * 256 + (size_t)n_targets * 4;
}

PCS_API int pcs_inverse_index_workspace(long long n_slots, long long n_targets, size_t* bytes) {
    PCS_CHECK_ARG(n_slots >= 1 && n_slots < (1ll << 31) && n_targets >= 1 && n_targets < (1ll << 31) && bytes,
                  "pcs_inverse_index_workspace: bad sizes");
    *bytes = inv_ws_bytes(n_slots, n_targets);
    return 0;
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
    hipStream_t s = as_stream(stream);
    int32_t* scratch = static_cast<int32_t*>(workspace);
    if (targets <= kRankMaxTargets) {
        // chunked stable counting sort (above): idx read twice, entries + offsets written
        ProbeScope pr(s, 0.0, 12.0 * (double)n + 4.0 * (double)(T + 1), "pcs::inverse_index<rank>");
        const int chunk = rank_chunk(targets), nch = (per_batch + chunk - 1) / chunk;
        int* hist = reinterpret_cast<int*>(workspace);   // B * nch * targets <= n + T ints (chunk >= targets)
        PCS_CHECK_ARG((size_t)B * nch * targets * 4 <= ws_bytes, "pcs_inverse_index: chunk histogram overflows");
        int nbits = 0;
        while ((1 << nbits) < targets) ++nbits;
        if (nch > 1)
            hipLaunchKernelGGL(inverse_count_kernel, dim3(nch, B), dim3(256), targets * sizeof(int), s, idx, per_batch,
                               targets, chunk, nch, hist);
        if (targets <= 4096)
            hipLaunchKernelGGL(inverse_rank_kernel<4>, dim3(nch, B), dim3(256), (4 * targets + 4) * sizeof(int), s,
                               idx, per_batch, targets, chunk, nch, B, nbits, hist, offsets, entries);
        else {
            static const hipError_t attr = hipFuncSetAttribute(
                reinterpret_cast<const void*>(&inverse_rank_kernel<2>), hipFuncAttributeMaxDynamicSharedMemorySize,
                (2 * kRankMaxTargets + 2) * (int)sizeof(int));
            (void)attr;
            hipLaunchKernelGGL(inverse_rank_kernel<2>, dim3(nch, B), dim3(128), (2 * targets + 2) * sizeof(int), s,
                               idx, per_batch, targets, chunk, nch, B, nbits, hist, offsets, entries);
        }
        return launch_status("pcs_inverse_index");
    }
    // algorithmic bytes of the map (both kernels): idx read, entries + offsets written
    ProbeScope pr(s, 0.0, 8.0 * (double)n + 4.0 * (double)(T + 1),
                  targets <= kInvLdsTargets ? "pcs::inverse_index+sort<true>" : "pcs::inverse_index+sort<false>");
    int* gcnt = reinterpret_cast<int*>(static_cast<char*>(workspace) + ((size_t)n * 4 + 255) / 256 * 256);
    if (targets <= kInvLdsTargets) {
        static const hipError_t attr = hipFuncSetAttribute(
            reinterpret_cast<const void*>(&inverse_index_kernel<true>), hipFuncAttributeMaxDynamicSharedMemorySize,
            (32 + kInvLdsTargets) * (int)sizeof(int));
        (void)attr;
        hipLaunchKernelGGL(inverse_index_kernel<true>, dim3(B), dim3(kInvThreads), (32 + targets) * sizeof(int), s,
                           idx, per_batch, targets, B, offsets, (int*)nullptr, scratch);
    } else {
        hipLaunchKernelGGL(inverse_index_kernel<false>, dim3(B), dim3(kInvThreads), 32 * sizeof(int), s, idx,
                           per_batch, targets, B, offsets, gcnt, scratch);
    }
    hipLaunchKernelGGL(inverse_sort_kernel, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, s, offsets, scratch, (int)T,
                       entries);
    return launch_status("pcs_inverse_index");
}

// grad_feats (B, N, D) = backward of group's feature gather (overwrites; no zero fill needed).
PCS_API int pcs_group_bwd_csr(const float* grad_out, int ld_gout, const int32_t* offsets, const int32_t* entries,
                              int B, int N, int D, float* grad_feats, void* stream) {
    PCS_CHECK_ARG(B >= 1 && N >= 1 && D >= 1 && ld_gout >= 3 + D, "pcs_group_bwd_csr: bad sizes");
    const long long total = (long long)B * N * D, targets = (long long)B * N;
    PCS_CHECK_ARG(total < (1ll << 31), "pcs_group_bwd_csr: too many elements");
    PCS_CHECK_ARG(grad_out && offsets && entries && grad_feats, "pcs_group_bwd_csr: null pointer");
    // algorithmic bytes (SURVEY.md 8(d) group bwd): the D gradient columns of every grouped row
    // read once, the source gradient written, the map read
    ProbeScope pr(as_stream(stream), 0.0, 8.0 * (double)total + 4.0 * (double)(targets + 1), "pcs::group_bwd_csr_kernel");
    hipLaunchKernelGGL(group_bwd_csr_kernel, dim3((unsigned)((targets + 3) / 4)), dim3(256), 0, as_stream(stream),
                       grad_out, ld_gout, offsets, entries, (int)targets, D, grad_feats);
    return launch_status("pcs_group_bwd_csr");
}

// grad_pts (B, M, D) = backward of interpolate's IDW gather (overwrites).
PCS_API int pcs_interp_bwd_csr(const float* grad_out, int ld_gout, int col_off, const float* dist,
                               const int32_t* offsets, const int32_t* entries, int B, int M, int D, float* grad_pts,
                               void* stream) {
    PCS_CHECK_ARG(B >= 1 && M >= 1 && D >= 1 && ld_gout >= col_off + D && col_off >= 0, "pcs_interp_bwd_csr: bad sizes");
    const long long total = (long long)B * M * D, targets = (long long)B * M;
    PCS_CHECK_ARG(total < (1ll << 31), "pcs_interp_bwd_csr: too many elements");
    PCS_CHECK_ARG(grad_out && dist && offsets && entries && grad_pts, "pcs_interp_bwd_csr: null pointer");
    const dim3 grid((unsigned)((targets + 3) / 4));
    const bool al = ld_gout % 4 == 0 && col_off % 4 == 0 && ((uintptr_t)grad_out | (uintptr_t)grad_pts) % 16 == 0;
    const int V = al && (D == 128 || D == 256) ? D / 64 : 1;
    ProbeScope pr(as_stream(stream), 0.0, 8.0 * (double)total + 4.0 * (double)(targets + 1),
                  V == 1 ? "pcs::interp_bwd_csr_kernel" : "pcs::interp_bwd_csr_vec_kernel<%d>", V);
    if (V == 2)
        hipLaunchKernelGGL(interp_bwd_csr_vec_kernel<2>, grid, dim3(256), 0, as_stream(stream), grad_out, ld_gout,
                           col_off, dist, offsets, entries, (int)targets, grad_pts);
    else if (V == 4)
        hipLaunchKernelGGL(interp_bwd_csr_vec_kernel<4>, grid, dim3(256), 0, as_stream(stream), grad_out, ld_gout,
                           col_off, dist, offsets, entries, (int)targets, grad_pts);
    else
        hipLaunchKernelGGL(interp_bwd_csr_kernel, grid, dim3(256), 0, as_stream(stream), grad_out, ld_gout, col_off,
                           dist, offsets, entries, (int)targets, D, grad_pts);
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
