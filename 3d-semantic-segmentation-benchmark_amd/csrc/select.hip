// Neighbour selection: ball query (reference `group`, models/utils/common.py:51-61)
// and k-nearest (reference `interpolate`, common.py:107-114), index-exact with
// PyTorch-CPU `topk(k, largest=False)`.
//
// CPU topk runs libstdc++ `partial_sort` (heap select) when k*64 <= n and
// `nth_element` (introselect) otherwise, over (value, index) pairs in index
// order.  Out-of-radius points carry +inf, so WHICH inf entries pad an
// underfull ball -- and which of several equal distances survive -- is decided
// by those algorithms.  We emulate both exactly (the
// algorithm is modelled and checked against torch.topk in
// tests/selection_model.py):
//
//  * heap path  (k*64 <= n): one WAVE per row; the k-heap lives in lanes
//    0..k-1 (one VGPR pair), heap surgery is wave-uniform scalar code using
//    v_readlane / v_writelane; distances stream in 64-point chunks and only
//    lanes beating the heap top (ballot) are pushed, in index order.
//  * intro path (k*64 >  n): one WAVE per row; the (value, index) array lives
//    in LDS; median-of-3 + Hoare partition rounds are run WAVE-PARALLEL via the
//    closed form (left/right stop lists + crossing rank found by binary search).
//  * three_nn (k == 3, n >= 192): one THREAD per query row, a register 3-heap,
//    reference points broadcast from LDS.
//
// Distances are the reference's un-fused ((dx*dx + dy*dy) + dz*dz) in fp32; a
// ball masks d > float32(r*r) to +inf (common.py:58-59).  Output index order is
// canonical (ascending distance, then index); only the SET is reference-defined
// for ties, and every consumer (max-pool, BN sums, IDW sum) is order-invariant
// up to fp32 summation order.
#include "pcs_common.hpp"

#include <algorithm>
#include <cmath>

namespace pcs {

constexpr unsigned kInfBits = 0x7f800000u;

typedef float f32x2 __attribute__((ext_vector_type(2)));

struct Geo {
    const float* cent;  // (B, R, 3) query / centroid coordinates
    const float* xyz;   // (B, N, 3) candidate coordinates
    int B, R, N, K;
    float r2;           // float32(r*r); ignored when !use_radius
    int use_radius;
    int* out_idx;       // (B, R, K)
    float* out_dist;    // optional (B, R, K) squared distances
};

__device__ __forceinline__ unsigned dist_bits(float d, const Geo& g) {
    if (g.use_radius && !(d <= g.r2)) return kInfBits;
    return fbits(d);
}

// ------------------------------------------------------------------ heap in lanes
struct LaneHeap {
    unsigned v;  // value bits of heap slot == lane
    unsigned i;  // index of heap slot == lane

    __device__ __forceinline__ unsigned gv(int s) const { return readlane_u(v, s); }
    __device__ __forceinline__ unsigned gi(int s) const { return readlane_u(i, s); }
    __device__ __forceinline__ void set(int s, unsigned vv, unsigned ii) {
        v = writelane_u(v, vv, s);
        i = writelane_u(i, ii, s);
    }
    __device__ __forceinline__ void move(int dst, int src) { set(dst, gv(src), gi(src)); }

    // libstdc++ std::__adjust_heap + __push_heap, comp = (a.v < b.v)
    __device__ void adjust(int hole, int len, unsigned val, unsigned vidx) {
        const int top = hole;
        int second = hole;
        while (second < (len - 1) / 2) {
            second = 2 * (second + 1);
            if (gv(second) < gv(second - 1)) second--;
            move(hole, second);
            hole = second;
        }
        if ((len & 1) == 0 && second == (len - 2) / 2) {
            second = 2 * (second + 1);
            move(hole, second - 1);
            hole = second - 1;
        }
        int parent = (hole - 1) / 2;
        while (hole > top && gv(parent) < val) {
            move(hole, parent);
            hole = parent;
            parent = (hole - 1) / 2;
        }
        set(hole, val, vidx);
    }

    __device__ void make(int len) {
        if (len < 2) return;
        int parent = (len - 2) / 2;
        while (true) {
            adjust(parent, len, gv(parent), gi(parent));
            if (parent == 0) break;
            parent--;
        }
    }
};

// write the k (value,index) pairs held by lanes < k in canonical order
__device__ __forceinline__ void emit_sorted(unsigned v, unsigned i, int k, int* out_idx, float* out_dist) {
    const int l = lane_id();
    int rank = 0;
    for (int j = 0; j < k; ++j) {
        const unsigned vj = readlane_u(v, j), ij = readlane_u(i, j);
        rank += (vj < v || (vj == v && ij < i)) ? 1 : 0;
    }
    if (l < k) {
        out_idx[rank] = (int)i;
        if (out_dist) out_dist[rank] = __uint_as_float(v);
    }
}


// ------------------------------------------------------------------ ball query: the unambiguous case
// A ball's candidates held in (value, index) slots: slot 0 = the queue's first K entries (lanes < K;
// +inf out of radius), slots 1..S = in-radius entries of index >= K, list entry 64 (s - 1) + lane in
// ascending index order (n of them).  When at least K of them are finite and the K-th smallest value
// is strictly below the (K+1)-th, BOTH libstdc++ selections the reference's topk runs (SURVEY.md
// Appendix A) return exactly the K smallest: partial_sort's heap keeps every excluded entry at or
// above its final top (entries only enter strictly below the top, and the top never rises), and
// nth_element partitions around the K-th.  Then the set is found by a radix search for the K-th
// smallest value bits -- no heap surgery.  Ties at the boundary and underfull balls (whose surviving
// infs the heap order picks) take the exact emulation.
template <int S>
__device__ bool ball_unambiguous(const unsigned (&vs)[S + 1], const unsigned (&xs)[S + 1], int K, int n, uint2* scratch,
                                 int* out_idx, float* out_dist) {
    const int lane = lane_id();
    int finite = 0;
#pragma unroll
    for (int u = 0; u <= S; ++u) finite += popc64(ballot(vs[u] != kInfBits && (u > 0 || lane < K)));
    if (finite < K) return false;
    // T = the smallest value bits with count(v <= T) >= K (values finite, below +inf bits)
    unsigned lo = 0u, hi = kInfBits - 1u;
    while (lo < hi) {
        const unsigned mid = lo + ((hi - lo) >> 1);
        int c = 0;
#pragma unroll
        for (int u = 0; u <= S; ++u) c += popc64(ballot(vs[u] <= mid && (u > 0 || lane < K)));
        if (c >= K) hi = mid;
        else lo = mid + 1u;
    }
    int base = 0;
    unsigned long long sel[S + 1];
#pragma unroll
    for (int u = 0; u <= S; ++u) {
        sel[u] = ballot(vs[u] <= lo && (u > 0 || lane < K));
        base += popc64(sel[u]);
    }
    if (base != K) return false;               // a tie straddles the K-th value
    base = 0;
#pragma unroll
    for (int u = 0; u <= S; ++u) {
        if ((sel[u] >> lane) & 1ull) scratch[base + popc64(sel[u] & lanemask_lt())] = make_uint2(vs[u], xs[u]);
        base += popc64(sel[u]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane < K) {
        // canonical order: ascending value, then index
        const uint2 me = scratch[lane];
        int rank = 0;
        for (int j = 0; j < K; ++j) {
            const uint2 o = scratch[j];
            rank += (o.x < me.x || (o.x == me.x && o.y < me.y)) ? 1 : 0;
        }
        out_idx[rank] = (int)me.y;
        if (out_dist) out_dist[rank] = __uint_as_float(me.x);
    }
    return true;
}

// the exact heap select over the same slots (partial_sort's make_heap on the first K entries, then
// the in-radius entries of index >= K in index order)
template <int S>
__device__ void ball_heap_slots(const unsigned (&vs)[S + 1], const unsigned (&xs)[S + 1], int K, int n, int* out_idx,
                                float* out_dist) {
    LaneHeap h;
    h.v = vs[0];
    h.i = xs[0];
    h.make(K);
    unsigned top = h.gv(0);
#pragma unroll
    for (int u = 1; u <= S; ++u) {
        unsigned long long mk = ballot(64 * (u - 1) + lane_id() < n && vs[u] < top);
        while (mk) {
            const int l = ffs64(mk);
            mk &= mk - 1;
            const unsigned v = readlane_u(vs[u], l);
            if (v < top) {
                h.adjust(0, K, v, readlane_u(xs[u], l));
                top = h.gv(0);
            }
        }
    }
    emit_sorted(h.v, h.i, K, out_idx, out_dist);
}

// 1024-thread blocks: 16 waves share one staged cloud (48 KB at N = 4096), so LDS allows
// 8 waves per SIMD instead of 3 -- the heap surgery is a latency-bound chain of
// v_readlane / SALU hops per wave, and occupancy is what hides it.
constexpr int kHeapBlock = 1024;

constexpr int kFastS = 2;                      // list slots per lane of the staged ball path (128 entries: 24 KB per
                                               // block, so two 1024-thread blocks still share a CU at N = 4096)

template <bool STAGE>
__global__ __launch_bounds__(kHeapBlock) void heap_select_kernel(Geo g, int rows_per_wave) {
    extern __shared__ __attribute__((aligned(16))) float s_xyz[];
    const int b = blockIdx.y;
    const float* X = g.xyz + (size_t)b * g.N * 3;
    if (STAGE) {
        for (int t = threadIdx.x; t < g.N * 3; t += blockDim.x) s_xyz[t] = X[t];
        __syncthreads();
    }
    const float* P = STAGE ? s_xyz : X;
    const int lane = lane_id();
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int K = g.K;
    // ball queries (staged cloud): per wave a 64 * kFastS-entry list of the in-radius entries of index >= K
    // and K output slots, after the cloud in the dynamic LDS
    uint2* wl = reinterpret_cast<uint2*>(s_xyz + ((size_t)g.N * 3 + 3) / 4 * 4) + (size_t)(threadIdx.x >> 6) * (64 * kFastS + 64);
    for (int rr = 0; rr < rows_per_wave; ++rr) {
        const int row = wave * rows_per_wave + rr;
        if (row >= g.R) break;
        const float* c = g.cent + ((size_t)b * g.R + row) * 3;
        const float cx = c[0], cy = c[1], cz = c[2];
        int* oi = g.out_idx + ((size_t)b * g.R + row) * K;
        float* od = g.out_dist ? g.out_dist + ((size_t)b * g.R + row) * K : nullptr;

        if (STAGE && g.use_radius) {
            // one pass over the cloud: the first K entries, and the in-radius ones of index >= K in order
            // (into a 64 * kFastS-entry list)
            unsigned vs[kFastS + 1], xs[kFastS + 1];
            int n = 0;
            for (int base = 0; base < g.N; base += kWave) {
                const int p = base + lane;
                unsigned v = kInfBits;
                if (p < g.N) v = dist_bits(sqdist_unfused(P[3 * p], P[3 * p + 1], P[3 * p + 2], cx, cy, cz), g);
                if (base == 0) { vs[0] = lane < K ? v : kInfBits; xs[0] = (unsigned)lane; }
                const bool in = p >= K && p < g.N && v != kInfBits;
                const unsigned long long m = ballot(in);
                const int pos = n + popc64(m & lanemask_lt());
                if (in && pos < 64 * kFastS) wl[pos] = make_uint2(v, (unsigned)p);
                n += popc64(m);
            }
            if (n <= 64 * kFastS) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int u = 1; u <= kFastS; ++u) {
                    const int j = 64 * (u - 1) + lane;
                    const uint2 e = j < n ? wl[j] : make_uint2(kInfBits, 0u);
                    vs[u] = e.x;
                    xs[u] = e.y;
                }
                __builtin_amdgcn_wave_barrier();
                if (!ball_unambiguous<kFastS>(vs, xs, K, n, wl + 64 * kFastS, oi, od))
                    ball_heap_slots<kFastS>(vs, xs, K, n, oi, od);
                continue;
            }
            // (more than 64 * kFastS in-radius entries: the exhaustive heap pass below)
        }

        LaneHeap h;
        h.v = kInfBits;
        h.i = 0;
        unsigned top = 0;
        for (int base = 0; base < g.N; base += kWave) {
            const int p = base + lane;
            unsigned v = kInfBits;
            if (p < g.N) v = dist_bits(sqdist_unfused(P[3 * p], P[3 * p + 1], P[3 * p + 2], cx, cy, cz), g);
            if (base == 0) {
                // heap = first K queue entries (K <= 64 <= N here)
                h.v = v;
                h.i = (unsigned)p;
                h.make(K);
                top = h.gv(0);
            }
            unsigned long long m = ballot(p >= K && p < g.N && v < top);
            while (m) {
                const int l = ffs64(m);
                m &= m - 1;
                const unsigned vv = readlane_u(v, l);
                if (vv < top) {
                    h.adjust(0, K, vv, (unsigned)(base + l));
                    top = h.gv(0);
                }
            }
        }
        emit_sorted(h.v, h.i, K, oi, od);
    }
}

// ------------------------------------------------------------------ introselect in LDS
struct RowLds {
    unsigned* V;        // n value bits
    unsigned short* I;  // n indices
    unsigned short* LA; // left-stop positions (ascending)
    unsigned short* RR; // right-stop positions (ascending)
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void lds_swap(RowLds& a, int x, int y) {
    // called by one lane
    const unsigned v = a.V[x];
    const unsigned short i = a.I[x];
    a.V[x] = a.V[y];
    a.I[x] = a.I[y];
    a.V[y] = v;
    a.I[y] = i;
}

// serial libstdc++ heap select over LDS (depth-limit fallback; lane 0 only)
__device__ void lds_adjust(RowLds& a, int first, int hole, int len, unsigned val, unsigned short vidx) {
    const int top = hole;
    int second = hole;
    unsigned* V = a.V + first;
    unsigned short* I = a.I + first;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (V[second] < V[second - 1]) second--;
        V[hole] = V[second];
        I[hole] = I[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        V[hole] = V[second - 1];
        I[hole] = I[second - 1];
        hole = second - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && V[parent] < val) {
        V[hole] = V[parent];
        I[hole] = I[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    V[hole] = val;
    I[hole] = vidx;
}

__device__ void lds_heap_select(RowLds& a, int first, int middle, int last) {
    const int len = middle - first;
    if (len >= 2) {
        int parent = (len - 2) / 2;
        while (true) {
            lds_adjust(a, first, parent, len, a.V[first + parent], a.I[first + parent]);
            if (parent == 0) break;
            parent--;
        }
    }
    for (int i = middle; i < last; ++i) {
        if (a.V[i] < a.V[first]) {
            const unsigned v = a.V[i];
            const unsigned short ix = a.I[i];
            a.V[i] = a.V[first];
            a.I[i] = a.I[first];
            lds_adjust(a, first, 0, len, v, ix);
        }
    }
}

// Hoare partition of [lo, hi) around pv, wave-parallel; returns the cut.
__device__ int partition_wave(RowLds& a, int lo, int hi, unsigned pv) {
    const int lane = lane_id();
    int nL = 0, nR = 0;
    for (int base = lo; base < hi; base += kWave) {
        const int p = base + lane;
        const bool in = p < hi;
        const unsigned v = in ? a.V[p] : 0u;
        const bool isL = in && v >= pv;   // left scan stops: !(v < pv)
        const bool isR = in && v <= pv;   // right scan stops: !(pv < v)
        const unsigned long long mL = ballot(isL), mR = ballot(isR);
        const unsigned long long lt = lanemask_lt();
        if (isL) a.LA[nL + popc64(mL & lt)] = (unsigned short)p;
        if (isR) a.RR[nR + popc64(mR & lt)] = (unsigned short)p;
        nL += popc64(mL);
        nR += popc64(mR);
    }
    wave_sync();
    // i* = first i with !(LA[i] < RR[nR-1-i])  (monotone predicate)
    int l0 = 0, l1 = nL < nR ? nL : nR;
    while (l0 < l1) {
        const int mid = (l0 + l1) >> 1;
        if (a.LA[mid] < a.RR[nR - 1 - mid]) l0 = mid + 1; else l1 = mid;
    }
    const int istar = l0;
    for (int i = lane; i < istar; i += kWave) {
        const int x = a.LA[i], y = a.RR[nR - 1 - i];
        const unsigned vx = a.V[x], vy = a.V[y];
        const unsigned short ix = a.I[x], iy = a.I[y];
        a.V[x] = vy;
        a.I[x] = iy;
        a.V[y] = vx;
        a.I[y] = ix;
    }
    int cut;
    if (nL == 0 && istar == 0) cut = hi;  // unreachable with a median-of-3 pivot
    else if (istar < nL && (istar == 0 || a.LA[istar] < a.RR[nR - istar])) cut = a.LA[istar];
    else cut = a.RR[nR - istar];
    wave_sync();
    return cut;
}

__device__ void move_median_to_first(RowLds& a, int result, int x, int y, int z) {
    const unsigned vx = a.V[x], vy = a.V[y], vz = a.V[z];
    int pick;
    if (vx < vy) {
        if (vy < vz) pick = y;
        else if (vx < vz) pick = z;
        else pick = x;
    } else if (vx < vz) pick = x;
    else if (vy < vz) pick = z;
    else pick = y;
    if (lane_id() == 0) lds_swap(a, result, pick);
    wave_sync();
}

// nth_element(first, first+nth, last) on the LDS row, libstdc++ __introselect
__device__ void introselect_wave(RowLds& a, int n, int nth) {
    int first = 0, last = n;
    int depth = 2 * (31 - __clz(n));
    while (last - first > 3) {
        if (depth == 0) {
            if (lane_id() == 0) {
                lds_heap_select(a, first, nth + 1, last);
                lds_swap(a, first, nth);
            }
            wave_sync();
            return;
        }
        --depth;
        const int mid = first + (last - first) / 2;
        move_median_to_first(a, first, first + 1, mid, last - 1);
        const int cut = partition_wave(a, first + 1, last, a.V[first]);
        if (cut <= nth) first = cut; else last = cut;
    }
    // insertion sort of <= 3 elements (stable under the strict comparator)
    if (lane_id() == 0) {
        for (int i = first + 1; i < last; ++i) {
            const unsigned v = a.V[i];
            const unsigned short ix = a.I[i];
            int j = i;
            while (j > first && v < a.V[j - 1]) {
                a.V[j] = a.V[j - 1];
                a.I[j] = a.I[j - 1];
                --j;
            }
            a.V[j] = v;
            a.I[j] = ix;
        }
    }
    wave_sync();
}

// LDS per wave: n*(4+2+2+2) bytes rounded to 16
__host__ __device__ constexpr int intro_row_bytes(int n) { return ((n * 10 + 15) / 16) * 16; }

template <bool STAGE>
__global__ __launch_bounds__(256) void intro_select_kernel(Geo g, int rows_per_wave) {
    extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
    const int b = blockIdx.y;
    const int n = g.N;
    const float* X = g.xyz + (size_t)b * n * 3;
    float* s_xyz = reinterpret_cast<float*>(s_raw);
    const int xyz_bytes = STAGE ? ((n * 12 + 15) / 16) * 16 : 0;
    if (STAGE) {
        for (int t = threadIdx.x; t < n * 3; t += blockDim.x) s_xyz[t] = X[t];
        __syncthreads();
    }
    const float* P = STAGE ? s_xyz : X;
    const int lane = lane_id();
    const int wib = threadIdx.x >> 6;
    unsigned char* mine = s_raw + xyz_bytes + wib * intro_row_bytes(n);
    RowLds a;
    a.V = reinterpret_cast<unsigned*>(mine);
    a.I = reinterpret_cast<unsigned short*>(mine + n * 4);
    a.LA = a.I + n;
    a.RR = a.LA + n;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int K = g.K;
    for (int rr = 0; rr < rows_per_wave; ++rr) {
        const int row = wave * rows_per_wave + rr;
        if (row >= g.R) break;
        const float* c = g.cent + ((size_t)b * g.R + row) * 3;
        const float cx = c[0], cy = c[1], cz = c[2];
        for (int p = lane; p < n; p += kWave) {
            a.V[p] = dist_bits(sqdist_unfused(P[3 * p], P[3 * p + 1], P[3 * p + 2], cx, cy, cz), g);
            a.I[p] = (unsigned short)p;
        }
        wave_sync();
        introselect_wave(a, n, K - 1);
        // first K entries are the set; emit them in canonical order
        int* oi = g.out_idx + ((size_t)b * g.R + row) * K;
        float* od = g.out_dist ? g.out_dist + ((size_t)b * g.R + row) * K : nullptr;
        for (int p = lane; p < K; p += kWave) {
            const unsigned v = a.V[p];
            const unsigned ix = a.I[p];
            int rank = 0;
            for (int q = 0; q < K; ++q) {
                const unsigned vq = a.V[q], iq = a.I[q];
                rank += (vq < v || (vq == v && iq < ix)) ? 1 : 0;
            }
            oi[rank] = (int)ix;
            if (od) od[rank] = __uint_as_float(v);
        }
        wave_sync();
    }
}

// ------------------------------------------------------------------ three_nn (k = 3)
struct H3 {
    float v0, v1, v2;
    int i0, i1, i2;
};

// libstdc++ adjust_heap(hole = 0, len = 3, value) specialised
__device__ __forceinline__ void adjust3(H3& h, float v, int i) {
    if (h.v2 < h.v1) {
        // second = 1
        if (h.v1 < v) { h.v0 = v; h.i0 = i; }
        else { h.v0 = h.v1; h.i0 = h.i1; h.v1 = v; h.i1 = i; }
    } else {
        // second = 2
        if (h.v2 < v) { h.v0 = v; h.i0 = i; }
        else { h.v0 = h.v2; h.i0 = h.i2; h.v2 = v; h.i2 = i; }
    }
}

__device__ __forceinline__ bool lt_vi(float va, int ia, float vb, int ib) { return va < vb || (va == vb && ia < ib); }

// ------------------------------------------------------------------ heap path over a cell grid
// The heap select (partial_sort) on a ball: the heap starts as the first k queue entries
// (indices 0..k-1, out-of-radius ones at +inf) and entry i >= k replaces the top only when its
// value is strictly below it -- an out-of-radius entry (+inf) never is.  So the only entries that
// can change the heap are the IN-RADIUS points with index >= k, and they act in ascending index
// order.  This kernel visits just those: one workgroup bins its cloud into cells of edge >= r
// (counting sort in LDS), so every in-radius point of a centroid lies in the 3 x 3 x 3 cells
// around the centroid's cell; a wave marks the in-radius points >= k of those cells in a bitmap
// of the cloud's indices, walks the bitmap in ascending index order (compacted into a list) and
// runs the same lane-heap surgery as heap_select_kernel on them -- the same heap states, so the
// same index set, ties and underfull balls included.  Work per centroid: the points of 27 cells
// instead of all N (PointNeXt SA1: ~600 of 24 576).
constexpr int kGridBlock = 1024;               // 16 waves share the cloud's grid
constexpr int kGridWaves = kGridBlock / kWave;
constexpr int kGridList = 512;                 // per-wave candidate list (u16), filled in rounds
constexpr int kGridU = 4;                      // 64-candidate batches with their loads in flight together
constexpr int kGridS = kGridList / 64;         // list slots per lane of the one-list (fast) path

struct GridLds {
    int* cend;                 // [ncells]: end of cell c in `sorted` (start = cend[c - 1], 0 for c = 0)
    unsigned short* sorted;    // [N]: point indices grouped by cell
    unsigned* bm;              // [waves][nw] candidate bitmaps
    unsigned short* list;      // [waves][kGridList]
};

__device__ __forceinline__ int grid_axis(float x, float lo, float inv, int n) {
    const float u = (x - lo) * inv;
    // NaN and below-range coordinates -> 0, above-range -> n - 1
    return u >= 1.f ? (int)fminf(u, (float)(n - 1)) : 0;
}

__global__ __launch_bounds__(kGridBlock) void grid_heap_select_kernel(Geo g, float cs0, int max_cells,
                                                                      int rows_per_wave) {
    extern __shared__ __attribute__((aligned(16))) unsigned char g_lds[];
    __shared__ float s_box[kGridWaves][6];
    __shared__ float s_geo[4];                 // lo x, y, z, 1 / cell edge
    __shared__ int s_dim[3];
    const int b = blockIdx.y, N = g.N, K = g.K;
    const int nw = (N + 31) >> 5;
    const float* X = g.xyz + (size_t)b * N * 3;
    GridLds L;
    size_t off = 0;
    L.cend = reinterpret_cast<int*>(g_lds + off);
    off += (size_t)max_cells * 4;
    L.sorted = reinterpret_cast<unsigned short*>(g_lds + off);
    off += ((size_t)N * 2 + 15) / 16 * 16;
    L.bm = reinterpret_cast<unsigned*>(g_lds + off);
    off += (size_t)kGridWaves * nw * 4;
    L.list = reinterpret_cast<unsigned short*>(g_lds + off);
    const float* P = X;                        // (clouds past 8192 points: coordinates from L2)
    const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;

    // ---- bounding box (NaN coordinates ignored by fminf / fmaxf)
    float bx[6] = {__builtin_inff(), __builtin_inff(), __builtin_inff(), -__builtin_inff(), -__builtin_inff(),
                   -__builtin_inff()};
    for (int p = tid; p < N; p += kGridBlock) {
        const float x = X[3 * p], y = X[3 * p + 1], z = X[3 * p + 2];
        bx[0] = fminf(bx[0], x); bx[1] = fminf(bx[1], y); bx[2] = fminf(bx[2], z);
        bx[3] = fmaxf(bx[3], x); bx[4] = fmaxf(bx[4], y); bx[5] = fmaxf(bx[5], z);
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1)
#pragma unroll
        for (int k = 0; k < 6; ++k) bx[k] = k < 3 ? fminf(bx[k], __shfl_xor(bx[k], m)) : fmaxf(bx[k], __shfl_xor(bx[k], m));
    if (lane == 0)
        for (int k = 0; k < 6; ++k) s_box[wv][k] = bx[k];
    __syncthreads();
    if (tid == 0) {
        float lo[3], ext[3];
        bool fin = true;
        for (int k = 0; k < 3; ++k) {
            float a = s_box[0][k], c = s_box[0][k + 3];
            for (int w = 1; w < kGridWaves; ++w) { a = fminf(a, s_box[w][k]); c = fmaxf(c, s_box[w][k + 3]); }
            lo[k] = a;
            ext[k] = c - a;
            fin = fin && ext[k] >= 0.f && ext[k] < 3.0e38f;
        }
        // cell edge: >= 1.02 r (cs0), and >= 2^-16 of the largest extent, so that with the fp32
        // rounding of (x - lo) * inv (<= 2^-22 of the extent / edge) two points within r land in
        // cells at most one apart on every axis; grown until the cell count fits the LDS table
        double cs = cs0;
        if (fin) cs = fmax(cs, (double)fmaxf(ext[0], fmaxf(ext[1], ext[2])) * (1.0 / 65536.0));
        long long n[3] = {1, 1, 1};
        for (int guard = 0; fin && guard < 64; ++guard) {
            for (int k = 0; k < 3; ++k) n[k] = (long long)((double)ext[k] / cs) + 1;
            if (n[0] * n[1] * n[2] <= max_cells) break;
            cs *= 1.25;
        }
        if (!fin || n[0] * n[1] * n[2] > max_cells) n[0] = n[1] = n[2] = 1;
        for (int k = 0; k < 3; ++k) { s_geo[k] = fin ? lo[k] : 0.f; s_dim[k] = (int)n[k]; }
        s_geo[3] = fin ? (float)(1.0 / cs) : 0.f;
    }
    __syncthreads();
    const float lox = s_geo[0], loy = s_geo[1], loz = s_geo[2], inv = s_geo[3];
    const int gx = s_dim[0], gy = s_dim[1], gz = s_dim[2];
    const int nc = gx * gy * gz;
    auto cell_of = [&](float x, float y, float z) {
        return grid_axis(x, lox, inv, gx) + gx * (grid_axis(y, loy, inv, gy) + gy * grid_axis(z, loz, inv, gz));
    };
    // ---- counting sort of the point indices by cell (the order inside a cell is irrelevant: the
    // bitmap restores index order)
    for (int c = tid; c < nc; c += kGridBlock) L.cend[c] = 0;
    __syncthreads();
    for (int p = tid; p < N; p += kGridBlock) atomicAdd(&L.cend[cell_of(P[3 * p], P[3 * p + 1], P[3 * p + 2])], 1);
    __syncthreads();
    {
        // exclusive scan of the counts: each thread a run of consecutive cells, then the runs
        const int per = (nc + kGridBlock - 1) / kGridBlock;
        const int c0 = tid * per, c1 = min(c0 + per, nc);
        int sum = 0;
        for (int c = c0; c < c1; ++c) sum += L.cend[c];
        int inc = sum;
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) {
            const int o = __shfl_up(inc, m);
            inc += lane >= m ? o : 0;
        }
        __shared__ int s_ws[kGridWaves];
        if (lane == 63) s_ws[wv] = inc;
        __syncthreads();
        int base = 0;
        for (int w = 0; w < wv; ++w) base += s_ws[w];
        int run = base + inc - sum;
        for (int c = c0; c < c1; ++c) {
            const int n = L.cend[c];
            L.cend[c] = run;                   // start of cell c, advanced to its end by the scatter
            run += n;
        }
    }
    __syncthreads();
    for (int p = tid; p < N; p += kGridBlock) {
        const int c = cell_of(P[3 * p], P[3 * p + 1], P[3 * p + 2]);
        L.sorted[atomicAdd(&L.cend[c], 1)] = (unsigned short)p;
    }
    __syncthreads();

    // ---- the rows: one wave each
    unsigned* bm = L.bm + (size_t)wv * nw;
    unsigned short* list = L.list + (size_t)wv * kGridList;
    const int wave = blockIdx.x * kGridWaves + wv;
    for (int rr = 0; rr < rows_per_wave; ++rr) {
        const int row = wave * rows_per_wave + rr;
        if (row >= g.R) break;
        const float* c = g.cent + ((size_t)b * g.R + row) * 3;
        const float cx = c[0], cy = c[1], cz = c[2];
        // the queue's first K entries (K <= 64 <= N): the heap's initial contents
        const unsigned v0 = dist_bits(sqdist_unfused(P[3 * lane], P[3 * lane + 1], P[3 * lane + 2], cx, cy, cz), g);
        for (int w = lane; w < nw; w += kWave) bm[w] = 0u;
        wave_sync();
        // in-radius points >= K of the 27 cells -> bitmap.  The x-adjacent cells of one (y, z) are one
        // run of `sorted`: lane q < 9 takes run q, the 9 runs are flattened into one index space and
        // walked GU x 64 entries at a time, all their coordinate loads in flight together
        const int ix = grid_axis(cx, lox, inv, gx), iy = grid_axis(cy, loy, inv, gy), iz = grid_axis(cz, loz, inv, gz);
        const int xl = max(ix - 1, 0), xh = min(ix + 1, gx - 1);
        int rbeg = 0, rlen = 0;
        if (lane < 9) {
            const int y = iy + lane % 3 - 1, z = iz + lane / 3 - 1;
            if (y >= 0 && y < gy && z >= 0 && z < gz) {
                const int cl = xl + gx * (y + gy * z), ch = xh + gx * (y + gy * z);
                rbeg = cl == 0 ? 0 : L.cend[cl - 1];
                rlen = L.cend[ch] - rbeg;
            }
        }
        int rinc = rlen;
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) {
            const int o = __shfl_up(rinc, m);
            rinc += lane >= m ? o : 0;
        }
        const int T = __builtin_amdgcn_readlane(rinc, 8);
        int pre[9], bg[9];
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            pre[q] = __builtin_amdgcn_readlane(rinc - rlen, q);
            bg[q] = __builtin_amdgcn_readlane(rbeg, q);
        }
        for (int j0 = 0; j0 < T; j0 += kGridU * kWave) {
            int pp[kGridU];
            float qx[kGridU], qy[kGridU], qz[kGridU];
#pragma unroll
            for (int u = 0; u < kGridU; ++u) {
                const int j = j0 + u * kWave + lane;
                int b0 = bg[0], p0 = pre[0];
#pragma unroll
                for (int q = 1; q < 9; ++q)
                    if (j >= pre[q]) { b0 = bg[q]; p0 = pre[q]; }
                pp[u] = j < T ? (int)L.sorted[b0 + j - p0] : -1;
            }
#pragma unroll
            for (int u = 0; u < kGridU; ++u) {
                const int p = pp[u] < 0 ? 0 : pp[u];
                qx[u] = P[3 * p]; qy[u] = P[3 * p + 1]; qz[u] = P[3 * p + 2];
            }
#pragma unroll
            for (int u = 0; u < kGridU; ++u) {
                const int p = pp[u];
                if (p >= K && sqdist_unfused(qx[u], qy[u], qz[u], cx, cy, cz) <= g.r2)
                    atomicOr(&bm[p >> 5], 1u << (p & 31));
            }
        }
        wave_sync();
        // ascending walk: lane l owns words [l * wpl, (l + 1) * wpl), its candidates land in the list
        // at its exclusive prefix; rounds of kGridList list entries
        const int wpl = (nw + kWave - 1) / kWave;
        const int w0 = min(lane * wpl, nw), w1 = min(w0 + wpl, nw);
        int cnt = 0;
        for (int w = w0; w < w1; ++w) cnt += __popc(bm[w]);
        int incl = cnt;
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) {
            const int o = __shfl_up(incl, m);
            incl += lane >= m ? o : 0;
        }
        const int total = __builtin_amdgcn_readlane(incl, 63);
        const int first = incl - cnt;
        int* oi = g.out_idx + ((size_t)b * g.R + row) * K;
        float* od = g.out_dist ? g.out_dist + ((size_t)b * g.R + row) * K : nullptr;
        if (total <= kGridList) {
            // one list: the candidates' values into slots, then the unambiguous K smallest or the heap
            int pos = first;
            for (int w = w0; w < w1; ++w) {
                unsigned m = bm[w];
                while (m) {
                    const int bit = __ffs(m) - 1;
                    m &= m - 1;
                    list[pos++] = (unsigned short)(32 * w + bit);
                }
            }
            wave_sync();
            unsigned vs[kGridS + 1], xs[kGridS + 1];
            vs[0] = lane < K ? v0 : kInfBits;
            xs[0] = (unsigned)lane;
#pragma unroll
            for (int u = 1; u <= kGridS; ++u) {
                const int j = 64 * (u - 1) + lane;
                xs[u] = j < total ? list[j] : 0u;
            }
#pragma unroll
            for (int u = 1; u <= kGridS; ++u) {
                const int j = 64 * (u - 1) + lane;
                const unsigned p = xs[u];
                vs[u] = j < total ? dist_bits(sqdist_unfused(P[3 * p], P[3 * p + 1], P[3 * p + 2], cx, cy, cz), g)
                                  : kInfBits;
            }
            wave_sync();
            if (!ball_unambiguous<kGridS>(vs, xs, K, total, reinterpret_cast<uint2*>(list), oi, od))
                ball_heap_slots<kGridS>(vs, xs, K, total, oi, od);
            wave_sync();
            continue;
        }
        // more candidates than one list: the exact heap over rounds of the list
        LaneHeap h;
        h.v = v0;
        h.i = (unsigned)lane;
        h.make(K);
        unsigned top = h.gv(0);
        for (int r0 = 0; r0 < total; r0 += kGridList) {
            // this round's entries [r0, r0 + kGridList)
            if (first < r0 + kGridList && first + cnt > r0) {
                int pos = first;
                for (int w = w0; w < w1 && pos < r0 + kGridList; ++w) {
                    unsigned m = bm[w];
                    while (m) {
                        const int bit = __ffs(m) - 1;
                        m &= m - 1;
                        if (pos >= r0 && pos < r0 + kGridList) list[pos - r0] = (unsigned short)(32 * w + bit);
                        ++pos;
                    }
                }
            }
            wave_sync();
            const int n = min(kGridList, total - r0);
            for (int base = 0; base < n; base += kGridU * kWave) {
                // GU x 64 candidates' coordinates in flight together, then the heap in list order
                unsigned vv[kGridU], pv[kGridU];
#pragma unroll
                for (int u = 0; u < kGridU; ++u) {
                    const int j = base + u * kWave + lane;
                    pv[u] = j < n ? list[j] : 0u;
                }
#pragma unroll
                for (int u = 0; u < kGridU; ++u) {
                    const int j = base + u * kWave + lane;
                    const unsigned p = pv[u];
                    vv[u] = j < n ? dist_bits(sqdist_unfused(P[3 * p], P[3 * p + 1], P[3 * p + 2], cx, cy, cz), g)
                                  : kInfBits;
                }
#pragma unroll
                for (int u = 0; u < kGridU; ++u) {
                    unsigned long long mk = ballot(vv[u] < top);
                    while (mk) {
                        const int l = ffs64(mk);
                        mk &= mk - 1;
                        const unsigned v = readlane_u(vv[u], l);
                        if (v < top) {
                            h.adjust(0, K, v, readlane_u(pv[u], l));
                            top = h.gv(0);
                        }
                    }
                }
            }
            wave_sync();
        }
        emit_sorted(h.v, h.i, K, oi, od);
    }
}

// LDS bytes of a grid launch (grid_heap_select_kernel's layout)
static size_t grid_lds_bytes(int N, int max_cells) {
    const size_t nw = (size_t)(N + 31) / 32;
    return (size_t)max_cells * 4 + ((size_t)N * 2 + 15) / 16 * 16 + (size_t)kGridWaves * nw * 4 +
           (size_t)kGridWaves * kGridList * 2;
}

template <bool STAGE>
__global__ __launch_bounds__(256) void three_nn_kernel(Geo g) {
    extern __shared__ __attribute__((aligned(16))) float s_xyz[];
    const int b = blockIdx.y;
    const int M = g.N;
    const float* X = g.xyz + (size_t)b * M * 3;
    if (STAGE) {
        for (int t = threadIdx.x; t < M * 3; t += blockDim.x) s_xyz[t] = X[t];
        __syncthreads();
    }
    const float* P = STAGE ? s_xyz : X;
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= g.R) return;
    const float* c = g.cent + ((size_t)b * g.R + row) * 3;
    const float qx = c[0], qy = c[1], qz = c[2];
    H3 h;
    h.v0 = sqdist_unfused(P[0], P[1], P[2], qx, qy, qz);
    h.v1 = sqdist_unfused(P[3], P[4], P[5], qx, qy, qz);
    h.v2 = sqdist_unfused(P[6], P[7], P[8], qx, qy, qz);
    h.i0 = 0; h.i1 = 1; h.i2 = 2;
    {   // make_heap(3): adjust(hole 0, len 3, original h0)
        const float v = h.v0;
        const int i = h.i0;
        adjust3(h, v, i);
    }
    // candidates in pairs on packed fp32 ops (v_pk_add/mul_f32, no contraction): the same
    // un-fused ((dx*dx + dy*dy) + dz*dz) roundings per component, half the VALU issues;
    // the heap still takes them one at a time, in index order
    const f32x2 q2x = {qx, qx}, q2y = {qy, qy}, q2z = {qz, qz};
    int m = 3;
    for (; m + 2 <= M; m += 2) {
        const float* p = P + 3 * m;
        const f32x2 dx = f32x2{p[0], p[3]} - q2x;
        const f32x2 dy = f32x2{p[1], p[4]} - q2y;
        const f32x2 dz = f32x2{p[2], p[5]} - q2z;
        const f32x2 d = (dx * dx + dy * dy) + dz * dz;
        if (d.x < h.v0) adjust3(h, d.x, m);
        if (d.y < h.v0) adjust3(h, d.y, m + 1);
    }
    for (; m < M; ++m) {
        const float d = sqdist_unfused(P[3 * m], P[3 * m + 1], P[3 * m + 2], qx, qy, qz);
        if (d < h.v0) adjust3(h, d, m);
    }
    // canonical ascending (distance, index)
    float a0 = h.v0, a1 = h.v1, a2 = h.v2;
    int j0 = h.i0, j1 = h.i1, j2 = h.i2;
    float tv; int ti;
    if (lt_vi(a1, j1, a0, j0)) { tv = a0; a0 = a1; a1 = tv; ti = j0; j0 = j1; j1 = ti; }
    if (lt_vi(a2, j2, a1, j1)) { tv = a1; a1 = a2; a2 = tv; ti = j1; j1 = j2; j2 = ti; }
    if (lt_vi(a1, j1, a0, j0)) { tv = a0; a0 = a1; a1 = tv; ti = j0; j0 = j1; j1 = ti; }
    int* oi = g.out_idx + ((size_t)b * g.R + row) * 3;
    oi[0] = j0; oi[1] = j1; oi[2] = j2;
    if (g.out_dist) {
        float* od = g.out_dist + ((size_t)b * g.R + row) * 3;
        od[0] = a0; od[1] = a1; od[2] = a2;
    }
}

constexpr int kStageMaxPoints = 8192;  // 96 KB of LDS
// the grid kernel where the exhaustive heap kernel cannot stage the cloud in LDS (N > 8192: it then
// streams every point of the cloud from L2 for every centroid); up to 8192 points the staged
// exhaustive scan measured as fast (PointNet++ SA1: 312 vs 280 us, profiles/r06_ballq.txt)
constexpr int kGridMinPoints = kStageMaxPoints + 1;
constexpr size_t kGridLdsMax = 160 * 1024 - 1024;   // dynamic LDS cap (the kernel's static arrays take < 1 KB)
// one row per wave on both paths: a prefetched plan's blocks then retire quickly and let the step
// stream's kernels in (profiles/r05_ab_geometry_blocks.txt)
constexpr int kRowsPerWave = 1;

static int run_select(Geo g, hipStream_t s, const char* what) {
    PCS_CHECK_ARG(g.B >= 0 && g.R >= 0 && g.N >= 1 && g.K >= 1, "%s: bad sizes B=%d R=%d N=%d K=%d", what, g.B,
                  g.R, g.N, g.K);
    PCS_CHECK_ARG(g.K <= g.N, "%s: k=%d out of range for %d points (torch.topk raises)", what, g.K, g.N);
    PCS_CHECK_ARG(g.N <= 65535, "%s: N=%d exceeds 65535", what, g.N);
    if (g.B == 0 || g.R == 0) return 0;
    const bool heap_path = (long long)g.K * 64 <= g.N;
    const bool stage = g.N <= kStageMaxPoints;
    const size_t xyz_lds = stage ? ((size_t)g.N * 12 + 15) / 16 * 16 : 0;
    // algorithmic work per launch: R x N un-fused distances (8 flops each) per cloud; bytes =
    // both point sets read once + the neighbour lists written (SURVEY.md 8(d) neighbour-op model)
    const double flops = 8.0 * g.B * (double)g.R * g.N;
    const double bytes = 12.0 * g.B * ((double)g.N + g.R) + 4.0 * g.B * (double)g.R * g.K * (g.out_dist ? 2 : 1);
    if (heap_path && g.K == 3 && !g.use_radius) {
        const dim3 grid((g.R + 255) / 256, g.B);
        ProbeScope pr(s, flops, bytes, "pcs::three_nn_kernel<%s>", stage ? "true" : "false");
        if (stage) hipLaunchKernelGGL(three_nn_kernel<true>, grid, dim3(256), xyz_lds, s, g);
        else hipLaunchKernelGGL(three_nn_kernel<false>, grid, dim3(256), 0, s, g);
        return launch_status(what);
    }
    if (heap_path && g.use_radius && g.K <= 64 && g.N >= kGridMinPoints) {
        // ball query on the heap path: over the cell grid (grid_heap_select_kernel), when its LDS fits
        const int cells = 8192;
        const size_t lds = grid_lds_bytes(g.N, cells);
        if (lds <= kGridLdsMax) {
            // rows per wave: about one workgroup per CU over the launch (each builds its cloud's grid)
            const long long waves_total = (long long)kGridWaves * 256;
            const int rpw = (int)std::max<long long>(1, ((long long)g.B * g.R + waves_total - 1) / waves_total);
            const int waves = (g.R + rpw - 1) / rpw;
            const dim3 grid((waves + kGridWaves - 1) / kGridWaves, g.B);
            const float cs0 = (float)(std::sqrt((double)g.r2) * 1.02) + 1e-30f;
            ProbeScope pr(s, flops, bytes, "pcs::grid_heap_select_kernel");
            static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&grid_heap_select_kernel),
                                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGridLdsMax);
            (void)attr;
            hipLaunchKernelGGL(grid_heap_select_kernel, grid, dim3(kGridBlock), lds, s, g, cs0, cells, rpw);
            return launch_status(what);
        }
    }
    if (heap_path) {
        PCS_CHECK_ARG(g.K <= 64, "%s: k=%d > 64 not supported on the heap path", what, g.K);
        const int rows_per_wave = kRowsPerWave;
        const int waves = (g.R + rows_per_wave - 1) / rows_per_wave;
        constexpr int wpb = kHeapBlock / kWave;
        const dim3 grid((waves + wpb - 1) / wpb, g.B);
        ProbeScope pr(s, flops, bytes, "pcs::heap_select_kernel<%s>", stage ? "true" : "false");
        // (ball queries: per wave 64 * kFastS list entries + 64 output slots of 8 B after the cloud)
        const size_t hl = xyz_lds + (g.use_radius ? (size_t)wpb * (64 * kFastS + 64) * 8 : 0);
        if (stage) {
            static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&heap_select_kernel<true>),
                                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                                               (int)(kStageMaxPoints * 12 + wpb * (64 * kFastS + 64) * 8));
            (void)attr;
            hipLaunchKernelGGL(heap_select_kernel<true>, grid, dim3(kHeapBlock), hl, s, g, rows_per_wave);
        }
        else hipLaunchKernelGGL(heap_select_kernel<false>, grid, dim3(kHeapBlock), 0, s, g, rows_per_wave);
        return launch_status(what);
    }
    // intro path: n < 64k <= 4096 for k <= 64
    PCS_CHECK_ARG(g.K <= 64, "%s: k=%d > 64 not supported", what, g.K);
    const int rows_per_wave = kRowsPerWave;
    const int waves = (g.R + rows_per_wave - 1) / rows_per_wave;
    const size_t row_lds = (size_t)intro_row_bytes(g.N);
    int wpb = 4;
    while (wpb > 1 && xyz_lds + wpb * row_lds > 64 * 1024) wpb >>= 1;
    const dim3 grid((waves + wpb - 1) / wpb, g.B);
    const size_t lds = xyz_lds + wpb * row_lds;
    ProbeScope pr(s, flops, bytes, "pcs::intro_select_kernel<%s>", stage ? "true" : "false");
    if (stage) hipLaunchKernelGGL(intro_select_kernel<true>, grid, dim3(64 * wpb), lds, s, g, rows_per_wave);
    else hipLaunchKernelGGL(intro_select_kernel<false>, grid, dim3(64 * wpb), lds, s, g, rows_per_wave);
    return launch_status(what);
}

}  // namespace pcs

// Reference: models/utils/common.py:51-61 (distances, radius mask, topk).
// out_idx (B, C, K) int32: the reference's neighbour set per centroid.
PCS_API int pcs_ball_query(const float* centroids, const float* xyz, int B, int C, int N, float r2, int K,
                           int32_t* out_idx, void* stream) {
    PCS_CHECK_ARG(centroids && xyz && out_idx, "pcs_ball_query: null pointer");
    pcs::Geo g{centroids, xyz, B, C, N, K, r2, 1, out_idx, nullptr};
    return pcs::run_select(g, pcs::as_stream(stream), "pcs_ball_query");
}

// Reference: models/utils/common.py:107-114 (distances, topk(k) smallest).
// query (B, N, 3) = coords_1, ref (B, M, 3) = coords_2; out (B, N, k).
PCS_API int pcs_knn_select(const float* query, const float* ref, int B, int N, int M, int k, int32_t* out_idx,
                           float* out_dist, void* stream) {
    PCS_CHECK_ARG(query && ref && out_idx, "pcs_knn_select: null pointer");
    pcs::Geo g{query, ref, B, N, M, k, 0.f, 0, out_idx, out_dist};
    return pcs::run_select(g, pcs::as_stream(stream), "pcs_knn_select");
}
