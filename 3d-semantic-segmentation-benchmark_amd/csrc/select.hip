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

// 1024-thread blocks: 16 waves share one staged cloud (48 KB at N = 4096), so LDS allows
// 8 waves per SIMD instead of 3 -- the heap surgery is a latency-bound chain of
// v_readlane / SALU hops per wave, and occupancy is what hides it.
constexpr int kHeapBlock = 1024;

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
    for (int rr = 0; rr < rows_per_wave; ++rr) {
        const int row = wave * rows_per_wave + rr;
        if (row >= g.R) break;
        const float* c = g.cent + ((size_t)b * g.R + row) * 3;
        const float cx = c[0], cy = c[1], cz = c[2];

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
        emit_sorted(h.v, h.i, K, g.out_idx + ((size_t)b * g.R + row) * K,
                    g.out_dist ? g.out_dist + ((size_t)b * g.R + row) * K : nullptr);
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
    if (heap_path) {
        PCS_CHECK_ARG(g.K <= 64, "%s: k=%d > 64 not supported on the heap path", what, g.K);
        const int rows_per_wave = kRowsPerWave;
        const int waves = (g.R + rows_per_wave - 1) / rows_per_wave;
        constexpr int wpb = kHeapBlock / kWave;
        const dim3 grid((waves + wpb - 1) / wpb, g.B);
        ProbeScope pr(s, flops, bytes, "pcs::heap_select_kernel<%s>", stage ? "true" : "false");
        if (stage) hipLaunchKernelGGL(heap_select_kernel<true>, grid, dim3(kHeapBlock), xyz_lds, s, g, rows_per_wave);
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
