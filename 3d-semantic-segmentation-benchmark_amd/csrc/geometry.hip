// Native geometry plan of a PointNet++-family forward: every neighbour structure of the
// network -- FPS per level (models/utils/common.py:6-34), its ball queries (common.py:37-61,
// against the previous level for SetAbstraction, against the centroids themselves for
// InvResMLP, common.py:288), the 3-NN of each FeaturePropagation (common.py:94-114) and the
// inverse (CSR) map of every neighbour table for the atomic-free gather backward -- enqueued
// by ONE host call on one stream (same kernels, same arguments as pcseg.common.GeometryPlan's
// Python path: bitwise the same plan), recording one caller event per level (the forward's SA
// level l waits on it) and one after the 3-NN.  With interp, every level's FPS and ball queries
// come first and the inverse maps (backward-only) after them, so a level's wait and the next
// level's FPS never queue behind a map.
//
// One call replaces ~20 Python-level launches (each with its own allocation, ctypes
// marshalling and caching-allocator stream bookkeeping): about 0.5 ms of host enqueue per
// PointNet++ step.  Outputs are caller-owned (one allocation on the Python side); the inverse
// maps share one scratch workspace, used in stream order.
#include "pcs_common.hpp"

#include <algorithm>

namespace pcs {

static size_t inv_scratch_bytes(long long n_slots, long long n_targets) {
    return ((size_t)n_slots * 4 + 255) / 256 * 256 + (size_t)n_targets * 4;
}

static int check_plan(int B, int N, const pcs_geo_level* lv, int L) {
    PCS_CHECK_ARG(B >= 1 && N >= 1 && lv && L >= 1 && L <= PCS_GEO_MAX_LEVELS, "pcs_geometry_plan: bad sizes B=%d N=%d L=%d",
                  B, N, L);
    int prev = N;
    for (int l = 0; l < L; ++l) {
        const pcs_geo_level& v = lv[l];
        PCS_CHECK_ARG(v.C >= 1 && v.C <= prev && v.nq >= 0 && v.nq <= PCS_GEO_MAX_QUERIES,
                      "pcs_geometry_plan: level %d: C=%lld nq=%lld (previous level %d points)", l, (long long)v.C,
                      (long long)v.nq, prev);
        for (int q = 0; q < v.nq; ++q) {
            const long long src = v.on_self[q] ? v.C : prev;
            PCS_CHECK_ARG(v.K[q] >= 1 && v.K[q] <= src && v.K[q] <= 64, "pcs_geometry_plan: level %d query %d: K=%lld", l,
                          q, (long long)v.K[q]);
        }
        prev = (int)v.C;
    }
    return 0;
}

// the inverse map of level v's ball query q (np = the previous level's point count)
static int ball_inverse(const pcs_geo_level& v, int q, int B, int np, void* ws, size_t ws_bytes, void* stream) {
    const int C = (int)v.C, K = (int)v.K[q], ns = v.on_self[q] ? C : np;
    PCS_CHECK_ARG(v.ball_off[q] && v.ball_ent[q], "pcs_geometry_plan: query %d: null map", q);
    return pcs_inverse_index(v.ball[q], B, C * K, ns, v.ball_off[q], v.ball_ent[q], ws, ws_bytes, stream);
}

}  // namespace pcs

using namespace pcs;

PCS_API int pcs_geometry_plan_workspace(int B, int N, const pcs_geo_level* lv, int L, int interp, int inverse,
                                        size_t* bytes) {
    if (int e = check_plan(B, N, lv, L)) return e;
    PCS_CHECK_ARG(bytes, "pcs_geometry_plan_workspace: null bytes");
    size_t m = 256;
    if (inverse) {
        long long prev = N;
        for (int l = 0; l < L; ++l) {
            for (int q = 0; q < lv[l].nq; ++q) {
                const long long src = lv[l].on_self[q] ? lv[l].C : prev;
                m = std::max(m, inv_scratch_bytes((long long)B * lv[l].C * lv[l].K[q], (long long)B * src));
            }
            if (interp) m = std::max(m, inv_scratch_bytes((long long)B * prev * 3, (long long)B * lv[l].C));
            prev = lv[l].C;
        }
    }
    *bytes = m;
    return 0;
}

// coords (B, N, 3); starts (L, B) int32 FPS start indices (the reference's torch.randint draw per
// level); lv[l]'s output pointers as documented in include/pcseg.h.
PCS_API int pcs_geometry_plan(const float* coords, int B, int N, const int32_t* starts, const pcs_geo_level* lv, int L,
                              int interp, int inverse, void* nn_event, void* ws, size_t ws_bytes, void* stream) {
    if (int e = check_plan(B, N, lv, L)) return e;
    size_t need = 0;
    pcs_geometry_plan_workspace(B, N, lv, L, interp, inverse, &need);
    PCS_CHECK_ARG(coords && starts && (ws || !inverse) && ws_bytes >= (inverse ? need : 0),
                  "pcs_geometry_plan: null pointer or workspace %zu < %zu bytes", ws_bytes, need);
    hipStream_t st = as_stream(stream);
    const float* prev = coords;
    int np = N;
    for (int l = 0; l < L; ++l) {
        const pcs_geo_level& v = lv[l];
        const int C = (int)v.C;
        PCS_CHECK_ARG(v.fps_idx && v.cent, "pcs_geometry_plan: level %d: null FPS output", l);
        if (int e = pcs_fps(prev, B, np, C, starts + (size_t)l * B, v.fps_idx, v.cent, stream)) return e;
        for (int q = 0; q < v.nq; ++q) {
            const float* src = v.on_self[q] ? v.cent : prev;
            const int ns = v.on_self[q] ? C : np;
            const int K = (int)v.K[q];
            PCS_CHECK_ARG(v.ball[q], "pcs_geometry_plan: level %d query %d: null ball output", l, q);
            if (int e = pcs_ball_query(v.cent, src, B, C, ns, (float)v.r2[q], K, v.ball[q], stream)) return e;
            if (inverse && !interp)
                if (int e = ball_inverse(v, q, B, np, ws, ws_bytes, stream)) return e;
        }
        if (v.event && hipEventRecord(static_cast<hipEvent_t>(v.event), st) != hipSuccess)
            return launch_status("pcs_geometry_plan: event record");
        prev = v.cent;
        np = C;
    }
    if (interp) {
        // the ball queries' inverse maps (read only by the backward) after every level's FPS and
        // ball queries: the forward's level-l wait then does not include them, nor does the next
        // level's FPS queue behind them; nn_event (after the 3-NN and their maps) covers them all
        np = N;
        for (int l = 0; l < L && inverse; ++l) {
            for (int q = 0; q < lv[l].nq; ++q)
                if (int e = ball_inverse(lv[l], q, B, np, ws, ws_bytes, stream)) return e;
            np = (int)lv[l].C;
        }
        // FP_L ... FP_1 (the reference's call order): 3-NN of level l's points among level l+1's
        for (int l = L - 1; l >= 0; --l) {
            const pcs_geo_level& v = lv[l];
            const float* fine = l == 0 ? coords : lv[l - 1].cent;
            const int nf = l == 0 ? N : (int)lv[l - 1].C;
            PCS_CHECK_ARG(v.nn_idx && v.nn_dist, "pcs_geometry_plan: level %d: null 3-NN output", l);
            if (int e = pcs_knn_select(fine, v.cent, B, nf, (int)v.C, 3, v.nn_idx, v.nn_dist, stream)) return e;
            if (inverse) {
                PCS_CHECK_ARG(v.nn_off && v.nn_ent, "pcs_geometry_plan: level %d: null 3-NN map", l);
                if (int e = pcs_inverse_index(v.nn_idx, B, nf * 3, (int)v.C, v.nn_off, v.nn_ent, ws, ws_bytes, stream))
                    return e;
            }
        }
        if (nn_event && hipEventRecord(static_cast<hipEvent_t>(nn_event), st) != hipSuccess)
            return launch_status("pcs_geometry_plan: event record");
    }
    return launch_status("pcs_geometry_plan");
}
