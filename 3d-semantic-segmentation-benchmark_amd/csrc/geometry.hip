// Native geometry plan of a PointNet++-family forward: every neighbour structure of the
// network -- FPS per level (models/utils/common.py:6-34), its ball queries (common.py:37-61,
// against the previous level for SetAbstraction, against the centroids themselves for
// InvResMLP, common.py:288), the 3-NN of each FeaturePropagation (common.py:94-114) and the
// inverse (CSR) map of every neighbour table for the atomic-free gather backward -- enqueued
// by ONE host call on one stream (same kernels, same arguments as pcseg.common.GeometryPlan's
// Python path: bitwise the same plan), recording one caller event per level (the forward's SA
// level l waits on it) and one after the 3-NN.  With interp, every level's FPS and ball queries
// come first and the inverse maps (backward-only) after them, so a level's wait and the next
// level's FPS never queue behind a map: all maps are one batched call at the end.
//
// One call replaces ~20 Python-level launches (each with its own allocation, ctypes
// marshalling and caching-allocator stream bookkeeping): about 0.5 ms of host enqueue per
// PointNet++ step.  Outputs are caller-owned (one allocation on the Python side); the inverse
// maps share one scratch workspace, used in stream order.
#include "pcs_common.hpp"

#include <algorithm>

namespace pcs {

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

// every inverse map of the plan (ball queries level by level, then with interp the 3-NN
// tables FP_L .. FP_1), as one pcs_inverse_index_batch: 3 launches for all of them
static int plan_maps(int B, int N, const pcs_geo_level* lv, int L, int interp, pcs_inverse_map* maps, int* n) {
    int np = N, k = 0;
    for (int l = 0; l < L; ++l) {
        const pcs_geo_level& v = lv[l];
        for (int q = 0; q < v.nq; ++q) {
            PCS_CHECK_ARG(v.ball_off[q] && v.ball_ent[q], "pcs_geometry_plan: level %d query %d: null map", l, q);
            maps[k++] = pcs_inverse_map{v.ball[q], (int)(v.C * v.K[q]), v.on_self[q] ? (int)v.C : np, v.ball_off[q],
                                        v.ball_ent[q]};
        }
        np = (int)v.C;
    }
    if (interp)
        for (int l = L - 1; l >= 0; --l) {
            const pcs_geo_level& v = lv[l];
            const int nf = l == 0 ? N : (int)lv[l - 1].C;
            PCS_CHECK_ARG(v.nn_off && v.nn_ent, "pcs_geometry_plan: level %d: null 3-NN map", l);
            maps[k++] = pcs_inverse_map{v.nn_idx, nf * 3, (int)v.C, v.nn_off, v.nn_ent};
        }
    *n = k;
    return 0;
}

constexpr int kPlanMaps = PCS_GEO_MAX_LEVELS * (PCS_GEO_MAX_QUERIES + 1);

}  // namespace pcs

using namespace pcs;

PCS_API int pcs_geometry_plan_workspace(int B, int N, const pcs_geo_level* lv, int L, int interp, int inverse,
                                        size_t* bytes) {
    if (int e = check_plan(B, N, lv, L)) return e;
    PCS_CHECK_ARG(bytes, "pcs_geometry_plan_workspace: null bytes");
    size_t m = 256;
    if (inverse) {
        pcs_inverse_map maps[kPlanMaps];
        int n = 0;
        // sizes only: the output pointers may still be null here
        int np = N;
        for (int l = 0; l < L; ++l) {
            for (int q = 0; q < lv[l].nq; ++q)
                maps[n++] = pcs_inverse_map{nullptr, (int)(lv[l].C * lv[l].K[q]), lv[l].on_self[q] ? (int)lv[l].C : np,
                                            nullptr, nullptr};
            np = (int)lv[l].C;
        }
        if (interp)
            for (int l = L - 1; l >= 0; --l)
                maps[n++] = pcs_inverse_map{nullptr, (l == 0 ? N : (int)lv[l - 1].C) * 3, (int)lv[l].C, nullptr, nullptr};
        if (n)
            if (int e = pcs_inverse_index_batch_workspace(maps, n, B, &m)) return e;
        m = std::max(m, (size_t)256);
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
        }
        if (inverse && !interp && v.nq) {
            // no 3-NN: the level's maps before its event (the backward's wait covers them)
            pcs_inverse_map maps[PCS_GEO_MAX_QUERIES];
            for (int q = 0; q < v.nq; ++q) {
                PCS_CHECK_ARG(v.ball_off[q] && v.ball_ent[q], "pcs_geometry_plan: level %d query %d: null map", l, q);
                maps[q] = pcs_inverse_map{v.ball[q], C * (int)v.K[q], v.on_self[q] ? C : np, v.ball_off[q],
                                          v.ball_ent[q]};
            }
            if (int e = pcs_inverse_index_batch(maps, (int)v.nq, B, ws, ws_bytes, stream)) return e;
        }
        if (v.event && hipEventRecord(static_cast<hipEvent_t>(v.event), st) != hipSuccess)
            return launch_status("pcs_geometry_plan: event record");
        prev = v.cent;
        np = C;
    }
    if (interp) {
        // FP_L ... FP_1 (the reference's call order): 3-NN of level l's points among level l+1's
        for (int l = L - 1; l >= 0; --l) {
            const pcs_geo_level& v = lv[l];
            const float* fine = l == 0 ? coords : lv[l - 1].cent;
            const int nf = l == 0 ? N : (int)lv[l - 1].C;
            PCS_CHECK_ARG(v.nn_idx && v.nn_dist, "pcs_geometry_plan: level %d: null 3-NN output", l);
            if (int e = pcs_knn_select(fine, v.cent, B, nf, (int)v.C, 3, v.nn_idx, v.nn_dist, stream)) return e;
        }
    }
    if (inverse && interp) {
        // the inverse maps (read only by the backward) after every FPS, ball query and 3-NN: no
        // level's wait and no FPS queues behind them; nn_event (after them) covers them all
        pcs_inverse_map maps[kPlanMaps];
        int n = 0;
        if (int e = plan_maps(B, N, lv, L, interp, maps, &n)) return e;
        if (n)
            if (int e = pcs_inverse_index_batch(maps, n, B, ws, ws_bytes, stream)) return e;
    }
    if (interp && nn_event && hipEventRecord(static_cast<hipEvent_t>(nn_event), st) != hipSuccess)
        return launch_status("pcs_geometry_plan: event record");
    return launch_status("pcs_geometry_plan");
}
