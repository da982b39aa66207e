// Launch probe of the engine GEMMs: while enabled (pcs_probe_begin .. pcs_probe_end),
// every pcs_gemm_rows / pcs_wgrad launch -- including those issued by pcs_mlp_forward /
// pcs_mlp_backward -- is bracketed by two HIP events recorded on the launch's own stream,
// together with the kernel name as rocprofv3 reports it and its algorithmic flops /
// bytes.  bench.py uses it for the live roofline of the dominant kernel.  Thread-safe:
// the autograd backward thread launches too.
#include <hip/hip_runtime.h>

#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "pcs_common.hpp"

namespace pcs {

struct ProbeRec {
    std::string name;
    double flops, bytes;
    hipEvent_t e0, e1;
    hipStream_t stream;
    std::function<void()> relaunch;   // the identical launch again (pcs_probe_replay)
};

static std::mutex g_probe_mu;
static bool g_probe_on = false;
static std::vector<ProbeRec> g_probe;

bool probe_enabled() { return g_probe_on; }

// returns the record index, or -1 (probe off / event failure); call before the launch
int probe_start(const char* name, double flops, double bytes, hipStream_t s, std::function<void()> relaunch) {
    if (!g_probe_on) return -1;
    ProbeRec r{name, flops, bytes, nullptr, nullptr, s, std::move(relaunch)};
    if (hipEventCreate(&r.e0) != hipSuccess || hipEventCreate(&r.e1) != hipSuccess) return -1;
    (void)hipEventRecord(r.e0, s);
    std::lock_guard<std::mutex> g(g_probe_mu);
    g_probe.push_back(r);
    return (int)g_probe.size() - 1;
}

void probe_stop(int idx, hipStream_t s) {
    if (idx < 0) return;
    hipEvent_t e;
    {
        std::lock_guard<std::mutex> g(g_probe_mu);
        e = g_probe[idx].e1;
    }
    (void)hipEventRecord(e, s);
}

static void probe_clear() {
    for (auto& r : g_probe) {
        (void)hipEventDestroy(r.e0);
        (void)hipEventDestroy(r.e1);
    }
    g_probe.clear();
}

// one wave sleeps until `ticks` of the 100 MHz realtime counter have passed
__global__ __launch_bounds__(64) void spin_kernel(unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(100);
}

}  // namespace pcs

using namespace pcs;

PCS_API int pcs_spin(int us, void* stream) {
    PCS_CHECK_ARG(us >= 0 && us <= 1000000, "pcs_spin: us=%d out of [0, 1e6]", us);
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, as_stream(stream), (unsigned long long)us * 100ull);
    return launch_status("pcs_spin");
}

PCS_API int pcs_probe_begin(void) {
    std::lock_guard<std::mutex> g(g_probe_mu);
    probe_clear();
    g_probe_on = true;
    return 0;
}

PCS_API int pcs_probe_end(void) {
    std::lock_guard<std::mutex> g(g_probe_mu);
    g_probe_on = false;
    return (int)g_probe.size();
}

// record i: kernel name (NUL-terminated, truncated to cap), algorithmic flops and bytes,
// elapsed milliseconds (waits for the stop event)
PCS_API int pcs_probe_get(int i, char* name, int cap, double* flops, double* bytes, float* ms) {
    hipEvent_t e0, e1;
    {
        std::lock_guard<std::mutex> g(g_probe_mu);
        PCS_CHECK_ARG(i >= 0 && i < (int)g_probe.size(), "pcs_probe_get: index %d of %zu", i, g_probe.size());
        const ProbeRec& r = g_probe[i];
        if (name && cap > 0) {
            strncpy(name, r.name.c_str(), cap - 1);
            name[cap - 1] = 0;
        }
        if (flops) *flops = r.flops;
        if (bytes) *bytes = r.bytes;
        e0 = r.e0;
        e1 = r.e1;
    }
    if (hipEventSynchronize(e1) != hipSuccess) return (int)hipErrorUnknown;
    float t = 0.f;
    const hipError_t err = hipEventElapsedTime(&t, e0, e1);
    if (err != hipSuccess) {
        set_error("pcs_probe_get: %s", hipGetErrorString(err));
        return (int)err;
    }
    if (ms) *ms = t;
    return 0;
}

// record i's stream (the hipStream_t its launch was enqueued on, as void*)
PCS_API int pcs_probe_stream(int i, void** stream) {
    std::lock_guard<std::mutex> g(g_probe_mu);
    PCS_CHECK_ARG(i >= 0 && i < (int)g_probe.size() && stream, "pcs_probe_stream: index %d of %zu", i,
                  g_probe.size());
    *stream = reinterpret_cast<void*>(g_probe[i].stream);
    return 0;
}

// record i's start and end in milliseconds after record 0's start (events on any stream of
// the device: the overlap of launches on different streams, e.g. a data gradient and the wgrad
// lane's weight gradient running beside it)
PCS_API int pcs_probe_times(int i, double* t0_ms, double* t1_ms) {
    hipEvent_t r0, e0, e1;
    {
        std::lock_guard<std::mutex> g(g_probe_mu);
        PCS_CHECK_ARG(i >= 0 && i < (int)g_probe.size() && t0_ms && t1_ms, "pcs_probe_times: index %d of %zu", i,
                      g_probe.size());
        r0 = g_probe[0].e0;
        e0 = g_probe[i].e0;
        e1 = g_probe[i].e1;
    }
    if (hipEventSynchronize(e1) != hipSuccess) return (int)hipErrorUnknown;
    float a = 0.f, b = 0.f;
    hipError_t err = hipEventElapsedTime(&a, r0, e0);
    if (err == hipSuccess) err = hipEventElapsedTime(&b, r0, e1);
    if (err != hipSuccess) {
        set_error("pcs_probe_times: %s", hipGetErrorString(err));
        return (int)err;
    }
    *t0_ms = a;
    *t1_ms = b;
    return 0;
}

// Re-issue every recorded launch of kernel `name` back to back, `reps` times (after one
// untimed pass), between two events on their stream: the average duration of one launch
// with the queue kept full, the figure rocprofv3 --stats reports as AverageNs for that
// kernel (the per-launch event brackets of a step also include launch gaps).  The
// launches rewrite their outputs (and accumulate into dW again): call after the timed run.
PCS_API int pcs_probe_replay(const char* name, int reps, float* us_per_launch, int* launches) {
    std::vector<ProbeRec> sel;
    {
        std::lock_guard<std::mutex> g(g_probe_mu);
        PCS_CHECK_ARG(!g_probe_on, "pcs_probe_replay: call after pcs_probe_end");
        for (const auto& r : g_probe)
            if (r.name == name && r.relaunch) sel.push_back(r);
    }
    PCS_CHECK_ARG(name && reps >= 1 && us_per_launch && !sel.empty(), "pcs_probe_replay: no launches of '%s'",
                  name ? name : "(null)");
    const hipStream_t s = sel[0].stream;
    for (const auto& r : sel) PCS_CHECK_ARG(r.stream == s, "pcs_probe_replay: launches of '%s' on different streams", name);
    for (const auto& r : sel) r.relaunch();
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return (int)hipErrorUnknown;
    (void)hipEventRecord(e0, s);
    for (int i = 0; i < reps; ++i)
        for (const auto& r : sel) r.relaunch();
    (void)hipEventRecord(e1, s);
    hipError_t err = hipEventSynchronize(e1);
    float ms = 0.f;
    if (err == hipSuccess) err = hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (err != hipSuccess) {
        set_error("pcs_probe_replay: %s", hipGetErrorString(err));
        return (int)err;
    }
    *us_per_launch = ms * 1e3f / (float)(reps * (int)sel.size());
    if (launches) *launches = (int)sel.size();
    return 0;
}
