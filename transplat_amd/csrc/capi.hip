// Library identification + the kernel-timing facility of the C-ABI (include/transplat_hip.h).
#include <stdio.h>

#include <vector>

#include "prof.h"

namespace tsplat {
namespace prof {

static int g_active = kNone;
static std::vector<hipEvent_t> g_ev;  // begin/end pairs
static size_t g_used = 0;             // events recorded
static bool g_open = false;

int active() { return g_active; }

static hipEvent_t next_event() {
    if (g_used >= g_ev.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        g_ev.push_back(e);
    }
    return g_ev[g_used++];
}

void begin(int, hipStream_t s) {
    if (g_open) return;
    hipEvent_t e = next_event();
    if (e) {
        hipEventRecord(e, s);
        g_open = true;
    }
}

void end(int, hipStream_t s) {
    if (!g_open) return;
    hipEvent_t e = next_event();
    if (e) hipEventRecord(e, s);
    g_open = false;
}

ExtEvents ext_events(int kid) {
    ExtEvents r;
    if (g_active != kid || g_open) return r;
    const size_t used = g_used;
    r.start = next_event();
    r.stop = next_event();
    if (!r.start || !r.stop) {  // keep begin / end pairs aligned
        g_used = used;
        r = ExtEvents{};
    }
    return r;
}

}  // namespace prof
}  // namespace tsplat

namespace tsplat {
int g_debug = 0;

int debug_check(const char* file, int line) {
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) return 0;
    fprintf(stderr, "[tsplat debug] %s:%d: %s\n", file, line, hipGetErrorString(e));
    return -1;
}
}  // namespace tsplat

extern "C" int tsplat_version(void) { return 1; }

extern "C" int tsplat_set_debug(int32_t on) {
    const int was = tsplat::g_debug;
    tsplat::g_debug = on != 0;
    return was;
}

extern "C" int tsplat_prof_enable(int32_t kernel_id) {
    using namespace tsplat::prof;
    if (kernel_id < 0 || kernel_id >= kNumKernels) return TSPLAT_EINVAL;
    g_active = kernel_id;
    g_used = 0;
    g_open = false;
    return TSPLAT_OK;
}

extern "C" int tsplat_prof_read(double* total_ms, int32_t* launches) {
    using namespace tsplat::prof;
    if (!total_ms || !launches) return TSPLAT_EINVAL;
    double tot = 0.0;
    int n = 0;
    for (size_t i = 0; i + 1 < g_used; i += 2) {
        if (hipEventSynchronize(g_ev[i + 1]) != hipSuccess) return TSPLAT_EHIP;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, g_ev[i], g_ev[i + 1]) != hipSuccess) return TSPLAT_EHIP;
        tot += ms;
        ++n;
    }
    *total_ms = tot;
    *launches = n;
    g_used = 0;
    g_open = false;
    return TSPLAT_OK;
}

// Diagnostic stage marks (tools/graph_stages.py, TSPLAT_MARKS=1): one lane writes the 100-MHz
// wall clock into buf[slot] when the launch runs on `stream` -- captured into a hipGraph like any
// launch, so the stage boundaries of a replayed step can be read back per stream
namespace tsplat {
__global__ void stamp_kernel(unsigned long long* buf, int slot) {
    if (threadIdx.x == 0) buf[slot] = wall_clock64();
}
}  // namespace tsplat

extern "C" int tsplat_timestamp(void* buf, int32_t slot, void* stream) {
    if (!buf || slot < 0) return TSPLAT_EINVAL;
    hipLaunchKernelGGL(tsplat::stamp_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (unsigned long long*)buf, slot);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
