// Shared helpers for the TranSplat gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/transplat_hip.h"

namespace tsplat {
// tsplat_set_debug (capi.hip): synchronise + check after every launch
extern int g_debug;
int debug_check(const char* file, int line);
}  // namespace tsplat

#define TSPLAT_CHECK_LAUNCH()                                                      \
    do {                                                                           \
        hipError_t _e = hipGetLastError();                                         \
        if (_e != hipSuccess) return TSPLAT_EHIP;                                  \
        if (tsplat::g_debug && tsplat::debug_check(__FILE__, __LINE__) != 0)       \
            return TSPLAT_EHIP;                                                    \
    } while (0)

#define TSPLAT_CHECK(expr)                                           \
    do {                                                             \
        hipError_t _e = (expr);                                      \
        if (_e != hipSuccess) return TSPLAT_EHIP;                    \
    } while (0)

namespace tsplat {

constexpr int kWave = 64;

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

__host__ __device__ inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ inline size_t ceil_div(size_t a, size_t b) { return (a + b - 1) / b; }

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks that the dispatcher deals round-robin over the 8 XCDs are renumbered so that
// each XCD walks a contiguous range of logical tiles (neighbouring tiles share L2 lines).
__device__ inline int xcd_remap(int bid, int nwg) {
    const int nxcd = 8;
    if (nwg < nxcd) return bid;
    int q = nwg / nxcd, r = nwg % nxcd;
    int xcd = bid % nxcd;
    int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + bid / nxcd;
}

}  // namespace tsplat
