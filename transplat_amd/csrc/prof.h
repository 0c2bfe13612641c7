// Optional per-kernel HIP-event timing (used by bench.py to measure one kernel's average launch
// duration on the stream it is launched on). Disabled by default: one branch per launch.
#pragma once

#include <hip/hip_ext.h>

#include "common.h"

namespace tsplat {
namespace prof {

enum KernelId : int {
    kNone = 0,
    kRasterPreprocess = 1,
    kRasterScan = 2,
    kRasterScatter = 3,
    kRasterRender = 4,
    kUvCoarse = 5,
    kUvCross = 6,
    kMsda = 7,
    kWinAttn = 8,
    kRasterAll = 9,   // the whole tsplat_raster_fwd launch sequence
    kGroupNorm = 10,  // both launches of tsplat_group_norm_fwd
    kUvCrossTable = 11,
    kLinear = 12,     // tsplat_linear_f32_fwd
    kMha = 13,        // tsplat_mha_f32_fwd
    kConv = 14,       // tsplat_conv2d_f32_fwd
    kWinoConv = 15,   // tsplat_conv3x3_wino_f32_fwd
    kGemmX3 = 16,     // tsplat_gemm_x3_fwd
    kNumKernels = 17,
};

int active();                 // kernel id being timed (0 = off)
void begin(int kid, hipStream_t s);
void end(int kid, hipStream_t s);

// Start / stop events for hipExtLaunchKernelGGL when `kid` is being timed (both null otherwise):
// the dispatch packet itself records them, so the pair brackets the kernel's execution as
// rocprof's dispatch timestamps do, without the separate event packets' dispatch gap.
struct ExtEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
ExtEvents ext_events(int kid);

}  // namespace prof
}  // namespace tsplat

#define TSPLAT_PROF_BEGIN(kid, s) \
    if (::tsplat::prof::active() == (kid)) ::tsplat::prof::begin((kid), (s))
#define TSPLAT_PROF_END(kid, s) \
    if (::tsplat::prof::active() == (kid)) ::tsplat::prof::end((kid), (s))
