// Bilinear upsampling (align_corners = True, integer factor) with the producing convolution's bias
// and the following activation in one pass, on gfx950.
//
// Semantics: reference src/model/encoder/matching/depth_predictor_trans.py (upsampler =
// Sequential(Conv2d, Upsample(scale_factor=4, mode="bilinear", align_corners=True), GELU)):
//   y = act(interpolate(conv_nobias(x)) + bias[c])
// the bias commutes with the interpolation (the four weights sum to 1). Index math follows
// torch's upsample_bilinear2d for align_corners: src = o * (in - 1) / (out - 1), i1 = i0 + (i0 < in - 1).
// HBM-bound: reads the small map (L2-resident), writes the 16x larger one once, float4 stores
// (4 consecutive output columns per thread) -- instead of the interpolation kernel plus a separate
// GELU pass over the full-resolution map.
#include "common.h"

namespace tsplat {
namespace upsample {

template <int ACT>
__device__ __forceinline__ float act(float v) {
    if (ACT == 2) return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));  // GELU (erf)
    if (ACT == 3) return fmaxf(v, 0.f);
    return v;
}

template <int ACT>
__global__ void __launch_bounds__(256) bilinear_ac_kernel(const float* __restrict__ x, const float* __restrict__ bias,
                                                          float* __restrict__ y, int c, int h, int w, int ho, int wo,
                                                          float rh, float rw, int total4) {
    // 32-bit index math (total4 < 2^31 checked on the host): 64-bit divisions cost ~100 VALU ops
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total4) return;
    const int wo4 = wo >> 2;
    const int rowi = i / wo4;
    const int ox0 = (i - rowi * wo4) * 4;
    const int nc = rowi / ho;
    const int oy = rowi - nc * ho;
    const float* src = x + (size_t)nc * h * w;
    const float b = bias ? bias[nc % c] : 0.f;
    const float hr = rh * (float)oy;
    const int h0 = (int)hr;
    const int h1 = h0 + (h0 < h - 1 ? 1 : 0);
    const float l1 = hr - (float)h0, l0 = 1.f - l1;
    const float* r0 = src + (long)h0 * w;
    const float* r1 = src + (long)h1 * w;
    float out[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float wr = rw * (float)(ox0 + j);
        const int w0 = (int)wr;
        const int w1 = w0 + (w0 < w - 1 ? 1 : 0);
        const float m1 = wr - (float)w0, m0 = 1.f - m1;
        const float v = l0 * (m0 * r0[w0] + m1 * r0[w1]) + l1 * (m0 * r1[w0] + m1 * r1[w1]);
        out[j] = act<ACT>(v + b);
    }
    *reinterpret_cast<float4*>(y + (size_t)rowi * wo + ox0) = make_float4(out[0], out[1], out[2], out[3]);
}

}  // namespace upsample
}  // namespace tsplat

extern "C" int tsplat_upsample_bilinear_act_fwd(const float* x, const float* bias, float* y, int32_t n, int32_t c,
                                                int32_t height, int32_t width, int32_t scale, int32_t act,
                                                void* stream_) {
    using namespace tsplat::upsample;
    if (!x || !y || n <= 0 || c <= 0 || height <= 0 || width <= 0 || scale < 1) return TSPLAT_EINVAL;
    const int ho = height * scale, wo = width * scale;
    if (wo % 4) return TSPLAT_EINVAL;
    const int64_t total4_64 = (int64_t)n * c * ho * (wo / 4);
    if (total4_64 >= (1ll << 31)) return TSPLAT_EINVAL;
    const int total4 = (int)total4_64;
    // align_corners = True scale, as torch computes it in float: (in - 1) / (out - 1)
    const float rh = ho > 1 ? (float)(height - 1) / (float)(ho - 1) : 0.f;
    const float rw = wo > 1 ? (float)(width - 1) / (float)(wo - 1) : 0.f;
    hipStream_t stream = (hipStream_t)stream_;
    const dim3 grid((unsigned)((total4 + 255) / 256)), block(256);
    switch (act) {
        case 0: hipLaunchKernelGGL(bilinear_ac_kernel<0>, grid, block, 0, stream, x, bias, y, c, height, width, ho, wo, rh, rw, total4); break;
        case 2: hipLaunchKernelGGL(bilinear_ac_kernel<2>, grid, block, 0, stream, x, bias, y, c, height, width, ho, wo, rh, rw, total4); break;
        case 3: hipLaunchKernelGGL(bilinear_ac_kernel<3>, grid, block, 0, stream, x, bias, y, c, height, width, ho, wo, rh, rw, total4); break;
        default: return TSPLAT_EINVAL;
    }
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
