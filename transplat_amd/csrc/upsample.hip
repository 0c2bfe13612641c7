// Bilinear upsampling (align_corners = True, integer factor) with the producing convolution's bias
// Built with -ffp-contract=off (transplat_amd/build.py): `hr - h0` contracted into
// fma(rh, oy, -h0) takes the interpolation weight from the unrounded source coordinate (up to one
// ulp of it, 1.5e-5 at 255) instead of torch's rounded one: 5.7e-5 off F.interpolate.
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

// Channels-last bilinear resize (align_corners = True, any output size): the DPT head's
// FeatureFusionBlock / final interpolations on its channels-last maps (reference
// src/depth_anything_v2/util/blocks.py FeatureFusionBlock.forward, dpt.py DPTHead.forward). One
// thread = one output pixel x 4 channels (float4 loads / stores along C).
__global__ void __launch_bounds__(256) bilinear_ac_nhwc_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                               int h, int w, int c4, int ho, int wo, float rh,
                                                               float rw, int total) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int cc = i % c4;
    const int pix = i / c4;
    const int ox = pix % wo;
    const int t = pix / wo;
    const int oy = t % ho, n = t / ho;
    const float hr = rh * (float)oy, wr = rw * (float)ox;
    const int h0 = (int)hr, w0 = (int)wr;
    const int h1 = h0 + (h0 < h - 1 ? 1 : 0), w1 = w0 + (w0 < w - 1 ? 1 : 0);
    const float l1 = hr - (float)h0, l0 = 1.f - l1, m1 = wr - (float)w0, m0 = 1.f - m1;
    const float4* src = reinterpret_cast<const float4*>(x) + (size_t)n * h * w * c4 + cc;
    const float4 a = src[((size_t)h0 * w + w0) * c4], b = src[((size_t)h0 * w + w1) * c4];
    const float4 cq = src[((size_t)h1 * w + w0) * c4], d = src[((size_t)h1 * w + w1) * c4];
    float4 o;
    o.x = l0 * (m0 * a.x + m1 * b.x) + l1 * (m0 * cq.x + m1 * d.x);
    o.y = l0 * (m0 * a.y + m1 * b.y) + l1 * (m0 * cq.y + m1 * d.y);
    o.z = l0 * (m0 * a.z + m1 * b.z) + l1 * (m0 * cq.z + m1 * d.z);
    o.w = l0 * (m0 * a.w + m1 * b.w) + l1 * (m0 * cq.w + m1 * d.w);
    reinterpret_cast<float4*>(y)[i] = o;
}

// F.interpolate(x, size, mode="bilinear", align_corners=True) on NCHW fp32 maps of any size (the
// DA-V2 input / depth resizes, reference encoder_trans.py, and the DINO feature resize,
// depth_predictor_trans.py): one thread per output element, consecutive threads along the output
// row (coalesced stores, neighbouring reads), so the work spreads over all N*C planes -- PyTorch's
// generic NCHW kernel loops over the N*C planes inside each output pixel's thread. Same
// arithmetic as torch's upsample_bilinear2d: source = dst * (in - 1) / (out - 1) in float.
__global__ void __launch_bounds__(256) bilinear_ac_nchw_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                               int h, int w, int ho, int wo, float rh, float rw,
                                                               size_t total) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int ox = (int)(i % wo);
    const size_t t = i / wo;
    const int oy = (int)(t % ho);
    const size_t plane = t / ho;
    const float hr = rh * (float)oy, wr = rw * (float)ox;
    const int h0 = (int)hr, w0 = (int)wr;
    const int h1 = h0 + (h0 < h - 1 ? 1 : 0), w1 = w0 + (w0 < w - 1 ? 1 : 0);
    const float l1 = hr - (float)h0, l0 = 1.f - l1, m1 = wr - (float)w0, m0 = 1.f - m1;
    const float* src = x + plane * h * w;
    const float a = src[(size_t)h0 * w + w0], b = src[(size_t)h0 * w + w1];
    const float cq = src[(size_t)h1 * w + w0], d = src[(size_t)h1 * w + w1];
    y[i] = l0 * (m0 * a + m1 * b) + l1 * (m0 * cq + m1 * d);
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

extern "C" int tsplat_resize_bilinear_nhwc_fwd(const float* x, float* y, int32_t n, int32_t height, int32_t width,
                                               int32_t c, int32_t out_height, int32_t out_width, void* stream_) {
    using namespace tsplat::upsample;
    if (!x || !y || n <= 0 || height <= 0 || width <= 0 || c <= 0 || c % 4 || out_height <= 0 || out_width <= 0)
        return TSPLAT_EINVAL;
    if ((uintptr_t)x % 16 || (uintptr_t)y % 16) return TSPLAT_EINVAL;
    const int64_t total64 = (int64_t)n * out_height * out_width * (c / 4);
    if (total64 >= (1ll << 31) || (int64_t)n * height * width * c >= (1ll << 31)) return TSPLAT_EINVAL;
    const int total = (int)total64;
    const float rh = out_height > 1 ? (float)(height - 1) / (float)(out_height - 1) : 0.f;
    const float rw = out_width > 1 ? (float)(width - 1) / (float)(out_width - 1) : 0.f;
    hipStream_t stream = (hipStream_t)stream_;
    hipLaunchKernelGGL(bilinear_ac_nhwc_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, x, y,
                       height, width, c / 4, out_height, out_width, rh, rw, total);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_resize_bilinear_nchw_fwd(const float* x, float* y, int32_t planes, int32_t height,
                                               int32_t width, int32_t out_height, int32_t out_width, void* stream_) {
    using namespace tsplat::upsample;
    if (!x || !y || planes <= 0 || height <= 0 || width <= 0 || out_height <= 0 || out_width <= 0)
        return TSPLAT_EINVAL;
    const size_t total = (size_t)planes * out_height * out_width;
    const float rh = out_height > 1 ? (float)(height - 1) / (float)(out_height - 1) : 0.f;
    const float rw = out_width > 1 ? (float)(width - 1) / (float)(out_width - 1) : 0.f;
    hipStream_t stream = (hipStream_t)stream_;
    hipLaunchKernelGGL(bilinear_ac_nchw_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, x, y,
                       height, width, out_height, out_width, rh, rw, total);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
