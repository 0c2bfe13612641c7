// Gaussian adapter: raw per-pixel head output -> world-space Gaussians, one thread per pixel.
//
// Fuses the reference's stage 5 (src/model/encoder/encoder_trans.py:294-353) and
// GaussianAdapter.forward (src/model/encoder/common/gaussian_adapter.py:48-96): sigmoid pixel
// offset, camera ray (get_world_rays, src/geometry/projection.py:91-114), means = o + d * depth,
// scale = (min + (max - min) sigmoid) * depth * multiplier, normalised xyzw quaternion ->
// R diag(s^2) R^T (gaussians.py:7-43) rotated to world by c2w, SH * mask rotated by the
// per-camera block-diagonal Wigner-D (misc/sh_rotation.py), opacity = map_pdf_to_opacity / gpp.
// The reference runs this as ~40 PyTorch launches including batched 3x3 GEMMs over 131k
// matrices (5.7 ms per scene measured on MI355X in r1); here it is one bandwidth-bound pass:
// 84 floats in, 88 floats out per Gaussian.
#include "common.h"
#include "prof.h"

namespace tsplat {
namespace adapter {

constexpr int kThreads = 256;
constexpr int kMaxSh = 25;

struct Params {
    int B, V, H, W, R, dsh;
    float smin, smax, op_exp, inv_gpp;
    int nchw;  // raw is the head's [(v b), R, H*W] map (channel stride H*W) instead of [b, v, HW, R]
};

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + __expf(-x)); }

// cams per (b, v): c2w R row-major (9), c2w t (3), K^-1 of the normalised intrinsics (9),
// scale multiplier (1)
template <int DSH>
__global__ void __launch_bounds__(kThreads)
adapter_kernel(Params p, const float* __restrict__ raw, const float* __restrict__ depths,
               const float* __restrict__ densities, const float* __restrict__ cams,
               const float* __restrict__ shrot, float* __restrict__ means, float* __restrict__ cov,
               float* __restrict__ harm, float* __restrict__ opac) {
    const int hw = p.H * p.W;
    const int bv = blockIdx.y;
    const int pix = blockIdx.x * kThreads + threadIdx.x;
    if (pix >= hw) return;
    const int b = bv / p.V, v = bv - b * p.V;
    const float* c = cams + (size_t)bv * 22;
    // channel k of this pixel's raw vector is r[k * cs]
    const size_t cs = p.nchw ? (size_t)hw : 1;
    const float* r = p.nchw ? raw + (size_t)(v * p.B + b) * p.R * hw + pix : raw + ((size_t)bv * hw + pix) * p.R;
    const size_t gi = (size_t)b * p.V * hw + (size_t)v * hw + pix;  // output index (b, v*HW + pix)
    const float depth = depths[(size_t)bv * hw + pix];

    // pixel-centre ray coordinate + learned sub-pixel offset
    const int py = pix / p.W, px = pix - py * p.W;
    const float fw = (float)p.W, fh = (float)p.H;
    const float x = ((float)px + 0.5f) / fw + (sigmoidf(r[0]) - 0.5f) * (1.0f / fw);
    const float y = ((float)py + 0.5f) / fh + (sigmoidf(r[cs]) - 0.5f) * (1.0f / fh);
    const float* ki = c + 12;
    float d0 = ki[0] * x + ki[1] * y + ki[2];
    float d1 = ki[3] * x + ki[4] * y + ki[5];
    float d2 = ki[6] * x + ki[7] * y + ki[8];
    const float dn = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
    d0 /= dn; d1 /= dn; d2 /= dn;
    const float* Rc = c;
    const float w0 = Rc[0] * d0 + Rc[1] * d1 + Rc[2] * d2;
    const float w1 = Rc[3] * d0 + Rc[4] * d1 + Rc[5] * d2;
    const float w2 = Rc[6] * d0 + Rc[7] * d1 + Rc[8] * d2;
    means[gi * 3 + 0] = c[9] + w0 * depth;
    means[gi * 3 + 1] = c[10] + w1 * depth;
    means[gi * 3 + 2] = c[11] + w2 * depth;

    // scales and quaternion -> covariance
    const float mult = c[21];
    float s[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) s[i] = (p.smin + (p.smax - p.smin) * sigmoidf(r[(2 + i) * cs])) * depth * mult;
    float qi = r[5 * cs], qj = r[6 * cs], qk = r[7 * cs], qr = r[8 * cs];
    const float qn = sqrtf(qi * qi + qj * qj + qk * qk + qr * qr) + 1e-8f;
    qi /= qn; qj /= qn; qk /= qn; qr /= qn;
    const float two_s = 2.0f / (qi * qi + qj * qj + qk * qk + qr * qr + 1e-8f);
    float Q[9] = {1 - two_s * (qj * qj + qk * qk), two_s * (qi * qj - qk * qr), two_s * (qi * qk + qj * qr),
                  two_s * (qi * qj + qk * qr), 1 - two_s * (qi * qi + qk * qk), two_s * (qj * qk - qi * qr),
                  two_s * (qi * qk - qj * qr), two_s * (qj * qk + qi * qr), 1 - two_s * (qi * qi + qj * qj)};
    // M = Rc Q diag(s): world covariance = M M^T
    float M[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            M[3 * i + j] = (Rc[3 * i] * Q[j] + Rc[3 * i + 1] * Q[3 + j] + Rc[3 * i + 2] * Q[6 + j]) * s[j];
    float* cv = cov + gi * 9;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            cv[3 * i + j] = M[3 * i] * M[3 * j] + M[3 * i + 1] * M[3 * j + 1] + M[3 * i + 2] * M[3 * j + 2];

    // SH: mask (0.1 * 0.25^l for l >= 1) then the block-diagonal rotation (fully unrolled)
    const float* D = shrot + (size_t)bv * DSH * DSH;
    float* hout = harm + gi * 3 * DSH;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        float sh[DSH];
        const float* rs = r + (9 + ch * DSH) * cs;
#pragma unroll
        for (int k = 0; k < DSH; ++k) {
            const int l = k < 1 ? 0 : (k < 4 ? 1 : (k < 9 ? 2 : (k < 16 ? 3 : 4)));
            const float mask = l == 0 ? 1.0f : (l == 1 ? 0.025f : (l == 2 ? 0.00625f : (l == 3 ? 0.0015625f : 0.000390625f)));
            sh[k] = rs[k * cs] * mask;
        }
#pragma unroll
        for (int ll = 0; ll * ll < DSH; ++ll) {
            const int o = ll * ll, n = 2 * ll + 1;
#pragma unroll
            for (int i = 0; i < n; ++i) {
                float acc = 0.f;
#pragma unroll
                for (int j = 0; j < n; ++j) acc += D[(o + i) * DSH + o + j] * sh[o + j];
                hout[ch * DSH + o + i] = acc;
            }
        }
    }

    // opacity = map_pdf_to_opacity(density) / gaussians_per_pixel
    const float pdf = densities[(size_t)bv * hw + pix];
    const float e = p.op_exp;
    opac[gi] = 0.5f * (1.0f - powf(1.0f - pdf, e) + powf(pdf, 1.0f / e)) * p.inv_gpp;
}

}  // namespace adapter
}  // namespace tsplat

using namespace tsplat;

extern "C" int tsplat_gaussian_adapter_fwd(const float* raw, const float* depths, const float* densities,
                                           const float* cams, const float* sh_rot, float* means,
                                           float* cov, float* harmonics, float* opacities, int32_t batch,
                                           int32_t views, int32_t height, int32_t width, int32_t raw_ch,
                                           int32_t d_sh, float scale_min, float scale_max,
                                           float opacity_exponent, int32_t gaussians_per_pixel,
                                           int32_t raw_nchw, void* stream_) {
    using namespace tsplat::adapter;
    if (!raw || !depths || !densities || !cams || !sh_rot || !means || !cov || !harmonics || !opacities)
        return TSPLAT_EINVAL;
    if (batch <= 0 || views <= 0 || height <= 0 || width <= 0 || d_sh <= 0 || d_sh > kMaxSh ||
        raw_ch != 9 + 3 * d_sh || gaussians_per_pixel != 1 || opacity_exponent <= 0.f)
        return TSPLAT_EINVAL;
    Params p{batch, views, height, width, raw_ch, d_sh, scale_min, scale_max, opacity_exponent,
             1.0f / (float)gaussians_per_pixel, raw_nchw ? 1 : 0};
    hipStream_t stream = (hipStream_t)stream_;
    dim3 grid(ceil_div(height * width, kThreads), batch * views);
#define TSPLAT_ADAPTER_LAUNCH(N)                                                                     \
    case N:                                                                                          \
        hipLaunchKernelGGL(adapter_kernel<N>, grid, dim3(kThreads), 0, stream, p, raw, depths, densities, \
                           cams, sh_rot, means, cov, harmonics, opacities);                          \
        break;
    switch (d_sh) {
        TSPLAT_ADAPTER_LAUNCH(1)
        TSPLAT_ADAPTER_LAUNCH(4)
        TSPLAT_ADAPTER_LAUNCH(9)
        TSPLAT_ADAPTER_LAUNCH(16)
        TSPLAT_ADAPTER_LAUNCH(25)
        default:
            return TSPLAT_EINVAL;
    }
#undef TSPLAT_ADAPTER_LAUNCH
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
