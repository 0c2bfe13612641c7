// Split-bf16 ("bf16x3") operand preparation for library GEMMs: x [rows, k] fp32 ->
// [rows, 3k] bf16 = [hi | hi | lo] (hi = bf16(x), lo = bf16(x - hi)). With the weight packed once as
// [W_hi | W_lo | W_hi] ([n, 3k]), ONE bf16 GEMM with fp32 accumulation and fp32 output computes
// x_hi W_hi + x_hi W_lo + x_lo W_hi = x W^T to <= 3 * 2^-18 relative per product: the nn.Linear
// layers of the fp32 path (DINOv2 qkv / proj / fc1 / fc2, reference src/depth_anything_v2/
// dinov2_layers/{attention,mlp}.py; the transformer FFN's mlp[0], multiview_transformer.py:327-407)
// in the stand-in for the reference's TF32 matmuls (src/main.py:15).
#include "common.h"

namespace tsplat {
namespace split {

__device__ __forceinline__ uint32_t bits(float v) { return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v); }

// one thread = 4 consecutive elements of a row (k % 4 == 0): one float4 in, three 8-B stores out
__global__ void __launch_bounds__(256) split3_kernel(const float4* __restrict__ x, uint2* __restrict__ out,
                                                     long long quads, int kq) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= quads) return;
    const long long row = i / kq;
    const int q = (int)(i - row * kq);
    const float4 v = x[i];
    const uint32_t h0 = bits(v.x) | (bits(v.y) << 16), h1 = bits(v.z) | (bits(v.w) << 16);
    const float r0 = v.x - __builtin_bit_cast(float, h0 << 16), r1 = v.y - __builtin_bit_cast(float, h0 & 0xffff0000u);
    const float r2 = v.z - __builtin_bit_cast(float, h1 << 16), r3 = v.w - __builtin_bit_cast(float, h1 & 0xffff0000u);
    const uint2 hi = make_uint2(h0, h1);
    const uint2 lo = make_uint2(bits(r0) | (bits(r1) << 16), bits(r2) | (bits(r3) << 16));
    uint2* o = out + row * 3 * kq + q;
    o[0] = hi;
    o[kq] = hi;
    o[2 * kq] = lo;
}

// weights [n, k] fp32 -> [n, 3k] bf16 = [hi | lo | hi]
__global__ void __launch_bounds__(256) split3_weight_kernel(const float4* __restrict__ w, uint2* __restrict__ out,
                                                            long long quads, int kq) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= quads) return;
    const long long row = i / kq;
    const int q = (int)(i - row * kq);
    const float4 v = w[i];
    const uint32_t h0 = bits(v.x) | (bits(v.y) << 16), h1 = bits(v.z) | (bits(v.w) << 16);
    const float r0 = v.x - __builtin_bit_cast(float, h0 << 16), r1 = v.y - __builtin_bit_cast(float, h0 & 0xffff0000u);
    const float r2 = v.z - __builtin_bit_cast(float, h1 << 16), r3 = v.w - __builtin_bit_cast(float, h1 & 0xffff0000u);
    const uint2 hi = make_uint2(h0, h1);
    const uint2 lo = make_uint2(bits(r0) | (bits(r1) << 16), bits(r2) | (bits(r3) << 16));
    uint2* o = out + row * 3 * kq + q;
    o[0] = hi;
    o[kq] = lo;
    o[2 * kq] = hi;
}

}  // namespace split
}  // namespace tsplat

using namespace tsplat;

extern "C" int tsplat_split_bf16x3(const float* x, void* out, int64_t rows, int32_t k, int32_t weight_order,
                                   void* stream_) {
    if (!x || !out || rows <= 0 || k <= 0 || k % 4) return TSPLAT_EINVAL;
    const long long quads = rows * (long long)(k / 4);
    const dim3 grid((unsigned)((quads + 255) / 256));
    if (weight_order)
        hipLaunchKernelGGL(split::split3_weight_kernel, grid, dim3(256), 0, (hipStream_t)stream_,
                           (const float4*)x, (uint2*)out, quads, k / 4);
    else
        hipLaunchKernelGGL(split::split3_kernel, grid, dim3(256), 0, (hipStream_t)stream_, (const float4*)x,
                           (uint2*)out, quads, k / 4);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
