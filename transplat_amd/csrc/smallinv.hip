// Batched inverses of tiny (2x2, 3x3, 4x4) fp32 matrices: the camera algebra of the encoder and
// decoder (pose inverses, K^-1, img2world, the rasterizer's view matrix; reference
// depth_predictor_trans.py:36-49,88-98, encoder_trans.py:181-190, cuda_splatting.py:93-96 call
// torch.inverse on them). One thread per matrix, Gauss-Jordan with partial pivoting (the
// LU-with-pivoting family torch.linalg.inv uses; results agree to rounding). One launch replaces
// rocsolver's getrf + getri chain of ~6 small launches per call site.
#include "common.h"

namespace tsplat {
namespace smallinv {

template <int D>
__global__ void __launch_bounds__(256) inverse_kernel(const float* __restrict__ in, float* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float a[D][2 * D];
#pragma unroll
    for (int r = 0; r < D; ++r)
#pragma unroll
        for (int c = 0; c < D; ++c) {
            a[r][c] = in[(size_t)i * D * D + r * D + c];
            a[r][D + c] = r == c ? 1.0f : 0.0f;
        }
#pragma unroll
    for (int col = 0; col < D; ++col) {
        // partial pivoting: the row with the largest |a[r][col]| among r >= col (static indices)
        int piv = col;
        float best = fabsf(a[col][col]);
#pragma unroll
        for (int r = col + 1; r < D; ++r)
            if (fabsf(a[r][col]) > best) {
                best = fabsf(a[r][col]);
                piv = r;
            }
#pragma unroll
        for (int r = col + 1; r < D; ++r) {
            if (r == piv) {
#pragma unroll
                for (int c = 0; c < 2 * D; ++c) {
                    const float t = a[col][c];
                    a[col][c] = a[r][c];
                    a[r][c] = t;
                }
            }
        }
        const float inv = 1.0f / a[col][col];
#pragma unroll
        for (int c = 0; c < 2 * D; ++c) a[col][c] *= inv;
#pragma unroll
        for (int r = 0; r < D; ++r) {
            if (r == col) continue;
            const float f = a[r][col];
#pragma unroll
            for (int c = 0; c < 2 * D; ++c) a[r][c] -= f * a[col][c];
        }
    }
#pragma unroll
    for (int r = 0; r < D; ++r)
#pragma unroll
        for (int c = 0; c < D; ++c) out[(size_t)i * D * D + r * D + c] = a[r][D + c];
}

}  // namespace smallinv
}  // namespace tsplat

extern "C" int tsplat_small_inverse(const float* in, float* out, int32_t n, int32_t dim, void* stream_) {
    using namespace tsplat::smallinv;
    if (!in || !out || n < 0 || dim < 2 || dim > 4) return TSPLAT_EINVAL;
    if (n == 0) return TSPLAT_OK;
    hipStream_t stream = (hipStream_t)stream_;
    const dim3 grid((n + 255) / 256);
    if (dim == 2)
        hipLaunchKernelGGL(inverse_kernel<2>, grid, dim3(256), 0, stream, in, out, n);
    else if (dim == 3)
        hipLaunchKernelGGL(inverse_kernel<3>, grid, dim3(256), 0, stream, in, out, n);
    else
        hipLaunchKernelGGL(inverse_kernel<4>, grid, dim3(256), 0, stream, in, out, n);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
