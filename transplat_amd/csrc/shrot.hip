// Per-camera real-SH rotation matrices (block-diagonal Wigner-D, degrees 0..4), one workgroup per
// camera, float64 inside.
//
// Restates misc/sh_rotation.py (the e3nn construction the reference calls in
// src/misc/sh_rotation.py:10-30): (alpha, beta, gamma) = matrix_to_angles(R) (Y-X-Y Euler angles
// read off R e_y), D^l = exp(alpha X_y) exp(beta X_x) exp(gamma X_y). In e3nn's real basis the
// y-rotation exp(t X_y) has two non-zeros per row -- cos(|m| t) on the diagonal and +-sin(|m| t)
// on the anti-diagonal -- and exp(t X_x) = P exp(t X_y) P^T with the constant P^l = exp(-pi/2 X_z)
// (host-computed once, `basis`). So D^l = Z(alpha) P Z(beta) P^T Z(gamma): two dense (2l+1)^3
// products plus sparse row/column mixes, instead of the ~600 tiny float64 GEMM / elementwise
// launches the matrix-exponential form costs per forward.
#include "common.h"

namespace tsplat {
namespace shrot {

constexpr int kThreads = 64;
constexpr int kMaxDeg = 4;
constexpr int kMaxN = 2 * kMaxDeg + 1;

// entry (r, c) of exp(t X_y) for degree l (indices 0..2l, m = index - l)
__device__ __forceinline__ double zrot(const double* cs, const double* sn, int l, int r, int c) {
    const int m = r - l;
    const int k = m < 0 ? -m : m;
    if (r == c) return cs[k];
    if (c == 2 * l - r) return m < 0 ? sn[k] : -sn[k];
    return 0.0;
}

__global__ void __launch_bounds__(kThreads)
shrot_kernel(const float* __restrict__ rot, const double* __restrict__ basis, float* __restrict__ out,
             int dsh, int ndeg) {
    __shared__ double ang[3];
    __shared__ double cs[3][kMaxN], sn[3][kMaxN];  // cos/sin(k * angle), k = 0..4
    __shared__ double A[kMaxN * kMaxN], T[kMaxN * kMaxN];
    const int cam = blockIdx.x;
    const int tid = threadIdx.x;
    const float* R = rot + 9 * cam;
    float* D = out + (size_t)cam * dsh * dsh;

    if (tid == 0) {
        // matrix_to_angles: x = normalize(R e_y); beta = acos(x_y); alpha = atan2(x_x, x_z);
        // gamma from the residual (Y(alpha) X(beta))^T R
        double x0 = R[1], x1 = R[4], x2 = R[7];
        const double nrm = fmax(sqrt(x0 * x0 + x1 * x1 + x2 * x2), 1e-12);
        x0 = fmin(fmax(x0 / nrm, -1.0), 1.0);
        x1 = fmin(fmax(x1 / nrm, -1.0), 1.0);
        x2 = fmin(fmax(x2 / nrm, -1.0), 1.0);
        const double b = acos(x1), a = atan2(x0, x2);
        const double ca = cos(a), sa = sin(a);
        // M = Y(a) X(b); rr = M^T R; only row 0 of rr is needed: rr[0][j] = sum_i M[i][0] R[i][j]
        // Y(a) = [[ca,0,sa],[0,1,0],[-sa,0,ca]], X(b) = [[1,0,0],[0,cb,-sb],[0,sb,cb]]
        // M[:,0] = Y(a) X(b) e_x = Y(a) e_x = (ca, 0, -sa)
        const double r00 = ca * R[0] - sa * R[6];
        const double r02 = ca * R[2] - sa * R[8];
        ang[0] = a;
        ang[1] = b;
        ang[2] = atan2(r02, r00);
    }
    __syncthreads();
    if (tid < 3 * (kMaxDeg + 1)) {
        const int which = tid / (kMaxDeg + 1), k = tid % (kMaxDeg + 1);
        const double t = ang[which] * (double)k;
        cs[which][k] = cos(t);
        sn[which][k] = sin(t);
    }
    for (int i = tid; i < dsh * dsh; i += kThreads) D[i] = 0.0f;
    __syncthreads();
    if (tid == 0) D[0] = 1.0f;

    const double* P = basis + 1;  // degree-0 block (1x1) first
    for (int l = 1; l < ndeg; ++l) {
        const int n = 2 * l + 1;
        // A = P Z(beta): column k mixes P's columns k and 2l - k
        for (int e = tid; e < n * n; e += kThreads) {
            const int i = e / n, k = e % n;
            double acc = P[i * n + k] * zrot(cs[1], sn[1], l, k, k);
            if (2 * l - k != k) acc += P[i * n + (2 * l - k)] * zrot(cs[1], sn[1], l, 2 * l - k, k);
            A[e] = acc;
        }
        __syncthreads();
        // T = A P^T
        for (int e = tid; e < n * n; e += kThreads) {
            const int i = e / n, j = e % n;
            double acc = 0.0;
            for (int k = 0; k < n; ++k) acc += A[i * n + k] * P[j * n + k];
            T[e] = acc;
        }
        __syncthreads();
        // D = Z(alpha) T Z(gamma)
        const int o = l * l;
        for (int e = tid; e < n * n; e += kThreads) {
            const int i = e / n, j = e % n;
            const int pi[2] = {i, 2 * l - i}, qj[2] = {j, 2 * l - j};
            double acc = 0.0;
            for (int u = 0; u < (pi[0] == pi[1] ? 1 : 2); ++u) {
                const double za = zrot(cs[0], sn[0], l, i, pi[u]);
                for (int w = 0; w < (qj[0] == qj[1] ? 1 : 2); ++w)
                    acc += za * T[pi[u] * n + qj[w]] * zrot(cs[2], sn[2], l, qj[w], j);
            }
            D[(o + i) * dsh + (o + j)] = (float)acc;
        }
        __syncthreads();
        P += n * n;
    }
}

}  // namespace shrot
}  // namespace tsplat

extern "C" int tsplat_sh_rotation_fwd(const float* rotations, const double* basis, float* out,
                                      int32_t num_cameras, int32_t d_sh, void* stream_) {
    using namespace tsplat::shrot;
    if (!rotations || !basis || !out || num_cameras <= 0) return TSPLAT_EINVAL;
    int ndeg = 0;
    while (ndeg * ndeg < d_sh) ++ndeg;
    if (ndeg * ndeg != d_sh || ndeg > kMaxDeg + 1) return TSPLAT_EINVAL;
    hipLaunchKernelGGL(shrot_kernel, dim3(num_cameras), dim3(kThreads), 0, (hipStream_t)stream_,
                       rotations, basis, out, d_sh, ndeg);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
