// GroupNorm (+ activation, + residual) over NCHW fp32: one launch when a group fits one
// workgroup's registers (<= 16,384 elements), else two.
//
// Replaces the GroupNorm -> SiLU/GELU (-> residual add) chains of the depth predictor's U-Nets
// and refine heads (reference src/model/encoder/matching/ldm_unet/{unet.py:177-370, util.py:
// 189-208}, depth_predictor_trans.py:142-206). PyTorch's ROCm GroupNorm launches one workgroup
// per (sample, group) for the moments -- 16-64 workgroups on a 256-CU part, 37 us per call in the
// r1 profile -- then a parameter kernel, an apply kernel and a separate activation.
// Here: (1) every group is split into 4096-element chunks; a chunk's workgroup reduces it to a
// Welford partial (mean, M2); (2) each apply workgroup combines its group's partials (Chan) and
// normalises its chunk with the activation and optional residual fused: x is read twice (the
// second time mostly from L2/MALL), y written once.
#include "common.h"
#include "prof.h"

namespace tsplat {
namespace gn {

constexpr int kThreads = 256;
constexpr int kChunk = 4096;  // elements per workgroup (16 per thread)

struct Welford {
    float n, mean, m2;
};

__device__ __forceinline__ Welford combine(Welford a, Welford b) {
    const float n = a.n + b.n;
    if (n == 0.f) return a;
    const float d = b.mean - a.mean;
    const float wb = b.n / n;
    return {n, a.mean + d * wb, a.m2 + b.m2 + d * d * a.n * wb};
}

__device__ __forceinline__ Welford push(Welford w, float x) {
    w.n += 1.f;
    const float d = x - w.mean;
    w.mean += d / w.n;
    w.m2 += d * (x - w.mean);
    return w;
}

__device__ __forceinline__ Welford wave_reduce(Welford w) {
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
        Welford o{__shfl_xor(w.n, off), __shfl_xor(w.mean, off), __shfl_xor(w.m2, off)};
        w = combine(w, o);
    }
    return w;
}

// activation I/O: fp32, or bf16 (config C3's bf16 dense layers: the convolutions around the norm
// read and write bf16, so the norm takes bf16 in and gives bf16 out, computing in fp32 -- the
// reference's GroupNorm32 normalises x.float() and casts back to x's dtype)
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const __bf16* p) { return (float)*p; }
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }
__device__ __forceinline__ void st1(__bf16* p, float v) { *p = (__bf16)v; }
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 ld4(const __bf16* p) {
    const bf16x4_t v = *reinterpret_cast<const bf16x4_t*>(p);
    return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ void st4(__bf16* p, float4 v) {
    *reinterpret_cast<bf16x4_t*>(p) = bf16x4_t{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
}

// Welford over this workgroup's chunk -> partials[seg * S + chunk] = (mean, M2)
// pb (may be null): per-channel bias of the producing convolution, added on the fly (the conv
// runs without its bias, so PyTorch's separate broadcast add disappears)
template <bool VEC, typename T>
__global__ void __launch_bounds__(kThreads)
stats_kernel(const T* __restrict__ x, const float* __restrict__ pb, float2* __restrict__ partials,
             int64_t L, int S, int HW, int cpg, int G) {
    const int chunk = blockIdx.x, seg = blockIdx.y, tid = threadIdx.x;
    const int64_t start = (int64_t)chunk * kChunk;
    const int n_local = (int)min((int64_t)kChunk, L - start);
    const T* p = x + (int64_t)seg * L + start;
    const int c0 = (seg % G) * cpg;
    Welford w{0.f, 0.f, 0.f};
    if (VEC) {
#pragma unroll
        for (int k = 0; k < kChunk / (4 * kThreads); ++k) {
            const int i = (k * kThreads + tid) * 4;
            if (i < n_local) {
                const float b = pb ? pb[c0 + (int)((start + i) / HW)] : 0.f;
                const float4 v = ld4(p + i);
                w = push(w, v.x + b);
                w = push(w, v.y + b);
                w = push(w, v.z + b);
                w = push(w, v.w + b);
            }
        }
    } else {
        for (int i = tid; i < n_local; i += kThreads)
            w = push(w, ld1(p + i) + (pb ? pb[c0 + (int)((start + i) / HW)] : 0.f));
    }
    w = wave_reduce(w);
    __shared__ Welford sw[kThreads / kWave];
    if ((tid & (kWave - 1)) == 0) sw[tid / kWave] = w;
    __syncthreads();
    if (tid == 0) {
        Welford t = sw[0];
#pragma unroll
        for (int i = 1; i < kThreads / kWave; ++i) t = combine(t, sw[i]);
        partials[(int64_t)seg * S + chunk] = make_float2(t.mean, t.m2);
    }
}

template <int ACT>
__device__ __forceinline__ float activate(float v) {
    if (ACT == 1) return v / (1.0f + expf(-v));                     // SiLU
    if (ACT == 2) return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));  // GELU (erf)
    if (ACT == 3) return fmaxf(v, 0.0f);                             // ReLU
    return v;
}

// after the residual add: ACT 3 is the UniMatch ResidualBlock ending relu(x + relu(norm(y)))
template <int ACT>
__device__ __forceinline__ float post_residual(float v) { return ACT == 3 ? fmaxf(v, 0.0f) : v; }

// The residual of element (sample n, channel ch, position p) at flat index e = (n C + ch) HW + p:
// res + e, or -- a residual given as the channel concatenation [res (c1 channels) | res2 (C - c1)]
// (a U-Net skip input, read in place) -- the element of whichever part holds channel ch
template <typename T>
__device__ __forceinline__ const T* res_at(const T* res, const T* res2, int c1, int C, int64_t e, int n, int ch,
                                           int HW) {
    if (c1 >= C) return res + e;
    const int64_t p = e - ((int64_t)n * C + ch) * HW;
    return ch < c1 ? res + ((int64_t)n * c1 + ch) * HW + p : res2 + ((int64_t)n * (C - c1) + (ch - c1)) * HW + p;
}

template <bool VEC, int ACT, bool RES, typename T>
__global__ void __launch_bounds__(kThreads)
apply_kernel(const T* __restrict__ x, const float* __restrict__ pb, const float2* __restrict__ partials,
             const float* __restrict__ gamma, const float* __restrict__ beta,
             const T* __restrict__ res, const T* __restrict__ res2, int c1, T* __restrict__ y, int64_t L, int S,
             int HW, int C, int cpg, int G, float eps) {
    const int chunk = blockIdx.x, seg = blockIdx.y, tid = threadIdx.x;
    __shared__ float s_scale_shift[2];
    if (tid < kWave) {
        // combine the group's S partials (chunk sizes are kChunk except the last)
        Welford w{0.f, 0.f, 0.f};
        for (int i = tid; i < S; i += kWave) {
            const float2 pm = partials[(int64_t)seg * S + i];
            const float n = (float)min((int64_t)kChunk, L - (int64_t)i * kChunk);
            w = combine(w, Welford{n, pm.x, pm.y});
        }
        w = wave_reduce(w);
        if (tid == 0) {
            s_scale_shift[0] = w.mean;
            s_scale_shift[1] = rsqrtf(w.m2 / (float)L + eps);
        }
    }
    __syncthreads();
    const float mean = s_scale_shift[0], rstd = s_scale_shift[1];
    const int g = seg % G;
    const int64_t start = (int64_t)chunk * kChunk;
    const int n_local = (int)min((int64_t)kChunk, L - start);
    const int64_t base = (int64_t)seg * L + start;
    if (VEC) {
#pragma unroll
        for (int k = 0; k < kChunk / (4 * kThreads); ++k) {
            const int i = (k * kThreads + tid) * 4;
            if (i < n_local) {
                const int c = g * cpg + (int)((start + i) / HW);  // HW % 4 == 0: one channel per float4
                const float sc = rstd * gamma[c];
                const float sh = beta[c] - sc * mean;
                const float b = pb ? pb[c] : 0.f;
                float4 v = ld4(x + base + i);
                v.x += b;
                v.y += b;
                v.z += b;
                v.w += b;
                v.x = activate<ACT>(v.x * sc + sh);
                v.y = activate<ACT>(v.y * sc + sh);
                v.z = activate<ACT>(v.z * sc + sh);
                v.w = activate<ACT>(v.w * sc + sh);
                if (RES) {
                    const float4 r = ld4(res_at(res, res2, c1, C, base + i, seg / G, c, HW));
                    v.x = post_residual<ACT>(v.x + r.x);
                    v.y = post_residual<ACT>(v.y + r.y);
                    v.z = post_residual<ACT>(v.z + r.z);
                    v.w = post_residual<ACT>(v.w + r.w);
                }
                st4(y + base + i, v);
            }
        }
    } else {
        for (int i = tid; i < n_local; i += kThreads) {
            const int c = g * cpg + (int)((start + i) / HW);
            const float sc = rstd * gamma[c];
            float v = activate<ACT>((ld1(x + base + i) + (pb ? pb[c] : 0.f)) * sc + (beta[c] - sc * mean));
            if (RES) v = post_residual<ACT>(v + ld1(res_at(res, res2, c1, C, base + i, seg / G, c, HW)));
            st1(y + base + i, v);
        }
    }
}

// Single-launch form for groups of at most 512 * NPT elements: one 512-thread workgroup per
// (sample, group) holds the group in registers (NPT floats per thread), reduces the mean and then
// the centred sum of squares (two exact block reductions, no partials), and writes
// act(norm) (+ residual) -- one read and one write of x, one launch instead of two.
constexpr int kFusedThreads = 512;

__device__ __forceinline__ float block_sum512(float v, float* red) {
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int w = threadIdx.x >> 6;
    __syncthreads();  // red may still be read from the previous reduction
    if ((threadIdx.x & (kWave - 1)) == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < kFusedThreads / kWave; ++i) t += red[i];
    return t;
}

template <int NPT, int ACT, bool RES, typename T>
__global__ void __launch_bounds__(kFusedThreads)
fused_kernel(const T* __restrict__ x, const float* __restrict__ pb, const float* __restrict__ gamma,
             const float* __restrict__ beta, const T* __restrict__ res, const T* __restrict__ res2, int c1,
             T* __restrict__ y, int L, int HW, int cpg, int G, float eps) {
    __shared__ float red[kFusedThreads / kWave];
    const int seg = blockIdx.x, tid = threadIdx.x;
    const int g = seg % G;
    const int64_t base = (int64_t)seg * L;
    float4 v[NPT / 4];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NPT / 4; ++k) {
        const int i = (k * kFusedThreads + tid) * 4;  // HW % 4 == 0: one channel per float4
        if (i < L) {
            v[k] = ld4(x + base + i);
            if (pb) {
                const float b = pb[g * cpg + i / HW];
                v[k].x += b;
                v[k].y += b;
                v[k].z += b;
                v[k].w += b;
            }
            s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
        }
    }
    const float mean = block_sum512(s, red) / (float)L;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NPT / 4; ++k) {
        const int i = (k * kFusedThreads + tid) * 4;
        if (i < L) {
            const float a = v[k].x - mean, b = v[k].y - mean, c = v[k].z - mean, d = v[k].w - mean;
            q += (a * a + b * b) + (c * c + d * d);
        }
    }
    const float rstd = rsqrtf(block_sum512(q, red) / (float)L + eps);
#pragma unroll
    for (int k = 0; k < NPT / 4; ++k) {
        const int i = (k * kFusedThreads + tid) * 4;
        if (i < L) {
            const int c = g * cpg + i / HW;
            const float sc = rstd * gamma[c], sh = beta[c] - sc * mean;
            float4 o;
            o.x = activate<ACT>(v[k].x * sc + sh);
            o.y = activate<ACT>(v[k].y * sc + sh);
            o.z = activate<ACT>(v[k].z * sc + sh);
            o.w = activate<ACT>(v[k].w * sc + sh);
            if (RES) {
                const float4 r = ld4(res_at(res, res2, c1, cpg * G, base + i, seg / G, c, HW));
                o.x = post_residual<ACT>(o.x + r.x);
                o.y = post_residual<ACT>(o.y + r.y);
                o.z = post_residual<ACT>(o.z + r.z);
                o.w = post_residual<ACT>(o.w + r.w);
            }
            st4(y + base + i, o);
        }
    }
}

}  // namespace gn
}  // namespace tsplat

using namespace tsplat;

extern "C" size_t tsplat_group_norm_workspace_bytes(int32_t n, int32_t c, int64_t hw, int32_t groups) {
    if (n <= 0 || c <= 0 || hw <= 0 || groups <= 0 || c % groups) return 0;
    const int64_t L = (int64_t)(c / groups) * hw;
    const int64_t S = (L + gn::kChunk - 1) / gn::kChunk;
    return (size_t)n * groups * S * sizeof(float2);
}

template <typename T>
static int group_norm_launch(const T* x, const float* pre_bias, const float* gamma, const float* beta,
                             const T* residual, T* y, void* workspace, int32_t n, int32_t c, int64_t hw,
                             int32_t groups, float eps, int32_t act, void* stream_, const T* residual2 = nullptr,
                             int32_t c1 = -1) {
    using namespace tsplat::gn;
    if (!x || !gamma || !beta || !y || !workspace) return TSPLAT_EINVAL;
    if (c1 < 0) c1 = c;  // one residual tensor
    if (c1 > c || (c1 < c && (!residual || !residual2 || c1 == 0))) return TSPLAT_EINVAL;
    if (n <= 0 || c <= 0 || hw <= 0 || groups <= 0 || c % groups || act < 0 || act > 3 ||
        hw > INT32_MAX)
        return TSPLAT_EINVAL;
    const int cpg = c / groups;
    const int64_t L = (int64_t)cpg * hw;
    const int64_t S = (L + kChunk - 1) / kChunk;
    if (S > INT32_MAX || (int64_t)n * groups > 65535) return TSPLAT_EINVAL;
    hipStream_t stream = (hipStream_t)stream_;
    const dim3 grid((unsigned)S, (unsigned)(n * groups));
    const uintptr_t al = 4 * sizeof(T);  // one vector of 4 elements
    const bool vec = (hw % 4 == 0) && ((uintptr_t)x % al == 0) && ((uintptr_t)y % al == 0) &&
                     (!residual || (uintptr_t)residual % al == 0) && (!residual2 || (uintptr_t)residual2 % al == 0);
    if (vec && L <= (int64_t)kFusedThreads * 32 && x != y) {
        // the whole group fits one workgroup's registers: single launch
        const int npt = L <= kFusedThreads * 4 ? 4 : L <= kFusedThreads * 8 ? 8 : L <= kFusedThreads * 16 ? 16 : 32;
        TSPLAT_PROF_BEGIN(prof::kGroupNorm, stream);
#define TSPLAT_GN_F(N, A, R)                                                                                  \
    hipLaunchKernelGGL((fused_kernel<N, A, R, T>), dim3((unsigned)(n * groups)), dim3(kFusedThreads), 0, stream, x, \
                       pre_bias, gamma, beta, residual, residual2, c1, y, (int)L, (int)hw, cpg, groups, eps)
#define TSPLAT_GN_FA(N, R)                   \
    switch (act) {                           \
        case 0: TSPLAT_GN_F(N, 0, R); break; \
        case 1: TSPLAT_GN_F(N, 1, R); break; \
        case 2: TSPLAT_GN_F(N, 2, R); break; \
        default: TSPLAT_GN_F(N, 3, R); break; \
    }
#define TSPLAT_GN_FN(N)                                                       \
    if (residual) { TSPLAT_GN_FA(N, true) } else { TSPLAT_GN_FA(N, false) }
        switch (npt) {
            case 4: TSPLAT_GN_FN(4); break;
            case 8: TSPLAT_GN_FN(8); break;
            case 16: TSPLAT_GN_FN(16); break;
            default: TSPLAT_GN_FN(32); break;
        }
#undef TSPLAT_GN_FN
#undef TSPLAT_GN_FA
#undef TSPLAT_GN_F
        TSPLAT_PROF_END(prof::kGroupNorm, stream);
        TSPLAT_CHECK_LAUNCH();
        return TSPLAT_OK;
    }
    float2* part = (float2*)workspace;
    TSPLAT_PROF_BEGIN(prof::kGroupNorm, stream);
    if (vec)
        hipLaunchKernelGGL((stats_kernel<true, T>), grid, dim3(kThreads), 0, stream, x, pre_bias, part, L, (int)S,
                           (int)hw, cpg, groups);
    else
        hipLaunchKernelGGL((stats_kernel<false, T>), grid, dim3(kThreads), 0, stream, x, pre_bias, part, L, (int)S,
                           (int)hw, cpg, groups);
    TSPLAT_CHECK_LAUNCH();
#define TSPLAT_GN_APPLY(V, A, R)                                                                   \
    hipLaunchKernelGGL((apply_kernel<V, A, R, T>), grid, dim3(kThreads), 0, stream, x, pre_bias, part, gamma,  \
                       beta, residual, residual2, c1, y, L, (int)S, (int)hw, c, cpg, groups, eps)
#define TSPLAT_GN_ACT(V, R)              \
    switch (act) {                       \
        case 0: TSPLAT_GN_APPLY(V, 0, R); break; \
        case 1: TSPLAT_GN_APPLY(V, 1, R); break; \
        case 2: TSPLAT_GN_APPLY(V, 2, R); break; \
        default: TSPLAT_GN_APPLY(V, 3, R); break; \
    }
    if (vec) {
        if (residual) { TSPLAT_GN_ACT(true, true) } else { TSPLAT_GN_ACT(true, false) }
    } else {
        if (residual) { TSPLAT_GN_ACT(false, true) } else { TSPLAT_GN_ACT(false, false) }
    }
#undef TSPLAT_GN_ACT
#undef TSPLAT_GN_APPLY
    TSPLAT_PROF_END(prof::kGroupNorm, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_group_norm_fwd(const float* x, const float* pre_bias, const float* gamma, const float* beta,
                                     const float* residual, float* y, void* workspace, int32_t n,
                                     int32_t c, int64_t hw, int32_t groups, float eps, int32_t act,
                                     void* stream_) {
    return group_norm_launch<float>(x, pre_bias, gamma, beta, residual, y, workspace, n, c, hw, groups, eps, act,
                                    stream_);
}

// tsplat_group_norm_fwd with the residual given as a channel concatenation read in place:
// channels [0, c1) from residual [n, c1, hw], [c1, c) from residual2 [n, c - c1, hw]
extern "C" int tsplat_group_norm_cat_res_fwd(const float* x, const float* pre_bias, const float* gamma,
                                             const float* beta, const float* residual, const float* residual2,
                                             int32_t c1, float* y, void* workspace, int32_t n, int32_t c, int64_t hw,
                                             int32_t groups, float eps, int32_t act, void* stream_) {
    if (c1 <= 0 || c1 >= c || !residual || !residual2) return TSPLAT_EINVAL;
    return group_norm_launch<float>(x, pre_bias, gamma, beta, residual, y, workspace, n, c, hw, groups, eps, act,
                                    stream_, residual2, c1);
}

extern "C" int tsplat_group_norm_bf16_fwd(const void* x, const float* pre_bias, const float* gamma,
                                          const float* beta, const void* residual, void* y, void* workspace,
                                          int32_t n, int32_t c, int64_t hw, int32_t groups, float eps, int32_t act,
                                          void* stream_) {
    return group_norm_launch<__bf16>((const __bf16*)x, pre_bias, gamma, beta, (const __bf16*)residual, (__bf16*)y,
                                     workspace, n, c, hw, groups, eps, act, stream_);
}

// ---------------------------------------------------------------------------------------------
// Convolution epilogue without normalisation: y = post(act(x + bias[c]) (+ residual)) over NCHW,
// one pass instead of PyTorch's bias add_ + activation (+ add) passes after a MIOpen convolution.
namespace tsplat {
namespace gn {

template <int ACT, bool RES>
__global__ void __launch_bounds__(kThreads)
bias_act_kernel(const float* __restrict__ x, const float* __restrict__ bias, const float* __restrict__ res,
                float* __restrict__ y, int n4, int hw4, int C) {
    const int i = blockIdx.x * kThreads + threadIdx.x;  // 32-bit index math (n4 < 2^31 checked)
    if (i >= n4) return;
    const int c = (i / hw4) % C;
    const float b = bias ? bias[c] : 0.f;
    float4 v = reinterpret_cast<const float4*>(x)[i];
    v.x = activate<ACT>(v.x + b);
    v.y = activate<ACT>(v.y + b);
    v.z = activate<ACT>(v.z + b);
    v.w = activate<ACT>(v.w + b);
    if (RES) {
        const float4 r = reinterpret_cast<const float4*>(res)[i];
        v.x = post_residual<ACT>(v.x + r.x);
        v.y = post_residual<ACT>(v.y + r.y);
        v.z = post_residual<ACT>(v.z + r.z);
        v.w = post_residual<ACT>(v.w + r.w);
    }
    reinterpret_cast<float4*>(y)[i] = v;
}

}  // namespace gn
}  // namespace tsplat

extern "C" int tsplat_bias_act_fwd(const float* x, const float* bias, const float* residual, float* y, int32_t n,
                                   int32_t c, int64_t hw, int32_t act, void* stream_) {
    using namespace tsplat::gn;
    if (!x || !y || n <= 0 || c <= 0 || hw <= 0 || hw % 4 || act < 0 || act > 3) return TSPLAT_EINVAL;
    if ((uintptr_t)x % 16 || (uintptr_t)y % 16 || (residual && (uintptr_t)residual % 16)) return TSPLAT_EINVAL;
    const int64_t n4 = (int64_t)n * c * hw / 4;
    if (n4 > INT32_MAX) return TSPLAT_EINVAL;
    hipStream_t stream = (hipStream_t)stream_;
    const dim3 grid((unsigned)((n4 + kThreads - 1) / kThreads));
#define TSPLAT_BA(A, R) \
    hipLaunchKernelGGL((bias_act_kernel<A, R>), grid, dim3(kThreads), 0, stream, x, bias, residual, y, (int)n4, (int)(hw / 4), c)
#define TSPLAT_BA_ACT(R)                   \
    switch (act) {                         \
        case 0: TSPLAT_BA(0, R); break;    \
        case 1: TSPLAT_BA(1, R); break;    \
        case 2: TSPLAT_BA(2, R); break;    \
        default: TSPLAT_BA(3, R); break;   \
    }
    if (residual) { TSPLAT_BA_ACT(true) } else { TSPLAT_BA_ACT(false) }
#undef TSPLAT_BA_ACT
#undef TSPLAT_BA
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

// ---------------------------------------------------------------------------------------------
// Channels-last form: y = act(x + bias[c]) (+ res1) (+ res2) over [rows, C] (NHWC maps, C % 4 == 0)
// -- the epilogues of the DPT head's bias-free MIOpen convolutions (ResidualConvUnit: bias + ReLU
// after conv1; bias + the unit's residual (+ the fusion block's skip) after conv2).
namespace tsplat {
namespace gn {

template <int ACT, int NRES>
__global__ void __launch_bounds__(kThreads)
bias_act_nhwc_kernel(const float* __restrict__ x, const float* __restrict__ bias, const float* __restrict__ r1,
                     const float* __restrict__ r2, float* __restrict__ y, int n4, int c4) {
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n4) return;
    float4 v = reinterpret_cast<const float4*>(x)[i];
    if (bias) {
        const float4 b = reinterpret_cast<const float4*>(bias)[i % c4];
        v.x += b.x;
        v.y += b.y;
        v.z += b.z;
        v.w += b.w;
    }
    v.x = activate<ACT>(v.x);
    v.y = activate<ACT>(v.y);
    v.z = activate<ACT>(v.z);
    v.w = activate<ACT>(v.w);
    if (NRES >= 1) {
        const float4 r = reinterpret_cast<const float4*>(r1)[i];
        v.x += r.x;
        v.y += r.y;
        v.z += r.z;
        v.w += r.w;
    }
    if (NRES >= 2) {
        const float4 r = reinterpret_cast<const float4*>(r2)[i];
        v.x += r.x;
        v.y += r.y;
        v.z += r.z;
        v.w += r.w;
    }
    reinterpret_cast<float4*>(y)[i] = v;
}

}  // namespace gn
}  // namespace tsplat

extern "C" int tsplat_bias_act_nhwc_fwd(const float* x, const float* bias, const float* res1, const float* res2,
                                        float* y, int64_t rows, int32_t c, int32_t act, void* stream_) {
    using namespace tsplat::gn;
    if (!x || !y || rows <= 0 || c <= 0 || c % 4 || !(act == 0 || act == 2 || act == 3)) return TSPLAT_EINVAL;
    if (res2 && !res1) return TSPLAT_EINVAL;
    if ((uintptr_t)x % 16 || (uintptr_t)y % 16 || (bias && (uintptr_t)bias % 16) || (res1 && (uintptr_t)res1 % 16) ||
        (res2 && (uintptr_t)res2 % 16))
        return TSPLAT_EINVAL;
    const int64_t n4 = rows * c / 4;
    if (n4 > INT32_MAX) return TSPLAT_EINVAL;
    hipStream_t stream = (hipStream_t)stream_;
    const dim3 grid((unsigned)((n4 + kThreads - 1) / kThreads));
    const int nres = res2 ? 2 : (res1 ? 1 : 0);
#define TSPLAT_BAN(A, R) \
    hipLaunchKernelGGL((bias_act_nhwc_kernel<A, R>), grid, dim3(kThreads), 0, stream, x, bias, res1, res2, y, (int)n4, c / 4)
#define TSPLAT_BAN_R(A)                  \
    switch (nres) {                      \
        case 0: TSPLAT_BAN(A, 0); break; \
        case 1: TSPLAT_BAN(A, 1); break; \
        default: TSPLAT_BAN(A, 2); break; \
    }
    if (act == 0) { TSPLAT_BAN_R(0) } else if (act == 2) { TSPLAT_BAN_R(2) } else { TSPLAT_BAN_R(3) }
#undef TSPLAT_BAN_R
#undef TSPLAT_BAN
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

// ---------------------------------------------------------------------------------------------
// Pre-norm transformer residual step of the DINOv2 blocks: x' = x + ls * y (LayerScale residual),
// n = LayerNorm(x') with the NEXT sub-layer's norm, one pass over the row (one wave per row).
namespace tsplat {
namespace gn {

// TY / TN: the sub-layer output y and the normalised n in fp32, or bf16 (bf16 dense mode: the
// linears read n and write y in bf16; the residual stream x stays fp32 as under autocast)
template <int V4, typename TY, typename TN>  // float4s per lane (dim = 256 V4)
__global__ void __launch_bounds__(kThreads)
residual_ln_kernel(const float* __restrict__ x, const TY* __restrict__ y, const float* __restrict__ ls,
                   const float* __restrict__ w, const float* __restrict__ b, float* __restrict__ x_out,
                   TN* __restrict__ n_out, int rows, float eps, int nslab) {
    const int row = blockIdx.x * (kThreads / kWave) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    constexpr int D = 256 * V4;
    const size_t off = (size_t)row * D;
    float4 v[V4];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < V4; ++k) {
        const int c = 4 * (lane + 64 * k);
        v[k] = *reinterpret_cast<const float4*>(x + off + c);
        if (y) {
            float4 t = ld4(y + off + c);
            // split-K slabs, summed in slab order (deterministic)
            for (int sl = 1; sl < nslab; ++sl) {
                const float4 u = ld4(y + (size_t)sl * rows * D + off + c);
                t.x += u.x;
                t.y += u.y;
                t.z += u.z;
                t.w += u.w;
            }
            float4 g = make_float4(1.f, 1.f, 1.f, 1.f);
            if (ls) g = *reinterpret_cast<const float4*>(ls + c);
            v[k].x += g.x * t.x;
            v[k].y += g.y * t.y;
            v[k].z += g.z * t.z;
            v[k].w += g.w * t.w;
        }
        s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const float mean = s * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < V4; ++k) {
        const float a = v[k].x - mean, bb = v[k].y - mean, cc = v[k].z - mean, d = v[k].w - mean;
        q += (a * a + bb * bb) + (cc * cc + d * d);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
    const float rstd = rsqrtf(q * (1.0f / D) + eps);
#pragma unroll
    for (int k = 0; k < V4; ++k) {
        const int c = 4 * (lane + 64 * k);
        if (x_out) *reinterpret_cast<float4*>(x_out + off + c) = v[k];
        const float4 g = *reinterpret_cast<const float4*>(w + c), bt = *reinterpret_cast<const float4*>(b + c);
        st4(n_out + off + c, make_float4((v[k].x - mean) * rstd * g.x + bt.x, (v[k].y - mean) * rstd * g.y + bt.y,
                                         (v[k].z - mean) * rstd * g.z + bt.z, (v[k].w - mean) * rstd * g.w + bt.w));
    }
}

}  // namespace gn
}  // namespace tsplat

template <typename TY, typename TN>
static int residual_ln_launch(const float* x, const TY* y, const float* ls, const float* ln_w, const float* ln_b,
                              float ln_eps, float* x_out, TN* n_out, int32_t rows, int32_t dim, void* stream_,
                              int32_t nslab = 1) {
    using namespace tsplat::gn;
    if (!x || !ln_w || !ln_b || !n_out || rows <= 0 || (ls && !y) || nslab < 1) return TSPLAT_EINVAL;
    if (y && !x_out) return TSPLAT_EINVAL;
    hipStream_t stream = (hipStream_t)stream_;
    const dim3 grid((rows + kThreads / kWave - 1) / (kThreads / kWave));
#define TSPLAT_RLN(V)                                                                                   \
    hipLaunchKernelGGL((residual_ln_kernel<V, TY, TN>), grid, dim3(kThreads), 0, stream, x, y, ls, ln_w, ln_b, \
                       x_out, n_out, rows, ln_eps, nslab)
    switch (dim) {
        case 256: TSPLAT_RLN(1); break;
        case 512: TSPLAT_RLN(2); break;
        case 768: TSPLAT_RLN(3); break;
        case 1024: TSPLAT_RLN(4); break;
        default: return TSPLAT_EINVAL;
    }
#undef TSPLAT_RLN
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_residual_ln_fwd(const float* x, const float* y, const float* ls, const float* ln_w,
                                      const float* ln_b, float ln_eps, float* x_out, float* n_out, int32_t rows,
                                      int32_t dim, void* stream_) {
    return residual_ln_launch<float, float>(x, y, ls, ln_w, ln_b, ln_eps, x_out, n_out, rows, dim, stream_);
}

extern "C" int tsplat_residual_ln_slabs_fwd(const float* x, const float* y, int32_t nslab, const float* ls,
                                            const float* ln_w, const float* ln_b, float ln_eps, float* x_out,
                                            float* n_out, int32_t rows, int32_t dim, void* stream_) {
    if (!y) return TSPLAT_EINVAL;
    return residual_ln_launch<float, float>(x, y, ls, ln_w, ln_b, ln_eps, x_out, n_out, rows, dim, stream_, nslab);
}

extern "C" int tsplat_residual_ln_bf16_fwd(const float* x, const void* y, const float* ls, const float* ln_w,
                                           const float* ln_b, float ln_eps, float* x_out, void* n_out, int32_t rows,
                                           int32_t dim, void* stream_) {
    return residual_ln_launch<__bf16, __bf16>(x, (const __bf16*)y, ls, ln_w, ln_b, ln_eps, x_out, (__bf16*)n_out,
                                              rows, dim, stream_);
}

// ---------------------------------------------------------------------------------------------
// LayerNorm over rows of 128 (the multi-view transformer's and the UV transformer's d_model) with
// an optional post-norm residual: out = [res +] LN(y). 32 lanes x float4 per row (two rows per
// wave), two-pass statistics in fp32; y and out in fp32 or bf16, res fp32. For the bf16 dense mode
// (config C3), where these norms otherwise run PyTorch's LayerNorm (65 us per call at batch 8 on
// 128-wide rows) between autocast casts (reference multiview_transformer.py:327-407 norm1 / norm2,
// utils/encoder.py:131-209 norms).
namespace tsplat {
namespace gn {

template <typename TY, typename TO>
__global__ void __launch_bounds__(kThreads)
ln128_kernel(const TY* __restrict__ y, const float* __restrict__ res, const float* __restrict__ w,
             const float* __restrict__ b, TO* __restrict__ out, int rows, float eps) {
    const int row = (blockIdx.x * kThreads + threadIdx.x) >> 5;
    const int l = threadIdx.x & 31;
    if (row >= rows) return;  // whole 32-lane halves leave together; the shuffles stay in a half
    const size_t off = (size_t)row * 128 + 4 * l;
    const float4 v = ld4(y + off);
    float s = (v.x + v.y) + (v.z + v.w);
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 32);
    const float mean = s * (1.0f / 128.0f);
    const float a = v.x - mean, bb = v.y - mean, c = v.z - mean, d = v.w - mean;
    float q = (a * a + bb * bb) + (c * c + d * d);
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) q += __shfl_xor(q, o, 32);
    const float rstd = rsqrtf(q * (1.0f / 128.0f) + eps);
    const float4 g = *reinterpret_cast<const float4*>(w + 4 * l), bt = *reinterpret_cast<const float4*>(b + 4 * l);
    float4 n = make_float4(a * rstd * g.x + bt.x, bb * rstd * g.y + bt.y, c * rstd * g.z + bt.z, d * rstd * g.w + bt.w);
    if (res) {
        const float4 r = *reinterpret_cast<const float4*>(res + off);
        n = make_float4(r.x + n.x, r.y + n.y, r.z + n.z, r.w + n.w);
    }
    st4(out + off, n);
}

}  // namespace gn
}  // namespace tsplat

extern "C" int tsplat_layer_norm128_fwd(const void* y, int32_t y_bf16, const float* residual, const float* ln_w,
                                        const float* ln_b, float ln_eps, void* out, int32_t out_bf16, int32_t rows,
                                        void* stream_) {
    using namespace tsplat::gn;
    if (!y || !ln_w || !ln_b || !out || rows <= 0) return TSPLAT_EINVAL;
    const uintptr_t al = y_bf16 ? 8 : 16;
    if ((uintptr_t)y % al || (uintptr_t)out % (out_bf16 ? 8 : 16) || (residual && (uintptr_t)residual % 16) ||
        (uintptr_t)ln_w % 16 || (uintptr_t)ln_b % 16)
        return TSPLAT_EINVAL;
    hipStream_t stream = (hipStream_t)stream_;
    const dim3 grid((unsigned)(((int64_t)rows * 32 + kThreads - 1) / kThreads));
#define TSPLAT_LN128(TY, TO)                                                                                 \
    hipLaunchKernelGGL((ln128_kernel<TY, TO>), grid, dim3(kThreads), 0, stream, (const TY*)y, residual, ln_w, ln_b, \
                       (TO*)out, rows, ln_eps)
    if (y_bf16 && out_bf16) TSPLAT_LN128(__bf16, __bf16);
    else if (y_bf16) TSPLAT_LN128(__bf16, float);
    else if (out_bf16) TSPLAT_LN128(float, __bf16);
    else TSPLAT_LN128(float, float);
#undef TSPLAT_LN128
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
