// Shifted-window cross/self attention of the multi-view transformer on gfx950 MFMA.
//
// Semantics: reference `single_head_split_window_attention`
// (src/model/encoder/backbone/multiview_transformer.py:57-206, both the 2-view and the multi-view
// branch) with the Swin mask of `generate_shift_window_attn_mask` (:17-54):
//   out[p] = softmax(q_p K_w^T / sqrt(C) + mask) V_w over the window w containing p, where windows
//   are the K x K splits of the map rolled by (-shift, -shift) (shift = window/2 on odd layers),
//   keys of m views are ordered pixel-major / view-minor and the -100 region mask is tiled
//   view-major, so key j uses mask column j mod L (the reference's V >= 3 indexing, reproduced).
// The roll, the window partition and the mask are index arithmetic here: nothing is materialised
// (the reference allocates rolled copies, a [K^2, L, L] mask and [8, L, L] fp32 scores per call).
//
// Kernel: flash-style, one workgroup = 4 waves = 64 queries of one window; each wave owns 16
// queries. Exact-fp32 MFMA (v_mfma_f32_16x16x4_f32) for both contractions:
//   S^T[key, q] = K Q^T   (keys on MFMA rows, queries on lanes -> per-query softmax stats are
//                          per-lane, no cross-lane transpose)
//   O^T[d, q]  += V^T P^T (the S^T accumulator IS the P^T B-operand: lane (q, g) holds keys
//                          16t + 4g + r in register (t, r), exactly what k-step 4t + r needs)
// K and V tiles of 64 keys are gathered by pixel index into LDS (K XOR-swizzled per 16-B chunk so
// the 16 row reads of a ds_read_b128 group hit distinct banks; V rows padded to 132 floats so the
// column reads of the two half-waves hit disjoint banks).
#include "common.h"
#include "prof.h"

namespace tsplat {
namespace winattn {

constexpr int kC = 128;          // channels (d_model of the reference transformer)
constexpr int kBQ = 64;          // queries per workgroup
constexpr int kBK = 64;          // keys per LDS tile
constexpr int kThreads = 256;
constexpr int kVStride = kC + 4;  // padded V row (floats)

typedef float floatx4 __attribute__((ext_vector_type(4)));

struct Params {
    int H, W, splits, shift, m, L;  // L = window pixels
    float scale;
};

// original pixel of in-window position t of window wi after the roll by -shift
__device__ __forceinline__ int win_pixel(const Params& p, int wi, int t) {
    const int wh = p.H / p.splits, ww = p.W / p.splits;
    const int sy = wi / p.splits, sx = wi % p.splits;
    const int ty = t / ww, tx = t - ty * ww;
    int y = sy * wh + ty + p.shift;
    int x = sx * ww + tx + p.shift;
    if (y >= p.H) y -= p.H;
    if (x >= p.W) x -= p.W;
    return y * p.W + x;
}

// Swin region id of in-window position t of window wi (on the rolled grid)
__device__ __forceinline__ int win_region(const Params& p, int wi, int t) {
    const int wh = p.H / p.splits, ww = p.W / p.splits;
    const int sy = wi / p.splits, sx = wi % p.splits;
    const int ty = t / ww, tx = t - ty * ww;
    const int Y = sy * wh + ty, X = sx * ww + tx;
    const int by = Y < p.H - wh ? 0 : (Y < p.H - wh / 2 ? 1 : 2);
    const int bx = X < p.W - ww ? 0 : (X < p.W - ww / 2 ? 1 : 2);
    return by * 3 + bx;
}

__global__ void __launch_bounds__(kThreads)
win_attn_f32_kernel(Params p, const float* __restrict__ q, const float* __restrict__ k,
                    const float* __restrict__ v, float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float sK[kBK * kC];
    __shared__ __attribute__((aligned(16))) float sV[kBK * kVStride];
    __shared__ int sKeyRegion[kBK];

    const int qblk = blockIdx.x, wi = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = lane >> 4, ql = lane & 15;
    const size_t HW = (size_t)p.H * p.W;
    const float* qb = q + (size_t)b * HW * kC;
    const float* kb = k + (size_t)b * p.m * HW * kC;
    const float* vb = v + (size_t)b * p.m * HW * kC;

    // this lane's query and its 32 channels [32g, 32g+32)
    const int tq = qblk * kBQ + wid * 16 + ql;
    const int qpix = win_pixel(p, wi, tq);
    const int qreg = p.shift ? win_region(p, wi, tq) : 0;
    float qr[32];
    {
        const float4* src = reinterpret_cast<const float4*>(qb + (size_t)qpix * kC + 32 * g);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float4 t4 = src[i];
            qr[4 * i] = t4.x * p.scale;
            qr[4 * i + 1] = t4.y * p.scale;
            qr[4 * i + 2] = t4.z * p.scale;
            qr[4 * i + 3] = t4.w * p.scale;
        }
    }

    floatx4 o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.f;

    const int nkeys = p.L * p.m;
    for (int k0 = 0; k0 < nkeys; k0 += kBK) {
        // ---- gather the K / V tile (64 keys x 128 ch) into LDS: 4 threads per key row
        {
            const int r = tid >> 2, part = tid & 3;  // row, 32-float quarter
            const int j = k0 + r;
            const int tk = j / p.m, vi = j - tk * p.m;
            const int kpix = win_pixel(p, wi, tk);
            const float4* ks = reinterpret_cast<const float4*>(kb + ((size_t)vi * HW + kpix) * kC + 32 * part);
            const float4* vs = reinterpret_cast<const float4*>(vb + ((size_t)vi * HW + kpix) * kC + 32 * part);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int chunk = part * 8 + i;               // 16-B chunk in the 512-B row
                const int phys = chunk ^ (r & 15);            // XOR swizzle (low 4 bits)
                *reinterpret_cast<float4*>(&sK[r * kC + phys * 4]) = ks[i];
                *reinterpret_cast<float4*>(&sV[r * kVStride + chunk * 4]) = vs[i];
            }
            if (part == 0 && p.shift) sKeyRegion[r] = win_region(p, wi, j % p.L);
        }
        __syncthreads();

        // ---- S^T = K Q^T for 4 tiles of 16 keys
        floatx4 s[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int row = 16 * t + ql;
            float kr[32];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int chunk = 8 * g + i;
                const float4 t4 = *reinterpret_cast<const float4*>(&sK[row * kC + ((chunk ^ (row & 15)) * 4)]);
                kr[4 * i] = t4.x;
                kr[4 * i + 1] = t4.y;
                kr[4 * i + 2] = t4.z;
                kr[4 * i + 3] = t4.w;
            }
            floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 32; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(kr[i], qr[i], acc, 0, 0, 0);
            s[t] = acc;
        }
        // ---- mask + online softmax (lane = query ql; keys 16t + 4g + r)
        float bmax = -INFINITY;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float x = s[t][r];
                if (p.shift) x += (sKeyRegion[16 * t + 4 * g + r] == qreg) ? 0.0f : -100.0f;
                s[t][r] = x;
                bmax = fmaxf(bmax, x);
            }
        bmax = fmaxf(bmax, __shfl_xor(bmax, 16));
        bmax = fmaxf(bmax, __shfl_xor(bmax, 32));
        const float m_new = fmaxf(m_run, bmax);
        const float corr = __expf(m_run - m_new);
        float bsum = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float e = __expf(s[t][r] - m_new);
                s[t][r] = e;
                bsum += e;
            }
        bsum += __shfl_xor(bsum, 16);
        bsum += __shfl_xor(bsum, 32);
        l_run = l_run * corr + bsum;
        m_run = m_new;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] *= corr;

        // ---- O^T += V^T P^T : k-step 4t + r covers keys 16t + 4g' + r
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            const int d = 16 * dt + ql;
            floatx4 acc = o[dt];
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float a = sV[(16 * t + 4 * g + r) * kVStride + d];
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, s[t][r], acc, 0, 0, 0);
                }
            o[dt] = acc;
        }
        __syncthreads();
    }

    // ---- epilogue: O^T[d = 16dt + 4g + r][q] / l -> out[qpix][d]
    const float inv = 1.0f / l_run;
    float* dst = out + ((size_t)b * HW + qpix) * kC + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
        float4 t4 = make_float4(o[dt][0] * inv, o[dt][1] * inv, o[dt][2] * inv, o[dt][3] * inv);
        *reinterpret_cast<float4*>(dst + 16 * dt) = t4;
    }
}

}  // namespace winattn
}  // namespace tsplat

using namespace tsplat;

extern "C" int tsplat_win_attn_fwd(const float* q, const float* k, const float* v, float* out,
                                   int32_t batch, int32_t height, int32_t width, int32_t channels,
                                   int32_t key_views, int32_t splits, int32_t with_shift,
                                   void* stream_) {
    using namespace tsplat::winattn;
    if (!q || !k || !v || !out) return TSPLAT_EINVAL;
    if (channels != kC || batch <= 0 || key_views <= 0 || splits <= 0) return TSPLAT_EINVAL;
    if (height % splits || width % splits) return TSPLAT_EINVAL;
    Params p;
    p.H = height;
    p.W = width;
    p.splits = splits;
    p.m = key_views;
    p.L = (height / splits) * (width / splits);
    p.shift = with_shift ? (height / splits) / 2 : 0;
    if (with_shift && (height / splits) / 2 != (width / splits) / 2) return TSPLAT_EINVAL;
    if (p.L % kBQ || (p.L * p.m) % kBK) return TSPLAT_EINVAL;
    p.scale = 1.0f / sqrtf((float)kC);
    hipStream_t stream = (hipStream_t)stream_;
    dim3 grid(p.L / kBQ, splits * splits, batch);
    TSPLAT_PROF_BEGIN(prof::kWinAttn, stream);
    hipLaunchKernelGGL(win_attn_f32_kernel, grid, dim3(kThreads), 0, stream, p, q, k, v, out);
    TSPLAT_PROF_END(prof::kWinAttn, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
