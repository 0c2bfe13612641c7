// 3x3 / stride 1 / pad 1 convolution as Winograd F(2x2, 3x3) on exact-fp32 MFMA, for the
// full-resolution and 64^2-128^2 convolutions of the depth predictor's heads and U-Nets
// (reference src/model/encoder/matching/depth_predictor_trans.py:110-125 to_gaussians /
// to_disparity, ldm_unet/unet.py ResBlock convolutions), which MIOpen runs with its VALU
// Winograd kernels (`miopenSp3AsmConv..._f2x3`, ~90 TFLOP/s direct-equivalent).
//
// y[n][co][2ty + i][2tx + j] = (A^T M A)[i][j], M[xi][co][t] = sum_ci U[xi][co][ci] V[xi][ci][t]:
//   V = B^T d B for the 4x4 input patch d of output tile t (rows 2ty - 1 .. 2ty + 2, zero outside),
//   U = G g G^T for the 3x3 filter g (precomputed once per weight version, tsplat_wino_weight_f32),
//   16 independent GEMMs (xi = 4 r + s) in v_mfma_f32_32x32x2_f32 -- 2.25x fewer products than
//   the direct convolution, at the same exact-fp32 MFMA rate.
// Workgroup = 4 waves = 32 output channels x 32 output tiles (2x2 pixels each, a TBY x TBX patch
// of tiles), wave w owns transform row r = w (xi = 4w .. 4w + 3: 64 accumulator registers).
// Per 8-channel chunk: every thread transforms one (tile, channel) patch into a double-buffered
// LDS image sV[xi][ci][tile] (loads of the next chunk issued before this chunk's MFMAs), one
// barrier, then 16 MFMAs per wave (A = the packed U fragment, 256 contiguous bytes per wave,
// prefetched a chunk ahead; B = one LDS float per lane). Epilogue: each wave folds its row of M
// into Z[r][j] = (M A)[r][j], the 4 rows meet in LDS, and Y = A^T Z + bias (+ ReLU / GELU) is
// stored as float2 pixel pairs.
#include <stdlib.h>

#include "common.h"
#include "prof.h"

namespace tsplat {
namespace wino {

constexpr int kThreads = 256;
constexpr int kCoB = 32;     // output channels per workgroup
constexpr int kTiles = 32;   // output tiles per workgroup
constexpr int kCiB = 8;      // channel padding granule; a chunk is CIB = 8 or 16 channels

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kMaxSrc = 6;  // input sources concatenated along channels (read in place)

struct Args {
    const float* src[kMaxSrc];  // source s: [n][cs[s]][h][w]; channel c of the conv input is
    int cs[kMaxSrc];            // channel c - (cs[0] + .. + cs[s-1]) of the source it falls in
    int nsrc;
    const float* u;      // packed U: [16][co_blocks][ci_pad / 2][2][32]
    const float* bias;   // [co] or null
    float* y;            // [n][co][h][w]
    int n, ci, h, w, co, ci_pad, co_blocks;
    int th, tw, tbx, tby, bx, by;  // tiles per image, tile-block shape, tile blocks per image row / column
    int act;             // 0 none, 1 ReLU, 2 GELU (erf)
};

__device__ __forceinline__ float act_fn(float v, int act) {
    if (act == 1) return fmaxf(v, 0.0f);
    if (act == 2) return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
    return v;
}

// U = G g G^T, G = [[1, 0, 0], [1/2, 1/2, 1/2], [1/2, -1/2, 1/2], [0, 0, 1]], packed as the A
// operand of v_mfma_f32_32x32x2_f32: lane l of k-step (ci pair) p reads U[co = 32 b + (l & 31)]
// [ci = 2 p + (l >> 5)], i.e. 64 consecutive floats. Padded co / ci entries are 0.
__global__ void __launch_bounds__(256) weight_kernel(const float* __restrict__ g, float* __restrict__ u, int co,
                                                     int ci, int ci_pad, int co_blocks) {
    const int idx = blockIdx.x * 256 + threadIdx.x;  // over co_blocks * 32 * ci_pad
    if (idx >= co_blocks * 32 * ci_pad) return;
    const int c = idx % ci_pad, o = idx / ci_pad;
    float k[3][3];
    const bool ok = o < co && c < ci;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) k[i][j] = ok ? g[((size_t)o * ci + c) * 9 + 3 * i + j] : 0.0f;
    float t[4][3];  // G g
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        t[0][j] = k[0][j];
        t[1][j] = 0.5f * (k[0][j] + k[1][j] + k[2][j]);
        t[2][j] = 0.5f * (k[0][j] - k[1][j] + k[2][j]);
        t[3][j] = k[2][j];
    }
    const int b = o / 32, ol = o % 32;
    const size_t plane = (size_t)co_blocks * ci_pad * 32;  // floats per xi
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float uu[4] = {t[r][0], 0.5f * (t[r][0] + t[r][1] + t[r][2]), 0.5f * (t[r][0] - t[r][1] + t[r][2]),
                             t[r][2]};
#pragma unroll
        for (int s = 0; s < 4; ++s)
            u[(4 * r + s) * plane + (((size_t)b * (ci_pad / 2) + c / 2) * 2 + (c & 1)) * 32 + ol] = uu[s];
    }
}

template <int CIB>
__global__ void __launch_bounds__(kThreads) conv_kernel(Args a) {
    constexpr int kP = CIB * kTiles / kThreads;  // (tile, channel) patches per thread per chunk
    __shared__ __attribute__((aligned(16))) float smem[2 * 16 * CIB * kTiles];  // sV x2, then Z
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int cob = blockIdx.y;
    const int blocks_per_img = a.bx * a.by;
    const int img = blockIdx.x / blocks_per_img, blk = blockIdx.x % blocks_per_img;
    const int ty0 = (blk / a.bx) * a.tby, tx0 = (blk % a.bx) * a.tbx;

    // this thread's transform slots: tile tt, channels cc + 8 k of each chunk
    const int tt = tid % kTiles, cc = tid / kTiles;
    const int ty = ty0 + tt / a.tbx, tx = tx0 + tt % a.tbx;
    const bool tile_ok = ty < a.th && tx < a.tw;
    const int y0 = 2 * ty - 1, x0 = 2 * tx - 1;
    const size_t hw = (size_t)a.h * a.w;
    // per-row / per-column validity of the 4x4 patch (zero padding)
    bool rok[4], cok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        rok[i] = tile_ok && y0 + i >= 0 && y0 + i < a.h;
        cok[i] = x0 + i >= 0 && x0 + i < a.w;
    }
    float d[kP][16];
    auto load_patch = [&](int chunk) {
#pragma unroll
        for (int k = 0; k < kP; ++k) {
            const int c = chunk * CIB + cc + 8 * k;
            // the source holding input channel c (channels past ci read the last one, zeroed)
            const float* src = nullptr;
            {
                int rem = min(c, a.ci - 1);
#pragma unroll
                for (int q = 0; q < kMaxSrc; ++q) {
                    if (q < a.nsrc && !src) {
                        if (rem < a.cs[q])
                            src = a.src[q] + ((size_t)img * a.cs[q] + rem) * hw;
                        else
                            rem -= a.cs[q];
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const bool ok = c < a.ci && rok[i] && cok[j];
                    d[k][4 * i + j] = ok ? src[(size_t)(y0 + i) * a.w + (x0 + j)] : 0.0f;
                }
        }
    };
    auto transform_store = [&](float* sV) {
#pragma unroll
        for (int k = 0; k < kP; ++k) {
            const float* dd = d[k];
            const int cl = cc + 8 * k;
            float t[16];  // B^T d
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                t[0 + j] = dd[0 + j] - dd[8 + j];
                t[4 + j] = dd[4 + j] + dd[8 + j];
                t[8 + j] = dd[8 + j] - dd[4 + j];
                t[12 + j] = dd[4 + j] - dd[12 + j];
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // (B^T d) B
                const float v0 = t[4 * r] - t[4 * r + 2], v1 = t[4 * r + 1] + t[4 * r + 2];
                const float v2 = t[4 * r + 2] - t[4 * r + 1], v3 = t[4 * r + 1] - t[4 * r + 3];
                sV[((4 * r + 0) * CIB + cl) * kTiles + tt] = v0;
                sV[((4 * r + 1) * CIB + cl) * kTiles + tt] = v1;
                sV[((4 * r + 2) * CIB + cl) * kTiles + tt] = v2;
                sV[((4 * r + 3) * CIB + cl) * kTiles + tt] = v3;
            }
        }
    };
    // A fragments of one chunk for this wave's 4 xi: [s][k-step]
    const size_t plane = (size_t)a.co_blocks * a.ci_pad * 32;
    const float* ub = a.u + (size_t)(4 * wid) * plane + (size_t)cob * (a.ci_pad / 2) * 64 + lane;
    float af[4][CIB / 2];
    auto load_a = [&](int chunk) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int kp = 0; kp < CIB / 2; ++kp) af[s][kp] = ub[s * plane + (size_t)(chunk * (CIB / 2) + kp) * 64];
    };

    floatx16 acc[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[s][r] = 0.0f;

    const int nchunks = a.ci_pad / CIB;
    load_patch(0);
    load_a(0);
    for (int ch = 0; ch < nchunks; ++ch) {
        float* sV = smem + (ch & 1) * (16 * CIB * kTiles);
        transform_store(sV);
        __syncthreads();  // sV(ch) complete; every wave is done with sV(ch - 2) = this buffer's last use
        float an[4][CIB / 2];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int kp = 0; kp < CIB / 2; ++kp) an[s][kp] = af[s][kp];
        if (ch + 1 < nchunks) {  // the next chunk's loads fly during this chunk's MFMAs
            load_patch(ch + 1);
            load_a(ch + 1);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const float* bsrc = sV + ((4 * wid + s) * CIB) * kTiles + lane;  // [2kp + (l >> 5)][l & 31]
#pragma unroll
            for (int kp = 0; kp < CIB / 2; ++kp)
                acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(an[s][kp], bsrc[2 * kp * kTiles], acc[s], 0, 0, 0);
        }
    }
    __syncthreads();  // all MFMAs' LDS reads done: smem becomes Z[r][j][co 32][tile 32]
    // C layout of 32x32x2: lane l holds tile l & 31, rows (co) (e & 3) + 8 (e >> 2) + 4 (l >> 5)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int col = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        const float z0 = acc[0][e] + acc[1][e] + acc[2][e];
        const float z1 = acc[1][e] - acc[2][e] - acc[3][e];
        smem[((wid * 2 + 0) * kCoB + col) * kTiles + (lane & 31)] = z0;
        smem[((wid * 2 + 1) * kCoB + col) * kTiles + (lane & 31)] = z1;
    }
    __syncthreads();
    const size_t out_img = (size_t)img * a.co * hw;
#pragma unroll
    for (int k = 0; k < (kCoB * kTiles) / kThreads; ++k) {
        const int pidx = tid + kThreads * k;
        const int col = pidx / kTiles, t2 = pidx % kTiles;
        const int o = cob * kCoB + col;
        const int oty = ty0 + t2 / a.tbx, otx = tx0 + t2 % a.tbx;
        if (o >= a.co || oty >= a.th || otx >= a.tw) continue;
        const float bv = a.bias ? a.bias[o] : 0.0f;
        float z[4][2];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 2; ++j) z[r][j] = smem[((r * 2 + j) * kCoB + col) * kTiles + t2];
        float* dst = a.y + out_img + (size_t)o * hw;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int py = 2 * oty + i;
            if (py >= a.h) continue;
            const float y0v = i == 0 ? z[0][0] + z[1][0] + z[2][0] : z[1][0] - z[2][0] - z[3][0];
            const float y1v = i == 0 ? z[0][1] + z[1][1] + z[2][1] : z[1][1] - z[2][1] - z[3][1];
            const float r0 = act_fn(y0v + bv, a.act), r1 = act_fn(y1v + bv, a.act);
            const int px = 2 * otx;
            float* p = dst + (size_t)py * a.w + px;
            if (px + 1 < a.w && ((reinterpret_cast<uintptr_t>(p) & 7) == 0)) {
                *reinterpret_cast<float2*>(p) = make_float2(r0, r1);
            } else {
                p[0] = r0;
                if (px + 1 < a.w) p[1] = r1;
            }
        }
    }
}

}  // namespace wino
}  // namespace tsplat

using namespace tsplat;

// input channels are padded to 16 (the larger chunk) in the packed filters
static int wino_ci_pad(int ci) { return (ci + 15) / 16 * 16; }

extern "C" size_t tsplat_wino_weight_floats(int32_t co, int32_t ci) {
    if (co <= 0 || ci <= 0) return 0;
    const int ci_pad = wino_ci_pad(ci);
    const int cob = (co + wino::kCoB - 1) / wino::kCoB;
    return (size_t)16 * cob * ci_pad * 32;
}

extern "C" int tsplat_wino_weight_f32(const float* weight, float* packed, int32_t co, int32_t ci, void* stream_) {
    if (!weight || !packed || co <= 0 || ci <= 0) return TSPLAT_EINVAL;
    const int ci_pad = wino_ci_pad(ci);
    const int cob = (co + wino::kCoB - 1) / wino::kCoB;
    const int total = cob * 32 * ci_pad;
    hipLaunchKernelGGL(wino::weight_kernel, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream_, weight,
                       packed, co, ci, ci_pad, cob);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

static int wino_launch(const float* const* srcs, const int32_t* chans, int32_t nsrc, const float* packed,
                       const float* bias, float* y, int32_t n, int32_t h, int32_t w, int32_t co, int32_t act,
                       void* stream_) {
    if (!srcs || !chans || nsrc <= 0 || nsrc > wino::kMaxSrc || !packed || !y || n <= 0 || h <= 0 || w <= 0 ||
        co <= 0 || act < 0 || act > 2)
        return TSPLAT_EINVAL;
    wino::Args a;
    int ci = 0;
    for (int q = 0; q < wino::kMaxSrc; ++q) {
        a.src[q] = q < nsrc ? srcs[q] : nullptr;
        a.cs[q] = q < nsrc ? chans[q] : 0;
        if (q < nsrc && (!srcs[q] || chans[q] <= 0)) return TSPLAT_EINVAL;
        ci += a.cs[q];
    }
    a.nsrc = nsrc;
    a.u = packed;
    a.bias = bias;
    a.y = y;
    a.n = n;
    a.ci = ci;
    a.h = h;
    a.w = w;
    a.co = co;
    a.ci_pad = wino_ci_pad(ci);
    a.co_blocks = (co + wino::kCoB - 1) / wino::kCoB;
    a.th = (h + 1) / 2;
    a.tw = (w + 1) / 2;
    // tile block of 32 tiles: the widest of 32 x 1, 16 x 2, 8 x 4 with the fewest padded tiles
    a.tbx = 32;
    {
        long best = -1;
        for (int tbx = 32; tbx >= 8; tbx /= 2) {
            const int tby = wino::kTiles / tbx;
            const long padded = (long)((a.tw + tbx - 1) / tbx) * tbx * ((a.th + tby - 1) / tby) * tby;
            if (best < 0 || padded < best) {
                best = padded;
                a.tbx = tbx;
            }
        }
    }
    a.tby = wino::kTiles / a.tbx;
    a.bx = (a.tw + a.tbx - 1) / a.tbx;
    a.by = (a.th + a.tby - 1) / a.tby;
    a.act = act;
    hipStream_t stream = (hipStream_t)stream_;
    TSPLAT_PROF_BEGIN(prof::kWinoConv, stream);
    // 8-channel chunks: 3 workgroups per CU (16-channel chunks, 2 per CU, measured 2-5 % slower;
    // TSPLAT_WINO_CIB=16 selects them). Two 32-channel output blocks per workgroup (128
    // accumulators per lane) spilled at 2 waves per SIMD and ran 1.3-2x slower.
    const char* e = getenv("TSPLAT_WINO_CIB");
    if (e && atoi(e) == 16)
        hipLaunchKernelGGL(wino::conv_kernel<16>, dim3(n * a.bx * a.by, a.co_blocks), dim3(wino::kThreads), 0,
                           stream, a);
    else
        hipLaunchKernelGGL(wino::conv_kernel<8>, dim3(n * a.bx * a.by, a.co_blocks), dim3(wino::kThreads), 0,
                           stream, a);
    TSPLAT_PROF_END(prof::kWinoConv, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_conv3x3_wino_f32_fwd(const float* x, const float* packed, const float* bias, float* y,
                                           int32_t n, int32_t ci, int32_t h, int32_t w, int32_t co, int32_t act,
                                           void* stream_) {
    return wino_launch(&x, &ci, 1, packed, bias, y, n, h, w, co, act, stream_);
}

extern "C" int tsplat_conv3x3_wino_cat_f32_fwd(const float* const* srcs, const int32_t* chans, int32_t nsrc,
                                               const float* packed, const float* bias, float* y, int32_t n,
                                               int32_t h, int32_t w, int32_t co, int32_t act, void* stream_) {
    return wino_launch(srcs, chans, nsrc, packed, bias, y, n, h, w, co, act, stream_);
}
