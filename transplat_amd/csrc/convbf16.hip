// 3x3 / stride 1 / pad 1 convolution on bf16 MFMA (config C3's dense layers) for gfx950.
//
// Semantics: F.conv2d(cat(srcs, 1), w, bias, stride 1, padding 1) under bf16 autocast (the
// reference's nn.Conv2d layers of the depth predictor U-Nets ldm_unet/unet.py:212-250 and its
// conv heads depth_predictor_trans.py:110-125, run by the C3 config in bf16): sources bf16 or fp32
// (rounded to bf16 on load, as autocast's cast would), weights and bias bf16, fp32 accumulation,
// bias (+ SiLU / GELU / ReLU) in fp32, output bf16 NCHW.
//
// Why: MIOpen runs these NCHW bf16 convolutions as im2col (`Im2d2Col_v2`) + GEMM or as CK NHWC
// kernels wrapped in NCHW<->NHWC `batched_transpose` launches; together ~6 ms of C3's 28 ms step.
// This kernel reads each NCHW input once into LDS and writes the NCHW output once.
//
// Implicit GEMM: Y[co][px] = sum_(tap, ci) W[co][tap, ci] X[ci][px + tap offset], one
// v_mfma_f32_32x32x16_bf16 per (tap, 16-channel chunk, 32 x 32 output tile):
//   A = W[co = 32 cb + c][ci = 16 k + 8 h + j]   (lane l = c + 32 h, element j; packed once on the host
//       as [co block][chunk][tap][64 lanes][8] bf16, one 16-B load per lane and tap);
//   B = X[ci = 16 k + 8 h + j][pixel p = c]      (one ds_read_b128 from the LDS tile);
//   C: lane holds pixel c, output channels 8 (r >> 2) + 4 h + (r & 3) in register r.
// Workgroup = 4 waves over a TH x TW pixel block (P = TH TW = 128 or 256 pixels) x 32 CT output
// channels: wave w takes co tile w % CT and NT = 2 column tiles of 32 pixels. Per chunk of 16 input
// channels the block plus a 1-row / 8-column halo is staged as [row][channel half][column][8
// channels] (each pixel's 8 channels of a half = one 16-B LDS word, so a wave's B reads are
// contiguous 16-lane runs): a thread loads 8 channels x 8 pixels (eight 16-B row segments of the
// NCHW map, coalesced across lanes), transposes them in registers, writes 8 LDS words. Double
// buffered, one barrier per chunk; the next chunk's loads and weights are in flight during the
// current chunk's 9 NT MFMAs. Epilogue: bias + act in fp32 -> bf16 tile [co][pixel] in LDS -> 16-B
// row stores.
#include <math.h>

#include "common.h"

namespace tsplat {
namespace convbf16 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kThreads = 256;
constexpr int kMaxSrc = 4;
constexpr int kNT = 2;  // 32-pixel column tiles per wave

struct Args {
    const void* src[kMaxSrc];
    int src_begin[kMaxSrc + 1];  // first concatenated channel of each source (src_begin[nsrc] = ci)
    int nsrc;
    const uint4* w;  // packed weights
    const float* bias;
    __bf16* y;
    int n, h, w_, ci, nchunk, co, act;
    int tiles_x, tiles_y;
};

__device__ __forceinline__ float act_fn(float v, int act) {
    if (act == 1) return v / (1.0f + __expf(-v));                       // SiLU
    if (act == 2) return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));  // GELU (erf)
    if (act == 3) return fmaxf(v, 0.0f);                                  // ReLU
    return v;
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
    const __bf16 a = (__bf16)lo, b = (__bf16)hi;
    return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}

// 8 bf16 pixels of one channel row segment (zeros outside the map / past the last channel)
template <bool F32>
__device__ __forceinline__ uint4 load8(const Args& a, int n, int c, int y, int x) {
    if (c >= a.ci || y < 0 || y >= a.h || x < 0 || x >= a.w_) return make_uint4(0u, 0u, 0u, 0u);
    int s = 0;
#pragma unroll
    for (int i = 1; i < kMaxSrc; ++i)
        if (i < a.nsrc && c >= a.src_begin[i]) s = i;
    const int cs = a.src_begin[s + 1] - a.src_begin[s];
    const size_t off = (((size_t)n * cs + (c - a.src_begin[s])) * a.h + y) * a.w_ + x;
    if constexpr (F32) {
        const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(a.src[s]) + off);
        const float4 u = p[0], v = p[1];
        return make_uint4(pack_bf16x2(u.x, u.y), pack_bf16x2(u.z, u.w), pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
    } else {
        return *reinterpret_cast<const uint4*>(reinterpret_cast<const __bf16*>(a.src[s]) + off);
    }
}

// 8 channels (in[j]: channel j, 8 pixels) -> 8 pixels (out[p]: 8 channels of pixel p)
__device__ __forceinline__ void transpose8(const uint4 (&in)[8], uint4 (&out)[8]) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {  // source dword d holds pixels 2d (low half) and 2d + 1
        uint32_t lo[4], hi[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t a = (&in[2 * e].x)[d], b = (&in[2 * e + 1].x)[d];
            lo[e] = (a & 0xffffu) | (b << 16);
            hi[e] = (a >> 16) | (b & 0xffff0000u);
        }
        out[2 * d] = make_uint4(lo[0], lo[1], lo[2], lo[3]);
        out[2 * d + 1] = make_uint4(hi[0], hi[1], hi[2], hi[3]);
    }
}

template <int TW, int CT, bool F32>
__global__ void __launch_bounds__(kThreads) conv3x3_bf16_kernel(Args a) {
    constexpr int P = 32 * (4 / CT) * kNT;  // pixels per workgroup
    constexpr int TH = P / TW;
    constexpr int LW = TW + 16;    // staged columns: x0 - 8 .. x0 + TW + 7
    constexpr int G = LW / 8;      // 8-pixel groups per staged row
    constexpr int kTasks = (TH + 2) * 2 * G;
    constexpr int kBuf = (TH + 2) * 2 * LW;  // 16-B words per buffer
    static_assert(kTasks <= kThreads, "one staging task per thread");
    static_assert(2 * kBuf * 16 >= 32 * CT * P * 2, "epilogue tile fits the staging buffers");
    __shared__ uint4 s_in[2][kBuf];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int c = lane & 31, h = lane >> 5;
    const int per_img = a.tiles_x * a.tiles_y;
    const int bx = blockIdx.x;
    const int n = bx / per_img, t = bx - n * per_img;
    const int y0 = (t / a.tiles_x) * TH, x0 = (t % a.tiles_x) * TW;
    const int ct = wid % CT, grp = wid / CT;
    const int cob = blockIdx.y * CT + ct;  // this wave's 32-channel output block

    // staging task: (row, channel half, 8-pixel group)
    const bool task = tid < kTasks;
    const int tg = tid % G, thf = (tid / G) & 1, trow = tid / (2 * G);
    uint4 st[8];
    auto load_chunk = [&](int k) {
        if (!task) return;
#pragma unroll
        for (int j = 0; j < 8; ++j) st[j] = load8<F32>(a, n, 16 * k + 8 * thf + j, y0 - 1 + trow, x0 - 8 + 8 * tg);
    };
    auto store_chunk = [&](int buf) {
        if (!task) return;
        uint4 px[8];
        transpose8(st, px);
        uint4* dst = &s_in[buf][(trow * 2 + thf) * LW + 8 * tg];
#pragma unroll
        for (int p = 0; p < 8; ++p) dst[p] = px[p];
    };
    // a wave whose 32-channel block lies past c_out (c_out not a multiple of 32 CT) reads no
    // weights and multiplies zeros; its outputs are never stored
    const bool cvalid = 32 * cob < a.co;
    const uint4* wsrc = a.w + (size_t)(cvalid ? cob : 0) * a.nchunk * 9 * 64 + lane;
    uint4 wf[9];
    auto load_w = [&](int k, uint4 (&dst)[9]) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) dst[tap] = cvalid ? wsrc[((size_t)k * 9 + tap) * 64] : make_uint4(0u, 0u, 0u, 0u);
    };

    // LDS word of (pixel p of column tile j) at tap (0, 0): row p / TW, column p % TW + 7
    int bbase[kNT];
#pragma unroll
    for (int k = 0; k < kNT; ++k) {
        const int p = 32 * (grp * kNT + k) + c;
        bbase[k] = ((p / TW) * 2 + h) * LW + (p % TW) + 7;
    }
    floatx16 acc[kNT];
#pragma unroll
    for (int k = 0; k < kNT; ++k)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[k][r] = 0.0f;

    load_chunk(0);
    load_w(0, wf);
    for (int k = 0; k < a.nchunk; ++k) {
        const int buf = k & 1;
        store_chunk(buf);
        __syncthreads();
        uint4 wn[9];
        if (k + 1 < a.nchunk) {
            load_chunk(k + 1);
            load_w(k + 1, wn);
        }
        const uint4* sb = s_in[buf];
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int off = (tap / 3) * 2 * LW + (tap % 3);
            const bf16x8 av = __builtin_bit_cast(bf16x8, wf[tap]);
#pragma unroll
            for (int j = 0; j < kNT; ++j) {
                const bf16x8 bv = __builtin_bit_cast(bf16x8, sb[bbase[j] + off]);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[j], 0, 0, 0);
            }
        }
        if (k + 1 < a.nchunk) {
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) wf[tap] = wn[tap];
        }
    }
    __syncthreads();  // every wave is done reading the staging buffers

    // epilogue: bias + act in fp32, bf16 tile [co_local][pixel] in LDS, then 16-B row stores
    __bf16* tile = reinterpret_cast<__bf16*>(&s_in[0][0]);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int col = 32 * ct + 8 * (r >> 2) + 4 * h + (r & 3);
        const int co = 32 * cob + 8 * (r >> 2) + 4 * h + (r & 3);
        const float b = (a.bias && co < a.co) ? a.bias[co] : 0.0f;
#pragma unroll
        for (int j = 0; j < kNT; ++j) tile[col * P + 32 * (grp * kNT + j) + c] = (__bf16)act_fn(acc[j][r] + b, a.act);
    }
    __syncthreads();
    constexpr int kItems = 32 * CT * P / 8;
#pragma unroll
    for (int i = tid; i < kItems; i += kThreads) {
        const int col = i / (P / 8), pg = i % (P / 8);
        const int co = 32 * CT * blockIdx.y + col;
        const int py = y0 + (8 * pg) / TW, px = x0 + (8 * pg) % TW;
        if (co < a.co && py < a.h && px < a.w_) {
            const uint4 v = *reinterpret_cast<const uint4*>(tile + col * P + 8 * pg);
            *reinterpret_cast<uint4*>(a.y + (((size_t)n * a.co + co) * a.h + py) * a.w_ + px) = v;
        }
    }
}

template <int TW, int CT>
static void launch_tw(const Args& a, bool f32, hipStream_t stream) {
    constexpr int P = 32 * (4 / CT) * kNT;
    constexpr int TH = P / TW;
    Args b = a;
    b.tiles_x = ceil_div(a.w_, TW);
    b.tiles_y = ceil_div(a.h, TH);
    dim3 grid(a.n * b.tiles_x * b.tiles_y, ceil_div(a.co, 32 * CT));
    if (f32)
        hipLaunchKernelGGL((conv3x3_bf16_kernel<TW, CT, true>), grid, dim3(kThreads), 0, stream, b);
    else
        hipLaunchKernelGGL((conv3x3_bf16_kernel<TW, CT, false>), grid, dim3(kThreads), 0, stream, b);
}

template <int CT>
static void launch_ct(const Args& a, bool f32, hipStream_t stream) {
    if (a.w_ >= 64)
        launch_tw<64, CT>(a, f32, stream);
    else if (a.w_ >= 32)
        launch_tw<32, CT>(a, f32, stream);
    else if (a.w_ >= 16)
        launch_tw<16, CT>(a, f32, stream);
    else
        launch_tw<8, CT>(a, f32, stream);
}

}  // namespace convbf16
}  // namespace tsplat

extern "C" size_t tsplat_conv3x3_bf16_weight_bytes(int32_t c_out, int32_t c_in) {
    if (c_out <= 0 || c_in <= 0) return 0;
    return (size_t)tsplat::ceil_div(c_out, 32) * tsplat::ceil_div(c_in, 16) * 9 * 64 * 16;
}

extern "C" int tsplat_conv3x3_bf16_fwd(const void* const* srcs, const int32_t* src_channels, int32_t nsrc,
                                       int32_t src_f32, const void* w_packed, const float* bias, void* y,
                                       int32_t batch, int32_t height, int32_t width, int32_t c_out, int32_t act,
                                       void* stream_) {
    using namespace tsplat::convbf16;
    if (!srcs || !src_channels || nsrc < 1 || nsrc > kMaxSrc || !w_packed || !y) return TSPLAT_EINVAL;
    if (batch <= 0 || height <= 0 || width <= 0 || c_out <= 0 || (width & 7) || act < 0 || act > 3)
        return TSPLAT_EINVAL;
    Args a{};
    int ci = 0;
    for (int s = 0; s < nsrc; ++s) {
        if (!srcs[s] || src_channels[s] <= 0 || (src_channels[s] & 7)) return TSPLAT_EINVAL;
        a.src[s] = srcs[s];
        a.src_begin[s] = ci;
        ci += src_channels[s];
        if ((int64_t)batch * src_channels[s] * height * width >= (1ll << 31)) return TSPLAT_EINVAL;
    }
    if ((int64_t)batch * c_out * height * width >= (1ll << 31)) return TSPLAT_EINVAL;
    a.src_begin[nsrc] = ci;
    for (int s = nsrc + 1; s <= kMaxSrc; ++s) a.src_begin[s] = ci;
    a.nsrc = nsrc;
    a.w = reinterpret_cast<const uint4*>(w_packed);
    a.bias = bias;
    a.y = reinterpret_cast<__bf16*>(y);
    a.n = batch;
    a.h = height;
    a.w_ = width;
    a.ci = ci;
    a.nchunk = tsplat::ceil_div(ci, 16);
    a.co = c_out;
    a.act = act;
    hipStream_t stream = (hipStream_t)stream_;
    if (c_out <= 32)
        launch_ct<1>(a, src_f32 != 0, stream);
    else
        launch_ct<2>(a, src_f32 != 0, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
