// 3x3 and 1x1 / stride 1 convolutions on bf16 MFMA (config C3's dense layers) for gfx950.
//
// Semantics: F.conv2d(up(cat(srcs, 1)), w, bias, stride 1, padding k // 2) under bf16 autocast, up =
// optional nearest 2x upsample (the U-Net Upsample block unet.py:105-137) read in place (the
// reference's nn.Conv2d layers of the depth predictor U-Nets ldm_unet/unet.py:212-250 and its
// conv heads depth_predictor_trans.py:110-125, run by the C3 config in bf16): sources bf16 or fp32
// (rounded to bf16 on load, as autocast's cast would), weights and bias bf16, fp32 accumulation,
// bias (+ SiLU / GELU / ReLU) in fp32, output bf16 NCHW.
//
// Why: MIOpen runs these NCHW bf16 convolutions as im2col (`Im2d2Col_v2`) + GEMM or as CK NHWC
// kernels wrapped in NCHW<->NHWC `batched_transpose` launches; together ~6 ms of C3's 28 ms step.
// This kernel reads each NCHW input once into LDS and writes the NCHW output once.
//
// Implicit GEMM: Y[co][px] = sum_(tap, ci) W[co][tap, ci] X[ci][px + tap offset] (9 taps or 1), one
// v_mfma_f32_32x32x16_bf16 per (tap, 16-channel chunk, 32 x 32 output tile):
//   A = W[co = 32 cb + c][ci = 16 k + 8 h + j]   (lane l = c + 32 h, element j; packed once on the host
//       as [co block][chunk][tap][64 lanes][8] bf16, one 16-B load per lane and tap);
//   B = X[ci = 16 k + 8 h + j][pixel p = c]      (one ds_read_b128 from the LDS tile);
//   C: lane holds pixel c, output channels 8 (r >> 2) + 4 h + (r & 3) in register r.
// Workgroup = 4 waves over a TH x TW pixel block (P = TH TW = 128 or 256 pixels) x 32 CT output
// channels: wave w takes co tile w % CT and NT = 2 column tiles of 32 pixels. Per chunk of 16 input
// channels the block (3x3: plus a 1-row / 8-column halo) is staged as [row][channel half][column][8
// channels] (each pixel's 8 channels of a half = one 16-B LDS word, so a wave's B reads are
// contiguous 16-lane runs): a thread loads 8 channels x 8 pixels (eight 16-B row segments of the
// NCHW map, coalesced across lanes), transposes them in registers, writes 8 LDS words. Double
// buffered, one barrier per chunk; the next chunk's loads and weights are in flight during the
// current chunk's 9 NT MFMAs. Epilogue: bias + act in fp32 -> bf16 tile [co][pixel] in LDS -> 16-B
// row stores.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "common.h"

namespace tsplat {
namespace convbf16 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kThreads = 256;
constexpr int kMaxSrc = 4;

struct Args {
    const void* src[kMaxSrc];
    int src_begin[kMaxSrc + 1];  // first concatenated channel of each source (src_begin[nsrc] = ci)
    int src_f32[kMaxSrc];        // per source: 1 fp32, 0 bf16 (the RAGGED loader reads it per channel)
    int nsrc;
    const uint4* w;  // packed weights
    const float* bias;
    __bf16* y;
    int n, h, w_, ci, nchunk, co, act;  // h, w_: OUTPUT size (= the convolved map's)
    int up;                              // 1: sources are [h / 2, w_ / 2], nearest-upsampled on load
    int tiles_x, tiles_y;
    int wg_target;  // workgroups per launch (all co blocks): a few per CU
    int occ4;       // bf16 sources: the occupancy-4 register allocation (default; C3 1057 vs 1042 views/s)
    int big;        // 3x3 with c_in * c_out >= TSPLAT_CONVBF16_BIG (default 96 * 96) and >= 192 workgroups:
                    // the register-blocked form (C3 1019 -> 1062 views/s, profiles/r3/convbf16)
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

__device__ __forceinline__ uint32_t dup_bf16(uint32_t v16) { return (v16 & 0xffffu) * 0x10001u; }

// The 8 x 8 block of one staging task: channels c0 .. c0 + 7 (c0 a multiple of 8, so all in one
// source) x pixels x .. x + 7 (x a multiple of 8) of row y of the convolved map, as 8 channel rows
// of 8 bf16; zeros outside the map or past the last channel. The source is chosen with constant
// kernel-argument indices (a runtime index into the argument arrays would be a memory load per
// access) and the 8 loads are independent.
template <bool F32>
__device__ __forceinline__ void load_block(const Args& a, int n, int c0, int y, int x, uint4 (&st)[8]) {
    if (c0 >= a.ci || y < 0 || y >= a.h || x < 0 || x >= a.w_) {
#pragma unroll
        for (int j = 0; j < 8; ++j) st[j] = make_uint4(0u, 0u, 0u, 0u);
        return;
    }
    const char* base = reinterpret_cast<const char*>(a.src[0]);
    int cb = 0, ce = a.src_begin[1];
#pragma unroll
    for (int i = 1; i < kMaxSrc; ++i) {
        if (i < a.nsrc && c0 >= a.src_begin[i]) {
            base = reinterpret_cast<const char*>(a.src[i]);
            cb = a.src_begin[i];
            ce = a.src_begin[i + 1];
        }
    }
    const int cs = ce - cb;
    constexpr int kEl = F32 ? 4 : 2;
    if (a.up) {  // source pixels x / 2 .. x / 2 + 3 of row y / 2, each used twice
        const int hs = a.h >> 1, ws = a.w_ >> 1;
        const size_t plane = (size_t)hs * ws;
        const char* p = base + ((((size_t)n * cs + (c0 - cb)) * hs + (y >> 1)) * ws + (x >> 1)) * kEl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if constexpr (F32) {
                const float4 u = *reinterpret_cast<const float4*>(p + j * plane * kEl);
                st[j] = make_uint4(pack_bf16x2(u.x, u.x), pack_bf16x2(u.y, u.y), pack_bf16x2(u.z, u.z),
                                   pack_bf16x2(u.w, u.w));
            } else {
                const uint2 u = *reinterpret_cast<const uint2*>(p + j * plane * kEl);
                st[j] = make_uint4(dup_bf16(u.x), dup_bf16(u.x >> 16), dup_bf16(u.y), dup_bf16(u.y >> 16));
            }
        }
        return;
    }
    const size_t plane = (size_t)a.h * a.w_;
    const char* p = base + ((((size_t)n * cs + (c0 - cb)) * a.h + y) * a.w_ + x) * kEl;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if constexpr (F32) {
            const float4* q = reinterpret_cast<const float4*>(p + j * plane * kEl);
            const float4 u = q[0], v = q[1];
            st[j] = make_uint4(pack_bf16x2(u.x, u.y), pack_bf16x2(u.z, u.w), pack_bf16x2(v.x, v.y),
                               pack_bf16x2(v.z, v.w));
        } else {
            st[j] = *reinterpret_cast<const uint4*>(p + j * plane * kEl);
        }
    }
}

// load_block for sources whose channel counts are not multiples of 8 or whose dtypes differ (the
// full-resolution heads read cat([features, images (3 channels), projection]) in place): each of
// the 8 channels picks its own source and dtype.
__device__ __forceinline__ void load_block_ragged(const Args& a, int n, int c0, int y, int x, uint4 (&st)[8]) {
    const bool inside = y >= 0 && y < a.h && x >= 0 && x < a.w_;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        st[j] = make_uint4(0u, 0u, 0u, 0u);
        if (!inside || c >= a.ci) continue;
        const char* base = reinterpret_cast<const char*>(a.src[0]);
        int cb = 0, ce = a.src_begin[1], f32 = a.src_f32[0];
#pragma unroll
        for (int i = 1; i < kMaxSrc; ++i) {
            if (i < a.nsrc && c >= a.src_begin[i]) {
                base = reinterpret_cast<const char*>(a.src[i]);
                cb = a.src_begin[i];
                ce = a.src_begin[i + 1];
                f32 = a.src_f32[i];
            }
        }
        const int cs = ce - cb;
        const int hs = a.up ? a.h >> 1 : a.h, ws = a.up ? a.w_ >> 1 : a.w_;
        const int ys = a.up ? y >> 1 : y, xs = a.up ? x >> 1 : x;
        const size_t e = (((size_t)n * cs + (c - cb)) * hs + ys) * ws + xs;
        if (f32) {
            const float* p = reinterpret_cast<const float*>(base) + e;
            if (a.up) {
                const float4 u = *reinterpret_cast<const float4*>(p);
                st[j] = make_uint4(pack_bf16x2(u.x, u.x), pack_bf16x2(u.y, u.y), pack_bf16x2(u.z, u.z),
                                   pack_bf16x2(u.w, u.w));
            } else {
                const float4 u = reinterpret_cast<const float4*>(p)[0], v = reinterpret_cast<const float4*>(p)[1];
                st[j] = make_uint4(pack_bf16x2(u.x, u.y), pack_bf16x2(u.z, u.w), pack_bf16x2(v.x, v.y),
                                   pack_bf16x2(v.z, v.w));
            }
        } else {
            const __bf16* p = reinterpret_cast<const __bf16*>(base) + e;
            if (a.up) {
                const uint2 u = *reinterpret_cast<const uint2*>(p);
                st[j] = make_uint4(dup_bf16(u.x), dup_bf16(u.x >> 16), dup_bf16(u.y), dup_bf16(u.y >> 16));
            } else {
                st[j] = *reinterpret_cast<const uint4*>(p);
            }
        }
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

// OCC: waves per SIMD the register allocation targets (2: no spills; 4, the default for bf16
// sources: more workgroups per CU to hide the staging loads' latency; same-box C3 1057 vs 1042
// views/s, profiles/r3/ab_r3d)
// SRC: 0 bf16 sources, 1 fp32 sources, 2 ragged / mixed (load_block_ragged)
// WCT x NT: 32-channel co tiles x 32-pixel column tiles per wave. (1, 2) = the small form, LDS
// epilogue; (2, 4) = the register-blocked form for the compute-heavy convolutions (full-resolution
// heads, 128-channel levels): per tap 2 A + 4 B LDS reads feed 8 MFMAs (the small form: 3 reads for
// 2), which takes the kernel off the LDS-bandwidth bound; its epilogue stores from registers.
template <int TW, int CT, int KS, int SRC, int OCC, int WCT, int NT>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(OCC))) conv_bf16_kernel(Args a) {
    constexpr int WR = CT / WCT;            // wave rows (co direction)
    constexpr int P = 32 * NT * (4 / WR);   // pixels per workgroup
    constexpr int TH = P / TW;
    constexpr int HY = KS / 2, HX = KS == 3 ? 8 : 0;  // staged halo rows / columns per side
    constexpr int NTAP = KS * KS;
    constexpr int LW = TW + 2 * HX;  // staged columns: x0 - HX .. x0 + TW + HX - 1
    constexpr int G = LW / 8;        // 8-pixel groups per staged row
    constexpr int SR = TH + 2 * HY;  // staged rows
    constexpr int kTasks = SR * 2 * G;
    constexpr int kBuf = SR * 2 * LW;  // 16-B words per buffer
    static_assert(kTasks <= kThreads, "one staging task per thread");
    static_assert(CT % WCT == 0 && 4 % WR == 0, "wave grid");
    constexpr bool kLdsEpi = WCT == 1;
    constexpr int kEpi = kLdsEpi ? 32 * CT * P * 2 / 16 : 0;  // bf16 epilogue tile [32 CT][P]
    constexpr int kW = CT * NTAP * 64;          // one chunk's A fragments of the CT co blocks
    constexpr int kWPer = (kW + kThreads - 1) / kThreads;
    __shared__ uint4 s_lds[2 * kBuf + 2 * kW + kEpi];
    uint4* const s_w = s_lds + 2 * kBuf;
    __bf16* const tile_out = reinterpret_cast<__bf16*>(s_lds + 2 * kBuf + 2 * kW);

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int c = lane & 31, h = lane >> 5;
    const int per_img = a.tiles_x * a.tiles_y;
    const int ntiles = a.n * per_img;
    const int ct0 = (wid % WR) * WCT, grp = wid / WR;  // this wave's first co tile, pixel group
    // this workgroup's pixel tiles: blockIdx.x, blockIdx.x + gridDim.x, ... (at least one)
    const int my_tiles = (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1;
    const int total = my_tiles * a.nchunk;  // flattened (tile, chunk) iterations
    auto tile_origin = [&](int ti, int& n, int& y0, int& x0) {
        const int t = (int)blockIdx.x + ti * (int)gridDim.x;
        n = t / per_img;
        const int r = t - n * per_img;
        y0 = (r / a.tiles_x) * TH;
        x0 = (r % a.tiles_x) * TW;
    };

    // staging task: (row, channel half, 8-pixel group)
    const bool task = tid < kTasks;
    const int tg = tid % G, thf = (tid / G) & 1, trow = tid / (2 * G);
    uint4 st[8];
    // the chunk's weights for all CT co blocks, [ct][tap][lane], staged through LDS with the input
    // (loaded once per workgroup instead of once per wave, one iteration ahead); a co block past
    // c_out reads zeros and its outputs are never stored
    uint4 wst[kWPer];
    auto load_iter = [&](int it) {
        const int ti = it / a.nchunk, k = it - ti * a.nchunk;
#pragma unroll
        for (int i = 0; i < kWPer; ++i) {
            const int idx = tid + i * kThreads;
            const int wct = idx / (NTAP * 64), rem = idx - wct * (NTAP * 64);
            const int wcob = blockIdx.y * CT + wct;
            wst[i] = (idx < kW && 32 * wcob < a.co)
                         ? a.w[((size_t)wcob * a.nchunk + k) * NTAP * 64 + rem]
                         : make_uint4(0u, 0u, 0u, 0u);
        }
        if (!task) return;
        int n, y0, x0;
        tile_origin(ti, n, y0, x0);
        if constexpr (SRC == 2)
            load_block_ragged(a, n, 16 * k + 8 * thf, y0 - HY + trow, x0 - HX + 8 * tg, st);
        else
            load_block<SRC == 1>(a, n, 16 * k + 8 * thf, y0 - HY + trow, x0 - HX + 8 * tg, st);
    };
    auto store_chunk = [&](int buf) {
#pragma unroll
        for (int i = 0; i < kWPer; ++i)
            if (tid + i * kThreads < kW) s_w[buf * kW + tid + i * kThreads] = wst[i];
        if (!task) return;
        uint4 px[8];
        transpose8(st, px);
        uint4* dst = s_lds + buf * kBuf + (trow * 2 + thf) * LW + 8 * tg;
#pragma unroll
        for (int p = 0; p < 8; ++p) dst[p] = px[p];
    };

    // LDS word of (pixel p of column tile j) at tap (0, 0): staged row p / TW, column p % TW + HX - KS / 2
    int bbase[NT];
#pragma unroll
    for (int k = 0; k < NT; ++k) {
        const int p = 32 * (grp * NT + k) + c;
        bbase[k] = ((p / TW) * 2 + h) * LW + (p % TW) + HX - KS / 2;
    }
    floatx16 acc[WCT][NT];

    // software pipeline over the flattened (tile, chunk) sequence: the loads of iteration it + 1
    // (next chunk, or the next tile's first chunk) fly during iteration it's MFMAs, so the
    // workgroup streams tiles instead of paying a memory round trip per tile
    load_iter(0);
    for (int it = 0; it < total; ++it) {
        const int ti = it / a.nchunk, k = it - ti * a.nchunk;
        const int buf = it & 1;
        store_chunk(buf);
        __syncthreads();
        if (it + 1 < total) load_iter(it + 1);
        if (k == 0) {
#pragma unroll
            for (int wc = 0; wc < WCT; ++wc)
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[wc][j][r] = 0.0f;
        }
        const uint4* sb = s_lds + buf * kBuf;
        const uint4* sw = s_w + buf * kW + ct0 * NTAP * 64 + lane;
#pragma unroll
        for (int tap = 0; tap < NTAP; ++tap) {
            const int off = (tap / KS) * 2 * LW + (tap % KS);
            bf16x8 av[WCT], bv[NT];
#pragma unroll
            for (int wc = 0; wc < WCT; ++wc) av[wc] = __builtin_bit_cast(bf16x8, sw[(wc * NTAP + tap) * 64]);
#pragma unroll
            for (int j = 0; j < NT; ++j) bv[j] = __builtin_bit_cast(bf16x8, sb[bbase[j] + off]);
#pragma unroll
            for (int wc = 0; wc < WCT; ++wc)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[wc][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[wc], bv[j], acc[wc][j], 0, 0, 0);
        }
        if (k + 1 == a.nchunk) {
            int n, y0, x0;
            tile_origin(ti, n, y0, x0);
            if constexpr (kLdsEpi) {
                // bias + act in fp32 -> bf16 [co_local][pixel] in its own LDS buffer (its previous
                // readers finished before this iteration's barrier) -> 16-B row stores
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int col = 32 * ct0 + 8 * (r >> 2) + 4 * h + (r & 3);
                    const int co = 32 * (blockIdx.y * CT + ct0) + 8 * (r >> 2) + 4 * h + (r & 3);
                    const float bias = (a.bias && co < a.co) ? a.bias[co] : 0.0f;
#pragma unroll
                    for (int j = 0; j < NT; ++j)
                        tile_out[col * P + 32 * (grp * NT + j) + c] = (__bf16)act_fn(acc[0][j][r] + bias, a.act);
                }
                __syncthreads();
                constexpr int kItems = 32 * CT * P / 8;
#pragma unroll
                for (int i = tid; i < kItems; i += kThreads) {
                    const int col = i / (P / 8), pg = i % (P / 8);
                    const int co = 32 * CT * blockIdx.y + col;
                    const int py = y0 + (8 * pg) / TW, px = x0 + (8 * pg) % TW;
                    if (co < a.co && py < a.h && px < a.w_) {
                        const uint4 v = *reinterpret_cast<const uint4*>(tile_out + col * P + 8 * pg);
                        *reinterpret_cast<uint4*>(a.y + (((size_t)n * a.co + co) * a.h + py) * a.w_ + px) = v;
                    }
                }
            } else {
                // straight from the accumulators: per register, 32 lanes store one co row's 32
                // consecutive pixels (64-B segments)
#pragma unroll
                for (int wc = 0; wc < WCT; ++wc)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int co = 32 * (blockIdx.y * CT + ct0 + wc) + 8 * (r >> 2) + 4 * h + (r & 3);
                        if (co >= a.co) continue;
                        const float bias = a.bias ? a.bias[co] : 0.0f;
#pragma unroll
                        for (int j = 0; j < NT; ++j) {
                            const int p = 32 * (grp * NT + j) + c;
                            const int py = y0 + p / TW, px = x0 + p % TW;
                            if (py < a.h && px < a.w_)
                                a.y[(((size_t)n * a.co + co) * a.h + py) * a.w_ + px] =
                                    (__bf16)act_fn(acc[wc][j][r] + bias, a.act);
                        }
                    }
            }
        }
    }
}

template <int TW, int CT, int KS, int WCT = 1, int NT = 2>
static void launch_tw(const Args& a, int src_mode, hipStream_t stream) {
    constexpr int P = 32 * NT * (4 / (CT / WCT));
    constexpr int TH = P / TW;
    Args b = a;
    b.tiles_x = ceil_div(a.w_, TW);
    b.tiles_y = ceil_div(a.h, TH);
    // enough workgroups to fill every CU a few times over; each streams its share of the tiles
    const int ntiles = a.n * b.tiles_x * b.tiles_y, cob = ceil_div(a.co, 32 * CT);
    // a multiple of 8 workgroups per output block: workgroup (x, y) is dispatched to XCD (x + y gx) % 8, so
    // the output blocks of one pixel tile then share an XCD and its L2 (the input tile is fetched once)
    const int want = std::max(8, a.wg_target / cob / 8 * 8);
    dim3 grid(std::min(ntiles, want), cob);
    if (src_mode == 2)
        hipLaunchKernelGGL((conv_bf16_kernel<TW, CT, KS, 2, 2, WCT, NT>), grid, dim3(kThreads), 0, stream, b);
    else if (src_mode == 1)
        hipLaunchKernelGGL((conv_bf16_kernel<TW, CT, KS, 1, 2, WCT, NT>), grid, dim3(kThreads), 0, stream, b);
    else if (a.occ4 && WCT == 1)
        hipLaunchKernelGGL((conv_bf16_kernel<TW, CT, KS, 0, 4, WCT, NT>), grid, dim3(kThreads), 0, stream, b);
    else
        hipLaunchKernelGGL((conv_bf16_kernel<TW, CT, KS, 0, 2, WCT, NT>), grid, dim3(kThreads), 0, stream, b);
}

template <int CT, int KS>
static void launch_ct(const Args& a, int src_mode, hipStream_t stream) {
    if (a.w_ >= 64)
        launch_tw<64, CT, KS>(a, src_mode, stream);
    else if (a.w_ >= 32)
        launch_tw<32, CT, KS>(a, src_mode, stream);
    else if (a.w_ >= 16)
        launch_tw<16, CT, KS>(a, src_mode, stream);
    else
        launch_tw<8, CT, KS>(a, src_mode, stream);
}

}  // namespace convbf16
}  // namespace tsplat

extern "C" size_t tsplat_conv2d_bf16_weight_bytes(int32_t c_out, int32_t c_in, int32_t ksize) {
    if (c_out <= 0 || c_in <= 0 || !(ksize == 1 || ksize == 3)) return 0;
    return (size_t)tsplat::ceil_div(c_out, 32) * tsplat::ceil_div(c_in, 16) * ksize * ksize * 64 * 16;
}

extern "C" int tsplat_conv2d_bf16_fwd(const void* const* srcs, const int32_t* src_channels, int32_t nsrc,
                                      const int32_t* src_f32, const void* w_packed, const float* bias, void* y,
                                      int32_t batch, int32_t height, int32_t width, int32_t c_out, int32_t ksize,
                                      int32_t upsample, int32_t act, void* stream_) {
    using namespace tsplat::convbf16;
    if (!srcs || !src_channels || !src_f32 || nsrc < 1 || nsrc > kMaxSrc || !w_packed || !y) return TSPLAT_EINVAL;
    if (batch <= 0 || height <= 0 || width <= 0 || c_out <= 0 || (width & 7) || act < 0 || act > 3)
        return TSPLAT_EINVAL;
    if (!(ksize == 1 || ksize == 3) || !(upsample == 0 || upsample == 1) || (upsample && (height & 1)))
        return TSPLAT_EINVAL;
    Args a{};
    int ci = 0;
    bool ragged = false;
    for (int s = 0; s < nsrc; ++s) {
        if (!srcs[s] || src_channels[s] <= 0 || !(src_f32[s] == 0 || src_f32[s] == 1)) return TSPLAT_EINVAL;
        ragged = ragged || (src_channels[s] & 7) || src_f32[s] != src_f32[0];
        a.src[s] = srcs[s];
        a.src_f32[s] = src_f32[s];
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
    a.up = upsample;
    {
        const char* e = getenv("TSPLAT_CONVBF16_WGS");  // A/B knob: workgroups per launch
        const char* o = getenv("TSPLAT_CONVBF16_OCC");  // "2": the spill-free allocation (A/B knob)
        a.occ4 = !(o && !strcmp(o, "2"));
        a.wg_target = e ? std::max(1, atoi(e)) : (a.occ4 ? 256 * 4 : 256 * 2);
        const char* bg = getenv("TSPLAT_CONVBF16_BIG");  // A/B knob: c_in * c_out threshold, 0 = off
        const long big_min = bg ? atol(bg) : 96L * 96L;
        // ... and only with enough 512-pixel tiles to fill the CUs (16 x 128 -> 128 at 32^2: 64
        // workgroups, 51 vs 25 us in the small form; at 64^2: 256, 79 vs 97 us for 256 -> 128)
        const long wgs = ((long)batch * height * width + 511) / 512 * ((c_out + 63) / 64);
        a.big = big_min > 0 && (long)ci * c_out >= big_min && wgs >= 192;
    }
    hipStream_t stream = (hipStream_t)stream_;
    const int f32 = ragged ? 2 : src_f32[0];  // loader mode
    if (ksize == 3) {
        if (a.big && c_out > 32 && width >= 32) {
            // register-blocked form: 64 co x 512 pixels per workgroup
            if (width >= 64)
                launch_tw<64, 2, 3, 2, 4>(a, f32, stream);
            else
                launch_tw<32, 2, 3, 2, 4>(a, f32, stream);
        } else if (c_out <= 32) {
            launch_ct<1, 3>(a, f32, stream);
        } else {
            launch_ct<2, 3>(a, f32, stream);
        }
    } else {
        if (c_out <= 32)
            launch_ct<1, 1>(a, f32, stream);
        else
            launch_ct<2, 1>(a, f32, stream);
    }
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
