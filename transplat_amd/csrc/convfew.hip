// 3x3 / stride 1 / pad 1 convolution of FEW-channel, full-resolution maps in split-bf16 ("bf16x3")
// precision: the refine U-Net's 32-channel 256^2 / 128^2 levels and the depth head
// (reference src/model/encoder/matching/depth_predictor_trans.py:138-160 refine_unet / to_disparity,
// ldm_unet/unet.py ResBlocks at model_channels = 32).
//
// Why not the Winograd kernel (winoconv3.hip) there: with 32-64 input channels a Winograd block has
// 2-4 chunks of work between its prologue (region loads, planes, A fragments) and its epilogue (Z
// fold, inverse transform, stores), so at b = 1 a 32 -> 32 conv over 2 x 256^2 ran at ~1.3 TB/s of
// its 34 MB of I/O (25-37 us per launch, 14 launches on the depth predictor's serial path). Here the
// product is a plain implicit GEMM -- out[co][px] = sum_(tap, ci) W[co][ci][tap] x[ci][px + tap],
// K = 9 ci -- whose input is staged ONCE per workgroup as an LDS image of the block's rows (+ 1-row /
// 4-column halo) in channel-innermost bf16 hi / lo form, so every MFMA B fragment (8 channels of one
// pixel) is one ds_read_b128 and the 9 taps re-read LDS, not memory.
//
// Workgroup: 4 waves, an output block of TR rows x 64 columns x 32 CB channels; units (32-pixel row
// segment, 32-channel output block) dealt round-robin to the waves, each unit one 32x32 fp32
// accumulator. Per 32-channel pass: stage the region (each thread item = 8 channels x 4 pixels: 8
// float4 loads -> 8 ds_write_b128 of hi / lo), barrier, then for tap x 16-channel chunk: A hi / lo
// fragments of the packed weight (kernels.conv_pack_weight_x3 layout, prefetched one k-step ahead),
// per unit B hi / lo from LDS and the three products lo*hi + hi*lo + hi*hi (<= 3 * 2^-18 relative per
// product, fp32 accumulation). Epilogue: + bias, activation, + residual(s), NCHW stores (32
// consecutive pixels per register and half-wave). ReLU-on-load and multi-source (concatenated) input
// as the Winograd kernel has them.
#include <stdlib.h>

#include "common.h"
#include "prof.h"

namespace tsplat {
namespace convfew {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kMaxSrc = 6;
constexpr int kCols = 64;            // output columns per workgroup
constexpr int kRC = kCols + 8;       // region columns: x0 - 4 .. x0 + 67 (16-B aligned float4 rows)
constexpr int kCP = 32;              // input channels per pass
constexpr int kPS = kCP + 8;         // bf16 per region pixel (padded: conflict-free b128 reads)
constexpr int kMaxCi = 128;

struct Args {
    const float* src[kMaxSrc];
    int cs[kMaxSrc];
    int nsrc;
    const uint4* wp;     // packed weight [cot][9][ng][hl][64 lanes] uint4 (8 bf16)
    const float* bias;   // [co] or null
    const float* res;    // [n][co][h][w] or null
    const float* res2;   // [n][co][h][w] or null
    float* y;            // [n][co][h][w]
    int n, ci, h, w, co, ng, cot;  // ng = ceil(ci / 16) chunks, cot = ceil(co / 32)
    int act;             // 0 none, 1 ReLU, 2 GELU (erf)
    int relu_in;
    int rb, cb;          // row / column blocks per image
    int abl;             // diagnostics only (TSPLAT_FEW_ABL): 1 no input loads, 2 no MFMAs, 4 no stores
};

__device__ __forceinline__ float act_fn(float v, int act) {
    if (act == 1) return fmaxf(v, 0.0f);
    if (act == 2) return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
    return v;
}

// plane of input channel c (concatenated sources), or null past the last channel; the source loop is
// unrolled so every a.src[q] / a.cs[q] is a constant kernel-argument offset (a runtime index into the
// argument struct would copy it to scratch)
__device__ __forceinline__ const float* plane(const Args& a, int img, int c) {
    const float* p = nullptr;
    if (c >= a.ci) return p;
#pragma unroll
    for (int q = 0; q < kMaxSrc; ++q) {
        if (!p && q < a.nsrc) {
            if (c < a.cs[q])
                p = a.src[q] + ((size_t)img * a.cs[q] + c) * ((size_t)a.h * a.w);
            else
                c -= a.cs[q];
        }
    }
    return p;
}

// The pass's A fragments live in registers (a wave needs only its own output block's 18 k-steps: 36
// uint4), loaded after the region is staged (the staging registers are dead then; the co-resident
// workgroup covers their latency), so the LDS holds just the image and two workgroups share a CU.
// (Measured against A staged in LDS with one workgroup per CU: 20.9 vs 24.1 us for 2 x 32 -> 32 at
// 256^2, tools/few_sweep.sh, profiles/r6/few_sweep.log.)
template <int TR, int CB>
__global__ void __launch_bounds__(256, 2) conv_kernel(Args a) {
    constexpr int R = TR + 2;                 // region rows
    constexpr int WPC = 4 / CB;               // waves per 32-channel output block
    constexpr int UPW = 2 * TR / WPC;         // 32-pixel row segments per wave
    static_assert(UPW >= 1 && (2 * TR) % WPC == 0, "segments per wave");
    constexpr int HL = R * kRC * kPS;         // bf16 per hi (or lo) image
    __shared__ __attribute__((aligned(16))) __bf16 sIn[2 * HL];
    __shared__ const float* sPlane[kMaxCi];  // every input channel's plane of this image

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int blk = blockIdx.x;
    const int img = blk / (a.rb * a.cb), rem = blk - img * (a.rb * a.cb);
    const int y0 = (rem / a.cb) * TR, x0 = (rem % a.cb) * kCols;
    const int cob0 = blockIdx.y * CB;  // first 32-channel output block of this workgroup
    const int cbw = wid / WPC, wi = wid % WPC;  // this wave's output block and its rank in it

    floatx16 acc[UPW];
#pragma unroll
    for (int u = 0; u < UPW; ++u)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[u][e] = 0.0f;
    // plane table (the concatenation's channel -> source lookup once per workgroup, not per load: the
    // per-load form compiled to branches around every load, each draining the ones in flight)
    for (int c = tid; c < kMaxCi; c += 256) sPlane[c] = plane(a, img, min(c, a.ci - 1));
    __syncthreads();

    // staging item it = (row * 18 + c4) * 4 + q: 8 channels (8 q ..) x 4 pixels (columns 4 c4 ..); q
    // fastest, so the 16-B LDS writes of 16 lanes hit 16 distinct bank quads (c4 stride 320 B = 16
    // banks, q stride 16 B), and each load instruction still reads 256-B runs of 4 planes; every
    // item's 8 float4 loads are issued before any is converted (one latency per pass)
    constexpr int ITEMS = (kCP / 8) * R * (kRC / 4);
    constexpr int IPT = (ITEMS + 255) / 256;
    auto stage = [&](int pass) __attribute__((always_inline)) {
        float4 v[IPT][8];
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const int it = tid + 256 * k;
            const int q = it & 3, c4 = (it >> 2) % (kRC / 4), row = (it >> 2) / (kRC / 4);
            const int y = y0 - 1 + row, x = x0 - 4 + 4 * c4;
            // a whole float4 is in or out of the map (w % 4 == 0). Loads stay unconditional (a branch
            // around each would drain the ones in flight): outside the map or past the last channel
            // they read a clamped in-map address and the value is replaced by zero (a shared zero
            // page instead was one hot L2 line for every halo load of the launch)
            const bool in = it < ITEMS && y >= 0 && y < a.h && x >= 0 && x < a.w;
            const int c0 = pass * kCP + 8 * q;
            const size_t po = (size_t)min(max(y, 0), a.h - 1) * a.w + min(max(x, 0), a.w - 4);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const bool ok = in && c0 + j < a.ci && !(a.abl & 1);
                const float* p = sPlane[min(c0 + j, kMaxCi - 1)] + po;
                // global address space: a pointer read from LDS would otherwise be a flat load, which
                // also counts against the LDS counter
                typedef float f4v __attribute__((ext_vector_type(4)));
                const f4v f = *(const __attribute__((address_space(1))) f4v*)p;
                v[k][j] = ok ? make_float4(f.x, f.y, f.z, f.w) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const int it = tid + 256 * k;
            if (it >= ITEMS) break;
            const int q = it & 3, c4 = (it >> 2) % (kRC / 4), row = (it >> 2) / (kRC / 4);
#pragma unroll
            for (int px = 0; px < 4; ++px) {
                bf16x8 hi, lo;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    float f = px == 0 ? v[k][j].x : px == 1 ? v[k][j].y : px == 2 ? v[k][j].z : v[k][j].w;
                    if (a.relu_in) f = fmaxf(f, 0.0f);
                    hi[j] = (__bf16)f;
                    lo[j] = (__bf16)(f - (float)hi[j]);
                }
                const int off = (row * kRC + 4 * c4 + px) * kPS + 8 * q;
                *reinterpret_cast<bf16x8*>(&sIn[off]) = hi;
                *reinterpret_cast<bf16x8*>(&sIn[HL + off]) = lo;
            }
        }
    };

    const int h = lane >> 5, n = lane & 31;
    const int passes = (a.ng + 1) / 2;
    uint4 ar[18][2];
    for (int pass = 0; pass < passes; ++pass) {
        if (pass) __syncthreads();  // every wave is done reading the previous pass's images
        stage(pass);
        {
            // this wave's A fragments of the pass (zero for a chunk past the last: its B rows are too)
            const int cot = min(cob0 + cbw, a.cot - 1);
#pragma unroll
            for (int ks = 0; ks < 18; ++ks) {
                const int g = 2 * pass + (ks & 1);
                const uint4* p = a.wp + ((((size_t)cot * 9 + (ks >> 1)) * a.ng + min(g, a.ng - 1)) * 2) * 64 + lane;
                ar[ks][0] = g < a.ng ? p[0] : make_uint4(0u, 0u, 0u, 0u);
                ar[ks][1] = g < a.ng ? p[64] : make_uint4(0u, 0u, 0u, 0u);
            }
        }
        __syncthreads();
        // 18 k-steps (tap, 16-channel chunk), unrolled: A from registers, B from LDS
        if (a.abl & 2) continue;
#pragma unroll
        for (int ks = 0; ks < 18; ++ks) {
            const int tap = ks >> 1, gl = ks & 1;
            const int dy = tap / 3, dx = tap - 3 * dy;  // region row i + dy, column j + dx + 3
            const bf16x8 ah = __builtin_bit_cast(bf16x8, ar[ks][0]);
            const bf16x8 al = __builtin_bit_cast(bf16x8, ar[ks][1]);
#pragma unroll
            for (int u = 0; u < UPW; ++u) {
                const int seg = wi + WPC * u;
                const int i = seg >> 1, j = (seg & 1) * 32 + n;
                const int off = ((i + dy) * kRC + j + dx + 3) * kPS + 16 * gl + 8 * h;
                const bf16x8 bh = *reinterpret_cast<const bf16x8*>(&sIn[off]);
                const bf16x8 bl = *reinterpret_cast<const bf16x8*>(&sIn[HL + off]);
                acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[u], 0, 0, 0);
                acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[u], 0, 0, 0);
                acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[u], 0, 0, 0);
            }
        }
    }

    // epilogue: register r of lane (n, h) = output channel 8 (r >> 2) + 4 h + (r & 3) of the wave's
    // block, pixel n of the segment
    const size_t hw = (size_t)a.h * a.w;
    if (a.abl & 4) {
        if (acc[0][0] == 12345.0f) a.y[0] = acc[UPW - 1][15];  // keep the accumulators live
        return;
    }
    // output tile through LDS (the input image is dead after the last MFMA): sOut[co][row][64 px],
    // then 16-B stores of whole 64-pixel rows (dword stores of 32-pixel runs, 64 per wave, ran at
    // ~1 TB/s: TSPLAT_FEW_ABL=4 measured the store phase at half the kernel)
    constexpr int CO = 32 * CB;
    static_assert(CO * TR * kCols * 4 <= 2 * HL * 2, "output tile fits the input image's LDS");
    float* sOut = reinterpret_cast<float*>(sIn);
    __syncthreads();  // every wave's last B reads are done
#pragma unroll
    for (int u = 0; u < UPW; ++u) {
        const int seg = wi + WPC * u;
        const int i = seg >> 1, j = (seg & 1) * 32 + n;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int col = 32 * cbw + 8 * (r >> 2) + 4 * h + (r & 3);
            sOut[(col * TR + i) * kCols + j] = acc[u][r];
        }
    }
    __syncthreads();
    constexpr int V4 = CO * TR * (kCols / 4);  // float4 of the tile
#pragma unroll 4
    for (int idx = tid; idx < V4; idx += 256) {
        const int c4 = idx % (kCols / 4), t2 = idx / (kCols / 4);
        const int i = t2 % TR, col = t2 / TR;
        const int o = 32 * cob0 + col, yy = y0 + i, xx = x0 + 4 * c4;
        if (o >= a.co || yy >= a.h || xx >= a.w) continue;  // w % 4 == 0: a float4 is whole
        const size_t off = ((size_t)img * a.co + o) * hw + (size_t)yy * a.w + xx;
        float4 v = *reinterpret_cast<const float4*>(&sOut[(col * TR + i) * kCols + 4 * c4]);
        const float bb = a.bias ? a.bias[o] : 0.0f;
        v = make_float4(act_fn(v.x + bb, a.act), act_fn(v.y + bb, a.act), act_fn(v.z + bb, a.act),
                        act_fn(v.w + bb, a.act));
        if (a.res) {
            const float4 r = *reinterpret_cast<const float4*>(a.res + off);
            v = make_float4(v.x + r.x, v.y + r.y, v.z + r.z, v.w + r.w);
        }
        if (a.res2) {
            const float4 r = *reinterpret_cast<const float4*>(a.res2 + off);
            v = make_float4(v.x + r.x, v.y + r.y, v.z + r.z, v.w + r.w);
        }
        *reinterpret_cast<float4*>(a.y + off) = v;
    }
}

}  // namespace convfew
}  // namespace tsplat

using namespace tsplat;

// Which (rows per block, output blocks per workgroup) form a launch of this shape takes, 0 = the
// shape is not one for this kernel. Rows: 8 where that still gives >= 256 workgroups, else 4, else 2.
// Which (rows per block, output blocks per workgroup) form a launch of this shape takes, 0 = the
// shape is not one for this kernel: 4-row blocks where that still gives >= 256 workgroups (two per
// CU), else 2-row ones; 64 output channels only in 2-row blocks (the LDS image of 4 rows is 69 KB).
extern "C" int32_t tsplat_conv3x3_few_form(int32_t n, int32_t ci, int32_t h, int32_t w, int32_t co) {
    if (n <= 0 || ci <= 0 || h <= 0 || w <= 0 || co <= 0 || w % 4 || co > 64 || ci > convfew::kMaxCi) return 0;
    const long cbk = (w + convfew::kCols - 1) / convfew::kCols;
    if (co > 32) return 22;
    if (const char* e = getenv("TSPLAT_FEW_TR")) {  // A/B knob: 4 or 2 rows per block
        const int tr = atoi(e);
        if (tr == 4 || tr == 2) return tr * 10 + 1;
    }
    return (long)n * ((h + 3) / 4) * cbk >= 256 ? 41 : 21;
}

extern "C" int tsplat_conv3x3_few_bf16x3_fwd(const float* const* srcs, const int32_t* chans, int32_t nsrc,
                                             const void* packed, const float* bias, const float* residual,
                                             const float* residual2, float* y, int32_t n, int32_t h, int32_t w,
                                             int32_t co, int32_t act, int32_t relu_in, void* stream_) {
    using namespace tsplat::convfew;
    if (!srcs || !chans || nsrc <= 0 || nsrc > kMaxSrc || !packed || !y || act < 0 || act > 2) return TSPLAT_EINVAL;
    Args a;
    int ci = 0;
    for (int q = 0; q < kMaxSrc; ++q) {
        a.src[q] = q < nsrc ? srcs[q] : nullptr;
        a.cs[q] = q < nsrc ? chans[q] : 0;
        if (q < nsrc && (!srcs[q] || chans[q] <= 0 || (reinterpret_cast<uintptr_t>(srcs[q]) & 15)))
            return TSPLAT_EINVAL;
        ci += a.cs[q];
    }
    const int form = tsplat_conv3x3_few_form(n, ci, h, w, co);
    if (!form) return TSPLAT_EINVAL;
    a.nsrc = nsrc;
    a.wp = (const uint4*)packed;
    a.bias = bias;
    a.res = residual;
    a.res2 = residual2;
    a.y = y;
    a.n = n;
    a.ci = ci;
    a.h = h;
    a.w = w;
    a.co = co;
    a.ng = (ci + 15) / 16;
    a.cot = (co + 31) / 32;
    a.act = act;
    a.relu_in = relu_in != 0;
    a.abl = getenv("TSPLAT_FEW_ABL") ? atoi(getenv("TSPLAT_FEW_ABL")) : 0;
    const int tr = form / 10, cb = form % 10;
    a.rb = (h + tr - 1) / tr;
    a.cb = (w + kCols - 1) / kCols;
    const dim3 grid(n * a.rb * a.cb, (a.cot + cb - 1) / cb);
    hipStream_t stream = (hipStream_t)stream_;
    const prof::ExtEvents ev = prof::ext_events(prof::kWinoConv);
#define TSPLAT_FEW(TR, CB)                                                                                 \
    hipExtLaunchKernelGGL((convfew::conv_kernel<TR, CB>), grid, dim3(256), 0, stream, ev.start, ev.stop, 0, a)
    switch (form) {
        case 41: TSPLAT_FEW(4, 1); break;
        case 21: TSPLAT_FEW(2, 1); break;
        default: TSPLAT_FEW(2, 2); break;
    }
#undef TSPLAT_FEW
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
