// Shifted-window cross/self attention of the multi-view transformer on gfx950 MFMA.
//
// Semantics: reference `single_head_split_window_attention`
// (src/model/encoder/backbone/multiview_transformer.py:57-206, both the 2-view and the multi-view
// branch) with the Swin mask of `generate_shift_window_attn_mask` (:17-54):
//   out[p] = softmax(q_p K_w^T / sqrt(C) + mask) V_w over the window w containing p, where windows
//   are the K x K splits of the map rolled by (-window_h/2, -window_w/2) on shifted layers,
//   keys of m views are ordered pixel-major / view-minor and the -100 region mask is tiled
//   view-major, so key j uses mask column j mod L (the reference's V >= 3 indexing, reproduced).
// The roll, the window partition and the mask are index arithmetic here: nothing is materialised
// (the reference allocates rolled copies, a [K^2, L, L] mask and [8, L, L] fp32 scores per call).
//
// Kernel: flash-style, one workgroup = 4 waves = 64 queries of one window; each wave owns 16
// queries. The keys of a window are split into ksplit ranges (one workgroup each, partials merged
// by a small combine kernel) so the 2-view 64x64 map (128 query blocks) still fills 256 CUs
// twice over; the next K/V tile's global loads are issued before the current tile's MFMAs.
// Exact-fp32 MFMA (v_mfma_f32_16x16x4_f32) for both contractions:
//   S^T[key, q] = K Q^T   (keys on MFMA rows, queries on lanes -> per-query softmax stats are
//                          per-lane, no cross-lane transpose)
//   O^T[d, q]  += V^T P^T (the S^T accumulator IS the P^T B-operand: lane (q, g) holds keys
//                          16t + 4g + r in register (t, r), exactly what k-step 4t + r needs)
// K and V tiles of 64 keys are gathered by pixel index into LDS (K XOR-swizzled per 16-B chunk so
// the 16 row reads of a ds_read_b128 group hit distinct banks; V rows padded to 132 floats so the
// column reads of the two half-waves hit disjoint banks).
#include <stdlib.h>
#include <string.h>

#include "common.h"
#include "prof.h"

namespace tsplat {
namespace winattn {

// TSPLAT_WA2_ABL (diagnostic builds only): removes one phase of the bf16 v2 loop -- 1 softmax,
// 2 PV MFMAs, 3 QK MFMAs, 4 next-tile gather + staging (results are wrong in such a build)
#ifndef TSPLAT_WA2_ABL
#define TSPLAT_WA2_ABL 0
#endif
constexpr int kAbl2 = TSPLAT_WA2_ABL;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kMaskLog2 = -100.0f * kLog2e;  // the reference's -100 mask, log2 domain

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// max of three scores as ONE gfx950 v_maximum3_f32 (IEEE-2019 maximum: NaN-propagating, so no
// canonicalising v_max_f32 x, x ahead of it as fmaxf's maxnum needs on MFMA results; the scores are
// finite, so the two agree). Compiler-visible on purpose: the hazard recognizer then pads the
// MFMA -> VALU read of the accumulators (s_nop 11 after a 32x32x16 chain). Round 5's inline-asm
// v_max3_f32 was invisible to it and read the last MFMA's destination 0 wait states after issue
// (a partial score, now and then: the bf16 v2 kernel's run-to-run drift). tests/test_isa_hazards.py
// checks every built code object for such a read.
__device__ __forceinline__ float max3_raw(float a, float b, float c) {
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}

// max / sum of lanes l and l ^ 32 (the two half-waves), in VALU via v_permlane32_swap instead of
// an LDS-routed ds_bpermute: swap(x, x) returns (x[row 0], x[row 1]) in every lane
__device__ __forceinline__ float halves_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float halves_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

#ifndef TSPLAT_WA_STAMP
#define TSPLAT_WA_STAMP 0  // diagnostic builds only (tools/build_stamp_wa.sh): per-workgroup phase clocks
#endif
#if TSPLAT_WA_STAMP
// [workgroup][16] uint64, written by thread 0 with vector stores: 0 wall clock at entry, 1 HW_ID |
// XCC_ID << 32, 2 shader clock at entry, 3 after the prologue barrier, 4 + t after key tile t
// (t < 8), 12 after the epilogue, 13 wall clock at the end
__device__ unsigned long long* g_wa_stamps = nullptr;
#define WA_STAMP(slot, val)                                                                          \
    do {                                                                                             \
        if (threadIdx.x == 0 && g_wa_stamps)                                                         \
            g_wa_stamps[(size_t)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 16 \
                        + (slot)] = (val);                                                           \
    } while (0)
#define WA_CLOCK() ((unsigned long long)__builtin_readcyclecounter())
#define WA_HWID()                                                                                    \
    ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |                      \
     ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32))
#else
#define WA_STAMP(slot, val) do {} while (0)
#endif

constexpr int kC = 128;          // channels (d_model of the reference transformer)
constexpr int kBQ = 64;          // queries per workgroup
constexpr int kBK = 64;          // keys per LDS tile
constexpr int kThreads = 256;
constexpr int kVStride = kC + 4;  // padded V row (floats)

typedef float floatx4 __attribute__((ext_vector_type(4)));

struct Params {
    int H, W, splits, shift, m, L;  // L = window pixels; shift != 0: shifted (masked) layer
    int shift_h, shift_w;           // roll of the shifted layer: half a window per axis
    int ksplit, keys_per_split;     // key range [s * keys_per_split, (s+1) * keys_per_split)
    int wh, ww, ww_log2;            // window rows / columns; log2(ww), or -1 if not a power of 2
    int kv_shift, nbatch;           // keys / values of query batch b come from batch (b + kv_shift) % nbatch
    float scale;
};

// t / ww and t % ww without a per-lane integer division when the window width is a power of 2
__device__ __forceinline__ void win_split(const Params& p, int t, int& ty, int& tx) {
    ty = p.ww_log2 >= 0 ? (t >> p.ww_log2) : t / p.ww;
    tx = t - ty * p.ww;
}

// split-key partials of one workgroup (64 queries): O (unnormalised, [64][128]), m, l
struct Partials {
    float* o;
    float* m;
    float* l;
};

// row of query t (in-window index) of window wi, batch b, key split ks in the partial arrays
__device__ __forceinline__ size_t pidx(const Params& p, int b, int wi, int ks, int t) {
    return (((size_t)b * p.splits * p.splits + wi) * p.ksplit + ks) * p.L + t;
}

// Logical (x, y, z) of this workgroup after the bijective XCD remap of its linear id: the
// dispatcher deals consecutive ids round-robin over the 8 XCDs, so without the remap the query
// blocks of one window (which all read the same K/V) would land on 8 different L2s.
__device__ __forceinline__ void xcd_block_coords(int& x, int& y, int& z) {
    const int X = gridDim.x, Y = gridDim.y;
    const int n = blockIdx.x + X * (blockIdx.y + Y * blockIdx.z);
    const int m = xcd_remap(n, X * Y * gridDim.z);
    x = m % X;
    y = (m / X) % Y;
    z = m / (X * Y);
}

// original pixel of in-window position t of window wi after the roll by -shift
__device__ __forceinline__ int win_pixel(const Params& p, int wi, int t) {
    const int sy = wi / p.splits, sx = wi - sy * p.splits;
    int ty, tx;
    win_split(p, t, ty, tx);
    int y = sy * p.wh + ty + p.shift_h;
    int x = sx * p.ww + tx + p.shift_w;
    if (y >= p.H) y -= p.H;
    if (x >= p.W) x -= p.W;
    return y * p.W + x;
}

// Swin region id of in-window position t of window wi (on the rolled grid)
__device__ __forceinline__ int win_region(const Params& p, int wi, int t) {
    const int sy = wi / p.splits, sx = wi - sy * p.splits;
    int ty, tx;
    win_split(p, t, ty, tx);
    const int Y = sy * p.wh + ty, X = sx * p.ww + tx;
    const int by = Y < p.H - p.wh ? 0 : (Y < p.H - p.wh / 2 ? 1 : 2);
    const int bx = X < p.W - p.ww ? 0 : (X < p.W - p.ww / 2 ? 1 : 2);
    return by * 3 + bx;
}

// key j of a window (pixel-major, view-minor over m key views): offset of its row in the
// [m, H*W] key/value maps and its mask region (mask column j mod L, the reference's tiling)
__device__ __forceinline__ void key_row(const Params& p, int wi, size_t HW, int j, size_t& off, int& region) {
    const int tk = p.m == 1 ? j : j / p.m, vi = j - tk * p.m;
    off = (size_t)vi * HW + win_pixel(p, wi, tk);
    region = p.shift ? win_region(p, wi, p.m == 1 ? j : j % p.L) : 0;
}

// K / V rows of one 64-key tile held in registers between the global gather and the LDS store
// (the next tile's loads are in flight while the current tile is computed)
struct TileRegs {
    float4 k[8], v[8];
};

__device__ __forceinline__ void load_tile(const Params& p, int wi, const float* kb, const float* vb,
                                          size_t HW, int k0, int tid, TileRegs& t, int& region) {
    const int r = tid >> 2, part = tid & 3;  // key row, 32-float quarter
    const int j = k0 + r;
    const int tk = j / p.m, vi = j - tk * p.m;
    const int kpix = win_pixel(p, wi, tk);
    const float4* ks = reinterpret_cast<const float4*>(kb + ((size_t)vi * HW + kpix) * kC + 32 * part);
    const float4* vs = reinterpret_cast<const float4*>(vb + ((size_t)vi * HW + kpix) * kC + 32 * part);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        t.k[i] = ks[i];
        t.v[i] = vs[i];
    }
    region = p.shift ? win_region(p, wi, j % p.L) : 0;
}

__device__ __forceinline__ void store_tile(float* sK, float* sV, int* sKeyRegion, int tid,
                                           const TileRegs& t, int region, bool shift) {
    const int r = tid >> 2, part = tid & 3;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int chunk = part * 8 + i;      // 16-B chunk in the 512-B row
        const int phys = chunk ^ (r & 15);   // XOR swizzle (low 4 bits)
        *reinterpret_cast<float4*>(&sK[r * kC + phys * 4]) = t.k[i];
        *reinterpret_cast<float4*>(&sV[r * kVStride + chunk * 4]) = t.v[i];
    }
    if (part == 0 && shift) sKeyRegion[r] = region;
}

// grid (query blocks, windows, batch * ksplit); ksplit > 1 writes Partials, else `out`
__global__ void __launch_bounds__(kThreads)
win_attn_f32_kernel(Params p, const float* __restrict__ q, const float* __restrict__ k,
                    const float* __restrict__ v, float* __restrict__ out, Partials part) {
    __shared__ __attribute__((aligned(16))) float sK[kBK * kC];
    __shared__ __attribute__((aligned(16))) float sV[kBK * kVStride];
    __shared__ int sKeyRegion[kBK];

    const int qblk = blockIdx.x, wi = blockIdx.y;
    const int b = blockIdx.z / p.ksplit, ks = blockIdx.z - b * p.ksplit;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = lane >> 4, ql = lane & 15;
    const size_t HW = (size_t)p.H * p.W;
    const float* qb = q + (size_t)b * HW * kC;
    const int bkv = p.kv_shift ? (b + p.kv_shift) % p.nbatch : b;
    const float* kb = k + (size_t)bkv * p.m * HW * kC;
    const float* vb = v + (size_t)bkv * p.m * HW * kC;

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

    const int kbeg = ks * p.keys_per_split, kend = kbeg + p.keys_per_split;
    TileRegs tr;
    int treg;
    load_tile(p, wi, kb, vb, HW, kbeg, tid, tr, treg);
    for (int k0 = kbeg; k0 < kend; k0 += kBK) {
        store_tile(sK, sV, sKeyRegion, tid, tr, treg, p.shift != 0);
        __syncthreads();
        if (k0 + kBK < kend) load_tile(p, wi, kb, vb, HW, k0 + kBK, tid, tr, treg);

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
        bmax = halves_max(bmax);
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
        bsum = halves_sum(bsum);
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

    if (p.ksplit == 1) {
        // ---- epilogue: O^T[d = 16dt + 4g + r][q] / l -> out[qpix][d]
        const float inv = 1.0f / l_run;
        float* dst = out + ((size_t)b * HW + qpix) * kC + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            float4 t4 = make_float4(o[dt][0] * inv, o[dt][1] * inv, o[dt][2] * inv, o[dt][3] * inv);
            *reinterpret_cast<float4*>(dst + 16 * dt) = t4;
        }
    } else {
        // ---- split-key partial: unnormalised O, running max and sum of this key range
        const size_t row = pidx(p, b, wi, ks, tq);
        float* dst = part.o + row * kC + 4 * g;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
            *reinterpret_cast<float4*>(dst + 16 * dt) = make_float4(o[dt][0], o[dt][1], o[dt][2], o[dt][3]);
        if (g == 0) {
            part.m[row] = m_run;
            part.l[row] = l_run;
        }
    }
}

// combine the ksplit partials of each query: out = sum_s e^(m_s - M) O_s / sum_s e^(m_s - M) l_s
// grid (L / 8, windows, batch); 32 threads per query, one float4 of channels each (1024+
// workgroups for the 2-view map: the partials are the only HBM/MALL traffic of the split)
__device__ __forceinline__ void store4(float* dst, float4 v) { *reinterpret_cast<float4*>(dst) = v; }
__device__ __forceinline__ void store4(__bf16* dst, float4 v) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<bf16x4*>(dst) = bf16x4{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
}

template <typename OutT>
__global__ void __launch_bounds__(kThreads)
win_attn_combine_kernel(Params p, Partials part, OutT* __restrict__ out) {
    const int wi = blockIdx.y, b = blockIdx.z;
    const int tq = blockIdx.x * (kThreads / 32) + (threadIdx.x >> 5), c4 = threadIdx.x & 31;
    const size_t HW = (size_t)p.H * p.W;
    float M = -INFINITY;
    for (int s = 0; s < p.ksplit; ++s) M = fmaxf(M, part.m[pidx(p, b, wi, s, tq)]);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    float L = 0.f;
    for (int s = 0; s < p.ksplit; ++s) {
        const size_t row = pidx(p, b, wi, s, tq);
        const float w = __expf(part.m[row] - M);
        L += w * part.l[row];
        const float4 t4 = reinterpret_cast<const float4*>(part.o + row * kC)[c4];
        acc.x += w * t4.x;
        acc.y += w * t4.y;
        acc.z += w * t4.z;
        acc.w += w * t4.w;
    }
    const float inv = 1.0f / L;
    const int qpix = win_pixel(p, wi, tq);
    store4(out + ((size_t)b * HW + qpix) * kC + 4 * c4, make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv));
}

// x32 / bf16 kernels store each wave's unnormalised O^T tile lane-contiguously: float4 number
// (dt * 4 + u) * 64 + lane of the wave's 16-KB slot holds O^T[d = 32 dt + 8u + 4h .. +3][query c]
// (lane = c + 32 h). Slot of (b, wi, ks, query block, wave) in the partial buffer (floats):
__device__ __forceinline__ size_t lane_tile_base(const Params& p, int b, int wi, int ks, int qblk, int wid) {
    const size_t nqb = (size_t)p.L / 128;
    return ((((size_t)b * p.splits * p.splits + wi) * p.ksplit + ks) * nqb + qblk) * 128 * kC + (size_t)wid * 32 * kC;
}

// combine for the lane-contiguous layout: grid (L / 128 * 16, windows, batch), 256 threads; a
// workgroup owns 256 consecutive float4s of one 128-query block (one wave slot's quarter, i.e.
// 32 queries): it forms those queries' weights e^(m_s - M) / L in LDS, then reads every partial
// float4 coalesced
template <typename OutT>
__global__ void __launch_bounds__(kThreads)
win_attn_combine_x32_kernel(Params p, Partials part, OutT* __restrict__ out) {
    __shared__ float s_w[8][32];
    const int qblk = blockIdx.x >> 4, part16 = blockIdx.x & 15, wi = blockIdx.y, b = blockIdx.z;
    const int t = threadIdx.x;
    const int idx = part16 * kThreads + t;  // float4 index within the 128-query block
    const int wid = idx >> 10, rem = idx & 1023, du = rem >> 6, lane = rem & 63;
    const int c = lane & 31, h = lane >> 5, dt = du >> 2, u = du & 3;
    const size_t HW = (size_t)p.H * p.W;
    if (t < 32) {
        const int tq = qblk * 128 + wid * 32 + t;
        float M = -INFINITY;
        for (int s = 0; s < p.ksplit; ++s) M = fmaxf(M, part.m[pidx(p, b, wi, s, tq)]);
        float L = 0.f;
        for (int s = 0; s < p.ksplit; ++s) {
            const size_t row = pidx(p, b, wi, s, tq);
            const float w = __expf(part.m[row] - M);
            s_w[s][t] = w;
            L += w * part.l[row];
        }
        const float inv = 1.0f / L;
        for (int s = 0; s < p.ksplit; ++s) s_w[s][t] *= inv;
    }
    __syncthreads();
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = 0; s < p.ksplit; ++s) {
        const float4 v = reinterpret_cast<const float4*>(part.o + lane_tile_base(p, b, wi, s, qblk, 0))[idx];
        const float w = s_w[s][c];
        acc.x += w * v.x;
        acc.y += w * v.y;
        acc.z += w * v.z;
        acc.w += w * v.w;
    }
    const int qpix = win_pixel(p, wi, qblk * 128 + wid * 32 + c);
    store4(out + ((size_t)b * HW + qpix) * kC + 32 * dt + 8 * u + 4 * h, acc);
}

// ============================================================================================
// 32x32x2 variant (window pixels % 128 == 0): one workgroup = 4 waves x 32 queries; every MFMA
// moves 32 FLOP per operand element (2x the 16x16x4 form) and has 64-cycle issue = dependent
// latency, so single accumulator chains run at rate. Operand maps (lane l, c = l & 31, h = l >> 5):
//   QK step i (0..63) contracts channels {i, 64 + i}: A = K[key c][64h + i] (LDS, K rows
//     XOR-swizzled by 16-B chunk), B = Q[query c][64h + i] (registers, pre-scaled);
//     S^T[key][q]: lane holds q = c, keys 8(r >> 2) + 4h + (r & 3) in register r.
//   PV step r contracts keys {8(r >> 2) + (r & 3) + 4h'}: B = the S^T register r itself,
//     A = V^T[d][that key] read as one ds_read_b128 per 4 steps from a transposed V tile.
// ============================================================================================
constexpr int kQW = 32;              // queries per wave
constexpr int kBQ3 = 4 * kQW;        // queries per workgroup
constexpr int kVtStride = kBK + 4;   // transposed V row (floats)

typedef float floatx16 __attribute__((ext_vector_type(16)));

// Staging is the T14 split of the key-pair kernel below: K(t+1) is loaded into registers during
// QK(t) and stored after the barrier that retires K(t); the same registers then carry V(t+1)
// during PV(t). Two barriers per tile, two workgroups per CU. (Round 4, measured slower and
// removed: Q and K by LDS-DMA in whole-row pieces with per-key offset tables, 60.4 vs 57.7 us at
// b = 2 -- the per-lane row gathers are not what bounds the prologue; profiles/r4/g25.)
__global__ void __launch_bounds__(kThreads, 2)
win_attn_f32x32_kernel(Params p, const float* __restrict__ q, const float* __restrict__ k,
                       const float* __restrict__ v, float* __restrict__ out, Partials part) {
    __shared__ __attribute__((aligned(16))) float sK[kBK * kC];
    __shared__ __attribute__((aligned(16))) float sVt[kC * kVtStride];
    __shared__ __attribute__((aligned(16))) int sKeyRegion[kBK];

    WA_STAMP(0, wall_clock64());
    WA_STAMP(1, WA_HWID());
    WA_STAMP(2, WA_CLOCK());
    int qblk, wi, bz;
    xcd_block_coords(qblk, wi, bz);
    const int b = bz / p.ksplit, ks = bz - b * p.ksplit;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int c = lane & 31, h = lane >> 5;
    const size_t HW = (size_t)p.H * p.W;
    const float* qb = q + (size_t)b * HW * kC;
    const int bkv = p.kv_shift ? (b + p.kv_shift) % p.nbatch : b;
    const float* kb = k + (size_t)bkv * p.m * HW * kC;
    const float* vb = v + (size_t)bkv * p.m * HW * kC;

    // staging: thread = (key row tid & 63, 32-channel quarter tid >> 6)
    const int grow = tid & 63, gpart = tid >> 6;
    const int kbeg = ks * p.keys_per_split, kend = kbeg + p.keys_per_split;
    float4 stg[8];
    int stg_region = 0;
    size_t stg_off = 0;
    auto load_k = [&](int k0) {
        key_row(p, wi, HW, k0 + grow, stg_off, stg_region);
        const float4* src = reinterpret_cast<const float4*>(kb + stg_off * kC + 32 * gpart);
#pragma unroll
        for (int i = 0; i < 8; ++i) stg[i] = src[i];
    };
    auto load_v = [&]() {
        const float4* src = reinterpret_cast<const float4*>(vb + stg_off * kC + 32 * gpart);
#pragma unroll
        for (int i = 0; i < 8; ++i) stg[i] = src[i];
    };
    auto store_k = [&]() {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int chunk = 8 * gpart + i;
            *reinterpret_cast<float4*>(&sK[grow * kC + ((chunk ^ (grow & 15)) * 4)]) = stg[i];
        }
        if (gpart == 0 && p.shift) sKeyRegion[grow] = stg_region;
    };
    auto store_v = [&]() {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int chunk = 8 * gpart + i;
            sVt[(4 * chunk + 0) * kVtStride + grow] = stg[i].x;
            sVt[(4 * chunk + 1) * kVtStride + grow] = stg[i].y;
            sVt[(4 * chunk + 2) * kVtStride + grow] = stg[i].z;
            sVt[(4 * chunk + 3) * kVtStride + grow] = stg[i].w;
        }
    };

    const int tq = qblk * kBQ3 + wid * kQW + c;
    const int qpix = win_pixel(p, wi, tq);
    const int qreg = p.shift ? win_region(p, wi, tq) : 0;
    // log2-domain scores (see the key-pair kernel)
    const float qscale = p.scale * kLog2e;
    float qr[64];
    auto load_q = [&]() {
        const float4* src = reinterpret_cast<const float4*>(qb + (size_t)qpix * kC + 64 * h);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float4 t4 = src[i];
            qr[4 * i] = t4.x * qscale;
            qr[4 * i + 1] = t4.y * qscale;
            qr[4 * i + 2] = t4.z * qscale;
            qr[4 * i + 3] = t4.w * qscale;
        }
    };
    floatx16 o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;

    {
        // prologue: tile 0's K and V rows are in flight together with Q (one exposed round trip)
        load_k(kbeg);
        float4 vrow[8];
        const float4* vsrc = reinterpret_cast<const float4*>(vb + stg_off * kC + 32 * gpart);
#pragma unroll
        for (int i = 0; i < 8; ++i) vrow[i] = vsrc[i];
        load_q();
        store_k();
#pragma unroll
        for (int i = 0; i < 8; ++i) stg[i] = vrow[i];
        store_v();
    }
    __syncthreads();
    WA_STAMP(3, WA_CLOCK());
    for (int k0 = kbeg; k0 < kend; k0 += kBK) {
        const bool has_next = k0 + kBK < kend;
        if (has_next) load_k(k0 + kBK);

        // ---- S^T = K Q^T, the two 32-key subtiles one after the other (a single 32x32x2 chain
        // runs at rate); the next K chunk is read from LDS before the current chunk's MFMAs
        floatx16 s[2];
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[sub][r] = 0.f;
            const int row = 32 * sub + c;
            auto kread = [&](int i4) {
                return *reinterpret_cast<const float4*>(&sK[row * kC + (((16 * h + i4) ^ (row & 15)) * 4)]);
            };
            float4 ka = kread(0);
#pragma unroll
            for (int i4 = 0; i4 < 16; ++i4) {
                const float4 nk = i4 + 1 < 16 ? kread(i4 + 1) : ka;
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x2f32(ka.x, qr[4 * i4 + 0], s[sub], 0, 0, 0);
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x2f32(ka.y, qr[4 * i4 + 1], s[sub], 0, 0, 0);
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x2f32(ka.z, qr[4 * i4 + 2], s[sub], 0, 0, 0);
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x2f32(ka.w, qr[4 * i4 + 3], s[sub], 0, 0, 0);
                ka = nk;
            }
        }
        // ---- mask + online softmax (lane = query c; its keys 32 sub + 8(r >> 2) + 4h + (r & 3))
        if (p.shift) {
            // region ids of the lane's 4-key runs as int4 LDS reads, branch-free select
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int4 rg = *reinterpret_cast<const int4*>(&sKeyRegion[32 * sub + 8 * u + 4 * h]);
                    s[sub][4 * u + 0] += rg.x == qreg ? 0.0f : kMaskLog2;
                    s[sub][4 * u + 1] += rg.y == qreg ? 0.0f : kMaskLog2;
                    s[sub][4 * u + 2] += rg.z == qreg ? 0.0f : kMaskLog2;
                    s[sub][4 * u + 3] += rg.w == qreg ? 0.0f : kMaskLog2;
                }
        }
        // row max as a v_max3 tree (16 instructions for 32 scores)
        float bmax = max3_raw(s[0][0], s[1][0], s[0][1]);
        bmax = max3_raw(bmax, s[1][1], s[0][2]);
#pragma unroll
        for (int r = 2; r < 15; ++r) bmax = max3_raw(bmax, s[1][r], s[0][r + 1]);
        bmax = fmaxf(bmax, s[1][15]);
        bmax = halves_max(bmax);
        const float m_new = fmaxf(m_run, bmax);
        if (__any(m_new > m_run)) {  // exact: corr == 1 for every lane otherwise
            const float corr = fast_exp2(m_run - m_new);
            l_run *= corr;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) o[dt] *= corr;
            m_run = m_new;
        }
        // s - m and the row sum on packed pairs (v_pk_add_f32: half the issue slots)
        typedef float f2v __attribute__((ext_vector_type(2)));
        const f2v nm2 = {-m_run, -m_run};
        f2v bsum2 = {0.f, 0.f};
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
                const f2v arg = (f2v){s[sub][r], s[sub][r + 1]} + nm2;
                const f2v e = {fast_exp2(arg.x), fast_exp2(arg.y)};
                s[sub][r] = e.x;
                s[sub][r + 1] = e.y;
                bsum2 += e;
            }
        l_run += halves_sum(bsum2.x + bsum2.y);

        __syncthreads();  // every wave is done with K(t) / regions(t)
        if (has_next) {
            store_k();
            load_v();
        }

        // ---- O^T += V^T P^T: per 4-key run, the four d tiles' chains interleaved
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int dp = 0; dp < 4; dp += 2) {
                    const float4 v0 = *reinterpret_cast<const float4*>(&sVt[(32 * dp + c) * kVtStride + 32 * sub + 8 * u + 4 * h]);
                    const float4 v1 = *reinterpret_cast<const float4*>(&sVt[(32 * dp + 32 + c) * kVtStride + 32 * sub + 8 * u + 4 * h]);
                    o[dp] = __builtin_amdgcn_mfma_f32_32x32x2f32(v0.x, s[sub][4 * u + 0], o[dp], 0, 0, 0);
                    o[dp + 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(v1.x, s[sub][4 * u + 0], o[dp + 1], 0, 0, 0);
                    o[dp] = __builtin_amdgcn_mfma_f32_32x32x2f32(v0.y, s[sub][4 * u + 1], o[dp], 0, 0, 0);
                    o[dp + 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(v1.y, s[sub][4 * u + 1], o[dp + 1], 0, 0, 0);
                    o[dp] = __builtin_amdgcn_mfma_f32_32x32x2f32(v0.z, s[sub][4 * u + 2], o[dp], 0, 0, 0);
                    o[dp + 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(v1.z, s[sub][4 * u + 2], o[dp + 1], 0, 0, 0);
                    o[dp] = __builtin_amdgcn_mfma_f32_32x32x2f32(v0.w, s[sub][4 * u + 3], o[dp], 0, 0, 0);
                    o[dp + 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(v1.w, s[sub][4 * u + 3], o[dp + 1], 0, 0, 0);
                }
        __syncthreads();  // every wave is done with V(t); K(t+1) is visible
        if (has_next) store_v();  // read after the next tile's first barrier
        if ((k0 - kbeg) / kBK < 8) WA_STAMP(4 + (k0 - kbeg) / kBK, WA_CLOCK());
    }

    // O^T[d = 32 dt + 8u + 4h + j][q = c] in o[dt][4u + j]
    if (p.ksplit == 1) {
        const float inv = 1.0f / l_run;
        float* dst = out + ((size_t)b * HW + qpix) * kC + 4 * h;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int u = 0; u < 4; ++u)
                *reinterpret_cast<float4*>(dst + 32 * dt + 8 * u) =
                    make_float4(o[dt][4 * u] * inv, o[dt][4 * u + 1] * inv, o[dt][4 * u + 2] * inv,
                                o[dt][4 * u + 3] * inv);
    } else {
        // lane-contiguous partial tile: each store instruction writes one 1-KB run
        const size_t row = pidx(p, b, wi, ks, tq);
        float4* dst = reinterpret_cast<float4*>(part.o + lane_tile_base(p, b, wi, ks, qblk, wid)) + lane;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int u = 0; u < 4; ++u)
                dst[(dt * 4 + u) * 64] = make_float4(o[dt][4 * u], o[dt][4 * u + 1], o[dt][4 * u + 2], o[dt][4 * u + 3]);
        if (h == 0) {
            part.m[row] = m_run * kLn2;  // natural-log domain for the combine
            part.l[row] = l_run;
        }
    }
    WA_STAMP(12, WA_CLOCK());
    WA_STAMP(13, wall_clock64());
}


// ============================================================================================
// bf16 operand types (the v2 / v3 kernels below)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
constexpr int kVtStrideH = kBK + 8;  // transposed V row (bf16 elements)

// ============================================================================================
// bf16 v2 (bf16 launches that need a key split): the round-1 bf16 kernel's operand maps, re-cut for the
// VALU budget beside 2.5 PF of matrix cores (one 32x32x16 MFMA = 32 cycles, of which 24 are free
// for vector issue):
//   * K / V / mask tiles double-buffered in LDS, one barrier per key tile (the next tile's rows,
//     loaded during this tile, are written to the other buffer after this tile's MFMAs);
//   * V stays row-major in LDS (16-B writes, the XOR image (b) of cdna_hip_programming.md T10) and
//     the PV A operand V^T[d][keys] comes from ds_read_b64_tr_b16: two transposed reads per
//     fragment instead of 16 two-byte transposing writes + shuffles per staged row;
//   * softmax in the log2 domain on the raw scores: one max3 tree, then exp2(fma(s, c, -m)) with
//     c = log2(e) / sqrt(C) -- no separate scale, subtract and log2(e) multiplies;
//   * deferred rescale (T13): the running max m moves only when a tile's max exceeds it by more
//     than kThr (log2 units), a wave-uniform branch, so P <= 2^kThr in bf16 (same relative
//     precision) and the 64-register O rescale and l update are skipped on almost every tile;
//   * the shifted-window mask rides on the QK^T MFMA: one extra k = 16 step per 32-key subtile
//     with A = kMaskBonus at the key's region slot (one-hot, from LDS) and B = 1 at the query's
//     region slot (registers), which adds kMaskBonus to every same-region score. Softmax is
//     invariant to a per-query shift, so this equals the reference's -100 on different-region
//     pairs up to the bonus's bf16 rounding: different-region weights are e^(-99.7) instead of
//     e^(-100) relative -- both below fp32's normal range, i.e. zero for the output.
// ============================================================================================
constexpr float kThr = 8.0f;             // deferred-rescale threshold (log2 units): P <= 256
constexpr float kMaskBonus = 1128.0f;    // bf16-exact; x 1/sqrt(128) = 99.7 (reference: 100)

// byte offset of 16-B chunk ch (0..15) of row r in a [rows][128 x bf16] tile, image (b) of T10:
// conflict-free for ds_read_b128 row reads and ds_read_b64_tr_b16 transposed reads alike
__device__ __forceinline__ int vimg_off(int r, int ch) {
    return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3)));
}

typedef short shortx4 __attribute__((ext_vector_type(4)));


__global__ void __launch_bounds__(kThreads, 2)
win_attn_bf16_v2_kernel(Params p, const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                        const __bf16* __restrict__ v, __bf16* __restrict__ out, Partials part) {
    // double-buffered K / V / mask tiles: one barrier per key tile
    __shared__ __attribute__((aligned(16))) __bf16 sKb[2][kBK * kC];
    __shared__ __attribute__((aligned(16))) unsigned char sVb[2][kBK * kC * 2];
    __shared__ __attribute__((aligned(16))) bf16x8 sMaskAb[2][kBK][2];  // one-hot key-region fragments

    int qblk, wi, bz;
    xcd_block_coords(qblk, wi, bz);
    const int b = bz / p.ksplit, ks = bz - b * p.ksplit;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int c = lane & 31, h = lane >> 5;
    const size_t HW = (size_t)p.H * p.W;
    const int kvb = (b + p.kv_shift) % p.nbatch;
    const __bf16* qb = q + (size_t)b * HW * kC;
    const __bf16* kb = k + (size_t)kvb * p.m * HW * kC;
    const __bf16* vb = v + (size_t)kvb * p.m * HW * kC;
    const float cl2 = p.scale * kLog2e;

    const int tq = qblk * kBQ3 + wid * kQW + c;
    const int qpix = win_pixel(p, wi, tq);
    bf16x8 qf[8];
    {
        const bf16x8* src = reinterpret_cast<const bf16x8*>(qb + (size_t)qpix * kC + 8 * h);
#pragma unroll
        for (int i = 0; i < 8; ++i) qf[i] = src[2 * i];
    }
    // mask B operand: B[k = 8h + j][query c] = 1 at the query's region slot
    bf16x8 qmask;
    {
        const int qreg = p.shift ? win_region(p, wi, tq) : 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) qmask[j] = (__bf16)(qreg == 8 * h + j ? 1.0f : 0.0f);
    }
    floatx16 o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;

    // gather: thread = (key row grow, 32-channel quarter gpart); the next tile's rows are loaded
    // into registers right after this tile's barrier and written to LDS after the end-of-tile
    // barrier (issue early / write late)
    const int grow = tid & 63, gpart = tid >> 6;
    const int kbeg = ks * p.keys_per_split, kend = kbeg + p.keys_per_split;
    bf16x8 kv[4], vv[4];
    int kreg = 0;
    auto gather = [&](int k0) {
        const int j = k0 + grow;
        const int tk = j / p.m, vi = j - tk * p.m;
        const int kpix = win_pixel(p, wi, tk);
        const bf16x8* ksrc = reinterpret_cast<const bf16x8*>(kb + ((size_t)vi * HW + kpix) * kC + 32 * gpart);
        const bf16x8* vsrc = reinterpret_cast<const bf16x8*>(vb + ((size_t)vi * HW + kpix) * kC + 32 * gpart);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            kv[i] = ksrc[i];
            vv[i] = vsrc[i];
        }
        kreg = p.shift ? win_region(p, wi, j % p.L) : 0;
    };
    auto stage = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int chunk = 4 * gpart + i;
            *reinterpret_cast<bf16x8*>(&sKb[buf][grow * kC + ((chunk ^ (grow & 15)) * 8)]) = kv[i];
            *reinterpret_cast<bf16x8*>(&sVb[buf][vimg_off(grow, chunk)]) = vv[i];
        }
        if (p.shift && gpart < 2) {
            bf16x8 a;
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = (__bf16)(kreg == 8 * gpart + j ? kMaskBonus : 0.0f);
            sMaskAb[buf][grow][gpart] = a;
        }
    };
    gather(kbeg);
    stage(0);
    __syncthreads();
    if (kbeg + kBK < kend) gather(kbeg + kBK);
    for (int k0 = kbeg, buf = 0; k0 < kend; k0 += kBK, buf ^= 1) {
        const __bf16* sK = sKb[buf];
        const unsigned char* sV = sVb[buf];
        const bf16x8(*sMaskA)[2] = sMaskAb[buf];

        // ---- S^T = K Q^T (+ the mask step), raw scores
        floatx16 s[2];
#pragma unroll
        for (int r = 0; r < 16; ++r) s[0][r] = s[1][r] = 0.f;
        {
            bf16x8 kk[2][8];
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int row = 32 * sub + c, chunk = 2 * i + h;
                    kk[sub][i] = *reinterpret_cast<const bf16x8*>(&sK[row * kC + ((chunk ^ (row & 15)) * 8)]);
                }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (kAbl2 == 3) {
                    s[0][i] += (float)kk[0][i][0];
                    s[1][i] += (float)kk[1][i][0];
                    continue;
                }
                s[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kk[0][i], qf[i], s[0], 0, 0, 0);
                s[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kk[1][i], qf[i], s[1], 0, 0, 0);
            }
            if (p.shift) {
                s[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sMaskA[c][h], qmask, s[0], 0, 0, 0);
                s[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sMaskA[32 + c][h], qmask, s[1], 0, 0, 0);
            }
        }
        // ---- online softmax (fp32, log2 domain), deferred rescale
        if (kAbl2 != 1) {
        float bmax = max3_raw(s[0][0], s[1][0], s[0][1]);
        bmax = max3_raw(bmax, s[1][1], s[0][2]);
#pragma unroll
        for (int r = 2; r < 15; ++r) bmax = max3_raw(bmax, s[1][r], s[0][r + 1]);
        bmax = fmaxf(bmax, s[1][15]);
        const float bm2 = halves_max(bmax) * cl2;
        if (__any(bm2 > m_run + kThr)) {
            const float m_new = fmaxf(m_run, bm2);
            const float corr = fast_exp2(m_run - m_new);
            l_run *= corr;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) o[dt] *= corr;
            m_run = m_new;
        }
        float bsum = 0.f;
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float e = fast_exp2(fmaf(s[sub][r], cl2, -m_run));
                s[sub][r] = e;
                bsum += e;
            }
        l_run += halves_sum(bsum);
        }

        // ---- O^T += V^T P^T: 4 k-steps of 16 keys; A = V^T by transposed LDS reads
#pragma unroll
        for (int ksx = 0; ksx < 4; ++ksx) {
            const int sub = ksx >> 1, st = ksx & 1;
            bf16x8 pf;
#pragma unroll
            for (int e = 0; e < 8; ++e) pf[e] = (__bf16)s[sub][8 * st + e];
            // group g = lane >> 4 reads the 4-key x 16-d block rows r0.., cols 32 dt + 16 (g & 1);
            // lane 4qq + pp of the group supplies row r0 + qq, chunk c0 + (pp >> 1), half pp & 1
            const int gi = lane & 15, qq = gi >> 2, pp = gi & 3;
            const int r0 = 16 * ksx + 4 * h + qq;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const int c0 = 4 * dt + 2 * ((lane >> 4) & 1) + (pp >> 1);
                const shortx4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (__attribute__((address_space(3))) shortx4*)(sV + vimg_off(r0, c0) + 8 * (pp & 1)));
                const shortx4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (__attribute__((address_space(3))) shortx4*)(sV + vimg_off(r0 + 8, c0) + 8 * (pp & 1)));
                typedef short shortx8 __attribute__((ext_vector_type(8)));
                const shortx8 vs = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                if (kAbl2 == 2) { o[dt][0] += (float)pf[0] + (float)vs[0]; continue; }
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, vs), pf, o[dt], 0, 0, 0);
            }
        }
        // write-late: the next tile's rows (loaded during this tile) go to the other buffer, whose
        // readers all passed the previous barrier; then the tile after that is requested
        if (k0 + kBK < kend && kAbl2 != 4) {
            stage(buf ^ 1);
            if (k0 + 2 * kBK < kend) gather(k0 + 2 * kBK);
        }
        __syncthreads();
    }

    // O^T[d = 32 dt + 8u + 4h + j][q = c] in o[dt][4u + j]
    if (p.ksplit == 1) {
        const float inv = 1.0f / l_run;
        __bf16* dst = out + ((size_t)b * HW + qpix) * kC + 4 * h;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int u = 0; u < 4; ++u)
                store4(dst + 32 * dt + 8 * u, make_float4(o[dt][4 * u] * inv, o[dt][4 * u + 1] * inv,
                                                          o[dt][4 * u + 2] * inv, o[dt][4 * u + 3] * inv));
    } else {
        const size_t row = pidx(p, b, wi, ks, tq);
        float4* dst = reinterpret_cast<float4*>(part.o + lane_tile_base(p, b, wi, ks, qblk, wid)) + lane;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int u = 0; u < 4; ++u)
                dst[(dt * 4 + u) * 64] = make_float4(o[dt][4 * u], o[dt][4 * u + 1], o[dt][4 * u + 2], o[dt][4 * u + 3]);
        if (h == 0) {
            part.m[row] = m_run * kLn2;  // the combine kernel takes natural-log maxima
            part.l[row] = l_run;
        }
    }
}

// ============================================================================================
// bf16 v3: 8 waves = two 4-wave groups (A: queries 0-127, B: 128-255 of a 256-query block) on the
// same K / V tiles, staggered by one phase so each SIMD pairs one group's MFMA phase with the other
// group's VALU phase (cdna_hip_programming.md / MI355X_MICROARCH.md "two waves per SIMD"):
//   group-local step s (A: s = i, B: s = i - 1 for global interval i, one s_barrier per interval)
//     s = 2t     (MFMA): O += V(t-1)^T P(t-1)^T (t >= 1), then S(t) = K(t) Q^T (+ mask step)
//     s = 2t + 1 (VALU): online softmax of S(t) -> P(t) (bf16), and staging: A writes its half of
//                        tile t + 1, B its half of tile t + 2, then each loads its next half.
// Tile u lives in LDS buffer u % 3 from its first write (interval 2u - 1 / 2u - 2) to its last
// read (B's PV at interval 2u + 3); three buffers keep every write after the previous occupant's
// last read (checked in the comments at the staging code). Operand maps, log2-domain softmax with
// deferred rescale and the mask step are those of win_attn_bf16_v2_kernel. ksplit == 1 only.
// ============================================================================================
constexpr int kThreads8 = 512;
constexpr int kBQ8 = 256;  // queries per workgroup
constexpr int kNBuf = 3;

__device__ __forceinline__ void lds_barrier() {
    // LDS writes complete, then the workgroup barrier; outstanding global loads (the prefetched
    // tile halves) stay in flight across it (a __syncthreads fence would drain them)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// LDS of v3: [K0 K1 K2][V0 V1 V2][M0 M1 M2]. K rows padded to 272 B and not swizzled: the QK^T
// operand reads (lane (c, h): row c, 16-B chunk 2i + h) then all sit at ONE per-lane address plus
// compile-time offsets, and a ds_read_b128 lane group's 16 rows land on 16 distinct 4-bank sets.
// V keeps image (b) (transposed tr16 reads), whose per-lane part takes 8 precomputed addresses.
// With the tile loop unrolled by three the ring-buffer offsets are immediates too.
constexpr int kKRowB = kC * 2 + 16;           // 272
constexpr int kKBufB = kBK * kKRowB;          // 17,408
constexpr int kVBufB = kBK * kC * 2;          // 16,384
constexpr int kMBufB = kBK * 2 * 16;          // 2,048 (one-hot mask fragments)
constexpr int kVOff = kNBuf * kKBufB;         // 52,224
constexpr int kMOff = kVOff + kNBuf * kVBufB; // 101,376
constexpr int kLds3 = kMOff + kNBuf * kMBufB; // 107,520

template <int N>
struct IC {
    static constexpr int value = N;
};

__global__ void __launch_bounds__(kThreads8, 1)
win_attn_bf16_v3_kernel(Params p, const __bf16* __restrict__ q, const __bf16* __restrict__ k,
                        const __bf16* __restrict__ v, __bf16* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[kLds3];
    WA_STAMP(0, wall_clock64());
    WA_STAMP(1, WA_HWID());
    WA_STAMP(2, WA_CLOCK());

    int qblk, wi, b;
    xcd_block_coords(qblk, wi, b);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wid >> 2, wq = wid & 3;
    const int c = lane & 31, h = lane >> 5;
    const size_t HW = (size_t)p.H * p.W;
    const int kvb = (b + p.kv_shift) % p.nbatch;
    const __bf16* qb = q + (size_t)b * HW * kC;
    const __bf16* kb = k + (size_t)kvb * p.m * HW * kC;
    const __bf16* vb = v + (size_t)kvb * p.m * HW * kC;
    const float cl2 = p.scale * kLog2e;

    const int tq = qblk * kBQ8 + grp * kBQ3 + wq * kQW + c;
    const int qpix = win_pixel(p, wi, tq);
    bf16x8 qf[8];
    {
        const bf16x8* src = reinterpret_cast<const bf16x8*>(qb + (size_t)qpix * kC + 8 * h);
#pragma unroll
        for (int i = 0; i < 8; ++i) qf[i] = src[2 * i];
    }
    bf16x8 qmask;
    {
        const int qreg = p.shift ? win_region(p, wi, tq) : 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) qmask[j] = (__bf16)(qreg == 8 * h + j ? 1.0f : 0.0f);
    }
    floatx16 o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;

    // per-lane LDS read addresses (byte offsets into smem), loop invariant
    const unsigned aK = c * kKRowB + h * 16;
    const unsigned aM = kMOff + c * 32 + h * 16;
    unsigned aV[2][4];  // [lo / hi key half][dt]: image (b) of keys 16 ksx + 4h + qq (+ 8)
    {
        const int gi = lane & 15, qq = gi >> 2, pp = gi & 3;
        const int x = 2 * ((lane >> 4) & 1) + (pp >> 1);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            aV[0][dt] = kVOff + 256 * (4 * h + qq) + 64 * (dt ^ qq) + 16 * (x ^ h) + 8 * (pp & 1);
            aV[1][dt] = kVOff + 256 * (4 * h + qq + 8) + 64 * (dt ^ qq) + 16 * (x ^ (h + 2)) + 8 * (pp & 1);
        }
    }

    // staging: a group moves its half of a tile: thread (key row grow, part gp) holds 16-B chunks
    // 8 grp + 2 gp + {0, 1} of the row's K and V (and, for gp == 0, the row's mask fragment grp).
    // (Round 6, measured slower and removed: whole 256-B rows per wave instruction -- K by two waves,
    // V by two, row offsets and mask regions shuffled -- 61.8 vs 51.1 us at B = 16 shifted, 51.5 vs
    // 49.0 unshifted; profiles/r6/wa_v3_rows.log)
    const int t8 = tid & 255, grow = t8 & 63, gp = t8 >> 6;
    const int ntiles = p.L * p.m / kBK;
    bf16x8 kv[2], vv[2];
    int kreg = 0;
    auto gather = [&](int tile) {
        const int j = tile * kBK + grow;
        int tk = j, vi = 0;
        if (p.m != 1) {  // (single key view: no division)
            tk = j / p.m;
            vi = j - tk * p.m;
        }
        const int kpix = win_pixel(p, wi, tk);
        const int ch0 = 8 * grp + 2 * gp;
        const bf16x8* ksrc = reinterpret_cast<const bf16x8*>(kb + ((size_t)vi * HW + kpix) * kC) + ch0;
        const bf16x8* vsrc = reinterpret_cast<const bf16x8*>(vb + ((size_t)vi * HW + kpix) * kC) + ch0;
        kv[0] = ksrc[0];
        kv[1] = ksrc[1];
        vv[0] = vsrc[0];
        vv[1] = vsrc[1];
        if (p.shift) kreg = win_region(p, wi, p.m == 1 ? j : j % p.L);
    };
    auto stage = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int chunk = 8 * grp + 2 * gp + i;
            *reinterpret_cast<bf16x8*>(smem + buf * kKBufB + grow * kKRowB + chunk * 16) = kv[i];
            *reinterpret_cast<bf16x8*>(smem + kVOff + buf * kVBufB + vimg_off(grow, chunk)) = vv[i];
        }
        if (p.shift && gp == 0) {
            bf16x8 a;
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = (__bf16)(kreg == 8 * grp + j ? kMaskBonus : 0.0f);
            *reinterpret_cast<bf16x8*>(smem + kMOff + buf * kMBufB + grow * 32 + grp * 16) = a;
        }
    };
    // prologue: tile 0 (both halves) and tile 1's B half in LDS; registers: A holds tile 1's half
    // (written in A's first VALU interval), B tile 2's (written in B's)
    gather(0);
    stage(0);
    if (grp == 1 && ntiles > 1) {
        gather(1);
        stage(1);
    }
    if (grp == 0 ? ntiles > 1 : ntiles > 2) gather(grp == 0 ? 1 : 2);
    lds_barrier();
    WA_STAMP(3, WA_CLOCK());
    // group B runs one interval behind A: one barrier before its loop (A: one after), so every
    // wave passes 2 (ntiles + 1) + 1 barriers
    if (grp == 1) lds_barrier();

    bf16x8 pf[4];
    // tile t (t % 3 == BUF); returns true after the final (PV-only) MFMA interval
    auto iter = [&](int t, auto bufc) -> bool {
        constexpr int BUF = decltype(bufc)::value;
        constexpr int PBUF = (BUF + 2) % 3;  // tile t - 1
        // ======== MFMA interval: O += V(t-1)^T P(t-1)^T, then S(t) = K(t) Q^T (+ mask step)
        if (t >= 1) {
#pragma unroll
            for (int ksx = 0; ksx < 4; ++ksx)
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) {
                    const int off = PBUF * kVBufB + 4096 * ksx;
                    const shortx4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (__attribute__((address_space(3))) shortx4*)(smem + aV[0][dt] + off));
                    const shortx4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (__attribute__((address_space(3))) shortx4*)(smem + aV[1][dt] + off));
                    typedef short shortx8 __attribute__((ext_vector_type(8)));
                    const shortx8 vs = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, vs), pf[ksx], o[dt], 0,
                                                                    0, 0);
                }
        }
        floatx16 sacc[2];
        if (t < ntiles) {
#pragma unroll
            for (int sub = 0; sub < 2; ++sub) {
                bf16x8 kk[8];
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    kk[i] = *reinterpret_cast<const bf16x8*>(smem + aK + BUF * kKBufB + sub * 32 * kKRowB + 32 * i);
                const floatx16 zero = {};
                sacc[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kk[0], qf[0], zero, 0, 0, 0);
#pragma unroll
                for (int i = 1; i < 8; ++i)
                    sacc[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kk[i], qf[i], sacc[sub], 0, 0, 0);
                if (p.shift)
                    sacc[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        *reinterpret_cast<const bf16x8*>(smem + aM + BUF * kMBufB + sub * 1024), qmask, sacc[sub], 0,
                        0, 0);
            }
        }
        lds_barrier();
        if (t < 8) WA_STAMP(4 + t, WA_CLOCK());
        if (t == ntiles) return true;
        // ======== VALU interval: staging, then the online softmax of S(t) -> P(t)
        // A writes tile t + 1 into buffer (t + 1) % 3, whose previous tile t - 2 was last read by
        // B's PV one interval earlier; B writes tile t + 2 into (t + 2) % 3, last read (tile t - 1)
        // by B's own PV in its previous interval. Both halves of tile u are in place before A's
        // QK(u).
        {
            const int wtile = t + 1 + grp;
            if (wtile < ntiles) {
                stage(grp == 0 ? (BUF + 1) % 3 : (BUF + 2) % 3);
                if (wtile + 1 < ntiles) gather(wtile + 1);
            }
        }
        float bmax = max3_raw(sacc[0][0], sacc[1][0], sacc[0][1]);
        bmax = max3_raw(bmax, sacc[1][1], sacc[0][2]);
#pragma unroll
        for (int r = 2; r < 15; ++r) bmax = max3_raw(bmax, sacc[1][r], sacc[0][r + 1]);
        bmax = fmaxf(bmax, sacc[1][15]);
        const float bm2 = halves_max(bmax) * cl2;
        if (__any(bm2 > m_run + kThr)) {
            const float m_new = fmaxf(m_run, bm2);
            const float corr = fast_exp2(m_run - m_new);
            l_run *= corr;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) o[dt] *= corr;
            m_run = m_new;
        }
        // scalar fma per score: the packed v_pk_fma / v_pk_add form measured 1.5 us slower at B = 16
        // (same box, profiles/r4/g22: 53.9 / 54.3 vs 52.2 / 52.9 us)
        float bsum = 0.f;
#pragma unroll
        for (int ksx = 0; ksx < 4; ++ksx)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float ex = fast_exp2(fmaf(sacc[ksx >> 1][8 * (ksx & 1) + e], cl2, -m_run));
                bsum += ex;
                pf[ksx][e] = (__bf16)ex;
            }
        l_run += halves_sum(bsum);
        lds_barrier();
        return false;
    };
    for (int t = 0;; t += 3) {
        if (iter(t, IC<0>{})) break;
        if (iter(t + 1, IC<1>{})) break;
        if (iter(t + 2, IC<2>{})) break;
    }
    if (grp == 0) lds_barrier();

    // O^T[d = 32 dt + 8u + 4h + j][q = c] in o[dt][4u + j]
    const float inv = 1.0f / l_run;
    __bf16* dst = out + ((size_t)b * HW + qpix) * kC + 4 * h;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int u = 0; u < 4; ++u)
            store4(dst + 32 * dt + 8 * u, make_float4(o[dt][4 * u] * inv, o[dt][4 * u + 1] * inv,
                                                      o[dt][4 * u + 2] * inv, o[dt][4 * u + 3] * inv));
    WA_STAMP(12, WA_CLOCK());
    WA_STAMP(13, wall_clock64());
}

// ============================================================================================
// bf16x3 ("split-bf16") form of the exact-fp32 128-query kernel: the C2 step's dense-precision
// mode (the reference runs both contractions as TF32 matmuls, src/main.py:15; gfx950 has no xf32
// MFMA). Every fp32 operand is x = xh + xl (xh = bf16(x), xl = bf16(x - xh)), every product
// xh yh + xh yl + xl yh on v_mfma_f32_32x32x16_bf16 with fp32 accumulation: <= ~3 * 2^-18 relative
// per product (TF32: 2^-11 per operand), at 3 / 16 of the exact-fp32 MFMA cycles.
//   * Q (fp32) is split in registers once per lane; K and V arrive pre-split (tsplat_split_kv_bf16x3:
//     every K / V row is staged by L / 128 query blocks, so splitting at staging would repeat it)
//     and are staged as hi / lo LDS images -- K row-major XOR-swizzled, V in the T10 image (b) read
//     transposed by ds_read_b64_tr_b16 (win_attn_bf16_v2_kernel's operand maps);
//   * softmax: raw fp32 scores, log2 domain, deferred rescale (P <= 2^kThr, split exactly as well);
//   * the shifted-window mask as the v2 kernel's extra MFMA step on the hi part (+kMaskBonus to
//     same-region scores: different-region weights e^-99.7 instead of e^-100, both 0 to fp32 output);
//   * K / V / mask tiles double-buffered, one barrier per tile; one workgroup per CU (132 KB LDS).
// Writes the same split-key partials (lane-contiguous O, natural-log m, l) as the exact kernel, so
// tsplat_linear_f32_attn_merge_fwd combines them in its operand staging unchanged.
// ============================================================================================
__device__ __forceinline__ void split8(const float (&x)[8], bf16x8& hi, bf16x8& lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        hi[j] = (__bf16)x[j];
        lo[j] = (__bf16)(x[j] - (float)hi[j]);
    }
}

__global__ void __launch_bounds__(kThreads, 1)
win_attn_x3_kernel(Params p, const float* __restrict__ q, const __bf16* __restrict__ khg,
                   const __bf16* __restrict__ klg, const __bf16* __restrict__ vhg, const __bf16* __restrict__ vlg,
                   float* __restrict__ out, Partials part) {
    __shared__ __attribute__((aligned(16))) __bf16 sKh[2][kBK * kC];
    __shared__ __attribute__((aligned(16))) __bf16 sKl[2][kBK * kC];
    __shared__ __attribute__((aligned(16))) unsigned char sVh[2][kBK * kC * 2];
    __shared__ __attribute__((aligned(16))) unsigned char sVl[2][kBK * kC * 2];
    __shared__ __attribute__((aligned(16))) bf16x8 sMaskAb[2][kBK][2];

    WA_STAMP(0, wall_clock64());
    WA_STAMP(1, WA_HWID());
    WA_STAMP(2, WA_CLOCK());
    // (tried: all key splits of a (batch, window) on one XCD, so Q is fetched into one L2 once --
    // prologue 10.2k vs 10.4k cycles, C2 unchanged, profiles/r5/x3/: the prologue is bound by the
    // chip-wide L2 -> CU ingest rate of a 256-CU burst, not by HBM bytes)
    int qblk, wi, bz;
    xcd_block_coords(qblk, wi, bz);
    const int b = bz / p.ksplit, ks = bz - b * p.ksplit;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int c = lane & 31, h = lane >> 5;
    const size_t HW = (size_t)p.H * p.W;
    const int kvb = (b + p.kv_shift) % p.nbatch;
    const size_t kvoff = (size_t)kvb * p.m * HW * kC;
    const float cl2 = p.scale * kLog2e;

    const int tq = qblk * kBQ3 + wid * kQW + c;
    const int qpix = win_pixel(p, wi, tq);
    bf16x8 qh[8], ql[8];
    bf16x8 qmask;
    {
        const int qreg = p.shift ? win_region(p, wi, tq) : 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) qmask[j] = (__bf16)(qreg == 8 * h + j ? 1.0f : 0.0f);
    }
    floatx16 o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;

    // gather: thread = (key row grow, 32-channel quarter gpart), hi and lo rows of K and V
    const int grow = tid & 63, gpart = tid >> 6;
    const int kbeg = ks * p.keys_per_split, kend = kbeg + p.keys_per_split;
    bf16x8 kvh[4], kvl[4], vvh[4], vvl[4];
    int kreg = 0;
    auto gather = [&](int k0) {
        const int j = k0 + grow;
        const int tk = j / p.m, vi = j - tk * p.m;
        const int kpix = win_pixel(p, wi, tk);
        const size_t off = kvoff + ((size_t)vi * HW + kpix) * kC + 32 * gpart;
        const bf16x8* a = reinterpret_cast<const bf16x8*>(khg + off);
        const bf16x8* bl = reinterpret_cast<const bf16x8*>(klg + off);
        const bf16x8* cv = reinterpret_cast<const bf16x8*>(vhg + off);
        const bf16x8* dv = reinterpret_cast<const bf16x8*>(vlg + off);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            kvh[i] = a[i];
            kvl[i] = bl[i];
            vvh[i] = cv[i];
            vvl[i] = dv[i];
        }
        kreg = p.shift ? win_region(p, wi, j % p.L) : 0;
    };
    auto stage = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int chunk = 4 * gpart + i;
            const int ko = grow * kC + ((chunk ^ (grow & 15)) * 8);
            *reinterpret_cast<bf16x8*>(&sKh[buf][ko]) = kvh[i];
            *reinterpret_cast<bf16x8*>(&sKl[buf][ko]) = kvl[i];
            *reinterpret_cast<bf16x8*>(&sVh[buf][vimg_off(grow, chunk)]) = vvh[i];
            *reinterpret_cast<bf16x8*>(&sVl[buf][vimg_off(grow, chunk)]) = vvl[i];
        }
        if (p.shift && gpart < 2) {
            bf16x8 a;
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = (__bf16)(kreg == 8 * gpart + j ? kMaskBonus : 0.0f);
            sMaskAb[buf][grow][gpart] = a;
        }
    };
    // prologue: the first tile's K / V loads go out before Q's, so stage(0) waits only for them;
    // Q[query c][16 i + 8 h .. + 7] is split into hi / lo (the B operand of k-step i) after it
    gather(kbeg);
    float4 qraw[16];
    {
        const float4* src = reinterpret_cast<const float4*>(q + ((size_t)b * HW + qpix) * kC + 8 * h);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            qraw[2 * i] = src[4 * i];
            qraw[2 * i + 1] = src[4 * i + 1];
        }
    }
    stage(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float4 a0 = qraw[2 * i], a1 = qraw[2 * i + 1];
        const float x[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        split8(x, qh[i], ql[i]);
    }
    __syncthreads();
    WA_STAMP(3, WA_CLOCK());
    if (kbeg + kBK < kend) gather(kbeg + kBK);
    for (int k0 = kbeg, buf = 0; k0 < kend; k0 += kBK, buf ^= 1) {
        // ---- S^T = K Q^T (+ the mask step): per 16-channel k-step kl qh + kh ql + kh qh
        floatx16 s[2];
#pragma unroll
        for (int r = 0; r < 16; ++r) s[0][r] = s[1][r] = 0.f;
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            const int row = 32 * sub + c;
            bf16x8 kh8[8], kl8[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int ko = row * kC + (((2 * i + h) ^ (row & 15)) * 8);
                kh8[i] = *reinterpret_cast<const bf16x8*>(&sKh[buf][ko]);
                kl8[i] = *reinterpret_cast<const bf16x8*>(&sKl[buf][ko]);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl8[i], qh[i], s[sub], 0, 0, 0);
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh8[i], ql[i], s[sub], 0, 0, 0);
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh8[i], qh[i], s[sub], 0, 0, 0);
            }
            if (p.shift)
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sMaskAb[buf][row][h], qmask, s[sub], 0, 0, 0);
        }
        // ---- online softmax (fp32, log2 domain), deferred rescale
        float bmax = max3_raw(s[0][0], s[1][0], s[0][1]);
        bmax = max3_raw(bmax, s[1][1], s[0][2]);
#pragma unroll
        for (int r = 2; r < 15; ++r) bmax = max3_raw(bmax, s[1][r], s[0][r + 1]);
        bmax = fmaxf(bmax, s[1][15]);
        const float bm2 = halves_max(bmax) * cl2;
        if (__any(bm2 > m_run + kThr)) {
            const float m_new = fmaxf(m_run, bm2);
            const float corr = fast_exp2(m_run - m_new);
            l_run *= corr;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) o[dt] *= corr;
            m_run = m_new;
        }
        float bsum = 0.f;
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float e = fast_exp2(fmaf(s[sub][r], cl2, -m_run));
                s[sub][r] = e;
                bsum += e;
            }
        l_run += halves_sum(bsum);

        // ---- O^T += V^T P^T: 4 k-steps of 16 keys, per d tile vl ph + vh pl + vh ph
        const int gi = lane & 15, qq = gi >> 2, pp = gi & 3;
#pragma unroll
        for (int ksx = 0; ksx < 4; ++ksx) {
            const int sub = ksx >> 1, st = ksx & 1;
            float pv[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) pv[e] = s[sub][8 * st + e];
            bf16x8 ph, pl;
            split8(pv, ph, pl);
            const int r0 = 16 * ksx + 4 * h + qq;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const int c0 = 4 * dt + 2 * ((lane >> 4) & 1) + (pp >> 1);
                const int a0 = vimg_off(r0, c0) + 8 * (pp & 1), a1 = vimg_off(r0 + 8, c0) + 8 * (pp & 1);
                typedef __attribute__((address_space(3))) shortx4 lds4;
                const shortx4 h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(sVh[buf] + a0));
                const shortx4 h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(sVh[buf] + a1));
                const shortx4 l0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(sVl[buf] + a0));
                const shortx4 l1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(sVl[buf] + a1));
                typedef short shortx8 __attribute__((ext_vector_type(8)));
                const shortx8 vh8 = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
                const shortx8 vl8 = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, vl8), ph, o[dt], 0, 0, 0);
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, vh8), pl, o[dt], 0, 0, 0);
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, vh8), ph, o[dt], 0, 0, 0);
            }
        }
        // write-late: the next tile's rows go to the other buffer (its readers passed the previous
        // barrier), then the tile after that is requested
        if (k0 + kBK < kend) {
            stage(buf ^ 1);
            if (k0 + 2 * kBK < kend) gather(k0 + 2 * kBK);
        }
        __syncthreads();
        if ((k0 - kbeg) / kBK < 8) WA_STAMP(4 + (k0 - kbeg) / kBK, WA_CLOCK());
    }

    // O^T[d = 32 dt + 8u + 4h + j][q = c] in o[dt][4u + j]
    if (p.ksplit == 1) {
        const float inv = 1.0f / l_run;
        float* dst = out + ((size_t)b * HW + qpix) * kC + 4 * h;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int u = 0; u < 4; ++u)
                store4(dst + 32 * dt + 8 * u, make_float4(o[dt][4 * u] * inv, o[dt][4 * u + 1] * inv,
                                                          o[dt][4 * u + 2] * inv, o[dt][4 * u + 3] * inv));
    } else {
        const size_t row = pidx(p, b, wi, ks, tq);
        float4* dst = reinterpret_cast<float4*>(part.o + lane_tile_base(p, b, wi, ks, qblk, wid)) + lane;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int u = 0; u < 4; ++u)
                dst[(dt * 4 + u) * 64] = make_float4(o[dt][4 * u], o[dt][4 * u + 1], o[dt][4 * u + 2], o[dt][4 * u + 3]);
        if (h == 0) {
            part.m[row] = m_run * kLn2;  // natural-log maxima for the combine
            part.l[row] = l_run;
        }
    }
    WA_STAMP(12, WA_CLOCK());
    WA_STAMP(13, wall_clock64());
}

// ============================================================================================
// bf16x3 v2 (round 6, default): 8 waves = two 4-wave groups on the SAME 128 queries; group g owns
// keys 32 g .. 32 g + 31 of every 64-key tile, i.e. its own half tiles (K hi / lo, V hi / lo: 32 KB,
// double-buffered per group, 128 KB in all), and keeps its own running (m, l, O); the two are
// combined through LDS at the end. The groups run win_attn_bf16_v3_kernel's one-phase stagger, so
// each SIMD pairs one group's MFMA phase (PV of the previous tile, QK of this one: 49 MFMAs) with
// the other group's VALU phase (softmax, P split, staging) instead of one wave doing both in turn
// (win_attn_x3_kernel: 6.4k cycles per tile for 3.1k of MFMAs):
//   group-local step s (group 0: s = i, group 1: s = i - 1 at global interval i, one barrier each)
//     s = 2t     (MFMA): O += V(t-1)^T P(t-1)^T (t >= 1), then S(t) = K(t) Q^T (+ mask step)
//     s = 2t + 1 (VALU): stage half tile t + 1 from registers into buffer (t + 1) % 2 (last read by
//                        PV(t - 1) in step 2t), request half tile t + 2, softmax of S(t) -> P(t).
// Q is loaded once per workgroup (512 threads, coalesced), split, and handed to both groups through
// LDS (the buffers-1 region, free until step 1). The mask A fragment is formed in registers from
// the key index. Operand maps, log2-domain softmax with deferred rescale, the mask step and the
// partials layout are those of win_attn_x3_kernel.
// ============================================================================================
constexpr int kHalfK = 32;                 // keys per group per tile
constexpr int kHImgB = kHalfK * kC * 2;    // one bf16 image of a half tile (8 KB)
constexpr int kX3BufB = 4 * kHImgB;        // Kh, Kl, Vh, Vl (32 KB)
constexpr int kX3GrpB = 2 * kX3BufB;       // two buffers per group (64 KB)
constexpr int kX3Lds = 2 * kX3GrpB;        // 128 KB

template <bool PRIO, bool WXCD>
__global__ void __launch_bounds__(kThreads8, 1)
win_attn_x3_v2_kernel(Params p, const float* __restrict__ q, const __bf16* __restrict__ khg,
                      const __bf16* __restrict__ klg, const __bf16* __restrict__ vhg, const __bf16* __restrict__ vlg,
                      float* __restrict__ out, Partials part) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[kX3Lds];

    WA_STAMP(0, wall_clock64());
    WA_STAMP(1, WA_HWID());
    WA_STAMP(2, WA_CLOCK());
    int qblk, wi, b, ks;
    if (WXCD) {
        // window-major XCD order: the remapped id walks query block, then key split, then window,
        // so the 8 x ksplit workgroups of one (batch, window) share an XCD (and its L2): Q is
        // fetched there once instead of once per key split's XCD
        const int X = gridDim.x, nwin = gridDim.y;
        const int n = blockIdx.x + X * (blockIdx.y + nwin * blockIdx.z);
        int m = xcd_remap(n, X * nwin * gridDim.z);
        qblk = m % X;
        m /= X;
        ks = m % p.ksplit;
        m /= p.ksplit;
        wi = m % nwin;
        b = m / nwin;
    } else {
        int bz;
        xcd_block_coords(qblk, wi, bz);
        b = bz / p.ksplit;
        ks = bz - b * p.ksplit;
    }
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wid >> 2, wq = wid & 3;
    const int c = lane & 31, h = lane >> 5;
    const size_t HW = (size_t)p.H * p.W;
    const int kvb = (b + p.kv_shift) % p.nbatch;
    const size_t kvoff = (size_t)kvb * p.m * HW * kC;
    const float cl2 = p.scale * kLog2e;
    const int kbeg = ks * p.keys_per_split;
    const int nt = p.keys_per_split / kBK;

    const int tq = qblk * kBQ3 + wq * kQW + c;
    // the query's region slot in the mask step's B operand (formed per tile: 4 registers fewer)
    const int qslot = (p.shift ? win_region(p, wi, tq) : 0) - 8 * h;

    // gather: wave wq of a group moves image wq (Kh, Kl, Vh, Vl) of its half tile, one 1-KB wave
    // instruction = 4 whole 256-B rows (16 lanes per row, lane = 16-B chunk: 8 cache lines per
    // instruction; a lane-per-row map touches 64 lines per instruction and ran the chip at ~9 B per
    // CU cycle). Lane c computes row c's offset (in rows); the 8 loads take theirs by shuffle.
    unsigned char* const gsm = smem + grp * kX3GrpB;
    const __bf16* const garr = (wq == 0 ? khg : wq == 1 ? klg : wq == 2 ? vhg : vlg) + kvoff;
    const int gch = lane & 15, gr = lane >> 4;  // chunk, row within a 4-row instruction
    bf16x8 gv[8];
    auto gather = [&](int t) {
        const int j = kbeg + t * kBK + kHalfK * grp + c;
        int tk = j, vi = 0;
        if (p.m != 1) {
            tk = j / p.m;
            vi = j - tk * p.m;
        }
        const int rowoff = vi * (int)HW + win_pixel(p, wi, tk);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int ro = __shfl(rowoff, 4 * i + gr, 64);
            gv[i] = *(reinterpret_cast<const bf16x8*>(garr + (size_t)ro * kC) + gch);
        }
    };
    auto stage = [&](int buf) {
        unsigned char* img = gsm + buf * kX3BufB + wq * kHImgB;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = 4 * i + gr;
            const int off = wq < 2 ? r * 256 + ((gch ^ (r & 15)) * 16) : vimg_off(r, gch);
            *reinterpret_cast<bf16x8*>(img + off) = gv[i];
        }
    };

    // prologue: half tile 0 staged, half tile 1 requested; Q (128 queries x 128 fp32) loaded by all
    // 512 threads (wave w, instruction i: rows 16 i + 2 w + {0, 1}, 32 lanes x 16 B per 512-B row),
    // split, and written as hi / lo images (row = query, 16-B chunk XOR-swizzled) into the
    // buffers-1 region of group 0 (hi) and group 1 (lo)
    gather(0);
    float4 qraw[8];
    const int c4 = lane & 31;  // float4 of the query row: channels 4 c4 .. 4 c4 + 3
    {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int qp = win_pixel(p, wi, qblk * kBQ3 + 16 * i + 2 * wid + h);
            qraw[i] = reinterpret_cast<const float4*>(q + ((size_t)b * HW + qp) * kC)[c4];
        }
    }
    stage(0);
    if (nt > 1) gather(1);  // in flight while Q is split
    {
        unsigned char* qh_img = smem + kX3BufB;            // group 0, buffer 1
        unsigned char* ql_img = smem + kX3GrpB + kX3BufB;  // group 1, buffer 1
        typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int row = 16 * i + 2 * wid + h;
            const float x[4] = {qraw[i].x, qraw[i].y, qraw[i].z, qraw[i].w};
            bf16x4v hi, lo;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                hi[e] = (__bf16)x[e];
                lo[e] = (__bf16)(x[e] - (float)hi[e]);
            }
            const int off = row * 256 + (((c4 >> 1) ^ (row & 15)) * 16) + 8 * (c4 & 1);
            *reinterpret_cast<bf16x4v*>(qh_img + off) = hi;
            *reinterpret_cast<bf16x4v*>(ql_img + off) = lo;
        }
    }
    lds_barrier();
    WA_STAMP(3, WA_CLOCK());
    bf16x8 qh[8], ql[8];
    {
        const unsigned char* qh_img = smem + kX3BufB;
        const unsigned char* ql_img = smem + kX3GrpB + kX3BufB;
        const int row = wq * kQW + c;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int off = row * 256 + (((2 * i + h) ^ (row & 15)) * 16);
            qh[i] = *reinterpret_cast<const bf16x8*>(qh_img + off);
            ql[i] = *reinterpret_cast<const bf16x8*>(ql_img + off);
        }
    }
    // group 1 runs one interval behind group 0 (its Q reads above finish before this barrier, i.e.
    // before group 0 stages half tile 1 over the Q images in its step 1)
    if (grp == 1) lds_barrier();
    // static priority for the second-dispatched half (MI355X_MICROARCH.md "Two waves per SIMD" 4)
    if (PRIO && grp == 1) __builtin_amdgcn_s_setprio(1);

    floatx16 o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;
    bf16x8 ph[2], pl[2];
    floatx16 sacc;

    // PV tr16 read addresses within a V image (keys 16 ksx + 4h + qq and + 8, d block dt)
    const int gi = lane & 15, qq = gi >> 2, pp = gi & 3;
    auto iter = [&](int t, auto bufc) -> bool {
        constexpr int BUF = decltype(bufc)::value;
        // ======== MFMA interval
        if (t >= 1) {
            const unsigned char* vh = gsm + (BUF ^ 1) * kX3BufB + 2 * kHImgB;
            const unsigned char* vl = vh + kHImgB;
#pragma unroll
            for (int ksx = 0; ksx < 2; ++ksx) {
                const int r0 = 16 * ksx + 4 * h + qq;
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) {
                    const int c0 = 4 * dt + 2 * ((lane >> 4) & 1) + (pp >> 1);
                    const int a0 = vimg_off(r0, c0) + 8 * (pp & 1), a1 = vimg_off(r0 + 8, c0) + 8 * (pp & 1);
                    typedef __attribute__((address_space(3))) shortx4 lds4;
                    const shortx4 h0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(vh + a0));
                    const shortx4 h1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(vh + a1));
                    const shortx4 l0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(vl + a0));
                    const shortx4 l1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)(vl + a1));
                    typedef short shortx8 __attribute__((ext_vector_type(8)));
                    const shortx8 vh8 = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
                    const shortx8 vl8 = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
                    o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, vl8), ph[ksx], o[dt], 0, 0, 0);
                    o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, vh8), pl[ksx], o[dt], 0, 0, 0);
                    o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, vh8), ph[ksx], o[dt], 0, 0, 0);
                }
            }
        }
        if (t < nt) {
            const unsigned char* kh = gsm + BUF * kX3BufB;
            const unsigned char* kl = kh + kHImgB;
            const floatx16 zero = {};
            sacc = zero;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int off = c * 256 + (((2 * i + h) ^ (c & 15)) * 16);
                const bf16x8 kh8 = *reinterpret_cast<const bf16x8*>(kh + off);
                const bf16x8 kl8 = *reinterpret_cast<const bf16x8*>(kl + off);
                sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kl8, qh[i], sacc, 0, 0, 0);
                sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh8, ql[i], sacc, 0, 0, 0);
                sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kh8, qh[i], sacc, 0, 0, 0);
            }
            if (p.shift) {
                // one-hot key-region A fragment of key row c (slots 8h .. 8h + 7)
                const int j = kbeg + t * kBK + kHalfK * grp + c;
                const int kreg = win_region(p, wi, p.m == 1 ? j : j % p.L);
                bf16x8 ma;
#pragma unroll
                for (int e = 0; e < 8; ++e) ma[e] = (__bf16)(kreg == 8 * h + e ? kMaskBonus : 0.0f);
                bf16x8 qmask;
#pragma unroll
                for (int e = 0; e < 8; ++e) qmask[e] = (__bf16)(qslot == e ? 1.0f : 0.0f);
                sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ma, qmask, sacc, 0, 0, 0);
            }
        }
        lds_barrier();
        if (t < 8) WA_STAMP(4 + t, WA_CLOCK());
        if (t == nt) return true;
        // ======== VALU interval: staging, then the online softmax of S(t) -> P(t)
        if (t + 1 < nt) {
            stage(BUF ^ 1);
            if (t + 2 < nt) gather(t + 2);
        }
        float bmax = max3_raw(sacc[0], sacc[1], sacc[2]);
#pragma unroll
        for (int r = 3; r < 15; r += 2) bmax = max3_raw(bmax, sacc[r], sacc[r + 1]);
        bmax = fmaxf(bmax, sacc[15]);
        const float bm2 = halves_max(bmax) * cl2;
        if (__any(bm2 > m_run + kThr)) {
            const float m_new = fmaxf(m_run, bm2);
            const float corr = fast_exp2(m_run - m_new);
            l_run *= corr;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) o[dt] *= corr;
            m_run = m_new;
        }
        float bsum = 0.f;
#pragma unroll
        for (int ksx = 0; ksx < 2; ++ksx) {
            float pv[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                pv[e] = fast_exp2(fmaf(sacc[8 * ksx + e], cl2, -m_run));
                bsum += pv[e];
            }
            split8(pv, ph[ksx], pl[ksx]);
        }
        l_run += halves_sum(bsum);
        lds_barrier();
        return false;
    };
    for (int t = 0;; t += 2) {
        if (iter(t, IC<0>{})) break;
        if (iter(t + 1, IC<1>{})) break;
    }
    if (grp == 0) lds_barrier();

    // combine the two key halves, split by d: group g finishes O^T rows d in [64 g, 64 g + 64)
    // (accumulators dt = 2 g, 2 g + 1) and parks the other half, plus its (m, l), for the other group
    float4* const park = reinterpret_cast<float4*>(smem);
    float2* const park_ml = reinterpret_cast<float2*>(smem + 2 * 4 * 8 * 64 * 16);
    auto finish = [&](auto gc) {
        constexpr int G = decltype(gc)::value;  // this group (static accumulator indices)
        float4* const mine = park + (size_t)(G * 4 + wq) * 8 * 64 + lane;
        const float4* const theirs = park + (size_t)((G ^ 1) * 4 + wq) * 8 * 64 + lane;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                constexpr int D0 = 2 * (G ^ 1);
                mine[(j * 4 + u) * 64] =
                    make_float4(o[D0 + j][4 * u], o[D0 + j][4 * u + 1], o[D0 + j][4 * u + 2], o[D0 + j][4 * u + 3]);
            }
        park_ml[(G * 4 + wq) * 64 + lane] = make_float2(m_run, l_run);
        lds_barrier();
        const float2 ml1 = park_ml[((G ^ 1) * 4 + wq) * 64 + lane];
        const float mm = fmaxf(m_run, ml1.x);
        const float f0 = fast_exp2(m_run - mm), f1 = fast_exp2(ml1.x - mm);
        l_run = l_run * f0 + ml1.y * f1;
        m_run = mm;
        constexpr int D = 2 * G;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float4 x = theirs[(j * 4 + u) * 64];
                o[D + j][4 * u] = o[D + j][4 * u] * f0 + x.x * f1;
                o[D + j][4 * u + 1] = o[D + j][4 * u + 1] * f0 + x.y * f1;
                o[D + j][4 * u + 2] = o[D + j][4 * u + 2] * f0 + x.z * f1;
                o[D + j][4 * u + 3] = o[D + j][4 * u + 3] * f0 + x.w * f1;
            }
        // O^T[d = 32 dt + 8u + 4h + j][q = c] in o[dt][4u + j]
        if (p.ksplit == 1) {
            const float inv = 1.0f / l_run;
            float* dst = out + ((size_t)b * HW + win_pixel(p, wi, tq)) * kC + 4 * h;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    store4(dst + 32 * (D + j) + 8 * u,
                           make_float4(o[D + j][4 * u] * inv, o[D + j][4 * u + 1] * inv, o[D + j][4 * u + 2] * inv,
                                       o[D + j][4 * u + 3] * inv));
        } else {
            float4* dst = reinterpret_cast<float4*>(part.o + lane_tile_base(p, b, wi, ks, qblk, wq)) + lane;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    dst[((D + j) * 4 + u) * 64] =
                        make_float4(o[D + j][4 * u], o[D + j][4 * u + 1], o[D + j][4 * u + 2], o[D + j][4 * u + 3]);
            if (G == 0 && h == 0) {
                const size_t row = pidx(p, b, wi, ks, tq);
                part.m[row] = m_run * kLn2;
                part.l[row] = l_run;
            }
        }
    };
    if (grp == 0)
        finish(IC<0>{});
    else
        finish(IC<1>{});
    WA_STAMP(12, WA_CLOCK());
    WA_STAMP(13, wall_clock64());
}

// K and V (fp32, n elements each) -> [kh | kl | vh | vl] bf16, x = xh + xl (see win_attn_x3_kernel)
__global__ void __launch_bounds__(256) split_kv_kernel(const float4* __restrict__ k, const float4* __restrict__ v,
                                                       __bf16* __restrict__ out, size_t n4) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const float4 x = blockIdx.y ? v[i] : k[i];
    typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
    bf16x4v hi, lo;
    const float e[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        hi[j] = (__bf16)e[j];
        lo[j] = (__bf16)(e[j] - (float)hi[j]);
    }
    bf16x4v* o = reinterpret_cast<bf16x4v*>(out + (size_t)blockIdx.y * 2 * (4 * n4));
    o[i] = hi;
    o[n4 + i] = lo;
}

}  // namespace winattn
}  // namespace tsplat

using namespace tsplat;

// keys are split so a launch fills the 256 CUs: >= 512 workgroups for the 16x16 kernel (two per
// CU), >= 256 for the 32x32 kernel (one per CU, software-pipelined)
static int choose_ksplit(int base_wgs, int key_tiles, int target) {
    int ks = 1;
    while (base_wgs * ks < target && ks * 2 <= key_tiles && key_tiles % (ks * 2) == 0 && ks < 8) ks *= 2;
    return ks;
}

// Tuning knobs (benchmarking only): TSPLAT_WINATTN=16 forces the 16x16x4 kernel;
// TSPLAT_WINATTN_KSPLIT forces the key split. (Round 4: the opt-in variants measured slower than the
// defaults -- the 16-query-wave x16 kernel, the key-pair kernel, the split-free quad kernel and the
// round-1 bf16 kernel -- were removed; DESIGN.md §3 keeps their measurements.)
static int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}
static bool env_is(const char* name, const char* val) {
    const char* e = getenv(name);
    return e && !strcmp(e, val);
}

// query-block size of the kernel used for window size L (128: 32x32x2 kernel, 64: 16x16x4)
static int query_block(int L) {
    if (env_is("TSPLAT_WINATTN", "16")) return tsplat::winattn::kBQ;
    return L % tsplat::winattn::kBQ3 == 0 ? tsplat::winattn::kBQ3 : tsplat::winattn::kBQ;
}
// 128-query kernel: one workgroup per CU is enough (measured: b = 2 at 256 workgroups beats 512,
// and the key-pair kernel); the 16x16x4 kernel wants two per CU
static int pick_ksplit(int base, int key_tiles, int qb) {
    const int forced = env_int("TSPLAT_WINATTN_KSPLIT", 0);
    if (forced > 0 && key_tiles % forced == 0) return forced;
    return choose_ksplit(base, key_tiles, qb == tsplat::winattn::kBQ3 ? 256 : 512);
}

extern "C" size_t tsplat_win_attn_workspace_bytes(int32_t batch, int32_t height, int32_t width,
                                                  int32_t key_views, int32_t splits) {
    using namespace tsplat::winattn;
    if (batch <= 0 || key_views <= 0 || splits <= 0 || height % splits || width % splits) return 0;
    const int L = (height / splits) * (width / splits);
    if (L % kBQ || (L * key_views) % kBK) return 0;
    const int base = (L / query_block(L)) * splits * splits * batch;
    const int ks = pick_ksplit(base, L * key_views / kBK, query_block(L));
    if (ks == 1) return 0;
    return (size_t)batch * splits * splits * ks * L * (kC + 2) * sizeof(float);
}

extern "C" int tsplat_win_attn_fwd(const float* q, const float* k, const float* v, float* out,
                                   void* workspace, int32_t batch, int32_t height, int32_t width,
                                   int32_t channels, int32_t key_views, int32_t splits,
                                   int32_t with_shift, void* stream_) {
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
    p.shift_h = with_shift ? (height / splits) / 2 : 0;
    p.shift_w = with_shift ? (width / splits) / 2 : 0;
    p.shift = with_shift ? 1 : 0;
    p.wh = height / splits;
    p.ww = width / splits;
    p.ww_log2 = (p.ww & (p.ww - 1)) == 0 ? __builtin_ctz(p.ww) : -1;
    p.kv_shift = 0;
    p.nbatch = batch;
    if (with_shift && (p.shift_h == 0 || p.shift_w == 0)) return TSPLAT_EINVAL;
    if (p.L % kBQ || (p.L * p.m) % kBK) return TSPLAT_EINVAL;
    p.scale = 1.0f / sqrtf((float)kC);
    hipStream_t stream = (hipStream_t)stream_;
    const int qb = query_block(p.L);
    const int base = (p.L / qb) * splits * splits * batch;
    p.ksplit = pick_ksplit(base, p.L * p.m / kBK, qb);
    p.keys_per_split = p.L * p.m / p.ksplit;
    Partials part{nullptr, nullptr, nullptr};
    if (p.ksplit > 1) {
        if (!workspace) return TSPLAT_EINVAL;
        const size_t n = (size_t)batch * splits * splits * p.ksplit * p.L;
        part.o = (float*)workspace;
        part.m = part.o + n * kC;
        part.l = part.m + n;
    }
    const dim3 grid(p.L / qb, splits * splits, batch * p.ksplit);
    TSPLAT_PROF_BEGIN(prof::kWinAttn, stream);
    if (qb == kBQ3)
        hipLaunchKernelGGL(win_attn_f32x32_kernel, grid, dim3(kThreads), 0, stream, p, q, k, v, out, part);
    else
        hipLaunchKernelGGL(win_attn_f32_kernel, grid, dim3(kThreads), 0, stream, p, q, k, v, out, part);
    if (p.ksplit > 1 && qb == kBQ3)
        hipLaunchKernelGGL(win_attn_combine_x32_kernel<float>, dim3(p.L / kBQ3 * 16, splits * splits, batch),
                           dim3(kThreads), 0, stream, p, part, out);
    else if (p.ksplit > 1)
        hipLaunchKernelGGL(win_attn_combine_kernel<float>, dim3(p.L / (kThreads / 32), splits * splits, batch),
                           dim3(kThreads), 0, stream, p, part, out);
    TSPLAT_PROF_END(prof::kWinAttn, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

// Key split the exact-fp32 128-query kernel uses for this launch shape (the same decision as
// tsplat_win_attn_fwd): > 1 means the call runs main + combine and tsplat_win_attn_partials_fwd
// may be used instead; 1 = no split; 0 = another kernel serves this shape.
extern "C" int32_t tsplat_win_attn_split(int32_t batch, int32_t height, int32_t width, int32_t key_views,
                                         int32_t splits) {
    using namespace tsplat::winattn;
    if (batch <= 0 || key_views <= 0 || splits <= 0 || height % splits || width % splits) return 0;
    const int L = (height / splits) * (width / splits);
    if (L % kBQ3 || (L * key_views) % kBK || getenv("TSPLAT_WINATTN")) return 0;
    const int base = (L / kBQ3) * splits * splits * batch;
    return pick_ksplit(base, L * key_views / kBK, kBQ3);
}

// The main kernel only: the split-key partials (O unnormalised, m in natural log, l) stay in
// `workspace` for a consumer that folds the combine into its own prologue (the merge projection,
// tsplat_linear_f32_attn_merge_fwd). Only for shapes where tsplat_win_attn_split() > 1.
extern "C" int tsplat_win_attn_partials_fwd(const float* q, const float* k, const float* v, void* workspace,
                                            int32_t batch, int32_t height, int32_t width, int32_t channels,
                                            int32_t key_views, int32_t splits, int32_t with_shift,
                                            int32_t key_batch_shift, void* stream_) {
    using namespace tsplat::winattn;
    if (!q || !k || !v || !workspace || channels != kC) return TSPLAT_EINVAL;
    if (key_batch_shift < 0 || key_batch_shift >= batch) return TSPLAT_EINVAL;
    const int ks = tsplat_win_attn_split(batch, height, width, key_views, splits);
    if (ks <= 1) return TSPLAT_EINVAL;
    Params p;
    p.H = height;
    p.W = width;
    p.splits = splits;
    p.m = key_views;
    p.L = (height / splits) * (width / splits);
    p.shift_h = with_shift ? (height / splits) / 2 : 0;
    p.shift_w = with_shift ? (width / splits) / 2 : 0;
    p.shift = with_shift ? 1 : 0;
    p.wh = height / splits;
    p.ww = width / splits;
    p.ww_log2 = (p.ww & (p.ww - 1)) == 0 ? __builtin_ctz(p.ww) : -1;
    p.kv_shift = 0;
    p.nbatch = batch;
    if (with_shift && (p.shift_h == 0 || p.shift_w == 0)) return TSPLAT_EINVAL;
    p.scale = 1.0f / sqrtf((float)kC);
    p.ksplit = ks;
    p.keys_per_split = p.L * p.m / p.ksplit;
    p.kv_shift = key_batch_shift;
    const size_t n = (size_t)batch * splits * splits * p.ksplit * p.L;
    Partials part{(float*)workspace, nullptr, nullptr};
    part.m = part.o + n * kC;
    part.l = part.m + n;
    hipStream_t stream = (hipStream_t)stream_;
    const prof::ExtEvents ev = prof::ext_events(prof::kWinAttn);  // kernel timestamps when timed
    hipExtLaunchKernelGGL(win_attn_f32x32_kernel, dim3(p.L / kBQ3, splits * splits, batch * p.ksplit),
                              dim3(kThreads), 0, stream, ev.start, ev.stop, 0, p, q, k, v, (float*)nullptr, part);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

#if TSPLAT_WA_STAMP
// diagnostic builds only: buffer of [workgroups][16] uint64 the next x32 launches stamp (null = off)
extern "C" int tsplat_win_attn_stamps(void* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(tsplat::winattn::g_wa_stamps), &buf, sizeof(buf)) == hipSuccess
               ? TSPLAT_OK : TSPLAT_EINVAL;
}
#endif

extern "C" size_t tsplat_win_attn_bf16_workspace_bytes(int32_t batch, int32_t height, int32_t width,
                                                       int32_t key_views, int32_t splits) {
    using namespace tsplat::winattn;
    if (batch <= 0 || key_views <= 0 || splits <= 0 || height % splits || width % splits) return 0;
    const int L = (height / splits) * (width / splits);
    if (L % kBQ3 || (L * key_views) % kBK) return 0;
    const int base = (L / kBQ3) * splits * splits * batch;
    const int ks = choose_ksplit(base, L * key_views / kBK, 512);
    if (ks == 1) return 0;
    return (size_t)batch * splits * splits * ks * L * (kC + 2) * sizeof(float);
}

extern "C" int tsplat_win_attn_bf16_shift_fwd(const void* q, const void* k, const void* v, void* out,
                                              void* workspace, int32_t batch, int32_t height, int32_t width,
                                              int32_t channels, int32_t key_views, int32_t splits,
                                              int32_t with_shift, int32_t key_batch_shift, void* stream_);

extern "C" int tsplat_win_attn_bf16_fwd(const void* q, const void* k, const void* v, void* out,
                                        void* workspace, int32_t batch, int32_t height, int32_t width,
                                        int32_t channels, int32_t key_views, int32_t splits,
                                        int32_t with_shift, void* stream_) {
    return tsplat_win_attn_bf16_shift_fwd(q, k, v, out, workspace, batch, height, width, channels, key_views, splits,
                                          with_shift, 0, stream_);
}

// tsplat_win_attn_bf16_fwd where query batch b attends to the keys / values of batch
// (b + key_batch_shift) % batch (the two-view cross pairing of forward_pair without a rolled copy)
extern "C" int tsplat_win_attn_bf16_shift_fwd(const void* q, const void* k, const void* v, void* out,
                                              void* workspace, int32_t batch, int32_t height, int32_t width,
                                              int32_t channels, int32_t key_views, int32_t splits,
                                              int32_t with_shift, int32_t key_batch_shift, void* stream_) {
    using namespace tsplat::winattn;
    if (!q || !k || !v || !out) return TSPLAT_EINVAL;
    if (key_batch_shift < 0 || key_batch_shift >= batch) return TSPLAT_EINVAL;
    if (channels != kC || batch <= 0 || key_views <= 0 || splits <= 0) return TSPLAT_EINVAL;
    if (height % splits || width % splits) return TSPLAT_EINVAL;
    Params p;
    p.H = height;
    p.W = width;
    p.splits = splits;
    p.m = key_views;
    p.L = (height / splits) * (width / splits);
    p.shift_h = with_shift ? (height / splits) / 2 : 0;
    p.shift_w = with_shift ? (width / splits) / 2 : 0;
    p.shift = with_shift ? 1 : 0;
    p.wh = height / splits;
    p.ww = width / splits;
    p.ww_log2 = (p.ww & (p.ww - 1)) == 0 ? __builtin_ctz(p.ww) : -1;
    p.kv_shift = key_batch_shift;
    p.nbatch = batch;
    if (with_shift && (p.shift_h == 0 || p.shift_w == 0)) return TSPLAT_EINVAL;
    if (p.L % kBQ3 || (p.L * p.m) % kBK) return TSPLAT_EINVAL;
    p.scale = 1.0f / sqrtf((float)kC);
    // v3 (8 staggered waves, 256 queries per workgroup, no key split) where the launch gives
    // >= 1 workgroup per CU without splitting keys; TSPLAT_WINATTN_BF16=v2 / v3 selects
    const bool v3 = p.L % kBQ8 == 0 &&
                    (env_is("TSPLAT_WINATTN_BF16", "v3") ||
                     (!getenv("TSPLAT_WINATTN_BF16") && (p.L / kBQ8) * splits * splits * batch >= 256));
    const int base = (p.L / kBQ3) * splits * splits * batch;
    p.ksplit = v3 ? 1 : choose_ksplit(base, p.L * p.m / kBK, 512);
    p.keys_per_split = p.L * p.m / p.ksplit;
    Partials part{nullptr, nullptr, nullptr};
    if (p.ksplit > 1) {
        if (!workspace) return TSPLAT_EINVAL;
        const size_t n = (size_t)batch * splits * splits * p.ksplit * p.L;
        part.o = (float*)workspace;
        part.m = part.o + n * kC;
        part.l = part.m + n;
    }
    hipStream_t stream = (hipStream_t)stream_;
    // the main kernel's own dispatch timestamps when timed (the split path's combine is not in it)
    const prof::ExtEvents ev = prof::ext_events(prof::kWinAttn);
    const __bf16 *qh = (const __bf16*)q, *kh = (const __bf16*)k, *vh = (const __bf16*)v;
    if (v3)
        hipExtLaunchKernelGGL(win_attn_bf16_v3_kernel, dim3(p.L / kBQ8, splits * splits, batch), dim3(kThreads8), 0,
                              stream, ev.start, ev.stop, 0, p, qh, kh, vh, (__bf16*)out);
    else
        hipExtLaunchKernelGGL(win_attn_bf16_v2_kernel, dim3(p.L / kBQ3, splits * splits, batch * p.ksplit),
                              dim3(kThreads), 0, stream, ev.start, ev.stop, 0, p, qh, kh, vh, (__bf16*)out, part);
    if (p.ksplit > 1)
        hipLaunchKernelGGL(win_attn_combine_x32_kernel<__bf16>, dim3(p.L / kBQ3 * 16, splits * splits, batch),
                           dim3(kThreads), 0, stream, p, part, (__bf16*)out);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}


// bf16x3 key / value split for tsplat_win_attn_x3_*: out = [kh | kl | vh | vl], each n bf16
extern "C" int tsplat_split_kv_bf16x3(const float* k, const float* v, void* out, int64_t n, void* stream_) {
    if (!k || !v || !out || n <= 0 || n % 4 || ((uintptr_t)k & 15) || ((uintptr_t)v & 15) || ((uintptr_t)out & 7))
        return TSPLAT_EINVAL;
    const size_t n4 = (size_t)n / 4;
    hipLaunchKernelGGL(tsplat::winattn::split_kv_kernel, dim3((unsigned)((n4 + 255) / 256), 2), dim3(256), 0,
                       (hipStream_t)stream_, (const float4*)k, (const float4*)v, (__bf16*)out, n4);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

static int x3_params(tsplat::winattn::Params& p, int32_t batch, int32_t height, int32_t width, int32_t channels,
                     int32_t key_views, int32_t splits, int32_t with_shift, int32_t key_batch_shift) {
    using namespace tsplat::winattn;
    if (channels != kC || batch <= 0 || key_views <= 0 || splits <= 0 || height % splits || width % splits)
        return TSPLAT_EINVAL;
    if (key_batch_shift < 0 || key_batch_shift >= batch) return TSPLAT_EINVAL;
    p.H = height;
    p.W = width;
    p.splits = splits;
    p.m = key_views;
    p.L = (height / splits) * (width / splits);
    p.shift_h = with_shift ? (height / splits) / 2 : 0;
    p.shift_w = with_shift ? (width / splits) / 2 : 0;
    p.shift = with_shift ? 1 : 0;
    p.wh = height / splits;
    p.ww = width / splits;
    p.ww_log2 = (p.ww & (p.ww - 1)) == 0 ? __builtin_ctz(p.ww) : -1;
    p.kv_shift = key_batch_shift;
    p.nbatch = batch;
    if (with_shift && (p.shift_h == 0 || p.shift_w == 0)) return TSPLAT_EINVAL;
    if (p.L % kBQ3 || (p.L * p.m) % kBK) return TSPLAT_EINVAL;
    p.scale = 1.0f / sqrtf((float)kC);
    // the exact kernel's key split (so the workspace / partials layout is the same)
    const int base = (p.L / kBQ3) * splits * splits * batch;
    p.ksplit = pick_ksplit(base, p.L * p.m / kBK, kBQ3);
    p.keys_per_split = p.L * p.m / p.ksplit;
    return TSPLAT_OK;
}

// the bf16x3 main kernel: the 8-wave two-group form (default) or the round-5 4-wave form
// (TSPLAT_WINATTN_X3=v1, the A/B knob); same grid, partials and output either way
static void launch_x3(const tsplat::winattn::Params& p, int splits, int batch, const float* q, const __bf16* kv,
                      size_t nkv, float* out, tsplat::winattn::Partials part, const tsplat::prof::ExtEvents& ev,
                      hipStream_t stream) {
    using namespace tsplat::winattn;
    const dim3 grid(p.L / kBQ3, splits * splits, batch * p.ksplit);
    if (env_is("TSPLAT_WINATTN_X3", "v1"))
        hipExtLaunchKernelGGL(win_attn_x3_kernel, grid, dim3(kThreads), 0, stream, ev.start, ev.stop, 0, p, q, kv,
                              kv + nkv, kv + 2 * nkv, kv + 3 * nkv, out, part);
    else if (env_is("TSPLAT_WINATTN_X3_PRIO", "0"))  // A/B knob: no static priority
        hipExtLaunchKernelGGL((win_attn_x3_v2_kernel<false, true>), grid, dim3(kThreads8), 0, stream, ev.start,
                              ev.stop, 0, p, q, kv, kv + nkv, kv + 2 * nkv, kv + 3 * nkv, out, part);
    else if (env_is("TSPLAT_WINATTN_X3_XCD", "split"))  // A/B knob: key-split-major XCD order
        hipExtLaunchKernelGGL((win_attn_x3_v2_kernel<true, false>), grid, dim3(kThreads8), 0, stream, ev.start,
                              ev.stop, 0, p, q, kv, kv + nkv, kv + 2 * nkv, kv + 3 * nkv, out, part);
    else  // window-major XCD order (profiles/r6/traffic_win_attn_x3_xcd.txt: fetch 17.4 vs 30.0 MB)
        hipExtLaunchKernelGGL((win_attn_x3_v2_kernel<true, true>), grid, dim3(kThreads8), 0, stream, ev.start,
                              ev.stop, 0, p, q, kv, kv + nkv, kv + 2 * nkv, kv + 3 * nkv, out, part);
}

// bf16x3 window attention, main kernel only (partials for the merge projection); kv_x3 =
// tsplat_split_kv_bf16x3(k, v) ([kh | kl | vh | vl], k / v [batch, key_views, H*W, 128]). Same
// shapes, key split and workspace as tsplat_win_attn_partials_fwd.
extern "C" int tsplat_win_attn_x3_partials_fwd(const float* q, const void* kv_x3, void* workspace, int32_t batch,
                                               int32_t height, int32_t width, int32_t channels, int32_t key_views,
                                               int32_t splits, int32_t with_shift, int32_t key_batch_shift,
                                               void* stream_) {
    using namespace tsplat::winattn;
    if (!q || !kv_x3 || !workspace) return TSPLAT_EINVAL;
    Params p;
    if (x3_params(p, batch, height, width, channels, key_views, splits, with_shift, key_batch_shift) != TSPLAT_OK)
        return TSPLAT_EINVAL;
    if (p.ksplit <= 1) return TSPLAT_EINVAL;
    const size_t n = (size_t)batch * splits * splits * p.ksplit * p.L;
    Partials part{(float*)workspace, nullptr, nullptr};
    part.m = part.o + n * kC;
    part.l = part.m + n;
    const size_t nkv = (size_t)batch * key_views * height * width * kC;
    const __bf16* kv = (const __bf16*)kv_x3;
    hipStream_t stream = (hipStream_t)stream_;
    const prof::ExtEvents ev = prof::ext_events(prof::kWinAttn);
    launch_x3(p, splits, batch, q, kv, nkv, (float*)nullptr, part, ev, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

// bf16x3 window attention, standalone (main + combine when the keys are split): out [batch, H*W,
// 128] fp32, the same result class as tsplat_win_attn_fwd at >= TF32 precision (tests, benchmarks)
extern "C" int tsplat_win_attn_x3_fwd(const float* q, const void* kv_x3, float* out, void* workspace, int32_t batch,
                                      int32_t height, int32_t width, int32_t channels, int32_t key_views,
                                      int32_t splits, int32_t with_shift, void* stream_) {
    using namespace tsplat::winattn;
    if (!q || !kv_x3 || !out) return TSPLAT_EINVAL;
    Params p;
    if (x3_params(p, batch, height, width, channels, key_views, splits, with_shift, 0) != TSPLAT_OK)
        return TSPLAT_EINVAL;
    Partials part{nullptr, nullptr, nullptr};
    if (p.ksplit > 1) {
        if (!workspace) return TSPLAT_EINVAL;
        const size_t n = (size_t)batch * splits * splits * p.ksplit * p.L;
        part.o = (float*)workspace;
        part.m = part.o + n * kC;
        part.l = part.m + n;
    }
    const size_t nkv = (size_t)batch * key_views * height * width * kC;
    const __bf16* kv = (const __bf16*)kv_x3;
    hipStream_t stream = (hipStream_t)stream_;
    const prof::ExtEvents ev = prof::ext_events(prof::kWinAttn);
    launch_x3(p, splits, batch, q, kv, nkv, out, part, ev, stream);
    if (p.ksplit > 1)
        hipLaunchKernelGGL(win_attn_combine_x32_kernel<float>, dim3(p.L / kBQ3 * 16, splits * splits, batch),
                           dim3(kThreads), 0, stream, p, part, out);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
