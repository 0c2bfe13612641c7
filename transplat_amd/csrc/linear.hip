// Row-block fp32 GEMM with fused epilogues for the multi-view transformer's linears on gfx950.
//
// Semantics (reference TransformerLayer.forward, src/model/encoder/backbone/multiview_transformer.py
// :327-407, single head, no biases): per layer
//   q, k, v = x Wq^T, y Wk^T, y Wv^T                        (q_proj / k_proj / v_proj)
//   m = norm1(attn Wmerge^T)                                 (merge + LayerNorm, eps 1e-5)
//   self layer:      out = x + m
//   cross/FFN layer: out = x + norm2(GELU([x | m] W1^T) W2^T) (mlp = Linear, exact GELU, Linear)
// One launch computes out[M, N] = epilogue([x1 | x2] W^T) with
//   x1 [M, k1], x2 [M, k2] (the concatenation is never materialised), W [N, k1 + k2] (nn.Linear),
//   epilogue = (+ bias) -> (exact-erf GELU) -> (LayerNorm over N = 128 with gamma / beta) ->
//   (+ residual [M, N]); "split" writes column block j of 128 to out + j * split_stride.
// Replaces per layer up to 11 PyTorch launches (3-4 hipBLASLt GEMMs, cat, GELU, 2 LayerNorms, add).
//
// Kernel: one workgroup = 4 waves = BM (32 or 64) rows x 128 columns; wave w owns columns
// [32 w, 32 w + 32) as BM / 32 v_mfma_f32_32x32x2_f32 accumulators (exact fp32). A = W (MFMA rows =
// output columns), B = X^T (MFMA columns = output rows), so lane (m, h) ends with 16 columns of ONE
// output row per accumulator: the row-wise LayerNorm needs only in-lane sums, one half-wave swap
// and a 4-wave LDS exchange. K is walked in 64-wide chunks staged through LDS (rows XOR-swizzled
// per 16-B chunk, ping-pong buffers) with two register stages in flight (see linear_f32_kernel).
#include "common.h"
#include "prof.h"

namespace tsplat {
namespace linear {

constexpr int kBN = 128;  // columns per workgroup
constexpr int kBK = 64;   // K chunk
constexpr int kThreads = 512;  // 8 waves: two per SIMD

enum Flags : int {
    kGelu = 1, kLayerNorm = 2, kResidual = 4, kSplit = 8, kBias = 16, kGeluIn = 32,
    kResPreLN = 64,  // with kResidual: the residual is added BEFORE the LayerNorm (post-norm layers)
    kReluIn = 128,   // ReLU applied to X as it is staged (the producing FFN layer's activation)
    kBf16x3 = 256,   // split-bf16 products (x = hi + lo; hi*hi + hi*lo + lo*hi on 32x32x16 bf16 MFMA)
    kXBf16 = 512,    // x1 is bf16 (widened exactly as it is staged; no x2)
    kOutBf16 = 1024, // the output is written as bf16 (round to nearest even; no residual)
};

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

struct Args {
    const float* x1;
    const float* x2;
    const float* w;
    const float* bias;
    const float* gamma;
    const float* beta;
    const float* res;
    float* out;
    long long split_stride;
    float eps;
    int k1, k2, M, N, flags;
    // X = combined split-key attention partials (tsplat_win_attn_partials_fwd layout), see
    // tsplat_linear_f32_attn_merge_fwd: o / m / l arrays and the window geometry
    const float* po;
    const float* pm;
    const float* pl;
    int aks, aH, aW, aS, aL, awh, aww, ash, asw;
    // kSplit outputs from column block x3_from on go to kv_x3 as bf16 hi / lo pairs (x = hi + lo):
    // block x3_from + i -> hi at kv_x3 + 2 i M 128, lo at kv_x3 + (2 i + 1) M 128 (the K / V operands
    // of tsplat_win_attn_x3_*); x3_from < 0: none
    __bf16* kv_x3;
    int x3_from;
};

constexpr int kMaxSplit = 8;

// Per-thread source of one X row when X is the attention output still split over key ranges:
// float offset of (row, split 0, this query's lane) in o, the split stride, the combine weights
struct AttnRow {
    size_t obase;
    float w[kMaxSplit];
};

__device__ __forceinline__ void attn_row(const Args& a, int m, AttnRow& r) {
    const int HW = a.aH * a.aW;
    const int b = m / HW, pix = m - b * HW;
    const int y = pix / a.aW, x = pix - y * a.aW;
    int Y = y - a.ash, X = x - a.asw;  // position on the rolled grid (the attention rolled by -shift)
    if (Y < 0) Y += a.aH;
    if (X < 0) X += a.aW;
    const int sy = Y / a.awh, sx = X / a.aww;
    const int wi = sy * a.aS + sx, t = (Y - sy * a.awh) * a.aww + (X - sx * a.aww);
    const size_t win = (size_t)b * a.aS * a.aS + wi;
    const int nqb = a.aL / 128;
    r.obase = ((win * a.aks * nqb + (t >> 7)) * 128 + 32 * ((t >> 5) & 3)) * 128 + 4 * (t & 31);
    float mx = -INFINITY;
#pragma unroll
    for (int s = 0; s < kMaxSplit; ++s)
        if (s < a.aks) mx = fmaxf(mx, a.pm[(win * a.aks + s) * a.aL + t]);
    float L = 0.f;
#pragma unroll
    for (int s = 0; s < kMaxSplit; ++s) {
        r.w[s] = 0.f;
        if (s < a.aks) {
            const size_t row = (win * a.aks + s) * a.aL + t;
            r.w[s] = __expf(a.pm[row] - mx);
            L += r.w[s] * a.pl[row];
        }
    }
    const float inv = 1.0f / L;
#pragma unroll
    for (int s = 0; s < kMaxSplit; ++s) r.w[s] *= inv;
}

// channels k .. k+3 of the combined attention row: O^T[d][q] float4 (dt * 4 + u) * 64 + lane of
// the wave slot holds d = 32 dt + 8 u + 4 h + (0..3) for lane = q + 32 h
__device__ __forceinline__ floatx4 attn_x4(const Args& a, const AttnRow& r, int k) {
    const size_t sstride = (size_t)(a.aL / 128) * 128 * 128;
    const size_t off = r.obase + ((size_t)(((k >> 5) * 4 + ((k >> 3) & 3)) * 64 + 32 * ((k >> 2) & 1))) * 4;
    floatx4 acc = (floatx4)(0.f);
#pragma unroll
    for (int s = 0; s < kMaxSplit; ++s)
        if (s < a.aks) acc += r.w[s] * *reinterpret_cast<const floatx4*>(a.po + off + s * sstride);
    return acc;
}

__device__ __forceinline__ float halves_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// One K chunk in flight in registers: thread = 16-B chunk (tid & 15) of rows (tid >> 4) + 32 i.
template <int BM>
struct Stage {
    floatx4 x[BM / 32], w[kBN / 32];
};

template <int BM, bool ATTN>
__device__ __forceinline__ void stage_load(const Args& a, int m0, int n0, int K, int ck, int tid, Stage<BM>& st,
                                           const AttnRow (&ar)[BM / 32]) {
    const int srow = tid >> 4, sq = tid & 15;
    const int k0 = ck * kBK;
    if (ATTN) {
#pragma unroll
        for (int i = 0; i < BM / 32; ++i)
            st.x[i] = m0 + srow + 32 * i < a.M ? attn_x4(a, ar[i], k0 + 4 * sq) : (floatx4)(0.f);
    } else {
        const bool first = k0 < a.k1;
        const float* xs = first ? a.x1 : a.x2;
        const int ld = first ? a.k1 : a.k2, kk = first ? k0 : k0 - a.k1;
        if (a.flags & kXBf16) {  // x1 bf16: 4 channels = 8 B, widened exactly
            typedef __bf16 bf16x4l __attribute__((ext_vector_type(4)));
            const __bf16* xb = reinterpret_cast<const __bf16*>(a.x1);
#pragma unroll
            for (int i = 0; i < BM / 32; ++i) {
                const int m = m0 + srow + 32 * i;
                st.x[i] = m < a.M ? __builtin_convertvector(
                                        *reinterpret_cast<const bf16x4l*>(xb + (size_t)m * a.k1 + k0 + 4 * sq), floatx4)
                                  : (floatx4)(0.f);
            }
        } else {
#pragma unroll
            for (int i = 0; i < BM / 32; ++i) {
                const int m = m0 + srow + 32 * i;
                st.x[i] = m < a.M ? *reinterpret_cast<const floatx4*>(xs + (size_t)m * ld + kk + 4 * sq) : (floatx4)(0.f);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < kBN / 32; ++i)
        st.w[i] = *reinterpret_cast<const floatx4*>(a.w + (size_t)(n0 + srow + 32 * i) * K + k0 + 4 * sq);
}

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// bf16x3 staging: a 256-B row holds the chunk's 64 channels as [hi: 8 units of 8 bf16 | lo: 8 units],
// 16-B unit u at slot u ^ (row & 15) (the fp32 image's swizzle); fp32 unit sq (channels 4 sq ..
// 4 sq + 3) is the (sq & 1) half of bf16 unit sq >> 1
__device__ __forceinline__ void store_split(char* base, int r, int sq, floatx4 v) {
    const bf16x4 hi = __builtin_convertvector(v, bf16x4);
    const bf16x4 lo = __builtin_convertvector(v - __builtin_convertvector(hi, floatx4), bf16x4);
    char* row = base + r * 256 + (sq & 1) * 8;
    *reinterpret_cast<bf16x4*>(row + (((sq >> 1) ^ (r & 15)) << 4)) = hi;
    *reinterpret_cast<bf16x4*>(row + (((8 + (sq >> 1)) ^ (r & 15)) << 4)) = lo;
}

template <int BM, bool X3>
__device__ __forceinline__ void stage_store(float* sX, float* sW, int tid, const Stage<BM>& st, bool gelu_in,
                                            bool relu_in) {
    const int srow = tid >> 4, sq = tid & 15;
#pragma unroll
    for (int i = 0; i < BM / 32; ++i) {
        const int r = srow + 32 * i;
        floatx4 x = st.x[i];
        if (gelu_in) x = (floatx4){gelu_erf(x.x), gelu_erf(x.y), gelu_erf(x.z), gelu_erf(x.w)};
        if (relu_in) x = (floatx4){fmaxf(x.x, 0.f), fmaxf(x.y, 0.f), fmaxf(x.z, 0.f), fmaxf(x.w, 0.f)};
        if (X3)
            store_split(reinterpret_cast<char*>(sX), r, sq, x);
        else
            *reinterpret_cast<floatx4*>(&sX[r * kBK + ((sq ^ (r & 15)) * 4)]) = x;
    }
#pragma unroll
    for (int i = 0; i < kBN / 32; ++i) {
        const int r = srow + 32 * i;
        if (X3)
            store_split(reinterpret_cast<char*>(sW), r, sq, st.w[i]);
        else
            *reinterpret_cast<floatx4*>(&sW[r * kBK + ((sq ^ (r & 15)) * 4)]) = st.w[i];
    }
}

// bf16x3 k-steps s0 .. s0 + NS - 1 of a chunk (16 channels each; lane half h supplies channels
// 16 s + 8 h .. + 7): A = W row wrow, B = X row xr, each as (hi, lo) bf16x8 from the split image
template <int NS>
__device__ __forceinline__ void chunk_mfma_x3(const float* sX, const float* sW, int wrow, int xr, int h, int s0,
                                              floatx16& acc) {
    const char* bx = reinterpret_cast<const char*>(sX) + xr * 256;
    const char* bw = reinterpret_cast<const char*>(sW) + wrow * 256;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const int u = 2 * (s0 + i) + h;
        const bf16x8 wh = *reinterpret_cast<const bf16x8*>(bw + ((u ^ (wrow & 15)) << 4));
        const bf16x8 wl = *reinterpret_cast<const bf16x8*>(bw + (((8 + u) ^ (wrow & 15)) << 4));
        const bf16x8 xh = *reinterpret_cast<const bf16x8*>(bx + ((u ^ (xr & 15)) << 4));
        const bf16x8 xl = *reinterpret_cast<const bf16x8*>(bx + (((8 + u) ^ (xr & 15)) << 4));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh, acc, 0, 0, 0);
    }
}

// chunk_mfma_x3 for two 32-row X groups (BM = 128): each W fragment pair feeds both accumulators
template <int NS>
__device__ __forceinline__ void chunk_mfma_x3_2(const float* sX, const float* sW, int wrow, int xr0, int xr1, int h,
                                                floatx16& acc0, floatx16& acc1) {
    const char* bx0 = reinterpret_cast<const char*>(sX) + xr0 * 256;
    const char* bx1 = reinterpret_cast<const char*>(sX) + xr1 * 256;
    const char* bw = reinterpret_cast<const char*>(sW) + wrow * 256;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const int u = 2 * i + h;
        const bf16x8 wh = *reinterpret_cast<const bf16x8*>(bw + ((u ^ (wrow & 15)) << 4));
        const bf16x8 wl = *reinterpret_cast<const bf16x8*>(bw + (((8 + u) ^ (wrow & 15)) << 4));
        const bf16x8 xh0 = *reinterpret_cast<const bf16x8*>(bx0 + ((u ^ (xr0 & 15)) << 4));
        const bf16x8 xl0 = *reinterpret_cast<const bf16x8*>(bx0 + (((8 + u) ^ (xr0 & 15)) << 4));
        const bf16x8 xh1 = *reinterpret_cast<const bf16x8*>(bx1 + ((u ^ (xr1 & 15)) << 4));
        const bf16x8 xl1 = *reinterpret_cast<const bf16x8*>(bx1 + (((8 + u) ^ (xr1 & 15)) << 4));
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh1, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl1, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh1, acc1, 0, 0, 0);
    }
}

// The k-steps of one chunk this wave owns: k-step t contracts chunk channels {t, 32 + t} (lane
// half h supplies channel 32 h + t), t in [8 q0, 8 q0 + 8 NQ) in 16-B units; rows xr0 .. xr0 + 31
template <int NQ>
__device__ __forceinline__ void chunk_mfma(const float* sX, const float* sW, int wrow, int xr, int h, int q0,
                                           floatx16& acc) {
    auto rd = [&](const float* base, int row, int q4) {
        const int lq = 8 * h + q0 + q4;  // logical 16-B chunk
        return *reinterpret_cast<const floatx4*>(&base[row * kBK + ((lq ^ (row & 15)) * 4)]);
    };
    floatx4 wn = rd(sW, wrow, 0), xn = rd(sX, xr, 0);
#pragma unroll
    for (int q4 = 0; q4 < NQ; ++q4) {
        // the next 16-B operands are read before this unit's four MFMAs
        const floatx4 wa = wn, xb = xn;
        if (q4 + 1 < NQ) {
            wn = rd(sW, wrow, q4 + 1);
            xn = rd(sX, xr, q4 + 1);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the MFMAs (no re-sinking)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.x, xb.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.y, xb.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.z, xb.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wa.w, xb.w, acc, 0, 0, 0);
    }
}

// 8 waves = 4 column blocks of 32 x 2. BM = 64: the second index is the row half (each wave one
// 32x32 accumulator over all of K). BM = 32 (grids too small to fill the chip with 64-row
// blocks): the second index is a K half inside every chunk, the halves are summed through LDS
// before the epilogue. Pipeline: LDS ping-pong (one barrier per chunk) and two register stages,
// so chunk t+2's global loads are issued before chunk t's MFMAs and stored to LDS only after
// chunk t+1's; the loop is unrolled by two so every register stage index is static.
template <int BM, bool ATTN, bool X3>
__global__ void __launch_bounds__(kThreads)
linear_f32_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) float sX[2][BM * kBK];
    __shared__ __attribute__((aligned(16))) float sW[2][kBN * kBK];
    __shared__ float sRed[4][BM];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int c = lane & 31, h = lane >> 5;
    const int cb = wid & 3, sel = wid >> 2;  // column block, row half (BM 64) or K half (BM 32)
    // XCD-aware order: ids are dealt (x fastest) round-robin over the 8 XCDs; remapped bijectively so
    // each XCD runs a contiguous range of (row block, column block) pairs with the column blocks of a
    // row block adjacent: the row block's X rows come from that XCD's L2 for all of them instead of
    // being re-fetched once per column block (x-fastest order)
    int mb, nb_;
    {
        const int nwg = gridDim.x * gridDim.y, id = blockIdx.x + blockIdx.y * gridDim.x;
        const int q = nwg / 8, r = nwg % 8, xcd = id % 8;
        const int logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
        mb = logical / gridDim.y;
        nb_ = logical - mb * gridDim.y;
    }
    const int m0 = mb * BM, n0 = nb_ * kBN;
    const int K = a.k1 + a.k2;
    const int nchunks = K / kBK;
    const int wrow = 32 * cb + c;                     // this lane's W row (output column)
    // this lane's X row (BM 128: and xr + 32, the second accumulator's)
    const int xr = BM == 128 ? 64 * sel + c : BM == 64 ? 32 * sel + c : c;
    const int q0 = BM == 32 ? 4 * sel : 0;            // first 16-B unit of the wave's k-steps
    constexpr int NQ = BM == 32 ? 4 : 8;
    static_assert(BM != 128 || (X3 && !ATTN), "128-row blocks: split-bf16 plain linears only");
    const bool gelu_in = a.flags & kGeluIn;  // GELU of the producing layer applied to X on its way to LDS
    const bool relu_in = a.flags & kReluIn;

    floatx16 acc, acc2;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = acc2[r] = 0.f;
    auto mfma_chunk = [&](const float* bx, const float* bw) {
        if constexpr (BM == 128)
            chunk_mfma_x3_2<4>(bx, bw, wrow, xr, xr + 32, h, acc, acc2);
        else if constexpr (X3)  // 4 bf16 k-steps per chunk: all of them (BM 64) or this wave's K half
            chunk_mfma_x3<BM == 64 ? 4 : 2>(bx, bw, wrow, xr, h, BM == 64 ? 0 : 2 * sel, acc);
        else
            chunk_mfma<NQ>(bx, bw, wrow, xr, h, q0, acc);
    };
    Stage<BM> s0, s1;
    AttnRow ar[BM / 32];
    if (ATTN) {
#pragma unroll
        for (int i = 0; i < BM / 32; ++i) {
            const int m = m0 + (tid >> 4) + 32 * i;
            if (m < a.M) attn_row(a, m, ar[i]);
        }
    }
    stage_load<BM, ATTN>(a, m0, n0, K, 0, tid, s0, ar);
    if (nchunks > 1) stage_load<BM, ATTN>(a, m0, n0, K, 1, tid, s1, ar);
    stage_store<BM, X3>(sX[0], sW[0], tid, s0, gelu_in, relu_in);
    __syncthreads();
    for (int ck = 0; ck < nchunks; ck += 2) {
        // even chunk ck (buffer 0); s1 holds chunk ck + 1, s0 is free
        if (ck + 2 < nchunks) stage_load<BM, ATTN>(a, m0, n0, K, ck + 2, tid, s0, ar);
        mfma_chunk(sX[0], sW[0]);
        if (ck + 1 >= nchunks) break;
        stage_store<BM, X3>(sX[1], sW[1], tid, s1, gelu_in, relu_in);
        __syncthreads();
        // odd chunk ck + 1 (buffer 1); s0 holds chunk ck + 2, s1 is free
        if (ck + 3 < nchunks) stage_load<BM, ATTN>(a, m0, n0, K, ck + 3, tid, s1, ar);
        mfma_chunk(sX[1], sW[1]);
        if (ck + 2 >= nchunks) break;
        stage_store<BM, X3>(sX[0], sW[0], tid, s0, gelu_in, relu_in);
        __syncthreads();
    }
    __syncthreads();  // every wave is done with the LDS tiles
    if (BM == 32) {   // sum the two K halves: waves 4..7 hand their accumulators to waves 0..3
        float* park = sW[0] + cb * 16 * 64;
        if (sel == 1) {
#pragma unroll
            for (int r = 0; r < 16; ++r) park[r * 64 + lane] = acc[r];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] += park[r * 64 + lane];
    }
    // BM = 32: waves 4..7 stay (for the barriers below) but store nothing
    const bool active = BM != 32 || sel == 0;

    // acc[r] = Y[row m0 + mr][column n0 + 32 cb + 8 (r >> 2) + 4 h + (r & 3)]. LayerNorm row
    // statistics: the 4 column-block waves of a row group exchange partial sums through sRed.
    // (a lambda: BM = 128 runs it for both accumulators; every wave calls it, so its barriers match)
    const int nb = n0 + 32 * cb + 4 * h;
    auto epilogue = [&](floatx16& y, const int mr) {
    const int m = m0 + mr;
    if (a.flags & kBias) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const floatx4 b = *reinterpret_cast<const floatx4*>(a.bias + nb + 8 * u);
            y[4 * u] += b.x;
            y[4 * u + 1] += b.y;
            y[4 * u + 2] += b.z;
            y[4 * u + 3] += b.w;
        }
    }
    if (a.flags & kGelu) {
#pragma unroll
        for (int r = 0; r < 16; ++r) y[r] = gelu_erf(y[r]);
    }
    if ((a.flags & kResidual) && (a.flags & kResPreLN) && m < a.M) {
        const float* rr = a.res + (size_t)m * a.N + nb;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const floatx4 r = *reinterpret_cast<const floatx4*>(rr + 8 * u);
            y[4 * u] += r.x;
            y[4 * u + 1] += r.y;
            y[4 * u + 2] += r.z;
            y[4 * u + 3] += r.w;
        }
    }
    if (a.flags & kLayerNorm) {  // N == 128: the workgroup holds whole rows
        float s = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) s += y[r];
        s = halves_sum(s);
        if (h == 0 && active) sRed[cb][mr] = s;
        __syncthreads();
        const float mean = (sRed[0][mr] + sRed[1][mr] + sRed[2][mr] + sRed[3][mr]) * (1.0f / kBN);
        __syncthreads();
        float v = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float d = y[r] - mean;
            v += d * d;
        }
        v = halves_sum(v);
        if (h == 0 && active) sRed[cb][mr] = v;
        __syncthreads();
        const float var = (sRed[0][mr] + sRed[1][mr] + sRed[2][mr] + sRed[3][mr]) * (1.0f / kBN);
        const float rstd = rsqrtf(var + a.eps);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const floatx4 g = *reinterpret_cast<const floatx4*>(a.gamma + nb + 8 * u);
            const floatx4 bt = *reinterpret_cast<const floatx4*>(a.beta + nb + 8 * u);
            y[4 * u] = (y[4 * u] - mean) * rstd * g.x + bt.x;
            y[4 * u + 1] = (y[4 * u + 1] - mean) * rstd * g.y + bt.y;
            y[4 * u + 2] = (y[4 * u + 2] - mean) * rstd * g.z + bt.z;
            y[4 * u + 3] = (y[4 * u + 3] - mean) * rstd * g.w + bt.w;
        }
    }
    if (!active || m >= a.M) return;
    if ((a.flags & kSplit) && a.x3_from >= 0 && nb / kBN >= a.x3_from) {
        typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
        const size_t blk = (size_t)(nb / kBN - a.x3_from) * 2;
        __bf16* hi = a.kv_x3 + blk * a.M * kBN + (size_t)m * kBN + nb % kBN;
        __bf16* lo = hi + (size_t)a.M * kBN;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            bf16x4v vh, vl;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                vh[j] = (__bf16)y[4 * u + j];
                vl[j] = (__bf16)(y[4 * u + j] - (float)vh[j]);
            }
            *reinterpret_cast<bf16x4v*>(hi + 8 * u) = vh;
            *reinterpret_cast<bf16x4v*>(lo + 8 * u) = vl;
        }
        return;
    }
    if (a.flags & kOutBf16) {  // bf16 output (same layouts; split_stride in elements)
        typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
        __bf16* ob = reinterpret_cast<__bf16*>(a.out) +
                     ((a.flags & kSplit) ? (size_t)(nb / kBN) * a.split_stride + (size_t)m * kBN + nb % kBN
                                         : (size_t)m * a.N + nb);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            bf16x4v vh;
#pragma unroll
            for (int j = 0; j < 4; ++j) vh[j] = (__bf16)y[4 * u + j];
            *reinterpret_cast<bf16x4v*>(ob + 8 * u) = vh;
        }
        return;
    }
    float* dst;
    int col0;
    if (a.flags & kSplit) {  // column block j of 128 -> its own [M, 128] matrix
        dst = a.out + (size_t)(nb / kBN) * a.split_stride + (size_t)m * kBN;
        col0 = nb % kBN;
    } else {
        dst = a.out + (size_t)m * a.N;
        col0 = nb;
    }
    const float* res = ((a.flags & kResidual) && !(a.flags & kResPreLN)) ? a.res + (size_t)m * a.N : nullptr;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        floatx4 o = {y[4 * u], y[4 * u + 1], y[4 * u + 2], y[4 * u + 3]};
        if (res) o += *reinterpret_cast<const floatx4*>(res + nb + 8 * u);
        *reinterpret_cast<floatx4*>(dst + col0 + 8 * u) = o;
    }
    };
    epilogue(acc, xr);
    if constexpr (BM == 128) epilogue(acc2, xr + 32);
}

}  // namespace linear
}  // namespace tsplat

using namespace tsplat;

static int launch_linear(tsplat::linear::Args a, void* stream_);

extern "C" int tsplat_linear_f32_fwd(const float* x1, int32_t k1, const float* x2, int32_t k2, const float* w,
                                     const float* bias, const float* ln_gamma, const float* ln_beta,
                                     float ln_eps, const float* residual, float* out, int64_t split_stride,
                                     int32_t M, int32_t N, int32_t flags, void* stream_) {
    using namespace tsplat::linear;
    if (!x1 || !w || !out || M <= 0 || N <= 0 || k1 <= 0 || k2 < 0) return TSPLAT_EINVAL;
    if (k1 % kBK || k2 % kBK || N % kBN || (k2 > 0 && !x2)) return TSPLAT_EINVAL;
    if ((flags & (kGeluIn | kReluIn)) && N != kBN) return TSPLAT_EINVAL;  // each X element staged once
    if ((flags & kResPreLN) && !(flags & kResidual)) return TSPLAT_EINVAL;
    if ((flags & kBias) && !bias) return TSPLAT_EINVAL;
    if ((flags & kLayerNorm) && (N != kBN || !ln_gamma || !ln_beta)) return TSPLAT_EINVAL;
    if ((flags & kResidual) && (!residual || (flags & kSplit))) return TSPLAT_EINVAL;
    if ((flags & kSplit) && split_stride < (int64_t)M * kBN) return TSPLAT_EINVAL;
    if ((flags & kXBf16) && (k2 > 0 || ((uintptr_t)x1 & 7))) return TSPLAT_EINVAL;
    if ((flags & kOutBf16) && ((flags & kResidual) || ((uintptr_t)out & 7))) return TSPLAT_EINVAL;
    Args a{x1, x2, w, bias, ln_gamma, ln_beta, residual, out, split_stride, ln_eps, k1, k2, M, N, flags};
    a.po = a.pm = a.pl = nullptr;
    a.kv_x3 = nullptr;
    a.x3_from = -1;
    return launch_linear(a, stream_);
}

// tsplat_linear_f32_fwd's split form with the column blocks from x3_from on written as bf16 hi / lo
// (see Args::kv_x3): the transformer's k / v projections straight into the bf16x3 attention's
// operand layout (no separate split pass). Blocks before x3_from go to out (fp32, split layout).
extern "C" int tsplat_linear_f32_split_x3_fwd(const float* x1, int32_t k1, const float* w, float* out, void* kv_x3,
                                             int32_t M, int32_t N, int32_t x3_from, int32_t flags, void* stream_) {
    using namespace tsplat::linear;
    if (!x1 || !w || !kv_x3 || M <= 0 || N <= 0 || k1 <= 0 || k1 % kBK || N % kBN) return TSPLAT_EINVAL;
    if (x3_from < 0 || x3_from >= N / kBN || (x3_from > 0 && !out)) return TSPLAT_EINVAL;
    if (flags & ~(kBf16x3 | kBias)) return TSPLAT_EINVAL;  // plain projections (the attention's q | k | v)
    if (((uintptr_t)kv_x3) & 7) return TSPLAT_EINVAL;
    Args a{x1, nullptr, w, nullptr, nullptr, nullptr, nullptr, out, (long long)M * kBN, 0.f, k1, 0, M, N,
           flags | kSplit};
    a.po = a.pm = a.pl = nullptr;
    a.kv_x3 = (__bf16*)kv_x3;
    a.x3_from = x3_from;
    return launch_linear(a, stream_);
}

static int launch_linear(tsplat::linear::Args a, void* stream_) {
    using namespace tsplat::linear;
    const int M = a.M, N = a.N, flags = a.flags;
    hipStream_t stream = (hipStream_t)stream_;
    TSPLAT_PROF_BEGIN(prof::kLinear, stream);
    // 64-row blocks when that still fills the 256 CUs, else 32-row blocks with the K halves split
    // over the wave pairs (a 128-column GEMM of 8,192 rows: 256 workgroups)
    const bool tall = (long long)((M + 63) / 64) * (N / kBN) >= 256;
    const dim3 g64((M + 63) / 64, N / kBN), g32((M + 31) / 32, N / kBN);
    // 128-row blocks (each W fragment feeds two accumulators: half the W staging and split work per
    // row) where they still make >= 512 workgroups (C3's 65,536-row layers); TSPLAT_LIN128=0: off
    static const bool lin128 = !getenv("TSPLAT_LIN128") || atoi(getenv("TSPLAT_LIN128")) != 0;
    const bool tall128 = lin128 && (long long)((M + 127) / 128) * (N / kBN) >= 512;
    if ((flags & kBf16x3) && tall128) {
        hipLaunchKernelGGL((linear_f32_kernel<128, false, true>), dim3((M + 127) / 128, N / kBN), dim3(kThreads), 0,
                           stream, a);
    } else if (flags & kBf16x3) {
        if (tall)
            hipLaunchKernelGGL((linear_f32_kernel<64, false, true>), g64, dim3(kThreads), 0, stream, a);
        else
            hipLaunchKernelGGL((linear_f32_kernel<32, false, true>), g32, dim3(kThreads), 0, stream, a);
    } else {
        if (tall)
            hipLaunchKernelGGL((linear_f32_kernel<64, false, false>), g64, dim3(kThreads), 0, stream, a);
        else
            hipLaunchKernelGGL((linear_f32_kernel<32, false, false>), g32, dim3(kThreads), 0, stream, a);
    }
    TSPLAT_PROF_END(prof::kLinear, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int32_t tsplat_win_attn_split(int32_t batch, int32_t height, int32_t width, int32_t key_views,
                                         int32_t splits);

extern "C" int tsplat_linear_f32_attn_merge_fwd(const float* partials, int32_t batch, int32_t height, int32_t width,
                                                int32_t key_views, int32_t splits, int32_t with_shift,
                                                const float* w, const float* ln_gamma, const float* ln_beta,
                                                float ln_eps, const float* residual, float* out, int32_t N,
                                                int32_t flags, void* stream_) {
    using namespace tsplat::linear;
    if (!partials || !w || !out || N <= 0 || N % kBN) return TSPLAT_EINVAL;
    const int ks = tsplat_win_attn_split(batch, height, width, key_views, splits);
    if (ks <= 1 || ks > kMaxSplit) return TSPLAT_EINVAL;
    if (flags & (kSplit | kGeluIn | kXBf16 | kOutBf16)) return TSPLAT_EINVAL;
    if ((flags & kLayerNorm) && (N != kBN || !ln_gamma || !ln_beta)) return TSPLAT_EINVAL;
    if ((flags & kResidual) && !residual) return TSPLAT_EINVAL;
    if (flags & kBias) return TSPLAT_EINVAL;
    const int M = batch * height * width;
    Args a{nullptr, nullptr, w, nullptr, ln_gamma, ln_beta, residual, out, 0, ln_eps, kBN, 0, M, N, flags};
    a.kv_x3 = nullptr;
    a.x3_from = -1;
    a.aks = ks;
    a.aH = height;
    a.aW = width;
    a.aS = splits;
    a.awh = height / splits;
    a.aww = width / splits;
    a.aL = a.awh * a.aww;
    a.ash = with_shift ? a.awh / 2 : 0;
    a.asw = with_shift ? a.aww / 2 : 0;
    const size_t n = (size_t)batch * splits * splits * ks * a.aL;
    a.po = partials;
    a.pm = partials + n * kBN;
    a.pl = a.pm + n;
    hipStream_t stream = (hipStream_t)stream_;
    TSPLAT_PROF_BEGIN(prof::kLinear, stream);
    if (flags & kBf16x3)
        hipLaunchKernelGGL((linear_f32_kernel<32, true, true>), dim3((M + 31) / 32, N / kBN), dim3(kThreads), 0, stream,
                           a);
    else
        hipLaunchKernelGGL((linear_f32_kernel<32, true, false>), dim3((M + 31) / 32, N / kBN), dim3(kThreads), 0,
                           stream, a);
    TSPLAT_PROF_END(prof::kLinear, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
