// Split-bf16 ("bf16x3") GEMM with fused bias / exact-GELU epilogue and split-K partial slabs, for the
// fp32 linears of the C2 step's bf16x3 dense mode that ran on hipBLASLt: DINOv2-B/14's qkv / proj /
// fc1 / fc2 at M = 650 rows (reference src/depth_anything_v2/dinov2_layers/attention.py:70-75,
// mlp.py:33-40; the reference runs them in TF32, src/main.py:15).
//
//   out[s][m][n] = sum over k in split s of x[m][k] w[n][k]   (+ bias[n] in slab 0, GELU if 1 split)
//
// Products as in the other bf16x3 kernels: x = xh + xl, w = wh + wl (hi = bf16(v), lo = bf16(v - hi)),
// x w ~ xh wh + xh wl + xl wh on v_mfma_f32_32x32x16_bf16 with fp32 accumulation (<= 3 * 2^-18
// relative per product; TF32 rounds each operand to 2^-11).
//
// Why a hand-written kernel: hipBLASLt's emulated-xf32 GEMMs raced inside the graphed two-stream
// step, and its exact-fp32 ones take 19-30 us per DINOv2 linear at M = 650
// (11 row blocks: the launch is operand-delivery-bound, not MFMA-bound). Here:
//   * W is split and packed once per weight version (tsplat_gemm_x3_pack) in MFMA A-fragment order
//     [n-tile 32][k-step 16][hi / lo][64 lanes][8 bf16], so a wave's fragment load is one contiguous
//     1-KB read (no LDS, each wave owns its 32 columns);
//   * x is read as fp32 with coalesced float4 rows, split in registers and written to LDS as B
//     fragments [hi / lo][k-step][m-tile][64 lanes][8 bf16] (lane slot XOR-swizzled by the k-step and
//     half so the 16-lane store groups hit 32 distinct banks; the fragment reads stay one
//     conflict-free ds_read_b128);
//   * workgroup = 64 rows x 128 columns, 4 waves (wave w: columns 32 w .. 32 w + 31, both 32-row
//     m-tiles: 6 MFMAs per 16-deep k-step on 4 LDS fragment reads and 2 fragment loads); K in
//     64-deep chunks, x double-buffered in LDS with one barrier per chunk, the chunk after next in
//     flight (x rows in registers, W fragments in a second register set);
//   * split-K: the K chunks are divided over `ksplit` workgroups per tile, each writing its own fp32
//     slab; the consumer (tsplat_residual_ln_slabs_fwd) sums the slabs in order, so the result is
//     deterministic and no atomics are needed;
//   * XCD-aware order: the workgroups of one column block (same W slice) are dealt to one XCD;
//   * the output tile goes through LDS and is stored as whole 512-B rows.
#include "common.h"
#include "prof.h"

namespace tsplat {
namespace gemm3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) f4v* gptr;  // global loads (not flat)

#ifndef TSPLAT_GEMM_WKMAJOR
#define TSPLAT_GEMM_WKMAJOR 1  // packed W k-step-major: a k-step's n-tiles adjacent
#endif
#ifndef TSPLAT_GEMM_SB
#define TSPLAT_GEMM_SB 0
#endif

constexpr int kBM = 64;       // rows per workgroup (2 m-tiles)
constexpr int kBN = 128;      // columns per workgroup (4 waves x 32)
constexpr int kBK = 64;       // K per chunk
constexpr int kSteps = kBK / 16;
#ifndef TSPLAT_GEMM_KG
#define TSPLAT_GEMM_KG 2
#endif
// k-groups: KG sets of 4 waves share each chunk's k-steps (2: two waves per SIMD, each with half the
// chunk's MFMAs, so one wave's LDS / barrier waits overlap the other's MFMAs); summed through LDS
constexpr int KG = TSPLAT_GEMM_KG;
constexpr int kThreads = 256 * KG;
constexpr int kSpw = 4 / KG;      // k-steps per wave and chunk
constexpr int kXr = 4 / KG;       // x float4 per thread and chunk
constexpr int kBufDw = 2 * kSteps * 2 * 64 * 4;  // dwords per x buffer: [hl][step][mt][lane][4 dw] = 4096
constexpr int kOutStride = kBN + 4;             // floats per row of the output tile in LDS
constexpr int kSmemDw = kBM * kOutStride > 2 * kBufDw ? kBM * kOutStride : 2 * kBufDw;

__device__ float4 g_zero16 = {0.f, 0.f, 0.f, 0.f};

#ifndef TSPLAT_GEMM_STAMP
#define TSPLAT_GEMM_STAMP 0  // diagnostic builds only: per-workgroup phase clocks (tools/gemm_stamps.py)
#endif
#if TSPLAT_GEMM_STAMP
__device__ unsigned long long* g_gemm_stamps = nullptr;
#define G_STAMP(slot)                                                                             \
    do {                                                                                          \
        if (threadIdx.x == 0 && g_gemm_stamps) g_gemm_stamps[(size_t)blockIdx.x * 8 + (slot)] = wall_clock64(); \
    } while (0)
#else
#define G_STAMP(slot) do {} while (0)
#endif

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((floatx2){a, b}, bf16x2));
}

// hi / lo bf16 halves of (a, b), each pair packed into one dword (a in the low half)
__device__ __forceinline__ void split_pair(float a, float b, uint32_t& hi, uint32_t& lo) {
    hi = pack_bf16(a, b);
    const float ah = __builtin_bit_cast(float, hi << 16), bh = __builtin_bit_cast(float, hi & 0xffff0000u);
    lo = pack_bf16(a - ah, b - bh);
}

// GELU with erf from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7 absolute, branch-free: one
// reciprocal, one exp2, five FMAs): the device library's erff (ranges, branches) made fc1's epilogue
// 4.8 of its 23.5 us (tools/gemm_stamps.py). The difference to the exact erf is below the bf16x3
// products' own rounding (~4e-6 relative).
__device__ __forceinline__ float gelu_erf(float v) {
    const float z = fabsf(v) * 0.70710678118654752f;
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
    float p = fmaf(1.061405429f, t, -1.453152027f);
    p = fmaf(p, t, 1.421413741f);
    p = fmaf(p, t, -0.284496736f);
    p = fmaf(p, t, 0.254829592f);
    const float e = 1.0f - p * t * __builtin_amdgcn_exp2f(-z * z * 1.44269504088896341f);
    return 0.5f * v * (1.0f + copysignf(e, v));
}

// W [n][k] fp32 -> [kcp][ntp][hl][64 lanes][8 bf16] (TSPLAT_GEMM_WKMAJOR; 0: [ntp][kcp][...]): lane (n & 31) + 32 ((k >> 3) & 1), element k & 7;
// rows n >= N and columns k >= K are zeros. One thread per (row, 8 consecutive k).
__global__ void __launch_bounds__(256) pack_kernel(const float* __restrict__ w, uint4* __restrict__ wp, int n_rows,
                                                   int k_cols, int ntp, int kcp) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long groups = 2LL * kcp;  // 8-wide k groups per row
    if (idx >= (long long)ntp * 32 * groups) return;
    const int n = (int)(idx / groups), g = (int)(idx % groups);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = 8 * g + j;
        v[j] = (n < n_rows && k < k_cols) ? w[(size_t)n * k_cols + k] : 0.0f;
    }
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) split_pair(v[2 * j], v[2 * j + 1], hi[j], lo[j]);
    const int kc = g >> 1, lane = (n & 31) + 32 * (g & 1);
#if TSPLAT_GEMM_WKMAJOR
    const size_t base = ((size_t)kc * ntp + (n >> 5)) * 128 + lane;
#else
    const size_t base = ((size_t)(n >> 5) * kcp + kc) * 128 + lane;
#endif
    wp[base] = make_uint4(hi[0], hi[1], hi[2], hi[3]);
    wp[base + 64] = make_uint4(lo[0], lo[1], lo[2], lo[3]);
}

struct Args {
    const float* x;    // [m][k] fp32, rows contiguous
    const uint4* w;    // packed W
    const float* bias; // [n] or null
    float* out;        // [ksplit][m][n]
    int m, n, k;
    int kcp;           // packed k-steps (a multiple of kSteps)
    int ntp;           // packed 32-row n-tiles
    int nchunk;        // K chunks = kcp / kSteps
    int cps;           // chunks per split
    int ksplit, act;
    int mb, nb;        // row / column blocks
};

__global__ void __launch_bounds__(kThreads, 2 / KG) gemm_x3_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) uint32_t smem[kSmemDw];
    // XCD-aware order: logical = (column block, split, row block) with the row block fastest; each XCD
    // takes a contiguous logical range, so the workgroups sharing one W slice share one L2
    G_STAMP(0);
    const int logical = xcd_remap(blockIdx.x, gridDim.x);
    const int mbk = logical % a.mb;
    const int rest = logical / a.mb;
    const int ks = rest % a.ksplit, nbk = rest / a.ksplit;
    const int c0 = ks * a.cps, c1 = min(c0 + a.cps, a.nchunk), nc = c1 - c0;

    const int tid = threadIdx.x, lane = tid & 63, w = (tid >> 6) & 3, g = tid >> 8;
#if TSPLAT_GEMM_WKMAJOR
    const uint4* wb = a.w + (size_t)(nbk * 4 + w) * 128 + lane;
    const size_t wstep = (size_t)a.ntp * 128;  // uint4 per k-step
#else
    const uint4* wb = a.w + (size_t)(nbk * 4 + w) * a.kcp * 128 + lane;
    const size_t wstep = 128;
#endif

    // x staging: thread = (row r0 + 16 KG i, float4 column c4), i < 4 / KG
    const int c4 = tid & 15, r0 = tid >> 4;
    const int st = c4 >> 2, sh = (c4 >> 1) & 1, jh = c4 & 1;
    int xoff[kXr];  // dword offset of this thread's hi pair in a buffer (lo at + kLoDw)
    const float* xrow[kXr];
    bool rok[kXr];
#pragma unroll
    for (int i = 0; i < kXr; ++i) {
        const int r = r0 + 16 * KG * i, gm = mbk * kBM + r;
        rok[i] = gm < a.m;
        xrow[i] = a.x + (size_t)(rok[i] ? gm : 0) * a.k + 4 * c4;
        const int slot = ((r & 31) + 32 * sh) ^ (2 * st + sh);
        xoff[i] = ((st * 2 + (r >> 5)) * 64 + slot) * 4 + 2 * jh;
    }
    constexpr int kLoDw = kSteps * 2 * 64 * 4;  // hl stride in dwords (2048)

    const std::integral_constant<int, 0> I0;
    const std::integral_constant<int, 1> I1;
    float4 xr[2][kXr];  // x rows of two chunks in flight: chunk c in set (c - c0) & 1
    uint4 wr[2][kSpw][2];  // this wave's k-steps g kSpw .. of a chunk
    floatx16 acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[t][e] = 0.0f;

    // unconditional loads (rows past M and columns past K read 16 zero bytes instead): a branch
    // around them would make the waits before the next store vmcnt(0), draining the W prefetch too
    auto gload_x = [&](int c, auto X) {
        const bool kok = c * kBK + 4 * c4 < a.k;
#pragma unroll
        for (int i = 0; i < kXr; ++i) {
            const float* p = rok[i] && kok ? xrow[i] + c * kBK : reinterpret_cast<const float*>(&g_zero16);
            const f4v v = *(gptr)p;
            xr[decltype(X)::value][i] = make_float4(v.x, v.y, v.z, v.w);
        }
    };
    auto gload_w = [&](int c, auto S) {
#pragma unroll
        for (int ss = 0; ss < kSpw; ++ss)
#pragma unroll
            for (int hl = 0; hl < 2; ++hl)
                wr[decltype(S)::value][ss][hl] = wb[((size_t)c * kSteps + g * kSpw + ss) * wstep + hl * 64];
    };
    auto store_x = [&](int buf, auto X) {
        uint32_t* b = smem + buf * kBufDw;
#pragma unroll
        for (int i = 0; i < kXr; ++i) {
            const float4 v = xr[decltype(X)::value][i];
            uint32_t h0, l0, h1, l1;
            split_pair(v.x, v.y, h0, l0);
            split_pair(v.z, v.w, h1, l1);
            *reinterpret_cast<uint2*>(b + xoff[i]) = make_uint2(h0, h1);
            *reinterpret_cast<uint2*>(b + kLoDw + xoff[i]) = make_uint2(l0, l1);
        }
    };
    // fragment reads of k-step s into register set F (the next step's reads are issued before the
    // current step's MFMAs, so only the first read of a chunk waits on LDS latency)
    bf16x8 xf[2][2][2];  // [set][m-tile][hi / lo]
    auto read_frags = [&](const uint32_t* b, int s, auto F) {
        const int slot = lane ^ (2 * s + (lane >> 5));
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const uint32_t* p = b + ((s * 2 + t) * 64 + slot) * 4;
            xf[decltype(F)::value][t][0] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p));
            xf[decltype(F)::value][t][1] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p + kLoDw));
        }
    };
    auto mma = [&](int buf, auto S) {
        const uint32_t* b = smem + buf * kBufDw;
        read_frags(b, g * kSpw, I0);
#pragma unroll
        for (int ss = 0; ss < kSpw; ++ss) {
            if (ss + 1 < kSpw) {
                if (ss & 1) read_frags(b, g * kSpw + ss + 1, I0);
                else read_frags(b, g * kSpw + ss + 1, I1);
            }
#if TSPLAT_GEMM_SB
            __builtin_amdgcn_sched_barrier(0);  // keep the next step's reads ahead of these MFMAs
#endif
            const bf16x8 wh = __builtin_bit_cast(bf16x8, wr[decltype(S)::value][ss][0]);
            const bf16x8 wl = __builtin_bit_cast(bf16x8, wr[decltype(S)::value][ss][1]);
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const bf16x8 xh = (ss & 1) ? xf[1][t][0] : xf[0][t][0];
                const bf16x8 xl = (ss & 1) ? xf[1][t][1] : xf[0][t][1];
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xh, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xl, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xh, acc[t], 0, 0, 0);
            }
        }
    };

    if (nc > 0) {
        // every load is unconditional (chunks past the split's last re-read the last one; their
        // registers are never consumed): a skipped load on one path would turn the waits of the
        // merged paths into vmcnt(0), draining the prefetch before the MFMAs
        const auto cl = [&](int c) { return min(c, c1 - 1); };
        gload_x(c0, I0);
        gload_w(c0, I0);
        gload_x(cl(c0 + 1), I1);
        gload_w(cl(c0 + 1), I1);
        store_x(0, I0);
        gload_x(cl(c0 + 2), I0);
        __syncthreads();
        G_STAMP(1);
        // step it (S = it & 1): MFMAs on x buffer S with W set S; x(it + 1) (loaded two steps ago, set
        // !S) to the other buffer (past the last chunk: a copy nobody reads); then the loads of x(it + 3)
        // into set !S and W(it + 2) into set S. x rows go first so that a store waits only for its own
        // rows and the W of its step.
        auto step = [&](int it, auto S) {
            constexpr int s_ = decltype(S)::value;
            const std::integral_constant<int, 1 - s_> NS;
            mma(s_, S);
            store_x(1 - s_, NS);
            gload_x(cl(c0 + it + 3), NS);
            gload_w(cl(c0 + it + 2), S);
            __syncthreads();
            if (it < 4) G_STAMP(2 + it);
        };
        int it = 0;
        for (; it + 1 < nc; it += 2) {
            step(it, I0);
            step(it + 1, I1);
        }
        if (it < nc) step(it, I0);
    }
    G_STAMP(6);

    // epilogue: accumulators -> LDS tile [64 rows][128 + 4] -> whole rows (+ bias, GELU) to the slab.
    // acc[t][e]: column (n) 32 w + (e & 3) + 8 (e >> 2) + 4 (lane >> 5), row (m) 32 t + (lane & 31)
    float* so = reinterpret_cast<float*>(smem);
    if constexpr (KG == 2) {
        // k-group 1's partial sums -> LDS [w][t][q][lane][4] -> added by k-group 0
        float4* ex = reinterpret_cast<float4*>(smem);
        if (g == 1) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    ex[((w * 2 + t) * 4 + q) * 64 + lane] =
                        make_float4(acc[t][4 * q], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]);
        }
        __syncthreads();
        if (g == 0) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 o = ex[((w * 2 + t) * 4 + q) * 64 + lane];
                    acc[t][4 * q] += o.x;
                    acc[t][4 * q + 1] += o.y;
                    acc[t][4 * q + 2] += o.z;
                    acc[t][4 * q + 3] += o.w;
                }
        }
        __syncthreads();
    }
    if (g == 0)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int mrow = 32 * t + (lane & 31), ncol = 32 * w + 8 * q + 4 * (lane >> 5);
            *reinterpret_cast<float4*>(so + mrow * kOutStride + ncol) =
                make_float4(acc[t][4 * q], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]);
        }
    __syncthreads();
    float* slab = a.out + (size_t)ks * a.m * a.n;
    const bool add_bias = a.bias && ks == 0;
#pragma unroll
    for (int i = 0; i < kBM * kBN / 4 / kThreads; ++i) {
        const int idx = tid + kThreads * i;
        const int mrow = idx >> 5, n4 = idx & 31;
        const int gm = mbk * kBM + mrow, gn = nbk * kBN + 4 * n4;
        if (gm >= a.m || gn >= a.n) continue;
        float4 v = *reinterpret_cast<const float4*>(so + mrow * kOutStride + 4 * n4);
        if (add_bias) {
            const float4 bb = *reinterpret_cast<const float4*>(a.bias + gn);
            v.x += bb.x;
            v.y += bb.y;
            v.z += bb.z;
            v.w += bb.w;
        }
        if (a.act == 1) v = make_float4(gelu_erf(v.x), gelu_erf(v.y), gelu_erf(v.z), gelu_erf(v.w));
        if (a.act == 2) {  // hi / lo bf16 images [m][n] at out and out + m n bf16 (the x3 MHA's operands)
            uint32_t h0, l0, h1, l1;
            split_pair(v.x, v.y, h0, l0);
            split_pair(v.z, v.w, h1, l1);
            uint2* ob = reinterpret_cast<uint2*>(a.out);
            const size_t e4 = ((size_t)gm * a.n + gn) / 4;
            ob[e4] = make_uint2(h0, h1);
            ob[e4 + (size_t)a.m * a.n / 4] = make_uint2(l0, l1);
            continue;
        }
        *reinterpret_cast<float4*>(slab + (size_t)gm * a.n + gn) = v;
    }
    G_STAMP(7);
}

}  // namespace gemm3
}  // namespace tsplat

using namespace tsplat::gemm3;

#if TSPLAT_GEMM_STAMP
extern "C" int tsplat_gemm_stamps(void* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_gemm_stamps), &buf, sizeof(buf)) == hipSuccess ? TSPLAT_OK : TSPLAT_EINVAL;
}
#endif

static void packed_dims(int n, int k, int& ntp, int& kcp) {
    ntp = tsplat::ceil_div(n, kBN) * (kBN / 32);
    kcp = tsplat::ceil_div(k, kBK) * kSteps;
}

extern "C" size_t tsplat_gemm_x3_pack_bytes(int32_t n, int32_t k) {
    if (n <= 0 || k <= 0) return 0;
    int ntp, kcp;
    packed_dims(n, k, ntp, kcp);
    return (size_t)ntp * kcp * 128 * sizeof(uint4);
}

extern "C" int tsplat_gemm_x3_pack(const float* w, void* wp, int32_t n, int32_t k, void* stream_) {
    if (!w || !wp || n <= 0 || k <= 0) return TSPLAT_EINVAL;
    int ntp, kcp;
    packed_dims(n, k, ntp, kcp);
    const long long threads = (long long)ntp * 32 * 2 * kcp;
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream_, w,
                       (uint4*)wp, n, k, ntp, kcp);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_gemm_x3_fwd(const float* x, const void* wp, const float* bias, float* out, int32_t m, int32_t n,
                                  int32_t k, int32_t ksplit, int32_t act, void* stream_) {
    if (!x || !wp || !out || m <= 0 || n <= 0 || k <= 0 || ksplit <= 0) return TSPLAT_EINVAL;
    // float4 rows: k and n multiples of 4, x / bias / out 16-B aligned
    if (k % 4 || n % 4 || ((uintptr_t)x & 15) || ((uintptr_t)out & 15) || (bias && ((uintptr_t)bias & 15)))
        return TSPLAT_EINVAL;
    if (act < 0 || act > 2) return TSPLAT_EINVAL;
    if (act && ksplit > 1) return TSPLAT_EINVAL;  // the activation needs the whole sum
    Args a{};
    a.x = x;
    a.w = (const uint4*)wp;
    a.bias = bias;
    a.out = out;
    a.m = m;
    a.n = n;
    a.k = k;
    packed_dims(n, k, a.ntp, a.kcp);
    a.nchunk = a.kcp / kSteps;
    if (ksplit > a.nchunk) return TSPLAT_EINVAL;
    a.cps = tsplat::ceil_div(a.nchunk, ksplit);
    if ((ksplit - 1) * a.cps >= a.nchunk) return TSPLAT_EINVAL;  // every split gets >= 1 chunk
    a.ksplit = ksplit;
    a.act = act;
    a.mb = tsplat::ceil_div(m, kBM);
    a.nb = tsplat::ceil_div(n, kBN);
    const long long grid = (long long)a.mb * a.nb * ksplit;
    if (grid > 0x7fffffff) return TSPLAT_EINVAL;
    TSPLAT_PROF_BEGIN(tsplat::prof::kGemmX3, (hipStream_t)stream_);
    hipLaunchKernelGGL(gemm_x3_kernel, dim3((unsigned)grid), dim3(kThreads), 0, (hipStream_t)stream_, a);
    TSPLAT_PROF_END(tsplat::prof::kGemmX3, (hipStream_t)stream_);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
