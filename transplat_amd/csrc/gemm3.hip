// Linear layer y = act(x W^T + bias) in split-bf16 ("bf16x3") precision on gfx950, for the fp32
// path's small-M library GEMMs: DINOv2 ViT-B's qkv / proj / fc1 (+ exact GELU) / fc2 at M = 650 rows
// (reference src/depth_anything_v2/dinov2_layers/{attention,mlp}.py, run by the reference in TF32,
// src/main.py:15). hipBLASLt's fp32 kernels reach 40-105 TF on these shapes and its bf16 ones are no
// faster at K' = 3K (profiles/r4/split_gemm.log): an M = 650 problem is a few hundred output tiles.
//
// x [M, K] fp32 is split while it is staged (x = hi + lo, hi = bf16(x), lo = bf16(x - hi)); W is
// packed once per weight version as [N][3K] bf16 = [hi | lo | hi] (tsplat_split_bf16x3 weight order;
// this kernel reads the hi and lo thirds). Each product is hi*hi + hi*lo + lo*hi: three
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation (<= 3 * 2^-18 relative per product).
//
// Workgroup: BM x 64 outputs, BM / 32 x 2 waves, each wave one 32 x 32 tile (MFMA rows = x rows m,
// columns = W rows n, so a lane ends with one output column and 16 rows: every store instruction
// writes 128-B row segments). K in 32-wide chunks through double-buffered LDS: x hi / lo and W hi / lo
// as [row][32 bf16] rows (64 B) with the 16-B chunk index XOR-swizzled by (row >> 2) & 3, so each
// 16-lane group of a ds_read_b128 hits 16 distinct 16-B slots; the next chunk's global loads are in
// registers during the current MFMAs, one barrier per chunk. Epilogue: + bias, exact-erf GELU.
//
// Pipelined form (`linear_pipe_kernel`, N % 128 == 0 and K % 64 == 0: every DINOv2 linear): the first
// form waited a full L2 round trip per 32-deep K step (one chunk of register prefetch). Here a 64 x
// 128 workgroup tile streams K in 64-deep stages through a 3-buffer LDS ring filled by LDS-DMA
// (`global_load_lds_dwordx4`: x as fp32 [64 rows][256 B], W hi / lo as [128 rows][hi 128 B | lo
// 128 B], each 16-B chunk XOR-swizzled by (row & 15) through the per-lane SOURCE address, so the
// ds_read_b128 fragment reads of each 16-lane group hit 16 distinct slots). Two stages are in flight
// while one is consumed (counted vmcnt, raw barriers: a __syncthreads fence would drain the DMA).
// Each wave owns 32 x 64 outputs: per 16-deep k-step it splits its x fragment once (8 fp32 -> hi /
// lo) and runs 6 MFMAs against the two W column tiles.
#include "common.h"

namespace tsplat {
namespace gemm3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kBN = 64;
constexpr int kBK = 32;

__device__ __forceinline__ uint32_t bits(float v) { return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v); }

// byte offset of 16-B chunk c (0..3) of row r in a [row][64 B] tile
__device__ __forceinline__ int swz(int r, int c) { return r * 64 + ((c ^ ((r >> 2) & 3)) << 4); }

template <int BM>
__global__ void __launch_bounds__(BM * 4) linear_kernel(const float* __restrict__ x, const uint4* __restrict__ w3,
                                                         const float* __restrict__ bias, float* __restrict__ y, int M,
                                                         int N, int K, int act) {
    constexpr int NT = BM * 4;          // threads
    constexpr int XL = BM * kBK / 4 / NT;     // float4 x loads per thread and chunk (2)
    constexpr int WL = kBN * kBK * 2 / 8 / NT;  // 16-B W loads (hi + lo) per thread and chunk
    __shared__ __attribute__((aligned(16))) char sX[2][2][BM * 64];   // [buf][hl][row][64 B]
    __shared__ __attribute__((aligned(16))) char sW[2][2][kBN * 64];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * kBN;
    const int nchunks = K / kBK;

    float4 xr[XL];
    uint4 wr[WL];
    auto gload = [&](int ck) {
        const int k0 = ck * kBK;
#pragma unroll
        for (int i = 0; i < XL; ++i) {
            const int idx = tid + NT * i, r = idx >> 3, q = idx & 7;  // row, float4 within the chunk row
            const int m = m0 + r;
            xr[i] = m < M ? *reinterpret_cast<const float4*>(x + (size_t)m * K + k0 + 4 * q)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < WL; ++i) {
            const int idx = tid + NT * i;  // (row, hl, 16-B chunk): 8 per row
            const int r = idx >> 3, hl = (idx >> 2) & 1, c = idx & 3;
            wr[i] = w3[((size_t)(n0 + r) * 3 * K + hl * K + k0) / 8 + c];
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < XL; ++i) {
            const int idx = tid + NT * i, r = idx >> 3, q = idx & 7;
            const float4 v = xr[i];
            const uint32_t h0 = bits(v.x) | (bits(v.y) << 16), h1 = bits(v.z) | (bits(v.w) << 16);
            const float e0 = v.x - __builtin_bit_cast(float, h0 << 16), e1 = v.y - __builtin_bit_cast(float, h0 & 0xffff0000u);
            const float e2 = v.z - __builtin_bit_cast(float, h1 << 16), e3 = v.w - __builtin_bit_cast(float, h1 & 0xffff0000u);
            const int off = swz(r, q >> 1) + (q & 1) * 8;
            *reinterpret_cast<uint2*>(&sX[buf][0][off]) = make_uint2(h0, h1);
            *reinterpret_cast<uint2*>(&sX[buf][1][off]) =
                make_uint2(bits(e0) | (bits(e1) << 16), bits(e2) | (bits(e3) << 16));
        }
#pragma unroll
        for (int i = 0; i < WL; ++i) {
            const int idx = tid + NT * i;
            const int r = idx >> 3, hl = (idx >> 2) & 1, c = idx & 3;
            *reinterpret_cast<uint4*>(&sW[buf][hl][swz(r, c)]) = wr[i];
        }
    };

    floatx16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    const int xrow = 32 * wm + (lane & 31), wrow = 32 * wn + (lane & 31), h = lane >> 5;

    gload(0);
    sstore(0);
    if (nchunks > 1) gload(1);
    __syncthreads();
    for (int ck = 0; ck < nchunks; ++ck) {
        const int buf = ck & 1;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {  // two 16-wide k-steps per chunk: 16-B chunk 2 ks + h
            const int c = 2 * ks + h;
            const bf16x8 xh = *reinterpret_cast<const bf16x8*>(&sX[buf][0][swz(xrow, c)]);
            const bf16x8 xl = *reinterpret_cast<const bf16x8*>(&sX[buf][1][swz(xrow, c)]);
            const bf16x8 wh = *reinterpret_cast<const bf16x8*>(&sW[buf][0][swz(wrow, c)]);
            const bf16x8 wl = *reinterpret_cast<const bf16x8*>(&sW[buf][1][swz(wrow, c)]);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xl, wh, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, wl, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xh, wh, acc, 0, 0, 0);
        }
        if (ck + 1 < nchunks) {
            sstore(buf ^ 1);  // buffer buf ^ 1 was last read in chunk ck - 1, before the last barrier
            if (ck + 2 < nchunks) gload(ck + 2);
            __syncthreads();
        }
    }

    // acc[e]: output row m0 + 32 wm + (e & 3) + 8 (e >> 2) + 4 h, column n0 + 32 wn + (lane & 31)
    const int n = n0 + 32 * wn + (lane & 31);
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int m = m0 + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (m < M) {
            float v = acc[e] + bv;
            if (act == 2) v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
            y[(size_t)m * N + n] = v;
        }
    }
}


// ---------------------------------------------------------------------------------------------
// pipelined form
constexpr int kPM = 64, kPN = 128, kPK = 64;       // workgroup tile, K stage depth
constexpr int kStages = 3;
constexpr int kXBytes = kPM * kPK * 4;             // 16 KB fp32 x stage
constexpr int kWBytes = kPN * kPK * 2 * 2;         // 32 KB W hi + lo stage
constexpr int kStageBytes = kXBytes + kWBytes;
constexpr int kGlds = (kStageBytes / 1024) / 4;    // LDS-DMA instructions per thread and stage (12)

typedef float f4v __attribute__((ext_vector_type(4)));

// (hi, lo) bf16x8 of 8 consecutive fp32 values: hi = bf16(v), lo = bf16(v - hi)
__device__ __forceinline__ void split8(const f4v a, const f4v b, bf16x8& hi, bf16x8& lo) {
    typedef float f8v __attribute__((ext_vector_type(8)));
    const f8v v = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    hi = __builtin_convertvector(v, bf16x8);
    const f8v h = __builtin_convertvector(hi, f8v);
    lo = __builtin_convertvector(v - h, bf16x8);
}

__global__ void __launch_bounds__(256, 1) linear_pipe_kernel(const float* __restrict__ x,
                                                              const __bf16* __restrict__ w3,
                                                              const float* __restrict__ bias, float* __restrict__ y,
                                                              int M, int N, int K, int act) {
    __shared__ __attribute__((aligned(1024))) char smem[kStages * kStageBytes];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int mblocks = (M + kPM - 1) / kPM, nblocks = N / kPN;
    // bijective XCD remap: the dispatcher deals ids round-robin over the 8 XCDs; consecutive
    // logical ids (same W column block) go to one XCD, so each W slice is read once per L2
    const int nwg = mblocks * nblocks, orig = blockIdx.x;
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    const int logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
    const int nb = logical / mblocks, mb = logical - nb * mblocks;
    const int m0 = mb * kPM, n0 = nb * kPN;
    const int nk = K / kPK;

    // LDS-DMA sources of this thread: piece = 1 KB = 4 rows x 256 B, lane (row 4 piece + (lane >> 4),
    // slot lane & 15) takes global chunk (lane & 15) ^ (row & 15)
    const int prow = lane >> 4, slot = lane & 15;
    const float* xsrc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // x pieces wid * 4 + i: rows 4 (4 wid + i) + prow
        const int row = 4 * (4 * wid + i) + prow;
        const int c = slot ^ (row & 15);
        xsrc[i] = x + (size_t)min(m0 + row, M - 1) * K + 4 * c;
    }
    const __bf16* wsrc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // W pieces wid * 8 + i: rows 4 (8 wid + i) + prow
        const int row = 4 * (8 * wid + i) + prow;
        const int c = slot ^ (row & 15);  // 0-7 hi chunks, 8-15 lo chunks
        wsrc[i] = w3 + (size_t)(n0 + row) * 3 * K + (c >> 3) * K + 8 * (c & 7);
    }
    auto issue = [&](int stage) {
        const int ks = min(stage, nk - 1);  // past the end: reload the last stage (unused, keeps counts)
        char* base = smem + (stage % kStages) * kStageBytes;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds(xsrc[i] + ks * kPK, base + (4 * wid + i) * 1024, 16, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            __builtin_amdgcn_global_load_lds(wsrc[i] + ks * kPK, base + kXBytes + (8 * wid + i) * 1024, 16, 0, 0);
    };

    const int wm = wid >> 1, wn = wid & 1, h = lane >> 5;
    const int arow = 32 * wm + (lane & 31);
    int brow[2];
    brow[0] = 64 * wn + (lane & 31);
    brow[1] = brow[0] + 32;
    floatx16 acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;

    issue(0);
    issue(1);
    for (int k = 0; k < nk; ++k) {
        issue(k + 2);
        // stage k landed (the two younger stages may still be in flight); then every wave's part
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kGlds) : "memory");
        __builtin_amdgcn_s_barrier();
        const char* sx = smem + (k % kStages) * kStageBytes;
        const char* sw = sx + kXBytes;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int c0 = 4 * s + 2 * h;
            const f4v a0 = *reinterpret_cast<const f4v*>(sx + arow * 256 + ((c0 ^ (arow & 15)) << 4));
            const f4v a1 = *reinterpret_cast<const f4v*>(sx + arow * 256 + (((c0 + 1) ^ (arow & 15)) << 4));
            bf16x8 ah, al;
            split8(a0, a1, ah, al);
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int n = brow[t], cb = 2 * s + h;
                const bf16x8 bh = *reinterpret_cast<const bf16x8*>(sw + n * 256 + ((cb ^ (n & 15)) << 4));
                const bf16x8 bl = *reinterpret_cast<const bf16x8*>(sw + n * 256 + (((cb + 8) ^ (n & 15)) << 4));
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[t], 0, 0, 0);
            }
        }
        // every wave is done reading buffer k % 3 before iteration k + 1 refills it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's unused reloads

    // acc[t][e]: output row m0 + 32 wm + (e & 3) + 8 (e >> 2) + 4 h, column n0 + brow[t]
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int n = n0 + brow[t];
        const float bv = bias ? bias[n] : 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int m = m0 + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
            if (m < M) {
                float v = acc[t][e] + bv;
                if (act == 2) v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
                y[(size_t)m * N + n] = v;
            }
        }
    }
}
}  // namespace gemm3
}  // namespace tsplat

using namespace tsplat;

extern "C" int tsplat_linear_bf16x3_fwd(const float* x, const void* w_packed, const float* bias, float* y, int32_t M,
                                        int32_t N, int32_t K, int32_t act, void* stream_) {
    using namespace tsplat::gemm3;
    if (!x || !w_packed || !y || M <= 0 || N <= 0 || K <= 0 || N % kBN || K % kBK || (act != 0 && act != 2))
        return TSPLAT_EINVAL;
    hipStream_t stream = (hipStream_t)stream_;
    if (N % kPN == 0 && K % kPK == 0 && !getenv("TSPLAT_LIN3_SIMPLE")) {
        const int wgs = (M + kPM - 1) / kPM * (N / kPN);
        hipLaunchKernelGGL(linear_pipe_kernel, dim3(wgs), dim3(256), 0, stream, x, (const __bf16*)w_packed, bias, y, M,
                           N, K, act);
        TSPLAT_CHECK_LAUNCH();
        return TSPLAT_OK;
    }
    // 64-row blocks while they give >= 256 workgroups, else 32-row blocks (2 waves)
    const long wg64 = (long)((M + 63) / 64) * (N / kBN);
    if (wg64 >= 256)
        hipLaunchKernelGGL(linear_kernel<64>, dim3((M + 63) / 64, N / kBN), dim3(256), 0, stream, x,
                           (const uint4*)w_packed, bias, y, M, N, K, act);
    else
        hipLaunchKernelGGL(linear_kernel<32>, dim3((M + 31) / 32, N / kBN), dim3(128), 0, stream, x,
                           (const uint4*)w_packed, bias, y, M, N, K, act);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
