// 3x3 / stride 1 / pad 1 convolution as Winograd F(2x2, 3x3) on split-bf16 ("bf16x3") MFMA: the
// fp32 dense-layer precision mode of the C2 step (the reference runs these convolutions in TF32,
// src/main.py:15 + cuDNN's default; gfx950 has no xf32 MFMA). Same convolutions as winoconv.hip
// (depth_predictor_trans.py:110-125 heads, ldm_unet/unet.py ResBlocks, the UniMatch CNN 3x3s).
//
// Every fp32 GEMM operand x is split as x = xh + xl (xh = bf16(x), xl = bf16(x - xh); x - xh is
// exact in fp32), and each product as xh yh + xh yl + xl yh -- three v_mfma_f32_32x32x16_bf16 with
// fp32 accumulation. The dropped xl yl term and xl's rounding leave <= 3 * 2^-18 relative per
// product (TF32 rounds each operand to 2^-11), at 3 / 16 of the exact-fp32 MFMA cycles.
//
// Winograd as in winoconv.hip: M[xi][co][t] = sum_ci U[xi][co][ci] V[xi][ci][t], V = B^T d B of the
// 4x4 input patch of output tile t, U = G g G^T (fp32, split once per weight version), y = A^T M A.
// Workgroup: 4 * CB * KS waves; CB 32-channel output blocks x T = 32 * NB output tiles; wave
// (k-group kg, co block hh, transform row r) owns the 4 GEMMs xi = 4 r + s of its co block for all
// NB tile blocks (4 * NB accumulator tiles). Per 16-channel chunk every thread transforms PP
// channel pairs of one tile, splits each V value into hi / lo bf16 and stores the pair as one dword of
//   sV[hl][xi][half 2][tile T][pair 4]   (pair 4 half + p = channels 8 half + 2p, + 1),
// so a B fragment (lane = tile n, half h: channels 8h .. 8h + 7) is one ds_read_b128, and a wave's
// stores (lanes = 16 tiles x 4 pairs) are 64 consecutive dwords. A = the packed U fragment, one
// 16-B load per (xi, hi / lo) and lane.
// Double-buffered sV, one barrier per chunk; the next chunk's patch loads and A fragments are in
// flight during the current MFMAs. KS = 2 splits the chunks of one output block over two k-groups
// (few-workgroup grids of the 32^2-64^2 maps); their Z slabs are summed in the epilogue.
#include <stdlib.h>

#include "common.h"
#include "prof.h"

#ifndef TSPLAT_W3_ABL
#define TSPLAT_W3_ABL 0  // diagnostic ablation builds only (tools/build_ablation_w3.sh)
#endif

namespace tsplat {
namespace wino3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kMaxSrc = 6;
constexpr int kMaxCiPad = 1024;
constexpr int kPersistCiPad = 512;  // the persistent form's plane table (keeps it at 2 workgroups / CU)

// 16 zero bytes every masked load reads instead (loads stay unconditional: a select of the address
// instead of an exec-masked branch with zero-initialised destinations per load)
__device__ uint4 g_zero16 = {0u, 0u, 0u, 0u};

#ifndef TSPLAT_W3_STAMP
#define TSPLAT_W3_STAMP 0  // diagnostic builds only (tools/build_stamp_w3.sh): per-workgroup phase clocks
#endif
#if TSPLAT_W3_STAMP
// [workgroup][8] 100-MHz wall clock at the phase boundaries, written by thread 0 (vector stores)
__device__ unsigned long long* g_w3_stamps = nullptr;
#define W3_STAMP(slot)                                                                                  \
    do {                                                                                                \
        if (threadIdx.x == 0 && g_w3_stamps)                                                            \
            g_w3_stamps[(size_t)(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (slot)] = wall_clock64();   \
    } while (0)
#else
#define W3_STAMP(slot) do {} while (0)
#endif

struct Args {
    const float* src[kMaxSrc];
    int cs[kMaxSrc];
    int nsrc;
    const uint4* u;      // packed U: [16 xi][cobs][nchunk][2 hl][64 lanes][8 bf16]
    const float* bias;   // [co] or null
    float* y;            // [n][co][h][w]
    int n, ci, h, w, co, ci_pad, cobs, nchunk;  // cobs: 32-channel blocks in the packing
    int th, tw, tbx, tby, bx, by;
    int act;             // 0 none, 1 ReLU, 2 GELU (erf)
    int relu_in;         // ReLU applied to the input as it is loaded (a pre-activation unit)
    const float* res;    // [n][co][h][w] added after the activation, or null
    const float* res2;   // a second such addend (the fusion block's skip), or null
    int cob_base;        // first 32-channel output block of this launch
};

__device__ __forceinline__ float act_fn(float v, int act) {
    if (act == 1) return fmaxf(v, 0.0f);
    if (act == 2) return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
    return v;
}

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

// (a, b) rounded to bf16 and packed (a in the low half): one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((floatx2){a, b}, bf16x2));
}

// hi / lo halves of the channel pair (a, b) as two packed dwords (channel a in the low half):
// cvt_pk, shift, and, two subtractions, cvt_pk
__device__ __forceinline__ void split_pair(float a, float b, uint32_t& hi, uint32_t& lo) {
    hi = pack_bf16(a, b);
    const float ah = __builtin_bit_cast(float, hi << 16), bh = __builtin_bit_cast(float, hi & 0xffff0000u);
    lo = pack_bf16(a - ah, b - bh);
}

// U = G g G^T (as winoconv.hip's weight_kernel), split into hi / lo bf16 and packed as the A operand
// of v_mfma_f32_32x32x16_bf16: lane l (co = 32 b + (l & 31), h = l >> 5), element j <- ci = 16 k + 8 h + j
__global__ void __launch_bounds__(256) weight_kernel(const float* __restrict__ g, __bf16* __restrict__ u, int co,
                                                     int ci, int ci_pad, int cobs) {
    const int idx = blockIdx.x * 256 + threadIdx.x;  // over cobs * 32 * ci_pad
    if (idx >= cobs * 32 * ci_pad) return;
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
    const int chunk = c / 16, h = (c >> 3) & 1, j = c & 7;
    const int nchunk = ci_pad / 16;
    const size_t lane = 32 * h + ol;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float uu[4] = {t[r][0], 0.5f * (t[r][0] + t[r][1] + t[r][2]), 0.5f * (t[r][0] - t[r][1] + t[r][2]),
                             t[r][2]};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const size_t base = ((((size_t)(4 * r + s) * cobs + b) * nchunk + chunk) * 2) * 64;
            const __bf16 hi = (__bf16)uu[s];
            const __bf16 lo = (__bf16)(uu[s] - (float)hi);
            u[((base + lane) * 8) + j] = hi;
            u[((base + 64 + lane) * 8) + j] = lo;
        }
    }
}

template <int T>
struct Patch {
    int img, y0, x0;
    bool rok[4], cok[4];

    __device__ __forceinline__ Patch(const Args& a, int blk_linear, int t) {
        const int blocks_per_img = a.bx * a.by;
        img = blk_linear / blocks_per_img;
        const int blk = blk_linear % blocks_per_img;
        const int ty = (blk / a.bx) * a.tby + t / a.tbx, tx = (blk % a.bx) * a.tbx + t % a.tbx;
        const bool tile_ok = ty < a.th && tx < a.tw;
        y0 = 2 * ty - 1;
        x0 = 2 * tx - 1;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            rok[i] = tile_ok && y0 + i >= 0 && y0 + i < a.h;
            cok[i] = x0 + i >= 0 && x0 + i < a.w;
        }
    }

    __device__ __forceinline__ void load(const Args& a, const float* const* planes, int c, float (&d)[16]) const {
#if TSPLAT_W3_ABL == 1  // diagnostic build: no patch loads
#pragma unroll
        for (int i = 0; i < 16; ++i) d[i] = (float)(c + i + x0) * 1e-3f;
        return;
#endif
        const __attribute__((address_space(1))) float* src =
            (const __attribute__((address_space(1))) float*)planes[min(c, a.ci_pad - 1)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool ok = c < a.ci && rok[i] && cok[j];
                d[4 * i + j] = ok ? src[(size_t)(y0 + i) * a.w + (x0 + j)] : 0.0f;
                if (a.relu_in) d[4 * i + j] = fmaxf(d[4 * i + j], 0.0f);
            }
    }
};

// V = B^T d B of the channel pair (da, db) -> hi / lo dwords of every xi into sV (this thread's tile
// and pair; xi stride 8 * T dwords, hl stride 16 * 8 * T)
template <int T>
__device__ __forceinline__ void transform_pair(const float (&da)[16], const float (&db)[16], uint32_t* sV) {
    float ta[16], tb[16];  // B^T d
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        ta[0 + j] = da[0 + j] - da[8 + j];
        ta[4 + j] = da[4 + j] + da[8 + j];
        ta[8 + j] = da[8 + j] - da[4 + j];
        ta[12 + j] = da[4 + j] - da[12 + j];
        tb[0 + j] = db[0 + j] - db[8 + j];
        tb[4 + j] = db[4 + j] + db[8 + j];
        tb[8 + j] = db[8 + j] - db[4 + j];
        tb[12 + j] = db[4 + j] - db[12 + j];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float va[4] = {ta[4 * r] - ta[4 * r + 2], ta[4 * r + 1] + ta[4 * r + 2], ta[4 * r + 2] - ta[4 * r + 1],
                             ta[4 * r + 1] - ta[4 * r + 3]};
        const float vb[4] = {tb[4 * r] - tb[4 * r + 2], tb[4 * r + 1] + tb[4 * r + 2], tb[4 * r + 2] - tb[4 * r + 1],
                             tb[4 * r + 1] - tb[4 * r + 3]};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            uint32_t hi, lo;
            split_pair(va[s], vb[s], hi, lo);
            sV[(4 * r + s) * 8 * T] = hi;
            sV[(16 + 4 * r + s) * 8 * T] = lo;
        }
    }
}

// Staged input (ST): per 16-channel chunk the tile block's input region -- rows 2 ty0 - 1 ..
// 2 (ty0 + TBY), columns from the 16-B-aligned 2 tx0 - 4, TBX / 2 + 2 float4 per row -- is loaded
// with coalesced float4 loads (a chunk ahead, in registers) into an LDS slot sIn[ch][row][col], and
// each thread reads its 4x4 patches from there: ~5 float4 loads per thread and chunk instead of 32
// predicated scalar ones (the map width must be a multiple of 4 and the sources 16-B aligned).
// sIn holds [16 channels][R rows][RP floats] with the channel stride padded by 8 floats (CS =
// R RP + 8, R RP being a multiple of 16 for every tile-block shape): a wave's patch reads (16 tiles
// x 4 channel pairs, pair p at channel stride 2 CS) then hit 2 distinct banks per tile column
// instead of one (2-way instead of 4-way conflicts)
template <int T>
struct Region {
    static constexpr int kPad = 8;
    static constexpr int kMaxFloats = T == 32 ? 16 * (4 * 72 + 8) : 16 * (4 * 136 + 8);  // largest [16][CS]
};

template <int CB, int NB, int KS, bool ST>
__global__ void __launch_bounds__(256 * CB * KS, (NB == 1 && CB * KS <= 2) ? 2 : 1) conv_kernel(Args a) {
    constexpr int T = 32 * NB;                 // tiles per workgroup
    constexpr int GT = 256 * CB;               // threads per k-group
    constexpr int PHR = GT / (4 * T);          // pair halves (4 pairs each) covered per pass
    constexpr int PP = PHR > 2 ? 1 : 2 / PHR;  // channel pairs per thread per chunk
    // more threads than channel pairs x tiles (64 co x 32 tiles): the waves of pair halves >= 2
    // skip the transform and only load, stage and multiply (their SIMDs' VALU goes to the others)
    constexpr bool XT = PHR > 2;
    static_assert(XT || PHR * PP == 2, "pairs per chunk");
    constexpr int BUF = 2 * 16 * 8 * T;        // dwords per sV buffer (hi + lo)
    constexpr int CO = 32 * CB;
    constexpr int NSV = ST ? 1 : 2;            // sV buffers per k-group
    constexpr int RGN = Region<T>::kMaxFloats; // floats per sIn slot
    // float4 region loads per thread and chunk: the largest R x C4 (72 for 32-tile blocks, 136 for
    // 64-tile ones) over the GT / 16 threads of a channel
    constexpr int NL = ((T == 32 ? 72 : 136) + GT / 16 - 1) / (GT / 16);
    // the pipeline's buffers, reused for the Z slabs after the last chunk (the larger of the two)
    constexpr int SMEM_PIPE = KS * (NSV * BUF + (ST ? 2 * RGN : 0));
    constexpr int SMEM = SMEM_PIPE > 8 * CO * T * KS ? SMEM_PIPE : 8 * CO * T * KS;
    __shared__ __attribute__((aligned(16))) uint32_t smem[SMEM];
    __shared__ const float* planes[kMaxCiPad];

    W3_STAMP(0);
    // XCD-aware order: the dispatcher deals workgroup ids (x fastest) round-robin over the 8 XCDs.
    // The bijective remap gives each XCD a contiguous range of (tile block, output block) pairs with
    // the output blocks of one tile block adjacent, so a tile block's input regions are fetched into
    // that XCD's L2 once for all its output blocks (x-fastest order re-read the whole input map from
    // HBM / MALL once per output block: 673 MB fetched for the 85 MB input of 2 x 163 -> 168 at 256^2,
    // profiles/r4/traffic_wino3_163x168_b1.json)
    int tbk, cbk;
    {
        const int nwg = gridDim.x * gridDim.y, id = blockIdx.x + blockIdx.y * gridDim.x;
        const int q = nwg / 8, r = nwg % 8, xcd = id % 8;
        const int logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
        tbk = logical / gridDim.y;
        cbk = logical - tbk * gridDim.y;
    }
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int kg = wid / (4 * CB), wg = wid % (4 * CB);
    const int hh = wg >> 2, rr = wg & 3;
    // transform slot: lane bits 0-1 = pair within a half (pl), then the tile, then the half (ph):
    // a wave's 64 lanes are 16 tiles x 4 pairs, so its sV dword stores are 64 consecutive dwords
    const int gtid = tid % GT;
    const int pl = gtid & 3, t = (gtid >> 2) % T, ph0 = (gtid >> 2) / T;
    const bool xf = !XT || ph0 < 2;  // this thread transforms (wave-uniform: a wave is 16 tiles of one ph0)
    const Patch<T> pt(a, tbk, t);

    for (int c = tid; c < a.ci_pad; c += 256 * CB * KS) {
        const float* src = nullptr;
        int rem = min(c, a.ci - 1);
        for (int q = 0; q < a.nsrc && !src; ++q) {
            if (rem < a.cs[q])
                src = a.src[q] + ((size_t)pt.img * a.cs[q] + rem) * ((size_t)a.h * a.w);
            else
                rem -= a.cs[q];
        }
        planes[c] = src;
    }
    __syncthreads();

    const int cob = a.cob_base + cbk * CB + hh;
    const bool co_ok = cob < a.cobs;
    // A fragments: [xi][cob][chunk][hl][lane] uint4
    const uint4* ub = a.u + ((size_t)(4 * rr) * a.cobs + (co_ok ? cob : 0)) * a.nchunk * 128 + lane;
    const size_t xi_stride = (size_t)a.cobs * a.nchunk * 128;
    uint4 af[4][2];
    // unconditional loads (a chunk past the last reads the last one's weights again: its B operand is
    // all zeros): a branch around them would make every later wait a vmcnt(0), draining the region
    // prefetch before the MFMAs
    auto load_a = [&](int chunk, int s0, int s1) {
        const size_t cofs = (size_t)min(chunk, a.nchunk - 1) * 128;
#pragma unroll
        for (int s = s0; s < s1; ++s)
#pragma unroll
            for (int hl = 0; hl < 2; ++hl) {
#if TSPLAT_W3_ABL == 3  // diagnostic build: no A loads
                af[s][hl] = make_uint4(chunk, s, hl, lane);
#else
                af[s][hl] = ub[s * xi_stride + cofs + hl * 64];
#endif
            }
    };

    floatx16 acc[4][NB];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[s][nb][e] = 0.0f;

    float d[PP][2][16];
    auto load_patches = [&](int chunk) {
        if (!xf) return;
#pragma unroll
        for (int q = 0; q < PP; ++q) {
            const int c0 = chunk * 16 + 2 * (4 * (ph0 + q * PHR) + pl);
            pt.load(a, planes, c0, d[q][0]);
            pt.load(a, planes, c0 + 1, d[q][1]);
        }
    };
    uint32_t* sG = smem + kg * (NSV * BUF + (ST ? 2 * RGN : 0));
    auto transform = [&](uint32_t* sV) {
        if (!xf) return;
#pragma unroll
        for (int q = 0; q < PP; ++q) transform_pair<T>(d[q][0], d[q][1], sV + ((ph0 + q * PHR) * T + t) * 4 + pl);
    };
    // staged region of the chunk: R rows x C4 float4 per channel, origin (ry0, rx0)
    const int blk = tbk % (a.bx * a.by);
    const int R = 2 * a.tby + 2, C4 = a.tbx / 2 + 2, RP = 4 * C4;
    const int ry0 = 2 * (blk / a.bx) * a.tby - 1, rx0 = 2 * (blk % a.bx) * a.tbx - 4;
    float* sIn = reinterpret_cast<float*>(sG + NSV * BUF);
    // DS: two register sets for the region loads (the 32-co forms have the registers): the loads of
    // chunk it + 3 are issued at iteration it and stored at it + 2, a whole iteration in flight
    // (tried and reverted: computing the next chunk's transform beside the MFMAs in registers,
    // sched_barrier-fenced quarters, one register set -- census 1695 vs 1637 us, C2 397.4 / 397.8 vs
    // 399.4 / 401.0 views/s, profiles/r4/g15/: the loop is bound by its VALU + LDS issue, not by the
    // phase order)
    constexpr bool DS = ST && CB == 1 && NB == 1;
    float4 gr[DS ? 2 : 1][ST ? NL : 1];
    // region loads: thread gtid stages channel gch = gtid / TPC of the chunk (one plane pointer per
    // chunk) and its elements j = sub + TPC k of that channel's R x C4 float4 ([row][c4] order). The
    // in-plane offset of element k (-1 outside the map or the region) does not depend on the chunk:
    // decomposed once, out of the loop (runtime divisions by C4)
    constexpr int TPC = GT / 16;
    const int gch = gtid / TPC, sub = gtid % TPC;
    int g_code[ST ? NL : 1];
#pragma unroll
    for (int k = 0; k < (ST ? NL : 0); ++k) {
        const int j = sub + TPC * k;
        const int row = j / C4, c4 = j - row * C4;
        const int y = ry0 + row, x = rx0 + 4 * c4;
        const bool ok = j < R * C4 && y >= 0 && y < a.h && x >= 0 && x < a.w;
        g_code[k] = ok ? y * a.w + x : -1;
    }
    // (S: register set, a compile-time constant -- std::integral_constant -- so the arrays stay in VGPRs)
    auto gload = [&](int chunk, auto S) {
        const int c = chunk * 16 + gch;
        // global address space: a plain pointer read from LDS would make these flat loads, which
        // count against the LDS counter too and wait on it
        typedef float f4v __attribute__((ext_vector_type(4)));
        typedef const __attribute__((address_space(1))) f4v* gptr;
        const float* plane = planes[min(c, a.ci_pad - 1)];
        const bool cok = c < a.ci;
#pragma unroll
        for (int k = 0; k < (ST ? NL : 0); ++k) {
            const float* addr = cok && g_code[k] >= 0 ? plane + g_code[k] : reinterpret_cast<const float*>(&g_zero16);
            const f4v v = *(gptr)addr;
            gr[decltype(S)::value][k] = make_float4(v.x, v.y, v.z, v.w);
        }
    };
    auto sstore = [&](int slot, auto S) {
        float4* dst = reinterpret_cast<float4*>(sIn + slot * RGN) + gch * ((R * RP + Region<T>::kPad) / 4);
#pragma unroll
        for (int k = 0; k < (ST ? NL : 0); ++k) {
            const int j = sub + TPC * k;
            float4 v = gr[decltype(S)::value][k];
            if (a.relu_in) v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
            if (j < R * C4) dst[j] = v;  // [ch][row][c4] with the padded channel stride
        }
    };
    auto read_patches = [&](int slot) {  // this thread's PP channel pairs of tile t from sIn
        if (!xf) return;
        const int tyl = t / a.tbx, txl = t - tyl * a.tbx;
        const float* base = sIn + slot * RGN + 2 * tyl * RP + 2 * txl + 3;
#pragma unroll
        for (int q = 0; q < PP; ++q)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const float* b = base + (2 * (4 * (ph0 + q * PHR) + pl) + e) * (R * RP + Region<T>::kPad);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) d[q][e][4 * i + j] = b[i * RP + j];
            }
    };
    // MFMAs of xi s0 .. s1 - 1 on buffer sV: B fragment of lane (n, h) = the 16 B of
    // [hl][xi][half h][tile 32 nb + n][4 pairs] (channels 8 h .. 8 h + 7), one ds_read_b128
    auto mfma = [&](const uint32_t* sV, int s0, int s1) {
#if TSPLAT_W3_ABL == 2  // diagnostic build: no MFMAs (the B reads stay)
        const uint32_t* bq = sV + ((lane >> 5) * T + (lane & 31)) * 4;
        for (int s = s0; s < s1; ++s) acc[s][0][0] += __builtin_bit_cast(float, bq[(4 * rr + s) * 8 * T]);
        return;
#endif
        const uint32_t* bb = sV + ((lane >> 5) * T + (lane & 31)) * 4;
#pragma unroll
        for (int s = s0; s < s1; ++s) {
            const int xi = 4 * rr + s;
            const bf16x8 ah = __builtin_bit_cast(bf16x8, af[s][0]);
            const bf16x8 al = __builtin_bit_cast(bf16x8, af[s][1]);
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) {
                const uint32_t* ph = bb + xi * 8 * T + 32 * nb * 4;
                const bf16x8 bh = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(ph));
                const bf16x8 bl = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(ph + 16 * 8 * T));
                acc[s][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[s][nb], 0, 0, 0);
                acc[s][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[s][nb], 0, 0, 0);
                acc[s][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[s][nb], 0, 0, 0);
            }
        }
    };

    // k-group kg takes chunks kg, kg + KS, ...; every group runs the same iteration count (a chunk
    // past the last one is all zeros) so the groups meet at every barrier
    const int iters = (a.nchunk + KS - 1) / KS;
    const std::integral_constant<int, 0> I0;
    const std::integral_constant<int, DS ? 1 : 0> I1;
    if constexpr (ST) {
        // single sV: store region(it + 1) | transform(it) | loads of region(it + 3) (DS) or it + 2 |
        // barrier | MFMAs(it) | barrier. Region r lives in register set r & 1 (DS) or set 0.
        gload(kg, I0);
        sstore(0, I0);
        gload(kg + KS, I1);
        if (DS) gload(kg + 2 * KS, I0);
        load_a(kg, 0, 4);
        __syncthreads();
        W3_STAMP(1);
        // S = the register set of region it + 1
        auto step = [&](int it, auto S) {
            const int ch = kg + it * KS;
            const bool more = it + 1 < iters;
            // the region of chunk it + 1 (its loads flew during the last iteration(s)) goes to LDS
            // first, so its registers are free again during the transform; slot (it + 1) & 1 was last
            // read by read_patches(it - 1), before the last barrier
            if (more) sstore((it + 1) & 1, S);
            read_patches(it & 1);
            transform(sG);
            // unconditional (past the last chunk: zero-page loads), see load_a
            gload(ch + (DS ? 3 : 2) * KS, S);
            __syncthreads();  // sV(it) complete
            mfma(sG, 0, 4);
            load_a(ch + KS, 0, 4);
            __syncthreads();  // every wave is done with sV(it) and with sIn slot it & 1
        };
        if constexpr (DS) {
            for (int it = 0; it < iters; it += 2) {
                step(it, I1);
                if (it + 1 < iters) step(it + 1, I0);
            }
        } else {
            for (int it = 0; it < iters; ++it) step(it, I0);
        }
    } else {
    load_patches(kg);
    load_a(kg, 0, 4);
    transform(sG);
    if (iters > 1) load_patches(kg + KS);
    __syncthreads();
    for (int it = 0; it < iters; ++it) {
        const int ch = kg + it * KS;
        const uint32_t* sV = sG + (it & 1) * BUF;
        const bool more = it + 1 < iters;
        mfma(sV, 0, 2);
        if (more) load_a(ch + KS, 0, 2);  // the first two xi's registers are free again
        if (more) {
            transform(sG + ((it + 1) & 1) * BUF);
            if (it + 2 < iters) load_patches(ch + 2 * KS);
        }
        mfma(sV, 2, 4);
        if (more) {
            load_a(ch + KS, 2, 4);
            __syncthreads();  // sV(it + 1) complete; every wave is done reading sV(it)
        }
    }
    }
    __syncthreads();  // all MFMAs' LDS reads done: smem becomes Z[kg][r][j][co CO][tile T]
    W3_STAMP(2);
    float* zs = reinterpret_cast<float*>(smem) + kg * (8 * CO * T);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int col = 32 * hh + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
            const int tt = 32 * nb + (lane & 31);
            zs[((rr * 2 + 0) * CO + col) * T + tt] = acc[0][nb][e] + acc[1][nb][e] + acc[2][nb][e];
            zs[((rr * 2 + 1) * CO + col) * T + tt] = acc[1][nb][e] - acc[2][nb][e] - acc[3][nb][e];
        }
    __syncthreads();
    const float* z0 = reinterpret_cast<const float*>(smem);
    if (KS > 1) {
        float* zw = reinterpret_cast<float*>(smem);
        for (int i = tid; i < 8 * CO * T; i += 256 * CB * KS) {
            float z = zw[i];
#pragma unroll
            for (int g2 = 1; g2 < KS; ++g2) z += zw[g2 * (8 * CO * T) + i];
            zw[i] = z;
        }
        __syncthreads();
    }
    const size_t hw = (size_t)a.h * a.w;
    for (int pidx = tid; pidx < CO * T; pidx += 256 * CB * KS) {
        const int col = pidx / T, t2 = pidx % T;
        const int o = (a.cob_base + cbk * CB) * 32 + col;
        const int oty = (blk / a.bx) * a.tby + t2 / a.tbx, otx = (blk % a.bx) * a.tbx + t2 % a.tbx;
        if (o >= a.co || oty >= a.th || otx >= a.tw) continue;
        const float bv = a.bias ? a.bias[o] : 0.0f;
        float z[4][2];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 2; ++j) z[r][j] = z0[((r * 2 + j) * CO + col) * T + t2];
        float* dst = a.y + ((size_t)pt.img * a.co + o) * hw;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int py = 2 * oty + i;
            if (py >= a.h) continue;
            const float y0v = i == 0 ? z[0][0] + z[1][0] + z[2][0] : z[1][0] - z[2][0] - z[3][0];
            const float y1v = i == 0 ? z[0][1] + z[1][1] + z[2][1] : z[1][1] - z[2][1] - z[3][1];
            float r0 = act_fn(y0v + bv, a.act), r1 = act_fn(y1v + bv, a.act);
            const int px = 2 * otx;
            float* p = dst + (size_t)py * a.w + px;
            const size_t off = ((size_t)pt.img * a.co + o) * hw + (size_t)py * a.w + px;
            if (a.res) {
                r0 += a.res[off];
                if (px + 1 < a.w) r1 += a.res[off + 1];
            }
            if (a.res2) {
                r0 += a.res2[off];
                if (px + 1 < a.w) r1 += a.res2[off + 1];
            }
            if (px + 1 < a.w && ((reinterpret_cast<uintptr_t>(p) & 7) == 0)) {
                *reinterpret_cast<float2*>(p) = make_float2(r0, r1);
            } else {
                p[0] = r0;
                if (px + 1 < a.w) p[1] = r1;
            }
        }
    }
    W3_STAMP(3);
}

// Persistent 32 co x 32 tile form for large maps with few input channels (the refine U-Net's
// 32-channel 256^2 levels: 2-4 chunks per output block, so a one-block workgroup was mostly its
// own prologue and epilogue -- region loads, planes, A fragments, Z fold, stores -- at ~12 us per
// workgroup round). Each workgroup walks tile blocks blockIdx.x, + gridDim.x, ... of output block
// blockIdx.y as one flat (block, chunk) sequence: the staged pipeline of conv_kernel<1, 1, 1, true>
// runs straight across block boundaries (the next block's regions load during this block's last
// MFMAs and its epilogue), and each block ends with the Z fold and the stores.
__global__ void __launch_bounds__(256, 2) conv_persist_kernel(Args a, int nblocks) {
    constexpr int T = 32, GT = 256;
    constexpr int BUF = 2 * 16 * 8 * T;
    constexpr int RGN = Region<T>::kMaxFloats;
    constexpr int NL = (72 + 15) / 16;  // float4 region loads per thread (R C4 <= 72 over 16 threads)
    constexpr int CO = 32;
    __shared__ __attribute__((aligned(16))) uint32_t smem[BUF + 2 * RGN];
    __shared__ const float* planes[kPersistCiPad];  // image 0's plane of each input channel
    __shared__ int cstride[kPersistCiPad];           // floats from one image's plane to the next's

    const int tid = threadIdx.x, lane = tid & 63, rr = tid >> 6;
    const int pl = tid & 3, t = (tid >> 2) % T, ph0 = (tid >> 2) / T;  // one channel pair per thread
    const size_t hw = (size_t)a.h * a.w;
    for (int c = tid; c < a.ci_pad; c += GT) {
        const float* src = nullptr;
        int rem = min(c, a.ci - 1), cs = 0;
        for (int q = 0; q < a.nsrc && !src; ++q) {
            if (rem < a.cs[q]) {
                src = a.src[q] + (size_t)rem * hw;
                cs = a.cs[q];
            } else {
                rem -= a.cs[q];
            }
        }
        planes[c] = src;
        cstride[c] = (int)(cs * hw);
    }

    const int cob = a.cob_base + blockIdx.y;
    // the epilogue's bias values (output channel cob * 32 + (tid + GT i) / T), loaded once: a load in
    // the per-block epilogue would wait vmcnt(0), draining the next block's region loads
    float bias_r[CO * T / GT];
#pragma unroll
    for (int i = 0; i < CO * T / GT; ++i) {
        const int o = cob * 32 + (tid + GT * i) / T;
        bias_r[i] = a.bias && o < a.co ? a.bias[o] : 0.0f;
    }
    const uint4* ub = a.u + ((size_t)(4 * rr) * a.cobs + cob) * a.nchunk * 128 + lane;
    const size_t xi_stride = (size_t)a.cobs * a.nchunk * 128;
    uint4 af[4][2];
    auto load_a = [&](int chunk) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int hl = 0; hl < 2; ++hl) af[s][hl] = ub[s * xi_stride + (size_t)chunk * 128 + hl * 64];
    };
    floatx16 acc[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[s][e] = 0.0f;

    const int R = 2 * a.tby + 2, C4 = a.tbx / 2 + 2, RP = 4 * C4;
    const int bpi = a.bx * a.by;  // tile blocks per image
    float* sIn = reinterpret_cast<float*>(smem + BUF);
    // region elements as in conv_kernel: channel gch = tid / 16 of the chunk, elements j = sub + 16 k
    // of its R x C4 float4; block-independent part (row << 12) | c4, -1 past the region
    const int gch = tid >> 4, sub = tid & 15;
    int g_pos[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        const int j = sub + 16 * k;
        const int row = j / C4, c4 = j - row * C4;
        g_pos[k] = j < R * C4 ? (row << 12) | c4 : -1;
    }
    // two register sets: the region of step g + 3 is loaded at step g and stored at step g + 2
    float4 gr[2][NL];
    // region loads of chunk `chunk` of the workgroup's jb-th tile block; origin of the tile block the
    // loads are for, recomputed (scalar divisions) only when it changes
    int o_jb = -1, img = 0, ry0 = 0, rx0 = 0;
    // (valid: a step of this workgroup; past its last one the loads read the zero page -- they stay
    // unconditional, see conv_kernel's load_a. S: register set, a compile-time constant)
    auto gload = [&](int jb, int chunk, bool valid, auto S) {
        if (jb != o_jb) {  // uniform
            const int bl = blockIdx.x + jb * gridDim.x;
            img = bl / bpi;
            const int blk = bl - img * bpi;
            ry0 = 2 * (blk / a.bx) * a.tby - 1;
            rx0 = 2 * (blk % a.bx) * a.tbx - 4;
            o_jb = jb;
        }
        const int c = chunk * 16 + gch;
        const bool cok = valid && c < a.ci;
        const int cc = min(c, a.ci_pad - 1);
        const float* plane = planes[cc] + (size_t)img * cstride[cc];
        typedef float f4v __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            const int code = g_pos[k];
            const int y = ry0 + ((code >> 12) & 4095), x = rx0 + 4 * (code & 4095);
            const bool ok = cok && code >= 0 && y >= 0 && y < a.h && x >= 0 && x < a.w;
            const float* addr = ok ? plane + (size_t)y * a.w + x : reinterpret_cast<const float*>(&g_zero16);
            const f4v v = *(const __attribute__((address_space(1))) f4v*)addr;
            gr[decltype(S)::value][k] = make_float4(v.x, v.y, v.z, v.w);
        }
    };
    auto sstore = [&](int slot, auto S) {
        float4* dst = reinterpret_cast<float4*>(sIn + slot * RGN) + gch * ((R * RP + Region<T>::kPad) / 4);
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            float4 v = gr[decltype(S)::value][k];
            if (a.relu_in) v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
            if (g_pos[k] >= 0) dst[sub + 16 * k] = v;
        }
    };
    float d[2][16];
    auto read_transform = [&](int slot) {
        const int tyl = t / a.tbx, txl = t - tyl * a.tbx;
        const float* base = sIn + slot * RGN + 2 * tyl * RP + 2 * txl + 3;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float* b = base + (2 * (4 * ph0 + pl) + e) * (R * RP + Region<T>::kPad);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) d[e][4 * i + j] = b[i * RP + j];
        }
        transform_pair<T>(d[0], d[1], smem + (ph0 * T + t) * 4 + pl);
    };

    const int nmine = (nblocks - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    const int G = nmine * a.nchunk;  // flat (block, chunk) steps of this workgroup
    if (G <= 0) return;              // uniform: no barrier below is reached by part of the group
    W3_STAMP(0);
    __syncthreads();                 // planes / cstride
    const std::integral_constant<int, 0> I0;
    const std::integral_constant<int, 1> I1;
    gload(0, 0, true, I0);
    sstore(0, I0);
    gload(1 / a.nchunk, 1 % a.nchunk, G > 1, I1);
    gload(2 / a.nchunk, 2 % a.nchunk, G > 2, I0);
    load_a(0);
    __syncthreads();
    W3_STAMP(1);
    int j = 0, c = 0;
    int nj = 3 / a.nchunk, nc = 3 % a.nchunk;  // (block, chunk) of step g + 3
    // S = the register set of step g + 1's region
    auto step = [&](int g, auto S) {
        if (g + 1 < G) sstore((g + 1) & 1, S);
        read_transform(g & 1);
        gload(nj, nc, g + 3 < G, S);
        if (++nc == a.nchunk) {
            nc = 0;
            ++nj;
        }
        __syncthreads();  // sV(g) complete
        const uint32_t* bb = smem + ((lane >> 5) * T + (lane & 31)) * 4;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int xi = 4 * rr + s;
            const bf16x8 ah = __builtin_bit_cast(bf16x8, af[s][0]);
            const bf16x8 al = __builtin_bit_cast(bf16x8, af[s][1]);
            const uint32_t* ph = bb + xi * 8 * T;
            const bf16x8 bh = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(ph));
            const bf16x8 bl = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(ph + 16 * 8 * T));
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[s], 0, 0, 0);
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[s], 0, 0, 0);
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[s], 0, 0, 0);
        }
        load_a(c + 1 < a.nchunk ? c + 1 : 0);  // unconditional (the last step's reload is unused)
        __syncthreads();  // every wave is done with sV(g) and with sIn slot g & 1
        if (++c < a.nchunk) return;
        // block j done: Z = M A through LDS (aliasing sV), then Y = A^T Z + bias (+ act, + residuals)
        if (j == 0) W3_STAMP(2);
        float* zs = reinterpret_cast<float*>(smem);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int col = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5), tt = lane & 31;
            zs[((rr * 2 + 0) * CO + col) * T + tt] = acc[0][e] + acc[1][e] + acc[2][e];
            zs[((rr * 2 + 1) * CO + col) * T + tt] = acc[1][e] - acc[2][e] - acc[3][e];
#pragma unroll
            for (int s = 0; s < 4; ++s) acc[s][e] = 0.0f;
        }
        __syncthreads();
        const int bl = blockIdx.x + j * gridDim.x;
        const int img = bl / bpi, blk = bl - img * bpi;
#pragma unroll
        for (int i = 0; i < CO * T / GT; ++i) {
            const int pidx = tid + GT * i;
            const int col = pidx / T, t2 = pidx % T;
            const int o = cob * 32 + col;
            const int oty = (blk / a.bx) * a.tby + t2 / a.tbx, otx = (blk % a.bx) * a.tbx + t2 % a.tbx;
            if (o >= a.co || oty >= a.th || otx >= a.tw) continue;
            const float bv = bias_r[i];
            float z[4][2];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int q = 0; q < 2; ++q) z[r][q] = zs[((r * 2 + q) * CO + col) * T + t2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int py = 2 * oty + i;
                if (py >= a.h) continue;
                const float y0v = i == 0 ? z[0][0] + z[1][0] + z[2][0] : z[1][0] - z[2][0] - z[3][0];
                const float y1v = i == 0 ? z[0][1] + z[1][1] + z[2][1] : z[1][1] - z[2][1] - z[3][1];
                float r0 = act_fn(y0v + bv, a.act), r1 = act_fn(y1v + bv, a.act);
                const int px = 2 * otx;
                const size_t off = ((size_t)img * a.co + o) * hw + (size_t)py * a.w + px;
                if (a.res) {
                    r0 += a.res[off];
                    if (px + 1 < a.w) r1 += a.res[off + 1];
                }
                if (a.res2) {
                    r0 += a.res2[off];
                    if (px + 1 < a.w) r1 += a.res2[off + 1];
                }
                float* p = a.y + off;
                if (px + 1 < a.w && ((reinterpret_cast<uintptr_t>(p) & 7) == 0)) {
                    *reinterpret_cast<float2*>(p) = make_float2(r0, r1);
                } else {
                    p[0] = r0;
                    if (px + 1 < a.w) p[1] = r1;
                }
            }
        }
        // Z read before the next block's transform overwrites it: LDS order only, a raw barrier (a
        // __syncthreads fence would wait for this block's output stores, vmcnt(0), and with them for
        // the next block's region loads already in flight)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (j == 0) W3_STAMP(3);
        c = 0;
        ++j;
    };
    for (int g = 0; g < G; g += 2) {
        step(g, I1);
        if (g + 1 < G) step(g + 1, I0);
    }
    W3_STAMP(4);
}

}  // namespace wino3
}  // namespace tsplat

using namespace tsplat;

#if TSPLAT_W3_STAMP
// diagnostic builds only: buffer of [workgroups][8] uint64 the next launches stamp (null = off)
extern "C" int tsplat_wino3_stamps(void* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(wino3::g_w3_stamps), &buf, sizeof(buf)) == hipSuccess ? TSPLAT_OK
                                                                                             : TSPLAT_EINVAL;
}
#endif

static int wino3_ci_pad(int ci) { return (ci + 15) / 16 * 16; }
static int wino3_cobs(int co) { return (co + 63) / 64 * 2; }

extern "C" size_t tsplat_wino_weight_bf16x3_bytes(int32_t co, int32_t ci) {
    if (co <= 0 || ci <= 0) return 0;
    return (size_t)16 * wino3_cobs(co) * wino3_ci_pad(ci) * 32 * 2 * 2;  // hi + lo bf16
}

extern "C" int tsplat_wino_weight_bf16x3(const float* weight, void* packed, int32_t co, int32_t ci, void* stream_) {
    if (!weight || !packed || co <= 0 || ci <= 0) return TSPLAT_EINVAL;
    const int ci_pad = wino3_ci_pad(ci);
    const int cobs = wino3_cobs(co);
    const int total = cobs * 32 * ci_pad;
    hipLaunchKernelGGL(wino3::weight_kernel, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream_, weight,
                       (__bf16*)packed, co, ci, ci_pad, cobs);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

// workgroup forms: 0 = auto, 1 = 32 co x 32 tiles (KS 1), 2 = 32 x 32 with two k-groups,
// 3 = 32 co x 64 tiles, 4 = 64 co x 64 tiles, 5 = persistent 32 x 32 (staged maps only),
// 6 = 64 co x 32 tiles (half the threads transform); staged input (Region) on top where the map
// allows it. (Round 6, tried and removed: 96 co x 32 tiles, 12 waves, to amortise the input transform
// over more outputs: the waves spilled at 170 registers, 472 vs 242 us for the gaussian head's
// 163 -> 168 at 256^2, profiles/r6/wino3_forms_head.log)
static int pick_form(int n, int th, int tw, int co) {
    if (const char* e = getenv("TSPLAT_WINO3_FORM")) {
        const int f = atoi(e);
        if (f >= 1 && f <= 6) return f;
    }
    // measured per census shape (tools/bench_wino3.py, profiles/r4/g17/bench_wino3.log, XCD-ordered
    // blocks): the 64 x 64 form above 128 workgroups (2 x 128 -> 64 at 144^2, 162 of them: 30.8 vs
    // 38.1 us for 32 x 32; at 128 -- 64 -> 64 at 128^2, 128 -> 256 at 64^2 -- half the CUs idle and
    // 32 x 32 wins), two k-groups where 32 x 32 workgroups would leave CUs idle, else 32 x 32 (the
    // persistent form measured 24.3 vs 23.1 us at 32 -> 32 / 256^2 once blocks were XCD-ordered, and
    // 23.9 vs 23.2 us with both chunks' A fragments held in registers for the whole walk, i.e. the
    // packed-U stream is not what bounds these few-channel maps, profiles/r4/g28; the 32 x 64 form
    // never)
    const long tiles = (long)n * th * tw;
    const int cob32 = (co + 31) / 32;
    const long wg64 = (tiles + 63) / 64 * ((co + 63) / 64);
    const long wg32 = (tiles + 31) / 32 * cob32;
    // 64 x 32 where it makes one or two workgroups per CU of a 64-channel-multiple output
    // (tools/wino3_forms.py, profiles/r5/forms/: 64 -> 64 at 128^2 16.2 vs 17.8 us, 128 -> 128 at 72^2
    // 21.7 vs 24.6, 96 -> 128 at 72^2 18.4 vs 20.6, 128 -> 256 at 64^2 24.3 vs 27.5; at 128 or
    // fewer workgroups and at 324 or more it loses, and at b = 8 everywhere)
    const long wg6 = (tiles + 31) / 32 * ((co + 63) / 64);
    // the persistent 32 x 32 form for 32-channel outputs over >= 2048 tile blocks (b = 8's 128^2 /
    // 256^2 refine U-Net levels, profiles/r5/late/wino3_forms_p5.log: 32 -> 32 at 256^2 141.6 vs 164.7
    // us, 64 -> 32 217.8 vs 250.0, 32 -> 32 at 128^2 39.0 vs 44.1; at b = 1's 1024 blocks it loses,
    // 25.2 vs 23.8); the launcher falls back to form 1 where it does not apply
    static const bool p5 = !getenv("TSPLAT_WINO3_P5") || atoi(getenv("TSPLAT_WINO3_P5")) != 0;  // A/B knob
    if (p5 && co <= 32 && wg32 >= 2048) return 5;
    static const bool f6 = !getenv("TSPLAT_WINO3_F6") || atoi(getenv("TSPLAT_WINO3_F6")) != 0;  // A/B knob
    if (f6 && co % 64 == 0 && wg6 >= 150 && wg6 <= 320) return 6;
    if (co > 32 && wg64 > 128) return 4;
    return wg32 <= 256 ? 2 : 1;
}

template <int CB, int NB, int KS>
static void launch(wino3::Args a, int blocks, bool staged, hipStream_t stream, hipEvent_t start, hipEvent_t stop,
                   int coblocks = -1) {
    if (coblocks < 0) coblocks = (a.co - 32 * a.cob_base + 32 * CB - 1) / (32 * CB);
    if (staged)
        hipExtLaunchKernelGGL((wino3::conv_kernel<CB, NB, KS, true>), dim3(blocks, coblocks), dim3(256 * CB * KS), 0,
                              stream, start, stop, 0, a);
    else
        hipExtLaunchKernelGGL((wino3::conv_kernel<CB, NB, KS, false>), dim3(blocks, coblocks), dim3(256 * CB * KS),
                              0, stream, start, stop, 0, a);
}

extern "C" int tsplat_conv3x3_wino_bf16x3_ex_fwd(const float* const* srcs, const int32_t* chans, int32_t nsrc,
                                                 const void* packed, const float* bias, const float* residual,
                                                 const float* residual2, float* y, int32_t n, int32_t h, int32_t w,
                                                 int32_t co, int32_t act, int32_t relu_in, void* stream_) {
    if (!srcs || !chans || nsrc <= 0 || nsrc > wino3::kMaxSrc || !packed || !y || n <= 0 || h <= 0 || w <= 0 ||
        co <= 0 || act < 0 || act > 2)
        return TSPLAT_EINVAL;
    wino3::Args a;
    int ci = 0;
    for (int q = 0; q < wino3::kMaxSrc; ++q) {
        a.src[q] = q < nsrc ? srcs[q] : nullptr;
        a.cs[q] = q < nsrc ? chans[q] : 0;
        if (q < nsrc && (!srcs[q] || chans[q] <= 0)) return TSPLAT_EINVAL;
        ci += a.cs[q];
    }
    a.nsrc = nsrc;
    a.u = (const uint4*)packed;
    a.bias = bias;
    a.y = y;
    a.n = n;
    a.ci = ci;
    a.h = h;
    a.w = w;
    a.co = co;
    a.ci_pad = wino3_ci_pad(ci);
    if (a.ci_pad > wino3::kMaxCiPad) return TSPLAT_EINVAL;
    a.cobs = wino3_cobs(co);
    a.nchunk = a.ci_pad / 16;
    a.th = (h + 1) / 2;
    a.tw = (w + 1) / 2;
    a.act = act;
    a.relu_in = relu_in != 0;
    a.res = residual;
    a.res2 = residual2;
    a.cob_base = 0;
    int form = pick_form(n, a.th, a.tw, co);
    // tile block: the widest of T x 1, T/2 x 2, T/4 x 4, T/8 x 8 with the fewest padded tiles; false
    // where the staged region loads' R x C4 <= 72 (32-tile blocks) / 136 (64-tile blocks) fails
    auto geometry = [&](int ttiles) {
        long best = -1;
        for (int tbx = ttiles; tbx >= ttiles / 8; tbx /= 2) {
            const int tby = ttiles / tbx;
            const long padded = (long)((a.tw + tbx - 1) / tbx) * tbx * ((a.th + tby - 1) / tby) * tby;
            if (best < 0 || padded < best) {
                best = padded;
                a.tbx = tbx;
            }
        }
        a.tby = ttiles / a.tbx;
        a.bx = (a.tw + a.tbx - 1) / a.tbx;
        a.by = (a.th + a.tby - 1) / a.tby;
        return (2 * a.tby + 2) * (a.tbx / 2 + 2) <= (ttiles == 32 ? 72 : 136);
    };
    if (!geometry(form == 3 || form == 4 ? 64 : 32)) return TSPLAT_EINVAL;
    const int blocks = n * a.bx * a.by;
    // staged input: float4 rows need a width that is a multiple of 4 and 16-B aligned sources
    bool staged = w % 4 == 0;
    for (int q = 0; q < nsrc; ++q) staged = staged && (reinterpret_cast<uintptr_t>(srcs[q]) & 15) == 0;
    if (const char* e = getenv("TSPLAT_WINO3_STAGE")) staged = staged && atoi(e) != 0;
    if (form == 5 && (!staged || a.ci_pad > wino3::kPersistCiPad)) form = 1;
    hipStream_t stream = (hipStream_t)stream_;
    const prof::ExtEvents ev = prof::ext_events(prof::kWinoConv);
    if (form == 5) {
        // about two workgroups per CU (68 KB of LDS each), each walking its share of the blocks
        int wgs = 512;
        if (const char* e = getenv("TSPLAT_WINO3_PWG")) wgs = std::max(1, atoi(e));
        const int cob32 = (co + 31) / 32;
        const int gx = std::max(1, std::min(blocks, (wgs + cob32 - 1) / cob32));
        hipExtLaunchKernelGGL(wino3::conv_persist_kernel, dim3(gx, cob32), dim3(256), 0, stream, ev.start, ev.stop, 0,
                              a, blocks);
        TSPLAT_CHECK_LAUNCH();
        return TSPLAT_OK;
    }
    // a 64-wide form over an output whose last 64-channel block is at most half used (the gaussian
    // head's 168 -> 84: 44 of 128 columns padding): the full 64-channel blocks on it, the rest as
    // 32 x 32 blocks (TSPLAT_WINO3_TAIL=0: off)
    static const bool tail = !getenv("TSPLAT_WINO3_TAIL") || atoi(getenv("TSPLAT_WINO3_TAIL")) != 0;
    if (form == 4 && tail && co > 64 && co % 64 != 0 && co % 64 <= 32) {
        launch<2, 2, 1>(a, blocks, staged, stream, ev.start, nullptr, co / 64);
        if (!geometry(32)) return TSPLAT_EINVAL;
        a.cob_base = (co / 64) * 2;
        launch<1, 1, 1>(a, n * a.bx * a.by, staged, stream, nullptr, ev.stop, 1);
        TSPLAT_CHECK_LAUNCH();
        return TSPLAT_OK;
    }
    switch (form) {
        case 4: launch<2, 2, 1>(a, blocks, staged, stream, ev.start, ev.stop); break;
        case 6: launch<2, 1, 1>(a, blocks, staged, stream, ev.start, ev.stop); break;
        case 3: launch<1, 2, 1>(a, blocks, staged, stream, ev.start, ev.stop); break;
        case 2: launch<1, 1, 2>(a, blocks, staged, stream, ev.start, ev.stop); break;
        default: launch<1, 1, 1>(a, blocks, staged, stream, ev.start, ev.stop); break;
    }
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_conv3x3_wino_bf16x3_cat_fwd(const float* const* srcs, const int32_t* chans, int32_t nsrc,
                                                  const void* packed, const float* bias, float* y, int32_t n,
                                                  int32_t h, int32_t w, int32_t co, int32_t act, void* stream_) {
    return tsplat_conv3x3_wino_bf16x3_ex_fwd(srcs, chans, nsrc, packed, bias, nullptr, nullptr, y, n, h, w, co, act, 0,
                                             stream_);
}

extern "C" int tsplat_conv3x3_wino_bf16x3_fwd(const float* x, const void* packed, const float* bias, float* y,
                                              int32_t n, int32_t ci, int32_t h, int32_t w, int32_t co, int32_t act,
                                              void* stream_) {
    return tsplat_conv3x3_wino_bf16x3_cat_fwd(&x, &ci, 1, packed, bias, y, n, h, w, co, act, stream_);
}
