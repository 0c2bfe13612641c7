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
// Two workgroup shapes over the same packed filters (one transform row r of 4 GEMMs per wave, 64
// accumulator registers):
//  * conv_kernel (4 waves): 32 output channels x 32 output tiles (2x2 pixels each, a TBY x TBX
//    patch of tiles). Per 8-channel chunk every thread transforms one (tile, channel) patch into a
//    double-buffered LDS image sV[xi][ci][tile] (the next chunk's loads fly during this chunk's
//    MFMAs), one barrier, 16 MFMAs per wave.
//  * conv64_kernel (8 waves): 64 output channels x 32 tiles, so each input transform feeds twice
//    the MFMAs; 16-channel chunks, 32 MFMAs per wave per chunk, and the transform of chunk c + 1
//    is done between the two halves of chunk c's MFMAs (its loads were issued a chunk earlier).
// A = the packed U fragment (float4 loads, prefetched a chunk ahead), B = one LDS float per lane.
// Epilogue: each wave folds its row of M into Z[r][j] = (M A)[r][j], the rows meet in LDS, and
// Y = A^T Z + bias (+ ReLU / GELU) is stored as float2 pixel pairs.
#include <stdlib.h>

#include "common.h"
#include "prof.h"

namespace tsplat {
namespace wino {

constexpr int kThreads = 256;
constexpr int kCoB = 32;     // output channels per workgroup
constexpr int kTiles = 32;   // output tiles per workgroup
constexpr int kCiB = 8;      // channels per chunk of conv_kernel (16 for conv64_kernel)
constexpr int kGroup = 16;   // packed-filter channel group: [xi][co block][group][lane][8 slots]

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kMaxSrc = 6;     // input sources concatenated along channels (read in place)
constexpr int kMaxCiPad = 1024;  // input channels (padded to 16) of one launch

struct Args {
    const float* src[kMaxSrc];  // source s: [n][cs[s]][h][w]; channel c of the conv input is
    int cs[kMaxSrc];            // channel c - (cs[0] + .. + cs[s-1]) of the source it falls in
    int nsrc;
    const float* u;      // packed U: [16][cobs][ci_pad / 16][64 lanes][8 slots]
    const float* bias;   // [co] or null
    float* y;            // [n][co][h][w]
    int n, ci, h, w, co, ci_pad, cobs;  // cobs = 32-channel blocks in the packing (even)
    int th, tw, tbx, tby, bx, by;  // tiles per image, tile-block shape, tile blocks per image row / column
    int act;             // 0 none, 1 ReLU, 2 GELU (erf)
    int cob_base;        // first 32-channel output block of this launch (a split launch's offset)
};

__device__ __forceinline__ float act_fn(float v, int act) {
    if (act == 1) return fmaxf(v, 0.0f);
    if (act == 2) return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
    return v;
}

// U = G g G^T, G = [[1, 0, 0], [1/2, 1/2, 1/2], [1/2, -1/2, 1/2], [0, 0, 1]], packed as the A
// operand of v_mfma_f32_32x32x2_f32: lane l (co = 32 b + (l & 31), k half h = l >> 5) of channel
// group gr holds 8 consecutive floats, slot 4 q + k <- ci = 16 gr + 8 q + 4 h + k, so an 8-channel
// chunk q is one float4 per lane and a 16-channel chunk two. MFMA k-step k of a chunk therefore
// pairs channels 4 h + k (the B operand reads the same rows). Padded co / ci entries are 0.
__device__ __forceinline__ int chunk_row(int h, int k) { return 8 * (k >> 2) + 4 * h + (k & 3); }

__global__ void __launch_bounds__(256) weight_kernel(const float* __restrict__ g, float* __restrict__ u, int co,
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
    const int gr = c / kGroup, rem = c % kGroup;
    const int q = rem >> 3, h = (rem >> 2) & 1, kk = rem & 3;
    const size_t plane = (size_t)cobs * ci_pad * 32;  // floats per xi
    const size_t off = (((size_t)b * (ci_pad / kGroup) + gr) * 64 + 32 * h + ol) * 8 + 4 * q + kk;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float uu[4] = {t[r][0], 0.5f * (t[r][0] + t[r][1] + t[r][2]), 0.5f * (t[r][0] - t[r][1] + t[r][2]),
                             t[r][2]};
#pragma unroll
        for (int s = 0; s < 4; ++s) u[(4 * r + s) * plane + off] = uu[s];
    }
}

// One thread's (tile, channel) transform slot: the 4x4 input patch of output tile tt of the
// workgroup's tile block, for channel cc of every chunk.
struct Patch {
    int img, tt, y0, x0;
    bool rok[4], cok[4];
    size_t hw;

    __device__ __forceinline__ Patch(const Args& a, int blk_linear, int tid) {
        const int blocks_per_img = a.bx * a.by;
        img = blk_linear / blocks_per_img;
        const int blk = blk_linear % blocks_per_img;
        const int ty0 = (blk / a.bx) * a.tby, tx0 = (blk % a.bx) * a.tbx;
        tt = tid % kTiles;
        const int ty = ty0 + tt / a.tbx, tx = tx0 + tt % a.tbx;
        const bool tile_ok = ty < a.th && tx < a.tw;
        y0 = 2 * ty - 1;
        x0 = 2 * tx - 1;
        hw = (size_t)a.h * a.w;
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // per-row / per-column validity (zero padding)
            rok[i] = tile_ok && y0 + i >= 0 && y0 + i < a.h;
            cok[i] = x0 + i >= 0 && x0 + i < a.w;
        }
    }

    // this image's plane of every (padded) input channel, in the source holding it (past ci: the
    // last channel's, never dereferenced); filled once per workgroup, so the per-chunk lookup is one
    // LDS read for concatenated inputs too
    __device__ __forceinline__ void fill_planes(const Args& a, const float** planes, int tid, int nthreads) const {
        for (int c = tid; c < a.ci_pad; c += nthreads) {
            const float* src = nullptr;
            int rem = min(c, a.ci - 1);
            for (int q = 0; q < a.nsrc && !src; ++q) {
                if (rem < a.cs[q])
                    src = a.src[q] + ((size_t)img * a.cs[q] + rem) * hw;
                else
                    rem -= a.cs[q];
            }
            planes[c] = src;
        }
    }

    // input channel c (channels past ci are zero). Loads stay predicated: unconditional loads from
    // clamped addresses with the zero padding applied in the transform measured slower (more
    // registers; 3 -> 2 waves per SIMD for conv_kernel).
    __device__ __forceinline__ void load(const Args& a, const float* const* planes, int c, float (&d)[16]) const {
        // global address space: a pointer read from LDS would otherwise make these flat loads
        const __attribute__((address_space(1))) float* src =
            (const __attribute__((address_space(1))) float*)planes[c];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool ok = c < a.ci && rok[i] && cok[j];
                d[4 * i + j] = ok ? src[(size_t)(y0 + i) * a.w + (x0 + j)] : 0.0f;
            }
    }

    // V = B^T d B into sV[xi][row][tile] (row stride kTiles, xi stride rows * kTiles)
    __device__ __forceinline__ void transform_store(const float (&dd)[16], float* sV, int row, int rows) const {
        float t[16];  // B^T d
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            t[0 + j] = dd[0 + j] - dd[8 + j];
            t[4 + j] = dd[4 + j] + dd[8 + j];
            t[8 + j] = dd[8 + j] - dd[4 + j];
            t[12 + j] = dd[4 + j] - dd[12 + j];
        }
        float* p = sV + row * kTiles + tt;
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // (B^T d) B
            p[(4 * r + 0) * rows * kTiles] = t[4 * r] - t[4 * r + 2];
            p[(4 * r + 1) * rows * kTiles] = t[4 * r + 1] + t[4 * r + 2];
            p[(4 * r + 2) * rows * kTiles] = t[4 * r + 2] - t[4 * r + 1];
            p[(4 * r + 3) * rows * kTiles] = t[4 * r + 1] - t[4 * r + 3];
        }
    }
};

// Z[r][j] = (M A)[r][j] of one wave's transform row r (acc[s] = M[4 r + s]) into
// zs[(r * 2 + j) * 1024 + co * 32 + tile]; C layout of 32x32x2: lane l holds tile l & 31, rows (co)
// (e & 3) + 8 (e >> 2) + 4 (l >> 5).
__device__ __forceinline__ void fold_row(const floatx16 (&acc)[4], float* zs, int r, int lane) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int col = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        zs[((r * 2 + 0) * kCoB + col) * kTiles + (lane & 31)] = acc[0][e] + acc[1][e] + acc[2][e];
        zs[((r * 2 + 1) * kCoB + col) * kTiles + (lane & 31)] = acc[1][e] - acc[2][e] - acc[3][e];
    }
}

// Y = A^T Z + bias (+ act) for output channel o (Z slab zs) and workgroup tile t2
__device__ __forceinline__ void store_tile(const Args& a, const float* zs, int col, int t2, int o, int img,
                                           int blk_linear) {
    const int blk = blk_linear % (a.bx * a.by);
    const int oty = (blk / a.bx) * a.tby + t2 / a.tbx, otx = (blk % a.bx) * a.tbx + t2 % a.tbx;
    if (o >= a.co || oty >= a.th || otx >= a.tw) return;
    const size_t hw = (size_t)a.h * a.w;
    const float bv = a.bias ? a.bias[o] : 0.0f;
    float z[4][2];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 2; ++j) z[r][j] = zs[((r * 2 + j) * kCoB + col) * kTiles + t2];
    float* dst = a.y + ((size_t)img * a.co + o) * hw;
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

// KS k-groups of 4 waves (KS = 2: 8 waves) split the 8-channel chunks of one 32 x 32 output block
// (group g takes chunks g, g + KS, ...; ci_pad / 8 is even, so both groups run the same number of
// iterations and meet at every barrier), each with its own double-buffered sV; their Z slabs are
// summed in the epilogue. For the few-workgroup grids of the 32^2-64^2 maps (one 4-wave workgroup
// per CU otherwise: one wave per SIMD through 16-32 serial chunks).
// XCD-aware (tile block, output block) order: the dispatcher deals workgroup ids (x fastest)
// round-robin over the 8 XCDs; remapped bijectively, each XCD runs a contiguous range of
// (tile block, output block) pairs with the output blocks of one tile block adjacent, so the tile
// block's input patches come from that XCD's L2 for all of them (x-fastest order re-reads the whole
// input once per output block; winoconv3.hip measured 673 -> 211 MB fetched for 163 -> 168 at 256^2)
__device__ __forceinline__ void xcd_tile_order(int& tb, int& cb) {
    const int nwg = gridDim.x * gridDim.y, id = blockIdx.x + blockIdx.y * gridDim.x;
    const int q = nwg / 8, r = nwg % 8, xcd = id % 8;
    const int logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
    tb = logical / gridDim.y;
    cb = logical - tb * gridDim.y;
}

template <int KS>
__global__ void __launch_bounds__(kThreads * KS) conv_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) float smem[KS * 2 * 16 * kCiB * kTiles];  // sV x2 per group, then Z
    __shared__ const float* planes[kMaxCiPad];
    const int kg = threadIdx.x / kThreads, tid = threadIdx.x % kThreads, lane = tid & 63, wid = tid >> 6;
    int tbk, cbk;
    xcd_tile_order(tbk, cbk);
    const int cob = a.cob_base + cbk;  // 32-channel output block
    const Patch pt(a, tbk, tid);
    const int cc = tid / kTiles;  // channel of each chunk this thread transforms
    float d[16];
    pt.fill_planes(a, planes, threadIdx.x, kThreads * KS);
    __syncthreads();

    // A fragments of one chunk for this wave's 4 xi: 8-channel chunk ch = half ch & 1 of group ch >> 1
    const size_t plane = (size_t)a.cobs * a.ci_pad * 32;
    const float* ub = a.u + (size_t)(4 * wid) * plane + (size_t)cob * (a.ci_pad / kGroup) * 512 + lane * 8;
    float4 af[4];
    auto load_a = [&](int chunk, float4 (&f)[4]) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
            f[s] = *reinterpret_cast<const float4*>(ub + s * plane + (size_t)(chunk >> 1) * 512 + 4 * (chunk & 1));
    };

    floatx16 acc[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[s][r] = 0.0f;

    const int nchunks = a.ci_pad / kCiB;  // even
    float* sG = smem + kg * (2 * 16 * kCiB * kTiles);
    pt.load(a, planes, kg * kCiB + cc, d);
    load_a(kg, af);
    for (int it = 0, ch = kg; ch < nchunks; ++it, ch += KS) {
        float* sV = sG + (it & 1) * (16 * kCiB * kTiles);
        pt.transform_store(d, sV, cc, kCiB);
        __syncthreads();  // sV(ch) complete; every wave is done with this buffer's previous chunk
        float4 an[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) an[s] = af[s];
        if (ch + KS < nchunks) {  // the next chunk's loads fly during this chunk's MFMAs
            pt.load(a, planes, (ch + KS) * kCiB + cc, d);
            load_a(ch + KS, af);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            // k-step k: lane half h reads channel row 4 h + k
            const float* bsrc = sV + ((4 * wid + s) * kCiB) * kTiles + (lane & 31) + 4 * kTiles * (lane >> 5);
            const float av[4] = {an[s].x, an[s].y, an[s].z, an[s].w};
#pragma unroll
            for (int k = 0; k < 4; ++k)
                acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[k], bsrc[k * kTiles], acc[s], 0, 0, 0);
        }
    }
    __syncthreads();  // all MFMAs' LDS reads done: smem becomes Z[group][r][j][co 32][tile 32]
    fold_row(acc, smem + kg * (8 * kCoB * kTiles), wid, lane);
    __syncthreads();
    if (KS > 1) {  // sum the groups' slabs into slab 0
        for (int i = threadIdx.x; i < 8 * kCoB * kTiles; i += kThreads * KS) {
            float z = smem[i];
#pragma unroll
            for (int g = 1; g < KS; ++g) z += smem[g * (8 * kCoB * kTiles) + i];
            smem[i] = z;
        }
        __syncthreads();
    }
    for (int pidx = threadIdx.x; pidx < kCoB * kTiles; pidx += kThreads * KS) {
        const int col = pidx / kTiles;
        store_tile(a, smem, col, pidx % kTiles, cob * kCoB + col, pt.img, tbk);
    }
}

// 8 waves: wave w = (co half hh = w >> 2, transform row r = w & 3); 16-channel chunks, thread tid
// transforms channel tid / 32 of each chunk (one patch). Per chunk c: A(c + 1) prefetch, MFMA
// k-steps 0..3, transform of patch c + 1 into the other sV buffer and the loads of patch c + 2,
// MFMA k-steps 4..7, one barrier.
constexpr int kThreads64 = 512;
constexpr int kCiB64 = 16;

__global__ void __launch_bounds__(kThreads64) conv64_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) float smem[2 * 16 * kCiB64 * kTiles];  // sV x2 (64 KB), then Z
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int hh = wid >> 2, rr = wid & 3;
    int tbk, cbk;
    xcd_tile_order(tbk, cbk);
    const int cob = cbk;  // 64-channel block = 32-channel blocks cob_base + 2 cob (+ 1)
    __shared__ const float* planes[kMaxCiPad];
    const Patch pt(a, tbk, tid);
    const int cc = tid / kTiles;
    float d[16];
    pt.fill_planes(a, planes, tid, kThreads64);
    __syncthreads();

    const size_t plane = (size_t)a.cobs * a.ci_pad * 32;
    const float* ub =
        a.u + (size_t)(4 * rr) * plane + (size_t)(a.cob_base + 2 * cob + hh) * (a.ci_pad / kGroup) * 512 + lane * 8;
    auto load_a = [&](int chunk, float4 (&f)[4][2]) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int q = 0; q < 2; ++q)
                f[s][q] = *reinterpret_cast<const float4*>(ub + s * plane + (size_t)chunk * 512 + 4 * q);
    };

    floatx16 acc[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[s][r] = 0.0f;

    // k-steps [q * 4, q * 4 + 4) of chunk ch (lane half h reads channel row chunk_row(h, k))
    auto mfma_half = [&](const float* sV, const float4 (&f)[4][2], int q) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const float* bsrc = sV + ((4 * rr + s) * kCiB64 + chunk_row(lane >> 5, 4 * q + k)) * kTiles + (lane & 31);
                const float av = k == 0 ? f[s][q].x : k == 1 ? f[s][q].y : k == 2 ? f[s][q].z : f[s][q].w;
                acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, *bsrc, acc[s], 0, 0, 0);
            }
    };

    const int nchunks = a.ci_pad / kCiB64;
    auto step = [&](int ch, const float4 (&cur)[4][2], float4 (&nxt)[4][2]) {
        const float* sV = smem + (ch & 1) * (16 * kCiB64 * kTiles);
        float* sN = smem + ((ch + 1) & 1) * (16 * kCiB64 * kTiles);
        const bool more = ch + 1 < nchunks;
        if (more) load_a(ch + 1, nxt);
        mfma_half(sV, cur, 0);
        if (more) {
            pt.transform_store(d, sN, cc, kCiB64);
            if (ch + 2 < nchunks) pt.load(a, planes, (ch + 2) * kCiB64 + cc, d);
        }
        mfma_half(sV, cur, 1);
        if (more) __syncthreads();  // sV(ch + 1) complete; every wave is done reading sV(ch)
    };
    float4 af[4][2], af2[4][2];
    pt.load(a, planes, cc, d);
    load_a(0, af);
    pt.transform_store(d, smem, cc, kCiB64);
    if (nchunks > 1) pt.load(a, planes, kCiB64 + cc, d);
    __syncthreads();
    for (int ch = 0; ch < nchunks; ch += 2) {
        step(ch, af, af2);
        if (ch + 1 < nchunks) step(ch + 1, af2, af);
    }
    __syncthreads();  // all MFMAs' LDS reads done: smem becomes Z[hh][r][j][co 32][tile 32]
    fold_row(acc, smem + hh * (8 * kCoB * kTiles), rr, lane);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < (2 * kCoB * kTiles) / kThreads64; ++k) {
        const int pidx = tid + kThreads64 * k;
        const int colg = pidx / kTiles;  // 0..63
        store_tile(a, smem + (colg >> 5) * (8 * kCoB * kTiles), colg & 31, pidx % kTiles,
                   a.cob_base * kCoB + cob * 64 + colg, pt.img,
                   tbk);
    }
}

}  // namespace wino
}  // namespace tsplat

using namespace tsplat;

// input channels are padded to the 16-channel group, output channels to 64 (an even number of
// 32-channel blocks, so both workgroup shapes read the same packing)
static int wino_ci_pad(int ci) { return (ci + wino::kGroup - 1) / wino::kGroup * wino::kGroup; }
static int wino_cobs(int co) { return (co + 63) / 64 * 2; }

extern "C" size_t tsplat_wino_weight_floats(int32_t co, int32_t ci) {
    if (co <= 0 || ci <= 0) return 0;
    return (size_t)16 * wino_cobs(co) * wino_ci_pad(ci) * 32;
}

extern "C" int tsplat_wino_weight_f32(const float* weight, float* packed, int32_t co, int32_t ci, void* stream_) {
    if (!weight || !packed || co <= 0 || ci <= 0) return TSPLAT_EINVAL;
    const int ci_pad = wino_ci_pad(ci);
    const int cob = wino_cobs(co);
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
    if (a.ci_pad > wino::kMaxCiPad) return TSPLAT_EINVAL;
    a.cobs = wino_cobs(co);
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
    const prof::ExtEvents ev = prof::ext_events(prof::kWinoConv);  // kernel timestamps when timed
    // 64-channel workgroups where they pad no more output channels than 32-channel ones and the
    // grid still covers most of the 256 CUs (measured per shape with tools/bench_wino.py: at 128
    // workgroups the 32-channel grid's 256 is faster, from 160 up the 64-channel one);
    // TSPLAT_WINO_WG=32 / 64 forces one shape.
    const int blocks = n * a.bx * a.by;
    const int cob32 = (co + wino::kCoB - 1) / wino::kCoB, cob64 = (co + 63) / 64;
    bool wide = cob32 % 2 == 0 && blocks * cob64 >= 160;
    // an odd number of 32-channel blocks on a big grid (168 -> 84 at 256^2): the even part as
    // 64-channel workgroups, the last block as a second, 32-channel launch
    bool split = cob32 % 2 == 1 && cob32 > 1 && blocks * (cob32 / 2) >= 160;
    if (const char* e = getenv("TSPLAT_WINO_WG")) {
        wide = atoi(e) == 64;
        split = false;
    }
    a.cob_base = 0;
    // 32-channel workgroups: split each block's chunks over two 4-wave groups while the grid alone
    // gives at most one workgroup per CU (TSPLAT_WINO_KS=1 / 2 forces)
    int ks = blocks * cob32 <= 256 ? 2 : 1;
    if (const char* e = getenv("TSPLAT_WINO_KS")) ks = atoi(e) == 2 ? 2 : 1;
    if (wide) {
        hipExtLaunchKernelGGL(wino::conv64_kernel, dim3(blocks, cob64), dim3(wino::kThreads64), 0, stream, ev.start,
                              ev.stop, 0, a);
    } else if (split) {
        hipExtLaunchKernelGGL(wino::conv64_kernel, dim3(blocks, cob32 / 2), dim3(wino::kThreads64), 0, stream,
                              ev.start, nullptr, 0, a);
        a.cob_base = cob32 - 1;
        hipExtLaunchKernelGGL(wino::conv_kernel<1>, dim3(blocks, 1), dim3(wino::kThreads), 0, stream, nullptr,
                              ev.stop, 0, a);
    } else if (ks == 2)
        hipExtLaunchKernelGGL(wino::conv_kernel<2>, dim3(blocks, cob32), dim3(2 * wino::kThreads), 0, stream,
                              ev.start, ev.stop, 0, a);
    else
        hipExtLaunchKernelGGL(wino::conv_kernel<1>, dim3(blocks, cob32), dim3(wino::kThreads), 0, stream, ev.start,
                              ev.stop, 0, a);
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
