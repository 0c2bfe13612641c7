// Depth-candidate correlation of the TranSplat cost volume on gfx950.
//
// Fuses, per (query pixel, depth candidate), what the reference does in four materialising steps:
//   calculate_grid (src/model/encoder/matching/depth_predictor_trans.py:11-57): back-project the
//     integer pixel with K^-1, rotate/translate into the other camera at depth 1/disp, project with
//     K, divide by max(z, 1e-3), normalise 2u/(W-1) - 1            -> grid [(v b), D, HW, 2], 8 MB
//   UVTransformerEncoder ref_3d = grid / 2 + 0.5 in (b v) order (utils/encoder.py:57-59)
//   mmcv ms_deform_attn bilinear sampling of the OTHER view's features at loc * size - 0.5 with
//     zero padding (attention.py:359 view flip; MSDA im2col)           -> [2, HW*D, C], 537 MB
//   correlation with the own feature: coarse sum_c / sqrt(C) (attention.py:542-547),
//     cross mean_c over softmax-weighted 4-point samples (attention.py:365-410)
// The grid is recomputed in registers from 2 x (K, K^-1, R, t) + D disparities, the sampled
// features never leave registers, and the only HBM traffic is the two channel-last feature maps
// (L2-resident), the per-(query, depth) offsets/weights of the cross layer, and the [.., D] output.
//
// Mapping: one workgroup per query pixel, 16 lanes per (query, depth) (8 channels per lane, so a
// 16-lane group reads one 512-B feature row as 16 x 32 B), 16 depths in flight per workgroup.
#include "common.h"
#include "prof.h"

#include <cstdlib>

namespace tsplat {
namespace corr {

constexpr int kC = 128;        // feature channels (= embed_dims)
constexpr int kThreads = 256;  // 16 groups of 16 lanes
constexpr int kGroups = kThreads / 16;
constexpr int kMaxPoints = 8;


struct Cam {
    float kinv[9], k[9], r[9], t[3];
};

struct Geo {
    int B, H, W, D;
};

// (b v)-ordered query n = 2b + v uses camera (v b) index v*B + b
__device__ __forceinline__ const float* cam_ptr(const float* cams, const Geo& g, int n) {
    const int b = n >> 1, v = n & 1;
    return cams + (size_t)(v * g.B + b) * 30;
}

// ray of integer pixel (x, y) in the own camera, rotated into the other: R K^-1 [x, y, 1]
__device__ __forceinline__ void pixel_ray(const float* c, float x, float y, float ray[3]) {
#pragma clang fp contract(off)
    const float* ki = c;
    const float* R = c + 18;
    const float p0 = ki[0] * x + ki[1] * y + ki[2];
    const float p1 = ki[3] * x + ki[4] * y + ki[5];
    const float p2 = ki[6] * x + ki[7] * y + ki[8];
    ray[0] = R[0] * p0 + R[1] * p1 + R[2] * p2;
    ray[1] = R[3] * p0 + R[4] * p1 + R[5] * p2;
    ray[2] = R[6] * p0 + R[7] * p1 + R[8] * p2;
}

// ref_3d of the ray at depth 1/disp: normalised grid coordinate / 2 + 0.5, in [0, 1] on-image
__device__ __forceinline__ void sample_ref(const float* c, const Geo& g, const float ray[3],
                                           float disp, float& rx, float& ry) {
#pragma clang fp contract(off)
    const float* K = c + 9;
    const float* t = c + 27;
    const float depth = 1.0f / disp;
    const float P0 = ray[0] * depth + t[0];
    const float P1 = ray[1] * depth + t[1];
    const float P2 = ray[2] * depth + t[2];
    const float u = K[0] * P0 + K[1] * P1 + K[2] * P2;
    const float v = K[3] * P0 + K[4] * P1 + K[5] * P2;
    const float w = fmaxf(K[6] * P0 + K[7] * P1 + K[8] * P2, 1e-3f);
    const float gx = 2.0f * (u / w) / (float)(g.W - 1) - 1.0f;
    const float gy = 2.0f * (v / w) / (float)(g.H - 1) - 1.0f;
    rx = gx / 2.0f + 0.5f;
    ry = gy / 2.0f + 0.5f;
}

// sampling position of depth sample `disp` in the other view's pixel grid (mmcv: loc * size - 0.5),
// with no fma contraction, so every kernel that places samples this way places them identically
// (the dedup kernels compare bit for bit; near w = 1e-3 the division amplifies a contraction's ulp)
__device__ __forceinline__ void sample_im(const float* c, const Geo& g, const float ray[3], float disp, float& xim,
                                          float& yim) {
#pragma clang fp contract(off)
    float rx, ry;
    sample_ref(c, g, ray, disp, rx, ry);
    xim = rx * (float)g.W - 0.5f;
    yim = ry * (float)g.H - 0.5f;
}

// bilinear sample (zero padding, mmcv ms_deform_attn_im2col_bilinear) of 8 channels [c0, c0+8)
// of a channel-last [H*W, C] map; accumulates w * value into acc
__device__ __forceinline__ void bilinear_acc8(const float* __restrict__ img, const Geo& g, float xim,
                                              float yim, float w, int c0, float acc[8]) {
    if (!(yim > -1.0f && xim > -1.0f && yim < (float)g.H && xim < (float)g.W)) return;
    const float fy = floorf(yim), fx = floorf(xim);
    const int y0 = (int)fy, x0 = (int)fx, y1 = y0 + 1, x1 = x0 + 1;
    const float ly = yim - fy, lx = xim - fx, hy = 1.0f - ly, hx = 1.0f - lx;
    const float w1 = hy * hx, w2 = hy * lx, w3 = ly * hx, w4 = ly * lx;
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
    auto corner = [&](int yy, int xx, float cw) {
        const float4* s = reinterpret_cast<const float4*>(img + ((size_t)yy * g.W + xx) * kC + c0);
        const float4 a = s[0], b = s[1];
        v[0] += cw * a.x; v[1] += cw * a.y; v[2] += cw * a.z; v[3] += cw * a.w;
        v[4] += cw * b.x; v[5] += cw * b.y; v[6] += cw * b.z; v[7] += cw * b.w;
    };
    if (y0 >= 0 && x0 >= 0) corner(y0, x0, w1);
    if (y0 >= 0 && x1 <= g.W - 1) corner(y0, x1, w2);
    if (y1 <= g.H - 1 && x0 >= 0) corner(y1, x0, w3);
    if (y1 <= g.H - 1 && x1 <= g.W - 1) corner(y1, x1, w4);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += w * v[i];
}

__device__ __forceinline__ float group_sum16(float x) {
    x += __shfl_xor(x, 1, 16);
    x += __shfl_xor(x, 2, 16);
    x += __shfl_xor(x, 4, 16);
    x += __shfl_xor(x, 8, 16);
    return x;
}

// ---- coarse: corr[n][p][d] = <sample(feat_other, loc(p, d)), feat_own[p]> / sqrt(C)
__global__ void __launch_bounds__(kThreads)
uv_coarse_kernel(Geo g, const float* __restrict__ feat, const float* __restrict__ cams,
                 const float* __restrict__ disp, float* __restrict__ out) {
    __shared__ float s_out[256];
    const int p = blockIdx.x, n = blockIdx.y;
    const int grp = threadIdx.x >> 4, gl = threadIdx.x & 15, c0 = gl * 8;
    const size_t HW = (size_t)g.H * g.W;
    const float* own = feat + (size_t)n * HW * kC;
    const float* other = feat + (size_t)(n ^ 1) * HW * kC;
    const float* c = cam_ptr(cams, g, n);
    const int b = n >> 1, v = n & 1;
    const float* dsp = disp + (size_t)(v * g.B + b) * g.D;
    float key[8];
    {
        const float4* s = reinterpret_cast<const float4*>(own + (size_t)p * kC + c0);
        const float4 a = s[0], bb = s[1];
        key[0] = a.x; key[1] = a.y; key[2] = a.z; key[3] = a.w;
        key[4] = bb.x; key[5] = bb.y; key[6] = bb.z; key[7] = bb.w;
    }
    float ray[3];
    pixel_ray(c, (float)(p % g.W), (float)(p / g.W), ray);
    const float inv_sqrt_c = 1.0f / sqrtf((float)kC);
    for (int d0 = 0; d0 < g.D; d0 += kGroups) {
        const int d = d0 + grp;
        float acc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = 0.f;
        if (d < g.D) {
            float rx, ry;
            sample_ref(c, g, ray, dsp[d], rx, ry);
            bilinear_acc8(other, g, rx * (float)g.W - 0.5f, ry * (float)g.H - 0.5f, 1.0f, c0, acc);
        }
        float part = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) part += acc[i] * key[i];
        part = group_sum16(part);
        if (gl == 0 && d < g.D) s_out[d & 255] = part * inv_sqrt_c;
        if (((d0 + kGroups) & 255) == 0 || d0 + kGroups >= g.D) {
            __syncthreads();
            const int base = d0 & ~255;
            const int cnt = min(256, g.D - base);
            if ((int)threadIdx.x < cnt) out[((size_t)n * HW + p) * g.D + base + threadIdx.x] = s_out[threadIdx.x];
            __syncthreads();
        }
    }
}

// ---- coarse, corner-deduplicated: corr(p, d) = sum_corner w_corner <F_other[corner], key_p> / sqrt(C)
// The D samples of a pixel lie on its epipolar segment in the other view and are uniform in
// disparity, so consecutive samples sit ~0.5 px apart and their bilinear corners repeat: at the
// production shape 512 corner reads (128 depths x 4) per pixel touch only ~130 distinct feature
// rows. One wave per query pixel:
//   1. each lane places S = D / 64 samples and marks their valid corners in a per-wave LDS bitmap
//      over the other view's H*W pixels (ds_or);
//   2. a wave scan of the bitmap's popcounts ranks the distinct corners and lists them;
//   3. each distinct corner's 128-wide dot with the own feature is computed ONCE (4 lanes per
//      corner, 32 channels = one 128-B line per lane, two xor-shuffles) into LDS;
//   4. each lane combines its samples' 4 weighted corner dots (rank = prefix + popcount below).
// On-chip feature traffic drops from 2 KB to ~0.5 KB per (pixel, depth) pair's share; the sum
// order differs from the sample-then-dot form only by rounding (tests hold 1e-4 absolute).
constexpr int kDedupWaves = 4;
constexpr int kDedupMaxS = 4;  // D <= 256

// WPE: waves per SIMD the register budget is sized for (5: 82 VGPRs, 1,280 of the production
// launch's 2,048 workgroups resident; 6: 80 VGPRs with 2 spilled, 1,536 resident)
template <int S, int WPE>
__global__ void __launch_bounds__(kDedupWaves * 64, WPE)
uv_coarse_dedup_kernel(Geo g, int nw, const float* __restrict__ feat, const float* __restrict__ cams,
                       const float* __restrict__ disp, float* __restrict__ out, int diag) {
    extern __shared__ unsigned smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = blockIdx.y;
    const int HW = g.H * g.W;
    const int p = blockIdx.x * kDedupWaves + wave;
    const bool active = p < HW;
    unsigned* bm = smem + (size_t)wave * (2 * nw + 8 * g.D);
    unsigned* pre = bm + nw;
    int* list = reinterpret_cast<int*>(pre + nw);
    float* dots = reinterpret_cast<float*>(list + 4 * g.D);
    // own feature (the dot operand: 8 lanes per corner, lane `sub` holds channels i*32 + sub*4 .. +3)
    // and this lane's disparities are loaded first: their latency overlaps sampling and ranking
    const int sub = lane & 7;
    const int pc = active ? p : 0;
    float4 key[4];
    {
        const float4* own = reinterpret_cast<const float4*>(feat + ((size_t)n * HW + pc) * kC) + sub;
#pragma unroll
        for (int i = 0; i < 4; ++i) key[i] = own[8 * i];
    }
    const float* c = cam_ptr(cams, g, n);
    const int b = n >> 1, v = n & 1;
    const float* dsp = disp + (size_t)(v * g.B + b) * g.D;
    float dv[S];
#pragma unroll
    for (int s = 0; s < S; ++s) dv[s] = dsp[min(lane + 64 * s, g.D - 1)];
    for (int i = lane; i < nw; i += 64) bm[i] = 0u;
    __syncthreads();

    // 1. samples -> bilinear corners (mmcv zero padding), marked in the bitmap. A corner that the
    //    previous depth sample (lane - 1, or lane 63 of the previous slice) also touches is not
    //    re-marked: consecutive samples share most corners, and same-word LDS atomics serialise.
    int cidx[S][4];
    float cw[S][4];
    const float fw = (float)g.W, fh = (float)g.H;
    float ray[3];
    pixel_ray(c, (float)(pc % g.W), (float)(pc / g.W), ray);
    int prev_cell = -1;  // previous sample's (y0 * W + x0) + (W + 1) offset code, -1 = none
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int d = lane + 64 * s;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            cidx[s][k] = -1;
            cw[s][k] = 0.f;
        }
        int y0 = 0, x0 = 0, cell = -1;
        if (active && d < g.D) {
            float xim, yim;
            sample_im(c, g, ray, dv[s], xim, yim);
            if (yim > -1.0f && xim > -1.0f && yim < fh && xim < fw) {
                const float fy = floorf(yim), fx = floorf(xim);
                y0 = (int)fy;
                x0 = (int)fx;
                const int y1 = y0 + 1, x1 = x0 + 1;
                const float ly = yim - fy, lx = xim - fx, hy = 1.0f - ly, hx = 1.0f - lx;
                if (y0 >= 0 && x0 >= 0) { cidx[s][0] = y0 * g.W + x0; cw[s][0] = hy * hx; }
                if (y0 >= 0 && x1 <= g.W - 1) { cidx[s][1] = y0 * g.W + x1; cw[s][1] = hy * lx; }
                if (y1 <= g.H - 1 && x0 >= 0) { cidx[s][2] = y1 * g.W + x0; cw[s][2] = ly * hx; }
                if (y1 <= g.H - 1 && x1 <= g.W - 1) { cidx[s][3] = y1 * g.W + x1; cw[s][3] = ly * lx; }
                cell = (y0 + 1) * (g.W + 2) + (x0 + 1);  // y0, x0 >= -1
            }
        }
        // the previous depth sample's cell: lane - 1 of this slice, lane 63 of the previous one
        int pcell = __shfl_up(cell, 1, 64);
        const int last = __shfl(cell, 63, 64);
        if (lane == 0) pcell = prev_cell;
        prev_cell = last;
        const int py0 = pcell >= 0 ? pcell / (g.W + 2) - 1 : -100, px0 = pcell >= 0 ? pcell % (g.W + 2) - 1 : -100;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int ci = cidx[s][k];
            if (ci < 0) continue;
            const int yy = y0 + (k >> 1), xx = x0 + (k & 1);
            const bool seen = yy >= py0 && yy <= py0 + 1 && xx >= px0 && xx <= px0 + 1;
            if (!seen) atomicOr(&bm[ci >> 5], 1u << (ci & 31));
        }
    }
    __syncthreads();
    if (diag == 1) { if (active) out[((size_t)n * HW + p) * g.D + lane] = (float)bm[lane] + key[0].x; return; }

    // 2. rank the distinct corners. Lane l holds word wb + l; the non-empty words are visited two
    //    at a time (a uniform loop over the ballot of non-empty words): half-wave h takes the h-th
    //    of the pair, lane l & 31 tests its bit. The words come from their owner lanes by
    //    v_readlane (a uniform index), not by an LDS read per iteration.
    int total = 0;
    for (int wb = 0; wb < nw; wb += 64) {
        const int wl = wb + lane;
        const unsigned mine = wl < nw ? bm[wl] : 0u;
        unsigned long long nz = __ballot(mine != 0u);
        while (nz) {
            const int i0 = __ffsll((long long)nz) - 1;
            nz &= nz - 1ull;
            const int i1 = nz ? __ffsll((long long)nz) - 1 : -1;
            if (nz) nz &= nz - 1ull;
            const unsigned b0 = (unsigned)__builtin_amdgcn_readlane((int)mine, i0);
            const unsigned b1 = i1 >= 0 ? (unsigned)__builtin_amdgcn_readlane((int)mine, i1) : 0u;
            const int h = lane >> 5, l = lane & 31;
            if (h == 0 || i1 >= 0) {
                const unsigned bits = h ? b1 : b0;
                const int w = wb + (h ? i1 : i0);
                const int base = total + (h ? __popc(b0) : 0);
                if ((bits >> l) & 1u) list[base + __popc(bits & ((1u << l) - 1u))] = w * 32 + l;
                if (l == 0) pre[w] = (unsigned)base;
            }
            total += __popc(b0) + __popc(b1);
        }
    }
    __syncthreads();
    if (diag == 2) { if (active) out[((size_t)n * HW + p) * g.D + lane] = (float)list[lane] + key[0].x; return; }

    // 3. one dot per distinct corner: 8 lanes per corner (each load instruction covers a full
    //    128-B line of 8 rows), 8 corners per pass, the next pass's rows in flight
    if (active) {
        const float4* other = reinterpret_cast<const float4*>(feat + (size_t)(n ^ 1) * HW * kC) + sub;
        const int jend = (total + 7) & ~7;  // same trip count for every lane (shuffles)
        auto load = [&](int jj, float4* x) {
            const float4* row = other + (size_t)(jj < total ? list[jj] : 0) * (kC / 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = row[8 * i];
        };
        auto dot = [&](int jj, const float4* x) {
            float a0 = 0.f, a1 = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a0 += x[i].x * key[i].x;
                a1 += x[i].y * key[i].y;
                a0 += x[i].z * key[i].z;
                a1 += x[i].w * key[i].w;
            }
            float acc = a0 + a1;
            acc += __shfl_xor(acc, 1, 8);
            acc += __shfl_xor(acc, 2, 8);
            acc += __shfl_xor(acc, 4, 8);
            if (jj < total && sub == 0) dots[jj] = acc;
        };
        float4 xa[4], xb[4];
        int j = lane >> 3;
        if (j < jend) load(j, xa);
        for (; j < jend; j += 16) {
            if (j + 8 < jend) load(j + 8, xb);
            dot(j, xa);
            if (j + 16 < jend) load(j + 16, xa);
            if (j + 8 < jend) dot(j + 8, xb);
        }
    }
    __syncthreads();
    if (diag == 3) { if (active) out[((size_t)n * HW + p) * g.D + lane] = dots[lane]; return; }
    if (!active) return;

    // 4. each sample = its corners' weighted dots (rank = word prefix + popcount below the bit)
    const float inv_sqrt_c = 1.0f / sqrtf((float)kC);
    float* o = out + ((size_t)n * HW + p) * g.D;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int d = lane + 64 * s;
        if (d >= g.D) continue;
        float val = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int ci = cidx[s][k];
            if (ci < 0) continue;
            const unsigned wd = bm[ci >> 5];
            const int rank = (int)pre[ci >> 5] + __popc(wd & ((1u << (ci & 31)) - 1u));
            val += cw[s][k] * dots[rank];
        }
        o[d] = val * inv_sqrt_c;
    }
}

// ---- coarse, run-deduplicated (round 6; default): the corner dedup above without the bitmap.
// A pixel's D samples walk its epipolar segment in depth order, so their bilinear cells
// (y0, x0) come in runs, and along a straight path (x and y each monotone) a corner shared by two
// distinct cells is shared by every cell between them: a corner is new exactly when the PREVIOUS
// distinct cell does not hold it. So, per wave (one query pixel), with no LDS bitmap, no ds_or
// atomics, no popcount scan over H*W / 32 words and no workgroup barrier:
//   1. each lane places its samples; a sample whose cell differs from the previous sample's is a
//      run head; a head's new corners (in bounds, outside the previous cell's 2 x 2) get ranks by a
//      ballot prefix sum and are listed; its other corners point at the previous cell's entry;
//   2. those pointers are resolved in place (chains of <= 3 cells on a monotone path; the loop
//      runs until none is left, so a non-monotone rounding step only costs an extra dot);
//   3. one dot per listed corner (the 8-lane row dot above, same sum order);
//   4. each sample reads its run's 4 corner ranks (one ds_read_b128) and combines as above.
// The result is the bitmap kernel's bit for bit (same dots, same per-sample sum order).
constexpr int kRunWaves = 4;

// LDS words per wave: src [D cells][4] ranks, then [4 D] corner pixels that the dot phase overwrites
// with the corners' dots (entry j is read by its 8 lanes before its dot is stored there)
__host__ __device__ inline int run_lds_words(int depths) { return 8 * depths; }

// LDS hand-off between the lanes of ONE wave (its LDS operations execute in order)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// WPE: waves per SIMD the register budget is sized for -- 8 (default for D <= 128: 60 VGPRs, one dot
// pass in flight per wave, all 2,048 workgroups of the production launch resident at once) or 6
// (73 VGPRs, two passes in flight; TSPLAT_CORR_RUN_WPE=6, and D > 128)
template <int S, int WPE>
__global__ void __launch_bounds__(kRunWaves * 64, WPE)
uv_coarse_run_kernel(Geo g, const float* __restrict__ feat, const float* __restrict__ cams,
                     const float* __restrict__ disp, float* __restrict__ out) {
    extern __shared__ int rsmem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = blockIdx.y;
    const int HW = g.H * g.W;
    const int p = blockIdx.x * kRunWaves + wave;
    if (p >= HW) return;  // wave-uniform; nothing below synchronises the workgroup
    int* src = rsmem + (size_t)wave * run_lds_words(g.D);
    int* list = src + 4 * g.D;
    float* dots = reinterpret_cast<float*>(list);

    // own feature (dot operand, 8 lanes per corner) and this lane's disparities first
    const int sub = lane & 7;
    float4 key[4];
    {
        const float4* own = reinterpret_cast<const float4*>(feat + ((size_t)n * HW + p) * kC) + sub;
#pragma unroll
        for (int i = 0; i < 4; ++i) key[i] = own[8 * i];
    }
    const float* c = cam_ptr(cams, g, n);
    const int b = n >> 1, v = n & 1;
    const float* dsp = disp + (size_t)(v * g.B + b) * g.D;
    float dv[S];
#pragma unroll
    for (int s = 0; s < S; ++s) dv[s] = dsp[min(lane + 64 * s, g.D - 1)];

    // 1. samples -> cells, run heads, new corners
    const unsigned long long lt = (1ull << lane) - 1ull, le = lt | (1ull << lane);
    const float fw = (float)g.W, fh = (float)g.H;
    float ray[3];
    pixel_ray(c, (float)(p % g.W), (float)(p / g.W), ray);
    int cell_of[S];    // the sample's run (distinct-cell) index, -1 = outside the sampling window
    float cw[S][4];
    int cells = 0, total = 0, prev_cell = -1;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int d = lane + 64 * s;
        int y0 = 0, x0 = 0, cell = -1, inb = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) cw[s][k] = 0.f;
        if (d < g.D) {
            float xim, yim;
            sample_im(c, g, ray, dv[s], xim, yim);
            if (yim > -1.0f && xim > -1.0f && yim < fh && xim < fw) {
                const float fy = floorf(yim), fx = floorf(xim);
                y0 = (int)fy;
                x0 = (int)fx;
                const int y1 = y0 + 1, x1 = x0 + 1;
                const float ly = yim - fy, lx = xim - fx, hy = 1.0f - ly, hx = 1.0f - lx;
                if (y0 >= 0 && x0 >= 0) { inb |= 1; cw[s][0] = hy * hx; }
                if (y0 >= 0 && x1 <= g.W - 1) { inb |= 2; cw[s][1] = hy * lx; }
                if (y1 <= g.H - 1 && x0 >= 0) { inb |= 4; cw[s][2] = ly * hx; }
                if (y1 <= g.H - 1 && x1 <= g.W - 1) { inb |= 8; cw[s][3] = ly * lx; }
                cell = (y0 + 1) * (g.W + 2) + (x0 + 1);  // y0, x0 >= -1
            }
        }
        // the previous depth sample's cell: lane - 1 of this slice, lane 63 of the previous one
        int pcell = __shfl_up(cell, 1, 64);
        const int last = __shfl(cell, 63, 64);
        if (lane == 0) pcell = prev_cell;
        prev_cell = last;
        const bool head = cell >= 0 && cell != pcell;
        const int py0 = pcell >= 0 ? pcell / (g.W + 2) - 1 : -100, px0 = pcell >= 0 ? pcell % (g.W + 2) - 1 : -100;
        int code[4], nnew = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int dy = y0 + (k >> 1) - py0, dx = x0 + (k & 1) - px0;
            if (!((inb >> k) & 1)) code[k] = -1;                                   // zero padding
            else if (dy >= 0 && dy <= 1 && dx >= 0 && dx <= 1) code[k] = -2 - (2 * dy + dx);  // previous cell's
            else code[k] = nnew++;                                               // new: local index
        }
        if (!head) nnew = 0;
        const unsigned long long hb = __ballot(head);
        const unsigned long long n0 = __ballot(nnew & 1), n1 = __ballot(nnew & 2), n2 = __ballot(nnew & 4);
        const int rbase = total + __popcll(n0 & lt) + 2 * __popcll(n1 & lt) + 4 * __popcll(n2 & lt);
        const int ci = cells + __popcll(hb & le) - 1;
        if (head) {
            int e[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                e[k] = code[k] >= 0 ? rbase + code[k] : code[k];
                if (code[k] >= 0) list[rbase + code[k]] = (y0 + (k >> 1)) * g.W + x0 + (k & 1);
            }
            *reinterpret_cast<int4*>(src + 4 * ci) = make_int4(e[0], e[1], e[2], e[3]);
        }
        cell_of[s] = cell >= 0 ? ci : -1;
        cells += __popcll(hb);
        total += __popcll(n0) + 2 * __popcll(n1) + 4 * __popcll(n2);
    }
    wave_lds_sync();

    // 2. a corner held by the previous cell takes that cell's entry (resolved in place; progress
    //    is guaranteed because cell 0 has no predecessor)
    for (;;) {
        bool pending = false;
        for (int c0 = 0; c0 < cells; c0 += 64) {
            const int ce = c0 + lane;
            if (ce < cells) {
                int4 e = *reinterpret_cast<const int4*>(src + 4 * ce);
                int ev[4] = {e.x, e.y, e.z, e.w};
                bool changed = false;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (ev[k] <= -2) {
                        const int r = src[4 * (ce - 1) + (-2 - ev[k])];
                        if (r > -2) {
                            ev[k] = r;
                            changed = true;
                        } else {
                            pending = true;
                        }
                    }
                if (changed) *reinterpret_cast<int4*>(src + 4 * ce) = make_int4(ev[0], ev[1], ev[2], ev[3]);
            }
        }
        wave_lds_sync();
        if (!__any(pending)) break;
    }

    // 3. one dot per listed corner: 8 lanes per corner, 8 corners per pass, the next pass in flight
    {
        const float4* other = reinterpret_cast<const float4*>(feat + (size_t)(n ^ 1) * HW * kC) + sub;
        const int jend = (total + 7) & ~7;
        auto load = [&](int jj, float4* x) {
            const float4* row = other + (size_t)(jj < total ? list[jj] : 0) * (kC / 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = row[8 * i];
        };
        auto dot = [&](int jj, const float4* x) {
            float a0 = 0.f, a1 = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a0 += x[i].x * key[i].x;
                a1 += x[i].y * key[i].y;
                a0 += x[i].z * key[i].z;
                a1 += x[i].w * key[i].w;
            }
            float acc = a0 + a1;
            acc += __shfl_xor(acc, 1, 8);
            acc += __shfl_xor(acc, 2, 8);
            acc += __shfl_xor(acc, 4, 8);
            if (jj < total && sub == 0) dots[jj] = acc;
        };
        if constexpr (WPE >= 8) {
            // one pass in flight per wave: at 8 waves per SIMD the other waves cover the latency
            for (int j = lane >> 3; j < jend; j += 8) {
                float4 xa[4];
                load(j, xa);
                dot(j, xa);
            }
        } else {
            float4 xa[4], xb[4];
            int j = lane >> 3;
            if (j < jend) load(j, xa);
            for (; j < jend; j += 16) {
                if (j + 8 < jend) load(j + 8, xb);
                dot(j, xa);
                if (j + 16 < jend) load(j + 16, xa);
                if (j + 8 < jend) dot(j + 8, xb);
            }
        }
    }
    wave_lds_sync();

    // 4. each sample = its run's corners' weighted dots
    const float inv_sqrt_c = 1.0f / sqrtf((float)kC);
    float* o = out + ((size_t)n * HW + p) * g.D;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int d = lane + 64 * s;
        if (d >= g.D) continue;
        float val = 0.f;
        if (cell_of[s] >= 0) {
            const int4 e = *reinterpret_cast<const int4*>(src + 4 * cell_of[s]);
            const int ev[4] = {e.x, e.y, e.z, e.w};
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (ev[k] >= 0) val += cw[s][k] * dots[ev[k]];
        }
        o[d] = val * inv_sqrt_c;
    }
}

// ---- cross: out[n][p][d] = mean_c key[p]_c * sum_pt softmax(logit)_pt sample(value_other, loc + off)
__global__ void __launch_bounds__(kThreads)
uv_cross_kernel(Geo g, int P, const float* __restrict__ value, const float* __restrict__ key,
                const float* __restrict__ cams, const float* __restrict__ disp,
                const float* __restrict__ offsets, const float* __restrict__ logits,
                float* __restrict__ out) {
    __shared__ float s_out[256];
    const int p = blockIdx.x, n = blockIdx.y;
    const int grp = threadIdx.x >> 4, gl = threadIdx.x & 15, c0 = gl * 8;
    const size_t HW = (size_t)g.H * g.W;
    const float* other = value + (size_t)(n ^ 1) * HW * kC;
    const float* c = cam_ptr(cams, g, n);
    const int b = n >> 1, v = n & 1;
    const float* dsp = disp + (size_t)(v * g.B + b) * g.D;
    const float* off = offsets + ((size_t)n * HW + p) * g.D * P * 2;
    const float* lg = logits + ((size_t)n * HW + p) * g.D * P;
    float kv[8];
    {
        const float4* s = reinterpret_cast<const float4*>(key + ((size_t)n * HW + p) * kC + c0);
        const float4 a = s[0], bb = s[1];
        kv[0] = a.x; kv[1] = a.y; kv[2] = a.z; kv[3] = a.w;
        kv[4] = bb.x; kv[5] = bb.y; kv[6] = bb.z; kv[7] = bb.w;
    }
    float ray[3];
    pixel_ray(c, (float)(p % g.W), (float)(p / g.W), ray);
    const float fw = (float)g.W, fh = (float)g.H;
    for (int d0 = 0; d0 < g.D; d0 += kGroups) {
        const int d = d0 + grp;
        float acc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = 0.f;
        if (d < g.D) {
            float rx, ry;
            sample_ref(c, g, ray, dsp[d], rx, ry);
            float e[kMaxPoints];
            float mx = -INFINITY;
            for (int pt = 0; pt < P; ++pt) mx = fmaxf(mx, lg[d * P + pt]);
            float ssum = 0.f;
            for (int pt = 0; pt < P; ++pt) {
                e[pt] = __expf(lg[d * P + pt] - mx);
                ssum += e[pt];
            }
            for (int pt = 0; pt < P; ++pt) {
                const float wgt = e[pt] / ssum;  // torch softmax over the points
                const float lx = rx + off[(d * P + pt) * 2] / fw;
                const float ly = ry + off[(d * P + pt) * 2 + 1] / fh;
                bilinear_acc8(other, g, lx * fw - 0.5f, ly * fh - 0.5f, wgt, c0, acc);
            }
        }
        float part = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) part += acc[i] * kv[i];
        part = group_sum16(part);
        if (gl == 0 && d < g.D) s_out[d & 255] = part * (1.0f / (float)kC);
        if (((d0 + kGroups) & 255) == 0 || d0 + kGroups >= g.D) {
            __syncthreads();
            const int base = d0 & ~255;
            const int cnt = min(256, g.D - base);
            if ((int)threadIdx.x < cnt) out[((size_t)n * HW + p) * g.D + base + threadIdx.x] = s_out[threadIdx.x];
            __syncthreads();
        }
    }
}

// ---- cross through a correlation table (the dot products factored out of the sampling):
//   mean_c key[p]_c * sum_pt w_pt bilinear(V_other)(loc)_c
//     = (1/C) sum_pt w_pt sum_corner b_corner * G[p][corner],   G = key V_other^T  [HW, HW]
// G comes from one library GEMM per (b v) (a plain batched GEMM, MFMA-bound); this kernel is then
// a pure gather: one thread per (pixel, depth), 4 points x 4 corners read from the pixel's 16-KB
// G row (L1/L2-resident), offsets and logits read coalesced (32 B + 16 B per thread). It replaces
// 16 x 512-B feature-row reads per (pixel, depth) -- 8.6 GB of L2 traffic per 2-view layer --
// by 16 x 4 B.
__global__ void __launch_bounds__(kThreads)
uv_cross_table_kernel(Geo g, int P, int C, const float* __restrict__ table, const float* __restrict__ cams,
                      const float* __restrict__ disp, const float* __restrict__ offsets,
                      const float* __restrict__ logits, float* __restrict__ out) {
    const int n = blockIdx.y;
    const size_t HW = (size_t)g.H * g.W;
    const size_t t = (size_t)blockIdx.x * kThreads + threadIdx.x;
    if (t >= HW * g.D) return;
    const int p = (int)(t / g.D), d = (int)(t - (size_t)p * g.D);
    const float* c = cam_ptr(cams, g, n);
    const int b = n >> 1, v = n & 1;
    const float* row = table + ((size_t)n * HW + p) * HW;
    const float* off = offsets + (((size_t)n * HW + p) * g.D + d) * P * 2;
    const float* lg = logits + (((size_t)n * HW + p) * g.D + d) * P;
    float ray[3];
    pixel_ray(c, (float)(p % g.W), (float)(p / g.W), ray);
    float rx, ry;
    sample_ref(c, g, ray, disp[(size_t)(v * g.B + b) * g.D + d], rx, ry);
    float e[kMaxPoints];
    float mx = -INFINITY;
    for (int pt = 0; pt < P; ++pt) mx = fmaxf(mx, lg[pt]);
    float ssum = 0.f;
    for (int pt = 0; pt < P; ++pt) {
        e[pt] = __expf(lg[pt] - mx);
        ssum += e[pt];
    }
    const float fw = (float)g.W, fh = (float)g.H;
    float acc = 0.f;
    for (int pt = 0; pt < P; ++pt) {
        const float wgt = e[pt] / ssum;
        const float xim = (rx + off[2 * pt] / fw) * fw - 0.5f;
        const float yim = (ry + off[2 * pt + 1] / fh) * fh - 0.5f;
        if (!(yim > -1.0f && xim > -1.0f && yim < fh && xim < fw)) continue;
        const float fy = floorf(yim), fx = floorf(xim);
        const int y0 = (int)fy, x0 = (int)fx, y1 = y0 + 1, x1 = x0 + 1;
        const float ly = yim - fy, lx = xim - fx, hy = 1.0f - ly, hx = 1.0f - lx;
        float val = 0.f;
        if (y0 >= 0 && x0 >= 0) val += hy * hx * row[y0 * g.W + x0];
        if (y0 >= 0 && x1 <= g.W - 1) val += hy * lx * row[y0 * g.W + x1];
        if (y1 <= g.H - 1 && x0 >= 0) val += ly * hx * row[y1 * g.W + x0];
        if (y1 <= g.H - 1 && x1 <= g.W - 1) val += ly * lx * row[y1 * g.W + x1];
        acc += wgt * val;
    }
    out[((size_t)n * HW + p) * g.D + d] = acc / (float)C;
}

// ---- single-level single-head MSDA: out[n][q] = sum_pt w_pt sample(value[n], loc_pt)
__global__ void __launch_bounds__(kThreads)
msda_kernel(Geo g, int Q, int P, const float* __restrict__ value, const float* __restrict__ loc,
            const float* __restrict__ weights, float* __restrict__ out) {
    const int n = blockIdx.y;
    const int q = blockIdx.x * kGroups + (threadIdx.x >> 4);
    const int gl = threadIdx.x & 15, c0 = gl * 8;
    if (q >= Q) return;
    const size_t HW = (size_t)g.H * g.W;
    const float* img = value + (size_t)n * HW * kC;
    const float* lc = loc + ((size_t)n * Q + q) * P * 2;
    const float* wt = weights + ((size_t)n * Q + q) * P;
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    for (int pt = 0; pt < P; ++pt)
        bilinear_acc8(img, g, lc[2 * pt] * (float)g.W - 0.5f, lc[2 * pt + 1] * (float)g.H - 0.5f, wt[pt],
                      c0, acc);
    float4* o = reinterpret_cast<float4*>(out + ((size_t)n * Q + q) * kC + c0);
    o[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    o[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
}

// ---- the same sampling from the raw projections (the UV self-attention's glue folded in,
// reference attention.py:232-262): per query q = y W + x, ow[n][q] holds the P (dx, dy) sampling
// offsets then the P attention logits (one linear's output, row stride `ows`); loc_pt = ref + off /
// (W, H) with ref = ((x + 0.5) / W, (y + 0.5) / H) (the reference points, encoder.py:61-71, same fp32
// operations), weights = softmax(logits) -- instead of the softmax, division and addition launches
// around msda_kernel.
__global__ void __launch_bounds__(kThreads)
msda_raw_kernel(Geo g, int Q, int P, const float* __restrict__ value, const float* __restrict__ ow, int ows,
                float* __restrict__ out) {
    const int n = blockIdx.y;
    const int q = blockIdx.x * kGroups + (threadIdx.x >> 4);
    const int gl = threadIdx.x & 15, c0 = gl * 8;
    if (q >= Q) return;
    const size_t HW = (size_t)g.H * g.W;
    const float* img = value + (size_t)n * HW * kC;
    const float* r = ow + ((size_t)n * Q + q) * ows;
    const float fw = (float)g.W, fh = (float)g.H;
    const int qy = q / g.W, qx = q - qy * g.W;
    const float rx = ((float)qx + 0.5f) / fw, ry = ((float)qy + 0.5f) / fh;
    float m = -INFINITY;
    for (int pt = 0; pt < P; ++pt) m = fmaxf(m, r[2 * P + pt]);
    float sum = 0.f;
    for (int pt = 0; pt < P; ++pt) sum += expf(r[2 * P + pt] - m);
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    for (int pt = 0; pt < P; ++pt) {
        const float wt = expf(r[2 * P + pt] - m) / sum;
        const float lx = rx + r[2 * pt] / fw, ly = ry + r[2 * pt + 1] / fh;
        bilinear_acc8(img, g, lx * fw - 0.5f, ly * fh - 0.5f, wt, c0, acc);
    }
    float4* o = reinterpret_cast<float4*>(out + ((size_t)n * Q + q) * kC + c0);
    o[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    o[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
}

// ---- mmcv ms_deform_attn_forward, general form: value [bs][num_keys][heads][hd] (level l's
// H_l x W_l map starts at key level_start[l]), sampling_loc [bs][nq][heads][L][P][2] (x, y in
// [0, 1]), attn_weight [bs][nq][heads][L][P] -> out [bs][nq][heads * hd]. One thread per (query,
// head, VEC channels): consecutive threads read consecutive channels of a value row. Sampling as
// mmcv's im2col bilinear: h = y H - 1/2, w = x W - 1/2, taken only for -1 < h < H, -1 < w < W,
// corners outside the map read as 0, val = w1 v1 + w2 v2 + w3 v3 + w4 v4, col += val * weight.
template <int VEC>
__global__ void __launch_bounds__(kThreads)
ms_deform_attn_kernel(const float* __restrict__ value, const int64_t* __restrict__ shapes,
                      const int64_t* __restrict__ starts, const float* __restrict__ loc,
                      const float* __restrict__ attw, float* __restrict__ out, int nk, int nh, int hd, int L,
                      int nq, int P, size_t total) {
    const size_t idx = (size_t)blockIdx.x * kThreads + threadIdx.x;
    if (idx >= total) return;
    const int groups = hd / VEC;
    const int cg = (int)(idx % groups);
    size_t t = idx / groups;
    const int head = (int)(t % nh);
    t /= nh;  // = b * nq + q
    const size_t b = t / nq;
    const size_t row = (size_t)nh * hd;  // floats per key
    const float* lw = attw + (t * nh + head) * (size_t)L * P;
    const float* ll = loc + (t * nh + head) * (size_t)L * P * 2;
    float acc[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
    for (int l = 0; l < L; ++l) {
        const int H = (int)shapes[2 * l], W = (int)shapes[2 * l + 1];
        const float* base = value + (b * nk + (size_t)starts[l]) * row + (size_t)head * hd + cg * VEC;
        for (int p = 0; p < P; ++p) {
            const float hi = ll[2 * (l * P + p) + 1] * (float)H - 0.5f;
            const float wi = ll[2 * (l * P + p)] * (float)W - 0.5f;
            const float wt = lw[l * P + p];
            if (!(hi > -1.0f && wi > -1.0f && hi < (float)H && wi < (float)W)) continue;
            const int h0 = (int)floorf(hi), w0 = (int)floorf(wi), h1 = h0 + 1, w1 = w0 + 1;
            const float lh = hi - (float)h0, lwt = wi - (float)w0, hh = 1.0f - lh, hwt = 1.0f - lwt;
            const float f1 = hh * hwt, f2 = hh * lwt, f3 = lh * hwt, f4 = lh * lwt;
            const bool ok1 = h0 >= 0 && w0 >= 0, ok2 = h0 >= 0 && w1 <= W - 1;
            const bool ok3 = h1 <= H - 1 && w0 >= 0, ok4 = h1 <= H - 1 && w1 <= W - 1;
            float v1[VEC], v2[VEC], v3[VEC], v4[VEC];
            auto fetch = [&](bool ok, int y, int x, float (&v)[VEC]) {
                if (ok) {
                    const float* src = base + ((size_t)y * W + x) * row;
                    if constexpr (VEC == 4) {
                        const float4 f = *reinterpret_cast<const float4*>(src);
                        v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
                    } else {
#pragma unroll
                        for (int i = 0; i < VEC; ++i) v[i] = src[i];
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < VEC; ++i) v[i] = 0.f;
                }
            };
            fetch(ok1, h0, w0, v1);
            fetch(ok2, h0, w1, v2);
            fetch(ok3, h1, w0, v3);
            fetch(ok4, h1, w1, v4);
#pragma unroll
            for (int i = 0; i < VEC; ++i) acc[i] += (f1 * v1[i] + f2 * v2[i] + f3 * v3[i] + f4 * v4[i]) * wt;
        }
    }
    float* o = out + (t * nh + head) * (size_t)hd + cg * VEC;
    if constexpr (VEC == 4) {
        *reinterpret_cast<float4*>(o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) o[i] = acc[i];
    }
}

}  // namespace corr
}  // namespace tsplat

using namespace tsplat;

extern "C" int tsplat_ms_deform_attn_fwd(const float* value, const int64_t* spatial_shapes,
                                         const int64_t* level_start_index, const float* sampling_loc,
                                         const float* attn_weight, float* out, int32_t batch, int32_t num_keys,
                                         int32_t num_heads, int32_t head_dim, int32_t num_levels,
                                         int32_t num_queries, int32_t num_points, int32_t im2col_step,
                                         void* stream_) {
    using namespace tsplat::corr;
    if (!value || !spatial_shapes || !level_start_index || !sampling_loc || !attn_weight || !out || batch <= 0 ||
        num_keys <= 0 || num_heads <= 0 || head_dim <= 0 || num_levels <= 0 || num_queries <= 0 ||
        num_points <= 0 || im2col_step <= 0)
        return TSPLAT_EINVAL;
    // mmcv: im2col_step_ = min(batch, im2col_step) must divide the batch (it only chunks the
    // batch for its column buffer; the result does not depend on it)
    const int step = im2col_step < batch ? im2col_step : batch;
    if (batch % step) return TSPLAT_EINVAL;
    const bool v4 = head_dim % 4 == 0 && ((uintptr_t)value & 15) == 0 && ((uintptr_t)out & 15) == 0;
    const size_t total = (size_t)batch * num_queries * num_heads * (head_dim / (v4 ? 4 : 1));
    hipStream_t stream = (hipStream_t)stream_;
    const dim3 grid((unsigned)ceil_div(total, (size_t)kThreads));
    TSPLAT_PROF_BEGIN(prof::kMsda, stream);
    if (v4)
        hipLaunchKernelGGL(ms_deform_attn_kernel<4>, grid, dim3(kThreads), 0, stream, value, spatial_shapes,
                           level_start_index, sampling_loc, attn_weight, out, num_keys, num_heads, head_dim,
                           num_levels, num_queries, num_points, total);
    else
        hipLaunchKernelGGL(ms_deform_attn_kernel<1>, grid, dim3(kThreads), 0, stream, value, spatial_shapes,
                           level_start_index, sampling_loc, attn_weight, out, num_keys, num_heads, head_dim,
                           num_levels, num_queries, num_points, total);
    TSPLAT_PROF_END(prof::kMsda, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_uv_coarse_fwd(const float* feat, const float* cams, const float* disp,
                                    float* out, int32_t batch, int32_t height, int32_t width,
                                    int32_t channels, int32_t depths, void* stream_) {
    using namespace tsplat::corr;
    if (!feat || !cams || !disp || !out || channels != kC || batch <= 0 || height <= 1 ||
        width <= 1 || depths <= 0)
        return TSPLAT_EINVAL;
    Geo g{batch, height, width, depths};
    hipStream_t stream = (hipStream_t)stream_;
    const int hw = height * width;
    const int nw = (hw + 31) / 32;
    const size_t lds = (size_t)kDedupWaves * (2 * nw + 8 * depths) * sizeof(unsigned);
    const int S = (depths + 63) / 64;
    TSPLAT_PROF_BEGIN(prof::kUvCoarse, stream);
    const char* denv = getenv("TSPLAT_CORR_DIAG");  // diagnostic builds: stop after phase 1 / 2 / 3
    const int diag = denv ? atoi(denv) : 0;
    const char* env = getenv("TSPLAT_UV_COARSE_DIRECT");  // A/B switch: the sample-then-dot kernel
    const char* benv = getenv("TSPLAT_UV_COARSE_BITMAP");  // A/B switch: the round-2 bitmap dedup kernel
    const size_t run_lds = (size_t)kRunWaves * run_lds_words(depths) * sizeof(int);
    if (S <= kDedupMaxS && run_lds <= 64 * 1024 && !(env && env[0] == '1') && !(benv && benv[0] == '1') && !diag) {
        const dim3 grid(ceil_div(hw, kRunWaves), 2 * batch), block(kRunWaves * 64);
        const char* renv = getenv("TSPLAT_CORR_RUN_WPE");
        const bool w8 = !renv || atoi(renv) != 6;
#define TSPLAT_UVR(SS)                                                                                           \
    do {                                                                                                         \
        if (w8)                                                                                                  \
            hipLaunchKernelGGL((uv_coarse_run_kernel<SS, 8>), grid, block, run_lds, stream, g, feat, cams, disp, out); \
        else                                                                                                     \
            hipLaunchKernelGGL((uv_coarse_run_kernel<SS, 6>), grid, block, run_lds, stream, g, feat, cams, disp, out); \
    } while (0)
        switch (S) {  // (S >= 3 spills at the 8-wave budget: 6)
            case 1: TSPLAT_UVR(1); break;
            case 2: TSPLAT_UVR(2); break;
            case 3: hipLaunchKernelGGL((uv_coarse_run_kernel<3, 6>), grid, block, run_lds, stream, g, feat, cams, disp, out); break;
            default: hipLaunchKernelGGL((uv_coarse_run_kernel<4, 6>), grid, block, run_lds, stream, g, feat, cams, disp, out); break;
        }
#undef TSPLAT_UVR
    } else if (S <= kDedupMaxS && lds <= 64 * 1024 && !(env && env[0] == '1')) {
        const dim3 grid(ceil_div(hw, kDedupWaves), 2 * batch), block(kDedupWaves * 64);
        // 6 waves per SIMD (default; profiles/r5/late/corr_wpe.txt: b = 8 120.5 -> 111.4 us, b = 1 24.3 /
        // 24.2 vs 24.2 / 24.6) or 5 (TSPLAT_CORR_WPE=5, the A/B knob)
        const char* wenv = getenv("TSPLAT_CORR_WPE");
        const bool w6 = !wenv || atoi(wenv) != 5;
#define TSPLAT_UVC(SS)                                                                                           \
    do {                                                                                                         \
        if (w6)                                                                                                  \
            hipLaunchKernelGGL((uv_coarse_dedup_kernel<SS, 6>), grid, block, lds, stream, g, nw, feat, cams, disp, \
                               out, diag);                                                                       \
        else                                                                                                     \
            hipLaunchKernelGGL((uv_coarse_dedup_kernel<SS, 5>), grid, block, lds, stream, g, nw, feat, cams, disp, \
                               out, diag);                                                                       \
    } while (0)
        switch (S) {
            case 1: TSPLAT_UVC(1); break;
            case 2: TSPLAT_UVC(2); break;
            case 3: TSPLAT_UVC(3); break;
            default: TSPLAT_UVC(4); break;
        }
#undef TSPLAT_UVC
    } else {
        hipLaunchKernelGGL(uv_coarse_kernel, dim3(hw, 2 * batch), dim3(kThreads), 0, stream, g, feat, cams, disp,
                           out);
    }
    TSPLAT_PROF_END(prof::kUvCoarse, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_uv_cross_fwd(const float* value, const float* key, const float* cams,
                                   const float* disp, const float* offsets, const float* logits,
                                   float* out, int32_t batch, int32_t height, int32_t width,
                                   int32_t channels, int32_t depths, int32_t points, void* stream_) {
    using namespace tsplat::corr;
    if (!value || !key || !cams || !disp || !offsets || !logits || !out || channels != kC ||
        batch <= 0 || height <= 1 || width <= 1 || depths <= 0 || points <= 0 || points > kMaxPoints)
        return TSPLAT_EINVAL;
    Geo g{batch, height, width, depths};
    hipStream_t stream = (hipStream_t)stream_;
    TSPLAT_PROF_BEGIN(prof::kUvCross, stream);
    hipLaunchKernelGGL(uv_cross_kernel, dim3(height * width, 2 * batch), dim3(kThreads), 0, stream,
                       g, points, value, key, cams, disp, offsets, logits, out);
    TSPLAT_PROF_END(prof::kUvCross, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_uv_cross_table_fwd(const float* table, const float* cams, const float* disp,
                                         const float* offsets, const float* logits, float* out,
                                         int32_t batch, int32_t height, int32_t width, int32_t channels,
                                         int32_t depths, int32_t points, void* stream_) {
    using namespace tsplat::corr;
    if (!table || !cams || !disp || !offsets || !logits || !out || channels <= 0 || batch <= 0 ||
        height <= 1 || width <= 1 || depths <= 0 || points <= 0 || points > kMaxPoints)
        return TSPLAT_EINVAL;
    Geo g{batch, height, width, depths};
    const size_t work = (size_t)height * width * depths;
    hipStream_t stream = (hipStream_t)stream_;
    TSPLAT_PROF_BEGIN(prof::kUvCrossTable, stream);
    hipLaunchKernelGGL(uv_cross_table_kernel, dim3((unsigned)ceil_div(work, (size_t)kThreads), 2 * batch),
                       dim3(kThreads), 0, stream, g, points, channels, table, cams, disp, offsets, logits, out);
    TSPLAT_PROF_END(prof::kUvCrossTable, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_msda_fwd(const float* value, const float* loc, const float* weights,
                               float* out, int32_t n, int32_t height, int32_t width,
                               int32_t channels, int32_t queries, int32_t points, void* stream_) {
    using namespace tsplat::corr;
    if (!value || !loc || !weights || !out || channels != kC || n <= 0 || height <= 0 ||
        width <= 0 || queries <= 0 || points <= 0)
        return TSPLAT_EINVAL;
    Geo g{1, height, width, 1};
    hipStream_t stream = (hipStream_t)stream_;
    TSPLAT_PROF_BEGIN(prof::kMsda, stream);
    hipLaunchKernelGGL(msda_kernel, dim3(ceil_div(queries, kGroups), n), dim3(kThreads), 0, stream, g,
                       queries, points, value, loc, weights, out);
    TSPLAT_PROF_END(prof::kMsda, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_msda_raw_fwd(const float* value, const float* ow, float* out, int32_t n, int32_t height,
                                   int32_t width, int32_t channels, int32_t points, int32_t ow_stride, void* stream_) {
    using namespace tsplat::corr;
    if (!value || !ow || !out || channels != kC || n <= 0 || height <= 0 || width <= 0 || points <= 0 ||
        ow_stride < 3 * points)
        return TSPLAT_EINVAL;
    Geo g{1, height, width, 1};
    const int queries = height * width;
    hipStream_t stream = (hipStream_t)stream_;
    TSPLAT_PROF_BEGIN(prof::kMsda, stream);
    hipLaunchKernelGGL(msda_raw_kernel, dim3(ceil_div(queries, kGroups), n), dim3(kThreads), 0, stream, g, queries,
                       points, value, ow, ow_stride, out);
    TSPLAT_PROF_END(prof::kMsda, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

// ---------------------------------------------------------------------------------------------
// Depth-candidate softmax head (reference depth_predictor_trans.py:170-180):
//   pdf = softmax(logits, dim = depth);  coarse = sum_d disp[d] * pdf[d];  pdf_max = max_d pdf[d]
// one thread per pixel over the D channel planes of [N, D, H*W] (coalesced across pixels); the
// [N, D, H, W] pdf is never written (nothing else reads it).
namespace tsplat {
namespace corr {

// 256 threads = 32 pixels x 8 depth slices (lanes of a wave: consecutive pixels of one slice, so
// every load is a 128-B row segment); each thread keeps its slice's logits in registers, the 8
// slices' (max, sum, weighted sum) merge through LDS. 256 workgroups at 64^2 x 2 instead of 32
// one-pixel-per-thread workgroups walking all 128 depths serially (58 us -> a few us).
constexpr int kSmPix = 32, kSmSlices = 8, kSmMaxPer = 32;

__global__ void __launch_bounds__(kSmPix * kSmSlices)
depth_softmax_kernel(const float* __restrict__ logits, const float* __restrict__ disp, float* __restrict__ coarse,
                     float* __restrict__ pmax, int D, int HW) {
    __shared__ float sm[3][kSmSlices][kSmPix];
    const int pl = threadIdx.x % kSmPix, sl = threadIdx.x / kSmPix;
    const int p = blockIdx.x * kSmPix + pl, n = blockIdx.y;
    const int per = (D + kSmSlices - 1) / kSmSlices;
    const int d0 = sl * per, d1 = min(D, d0 + per);
    const int pc = min(p, HW - 1);
    const float* l = logits + (size_t)n * D * HW + pc;
    const float* dv = disp + (size_t)n * D;
    float v[kSmMaxPer];
#pragma unroll
    for (int k = 0; k < kSmMaxPer; ++k) v[k] = (k < d1 - d0) ? l[(size_t)(d0 + k) * HW] : -INFINITY;
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < kSmMaxPer; ++k) m = fmaxf(m, v[k]);
    float s = 0.f, w = 0.f;
#pragma unroll
    for (int k = 0; k < kSmMaxPer; ++k) {
        if (k < d1 - d0) {
            const float e = expf(v[k] - m);
            s += e;
            w += e * dv[d0 + k];
        }
    }
    sm[0][sl][pl] = m;
    sm[1][sl][pl] = s;
    sm[2][sl][pl] = w;
    __syncthreads();
    if (sl != 0 || p >= HW) return;
    float M = -INFINITY;
#pragma unroll
    for (int k = 0; k < kSmSlices; ++k) M = fmaxf(M, sm[0][k][pl]);
    float S = 0.f, W = 0.f;
#pragma unroll
    for (int k = 0; k < kSmSlices; ++k) {
        const float mk = sm[0][k][pl];
        const float a = mk == -INFINITY ? 0.f : expf(mk - M);
        S += a * sm[1][k][pl];
        W += a * sm[2][k][pl];
    }
    coarse[(size_t)n * HW + p] = W / S;
    pmax[(size_t)n * HW + p] = 1.0f / S;  // = exp(M - M) / S, the largest pdf entry
}

}  // namespace corr
}  // namespace tsplat

extern "C" int tsplat_depth_softmax_fwd(const float* logits, const float* disp, float* coarse, float* pdf_max,
                                        int32_t n, int32_t depths, int32_t hw, void* stream_) {
    using namespace tsplat::corr;
    if (!logits || !disp || !coarse || !pdf_max || n <= 0 || depths <= 0 || hw <= 0 || n > 65535)
        return TSPLAT_EINVAL;
    if (depths > kSmSlices * kSmMaxPer) return TSPLAT_EINVAL;
    hipStream_t stream = (hipStream_t)stream_;
    hipLaunchKernelGGL(depth_softmax_kernel, dim3((hw + kSmPix - 1) / kSmPix, n), dim3(kSmPix * kSmSlices), 0, stream,
                       logits, disp, coarse, pdf_max, depths, hw);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

// ---------------------------------------------------------------------------------------------
// Depth head tail (reference depth_predictor_trans.py:480-491): from the refined full-resolution
// disparity and the to_disparity head's two channels (delta, raw density) of map (v b) index m,
//   depth   = 1 / clamp(fullres + delta, 1 / far, 1 / near)      (the reference's fp32 operations)
//   density = sigmoid(raw)
// written straight into the [b, v, h w] layouts the Gaussian adapter reads -- one launch for what
// was nine elementwise ones (sigmoid, add, reciprocals, clamp, the (v b) -> (b v) repeats).
namespace tsplat {
namespace corr {
__global__ void __launch_bounds__(256) depth_tail_kernel(const float* __restrict__ fullres, const float* __restrict__ head,
                                                         const float* __restrict__ near, const float* __restrict__ far,
                                                         float* __restrict__ depth, float* __restrict__ density, int b,
                                                         int v, int hw) {
    const int m = blockIdx.y;  // (v b) map index
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= hw) return;
    const int vi = m / b, bi = m - vi * b;
    const int bv = bi * v + vi;  // near / far are [b, v]
    const float lo = 1.0f / far[bv], hi = 1.0f / near[bv];
    const float d = fullres[(size_t)m * hw + p] + head[((size_t)m * 2) * hw + p];
    const float c = fminf(fmaxf(d, lo), hi);
    const float raw = head[((size_t)m * 2 + 1) * hw + p];
    depth[(size_t)bv * hw + p] = 1.0f / c;
    density[(size_t)bv * hw + p] = 1.0f / (1.0f + expf(-raw));
}
}  // namespace corr
}  // namespace tsplat

extern "C" int tsplat_depth_tail_fwd(const float* fullres, const float* head, const float* near, const float* far,
                                     float* depth, float* density, int32_t batch, int32_t views, int32_t hw,
                                     void* stream_) {
    using namespace tsplat::corr;
    if (!fullres || !head || !near || !far || !depth || !density || batch <= 0 || views <= 0 || hw <= 0)
        return TSPLAT_EINVAL;
    hipLaunchKernelGGL(depth_tail_kernel, dim3((hw + 255) / 256, batch * views), dim3(256), 0, (hipStream_t)stream_,
                       fullres, head, near, far, depth, density, batch, views, hw);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
