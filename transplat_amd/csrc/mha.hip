// Dense multi-head self-attention of the Depth-Anything-V2 ViT-B encoder (DINOv2) on gfx950,
// exact fp32 MFMA.
//
// Semantics: reference src/depth_anything_v2/dinov2_layers/attention.py Attention.forward,
//   qkv = x Wqkv^T + b  -> [B, N, 3, H, 64];  out = softmax(q k^T * scale) v  -> [B, N, H, 64]
// (torch.nn.functional.scaled_dot_product_attention, no mask, no dropout). The kernel reads q, k, v
// straight from the qkv projection's output and writes the [B, N, H * 64] layout the output
// projection consumes, so the permute / transpose copies around SDPA disappear.
//
// Shape at 256x256 input: 2 images x 12 heads, N = 325 tokens (1 + 18 x 18), head dim 64:
// 0.65 GFLOP per call. Mapping: one workgroup = 4 waves on the same 32 queries of one (image,
// head); wave w walks the w-th quarter of the keys in 32-key tiles with no LDS and no barrier
// (each lane loads its own key row for S^T = K Q^T and one 128-B V segment per k-step for
// O^T += V^T P^T, the next tile prefetched into registers), and the four (max, sum, O) partials are
// merged once through LDS. 24 x 11 query blocks = 264 workgroups, ~1 wave per SIMD.
#include <string.h>

#include "common.h"
#include "prof.h"

namespace tsplat {
namespace mha {

constexpr int kD = 64;   // head dim
constexpr int kQW = 32;  // queries per workgroup (one MFMA tile)
constexpr int kKT = 32;  // keys per tile
constexpr int kThreads = 256;
constexpr float kLog2e = 1.4426950408889634f;

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float halves_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float halves_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// lanes l and l ^ 16 (v_permlane16_swap exchanges 16-lane rows 0 <-> 1 and 2 <-> 3, VALU only)
__device__ __forceinline__ float rows_max(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float rows_sum(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

struct Tile {
    floatx4 k[8];  // this lane's key row, dims 32 h .. 32 h + 31
    float v[32];   // V[key 8u + 4h + j][32 dt + c] for (u, j, dt): index (u * 4 + j) * 2 + dt
};

__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2, 2)))
mha_f32_kernel(const float* __restrict__ qkv, float* __restrict__ out, int N, int H, float scale) {
    __shared__ float sO[4][2][16][64];
    __shared__ float sML[4][2][kQW];

    const int qblk = blockIdx.x, bh = blockIdx.y;
    const int b = bh / H, head = bh - b * H;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int c = lane & 31, h = lane >> 5;
    const size_t tok = (size_t)3 * H * kD;  // floats per token row of qkv
    const float* base = qkv + (size_t)b * N * tok + (size_t)head * kD;
    const float* qb = base;
    const float* kb = base + (size_t)H * kD;
    const float* vb = base + (size_t)2 * H * kD;

    // keys of this wave: a quarter of N, in 32-key tiles (the last tile masked past N)
    const int per = (N + 3) / 4;
    const int k_lo = wid * per, k_hi = min(N, k_lo + per);
    const int q = qblk * kQW + c;
    const bool qvalid = q < N;

    float qr[32];
    {
        const float qs = scale * kLog2e;
        const floatx4* src = reinterpret_cast<const floatx4*>(qb + (size_t)(qvalid ? q : 0) * tok + 32 * h);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const floatx4 t = src[i];
            qr[4 * i] = t.x * qs;
            qr[4 * i + 1] = t.y * qs;
            qr[4 * i + 2] = t.z * qs;
            qr[4 * i + 3] = t.w * qs;
        }
    }
    auto load_tile = [&](int k0, Tile& t) {
        const int kr = min(k0 + c, N - 1);  // clamped row; masked below
        const floatx4* ks = reinterpret_cast<const floatx4*>(kb + (size_t)kr * tok + 32 * h);
#pragma unroll
        for (int i = 0; i < 8; ++i) t.k[i] = ks[i];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int vr = min(k0 + 8 * u + 4 * h + j, N - 1);
                const float* vs = vb + (size_t)vr * tok + c;
                t.v[(u * 4 + j) * 2] = vs[0];
                t.v[(u * 4 + j) * 2 + 1] = vs[32];
            }
    };

    floatx16 o[2];
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;
    Tile cur, nxt;
    if (k_lo < k_hi) load_tile(k_lo, cur);
    for (int k0 = k_lo; k0 < k_hi; k0 += kKT) {
        const bool has_next = k0 + kKT < k_hi;
        if (has_next) load_tile(k0 + kKT, nxt);
        // S^T[key 8(r >> 2) + 4h + (r & 3)][query c]; k-step t contracts dims {t, 32 + t}
        floatx16 s;
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            s = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.k[i].x, qr[4 * i + 0], s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.k[i].y, qr[4 * i + 1], s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.k[i].z, qr[4 * i + 2], s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.k[i].w, qr[4 * i + 3], s, 0, 0, 0);
        }
        // keys past this wave's range score -inf (their exp is exactly 0)
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (k0 + 8 * (r >> 2) + 4 * h + (r & 3) >= k_hi) s[r] = -INFINITY;
        float bmax = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) bmax = fmaxf(bmax, s[r]);
        bmax = halves_max(bmax);
        const float m_new = fmaxf(m_run, bmax);
        if (__any(m_new > m_run)) {
            const float corr = __builtin_amdgcn_exp2f(m_run - m_new);
            l_run *= corr;
            o[0] *= corr;
            o[1] *= corr;
            m_run = m_new;
        }
        float bsum = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float e = __builtin_amdgcn_exp2f(s[r] - m_run);
            s[r] = e;
            bsum += e;
        }
        l_run += halves_sum(bsum);
        // O^T[d = 32 dt + 8(r >> 2) + 4h + (r & 3)][query c] += V^T P^T, k-step (u, j) contracts keys
        // {8u + j, 8u + 4 + j} (lane halves): B = the S^T register 4u + j itself
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                o[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.v[(u * 4 + j) * 2], s[4 * u + j], o[0], 0, 0, 0);
                o[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur.v[(u * 4 + j) * 2 + 1], s[4 * u + j], o[1], 0, 0, 0);
            }
        if (has_next) cur = nxt;
    }

    // merge the four key quarters: waves 0 and 1 finish d tiles 0 and 1
    if (h == 0) {
        sML[wid][0][c] = m_run;
        sML[wid][1][c] = l_run;
    }
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) sO[wid][dt][r][lane] = o[dt][r];
    __syncthreads();
    if (wid >= 2 || !qvalid) return;
    float mw[4], M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        mw[w] = sML[w][0][c];
        M = fmaxf(M, mw[w]);
    }
    float a[4], L = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        a[w] = mw[w] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mw[w] - M);
        L += a[w] * sML[w][1][c];
    }
    const float inv = 1.0f / L;
    float acc[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) t += a[w] * sO[w][wid][r][lane];
        acc[r] = t * inv;
    }
    // out[b][q][head][d], d = 32 wid + 8u + 4h + (0..3) in acc[4u .. 4u + 3]
    float* dst = out + (((size_t)b * N + q) * H + head) * kD + 32 * wid + 4 * h;
#pragma unroll
    for (int u = 0; u < 4; ++u)
        *reinterpret_cast<floatx4*>(dst + 8 * u) = (floatx4){acc[4 * u], acc[4 * u + 1], acc[4 * u + 2], acc[4 * u + 3]};
}

// ---------------------------------------------------------------------------------------------
// Channels-first legacy QKV attention of the depth predictor U-Nets (head dim 32).
//
// Semantics: reference src/model/encoder/matching/ldm_unet/unet.py QKVAttentionLegacy.forward:
// per (batch, head), rows q | k | v (channels-first), out = einsum("bts,bcs->bct",
// softmax((q * s)^T (k * s)), v) with s = 32^(-1/4) (applied once to the dot product here:
// s^2 = 1/sqrt(32)). use_cross_view_self_attn folds the V views into the token axis
// ("(v b) n t -> b n (v t)"): the kernel reads qkv [(v b), 3 * heads * 32, t] and writes out
// [(v b), heads * 32, t] in that layout directly (token T' = view * t + i), so the two rearrange
// copies disappear.
// At 16^2 x 2 views T = 512; 1 or 4 heads: latency-bound, so one workgroup = 8 waves on 32
// queries, each wave walking an eighth of the keys (no LDS, no barrier in the loop; channels-first
// rows make the K / Q operand loads coalesced across lanes and each lane's V run contiguous), the
// eight (max, sum, O) partials merged once through LDS.
constexpr int kCfD = 32;
constexpr int kCfWaves = 8;

__global__ void __launch_bounds__(kCfWaves * 64)
mha_cf32_kernel(const float* __restrict__ qkv, float* __restrict__ out, int B, int H, int tl, int T, float scale) {
    __shared__ float sO[kCfWaves][16][64];
    __shared__ float sML[kCfWaves][2][kQW];

    const int qblk = blockIdx.x, bh = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int c = lane & 31, h = lane >> 5;
    const int b = bh / H, head = bh - b * H;
    // element (row, token) of this (batch, head): view = token / tl
    const size_t vstride = (size_t)B * 3 * H * kCfD * tl;  // between views
    const float* base = qkv + ((size_t)b * 3 * H + (size_t)head * 3) * kCfD * tl;
    auto at = [&](int row, int tok) -> const float* {
        const int vw = tok / tl;
        return base + vw * vstride + (size_t)row * tl + (tok - vw * tl);
    };

    const int per = (T + kCfWaves - 1) / kCfWaves;
    const int k_lo = min(T, wid * per), k_hi = min(T, k_lo + per);
    const int q = qblk * kQW + c;
    const bool qvalid = q < T;

    // k-step t contracts dims {t, 16 + t}: this lane holds dim 16 h + t
    float qr[16];
    {
        const float qs = scale * kLog2e;
        const int qc = qvalid ? q : 0;
        const float* qp = at(16 * h, qc);
#pragma unroll
        for (int t = 0; t < 16; ++t) qr[t] = qp[(size_t)t * tl] * qs;
    }
    floatx16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;
    // this lane's K column (16 dims) and V row segment (16 keys) of a 32-key tile, the next tile's
    // loads issued before the current tile's MFMAs (a scheduling barrier keeps them there)
    auto load_tile = [&](int k0, float* kv, float* vv) {
        const int kr = min(k0 + c, T - 1);
        const float* kp = at(kCfD + 16 * h, kr);
#pragma unroll
        for (int t = 0; t < 16; ++t) kv[t] = kp[(size_t)t * tl];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) vv[u * 4 + j] = *at(2 * kCfD + c, min(k0 + 8 * u + 4 * h + j, T - 1));
    };
    float kv[16], vv[16], nk[16], nv[16];
    if (k_lo < k_hi) load_tile(k_lo, kv, vv);
    for (int k0 = k_lo; k0 < k_hi; k0 += kKT) {
        const bool has_next = k0 + kKT < k_hi;
        if (has_next) load_tile(k0 + kKT, nk, nv);
        __builtin_amdgcn_sched_barrier(0);
        // S^T[key 8(r >> 2) + 4h + (r & 3)][query c] = sum_d K[d][key] Q[d][query]
        floatx16 s;
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
        for (int t = 0; t < 16; ++t) s = __builtin_amdgcn_mfma_f32_32x32x2f32(kv[t], qr[t], s, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (k0 + 8 * (r >> 2) + 4 * h + (r & 3) >= k_hi) s[r] = -INFINITY;
        float bmax = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) bmax = fmaxf(bmax, s[r]);
        bmax = halves_max(bmax);
        const float m_new = fmaxf(m_run, bmax);
        if (__any(m_new > m_run)) {
            const float corr = __builtin_amdgcn_exp2f(m_run - m_new);
            l_run *= corr;
            o *= corr;
            m_run = m_new;
        }
        float bsum = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float e = __builtin_amdgcn_exp2f(s[r] - m_run);
            s[r] = e;
            bsum += e;
        }
        l_run += halves_sum(bsum);
        // O^T[d = 8(r >> 2) + 4h + (r & 3)][query c] += V^T P^T; k-step (u, j): keys {8u + j, 8u + 4 + j}
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) o = __builtin_amdgcn_mfma_f32_32x32x2f32(vv[u * 4 + j], s[4 * u + j], o, 0, 0, 0);
        if (has_next) {
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                kv[t] = nk[t];
                vv[t] = nv[t];
            }
        }
    }

    if (h == 0) {
        sML[wid][0][c] = m_run;
        sML[wid][1][c] = l_run;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) sO[wid][r][lane] = o[r];
    __syncthreads();
    // wave w finishes registers r = 2w, 2w + 1 of the merged tile
    if (!qvalid) return;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < kCfWaves; ++w) M = fmaxf(M, sML[w][0][c]);
    float a[kCfWaves], L = 0.f;
#pragma unroll
    for (int w = 0; w < kCfWaves; ++w) {
        const float mw = sML[w][0][c];
        a[w] = mw == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mw - M);
        L += a[w] * sML[w][1][c];
    }
    const float inv = 1.0f / L;
    const int vw = q / tl;
    float* dst = out + (((size_t)vw * B + b) * H + head) * kCfD * tl + (q - vw * tl);
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        const int r = 2 * wid + rr;
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < kCfWaves; ++w) t += a[w] * sO[w][r][lane];
        const int d = 8 * (r >> 2) + 4 * h + (r & 3);
        dst[(size_t)d * tl] = t * inv;
    }
}

// ---------------------------------------------------------------------------------------------
// The same attention on 16-query blocks with v_mfma_f32_16x16x4_f32 (the same fp32 FLOP rate as
// the 32x32x2 form). Why: at the DINOv2 shape the 32-query kernel makes 24 x 11 = 264 workgroups of
// 4 waves at 1 wave per SIMD (276 registers), so 8 CUs run a second workgroup after the first and a
// lone wave per SIMD exposes every load and softmax latency (SQ counters: 63 % of wave time in
// issue stalls). Here: 24 x 21 = 504 workgroups of W waves on 16 queries, each wave a tile-aligned
// share of the 16-key tiles (no per-wave key-range masking), ~100 registers, so every workgroup is
// resident at once and a SIMD's waves overlap one's softmax with another's MFMAs.
// Operand maps (lane = 16 g + c):
//   S^T = K Q^T, k-step t contracts dim 16 g + t at lane group g (any dim permutation is a valid
//     contraction order as long as A and B agree): A = K[key c][16 g + t], B = Q[query c][16 g + t]
//     -> each lane's K and Q operands are one 64-B contiguous run; s[i] = S^T[key 4 g + i][query c];
//   O^T += V^T P^T, k-step t contracts keys {4 g + t}: B = P^T[key 4 g + t][query c] = s[t] itself,
//     A = V[key 4 g + t][16 dt + c]; o[dt][i] = O^T[d = 16 dt + 4 g + i][query c].
// Per-query softmax statistics reduce over the 4 registers and the 4 lane groups.
template <int W>
__global__ void __launch_bounds__(W * 64)
mha16_f32_kernel(const float* __restrict__ qkv, float* __restrict__ out, int N, int H, float scale,
                 const float* __restrict__ bias) {
    __shared__ float sO[W][16][64];
    __shared__ float sML[W][2][16];

    // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs, so consecutive linear ids
    // would spread one (image, head)'s query blocks over every XCD's L2; remapped, XCD x runs the
    // logical ids [x * total / 8, (x + 1) * total / 8), i.e. whole (image, head) K / V sets
    const int nq = gridDim.x, total = nq * gridDim.y;
    int lin = blockIdx.x + blockIdx.y * nq;
    if ((total & 7) == 0) lin = (lin & 7) * (total >> 3) + (lin >> 3);
    const int bh = lin / nq, qblk = lin - bh * nq;
    const int b = bh / H, head = bh - b * H;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int c = lane & 15, g = lane >> 4;
    const size_t tok = (size_t)3 * H * kD;
    const float* base = qkv + (size_t)b * N * tok + (size_t)head * kD;
    const float* kb = base + (size_t)H * kD;
    const float* vb = base + (size_t)2 * H * kD;

    const int nt = (N + 15) / 16;
    const int t_lo = wid * nt / W, t_hi = (wid + 1) * nt / W;
    const int q = qblk * 16 + c;

    float qr[16];
    {
        const float qs = scale * kLog2e;
        const floatx4* src = reinterpret_cast<const floatx4*>(base + (size_t)min(q, N - 1) * tok + 16 * g);
        // the projection's bias (bias != null: qkv holds x W^T without it): q's part added here; k's part
        // shifts every score of a query by the same b_k . q, which the softmax cancels, so it is
        // dropped; v's part is added to the normalised output (the weights sum to 1)
        const floatx4* bq = reinterpret_cast<const floatx4*>(bias + (size_t)head * kD + 16 * g);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const floatx4 t = bias ? src[i] + bq[i] : src[i];
            qr[4 * i] = t.x * qs;
            qr[4 * i + 1] = t.y * qs;
            qr[4 * i + 2] = t.z * qs;
            qr[4 * i + 3] = t.w * qs;
        }
    }
    struct Tile16 {
        floatx4 k[4];  // K[key c][16 g .. 16 g + 15]
        float v[16];   // V[key 4 g + t][16 dt + c] at t * 4 + dt
    };
    auto load_tile = [&](int tile, Tile16& T) {
        const int k0 = tile * 16;
        const floatx4* ks = reinterpret_cast<const floatx4*>(kb + (size_t)min(k0 + c, N - 1) * tok + 16 * g);
#pragma unroll
        for (int i = 0; i < 4; ++i) T.k[i] = ks[i];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const float* vs = vb + (size_t)min(k0 + 4 * g + t, N - 1) * tok + c;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) T.v[t * 4 + dt] = vs[16 * dt];
        }
    };

    floatx4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = (floatx4){0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.f;
    Tile16 cur, nxt;
    if (t_lo < t_hi) load_tile(t_lo, cur);
    for (int tile = t_lo; tile < t_hi; ++tile) {
        const bool has_next = tile + 1 < t_hi;
        if (has_next) load_tile(tile + 1, nxt);
        // two independent accumulation chains (dims 16 g + 0..7 / 8..15), summed once
        floatx4 s = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            s = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.k[i].x, qr[4 * i + 0], s, 0, 0, 0);
            s2 = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.k[i + 2].x, qr[4 * i + 8], s2, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.k[i].y, qr[4 * i + 1], s, 0, 0, 0);
            s2 = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.k[i + 2].y, qr[4 * i + 9], s2, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.k[i].z, qr[4 * i + 2], s, 0, 0, 0);
            s2 = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.k[i + 2].z, qr[4 * i + 10], s2, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.k[i].w, qr[4 * i + 3], s, 0, 0, 0);
            s2 = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.k[i + 2].w, qr[4 * i + 11], s2, 0, 0, 0);
        }
        s += s2;
        // keys past N (the last tile only) score -inf: their exp is exactly 0
        const int kg = tile * 16 + 4 * g;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (kg + i >= N) s[i] = -INFINITY;
        float bmax = fmaxf(fmaxf(s[0], s[1]), fmaxf(s[2], s[3]));
        bmax = halves_max(rows_max(bmax));
        const float m_new = fmaxf(m_run, bmax);  // finite: every tile holds a key < N
        if (__any(m_new > m_run)) {
            const float corr = __builtin_amdgcn_exp2f(m_run - m_new);
            l_run *= corr;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) o[dt] *= corr;
            m_run = m_new;
        }
        float bsum = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            s[i] = __builtin_amdgcn_exp2f(s[i] - m_run);
            bsum += s[i];
        }
        l_run += halves_sum(rows_sum(bsum));
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.v[t * 4 + dt], s[t], o[dt], 0, 0, 0);
        if (has_next) cur = nxt;
    }

    // merge the W key shares
    if (g == 0) {
        sML[wid][0][c] = m_run;
        sML[wid][1][c] = l_run;
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) sO[wid][dt * 4 + i][lane] = o[dt][i];
    __syncthreads();
    // 16 queries x 16 runs of 4 dims: run j holds d = 4 j .. 4 j + 3 = 16 dt + 4 g' + i (dt = j >> 2,
    // g' = j & 3) of query qq, i.e. sO[w][4 dt + i][16 g' + qq]
    if (tid >= 256) return;
    const int qq = tid >> 4, j = tid & 15;
    const int qo = qblk * 16 + qq;
    if (qo >= N) return;
    float mw[W], M = -INFINITY;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        mw[w] = sML[w][0][qq];
        M = fmaxf(M, mw[w]);
    }
    float a[W], L = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        a[w] = mw[w] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mw[w] - M);
        L += a[w] * sML[w][1][qq];
    }
    const float inv = 1.0f / L;
    float acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < W; ++w) t += a[w] * sO[w][(j >> 2) * 4 + i][(j & 3) * 16 + qq];
        acc[i] = t * inv;
        if (bias) acc[i] += bias[(size_t)(2 * H + head) * kD + 4 * j + i];
    }
    float* dst = out + (((size_t)b * N + qo) * H + head) * kD + 4 * j;
    *reinterpret_cast<floatx4*>(dst) = (floatx4){acc[0], acc[1], acc[2], acc[3]};
}

// ---------------------------------------------------------------------------------------------
// Split-bf16 ("bf16x3") form of mha16_f32_kernel for the dense-layer mode of the C2 step (the
// reference's attention matmuls run under TF32, src/main.py:15). The projection output (+ its bias)
// is split once per call by split_qkv_kernel into hi / lo bf16 images (x = hi + lo, |x - hi - lo| <=
// 2^-16 |x|), and every product is hi*hi + hi*lo + lo*hi with fp32 accumulation:
//   S^T = K Q^T: two k-steps of v_mfma_f32_16x16x32_bf16 (lane group g holds dims 16 g + 8 s .. + 7 of
//     its key row / query row in k-step s) x 3 terms, instead of 16 v_mfma_f32_16x16x4_f32;
//   O^T += V^T P^T: per 16-dim block dt, v_mfma_f32_16x16x16_bf16 (A = V[key 4 g + j][16 dt + c],
//     B = the lane's own 4 probabilities, split) x 3 terms, instead of 16 fp32 MFMAs.
// Same operand / output maps, softmax and merge as mha16_f32_kernel; the biases live in the split
// image (q's scaled by scale * log2 e in registers after re-joining hi + lo exactly).
__global__ void __launch_bounds__(256) split_qkv_kernel(const float4* __restrict__ x, const float* __restrict__ bias,
                                                        int cols4, int64_t n4, uint2* __restrict__ hi,
                                                        uint2* __restrict__ lo) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        float4 v = x[i];
        if (bias) {
            const float4 b = reinterpret_cast<const float4*>(bias)[i % cols4];
            v.x += b.x;
            v.y += b.y;
            v.z += b.z;
            v.w += b.w;
        }
        const floatx4 f = {v.x, v.y, v.z, v.w};
        const bf16x4 h = __builtin_convertvector(f, bf16x4);
        const bf16x4 l = __builtin_convertvector(f - __builtin_convertvector(h, floatx4), bf16x4);
        hi[i] = __builtin_bit_cast(uint2, h);
        lo[i] = __builtin_bit_cast(uint2, l);
    }
}

typedef __bf16 bf16x8m __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4m __attribute__((ext_vector_type(4)));
typedef short shortx4m __attribute__((ext_vector_type(4)));

template <int W>
__global__ void __launch_bounds__(W * 64)
mha16_x3_kernel(const __bf16* __restrict__ qh_img, const __bf16* __restrict__ ql_img, float* __restrict__ out, int N,
                int H, float scale) {
    __shared__ float sO[W][16][64];
    __shared__ float sML[W][2][16];

    const int nq = gridDim.x, total = nq * gridDim.y;
    int lin = blockIdx.x + blockIdx.y * nq;
    if ((total & 7) == 0) lin = (lin & 7) * (total >> 3) + (lin >> 3);
    const int bh = lin / nq, qblk = lin - bh * nq;
    const int b = bh / H, head = bh - b * H;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int c = lane & 15, g = lane >> 4;
    const size_t tok = (size_t)3 * H * kD;
    const size_t off0 = (size_t)b * N * tok + (size_t)head * kD;
    const __bf16* kh_b = qh_img + off0 + (size_t)H * kD;
    const __bf16* kl_b = ql_img + off0 + (size_t)H * kD;
    const __bf16* vh_b = qh_img + off0 + (size_t)2 * H * kD;
    const __bf16* vl_b = ql_img + off0 + (size_t)2 * H * kD;

    const int nt = (N + 15) / 16;
    const int t_lo = wid * nt / W, t_hi = (wid + 1) * nt / W;
    const int q = qblk * 16 + c;

    // this lane's query row, dims 16 g .. 16 g + 15: re-joined (exact), scaled, split again
    bf16x8m qh[2], ql[2];
    {
        const float qs = scale * kLog2e;
        const size_t qo = off0 + (size_t)min(q, N - 1) * tok + 16 * g;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const bf16x8m h = *reinterpret_cast<const bf16x8m*>(qh_img + qo + 8 * s2);
            const bf16x8m l = *reinterpret_cast<const bf16x8m*>(ql_img + qo + 8 * s2);
            typedef float floatx8 __attribute__((ext_vector_type(8)));
            const floatx8 f = (__builtin_convertvector(h, floatx8) + __builtin_convertvector(l, floatx8)) * qs;
            qh[s2] = __builtin_convertvector(f, bf16x8m);
            ql[s2] = __builtin_convertvector(f - __builtin_convertvector(qh[s2], floatx8), bf16x8m);
        }
    }
    struct TileX3 {
        bf16x8m kh[2], kl[2];      // K[key c][16 g + 8 s .. + 7]
        __bf16 vh[16], vl[16];     // V[key 4 g + t][16 dt + c] at t * 4 + dt
    };
    auto load_tile = [&](int tile, TileX3& T) {
        const int k0 = tile * 16;
        const size_t ko = (size_t)min(k0 + c, N - 1) * tok + 16 * g;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            T.kh[s2] = *reinterpret_cast<const bf16x8m*>(kh_b + ko + 8 * s2);
            T.kl[s2] = *reinterpret_cast<const bf16x8m*>(kl_b + ko + 8 * s2);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const size_t vo = (size_t)min(k0 + 4 * g + t, N - 1) * tok + c;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                T.vh[t * 4 + dt] = vh_b[vo + 16 * dt];
                T.vl[t * 4 + dt] = vl_b[vo + 16 * dt];
            }
        }
    };

    floatx4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = (floatx4){0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.f;
    TileX3 cur, nxt;
    if (t_lo < t_hi) load_tile(t_lo, cur);
    for (int tile = t_lo; tile < t_hi; ++tile) {
        const bool has_next = tile + 1 < t_hi;
        if (has_next) load_tile(tile + 1, nxt);
        floatx4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.kl[s2], qh[s2], s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.kh[s2], ql[s2], s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.kh[s2], qh[s2], s, 0, 0, 0);
        }
        const int kg = tile * 16 + 4 * g;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (kg + i >= N) s[i] = -INFINITY;
        float bmax = fmaxf(fmaxf(s[0], s[1]), fmaxf(s[2], s[3]));
        bmax = halves_max(rows_max(bmax));
        const float m_new = fmaxf(m_run, bmax);
        if (__any(m_new > m_run)) {
            const float corr = __builtin_amdgcn_exp2f(m_run - m_new);
            l_run *= corr;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) o[dt] *= corr;
            m_run = m_new;
        }
        float bsum = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            s[i] = __builtin_amdgcn_exp2f(s[i] - m_run);
            bsum += s[i];
        }
        l_run += halves_sum(rows_sum(bsum));
        const bf16x4m ph = __builtin_convertvector(s, bf16x4m);
        const bf16x4m pl = __builtin_convertvector(s - __builtin_convertvector(ph, floatx4), bf16x4m);
        const shortx4m phs = __builtin_bit_cast(shortx4m, ph), pls = __builtin_bit_cast(shortx4m, pl);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            const bf16x4m vh4 = {cur.vh[dt], cur.vh[4 + dt], cur.vh[8 + dt], cur.vh[12 + dt]};
            const bf16x4m vl4 = {cur.vl[dt], cur.vl[4 + dt], cur.vl[8 + dt], cur.vl[12 + dt]};
            const shortx4m vhs = __builtin_bit_cast(shortx4m, vh4), vls = __builtin_bit_cast(shortx4m, vl4);
            o[dt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vls, phs, o[dt], 0, 0, 0);
            o[dt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vhs, pls, o[dt], 0, 0, 0);
            o[dt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vhs, phs, o[dt], 0, 0, 0);
        }
        if (has_next) cur = nxt;
    }

    if (g == 0) {
        sML[wid][0][c] = m_run;
        sML[wid][1][c] = l_run;
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) sO[wid][dt * 4 + i][lane] = o[dt][i];
    __syncthreads();
    if (tid >= 256) return;
    const int qq = tid >> 4, j = tid & 15;
    const int qo = qblk * 16 + qq;
    if (qo >= N) return;
    float mw[W], M = -INFINITY;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        mw[w] = sML[w][0][qq];
        M = fmaxf(M, mw[w]);
    }
    float a[W], L = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        a[w] = mw[w] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mw[w] - M);
        L += a[w] * sML[w][1][qq];
    }
    const float inv = 1.0f / L;
    float acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < W; ++w) t += a[w] * sO[w][(j >> 2) * 4 + i][(j & 3) * 16 + qq];
        acc[i] = t * inv;
    }
    float* dst = out + (((size_t)b * N + qo) * H + head) * kD + 4 * j;
    *reinterpret_cast<floatx4*>(dst) = (floatx4){acc[0], acc[1], acc[2], acc[3]};
}

}  // namespace mha
}  // namespace tsplat

extern "C" int tsplat_mha_bias_f32_fwd(const float* qkv, const float* bias, float* out, int32_t batch,
                                       int32_t tokens, int32_t heads, int32_t head_dim, float scale, void* stream_);

extern "C" int tsplat_mha_f32_fwd(const float* qkv, float* out, int32_t batch, int32_t tokens, int32_t heads,
                                  int32_t head_dim, float scale, void* stream_) {
    return tsplat_mha_bias_f32_fwd(qkv, nullptr, out, batch, tokens, heads, head_dim, scale, stream_);
}

extern "C" int tsplat_mha_bias_f32_fwd(const float* qkv, const float* bias, float* out, int32_t batch,
                                       int32_t tokens, int32_t heads, int32_t head_dim, float scale, void* stream_) {
    using namespace tsplat::mha;
    if (!qkv || !out || batch <= 0 || tokens <= 0 || heads <= 0 || head_dim != kD) return TSPLAT_EINVAL;
    if ((int64_t)batch * heads > 65535 || (reinterpret_cast<uintptr_t>(bias) & 15)) return TSPLAT_EINVAL;
    hipStream_t stream = (hipStream_t)stream_;
    // TSPLAT_MHA: "16" (default, 4 waves per 16-query block), "16x8" (8 waves), "32" (the
    // 32-query kernel); A/B knob. The bias form is the default kernel's.
    const char* env = getenv("TSPLAT_MHA");
    const int form = !env || bias ? 0 : (!strcmp(env, "32") ? 2 : (!strcmp(env, "16x8") ? 1 : 0));
    TSPLAT_PROF_BEGIN(tsplat::prof::kMha, stream);
    if (form == 2)
        hipLaunchKernelGGL(mha_f32_kernel, dim3((tokens + kQW - 1) / kQW, batch * heads), dim3(kThreads), 0, stream,
                           qkv, out, tokens, heads, scale);
    else if (form == 1)
        hipLaunchKernelGGL(mha16_f32_kernel<8>, dim3((tokens + 15) / 16, batch * heads), dim3(512), 0, stream, qkv,
                           out, tokens, heads, scale, nullptr);
    else
        hipLaunchKernelGGL(mha16_f32_kernel<4>, dim3((tokens + 15) / 16, batch * heads), dim3(256), 0, stream, qkv,
                           out, tokens, heads, scale, bias);
    TSPLAT_PROF_END(tsplat::prof::kMha, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" int tsplat_qkv_attention_cf_fwd(const float* qkv, float* out, int32_t batch, int32_t heads,
                                           int32_t views, int32_t tokens_per_view, int32_t head_dim, float scale,
                                           void* stream_) {
    using namespace tsplat::mha;
    if (!qkv || !out || batch <= 0 || heads <= 0 || views <= 0 || tokens_per_view <= 0 || head_dim != kCfD)
        return TSPLAT_EINVAL;
    if ((int64_t)batch * heads > 65535 || (int64_t)views * tokens_per_view >= (1 << 30)) return TSPLAT_EINVAL;
    const int tokens = views * tokens_per_view;
    hipStream_t stream = (hipStream_t)stream_;
    TSPLAT_PROF_BEGIN(tsplat::prof::kMha, stream);
    hipLaunchKernelGGL(mha_cf32_kernel, dim3((tokens + kQW - 1) / kQW, batch * heads), dim3(kCfWaves * 64), 0, stream,
                       qkv, out, batch, heads, tokens_per_view, tokens, scale);
    TSPLAT_PROF_END(tsplat::prof::kMha, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

extern "C" size_t tsplat_mha_x3_workspace_bytes(int32_t batch, int32_t tokens, int32_t heads, int32_t head_dim) {
    if (batch <= 0 || tokens <= 0 || heads <= 0 || head_dim <= 0) return 0;
    return (size_t)2 * batch * tokens * 3 * heads * head_dim * sizeof(__bf16);
}

extern "C" int tsplat_mha_x3_fwd(const float* qkv, const float* bias, float* out, void* workspace, int32_t batch,
                                 int32_t tokens, int32_t heads, int32_t head_dim, float scale, void* stream_) {
    using namespace tsplat::mha;
    if (!qkv || !out || !workspace || batch <= 0 || tokens <= 0 || heads <= 0 || head_dim != kD) return TSPLAT_EINVAL;
    if ((int64_t)batch * heads > 65535 || (reinterpret_cast<uintptr_t>(bias) & 15) ||
        (reinterpret_cast<uintptr_t>(qkv) & 15) || (reinterpret_cast<uintptr_t>(workspace) & 15))
        return TSPLAT_EINVAL;
    hipStream_t stream = (hipStream_t)stream_;
    const int64_t n = (int64_t)batch * tokens * 3 * heads * kD;
    __bf16* hi = (__bf16*)workspace;
    __bf16* lo = hi + n;
    const int64_t n4 = n / 4;
    const int blocks = (int)((n4 + 255) / 256 < 4096 ? (n4 + 255) / 256 : 4096);
    TSPLAT_PROF_BEGIN(tsplat::prof::kMha, stream);
    hipLaunchKernelGGL(split_qkv_kernel, dim3(blocks), dim3(256), 0, stream, (const float4*)qkv, bias,
                       3 * heads * kD / 4, n4, (uint2*)hi, (uint2*)lo);
    hipLaunchKernelGGL(mha16_x3_kernel<4>, dim3((tokens + 15) / 16, batch * heads), dim3(256), 0, stream, hi, lo, out,
                       tokens, heads, scale);
    TSPLAT_PROF_END(tsplat::prof::kMha, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

// The same attention on q / k / v already split into hi / lo bf16 images ([batch, tokens, 3 heads
// kD] each, the qkv projection's bias included): written by the projection GEMM's epilogue
// (tsplat_gemm_x3_fwd act 2), so the split pass and the fp32 qkv round trip are gone.
extern "C" int tsplat_mha_x3_presplit_fwd(const void* qkv_hi, const void* qkv_lo, float* out, int32_t batch,
                                          int32_t tokens, int32_t heads, int32_t head_dim, float scale,
                                          void* stream_) {
    using namespace tsplat::mha;
    if (!qkv_hi || !qkv_lo || !out || batch <= 0 || tokens <= 0 || heads <= 0 || head_dim != kD) return TSPLAT_EINVAL;
    if ((int64_t)batch * heads > 65535 || (reinterpret_cast<uintptr_t>(qkv_hi) & 15) ||
        (reinterpret_cast<uintptr_t>(qkv_lo) & 15) ||
        (const char*)qkv_lo - (const char*)qkv_hi != (int64_t)batch * tokens * 3 * heads * kD * 2)
        return TSPLAT_EINVAL;  // the kernel takes lo at hi + n (one workspace-shaped image)
    hipStream_t stream = (hipStream_t)stream_;
    TSPLAT_PROF_BEGIN(tsplat::prof::kMha, stream);
    hipLaunchKernelGGL(mha16_x3_kernel<4>, dim3((tokens + 15) / 16, batch * heads), dim3(256), 0, stream,
                       (const __bf16*)qkv_hi, (const __bf16*)qkv_lo, out, tokens, heads, scale);
    TSPLAT_PROF_END(tsplat::prof::kMha, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
