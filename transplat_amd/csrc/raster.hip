// Gaussian-splat forward rasterizer for gfx950 (MI355X).
//
// Algorithm = the graphdeco forward rasterizer behind `GaussianRasterizer` as called by
// `render_cuda` (reference src/model/decoder/cuda_splatting.py:56-136): preprocess (cull at
// z_view <= 0.2, EWA 2-D covariance with the 1.3*tan(fov) clamp and +0.3 low-pass, conic, 3-sigma
// radius, 16x16 tile rect, SH -> RGB), binning of (Gaussian, tile) instances, front-to-back depth
// order per tile, alpha blending with the 1/255 skip, 0.99 cap and T < 1e-4 stop.
//
// MI355X-first structure (not a translation of the CUDA one):
//   * every view of every scene is rendered by ONE set of launches (blockIdx.y = view); the
//     reference loops views in Python with two host syncs per view;
//   * no global radix sort: tiles are binned by a block-aggregated counting pass (LDS histogram,
//     one global atomic per (block, tile)), and each tile's list is ordered inside the render
//     kernel, keyed (depth bits << 32 | gaussian id) -- exactly the (depth, id) order of the
//     reference's stable sort over id-ordered duplicates -- by an LDS counting sort on the depth
//     bits with a per-bucket rank fix-up (a bitonic network for short or clustered lists);
//   * one 64-byte record per (view, Gaussian) (mean, ellipse extents, conic, opacity, rgb, cull
//     constants), so the render kernel's gather of an entry touches one cache line;
//   * the blend is scalar fp32 (v_pk_fma_f32 has v_fma_f32's FLOP rate and packing costs moves;
//     built with -fno-slp-vectorize), 4 entries per LDS read group.
//
// Floating point: contraction is OFF in this file, so the view-space depth (the sort key) is the
// reference's transformPoint4x3 expression bit for bit -- the front-to-back order, ties included,
// is exactly the reference's. Everything else is this kernel's own arithmetic: the EWA covariance
// as (J R) Sigma (J R)^T, the power in the log2 domain (log2 e folded into the stored conic) and
// the hardware exp2 (v_exp_f32). Parity is held against oracle/raster_ref.c's LITERAL restatement
// of the upstream expressions to L-inf 1e-4, excluding only the pixels whose blend decisions the
// oracle flags as within a rounding margin of their thresholds (tests/test_raster.py).
#pragma clang fp contract(off)

#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "common.h"
#include "prof.h"

namespace tsplat {
namespace raster {

constexpr int kTile = 16;                 // BLOCK_X = BLOCK_Y of the reference rasterizer
constexpr int kTileThreads = kTile * kTile;
constexpr int kSortCap = 4096;            // tile lists up to this length are sorted in LDS
constexpr int kPreThreads = 256;
constexpr size_t kMaxLdsBytes = 160 * 1024;  // gfx950 LDS per workgroup
constexpr int kRecBytes = 64;             // per-(view, Gaussian) record (Workspace::rec)
constexpr int kRecFields = 9;             // x, y, conic a b c, opacity, r g b

__constant__ float kSH_C0 = 0.28209479177387814f;
__constant__ float kSH_C1 = 0.4886025119029199f;
__constant__ float kSH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                                -1.0925484305920792f, 0.5462742152960396f};
__constant__ float kSH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                                0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                                -0.5900435899266435f};
// Degree-4 real SH constants (same sign convention as the lower degrees).
__constant__ float kSH_C4[9] = {2.5033429417967046f, -1.7701307697799304f, 0.9461746957575601f,
                                -0.6690465435572892f, 0.10578554691520431f, -0.6690465435572892f,
                                0.47308734787878004f, -1.7701307697799304f, 0.6258357354491761f};

struct Workspace {
    // [V*G] 64-byte records, one per (view, Gaussian), so the render kernel's gather of an entry
    // touches one cache line (three SoA arrays cost three lines per entry):
    //   rec[4i + 0] pixel-space mean + half-extents of the alpha >= 1/255 ellipse
    //   rec[4i + 1] conic (a, b, c) as log2(e) (-a/2, -b, -c/2) (the blend's log2-domain power
    //               form) + opacity
    //   rec[4i + 2] rgb + view-space depth
    //   rec[4i + 3] block-cull constants: threshold q, -b/a, -b/c (ellipse_meets_block)
    float4* rec;
    uint32_t* counts;    // [V*T]
    uint32_t* offsets;   // [V*T + 1]
    uint32_t* cursor;    // [V*T]
    uint64_t* keys;      // [capacity]
};

__host__ __device__ inline Workspace carve(void* base, int G, int V, int T, int capacity,
                                           size_t* total) {
    Workspace w;
    size_t off = 0;
    char* p = (char*)base;
    auto take = [&](size_t bytes) {
        char* r = p ? p + off : nullptr;
        off = align_up(off + bytes, 256);
        return r;
    };
    size_t n = (size_t)V * G;
    w.rec = (float4*)take(n * kRecBytes);
    // counts + cursor contiguous so one memset clears both
    w.counts = (uint32_t*)take((size_t)2 * V * T * sizeof(uint32_t));
    w.cursor = w.counts ? w.counts + (size_t)V * T : nullptr;
    w.offsets = (uint32_t*)take(((size_t)V * T + 1) * sizeof(uint32_t));
    w.keys = (uint64_t*)take((size_t)capacity * sizeof(uint64_t));
    if (total) *total = off;
    return w;
}

struct Params {
    int G, V, vps, H, W, M, deg, tiles_x, tiles_y, T, capacity;
    int diag;  // timing diagnostics only (TSPLAT_RASTER_DIAG; output is wrong when != 0)
    int count_sort;  // 1: counting sort for long tile lists (default); 0: bitonic only (A/B)
    int view_rot;    // render: view v's workgroups take tiles rotated by v * view_rot (load balance)
    int sh_vec4;     // preprocess: every wave's SH block is 16-byte aligned (16-byte staging loads)
};

__device__ __forceinline__ void get_rect(float px, float py, int r, int tx, int ty, int& x0,
                                         int& y0, int& x1, int& y1) {
    // (int) truncation and clamps exactly as the reference getRect (auxiliary.h)
    x0 = min(tx, max(0, (int)((px - (float)r) / (float)kTile)));
    y0 = min(ty, max(0, (int)((py - (float)r) / (float)kTile)));
    x1 = min(tx, max(0, (int)((px + (float)r + (float)(kTile - 1)) / (float)kTile)));
    y1 = min(ty, max(0, (int)((py + (float)r + (float)(kTile - 1)) / (float)kTile)));
}

__device__ __forceinline__ void sh_to_rgb(const float* __restrict__ sh, int M, int deg, float dx,
                                          float dy, float dz, float out[3]) {
    // sh is colour-major [3][M]; coefficient k of channel c is sh[c*M + k]
    float len = sqrtf(dx * dx + dy * dy + dz * dz);
    float x = dx / len, y = dy / len, z = dz / len;
    float xx = x * x, yy = y * y, zz = z * z;
    float xy = x * y, yz = y * z, xz = x * z;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float* s = sh + c * M;
        float r = kSH_C0 * s[0];
        if (deg > 0) {
            r = r - kSH_C1 * y * s[1] + kSH_C1 * z * s[2] - kSH_C1 * x * s[3];
            if (deg > 1) {
                r = r + kSH_C2[0] * xy * s[4] + kSH_C2[1] * yz * s[5] +
                    kSH_C2[2] * (2.0f * zz - xx - yy) * s[6] + kSH_C2[3] * xz * s[7] +
                    kSH_C2[4] * (xx - yy) * s[8];
                if (deg > 2) {
                    r = r + kSH_C3[0] * y * (3.0f * xx - yy) * s[9] + kSH_C3[1] * xy * z * s[10] +
                        kSH_C3[2] * y * (4.0f * zz - xx - yy) * s[11] +
                        kSH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * s[12] +
                        kSH_C3[4] * x * (4.0f * zz - xx - yy) * s[13] +
                        kSH_C3[5] * z * (xx - yy) * s[14] + kSH_C3[6] * x * (xx - 3.0f * yy) * s[15];
                    if (deg > 3) {
                        r = r + kSH_C4[0] * xy * (xx - yy) * s[16] +
                            kSH_C4[1] * yz * (3.0f * xx - yy) * s[17] +
                            kSH_C4[2] * xy * (7.0f * zz - 1.0f) * s[18] +
                            kSH_C4[3] * yz * (7.0f * zz - 3.0f) * s[19] +
                            kSH_C4[4] * (zz * (35.0f * zz - 30.0f) + 3.0f) * s[20] +
                            kSH_C4[5] * xz * (7.0f * zz - 3.0f) * s[21] +
                            kSH_C4[6] * (xx - yy) * (7.0f * zz - 1.0f) * s[22] +
                            kSH_C4[7] * xz * (xx - 3.0f * yy) * s[23] +
                            kSH_C4[8] * (xx * (xx - 3.0f * yy) - yy * (3.0f * xx - yy)) * s[24];
                    }
                }
            }
        }
        r = r + 0.5f;
        out[c] = fmaxf(r, 0.0f);
    }
}

// --- K0: clear the per-tile counters (a kernel, not hipMemsetAsync: a memset captured into a
// hipGraph was observed on ROCm 7.2 to leave garbage in the counters on the second replay) ---
__global__ void __launch_bounds__(256) zero_kernel(uint4* __restrict__ p, size_t n4) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        p[i] = make_uint4(0u, 0u, 0u, 0u);
}

// --- K1: preprocess + per-tile instance counts ----------------------------------------------
// One thread per Gaussian for ALL views of its scene (blockIdx.y = scene): the scene-level inputs
// (mean, covariance, opacity, SH) are read once, not once per view. The SH block of a wave's 64
// Gaussians ([64][3][M] floats, contiguous) is staged into LDS by coalesced 16-byte loads: read
// per thread in place, every load instruction of the wave touches 64 cache lines (a 3M-float
// stride), which made the SH reads half of this kernel's time (TSPLAT_RASTER_DIAG=7 skips them).
constexpr int kMaxShFloats = 75;  // 3 (deg 4 + 1)^2
constexpr int kShStageIt = (kWave * kMaxShFloats / 4 + kWave - 1) / kWave;  // float4s per lane
__global__ void __launch_bounds__(kPreThreads)
preprocess_kernel(Params p, const float* __restrict__ means, const float* __restrict__ cov,
                  const float* __restrict__ shs, const float* __restrict__ opacity,
                  const float* __restrict__ viewmat, const float* __restrict__ projmat,
                  const float* __restrict__ campos, const float* __restrict__ tanfov,
                  const float* __restrict__ scene_scale, int32_t* __restrict__ out_radii,
                  Workspace ws) {
    extern __shared__ uint32_t hist[];  // [T]
    __shared__ __attribute__((aligned(16))) float s_sh[kPreThreads * kMaxShFloats];
    const int scene = blockIdx.y;
    const int lane = threadIdx.x % kWave, wid = threadIdx.x / kWave;
    const int g = blockIdx.x * kPreThreads + threadIdx.x;
    const int nf = 3 * p.M;
    const size_t sg = (size_t)scene * p.G + g;
    float* my_sh = s_sh + (size_t)threadIdx.x * nf;
    // the SH block's 16-byte loads are issued first and stay in flight through the geometry pass
    // below (pass 1: projection, EWA covariance, records without colour, tile counts, per view);
    // pass 2 stores them to LDS and evaluates the colours of every view
    const int gw0 = blockIdx.x * kPreThreads + wid * kWave;
    const int sh_total = max(0, min(kWave, p.G - gw0)) * nf;
    const float* sh_src = shs + (size_t)nf * ((size_t)scene * p.G + gw0);
    float* sh_dst = s_sh + (size_t)wid * kWave * nf;
    const bool stage4 = p.sh_vec4 && p.diag != 7;
    const int t4 = stage4 ? sh_total / 4 : 0;
    // 19 named registers, loaded unconditionally at a clamped index (held in an array across the
    // geometry pass, the staging lived in scratch memory)
    const float4* sh_src4 = reinterpret_cast<const float4*>(sh_src);
    const int t4c = max(t4 - 1, 0);
    const bool any4 = t4 > 0;
#define TSPLAT_SH_LD(e) \
    float4 shr##e = any4 ? sh_src4[min(lane + (e) * kWave, t4c)] : make_float4(0.f, 0.f, 0.f, 0.f);
    TSPLAT_SH_LD(0) TSPLAT_SH_LD(1) TSPLAT_SH_LD(2) TSPLAT_SH_LD(3) TSPLAT_SH_LD(4) TSPLAT_SH_LD(5)
    TSPLAT_SH_LD(6) TSPLAT_SH_LD(7) TSPLAT_SH_LD(8) TSPLAT_SH_LD(9) TSPLAT_SH_LD(10) TSPLAT_SH_LD(11)
    TSPLAT_SH_LD(12) TSPLAT_SH_LD(13) TSPLAT_SH_LD(14) TSPLAT_SH_LD(15) TSPLAT_SH_LD(16) TSPLAT_SH_LD(17)
    TSPLAT_SH_LD(18)
#undef TSPLAT_SH_LD
    static_assert(kShStageIt == 19, "staging registers are spelled out for 19 float4s per lane");
    // scene-level inputs, once for all views
    float m0 = 0.f, m1 = 0.f, m2 = 0.f, k00 = 0.f, k01 = 0.f, k02 = 0.f, k11 = 0.f, k12 = 0.f, k22 = 0.f,
          o = 0.f;
    if (g < p.G) {
        m0 = means[3 * sg];
        m1 = means[3 * sg + 1];
        m2 = means[3 * sg + 2];
        const float* C = cov + 9 * sg;
        k00 = C[0];
        k01 = C[1];
        k02 = C[2];
        k11 = C[4];
        k12 = C[5];
        k22 = C[8];
        o = opacity[sg];
    }

    uint32_t okmask = 0;  // bit vv: the Gaussian is rendered in view vv (vps <= 32, host-checked)
    for (int vv = 0; vv < p.vps; ++vv) {
        const int v = scene * p.vps + vv;
        for (int i = threadIdx.x; i < p.T; i += kPreThreads) hist[i] = 0;
        __syncthreads();  // hist cleared
        if (g < p.G) {
            const size_t vg = (size_t)v * p.G + g;
            const float* vm = viewmat + 16 * v;
            const float* pm = projmat + 16 * v;
            const float s = scene_scale[2 * v], s2 = scene_scale[2 * v + 1];
            int radius = 0;
            // scale-invariant rendering: means * s, cov * s^2 (cuda_splatting.py:73-80)
            const float mx = m0 * s, my = m1 * s, mz = m2 * s;
            // in_frustum: view-space depth test (auxiliary.h in_frustum)
            const float vx = vm[0] * mx + vm[4] * my + vm[8] * mz + vm[12];
            const float vy = vm[1] * mx + vm[5] * my + vm[9] * mz + vm[13];
            const float vz = vm[2] * mx + vm[6] * my + vm[10] * mz + vm[14];
            bool ok = vz > 0.2f;
            float px = 0.f, py = 0.f, conic_a = 0.f, conic_b = 0.f, conic_c = 0.f;
            float cov_a = 0.f, cov_c = 0.f;
            int x0 = 0, y0 = 0, x1 = 0, y1 = 0;
            if (ok) {
                const float hx = pm[0] * mx + pm[4] * my + pm[8] * mz + pm[12];
                const float hy = pm[1] * mx + pm[5] * my + pm[9] * mz + pm[13];
                const float hw = pm[3] * mx + pm[7] * my + pm[11] * mz + pm[15];
                const float pw = 1.0f / (hw + 0.0000001f);
                const float ndc_x = hx * pw, ndc_y = hy * pw;
                const float c00 = k00 * s2, c01 = k01 * s2, c02 = k02 * s2;
                const float c11 = k11 * s2, c12 = k12 * s2, c22 = k22 * s2;
                // EWA splatting (computeCov2D)
                const float tfx = tanfov[2 * v], tfy = tanfov[2 * v + 1];
                const float fx = (float)p.W / (2.0f * tfx), fy = (float)p.H / (2.0f * tfy);
                const float limx = 1.3f * tfx, limy = 1.3f * tfy;
                const float tz = vz;
                const float tx = fminf(limx, fmaxf(-limx, vx / tz)) * tz;
                const float ty = fminf(limy, fmaxf(-limy, vy / tz)) * tz;
                const float j00 = fx / tz, j02 = -(fx * tx) / (tz * tz);
                const float j11 = fy / tz, j12 = -(fy * ty) / (tz * tz);
                // M = J * R_w2c, R[r][c] = vm[c*4 + r]
                const float n00 = j00 * vm[0] + j02 * vm[2];
                const float n01 = j00 * vm[4] + j02 * vm[6];
                const float n02 = j00 * vm[8] + j02 * vm[10];
                const float n10 = j11 * vm[1] + j12 * vm[2];
                const float n11 = j11 * vm[5] + j12 * vm[6];
                const float n12 = j11 * vm[9] + j12 * vm[10];
                const float u00 = n00 * c00 + n01 * c01 + n02 * c02;
                const float u01 = n00 * c01 + n01 * c11 + n02 * c12;
                const float u02 = n00 * c02 + n01 * c12 + n02 * c22;
                const float u10 = n10 * c00 + n11 * c01 + n12 * c02;
                const float u11 = n10 * c01 + n11 * c11 + n12 * c12;
                const float u12 = n10 * c02 + n11 * c12 + n12 * c22;
                const float a = u00 * n00 + u01 * n01 + u02 * n02 + 0.3f;
                const float b = u00 * n10 + u01 * n11 + u02 * n12;
                const float c = u10 * n10 + u11 * n11 + u12 * n12 + 0.3f;
                const float det = a * c - b * b;
                cov_a = a;
                cov_c = c;
                ok = det != 0.0f;
                if (ok) {
                    const float det_inv = 1.0f / det;
                    conic_a = c * det_inv;
                    conic_b = -b * det_inv;
                    conic_c = a * det_inv;
                    const float mid = 0.5f * (a + c);
                    const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
                    const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
                    radius = (int)ceilf(3.0f * sqrtf(fmaxf(l1, l2)));
                    px = ((ndc_x + 1.0f) * (float)p.W - 1.0f) * 0.5f;
                    py = ((ndc_y + 1.0f) * (float)p.H - 1.0f) * 0.5f;
                    get_rect(px, py, radius, p.tiles_x, p.tiles_y, x0, y0, x1, y1);
                    ok = (x1 - x0) * (y1 - y0) != 0;
                }
            }
            if (ok) {
                okmask |= 1u << vv;
                // Conservative half-extents of the region where o * exp(power) >= 1/255 (power =
                // -Q/2, Q <= 2 ln(255 o)); lets a wave skip Gaussians that miss its 8x8 pixels.
                // Pure culling: pixels inside keep the exact reference arithmetic.
                float ex = INFINITY, ey = INFINITY;
                if (o == o) {
                    const float q = 2.0f * logf(255.0f * o);
                    if (q < 0.0f) {
                        ex = ey = -1.0f;  // alpha < 1/255 everywhere
                    } else if (cov_a > 0.0f && cov_c > 0.0f && q < INFINITY) {
                        ex = sqrtf(q * cov_a) * 1.001f + 0.01f;
                        ey = sqrtf(q * cov_c) * 1.001f + 0.01f;
                    }
                }
                float4* rec = ws.rec + 4 * vg;
                rec[0] = make_float4(px, py, ex, ey);
                // power * log2(e): alpha = o * 2^(power2) is one v_exp_f32 in the blend
                constexpr float kLog2e = 1.44269504088896341f;
                rec[1] = make_float4(-0.5f * kLog2e * conic_a, -kLog2e * conic_b, -0.5f * kLog2e * conic_c, o);
                // cull threshold in the same log2 units as the stored conic: 2 log2(255 o), + margins
                rec[3] = make_float4(2.0f * __log2f(255.0f * o) * 1.001f + 1.5e-3f,
                                     -conic_b * __builtin_amdgcn_rcpf(conic_a),
                                     -conic_b * __builtin_amdgcn_rcpf(conic_c), 0.0f);
                for (int ty = y0; ty < y1; ++ty)
                    for (int tx = x0; tx < x1; ++tx) atomicAdd(&hist[ty * p.tiles_x + tx], 1u);
            } else {
                radius = 0;
            }
            out_radii[vg] = radius;
        }
        __syncthreads();
        uint32_t* gcount = ws.counts + (size_t)v * p.T;
        for (int i = threadIdx.x; i < p.T; i += kPreThreads)
            if (hist[i]) atomicAdd(&gcount[i], hist[i]);
        // the next view's clear of hist[i] is by this same thread, after its read above
    }

    // pass 2: the staged SH to LDS (this wave's own block: a wave barrier orders it), then colours
    float4* sh_dst4 = reinterpret_cast<float4*>(sh_dst);
#define TSPLAT_SH_ST(e) \
    if (lane + (e) * kWave < t4) sh_dst4[lane + (e) * kWave] = shr##e;
    TSPLAT_SH_ST(0) TSPLAT_SH_ST(1) TSPLAT_SH_ST(2) TSPLAT_SH_ST(3) TSPLAT_SH_ST(4) TSPLAT_SH_ST(5)
    TSPLAT_SH_ST(6) TSPLAT_SH_ST(7) TSPLAT_SH_ST(8) TSPLAT_SH_ST(9) TSPLAT_SH_ST(10) TSPLAT_SH_ST(11)
    TSPLAT_SH_ST(12) TSPLAT_SH_ST(13) TSPLAT_SH_ST(14) TSPLAT_SH_ST(15) TSPLAT_SH_ST(16) TSPLAT_SH_ST(17)
    TSPLAT_SH_ST(18)
#undef TSPLAT_SH_ST
    if (p.diag != 7)
        for (int i = 4 * t4 + lane; i < sh_total; i += kWave) sh_dst[i] = sh_src[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int vv = 0; vv < p.vps; ++vv) {
        if (!((okmask >> vv) & 1u)) continue;
        const int v = scene * p.vps + vv;
        const float* vm = viewmat + 16 * v;
        const float s = scene_scale[2 * v];
        const float mx = m0 * s, my = m1 * s, mz = m2 * s;
        const float vz = vm[2] * mx + vm[6] * my + vm[10] * mz + vm[14];  // as in pass 1, bit for bit
        float rgb[3] = {0.5f, 0.5f, 0.5f};
        const float* cp = campos + 3 * v;
        if (p.diag != 7) sh_to_rgb(my_sh, p.M, p.deg, mx - cp[0], my - cp[1], mz - cp[2], rgb);
        ws.rec[4 * ((size_t)v * p.G + g) + 2] = make_float4(rgb[0], rgb[1], rgb[2], vz);
    }
}

// --- K3: scatter (gaussian, tile) instances into per-tile ranges ------------------------------
// The exclusive scan of the V*T tile counts is folded in (it was a single-workgroup launch of its
// own): each workgroup sums the counts of the views before its own and scans its view's T counts
// in LDS; the x = 0 workgroup of each view publishes that view's offsets for the render kernel,
// and the last view's also the total (offsets[V T]) and the capacity-overflow status.
__device__ __forceinline__ uint32_t block_sum_u32(uint32_t x, uint32_t* red) {
    const int lane = threadIdx.x % kWave, wid = threadIdx.x / kWave;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o);
    if (lane == 0) red[wid] = x;
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kPreThreads / kWave; ++w) t += red[w];
    return t;
}

__global__ void __launch_bounds__(kPreThreads)
scatter_kernel(Params p, const int32_t* __restrict__ radii, Workspace ws, int32_t* __restrict__ status) {
    extern __shared__ uint32_t lds[];  // hist[T], base[T], pre[T]
    uint32_t* hist = lds;
    uint32_t* base = lds + p.T;
    uint32_t* pre = lds + 2 * p.T;
    __shared__ uint32_t red[2][kPreThreads / kWave];
    const int v = blockIdx.y;
    const int g = blockIdx.x * kPreThreads + threadIdx.x;
    const int lane = threadIdx.x % kWave, wid = threadIdx.x / kWave;
    for (int i = threadIdx.x; i < p.T; i += kPreThreads) hist[i] = 0;
    // this view's tile counts: thread t owns the contiguous segment [t k, t k + k), k = ceil(T / 256)
    const uint32_t* vcount = ws.counts + (size_t)v * p.T;
    const int seg = (p.T + kPreThreads - 1) / kPreThreads;
    const int s0 = min(p.T, (int)threadIdx.x * seg), s1 = min(p.T, s0 + seg);
    uint32_t own = 0;
    for (int i = s0; i < s1; ++i) own += vcount[i];
    uint32_t prior = 0;  // counts of the views before this one
    for (size_t i = threadIdx.x; i < (size_t)v * p.T; i += kPreThreads) prior += ws.counts[i];
    prior = block_sum_u32(prior, red[0]);  // (its barrier also orders the hist clear)
    uint32_t incl = own;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, d, kWave);
        if (lane >= d) incl += y;
    }
    if (lane == kWave - 1) red[1][wid] = incl;
    __syncthreads();
    uint32_t run = prior + incl - own;
    for (int w = 0; w < wid; ++w) run += red[1][w];
    for (int i = s0; i < s1; ++i) {
        pre[i] = run;
        run += vcount[i];
    }
    if (blockIdx.x == 0) {
        uint32_t* off = ws.offsets + (size_t)v * p.T;
        for (int i = s0; i < s1; ++i) off[i] = pre[i];
        if (v == p.V - 1 && threadIdx.x == kPreThreads - 1) {  // holds the view's last segment
            ws.offsets[(size_t)p.V * p.T] = run;
            if (run > (uint32_t)p.capacity) atomicOr(status, 1);
        }
    }
    __syncthreads();
    int r = 0, x0 = 0, y0 = 0, x1 = 0, y1 = 0;
    uint64_t key_lo = 0, depth_bits = 0;
    const size_t vg = (size_t)v * p.G + g;
    if (g < p.G) {
        r = radii[vg];
        if (r > 0) {
            const float4 xy = ws.rec[4 * vg];
            get_rect(xy.x, xy.y, r, p.tiles_x, p.tiles_y, x0, y0, x1, y1);
            depth_bits = (uint64_t)__float_as_uint(ws.rec[4 * vg + 2].w);
            key_lo = (uint64_t)(uint32_t)g;
            for (int ty = y0; ty < y1; ++ty)
                for (int tx = x0; tx < x1; ++tx) atomicAdd(&hist[ty * p.tiles_x + tx], 1u);
        }
    }
    __syncthreads();
    uint32_t* gcur = ws.cursor + (size_t)v * p.T;
    for (int i = threadIdx.x; i < p.T; i += kPreThreads) {
        uint32_t h = hist[i];
        base[i] = h ? pre[i] + atomicAdd(&gcur[i], h) : 0u;
        hist[i] = 0;
    }
    __syncthreads();
    if (r > 0) {
        const uint64_t key = (depth_bits << 32) | key_lo;
        for (int ty = y0; ty < y1; ++ty)
            for (int tx = x0; tx < x1; ++tx) {
                const int t = ty * p.tiles_x + tx;
                const uint32_t pos = base[t] + atomicAdd(&hist[t], 1u);
                if (pos < (uint32_t)p.capacity) ws.keys[pos] = key;
            }
    }
}

// Bitonic sort (all-ascending "mirror" network) of n keys held in `buf`, virtual length
// next_pow2(n); positions >= n behave as +inf and never move, so no padding is written.
template <typename Ptr>
__device__ __forceinline__ void bitonic_sort(Ptr buf, int n) {
    int logP = 0;
    while ((1 << logP) < n) ++logP;
    const int half = (1 << logP) >> 1;
    for (int lk = 1; lk <= logP; ++lk) {
        for (int lj = lk - 1; lj >= 0; --lj) {
            const int j = 1 << lj;
            for (int i = threadIdx.x; i < half; i += kTileThreads) {
                const int blk = i >> lj, q = i & (j - 1);
                int a, b;
                if (lj == lk - 1) {  // first step of a merge: compare mirrored pairs
                    a = (blk << (lj + 1)) + q;
                    b = (blk << (lj + 1)) + (2 * j - 1 - q);
                } else {
                    a = (blk << (lj + 1)) + q;
                    b = a + j;
                }
                if (b < n) {
                    const uint64_t ka = buf[a], kb = buf[b];
                    if (ka > kb) {
                        buf[a] = kb;
                        buf[b] = ka;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// Register-resident bitonic sort of the n <= kSortCap keys in `buf` (LDS), ascending. Thread t
// holds positions t*E .. t*E + E - 1 (E = P / 256 for P = next_pow2(n) >= 256; positions >= n
// are +inf). The network is unrolled at compile time (template over log2 P), so every register
// index is static: stages whose partner distance j is below E run in registers, j < 64 E
// exchange with the partner lane by shuffles, and only j >= 64 E (at most 3 stages for 4096
// keys) go through LDS with barriers -- instead of one barrier-separated LDS pass per stage.
template <int E>
__device__ __forceinline__ void cas_step(uint64_t (&v)[E], int t, int k, int j, uint64_t* buf) {
    if (j < E) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int f = e ^ j;
            if (f > e) {
                const bool asc = (((t * E + e) & k) == 0);
                const uint64_t a = v[e], b = v[f];
                const bool sw = asc ? (a > b) : (a < b);
                v[e] = sw ? b : a;
                v[f] = sw ? a : b;
            }
        }
    } else if (j < 64 * E) {
        const int lane_xor = j / E;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int i = t * E + e;
            const uint32_t lo = __shfl_xor((uint32_t)v[e], lane_xor);
            const uint32_t hi = __shfl_xor((uint32_t)(v[e] >> 32), lane_xor);
            const uint64_t other = ((uint64_t)hi << 32) | lo;
            const bool take_min = ((i & j) == 0) == ((i & k) == 0);
            const uint64_t mn = v[e] < other ? v[e] : other, mx = v[e] < other ? other : v[e];
            v[e] = take_min ? mn : mx;
        }
    } else {
        __syncthreads();  // previous readers of buf are done
#pragma unroll
        for (int e = 0; e < E; ++e) buf[t * E + e] = v[e];
        __syncthreads();
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int i = t * E + e;
            const uint64_t other = buf[i ^ j];
            const bool take_min = ((i & j) == 0) == ((i & k) == 0);
            const uint64_t mn = v[e] < other ? v[e] : other, mx = v[e] < other ? other : v[e];
            v[e] = take_min ? mn : mx;
        }
    }
}

template <int LOGP>
__device__ __forceinline__ void bitonic_sort_regs_p(uint64_t* buf, int n) {
    constexpr int P = 1 << LOGP;
    constexpr int E = P / kTileThreads;
    const int t = threadIdx.x;
    uint64_t v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = t * E + e;
        v[e] = i < n ? buf[i] : ~0ull;
    }
#pragma unroll
    for (int lk = 1; lk <= LOGP; ++lk)
#pragma unroll
        for (int lj = lk - 1; lj >= 0; --lj) cas_step<E>(v, t, 1 << lk, 1 << lj, buf);
    __syncthreads();
    // sorted gaussian ids (the keys' low words) as a uint32 list at the start of buf
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = t * E + e;
        if (i < n) reinterpret_cast<uint32_t*>(buf)[i] = (uint32_t)v[e];
    }
    __syncthreads();
}

__device__ __forceinline__ void bitonic_sort_regs(uint64_t* buf, int n) {
    if (n <= 256) bitonic_sort_regs_p<8>(buf, n);
    else if (n <= 512) bitonic_sort_regs_p<9>(buf, n);
    else if (n <= 1024) bitonic_sort_regs_p<10>(buf, n);
    else if (n <= 2048) bitonic_sort_regs_p<11>(buf, n);
    else bitonic_sort_regs_p<12>(buf, n);
}

// Counting sort of a tile list on its depth bits, for lists longer than one bitonic register pass.
// Depths are positive floats, so their bit patterns order like the depths. bucket(d) = (d - dmin)
// >> s, with s the smallest shift that maps the tile's depth-bit range onto <= kBuckets buckets:
// monotone in depth, so concatenating the buckets in order is a depth order. Each thread holds E
// keys in registers (key i = t + 256 e, one coalesced load batch); the keys are scattered to their
// bucket's slice of `out` by LDS atomics, and a key's final slot in its bucket -- almost always 0-2
// keys -- is its bucket start + the number of bucket members with a smaller (depth bits << 32 | id)
// key, so the result is exactly the ascending key order the bitonic network produces. A tile
// whose depths cluster (some bucket holds more than kFixMax keys) returns false before anything
// is written and takes the bitonic path.
constexpr int kBuckets = 2048;
constexpr int kBucketBits = 11;
constexpr int kFixMax = 32;

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o));
    return x;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o));
    return x;
}

template <int E>
__device__ bool counting_sort_e(const uint64_t* __restrict__ keys, int n, uint64_t* out, uint32_t* cnt,
                                uint32_t* red) {
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
    constexpr int kPer = kBuckets / kTileThreads;  // consecutive buckets per thread in the scan
    uint64_t k[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = tid + e * kTileThreads;
        k[e] = i < n ? keys[i] : ~0ull;
    }
    for (int i = tid; i < kBuckets; i += kTileThreads) cnt[i] = 0;
    if (tid == 0) {
        red[0] = 0xffffffffu;
        red[1] = 0u;
        red[2] = 0u;
    }
    uint32_t lo = 0xffffffffu, hi = 0u;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if (tid + e * kTileThreads < n) {
            const uint32_t d = (uint32_t)(k[e] >> 32);
            lo = min(lo, d);
            hi = max(hi, d);
        }
    }
    lo = wave_min_u32(lo);
    hi = wave_max_u32(hi);
    __syncthreads();  // red and cnt initialised
    if (lane == 0) {
        atomicMin(&red[0], lo);
        atomicMax(&red[1], hi);
    }
    __syncthreads();
    const uint32_t dmin = red[0], range = red[1] - dmin;
    const int bits = range ? 32 - __clz(range) : 0;
    const int sh = bits > kBucketBits ? bits - kBucketBits : 0;
    uint32_t bk[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const bool valid = tid + e * kTileThreads < n;
        bk[e] = valid ? ((uint32_t)(k[e] >> 32) - dmin) >> sh : 0u;
        if (valid) atomicAdd(&cnt[bk[e]], 1u);
    }
    __syncthreads();
    // exclusive scan of the bucket counts (thread t owns buckets kPer t .. kPer t + kPer - 1) and
    // the largest bucket
    uint32_t c[kPer];
    uint32_t sum = 0, mx = 0;
#pragma unroll
    for (int e = 0; e < kPer; ++e) {
        c[e] = cnt[tid * kPer + e];
        sum += c[e];
        mx = max(mx, c[e]);
    }
    uint32_t incl = sum;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, kWave);
        if (lane >= d) incl += y;
    }
    mx = wave_max_u32(mx);
    __shared__ uint32_t wtot[kTileThreads / kWave];
    if (lane == kWave - 1) wtot[wid] = incl;
    if (lane == 0) atomicMax(&red[2], mx);
    __syncthreads();
    if (red[2] > (uint32_t)kFixMax) return false;  // uniform: every thread read the same value
    uint32_t run = incl - sum;
    for (int w = 0; w < wid; ++w) run += wtot[w];
#pragma unroll
    for (int e = 0; e < kPer; ++e) {
        cnt[tid * kPer + e] = run;
        run += c[e];
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e)
        if (tid + e * kTileThreads < n) out[atomicAdd(&cnt[bk[e]], 1u)] = k[e];
    __syncthreads();  // cnt[b] is now the end of bucket b
    uint32_t slot[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t b = tid + e * kTileThreads < n ? bk[e] : 0u;  // padding keys: any bucket
        const uint32_t s0 = b ? cnt[b - 1] : 0u, s1 = cnt[b];
        uint32_t r = 0;
        for (uint32_t j = s0; j < s1; ++j) r += out[j] < k[e];
        slot[e] = s0 + r;
    }
    __syncthreads();
    // every read of the 64-bit keys is done: leave the sorted gaussian ids (the keys' low words)
    // as a uint32 list at the start of the same LDS region
#pragma unroll
    for (int e = 0; e < E; ++e)
        if (tid + e * kTileThreads < n) reinterpret_cast<uint32_t*>(out)[slot[e]] = (uint32_t)k[e];
    __syncthreads();
    return true;
}

__device__ __forceinline__ bool counting_sort(const uint64_t* __restrict__ keys, int n, uint64_t* out,
                                              uint32_t* cnt, uint32_t* red) {
    if (n <= 2 * kTileThreads) return counting_sort_e<2>(keys, n, out, cnt, red);
    if (n <= 4 * kTileThreads) return counting_sort_e<4>(keys, n, out, cnt, red);
    if (n <= 8 * kTileThreads) return counting_sort_e<8>(keys, n, out, cnt, red);
    return counting_sort_e<16>(keys, n, out, cnt, red);
}

// Exact culling of one Gaussian against a pixel block: does the alpha >= 1/255 ellipse
// {d : a dx^2 + 2 b dx dy + c dy^2 <= q}, q = 2 ln(255 o), meet the rectangle of pixel centres
// [x0, x1] x [y0, y1]? The minimum of the (convex) quadratic over the rectangle is 0 when the
// centre is inside, else it lies on an edge (1-D minimisation, clamped). Conservative margins
// (relative 1e-3 on q plus 1e-3 absolute) keep every contributing Gaussian (the blend's float
// arithmetic differs from this by a few ulps), so images are unchanged; culls the corners the
// axis-aligned box test keeps for rotated / elongated splats.
__device__ __forceinline__ bool ellipse_meets_block(float mx, float my, float4 co, float4 cull, float x0, float x1,
                                                    float y0, float y1) {
    // co = log2(e) (-a/2, -b, -c/2) and o as stored; cull = (2 log2(255 o) * 1.001 + 1.5e-3, -b/a,
    // -b/c): Q and q both carry the log2(e) factor,
    // precomputed per (view, Gaussian) by the preprocess kernel (approximate reciprocals: a clamped
    // minimiser off by an ulp raises Q by O(ulp^2), far inside the margins above)
    const float a = -2.0f * co.x, b = -co.y, c = -2.0f * co.z;
    const float q = cull.x, kba = cull.y, kbc = cull.z;
    const float X0 = x0 - mx, X1 = x1 - mx, Y0 = y0 - my, Y1 = y1 - my;
    if (X0 <= 0.f && X1 >= 0.f && Y0 <= 0.f && Y1 >= 0.f) return true;
    if (!(a > 0.f && c > 0.f)) return true;  // degenerate: keep (the box test decided)
    // Q(dx, dy) = dx (a dx + 2 b dy) + c dy^2; along x = X the minimiser is dy = X (-b / c)
    const float b2 = 2.0f * b;
    auto Qf = [&](float dx, float dy) { return fmaf(dx, fmaf(b2, dy, a * dx), c * dy * dy); };
    const float qx0 = Qf(X0, fminf(fmaxf(X0 * kbc, Y0), Y1));
    const float qx1 = Qf(X1, fminf(fmaxf(X1 * kbc, Y0), Y1));
    const float qy0 = Qf(fminf(fmaxf(Y0 * kba, X0), X1), Y0);
    const float qy1 = Qf(fminf(fmaxf(Y1 * kba, X0), X1), Y1);
    return fminf(fminf(qx0, qx1), fminf(qy0, qy1)) <= q;
}

// --- K4: per-tile depth sort + front-to-back alpha blending ---------------------------------
// One workgroup per (tile, view); the tile list is sorted in LDS (counting sort, or the bitonic
// network), then each wave owns
// an 8x8 pixel block and walks the sorted list on its own in 64-entry chunks (no workgroup
// barriers, so a wave never waits for a busier neighbour): the chunk's records are fetched one
// chunk ahead, the entries whose alpha >= 1/255 box can touch the block are compacted in depth
// order into the wave's LDS slot (conservative, so exact) and blended branch-free; the wave
// leaves as soon as all its 64 pixels are saturated.
__global__ void __launch_bounds__(kTileThreads)
render_kernel(Params p, const float* __restrict__ bg, float* __restrict__ out_color,
              Workspace ws) {
    __shared__ uint64_t skeys[kSortCap];
    __shared__ uint32_t s_cnt[kBuckets];
    __shared__ uint32_t s_red[4];
    // per-wave compacted records of the current 64-entry chunk (waves progress independently),
    // field-major: one ds_read_b128 of a field gives 4 consecutive entries = 2 packed pairs
    __shared__ __attribute__((aligned(16))) float s_rec[kTileThreads / kWave][kRecFields][kWave];

    const int v = blockIdx.y;
    // Workgroup (tile, v) and (tile, v') share an XCD and a CU slot in dispatch order, and a
    // tile's cost is similar across the target views of a scene (central tiles are the heavy
    // ones), so without the per-view rotation every CU would get the same tile three times.
    // Rotating by whole tile rows keeps each XCD's band of rows contiguous (L2 reuse of records).
    int tile = xcd_remap(blockIdx.x, gridDim.x) + v * p.view_rot;
    tile %= p.T;
    const uint64_t t_begin = p.diag == 5 ? __builtin_amdgcn_s_memtime() : 0;
    int d_entries = 0, d_chunks = 0;  // diag 5 only
    const int tx = tile % p.tiles_x, ty = tile / p.tiles_x;
    const int t_idx = v * p.T + tile;
    uint32_t start = ws.offsets[t_idx];
    uint32_t end = ws.offsets[t_idx + 1];
    if (end > (uint32_t)p.capacity) end = (uint32_t)p.capacity;
    if (start > end) start = end;
    const int n = (int)(end - start);

    uint64_t* gkeys = ws.keys + start;
    const bool in_lds = n <= kSortCap;
    if (in_lds) {
        // lists longer than one register pass: counting sort on the depth bits (falls back to the
        // bitonic network when the tile's depths cluster)
        const bool try_count = p.count_sort && n > kTileThreads && p.diag != 3;
        const bool counted = try_count && counting_sort(gkeys, n, skeys, s_cnt, s_red);
        if (!counted) {
            for (int i = threadIdx.x; i < n; i += kTileThreads) skeys[i] = gkeys[i];
            __syncthreads();
            if (p.diag == 3) return;  // key load only
            bitonic_sort_regs(skeys, n);
        }
        if (p.diag == 2) return;  // key load + sort
    } else {
        bitonic_sort(gkeys, n);  // rare: very long tile list, sorted in place in global memory
    }
    // no workgroup barrier below this point: each wave walks the sorted list on its own

    const int wid = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    const int lx = (wid & 1) * 8 + (lane & 7), ly = (wid >> 1) * 8 + (lane >> 3);
    const int pxi = tx * kTile + lx, pyi = ty * kTile + ly;
    const float wx0 = (float)(tx * kTile + (wid & 1) * 8), wx1 = wx0 + 7.0f;
    const float wy0 = (float)(ty * kTile + (wid >> 1) * 8), wy1 = wy0 + 7.0f;
    const bool inside = pxi < p.W && pyi < p.H;
    bool done = !inside;
    const float pfx = (float)pxi, pfy = (float)pyi;
    float T = 1.0f;
    float C0 = 0.f, C1 = 0.f, C2 = 0.f;
    const size_t vbase = (size_t)v * p.G;
    const uint64_t lt_mask = (1ull << lane) - 1ull;
    float (*w_rec)[kWave] = s_rec[wid];

    // power = -0.5 (a dx^2 + c dy^2) - b dx dy, alpha = min(0.99, o e^power), T' = T (1 - alpha),
    // C += rgb alpha T (reference renderCUDA), here with the power scaled by log2(e) so that
    // e^power = 2^power2 is one v_exp_f32, and the quadratic in Horner form (2 FMAs + 3 multiplies).
    // Scalar fp32 on purpose: v_pk_fma_f32 has the same FLOP rate as v_fma_f32 (twice the cycles),
    // and packing the operands costs register moves.
    auto blend = [&](float x, float y, float ca, float cb, float cc, float o, float r, float g, float bl) {
        // (ca, cb, cc) = log2(e) (-a/2, -b, -c/2): power2 = dy (cc dy + cb dx) + (ca dx) dx
        const float dx = x - pfx, dy = y - pfy;
        const float power2 = fmaf(dy, fmaf(cc, dy, cb * dx), (ca * dx) * dx);
        const float alpha = fminf(0.99f, o * __builtin_amdgcn_exp2f(power2));
        const float test_T = fmaf(-alpha, T, T);
        // reference order: skip power > 0, skip alpha < 1/255, stop if test_T < 1e-4
        const bool contrib = !done && !(power2 > 0.0f) && !(alpha < 1.0f / 255.0f);
        const bool stop = contrib && (test_T < 0.0001f);
        const bool acc = contrib && !stop;
        const float w = acc ? alpha * T : 0.0f;  // a skipped entry adds c * 0 = +0: C unchanged
        C0 = fmaf(r, w, C0);
        C1 = fmaf(g, w, C1);
        C2 = fmaf(bl, w, C2);
        T = acc ? test_T : T;
        done = done || stop;
    };

    struct Quad {
        float4 f[kRecFields];
    };
    auto load_quad = [&](int i, Quad& q) {
#pragma unroll
        for (int f = 0; f < kRecFields; ++f) q.f[f] = *reinterpret_cast<const float4*>(&w_rec[f][i]);
    };
    auto blend_quad = [&](const Quad& q) {
        const float4* f = q.f;
        blend(f[0].x, f[1].x, f[2].x, f[3].x, f[4].x, f[5].x, f[6].x, f[7].x, f[8].x);
        blend(f[0].y, f[1].y, f[2].y, f[3].y, f[4].y, f[5].y, f[6].y, f[7].y, f[8].y);
        blend(f[0].z, f[1].z, f[2].z, f[3].z, f[4].z, f[5].z, f[6].z, f[7].z, f[8].z);
        blend(f[0].w, f[1].w, f[2].w, f[3].w, f[4].w, f[5].w, f[6].w, f[7].w, f[8].w);
    };

    const uint32_t* sids = reinterpret_cast<const uint32_t*>(skeys);  // sorted ids (n <= kSortCap)
    auto walk = [&](auto lds_tag) {
        constexpr bool kInLds = decltype(lds_tag)::value;
        // this lane's record of the next 64-entry chunk, fetched one chunk ahead
        float4 r_xy = make_float4(0.f, 0.f, 0.f, 0.f), r_co = r_xy, r_rgb = r_xy, r_cull = r_xy;
        bool r_valid = false;
        auto fetch = [&](int k) {
            r_valid = k < n;
            if (r_valid) {
                // the list's address space is static here, so the LDS read is a ds_read (a generic
                // load would wait on every outstanding load, the previous chunk's prefetch included)
                uint32_t gid;
                if constexpr (kInLds)
                    gid = sids[k];
                else
                    gid = (uint32_t)gkeys[k];
                const float4* rec = ws.rec + 4 * (vbase + gid);
                r_xy = rec[0];
                r_co = rec[1];
                r_rgb = rec[2];
                r_cull = rec[3];
            }
        };
        fetch(lane);
        for (int c0 = 0; c0 < n; c0 += kWave) {
            if (__all(done)) break;
            const float4 xy = r_xy, co = r_co, rgb = r_rgb, cull = r_cull;
            const bool valid = r_valid;
            fetch(c0 + kWave + lane);
            // order-preserving compaction of the chunk's entries whose alpha >= 1/255 box touches
            // this wave's 8x8 block
            bool hit = valid && !(xy.x + xy.z < wx0 || xy.x - xy.z > wx1 || xy.y + xy.w < wy0 ||
                                  xy.y - xy.w > wy1);
            if (hit) hit = ellipse_meets_block(xy.x, xy.y, co, cull, wx0, wx1, wy0, wy1);
            const uint64_t mask = __ballot(hit);
            const int m = p.diag == 4 ? 0 : __popcll(mask);
            d_entries += m;
            ++d_chunks;
            if (hit) {
                const int pos = __popcll(mask & lt_mask);
                w_rec[0][pos] = xy.x;
                w_rec[1][pos] = xy.y;
                w_rec[2][pos] = co.x;
                w_rec[3][pos] = co.y;
                w_rec[4][pos] = co.z;
                w_rec[5][pos] = co.w;
                w_rec[6][pos] = rgb.x;
                w_rec[7][pos] = rgb.y;
                w_rec[8][pos] = rgb.z;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // groups of 4 entries: one ds_read_b128 per field
            const int m4 = m & ~3;
            for (int i = 0; i < m4; i += 4) {
                Quad q;
                load_quad(i, q);
                blend_quad(q);
            }
            for (int i = m4; i < m; ++i)
                blend(w_rec[0][i], w_rec[1][i], w_rec[2][i], w_rec[3][i], w_rec[4][i], w_rec[5][i], w_rec[6][i],
                      w_rec[7][i], w_rec[8][i]);
            __builtin_amdgcn_wave_barrier();  // reads of this chunk's records precede the next writes
        }
    };
    if (in_lds)
        walk(std::true_type{});
    else
        walk(std::false_type{});
    if (p.diag == 5) {  // per-wave cost instead of colours: cycles since the start, entries, chunks
        C0 = (float)(__builtin_amdgcn_s_memtime() - t_begin);
        C1 = (float)d_entries;
        C2 = (float)d_chunks;
        T = 0.0f;
    }
    if (inside) {
        const size_t hw = (size_t)p.H * p.W;
        float* o = out_color + (size_t)v * 3 * hw + (size_t)pyi * p.W + pxi;
        const float* bgv = bg + 3 * v;
        o[0] = C0 + T * bgv[0];
        o[hw] = C1 + T * bgv[1];
        o[2 * hw] = C2 + T * bgv[2];
    }
}

}  // namespace raster
}  // namespace tsplat

using namespace tsplat;
using namespace tsplat::raster;

extern "C" size_t tsplat_raster_workspace_bytes(int32_t G, int32_t V, int32_t H, int32_t W,
                                                int32_t capacity) {
    const int T = ceil_div(W, kTile) * ceil_div(H, kTile);
    size_t total = 0;
    carve(nullptr, G, V, T, capacity, &total);
    return total;
}

extern "C" size_t tsplat_raster_num_rendered_offset(int32_t G, int32_t V, int32_t H, int32_t W) {
    const int T = ceil_div(W, kTile) * ceil_div(H, kTile);
    const Workspace w = carve((void*)(uintptr_t)0x100000, G, V, T, 1, nullptr);  // layout only
    return (size_t)((char*)(w.offsets + (size_t)V * T) - (char*)(uintptr_t)0x100000);
}

extern "C" int tsplat_raster_fwd(const tsplat_raster_desc* d, const float* means, const float* cov,
                                 const float* shs, const float* opacity, const float* viewmat,
                                 const float* projmat, const float* campos, const float* tanfov,
                                 const float* bg, const float* scene_scale, float* out_color,
                                 int32_t* out_radii, void* workspace, int32_t* status,
                                 void* stream_) {
    if (!d || !means || !cov || !shs || !opacity || !viewmat || !projmat || !campos || !tanfov ||
        !bg || !scene_scale || !out_color || !out_radii || !workspace || !status)
        return TSPLAT_EINVAL;
    if (d->num_gaussians <= 0 || d->num_views <= 0 || d->views_per_scene <= 0 ||
        d->num_views % d->views_per_scene != 0 || d->height <= 0 || d->width <= 0 ||
        d->sh_coeffs <= 0 || d->sh_degree < 0 || d->sh_degree > 4 ||
        (d->sh_degree + 1) * (d->sh_degree + 1) > d->sh_coeffs || d->capacity <= 0)
        return TSPLAT_EINVAL;
    hipStream_t stream = (hipStream_t)stream_;
    Params p;
    p.G = d->num_gaussians;
    p.V = d->num_views;
    p.vps = d->views_per_scene;
    p.H = d->height;
    p.W = d->width;
    p.M = d->sh_coeffs;
    p.deg = d->sh_degree;
    p.tiles_x = ceil_div(p.W, kTile);
    p.tiles_y = ceil_div(p.H, kTile);
    p.T = p.tiles_x * p.tiles_y;
    p.capacity = d->capacity;
    {
        const char* e = getenv("TSPLAT_RASTER_DIAG");
        p.diag = e ? atoi(e) : 0;
        const char* s = getenv("TSPLAT_RASTER_SORT");
        p.count_sort = !(s && !strcmp(s, "bitonic"));
        // rotation per view: about T / 3 tiles, rounded to whole rows (TSPLAT_RASTER_ROT=0: off)
        const char* r = getenv("TSPLAT_RASTER_ROT");
        const int rows = (p.tiles_y + 1) / 3;
        p.view_rot = (r && !strcmp(r, "0")) ? 0 : rows * p.tiles_x;
    }
    // every argument check before the first launch (a rejected call queues nothing)
    if (3 * p.M > kMaxShFloats || p.vps > 32) return TSPLAT_EINVAL;
    // scatter keeps 3 T uint32 of per-tile counters in LDS: up to gfx950's 160 KB per workgroup
    // (13,653 16x16 tiles, about 1860 x 1860 px); above 64 KB the kernel's dynamic-LDS limit is raised
    const size_t scatter_lds = (size_t)p.T * 3 * sizeof(uint32_t);
    if (scatter_lds > kMaxLdsBytes) return TSPLAT_EINVAL;
    if (scatter_lds > 64 * 1024 &&
        hipFuncSetAttribute(reinterpret_cast<const void*>(&scatter_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)scatter_lds) != hipSuccess)
        return TSPLAT_EINVAL;
    Workspace ws = carve(workspace, p.G, p.V, p.T, p.capacity, nullptr);

    TSPLAT_PROF_BEGIN(prof::kRasterAll, stream);
    {
        // counts + cursor: 2 V T uint32, padded by carve()'s 256-byte alignment to whole uint4s
        const size_t n4 = ceil_div((size_t)2 * p.V * p.T, (size_t)4);
        const int blocks = (int)std::min<size_t>(ceil_div(n4, (size_t)256), 1024);
        hipLaunchKernelGGL(zero_kernel, dim3(blocks), dim3(256), 0, stream, (uint4*)ws.counts, n4);
        TSPLAT_CHECK_LAUNCH();
    }
    const int scenes = p.V / p.vps;
    // a wave's SH block starts at 3 M (scene G + 64 k) floats: 16-byte aligned when the base is
    // and 3 M G is a multiple of 4 (or there is one scene)
    p.sh_vec4 = ((uintptr_t)shs % 16 == 0) && (scenes == 1 || ((size_t)3 * p.M * p.G) % 4 == 0);
    dim3 pre_grid(ceil_div(p.G, kPreThreads), p.V);
    TSPLAT_PROF_BEGIN(prof::kRasterPreprocess, stream);
    hipLaunchKernelGGL(preprocess_kernel, dim3(ceil_div(p.G, kPreThreads), scenes), dim3(kPreThreads),
                       p.T * sizeof(uint32_t),
                       stream, p, means, cov, shs, opacity, viewmat, projmat, campos, tanfov,
                       scene_scale, out_radii, ws);
    TSPLAT_PROF_END(prof::kRasterPreprocess, stream);
    TSPLAT_CHECK_LAUNCH();
    TSPLAT_PROF_BEGIN(prof::kRasterScatter, stream);
    hipLaunchKernelGGL(scatter_kernel, pre_grid, dim3(kPreThreads), 3 * p.T * sizeof(uint32_t),
                       stream, p, (const int32_t*)out_radii, ws, status);
    TSPLAT_PROF_END(prof::kRasterScatter, stream);
    TSPLAT_CHECK_LAUNCH();
    TSPLAT_PROF_BEGIN(prof::kRasterRender, stream);
    hipLaunchKernelGGL(render_kernel, dim3(p.T, p.V), dim3(kTileThreads), 0, stream, p, bg,
                       out_color, ws);
    TSPLAT_PROF_END(prof::kRasterRender, stream);
    TSPLAT_PROF_END(prof::kRasterAll, stream);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}

// ---------------------------------------------------------------------------------------------
// Per-view camera constants of render_cuda (reference src/model/decoder/cuda_splatting.py:56-96,
// get_fov projection.py:233-247, get_projection_matrix cuda_splatting.py:26-53) in one launch,
// one thread per view: scale invariance (t, near, far scaled by 1/near), fov from K^-1 applied
// to the image-edge midpoints, tan(fov / 2), the projection matrix, view = inverse(c2w)^T,
// full = view @ proj^T. Replaces ~40 tiny PyTorch launches per decoder call.
namespace tsplat {
namespace raster {

template <int D>
__device__ void gj_inverse(const float* a_in, float* out) {
    float a[D][2 * D];
    for (int r = 0; r < D; ++r)
        for (int c = 0; c < D; ++c) {
            a[r][c] = a_in[r * D + c];
            a[r][D + c] = r == c ? 1.0f : 0.0f;
        }
    for (int col = 0; col < D; ++col) {
        int piv = col;
        for (int r = col + 1; r < D; ++r)
            if (fabsf(a[r][col]) > fabsf(a[piv][col])) piv = r;
        if (piv != col)
            for (int c = 0; c < 2 * D; ++c) {
                const float t = a[col][c];
                a[col][c] = a[piv][c];
                a[piv][c] = t;
            }
        const float inv = 1.0f / a[col][col];
        for (int c = 0; c < 2 * D; ++c) a[col][c] *= inv;
        for (int r = 0; r < D; ++r) {
            if (r == col) continue;
            const float f = a[r][col];
            for (int c = 0; c < 2 * D; ++c) a[r][c] -= f * a[col][c];
        }
    }
    for (int r = 0; r < D; ++r)
        for (int c = 0; c < D; ++c) out[r * D + c] = a[r][D + c];
}

__global__ void cameras_kernel(const float* __restrict__ ext, const float* __restrict__ intr,
                               const float* __restrict__ near_in, const float* __restrict__ far_in,
                               const float* __restrict__ bg_in, int bg_per_view, int scale_invariant, int V,
                               float* __restrict__ viewmat, float* __restrict__ projmat, float* __restrict__ campos,
                               float* __restrict__ tanfov, float* __restrict__ bg_out, float* __restrict__ scale_out) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    float e[16];
    for (int i = 0; i < 16; ++i) e[i] = ext[v * 16 + i];
    float nr = near_in[v], fr = far_in[v], s = 1.0f;
    if (scale_invariant) {
        s = 1.0f / nr;
        e[3] *= s;
        e[7] *= s;
        e[11] *= s;
        nr *= s;
        fr *= s;
    }
    float ki[9];
    gj_inverse<3>(intr + v * 9, ki);
    auto dir = [&](float x, float y, float d[3]) {
        float n2 = 0.f;
        for (int r = 0; r < 3; ++r) {
            d[r] = ki[3 * r] * x + ki[3 * r + 1] * y + ki[3 * r + 2];
            n2 += d[r] * d[r];
        }
        const float n = sqrtf(n2);
        for (int r = 0; r < 3; ++r) d[r] /= n;
    };
    float l[3], r_[3], t[3], b[3];
    dir(0.f, 0.5f, l);
    dir(1.f, 0.5f, r_);
    dir(0.5f, 0.f, t);
    dir(0.5f, 1.f, b);
    const float fov_x = acosf(l[0] * r_[0] + l[1] * r_[1] + l[2] * r_[2]);
    const float fov_y = acosf(t[0] * b[0] + t[1] * b[1] + t[2] * b[2]);
    const float tx = tanf(0.5f * fov_x), ty = tanf(0.5f * fov_y);
    // projection P (row-major), as get_projection_matrix builds it
    const float top = ty * nr, bottom = -top, right = tx * nr, left = -right;
    float P[16] = {0.f};
    P[0] = 2 * nr / (right - left);
    P[5] = 2 * nr / (top - bottom);
    P[2] = (right + left) / (right - left);
    P[6] = (top + bottom) / (top - bottom);
    P[14] = 1.0f;
    P[10] = fr / (fr - nr);
    P[11] = -(fr * nr) / (fr - nr);
    float w2c[16];
    gj_inverse<4>(e, w2c);
    // view_matrix = w2c^T; full = view_matrix @ P^T -> full[i][j] = sum_k w2c[k][i] P[j][k]
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            viewmat[v * 16 + i * 4 + j] = w2c[j * 4 + i];
            float acc = 0.f;
            for (int k = 0; k < 4; ++k) acc += w2c[k * 4 + i] * P[j * 4 + k];
            projmat[v * 16 + i * 4 + j] = acc;
        }
    campos[v * 3 + 0] = e[3];
    campos[v * 3 + 1] = e[7];
    campos[v * 3 + 2] = e[11];
    tanfov[v * 2 + 0] = tx;
    tanfov[v * 2 + 1] = ty;
    for (int c = 0; c < 3; ++c) bg_out[v * 3 + c] = bg_in[(bg_per_view ? v * 3 : 0) + c];
    scale_out[v * 2 + 0] = s;
    scale_out[v * 2 + 1] = s * s;
}

}  // namespace raster
}  // namespace tsplat

extern "C" int tsplat_raster_cameras(const float* extrinsics, const float* intrinsics, const float* near,
                                     const float* far, const float* bg, int32_t bg_per_view, int32_t scale_invariant,
                                     int32_t num_views, float* viewmat, float* projmat, float* campos, float* tanfov,
                                     float* bg_out, float* scale, void* stream_) {
    if (!extrinsics || !intrinsics || !near || !far || !bg || !viewmat || !projmat || !campos || !tanfov ||
        !bg_out || !scale || num_views <= 0)
        return TSPLAT_EINVAL;
    hipStream_t stream = (hipStream_t)stream_;
    hipLaunchKernelGGL(tsplat::raster::cameras_kernel, dim3((num_views + 63) / 64), dim3(64), 0, stream, extrinsics,
                       intrinsics, near, far, bg, bg_per_view, scale_invariant, num_views, viewmat, projmat, campos,
                       tanfov, bg_out, scale);
    TSPLAT_CHECK_LAUNCH();
    return TSPLAT_OK;
}
