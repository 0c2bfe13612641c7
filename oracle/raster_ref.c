/*
 * oracle/raster_ref.c — TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
 *
 * Scalar CPU restatement of the forward Gaussian rasterizer that the reference calls through
 * `GaussianRasterizer` (diff-gaussian-rasterization-modified, git dependency in the reference's
 * requirements.txt:17, un-vendored and unpinned -> the upstream graphdeco forward algorithm is
 * restated here). Call-site conventions follow render_cuda (reference
 * src/model/decoder/cuda_splatting.py:56-136):
 *   - scale invariance: means * (1/near), cov * (1/near)^2            (:73-80)
 *   - cov3D_precomp = upper triangle (xx, xy, xz, yy, yz, zz)          (:124,132)
 *   - shs = harmonics transposed to [G, M, 3]; degree = isqrt(M) - 1   (:82-84)
 *   - viewmatrix = inverse(c2w)^T, projmatrix = viewmatrix @ P^T       (:93-96)
 * Rasterizer stages restated (graphdeco forward.cu):
 *   preprocess: in_frustum (z_view <= 0.2 culled), p_proj = full * p / (w + 1e-7),
 *     computeCov2D (EWA, tx/tz and ty/tz clamped to +-1.3 tan(fov/2), +0.3 on the diagonal),
 *     det == 0 culled, conic, lambda = mid +- sqrt(max(0.1, mid^2 - det)), r = ceil(3 sqrt(lmax)),
 *     ndc2Pix, getRect (16x16 tiles, (int) truncation), empty rect culled, SH -> RGB (+0.5, >= 0)
 *   binning: every (gaussian, tile) instance ordered by (tile, depth, gaussian id) — the order of
 *     the stable radix sort over id-ordered duplicates keyed (tile << 32 | depth bits)
 *   render: per pixel at integer coordinates, front to back (explicit fmaf where the kernel uses
 *     v_fma_f32, identical sequence): power = -0.5(a dx^2 + c dy^2) - b dx dy, evaluated as
 *     fmaf(dy, fmaf(-c/2, dy, -b dx), (-a/2 dx) dx) (the reference's CUDA build contracts its
 *     expression into FMAs too; the exact op order is the rasterizer's choice, not a semantic),
 *     skip power > 0, alpha = min(0.99, o exp(power)), skip alpha < 1/255, stop when
 *     T (1 - alpha) < 1e-4, C += rgb alpha T; out = C + T bg.
 * Parity: unpinned against the reference CUDA binary (not available anywhere);
 * the op sequence (and the exp polynomial) is kept identical to the HIP kernel so the two agree
 * bit for bit on identical inputs. Compile with -O2 -ffp-contract=off (see oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define TILE 16

static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};
static const float SH_C4[9] = {2.5033429417967046f, -1.7701307697799304f, 0.9461746957575601f,
                               -0.6690465435572892f, 0.10578554691520431f, -0.6690465435572892f,
                               0.47308734787878004f, -1.7701307697799304f, 0.6258357354491761f};

static float bits_to_float(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static uint32_t float_to_bits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

/* exp(x), x <= 0: Cephes reduction + degree-5 polynomial with explicit fmaf (same op order as
 * the kernel; fmaf is correctly rounded on both sides). */
static float ref_exp_neg(float x) {
    if (x < -87.0f) return 0.0f;
    const float kf = rintf(x * 1.44269504088896341f);
    float r = fmaf(kf, -0.693359375f, x);
    r = fmaf(kf, 2.12194440e-4f, r);
    const float z = r * r;
    float p = 1.9875691500e-4f;
    p = fmaf(p, r, 1.3981999507e-3f);
    p = fmaf(p, r, 8.3334519073e-3f);
    p = fmaf(p, r, 4.1665795894e-2f);
    p = fmaf(p, r, 1.6666665459e-1f);
    p = fmaf(p, r, 5.0000001201e-1f);
    p = fmaf(p, z, r) + 1.0f;
    const int k = (int)kf;
    return p * bits_to_float((uint32_t)(k + 127) << 23);
}

static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }

static void get_rect(float px, float py, int r, int tx, int ty, int* x0, int* y0, int* x1, int* y1) {
    *x0 = imin(tx, imax(0, (int)((px - (float)r) / (float)TILE)));
    *y0 = imin(ty, imax(0, (int)((py - (float)r) / (float)TILE)));
    *x1 = imin(tx, imax(0, (int)((px + (float)r + (float)(TILE - 1)) / (float)TILE)));
    *y1 = imin(ty, imax(0, (int)((py + (float)r + (float)(TILE - 1)) / (float)TILE)));
}

/* computeColorFromSH, coefficient k of channel c at sh[c*M + k] */
static void sh_to_rgb(const float* sh, int M, int deg, float dx, float dy, float dz, float out[3]) {
    float len = sqrtf(dx * dx + dy * dy + dz * dz);
    float x = dx / len, y = dy / len, z = dz / len;
    float xx = x * x, yy = y * y, zz = z * z;
    float xy = x * y, yz = y * z, xz = x * z;
    for (int c = 0; c < 3; ++c) {
        const float* s = sh + c * M;
        float r = SH_C0 * s[0];
        if (deg > 0) {
            r = r - SH_C1 * y * s[1] + SH_C1 * z * s[2] - SH_C1 * x * s[3];
            if (deg > 1) {
                r = r + SH_C2[0] * xy * s[4] + SH_C2[1] * yz * s[5] +
                    SH_C2[2] * (2.0f * zz - xx - yy) * s[6] + SH_C2[3] * xz * s[7] +
                    SH_C2[4] * (xx - yy) * s[8];
                if (deg > 2) {
                    r = r + SH_C3[0] * y * (3.0f * xx - yy) * s[9] + SH_C3[1] * xy * z * s[10] +
                        SH_C3[2] * y * (4.0f * zz - xx - yy) * s[11] +
                        SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * s[12] +
                        SH_C3[4] * x * (4.0f * zz - xx - yy) * s[13] +
                        SH_C3[5] * z * (xx - yy) * s[14] + SH_C3[6] * x * (xx - 3.0f * yy) * s[15];
                    if (deg > 3) {
                        r = r + SH_C4[0] * xy * (xx - yy) * s[16] +
                            SH_C4[1] * yz * (3.0f * xx - yy) * s[17] +
                            SH_C4[2] * xy * (7.0f * zz - 1.0f) * s[18] +
                            SH_C4[3] * yz * (7.0f * zz - 3.0f) * s[19] +
                            SH_C4[4] * (zz * (35.0f * zz - 30.0f) + 3.0f) * s[20] +
                            SH_C4[5] * xz * (7.0f * zz - 3.0f) * s[21] +
                            SH_C4[6] * (xx - yy) * (7.0f * zz - 1.0f) * s[22] +
                            SH_C4[7] * xz * (xx - 3.0f * yy) * s[23] +
                            SH_C4[8] * (xx * (xx - 3.0f * yy) - yy * (3.0f * xx - yy)) * s[24];
                    }
                }
            }
        }
        r = r + 0.5f;
        out[c] = r > 0.0f ? r : 0.0f;
    }
}

typedef struct {
    float px, py, ca, cb, cc, op, r, g, b, depth;
} Rec;

static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : (x > y);
}

/*
 * Render one view. Inputs use the same layouts as tsplat_raster_fwd for one view/scene:
 * means[G*3], cov[G*9], shs[G*3*M], opacity[G], viewmat[16], projmat[16] (column-major),
 * campos[3], tanfov[2], bg[3], scale[2] = (s, s*s). Outputs out_color[3*H*W], out_radii[G].
 * Returns the number of (gaussian, tile) instances, or -1 on allocation failure.
 */
/* OpenMP over Gaussians (preprocess) and tiles (sort, blend): every thread writes disjoint
 * outputs, so the image is bit-identical for any thread count. n <= 0 leaves the default. */
void tsplat_ref_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

int tsplat_ref_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

long tsplat_ref_raster_view(int G, int H, int W, int M, int deg, const float* means,
                            const float* cov, const float* shs, const float* opacity,
                            const float* vm, const float* pm, const float* campos,
                            const float* tanfov, const float* bg, const float* scale,
                            float* out_color, int32_t* out_radii) {
    const int tiles_x = (W + TILE - 1) / TILE, tiles_y = (H + TILE - 1) / TILE;
    const int T = tiles_x * tiles_y;
    const float s = scale[0], s2 = scale[1];
    Rec* rec = (Rec*)malloc(sizeof(Rec) * (size_t)(G > 0 ? G : 1));
    long* counts = (long*)calloc((size_t)T + 1, sizeof(long));
    if (!rec || !counts) return -1;

#pragma omp parallel for schedule(static)
    for (int g = 0; g < G; ++g) {
        int radius = 0;
        out_radii[g] = 0;
        const float mx = means[3 * g] * s, my = means[3 * g + 1] * s, mz = means[3 * g + 2] * s;
        const float vx = vm[0] * mx + vm[4] * my + vm[8] * mz + vm[12];
        const float vy = vm[1] * mx + vm[5] * my + vm[9] * mz + vm[13];
        const float vz = vm[2] * mx + vm[6] * my + vm[10] * mz + vm[14];
        if (!(vz > 0.2f)) continue;
        const float hx = pm[0] * mx + pm[4] * my + pm[8] * mz + pm[12];
        const float hy = pm[1] * mx + pm[5] * my + pm[9] * mz + pm[13];
        const float hw = pm[3] * mx + pm[7] * my + pm[11] * mz + pm[15];
        const float pw = 1.0f / (hw + 0.0000001f);
        const float ndc_x = hx * pw, ndc_y = hy * pw;
        const float* C = cov + 9 * (size_t)g;
        const float c00 = C[0] * s2, c01 = C[1] * s2, c02 = C[2] * s2;
        const float c11 = C[4] * s2, c12 = C[5] * s2, c22 = C[8] * s2;
        const float tfx = tanfov[0], tfy = tanfov[1];
        const float fx = (float)W / (2.0f * tfx), fy = (float)H / (2.0f * tfy);
        const float limx = 1.3f * tfx, limy = 1.3f * tfy;
        const float tz = vz;
        float tx = vx / tz, ty = vy / tz;
        tx = fminf(limx, fmaxf(-limx, tx)) * tz;
        ty = fminf(limy, fmaxf(-limy, ty)) * tz;
        const float j00 = fx / tz, j02 = -(fx * tx) / (tz * tz);
        const float j11 = fy / tz, j12 = -(fy * ty) / (tz * tz);
        const float m00 = j00 * vm[0] + j02 * vm[2];
        const float m01 = j00 * vm[4] + j02 * vm[6];
        const float m02 = j00 * vm[8] + j02 * vm[10];
        const float m10 = j11 * vm[1] + j12 * vm[2];
        const float m11 = j11 * vm[5] + j12 * vm[6];
        const float m12 = j11 * vm[9] + j12 * vm[10];
        const float u00 = m00 * c00 + m01 * c01 + m02 * c02;
        const float u01 = m00 * c01 + m01 * c11 + m02 * c12;
        const float u02 = m00 * c02 + m01 * c12 + m02 * c22;
        const float u10 = m10 * c00 + m11 * c01 + m12 * c02;
        const float u11 = m10 * c01 + m11 * c11 + m12 * c12;
        const float u12 = m10 * c02 + m11 * c12 + m12 * c22;
        const float a = u00 * m00 + u01 * m01 + u02 * m02 + 0.3f;
        const float b = u00 * m10 + u01 * m11 + u02 * m12;
        const float c = u10 * m10 + u11 * m11 + u12 * m12 + 0.3f;
        const float det = a * c - b * b;
        if (det == 0.0f) continue;
        const float det_inv = 1.0f / det;
        const float mid = 0.5f * (a + c);
        const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
        const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
        radius = (int)ceilf(3.0f * sqrtf(fmaxf(l1, l2)));
        const float px = ((ndc_x + 1.0f) * (float)W - 1.0f) * 0.5f;
        const float py = ((ndc_y + 1.0f) * (float)H - 1.0f) * 0.5f;
        int x0, y0, x1, y1;
        get_rect(px, py, radius, tiles_x, tiles_y, &x0, &y0, &x1, &y1);
        if ((x1 - x0) * (y1 - y0) == 0) continue;
        float rgb[3];
        sh_to_rgb(shs + (size_t)3 * M * g, M, deg, mx - campos[0], my - campos[1], mz - campos[2], rgb);
        Rec* q = &rec[g];
        q->px = px;
        q->py = py;
        /* conic (A, B, C) = (c, -b, a) / det, stored as (-A/2, -B, -C/2) (exact scalings) for
         * the blend's power = dy (-C/2 dy - B dx) + (-A/2 dx) dx */
        q->ca = -0.5f * (c * det_inv);
        q->cb = -(-b * det_inv);
        q->cc = -0.5f * (a * det_inv);
        q->op = opacity[g];
        q->r = rgb[0];
        q->g = rgb[1];
        q->b = rgb[2];
        q->depth = vz;
        out_radii[g] = radius;
    }
    /* per-tile counts (serial: cheap, and keeps the parallel preprocess free of shared writes) */
    for (int g = 0; g < G; ++g) {
        if (out_radii[g] <= 0) continue;
        int x0, y0, x1, y1;
        get_rect(rec[g].px, rec[g].py, out_radii[g], tiles_x, tiles_y, &x0, &y0, &x1, &y1);
        for (int yy = y0; yy < y1; ++yy)
            for (int xx = x0; xx < x1; ++xx) counts[yy * tiles_x + xx]++;
    }

    /* per-tile lists keyed (depth bits << 32 | id), sorted ascending */
    long* offs = (long*)calloc((size_t)T + 1, sizeof(long));
    long total = 0;
    for (int t = 0; t < T; ++t) {
        offs[t] = total;
        total += counts[t];
    }
    offs[T] = total;
    uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(total > 0 ? total : 1));
    long* cur = (long*)calloc((size_t)T, sizeof(long));
    if (!offs || !keys || !cur) return -1;
    for (int g = 0; g < G; ++g) {
        if (out_radii[g] <= 0) continue;
        int x0, y0, x1, y1;
        get_rect(rec[g].px, rec[g].py, out_radii[g], tiles_x, tiles_y, &x0, &y0, &x1, &y1);
        const uint64_t key = ((uint64_t)float_to_bits(rec[g].depth) << 32) | (uint32_t)g;
        for (int yy = y0; yy < y1; ++yy)
            for (int xx = x0; xx < x1; ++xx) {
                const int t = yy * tiles_x + xx;
                keys[offs[t] + cur[t]++] = key;
            }
    }
#pragma omp parallel for schedule(dynamic)
    for (int t = 0; t < T; ++t) qsort(keys + offs[t], (size_t)(offs[t + 1] - offs[t]), 8, cmp_u64);

    const size_t hwn = (size_t)H * W;
#pragma omp parallel for schedule(dynamic)
    for (int t = 0; t < T; ++t) {
        const int tx = t % tiles_x, ty = t / tiles_x;
        for (int ly = 0; ly < TILE; ++ly)
            for (int lx = 0; lx < TILE; ++lx) {
                const int pxi = tx * TILE + lx, pyi = ty * TILE + ly;
                if (pxi >= W || pyi >= H) continue;
                const float pfx = (float)pxi, pfy = (float)pyi;
                float Tr = 1.0f, C0 = 0.f, C1 = 0.f, C2 = 0.f;
                for (long k = offs[t]; k < offs[t + 1]; ++k) {
                    const Rec* q = &rec[(uint32_t)(keys[k] & 0xffffffffu)];
                    const float dx = q->px - pfx, dy = q->py - pfy;
                    const float power = fmaf(dy, fmaf(q->cc, dy, q->cb * dx), (q->ca * dx) * dx);
                    if (power > 0.0f) continue;
                    const float alpha = fminf(0.99f, q->op * ref_exp_neg(power));
                    if (alpha < 1.0f / 255.0f) continue;
                    const float test_T = fmaf(-alpha, Tr, Tr);
                    if (test_T < 0.0001f) break;
                    const float w = alpha * Tr;
                    C0 = fmaf(q->r, w, C0);
                    C1 = fmaf(q->g, w, C1);
                    C2 = fmaf(q->b, w, C2);
                    Tr = test_T;
                }
                const size_t pix = (size_t)pyi * W + pxi;
                out_color[pix] = C0 + Tr * bg[0];
                out_color[hwn + pix] = C1 + Tr * bg[1];
                out_color[2 * hwn + pix] = C2 + Tr * bg[2];
            }
    }
    free(rec);
    free(counts);
    free(offs);
    free(keys);
    free(cur);
    return total;
}
