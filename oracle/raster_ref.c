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
#include <stdio.h>
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

/* ============================================================================================
 * LITERAL mode: the upstream graphdeco forward written as its source states it, independent of
 * the HIP kernel's arithmetic (the kernel reorders the power, folds log2 e into the conic and
 * uses the hardware exp2). Op order followed term by term (compiled with -ffp-contract=off, i.e.
 * plain IEEE ops; nvcc's default --fmad=true would contract some of these, which is rounding-
 * level and is covered by the margins below):
 *   forward.cu preprocessCUDA / in_frustum (auxiliary.h): p_hom = transformPoint4x4(p, proj),
 *     p_w = 1 / (p_hom.w + 0.0000001f), p_view = transformPoint4x3(p, view), cull p_view.z <= 0.2
 *   computeCov2D: t clamped by 1.3 tan(fov / 2); J and W as glm::mat3 (column-major); T = W * J;
 *     cov = transpose(T) * transpose(Vrk) * T evaluated left to right with glm's mat3 product
 *     (Result[i][r] = A[0][r] B[i][0] + A[1][r] B[i][1] + A[2][r] B[i][2]); +0.3 on the diagonal
 *   det, det_inv = 1.f / det, conic = (c, -b, a) det_inv, mid, lambda1/2, r = ceil(3 sqrt(lmax))
 *   ndc2Pix(v, S) = ((v + 1.0) * S - 1.0) * 0.5 -- DOUBLE constants, so evaluated in double
 *   renderCUDA: d = xy - pixf; power = -0.5f * (con.x * d.x * d.x + con.z * d.y * d.y)
 *     - con.y * d.x * d.y; skip power > 0; alpha = min(0.99f, o * exp(power)) (libm expf);
 *     skip alpha < 1/255; test_T = T * (1 - alpha); stop (done) if test_T < 0.0001f;
 *     C += feature * alpha * T; T = test_T; out = C + T * bg.
 *
 * Threshold flags (out_flag / out_gflag, optional): the blend has discontinuous decisions
 * (z <= 0.2 cull, ceil of the radius, the (int) tile rect, power > 0, alpha < 1/255, T < 1e-4).
 * An implementation whose rounding differs from this one by a few ulps (any GPU kernel) may take
 * the other side of a decision that sits within that distance, changing a pixel by up to ~1/255.
 * Every decision is therefore also evaluated in a double-precision shadow (preprocess in double,
 * the blend's power / alpha / T in double along the float path's own decisions), and a decision
 * counts as ambiguous when the float value is within margin = 8 |float - double| + 16 ulp-scale
 * of its threshold. Pixels with an ambiguous decision (and Gaussians with an ambiguous radius,
 * rect or cull) are flagged; a parity test may exclude exactly those and must report how many.
 * Extra tiles that an ambiguous rect or radius could add are walked too, flagging the pixels
 * where that Gaussian would contribute, without blending it.
 * ============================================================================================ */

typedef struct {
    float px, py, A, B, C, op, r, g, b, depth;  /* literal float values, conic (A, B, C) */
    double pxd, pyd, Ad, Bd, Cd;                 /* double shadow */
    int x0, y0, x1, y1;                          /* nominal rect (empty when culled) */
    int ox0, oy0, ox1, oy1;                      /* outer rect (walked) */
    int ix0, iy0, ix1, iy1;                      /* inner rect (certain) */
} LRec;

typedef float gmat3[3][3]; /* glm layout: m[column][row] */

static void gmul(gmat3 A, gmat3 B, gmat3 R) {
    for (int i = 0; i < 3; ++i)
        for (int r = 0; r < 3; ++r) R[i][r] = A[0][r] * B[i][0] + A[1][r] * B[i][1] + A[2][r] * B[i][2];
}
static void gtrans(gmat3 A, gmat3 R) {
    for (int i = 0; i < 3; ++i)
        for (int r = 0; r < 3; ++r) R[i][r] = A[r][i];
}
typedef double dmat3[3][3];
static void dmul(dmat3 A, dmat3 B, dmat3 R) {
    for (int i = 0; i < 3; ++i)
        for (int r = 0; r < 3; ++r) R[i][r] = A[0][r] * B[i][0] + A[1][r] * B[i][1] + A[2][r] * B[i][2];
}
static void dtrans(dmat3 A, dmat3 R) {
    for (int i = 0; i < 3; ++i)
        for (int r = 0; r < 3; ++r) R[i][r] = A[r][i];
}

static const double kEps = 1.1920928955078125e-07; /* FLT_EPSILON */

/* out_flag bits: which decision was ambiguous at the pixel */
enum { kFlagRect = 1, kFlagPower = 2, kFlagAlpha = 4, kFlagT = 8 };

static int rect_area(int x0, int y0, int x1, int y1) { return (x1 - x0) * (y1 - y0); }

long tsplat_ref_raster_view_literal(int G, int H, int W, int M, int deg, const float* means,
                                    const float* cov, const float* shs, const float* opacity,
                                    const float* vm, const float* pm, const float* campos,
                                    const float* tanfov, const float* bg, const float* scale,
                                    float* out_color, int32_t* out_radii, uint8_t* out_flag,
                                    uint8_t* out_gflag) {
    const int tiles_x = (W + TILE - 1) / TILE, tiles_y = (H + TILE - 1) / TILE;
    const int T = tiles_x * tiles_y;
    const float s = scale[0], s2 = scale[1];
    const int flags = out_flag != NULL;
    LRec* rec = (LRec*)malloc(sizeof(LRec) * (size_t)(G > 0 ? G : 1));
    long* counts = (long*)calloc((size_t)T + 1, sizeof(long));
    if (!rec || !counts) return -1;

#pragma omp parallel for schedule(static)
    for (int g = 0; g < G; ++g) {
        LRec* q = &rec[g];
        memset(q, 0, sizeof(*q));
        out_radii[g] = 0;
        if (out_gflag) out_gflag[g] = 0;
        /* render_cuda hands the rasterizer means * s and cov * s^2 (cuda_splatting.py:73-80) */
        const float p0 = means[3 * g] * s, p1 = means[3 * g + 1] * s, p2 = means[3 * g + 2] * s;
        const float* Cm = cov + 9 * (size_t)g;
        const float cv[6] = {Cm[0] * s2, Cm[1] * s2, Cm[2] * s2, Cm[4] * s2, Cm[5] * s2, Cm[8] * s2};
        /* transformPoint4x4 / 4x3 */
        const float hx = pm[0] * p0 + pm[4] * p1 + pm[8] * p2 + pm[12];
        const float hy = pm[1] * p0 + pm[5] * p1 + pm[9] * p2 + pm[13];
        const float hw = pm[3] * p0 + pm[7] * p1 + pm[11] * p2 + pm[15];
        const float p_w = 1.0f / (hw + 0.0000001f);
        const float prx = hx * p_w, pry = hy * p_w;
        const float tvx = vm[0] * p0 + vm[4] * p1 + vm[8] * p2 + vm[12];
        const float tvy = vm[1] * p0 + vm[5] * p1 + vm[9] * p2 + vm[13];
        const float tvz = vm[2] * p0 + vm[6] * p1 + vm[10] * p2 + vm[14];
        /* double shadow of the same chain */
        const double d0 = p0, d1 = p1, d2 = p2;
        const double hxd = (double)pm[0] * d0 + (double)pm[4] * d1 + (double)pm[8] * d2 + pm[12];
        const double hyd = (double)pm[1] * d0 + (double)pm[5] * d1 + (double)pm[9] * d2 + pm[13];
        const double hwd = (double)pm[3] * d0 + (double)pm[7] * d1 + (double)pm[11] * d2 + pm[15];
        const double pwd = 1.0 / (hwd + 0.0000001);
        const double tvxd = (double)vm[0] * d0 + (double)vm[4] * d1 + (double)vm[8] * d2 + vm[12];
        const double tvyd = (double)vm[1] * d0 + (double)vm[5] * d1 + (double)vm[9] * d2 + vm[13];
        const double tvzd = (double)vm[2] * d0 + (double)vm[6] * d1 + (double)vm[10] * d2 + vm[14];
        const double zscale = fabs(vm[2] * p0) + fabs(vm[6] * p1) + fabs(vm[10] * p2) + fabs(vm[14]);
        const double mz = 8.0 * fabs((double)tvz - tvzd) + 16.0 * kEps * zscale;
        int unc = fabs((double)tvz - 0.2) <= mz;
        const int culled = !(tvz > 0.2f);
        if (culled && !unc) continue;
        if (!(tvz > 0.0f)) continue; /* behind the camera: no image position to speak of */

        /* computeCov2D (float, glm order) */
        const float tfx = tanfov[0], tfy = tanfov[1];
        const float focal_x = (float)W / (2.0f * tfx), focal_y = (float)H / (2.0f * tfy);
        const float limx = 1.3f * tfx, limy = 1.3f * tfy;
        const float txtz = tvx / tvz, tytz = tvy / tvz;
        const float tx = fminf(limx, fmaxf(-limx, txtz)) * tvz;
        const float ty = fminf(limy, fmaxf(-limy, tytz)) * tvz;
        gmat3 J = {{focal_x / tvz, 0.0f, -(focal_x * tx) / (tvz * tvz)},
                   {0.0f, focal_y / tvz, -(focal_y * ty) / (tvz * tvz)},
                   {0.0f, 0.0f, 0.0f}};
        gmat3 Wm = {{vm[0], vm[4], vm[8]}, {vm[1], vm[5], vm[9]}, {vm[2], vm[6], vm[10]}};
        gmat3 Vrk = {{cv[0], cv[1], cv[2]}, {cv[1], cv[3], cv[4]}, {cv[2], cv[4], cv[5]}};
        gmat3 Tm, Tt, Vt, TtVt, cv2;
        gmul(Wm, J, Tm);
        gtrans(Tm, Tt);
        gtrans(Vrk, Vt);
        gmul(Tt, Vt, TtVt);
        gmul(TtVt, Tm, cv2);
        cv2[0][0] += 0.3f;
        cv2[1][1] += 0.3f;
        const float ca = cv2[0][0], cb = cv2[0][1], cc = cv2[1][1];
        const float det = ca * cc - cb * cb;
        if (det == 0.0f) continue;
        const float det_inv = 1.f / det;
        q->A = cc * det_inv;
        q->B = -cb * det_inv;
        q->C = ca * det_inv;
        const float mid = 0.5f * (ca + cc);
        const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
        const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
        const float rf = 3.f * sqrtf(fmaxf(lambda1, lambda2));
        const int radius = (int)ceilf(rf);
        q->px = (float)((((double)prx + 1.0) * (double)W - 1.0) * 0.5);
        q->py = (float)((((double)pry + 1.0) * (double)H - 1.0) * 0.5);

        /* double shadow of computeCov2D, conic, radius, pixel position */
        const double tfxd = tfx, tfyd = tfy;
        const double fxd = (double)W / (2.0 * tfxd), fyd = (double)H / (2.0 * tfyd);
        const double txd = fmin(1.3 * tfxd, fmax(-1.3 * tfxd, tvxd / tvzd)) * tvzd;
        const double tyd = fmin(1.3 * tfyd, fmax(-1.3 * tfyd, tvyd / tvzd)) * tvzd;
        dmat3 Jd = {{fxd / tvzd, 0.0, -(fxd * txd) / (tvzd * tvzd)},
                    {0.0, fyd / tvzd, -(fyd * tyd) / (tvzd * tvzd)},
                    {0.0, 0.0, 0.0}};
        dmat3 Wd = {{vm[0], vm[4], vm[8]}, {vm[1], vm[5], vm[9]}, {vm[2], vm[6], vm[10]}};
        dmat3 Vd = {{cv[0], cv[1], cv[2]}, {cv[1], cv[3], cv[4]}, {cv[2], cv[4], cv[5]}};
        dmat3 Td, Ttd, Vtd, TVd, c2d;
        dmul(Wd, Jd, Td);
        dtrans(Td, Ttd);
        dtrans(Vd, Vtd);
        dmul(Ttd, Vtd, TVd);
        dmul(TVd, Td, c2d);
        const double cad = c2d[0][0] + 0.3, cbd = c2d[0][1], ccd = c2d[1][1] + 0.3;
        const double detd = cad * ccd - cbd * cbd;
        q->Ad = ccd / detd;
        q->Bd = -cbd / detd;
        q->Cd = cad / detd;
        const double midd = 0.5 * (cad + ccd);
        const double l1d = midd + sqrt(fmax(0.1, midd * midd - detd));
        const double l2d = midd - sqrt(fmax(0.1, midd * midd - detd));
        const double rfd = 3.0 * sqrt(fmax(l1d, l2d));
        q->pxd = ((hxd * pwd) + 1.0) * (double)W * 0.5 - 0.5;
        q->pyd = ((hyd * pwd) + 1.0) * (double)H * 0.5 - 0.5;

        /* radius and rect ambiguity */
        const double mr = 8.0 * fabs((double)rf - rfd) + 16.0 * kEps * rf;
        const int r_lo = (int)ceil(rf - mr), r_hi = (int)ceil(rf + mr);
        unc |= r_lo != r_hi;
        const double mpx = 8.0 * fabs((double)q->px - q->pxd) + 4.0 * kEps * (fabs(q->px) + (double)W);
        const double mpy = 8.0 * fabs((double)q->py - q->pyd) + 4.0 * kEps * (fabs(q->py) + (double)H);
        get_rect(q->px, q->py, radius, tiles_x, tiles_y, &q->x0, &q->y0, &q->x1, &q->y1);
        int ax0, ay0, ax1, ay1, bx0, by0, bx1, by1;
        /* outer: largest radius, position pushed outwards on each side; inner: the opposite */
        get_rect((float)(q->px - mpx), (float)(q->py - mpy), r_hi, tiles_x, tiles_y, &ax0, &ay0, &bx1, &by1);
        get_rect((float)(q->px + mpx), (float)(q->py + mpy), r_hi, tiles_x, tiles_y, &bx0, &by0, &ax1, &ay1);
        q->ox0 = imin(ax0, q->x0);
        q->oy0 = imin(ay0, q->y0);
        q->ox1 = imax(ax1, q->x1);
        q->oy1 = imax(ay1, q->y1);
        get_rect((float)(q->px + mpx), (float)(q->py + mpy), r_lo, tiles_x, tiles_y, &ax0, &ay0, &bx1, &by1);
        get_rect((float)(q->px - mpx), (float)(q->py - mpy), r_lo, tiles_x, tiles_y, &bx0, &by0, &ax1, &ay1);
        q->ix0 = imax(ax0, q->x0);
        q->iy0 = imax(ay0, q->y0);
        q->ix1 = imin(ax1, q->x1);
        q->iy1 = imin(ay1, q->y1);
        if (culled) { /* ambiguous cull: nothing is certain, nothing nominal */
            q->x0 = q->x1 = q->y0 = q->y1 = 0;
            q->ix0 = q->ix1 = q->iy0 = q->iy1 = 0;
        }
        if (q->ix1 < q->ix0) q->ix1 = q->ix0;
        if (q->iy1 < q->iy0) q->iy1 = q->iy0;
        unc |= q->ox0 != q->ix0 || q->oy0 != q->iy0 || q->ox1 != q->ix1 || q->oy1 != q->iy1;
        if (out_gflag) out_gflag[g] = (uint8_t)unc;
        if (rect_area(q->ox0, q->oy0, q->ox1, q->oy1) == 0) continue;
        float rgb[3];
        sh_to_rgb(shs + (size_t)3 * M * g, M, deg, p0 - campos[0], p1 - campos[1], p2 - campos[2], rgb);
        q->op = opacity[g];
        q->r = rgb[0];
        q->g = rgb[1];
        q->b = rgb[2];
        q->depth = tvz;
        if (!culled && rect_area(q->x0, q->y0, q->x1, q->y1) != 0) out_radii[g] = radius;
        else {
            q->x0 = q->x1 = q->y0 = q->y1 = 0;
        }
        if (!flags) { /* plain literal render: walk the nominal rect only */
            q->ox0 = q->x0; q->oy0 = q->y0; q->ox1 = q->x1; q->oy1 = q->y1;
        }
    }
    for (int g = 0; g < G; ++g) {
        const LRec* q = &rec[g];
        for (int yy = q->oy0; yy < q->oy1; ++yy)
            for (int xx = q->ox0; xx < q->ox1; ++xx) counts[yy * tiles_x + xx]++;
    }
    long* offs = (long*)calloc((size_t)T + 1, sizeof(long));
    long total = 0, nominal = 0;
    for (int t = 0; t < T; ++t) {
        offs[t] = total;
        total += counts[t];
    }
    offs[T] = total;
    uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(total > 0 ? total : 1));
    long* cur = (long*)calloc((size_t)T, sizeof(long));
    if (!offs || !keys || !cur) return -1;
    for (int g = 0; g < G; ++g) {
        const LRec* q = &rec[g];
        const uint64_t key = ((uint64_t)float_to_bits(q->depth) << 32) | (uint32_t)g;
        nominal += (long)rect_area(q->x0, q->y0, q->x1, q->y1);
        for (int yy = q->oy0; yy < q->oy1; ++yy)
            for (int xx = q->ox0; xx < q->ox1; ++xx) {
                const int t = yy * tiles_x + xx;
                keys[offs[t] + cur[t]++] = key;
            }
    }
#pragma omp parallel for schedule(dynamic)
    for (int t = 0; t < T; ++t) qsort(keys + offs[t], (size_t)(offs[t + 1] - offs[t]), 8, cmp_u64);

    const size_t hwn = (size_t)H * W;
    const float a_min = 1.0f / 255.0f;
    /* diagnostics: TSPLAT_REF_DEBUG_PIXEL=x,y prints that pixel's flagged-mode blend, entry by entry */
    int dbx = -1, dby = -1;
    {
        const char* e = getenv("TSPLAT_REF_DEBUG_PIXEL");
        if (e && sscanf(e, "%d,%d", &dbx, &dby) != 2) dbx = dby = -1;
    }
#pragma omp parallel for schedule(dynamic)
    for (int t = 0; t < T; ++t) {
        const int tx = t % tiles_x, ty = t / tiles_x;
        for (int ly = 0; ly < TILE; ++ly)
            for (int lx = 0; lx < TILE; ++lx) {
                const int pxi = tx * TILE + lx, pyi = ty * TILE + ly;
                if (pxi >= W || pyi >= H) continue;
                const float pfx = (float)pxi, pfy = (float)pyi;
                float Tr = 1.0f, C0 = 0.f, C1 = 0.f, C2 = 0.f;
                double Td = 1.0;
                int flag = 0, n_acc = 0;
                for (long k = offs[t]; k < offs[t + 1]; ++k) {
                    const LRec* q = &rec[(uint32_t)(keys[k] & 0xffffffffu)];
                    const int in_nom = tx >= q->x0 && tx < q->x1 && ty >= q->y0 && ty < q->y1;
                    const float dx = q->px - pfx, dy = q->py - pfy;
                    const float power = -0.5f * (q->A * dx * dx + q->C * dy * dy) - q->B * dx * dy;
                    if (!flags) {
                        if (power > 0.0f) continue;
                        const float alpha = fminf(0.99f, q->op * expf(power));
                        if (alpha < a_min) continue;
                        const float test_T = Tr * (1 - alpha);
                        if (test_T < 0.0001f) break;
                        C0 += q->r * alpha * Tr;
                        C1 += q->g * alpha * Tr;
                        C2 += q->b * alpha * Tr;
                        Tr = test_T;
                        continue;
                    }
                    const int certain = tx >= q->ix0 && tx < q->ix1 && ty >= q->iy0 && ty < q->iy1;
                    const double dxd = q->pxd - pfx, dyd = q->pyd - pfy;
                    const double pd = -0.5 * (q->Ad * dxd * dxd + q->Cd * dyd * dyd) - q->Bd * dxd * dyd;
                    const double S = 0.5 * (fabs(q->A * dx * dx) + fabs(q->C * dy * dy)) + fabs(q->B * dx * dy);
                    const double mp = 4.0 * fabs((double)power - pd) + 8.0 * kEps * S;
                    /* could this entry contribute here in a slightly different rounding? */
                    const double a_hi = fmin(0.99, q->op * exp(fmin(0.0, (double)power + mp)));
                    const int may_contrib = a_hi >= (double)a_min * (1.0 - 1e-6);
                    if (!in_nom) { /* only an ambiguous rect / radius / cull walks this tile */
                        if (may_contrib) flag |= kFlagRect;
                        continue;
                    }
                    if (!certain && may_contrib) flag |= kFlagRect;
                    if (power > 0.0f) {
                        if (may_contrib) flag |= kFlagPower; /* skipped here, maybe not elsewhere */
                        continue;
                    }
                    if (mp > 0.0 && (double)power + mp > 0.0 && may_contrib) flag |= kFlagPower;
                    const float alpha = fminf(0.99f, q->op * expf(power));
                    const double ad = fmin(0.99, q->op * exp(pd));
                    const double ma = 4.0 * fabs((double)alpha - ad) + (double)alpha * (mp + 8.0 * kEps);
                    if (fabs((double)alpha - (double)a_min) <= ma) flag |= kFlagAlpha;
                    if (pxi == dbx && pyi == dby)
                        fprintf(stderr, "dbg k=%ld g=%u power=%.9g pd=%.9g mp=%.3g S=%.3g alpha=%.9g ad=%.9g ma=%.3g "
                                "T=%.9g flag=%d\n", k - offs[t], (unsigned)(keys[k] & 0xffffffffu), power, pd, mp, S,
                                alpha, ad, ma, Tr, flag);
                    if (alpha < a_min) continue;
                    const float test_T = Tr * (1 - alpha);
                    const double tTd = Td * (1.0 - ad);
                    ++n_acc;
                    const double mT = 4.0 * fabs((double)test_T - tTd) + 8.0 * kEps * n_acc * (double)test_T;
                    if (fabs((double)test_T - 0.0001) <= mT) flag |= kFlagT;
                    if (test_T < 0.0001f) break;
                    C0 += q->r * alpha * Tr;
                    C1 += q->g * alpha * Tr;
                    C2 += q->b * alpha * Tr;
                    Tr = test_T;
                    Td = tTd;
                }
                const size_t pix = (size_t)pyi * W + pxi;
                out_color[pix] = C0 + Tr * bg[0];
                out_color[hwn + pix] = C1 + Tr * bg[1];
                out_color[2 * hwn + pix] = C2 + Tr * bg[2];
                if (flags) out_flag[pix] = (uint8_t)flag;
            }
    }
    free(rec);
    free(counts);
    free(offs);
    free(keys);
    free(cur);
    return nominal;
}
