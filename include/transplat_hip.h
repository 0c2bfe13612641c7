/*
 * transplat_hip.h — C-ABI of the MI355X (gfx950) TranSplat inference hot path.
 *
 * Every entry point is `extern "C"`, takes plain device pointers + sizes and an explicit
 * hipStream_t (passed as void*), allocates nothing, and returns an int status:
 *   0 = OK, TSPLAT_EINVAL = bad argument, TSPLAT_EHIP = HIP launch error.
 * All pointers are device-resident and owned by the caller (the PyTorch caching allocator on
 * the Python side). Calls are thread-compatible (one stream per thread), never thread-safe
 * on a shared workspace. No entry point synchronises the stream.
 *
 * Reference interfaces replaced (paths relative to the reference repo):
 *   - rasterizer: `GaussianRasterizer(GaussianRasterizationSettings(...))(means3D, means2D,
 *     shs, colors_precomp, opacities, cov3D_precomp)` called once per view inside the Python
 *     loop of `render_cuda` (src/model/decoder/cuda_splatting.py:100-135), i.e. the
 *     third-party `diff_gaussian_rasterization._C.rasterize_gaussians` forward.
 *   - depth-candidate correlation: `UVCoarseAttention.forward` / `UVCrossAttention.forward`
 *     (src/model/utils/attention.py:468-551 / :329-416) together with `calculate_grid`
 *     (src/model/encoder/matching/depth_predictor_trans.py:11-57) and mmcv's
 *     `ext_module.ms_deform_attn_forward`
 *     (src/model/utils/multi_scale_deformable_attn_function.py:111-117).
 *   - window attention: `single_head_split_window_attention`
 *     (src/model/encoder/backbone/multiview_transformer.py:57-206) with the shifted-window
 *     mask of `generate_shift_window_attn_mask` (:17-54).
 */
#ifndef TRANSPLAT_HIP_H
#define TRANSPLAT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSPLAT_OK 0
#define TSPLAT_EINVAL (-1)
#define TSPLAT_EHIP (-2)

/* Library version / build identification (for the smoke check and the loader). */
int tsplat_version(void);

/* Debug mode (the upstream rasterizer's `debug` setting, GaussianRasterizationSettings.debug as
 * passed by src/model/decoder/cuda_splatting.py:120, whose CHECK_CUDA synchronises and checks
 * after every kernel): with on != 0 every launch of every entry point is followed by a device
 * synchronisation and an error check, and a failure prints the failing source line to stderr and
 * returns TSPLAT_EHIP from the entry point that launched it. Not usable inside hipGraph capture
 * (the Python side refuses). Returns the previous setting. */
int tsplat_set_debug(int32_t on);

/* Per-kernel timing with HIP events recorded on the launch stream around every launch of ONE
 * kernel (ids: 1 raster preprocess, 2 raster scan, 3 raster scatter, 4 raster render,
 * 5 uv coarse correlation, 6 uv cross correlation, 7 msda, 8 window attention, 9 the whole
 * rasterizer launch sequence, 10 group norm (both launches), 11 uv cross through the
 * correlation table; 0 = off).
 * tsplat_prof_read waits for the recorded events, returns the summed duration and the number of
 * launches timed since the last enable/read, and resets the record. Used by bench.py only. */
int tsplat_prof_enable(int32_t kernel_id);
int tsplat_prof_read(double* total_ms, int32_t* launches);

/* ------------------------------------------------------------------------------------------
 * Gaussian-splat forward rasterizer (graphdeco forward algorithm: preprocess, per-tile binning,
 * depth sort, front-to-back alpha blending), all views of all scenes in ONE set of launches.
 *
 * View v renders the Gaussians of scene (v / views_per_scene); Gaussian arrays are
 * [num_scenes, G, ...] with num_scenes = num_views / views_per_scene.
 * Layouts (fp32, contiguous):
 *   means      [S, G, 3]
 *   cov        [S, G, 3, 3]     full symmetric 3x3 (upper triangle read, as the reference's
 *                               cov3D_precomp = cov[:, row, col] with triu_indices(3,3))
 *   shs        [S, G, 3, M]     colour-major SH (the Gaussians.harmonics layout; the reference
 *                               transposes it to [G, M, 3] before the call)
 *   opacity    [S, G]
 *   viewmat    [V, 16]          view matrix, column-major (= inverse(c2w)^T row-major)
 *   projmat    [V, 16]          full projection, column-major (viewmat @ P^T)
 *   campos     [V, 3]           camera centre (scaled c2w[:3, 3])
 *   tanfov     [V, 2]           tan(fov_x/2), tan(fov_y/2)
 *   bg         [V, 3]           background colour
 *   scene_scale[V, 2]           (s, s*s) scale-invariance factors applied to means / cov
 * Outputs:
 *   out_color  [V, 3, H, W]
 *   out_radii  [V, G] int32     (0 = culled), the rasterizer's `radii`
 * Workspace: tsplat_raster_workspace_bytes(G, V, H, W, capacity) bytes, 256-byte aligned.
 * `capacity` bounds the number of (Gaussian, tile) instances; if a call needs more, the sticky
 * int at `status` gets bit 0 set and the image is incomplete (the Python side checks it).
 * ---------------------------------------------------------------------------------------- */
typedef struct tsplat_raster_desc {
    int32_t num_gaussians;    /* G per scene */
    int32_t num_views;        /* V total views = num_scenes * views_per_scene */
    int32_t views_per_scene;
    int32_t height;
    int32_t width;
    int32_t sh_coeffs;        /* M = coefficients stored per colour channel ((deg+1)^2) */
    int32_t sh_degree;        /* degree evaluated; 3 = upstream graphdeco, 4 = full degree-4 */
    int32_t capacity;         /* instance capacity of the workspace */
} tsplat_raster_desc;

size_t tsplat_raster_workspace_bytes(int32_t num_gaussians, int32_t num_views, int32_t height,
                                     int32_t width, int32_t capacity);

/* Byte offset inside the workspace of the uint32 total of (Gaussian, tile) instances the last
 * tsplat_raster_fwd on that workspace generated: the reference forward's `num_rendered`
 * (rasterize_points.cu RasterizeGaussiansCUDA return value). Valid after the call's stream
 * completes; it may exceed `capacity` (then the status bit is set). */
size_t tsplat_raster_num_rendered_offset(int32_t num_gaussians, int32_t num_views, int32_t height,
                                         int32_t width);

int tsplat_raster_fwd(const tsplat_raster_desc* desc,
                      const float* means, const float* cov, const float* shs,
                      const float* opacity, const float* viewmat, const float* projmat,
                      const float* campos, const float* tanfov, const float* bg,
                      const float* scene_scale,
                      float* out_color, int32_t* out_radii,
                      void* workspace, int32_t* status, void* stream);


/* Depth-candidate softmax head (reference depth_predictor_trans.py:170-180): logits [n, depths, hw]
 * (NCHW), disp [n, depths] -> coarse [n, hw] = sum_d disp softmax_d, pdf_max [n, hw] = max_d softmax_d;
 * depths <= 256. */
int tsplat_depth_softmax_fwd(const float* logits, const float* disp, float* coarse, float* pdf_max, int32_t n,
                             int32_t depths, int32_t hw, void* stream);

/* Depth head tail (reference src/model/encoder/matching/depth_predictor_trans.py:480-491): fullres
 * [v b][h w] refined disparity, head [v b][2][h w] (the to_disparity output: delta, raw density), near
 * / far [b][v] -> depth [b][v][h w] = 1 / clamp(fullres + delta, 1 / far, 1 / near), density
 * [b][v][h w] = sigmoid(raw). */
int tsplat_depth_tail_fwd(const float* fullres, const float* head, const float* near, const float* far, float* depth,
                          float* density, int32_t batch, int32_t views, int32_t hw, void* stream);

/* Per-view camera constants of render_cuda (reference cuda_splatting.py:56-96 with get_fov and
 * get_projection_matrix) from extrinsics [V, 4, 4] (c2w), normalised intrinsics [V, 3, 3], near
 * and far [V], bg [V, 3] (bg_per_view) or [3]: writes the viewmat / projmat / campos / tanfov / bg
 * / scale arrays tsplat_raster_fwd takes (one thread per view; scale_invariant as render_cuda). */
int tsplat_raster_cameras(const float* extrinsics, const float* intrinsics, const float* near, const float* far,
                          const float* bg, int32_t bg_per_view, int32_t scale_invariant, int32_t num_views,
                          float* viewmat, float* projmat, float* campos, float* tanfov, float* bg_out, float* scale,
                          void* stream);

/* ------------------------------------------------------------------------------------------
 * Depth-candidate correlation (cost volume), all fp32, channel-last features.
 * Queries are (b v)-ordered: n = 2*b + v (the UVTransformerEncoder layout, utils/encoder.py:44);
 * cameras and disparities are (v b)-ordered: index v*batch + b (prepare_feat_proj_data_lists).
 *   cams [2*batch, 30] = K^-1 (9, row-major), K (9), R (9) = pose[:3,:3], t (3) = pose[:3,3] of
 *                        the relative pose own -> other camera, pixel-unit intrinsics
 *   disp [2*batch, depths] inverse-depth candidates
 * Only two views are supported (the reference's match_two pairs views for V > 2).
 * ---------------------------------------------------------------------------------------- */

/* UVCoarseAttention + calculate_grid: out[n, p, d] = <bilinear(feat[n^1], ref_3d(p, d)),
 * feat[n, p]> / sqrt(C). feat [2*batch, H*W, C]; out [2*batch, H*W, depths]; C must be 128. */
int tsplat_uv_coarse_fwd(const float* feat, const float* cams, const float* disp, float* out,
                         int32_t batch, int32_t height, int32_t width, int32_t channels,
                         int32_t depths, void* stream);

/* UVCrossAttention core: out[n, p, d] = mean_c key[n, p, c] * sum_pt softmax(logits[n, p, d, :])_pt
 * * bilinear(value[n^1], ref_3d(p, d) + offsets[n, p, d, pt, :] / (W, H))_c.
 * value = value_proj output per view (un-flipped), key = raw own feature, both [2*batch, H*W, C];
 * offsets [2*batch, H*W, depths*points*2]; logits [2*batch, H*W, depths*points];
 * out [2*batch, H*W, depths]; points <= 8. */
int tsplat_uv_cross_fwd(const float* value, const float* key, const float* cams,
                        const float* disp, const float* offsets, const float* logits, float* out,
                        int32_t batch, int32_t height, int32_t width, int32_t channels,
                        int32_t depths, int32_t points, void* stream);

/* Fine cross correlation, table form: identical semantics to tsplat_uv_cross_fwd with the
 * channel dot products precomputed, table[(b v)][p][q] = sum_c key[p][c] value_other[q][c]
 * ([2*batch, H*W, H*W] fp32, e.g. one batched library GEMM), so each (pixel, depth) gathers
 * 4 points x 4 bilinear corners of scalars: out = (1/channels) sum_pt softmax_pt sum_corner
 * b * table[p][corner]. Same cams / disp / offsets / logits / out layouts. */
int tsplat_uv_cross_table_fwd(const float* table, const float* cams, const float* disp, const float* offsets,
                              const float* logits, float* out, int32_t batch, int32_t height, int32_t width,
                              int32_t channels, int32_t depths, int32_t points, void* stream);

/* Single-level single-head multi-scale deformable attention (mmcv ms_deform_attn_forward with
 * num_levels = num_heads = 1): out[i, q] = sum_pt weights[i, q, pt] * bilinear(value[i],
 * loc[i, q, pt] * (W, H) - 0.5). value [n, H*W, C], loc [n, queries, points, 2] in [0, 1],
 * weights [n, queries, points] (already softmax-normalised), out [n, queries, C]. */
int tsplat_msda_fwd(const float* value, const float* loc, const float* weights, float* out,
                    int32_t n, int32_t height, int32_t width, int32_t channels, int32_t queries,
                    int32_t points, void* stream);

/* tsplat_msda_fwd from the raw projections of the UV self-attention (reference
 * src/model/utils/attention.py:232-262 UVSelfAttention.forward after its two linears): ow [n][h w]
 * rows of ow_stride floats holding the points' (dx, dy) sampling offsets then their attention
 * logits; the query grid's reference points ((x + 0.5) / w, (y + 0.5) / h), loc = ref + off / (w,
 * h) and the softmax over the points are computed in the kernel. out [n, h w, 128]. */
int tsplat_msda_raw_fwd(const float* value, const float* ow, float* out, int32_t n, int32_t height, int32_t width,
                        int32_t channels, int32_t points, int32_t ow_stride, void* stream);

/* Multi-scale deformable attention with mmcv's ms_deform_attn_forward contract (replaces
 * ext_module.ms_deform_attn_forward called from the reference's
 * MultiScaleDeformableAttnFunction_fp32.forward, src/model/utils/multi_scale_deformable_attn_function.py:111-117,
 * itself reached from src/model/utils/attention.py:265-267): value [batch, num_keys, num_heads, head_dim],
 * spatial_shapes [num_levels, 2] int64 (h, w) and level_start_index [num_levels] int64 (first key
 * of each level) in device memory, sampling_loc [batch, num_queries, num_heads, num_levels,
 * num_points, 2] (x, y in [0, 1]), attn_weight [batch, num_queries, num_heads, num_levels,
 * num_points] -> out [batch, num_queries, num_heads * head_dim], fp32. Bilinear sampling at
 * (x W - 1/2, y H - 1/2) with zero padding, as mmcv. im2col_step: as mmcv, min(batch,
 * im2col_step) must divide batch (TSPLAT_EINVAL otherwise); it does not change the result.
 * num_keys must equal sum_l h_l w_l (not checked: the shapes live on the device). */
int tsplat_ms_deform_attn_fwd(const float* value, const int64_t* spatial_shapes, const int64_t* level_start_index,
                              const float* sampling_loc, const float* attn_weight, float* out, int32_t batch,
                              int32_t num_keys, int32_t num_heads, int32_t head_dim, int32_t num_levels,
                              int32_t num_queries, int32_t num_points, int32_t im2col_step, void* stream);

/* Real-SH rotation matrices, block-diagonal over degrees 0..isqrt(d_sh)-1 (<= 4), one per
 * camera: replaces the reference's e3nn call chain in rotate_sh (src/misc/sh_rotation.py:10-30:
 * matrix_to_angles + wigner_D per degree). rotations [n, 3, 3] row-major float32 (the c2w
 * rotation); basis = the constant e3nn x-to-y basis change P^l = exp(-pi/2 X_z), degrees 0..4
 * packed row-major (1 + 9 + 25 + 49 + 81 = 165 float64, misc/sh_rotation.x_basis_packed);
 * out [n, d_sh, d_sh] float32 (zeros off the diagonal blocks). */
int tsplat_sh_rotation_fwd(const float* rotations, const double* basis, float* out, int32_t num_cameras,
                           int32_t d_sh, void* stream);

/* GroupNorm over NCHW fp32 with the producing convolution's bias, the following activation and
 * the residual add fused: y = act(group_norm(x + pre_bias[c]) * gamma + beta) [+ residual],
 * act 0 none, 1 SiLU, 2 GELU (erf), 3 ReLU, where with a residual 3 also applies ReLU after the
 * add (y = relu(residual + relu(norm)), the UniMatch ResidualBlock ending with InstanceNorm =
 * GroupNorm(groups = C), reference src/model/encoder/backbone/unimatch/backbone.py ResidualBlock);
 * pre_bias and residual may be NULL.
 * Replaces the U-Net / refine-head chains GroupNorm32 -> SiLU (-> + skip) and GroupNorm -> GELU
 * (reference src/model/encoder/matching/ldm_unet/unet.py:177-370, util.py:189-208,
 * depth_predictor_trans.py:142-206; torch.nn.functional.group_norm semantics: biased variance,
 * rsqrt(var + eps)). workspace: tsplat_group_norm_workspace_bytes(n, c, hw, groups) bytes.
 * residual may be NULL; x, residual and y are [n, c, hw] contiguous, y may not alias x. */
size_t tsplat_group_norm_workspace_bytes(int32_t n, int32_t c, int64_t hw, int32_t groups);
int tsplat_group_norm_fwd(const float* x, const float* pre_bias, const float* gamma, const float* beta,
                          const float* residual,
                          float* y, void* workspace, int32_t n, int32_t c, int64_t hw, int32_t groups,
                          float eps, int32_t act, void* stream);
/* The same with the residual given as the channel concatenation [residual | residual2] read in
 * place (the U-Net output blocks' identity skip over cat([h, skip]), reference unet.py:177-300):
 * channels [0, c1) from residual [n, c1, hw], channels [c1, c) from residual2 [n, c - c1, hw];
 * 0 < c1 < c. */
int tsplat_group_norm_cat_res_fwd(const float* x, const float* pre_bias, const float* gamma, const float* beta,
                                  const float* residual, const float* residual2, int32_t c1, float* y,
                                  void* workspace, int32_t n, int32_t c, int64_t hw, int32_t groups, float eps,
                                  int32_t act, void* stream);
/* The same with bf16 x / residual / y (fp32 statistics, gamma, beta, pre_bias): the bf16
 * dense-layer mode (config C3), where the surrounding convolutions read and write bf16 -- the
 * reference's GroupNorm32 likewise normalises x.float() and casts back to x's dtype
 * (ldm_unet/util.py GroupNorm32.forward). */
int tsplat_group_norm_bf16_fwd(const void* x, const float* pre_bias, const float* gamma, const float* beta,
                               const void* residual, void* y, void* workspace, int32_t n, int32_t c, int64_t hw,
                               int32_t groups, float eps, int32_t act, void* stream);

/* Convolution epilogue without a norm: y = act(x + bias[c]) [+ residual] over [n, c, hw] fp32
 * (act as above; 3 with a residual = relu(residual + relu(.))), hw % 4 == 0, 16-B aligned; y may
 * alias x. Replaces the bias add_ + activation (+ residual add) passes after a MIOpen convolution
 * (reference depth_predictor_trans.py:151-206 conv -> GELU heads, depth_anything_v2/util/blocks.py
 * ResidualConvUnit relu -> conv -> relu -> conv -> + x). bias may be NULL. */
int tsplat_bias_act_fwd(const float* x, const float* bias, const float* residual, float* y, int32_t n, int32_t c,
                        int64_t hw, int32_t act, void* stream);

/* Channels-last conv epilogue: y [rows, c] = act(x + bias[c]) (+ res1) (+ res2), NHWC maps with
 * c % 4 == 0, 16-byte aligned; act 0 none, 2 GELU (erf), 3 ReLU (before the residuals). The
 * Depth-Anything DPT ResidualConvUnit / FeatureFusionBlock (reference
 * src/depth_anything_v2/util/blocks.py:73-150) after bias-free MIOpen convolutions: conv1 -> bias +
 * ReLU, conv2 -> bias + unit residual (+ the fusion block's skip). x may equal y. */
int tsplat_bias_act_nhwc_fwd(const float* x, const float* bias, const float* res1, const float* res2, float* y,
                             int64_t rows, int32_t c, int32_t act, void* stream);

/* Pre-norm residual step of the DINOv2 blocks (reference dinov2_layers/block.py Block.forward:
 * x = x + ls(sublayer(norm(x)))): x_out = x + ls * y, n_out = LayerNorm(x_out; ln_w, ln_b, ln_eps)
 * with the NEXT sub-layer's norm, over rows of dim 256 / 512 / 768 / 1024 fp32. y may be NULL
 * (plain LayerNorm of x, x_out unused), ls may be NULL (no LayerScale). */
int tsplat_residual_ln_fwd(const float* x, const float* y, const float* ls, const float* ln_w, const float* ln_b,
                           float ln_eps, float* x_out, float* n_out, int32_t rows, int32_t dim, void* stream);
/* The same with a bf16 sub-layer output y and a bf16 n_out (bf16 dense mode: the linears read and
 * write bf16), the residual stream x / x_out and all statistics fp32 -- what autocast computes
 * (LayerNorm in fp32, cast to bf16 by the next linear). */
/* LayerNorm over rows of 128 with an optional post-norm residual: out = [residual +] LN(y; ln_w,
 * ln_b, ln_eps), y and out fp32 or bf16 (y_bf16 / out_bf16), residual fp32 or NULL. The multi-view
 * transformer's norm1 / norm2 with `source + message` (reference multiview_transformer.py:327-407)
 * and the UV encoder layer's norms (utils/encoder.py:131-209) in the bf16 dense mode. */
int tsplat_layer_norm128_fwd(const void* y, int32_t y_bf16, const float* residual, const float* ln_w,
                             const float* ln_b, float ln_eps, void* out, int32_t out_bf16, int32_t rows,
                             void* stream);
int tsplat_residual_ln_bf16_fwd(const float* x, const void* y, const float* ls, const float* ln_w, const float* ln_b,
                                float ln_eps, float* x_out, void* n_out, int32_t rows, int32_t dim, void* stream);

/* ------------------------------------------------------------------------------------------
 * Gaussian adapter (encoder stage 5 + GaussianAdapter.forward, reference
 * src/model/encoder/encoder_trans.py:294-353, common/gaussian_adapter.py:48-96), one pass:
 *   raw [batch, views, H*W, raw_ch] head output (2 offset + 3 scale + 4 xyzw quaternion +
 *       3*d_sh SH, raw_ch = 9 + 3*d_sh); depths, densities [batch, views, H*W];
 *   cams [batch*views, 22] = c2w R (9, row-major), c2w t (3), K^-1 of the normalised
 *       intrinsics (9), scale multiplier 0.1 * sum(K[:2,:2]^-1 (1/W, 1/H)) (1);
 *   sh_rot [batch*views, d_sh, d_sh] block-diagonal real-SH rotation of c2w R (e3nn wigner_D);
 *   outputs means [batch, views*H*W, 3], cov [.., 3, 3], harmonics [.., 3, d_sh], opacities [..];
 *   opacity = 0.5 (1 - (1 - pdf)^e + pdf^(1/e)) / gaussians_per_pixel (map_pdf_to_opacity).
 *   raw_nchw != 0: raw is the head's output map [views * batch, raw_ch, H*W] as the convolution
 *   wrote it ((v b) order, channel stride H*W), read in place instead of its [b, v, HW, c] copy.
 * ---------------------------------------------------------------------------------------- */
int tsplat_gaussian_adapter_fwd(const float* raw, const float* depths, const float* densities,
                                const float* cams, const float* sh_rot, float* means, float* cov,
                                float* harmonics, float* opacities, int32_t batch, int32_t views,
                                int32_t height, int32_t width, int32_t raw_ch, int32_t d_sh,
                                float scale_min, float scale_max, float opacity_exponent,
                                int32_t gaussians_per_pixel, int32_t raw_nchw, void* stream);

/* ------------------------------------------------------------------------------------------
 * Shifted-window attention of the multi-view transformer (exact fp32 MFMA):
 *   q [batch, H*W, C]; k, v [batch, key_views, H*W, C] (key_views = 1 for two views);
 *   out [batch, H*W, C]; C must be 128; window pixels and window pixels * key_views must be
 *   multiples of 64. with_shift rolls by half a window per axis and applies the -100 region mask.
 *   Replaces single_head_split_window_attention (reference
 *   src/model/encoder/backbone/multiview_transformer.py:57-206).
 *   workspace: tsplat_win_attn_workspace_bytes(...) bytes (split-key partials; may be 0, then
 *   workspace may be NULL).
 * ---------------------------------------------------------------------------------------- */
size_t tsplat_win_attn_workspace_bytes(int32_t batch, int32_t height, int32_t width, int32_t key_views,
                                       int32_t splits);
int tsplat_win_attn_fwd(const float* q, const float* k, const float* v, float* out, void* workspace,
                        int32_t batch, int32_t height, int32_t width, int32_t channels,
                        int32_t key_views, int32_t splits, int32_t with_shift, void* stream);

/* Split-key form of the same attention for a consumer that folds the combine into its own
 * prologue: tsplat_win_attn_split() returns the key split the 128-query kernel uses for the shape
 * (> 1: split, 1: none, 0: another kernel serves it); tsplat_win_attn_partials_fwd runs only the
 * main kernel and leaves the partials (unnormalised O, max in natural log, sum) in workspace
 * (tsplat_win_attn_workspace_bytes bytes), for tsplat_linear_f32_attn_merge_fwd. Query batch b
 * attends to the keys / values of batch (b + key_batch_shift) % batch: with the two views stacked
 * [v0; v1], shift = batch / 2 is the reference's cross-view pairing (batch_features,
 * multiview_transformer.py:495-515) without building the swapped copy. */
int32_t tsplat_win_attn_split(int32_t batch, int32_t height, int32_t width, int32_t key_views, int32_t splits);
int tsplat_win_attn_partials_fwd(const float* q, const float* k, const float* v, void* workspace, int32_t batch,
                                 int32_t height, int32_t width, int32_t channels, int32_t key_views,
                                 int32_t splits, int32_t with_shift, int32_t key_batch_shift, void* stream);

/* bf16x3 ("split-bf16") form of the same fp32 attention -- the C2 step's dense-precision mode: the
 * reference runs QK^T and PV as TF32 matmuls (multiview_transformer.py:57-206 under
 * set_float32_matmul_precision('high'), src/main.py:15). Every fp32 operand x = xh + xl (bf16
 * hi / lo), each product xh yh + xh yl + xl yh on bf16 MFMA with fp32 accumulation and an fp32
 * softmax: <= ~3 * 2^-18 relative per product (TF32: 2^-11 per operand). Window pixels must be a
 * multiple of 128. kv_x3 = [kh | kl | vh | vl] bf16, each batch * key_views * H * W * 128 elements,
 * from tsplat_split_kv_bf16x3(k, v, kv_x3, n = that count). q / out fp32 as tsplat_win_attn_fwd;
 * workspace and key split as tsplat_win_attn_fwd / _partials_fwd (same partials layout, so
 * tsplat_linear_f32_attn_merge_fwd consumes the _x3_partials_fwd output unchanged). */
int tsplat_split_kv_bf16x3(const float* k, const float* v, void* kv_x3, int64_t n, void* stream);
/* The transformer's q | k | v (or k | v) projection writing its column blocks 128-wide as
 * tsplat_linear_f32_fwd's split form does, except that blocks j >= x3_from land in kv_x3 as bf16
 * hi / lo (block x3_from + i: hi at kv_x3 + 2 i M 128, lo at kv_x3 + (2 i + 1) M 128 elements) --
 * the [kh | kl | vh | vl] operand of tsplat_win_attn_x3_* without a separate split pass. Blocks
 * j < x3_from go to out + j M 128 (fp32). x1 [M, k1], w [N, k1], k1 % 64 == 0, N % 128 == 0;
 * flags: 256 = bf16x3 products (else exact fp32). */
int tsplat_linear_f32_split_x3_fwd(const float* x1, int32_t k1, const float* w, float* out, void* kv_x3, int32_t M,
                                   int32_t N, int32_t x3_from, int32_t flags, void* stream);
int tsplat_win_attn_x3_fwd(const float* q, const void* kv_x3, float* out, void* workspace, int32_t batch,
                           int32_t height, int32_t width, int32_t channels, int32_t key_views, int32_t splits,
                           int32_t with_shift, void* stream);
int tsplat_win_attn_x3_partials_fwd(const float* q, const void* kv_x3, void* workspace, int32_t batch, int32_t height,
                                    int32_t width, int32_t channels, int32_t key_views, int32_t splits,
                                    int32_t with_shift, int32_t key_batch_shift, void* stream);

/* bf16 variant (config C3): q, k, v, out are bf16 (raw 16-bit storage), same layouts and
 * semantics; bf16 MFMA with fp32 accumulation and an fp32 softmax (P rounded to bf16 for the
 * PV product). Window pixels must be a multiple of 128. */
size_t tsplat_win_attn_bf16_workspace_bytes(int32_t batch, int32_t height, int32_t width, int32_t key_views,
                                            int32_t splits);
int tsplat_win_attn_bf16_fwd(const void* q, const void* k, const void* v, void* out, void* workspace,
                             int32_t batch, int32_t height, int32_t width, int32_t channels,
                             int32_t key_views, int32_t splits, int32_t with_shift, void* stream);
/* The same with query batch b reading the keys / values of batch (b + key_batch_shift) % batch, the
 * two-view cross pairing (reference batch_features, multiview_transformer.py:495-515) as index
 * arithmetic instead of a rolled copy; 0 <= key_batch_shift < batch. */
int tsplat_win_attn_bf16_shift_fwd(const void* q, const void* k, const void* v, void* out, void* workspace,
                                   int32_t batch, int32_t height, int32_t width, int32_t channels,
                                   int32_t key_views, int32_t splits, int32_t with_shift,
                                   int32_t key_batch_shift, void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused linear of the multi-view transformer (exact fp32 MFMA), replacing the nn.Linear +
 * torch.cat + nn.GELU + nn.LayerNorm + residual-add chains of TransformerLayer.forward
 * (reference src/model/encoder/backbone/multiview_transformer.py:327-407):
 *   out[M, N] = epilogue([x1 | x2] w^T), x1 [M, k1], x2 [M, k2] (x2 may be NULL when k2 = 0),
 *   w [N, k1 + k2] row-major (nn.Linear weight); k1, k2 multiples of 64, N a multiple of 128.
 *   flags: 16 + bias[N]; 1 exact-erf GELU; 2 LayerNorm over the row (N must be 128; biased
 *   variance, rsqrt(var + ln_eps), ln_gamma / ln_beta [128]); 4 + residual [M, N];
 *   8 split: column block j of 128 is written to out + j * split_stride as its own [M, 128]
 *   matrix (not with 4); 32 GELU of the INPUT: exact-erf GELU applied to [x1 | x2] as it is
 *   loaded (the producing layer's activation; N must be 128); 128 ReLU of the input (same rule);
 *   64 with 4: the residual is added BEFORE the LayerNorm (post-norm layers: LN(x W^T + b + r));
 *   256 bf16x3 products: x and w split as hi + lo bf16 while staged, hi*hi + hi*lo + lo*hi on
 *   v_mfma_f32_32x32x16_bf16 with fp32 accumulation (<= 3 * 2^-18 relative per product, the
 *   stand-in for the reference's TF32, src/main.py:15); default exact fp32;
 *   512 x1 is bf16 [M, k1] (pass it as x1; k2 must be 0), widened exactly while staged;
 *   1024 out is bf16 (rounded to nearest even; split_stride then counts bf16 elements; not with 4).
 *   Epilogues applied in that order.
 * ---------------------------------------------------------------------------------------- */
int tsplat_linear_f32_fwd(const float* x1, int32_t k1, const float* x2, int32_t k2, const float* w,
                          const float* bias, const float* ln_gamma, const float* ln_beta, float ln_eps,
                          const float* residual, float* out, int64_t split_stride, int32_t M, int32_t N,
                          int32_t flags, void* stream);

/* The merge projection of a transformer layer reading the attention output still split over
 * key ranges: out = epilogue(combine(partials) w^T) with combine = sum_s e^(m_s - M) O_s /
 * sum_s e^(m_s - M) l_s per query (the combine launch of tsplat_win_attn_fwd, moved into this
 * kernel's operand staging). partials as left by tsplat_win_attn_partials_fwd for the same
 * (batch, height, width, key_views, splits, with_shift); out [batch, height*width, N] in pixel
 * order; w [N, 128]; flags as tsplat_linear_f32_fwd (2 LayerNorm, 4 residual, 256 bf16x3; no 8/16/32). */
int tsplat_linear_f32_attn_merge_fwd(const float* partials, int32_t batch, int32_t height, int32_t width,
                                     int32_t key_views, int32_t splits, int32_t with_shift, const float* w,
                                     const float* ln_gamma, const float* ln_beta, float ln_eps,
                                     const float* residual, float* out, int32_t N, int32_t flags, void* stream);

/* Batched inverse of n row-major dim x dim fp32 matrices (dim 2..4): the camera algebra's
 * torch.inverse calls (reference depth_predictor_trans.py:36-49,88-98, encoder_trans.py:181-190,
 * cuda_splatting.py:93-96), Gauss-Jordan with partial pivoting, one thread per matrix. */
int tsplat_small_inverse(const float* in, float* out, int32_t n, int32_t dim, void* stream);

/* Dense multi-head self-attention of the DINOv2 ViT-B encoder (exact fp32 MFMA), replacing
 * scaled_dot_product_attention + its permute / transpose copies in Attention.forward (reference
 * src/depth_anything_v2/dinov2_layers/attention.py): qkv [batch, tokens, 3, heads, head_dim] (the
 * qkv Linear's output as it is), out [batch, tokens, heads, head_dim] = softmax(q k^T * scale) v.
 * head_dim must be 64. */
int tsplat_mha_f32_fwd(const float* qkv, float* out, int32_t batch, int32_t tokens, int32_t heads,
                       int32_t head_dim, float scale, void* stream);
/* The same with the qkv projection's bias folded in: qkv holds x W^T WITHOUT the bias and bias is
 * its [3 * heads * 64] vector (16-B aligned): q + b_q is formed on load, b_k is dropped (it adds
 * b_k . q to every score of a query, which the softmax cancels) and b_v is added to the normalised
 * output -- the reference Attention.forward on qkv = Linear(x) with bias (dinov2_layers/attention.py),
 * one elementwise pass fewer. bias = NULL is tsplat_mha_f32_fwd. */
int tsplat_mha_bias_f32_fwd(const float* qkv, const float* bias, float* out, int32_t batch, int32_t tokens,
                            int32_t heads, int32_t head_dim, float scale, void* stream);
/* The same attention in split-bf16 ("bf16x3") precision, the dense-layer mode of the C2 step (the
 * reference's SDPA matmuls run under TF32, src/main.py:15): qkv (+ bias, may be NULL) is split once
 * into hi / lo bf16 images in workspace (tsplat_mha_x3_workspace_bytes), and QK^T / PV run as
 * hi*hi + hi*lo + lo*hi on v_mfma_f32_16x16x32_bf16 / 16x16x16_bf16 with fp32 accumulation and the
 * fp32 online softmax of tsplat_mha_f32_fwd. qkv, bias and workspace 16-B aligned. */
/* tsplat_mha_x3_fwd on qkv already split into hi / lo bf16 images (bias included), lo = hi + batch
 * tokens 3 heads head_dim elements (tsplat_gemm_x3_fwd act 2 writes them so). */
int tsplat_mha_x3_presplit_fwd(const void* qkv_hi, const void* qkv_lo, float* out, int32_t batch, int32_t tokens,
                               int32_t heads, int32_t head_dim, float scale, void* stream);
size_t tsplat_mha_x3_workspace_bytes(int32_t batch, int32_t tokens, int32_t heads, int32_t head_dim);
int tsplat_mha_x3_fwd(const float* qkv, const float* bias, float* out, void* workspace, int32_t batch,
                      int32_t tokens, int32_t heads, int32_t head_dim, float scale, void* stream);

/* Legacy channels-first QKV attention of the depth predictor U-Nets (exact fp32 MFMA), replacing
 * QKVAttentionLegacy.forward (reference src/model/encoder/matching/ldm_unet/unet.py:510-552) with
 * use_cross_view_self_attn folding the views into the tokens: qkv [views * batch, 3 * heads * 32,
 * tokens_per_view] ((v b) order, per head rows q | k | v), out [views * batch, heads * 32,
 * tokens_per_view] = softmax over all views' tokens of q.k * scale, times v. views = 1 for plain
 * self-attention. head_dim must be 32; scale multiplies the dot product (the reference's
 * (q / ch^(1/4)).(k / ch^(1/4)) is scale = ch^(-1/2)). */
int tsplat_qkv_attention_cf_fwd(const float* qkv, float* out, int32_t batch, int32_t heads, int32_t views,
                                int32_t tokens_per_view, int32_t head_dim, float scale, void* stream);

/* Direct convolution of the depth predictor U-Nets' low-resolution levels (exact fp32 MFMA),
 * replacing MIOpen for nn.Conv2d in reference src/model/encoder/matching/ldm_unet/unet.py (ResBlock
 * in/out convs unet.py:212-250 and 1x1 skip unet.py:258-266, Downsample unet.py:140-170, Upsample
 * unet.py:105-137): y [batch, c_out, hout, wout] = conv(x, w, bias, stride, padding = ksize / 2)
 * with x = cat([x1 (c1 channels), x2 (c2 channels, may be 0)], dim 1) [batch, c1 + c2, height, width]
 * read in place, nearest-upsampled 2x first when upsample = 1. ksize 1 or 3, stride 1 or 2 (not
 * with upsample; the strided 1x1 is the UniMatch CNN's shortcut), c1 and c2 even. w_packed is the weight [c_out, cin, k, k] laid out as
 * [ceil(c_out / 32)][k * k][cin / 2][2][32] (zero rows past c_out); bias may be null. ksplit
 * (1..16) waves share one 32 x 32 output tile. */
int tsplat_conv2d_f32_fwd(const float* x1, int32_t c1, const float* x2, int32_t c2, const float* w_packed,
                          const float* bias, float* y, int32_t batch, int32_t height, int32_t width, int32_t c_out,
                          int32_t ksize, int32_t stride, int32_t upsample, int32_t ksplit, void* stream);

/* tsplat_conv2d_f32_fwd with the input-channel pairs of each 32 x 32 output tile also split over
 * zsplit (1..64) workgroups, for few-tile maps with long reductions (the same nn.Conv2d layers at
 * 9^2-32^2, and the Depth-Anything DPT's tiny stride-2 768-channel level, reference
 * src/depth_anything_v2/dpt.py:117-151). partials: device workspace of ceil(npx / 32) *
 * ceil(c_out / 32) * zsplit * 1024 floats; counters: that many (tiles) int32 arrival counters, zero
 * on entry and left zero on return (the last workgroup of a tile resets its counter), so one buffer
 * serves every launch on one stream. The result does not depend on which workgroup finishes last
 * (partials summed in z order). zsplit = 1 is tsplat_conv2d_f32_fwd. */
int tsplat_conv2d_f32_zsplit_fwd(const float* x1, int32_t c1, const float* x2, int32_t c2, const float* w_packed,
                                 const float* bias, float* y, int32_t batch, int32_t height, int32_t width,
                                 int32_t c_out, int32_t ksize, int32_t stride, int32_t upsample, int32_t ksplit,
                                 int32_t zsplit, float* partials, int32_t* counters, void* stream);

/* tsplat_conv2d_f32_zsplit_fwd in split-bf16 ("bf16x3", the bf16x3 dense mode's precision: each
 * product as hi*hi + hi*lo + lo*hi of x = hi + lo bf16 on bf16 MFMA, fp32 accumulation, <= ~3 * 2^-18
 * relative per product -- finer than the reference's TF32, src/main.py:15). Same layers, arguments
 * and workspaces, except: c1 and c2 any positive / non-negative counts (not only even), and
 * w_packed is the weight as bf16 hi / lo fragments [ceil(c_out / 32)][k * k][ceil(cin / 16)][2 (hi,
 * lo)][64][8] (element (l, j) of fragment (cot, tap, g): c_out 32 cot + (l & 31), cin 16 g + 8 (l >> 5)
 * + j; zero past c_out / cin). */
int tsplat_conv2d_bf16x3_fwd(const float* x1, int32_t c1, const float* x2, int32_t c2, const void* w_packed,
                             const float* bias, float* y, int32_t batch, int32_t height, int32_t width,
                             int32_t c_out, int32_t ksize, int32_t stride, int32_t upsample, int32_t ksplit,
                             int32_t zsplit, float* partials, int32_t* counters, void* stream);

/* 3x3 / stride 1 / padding 1 convolution as Winograd F(2x2, 3x3) on exact-fp32 MFMA (replaces the
 * nn.Conv2d(c_in, c_out, 3, 1, 1) calls of the depth predictor's full-resolution heads and U-Net
 * levels, reference src/model/encoder/matching/depth_predictor_trans.py:110-125 and
 * ldm_unet/unet.py ResBlock, which PyTorch hands to MIOpen). x [batch, c_in, height, width] and
 * y [batch, c_out, height, width] NCHW fp32; w_packed = tsplat_wino_weight_f32(weight) (the
 * transformed filters G g G^T, tsplat_wino_weight_floats(c_out, c_in) floats); bias may be null;
 * y = act(conv(x) + bias), act 0 none, 1 ReLU, 2 GELU (erf). */
size_t tsplat_wino_weight_floats(int32_t c_out, int32_t c_in);
int tsplat_wino_weight_f32(const float* weight, float* w_packed, int32_t c_out, int32_t c_in, void* stream);
int tsplat_conv3x3_wino_f32_fwd(const float* x, const float* w_packed, const float* bias, float* y, int32_t batch,
                                int32_t c_in, int32_t height, int32_t width, int32_t c_out, int32_t act,
                                void* stream);
/* The same on the channel concatenation of n_src (1..6) NCHW inputs, read in place (replaces the
 * torch.cat feeding the reference's to_gaussians head, depth_predictor_trans.py:486-489, and the
 * U-Net output blocks' skip concatenation, ldm_unet/unet.py:1130): srcs / chans are HOST arrays of
 * n_src device pointers [batch, chans[s], height, width] and their channel counts (sum = c_in). */
int tsplat_conv3x3_wino_cat_f32_fwd(const float* const* srcs, const int32_t* chans, int32_t n_src,
                                    const float* w_packed, const float* bias, float* y, int32_t batch,
                                    int32_t height, int32_t width, int32_t c_out, int32_t act, void* stream);

/* The same Winograd convolutions in split-bf16 ("bf16x3") precision, the C2 step's dense-layer
 * mode standing in for the reference's TF32 (src/main.py:15 + cuDNN's TF32 convolutions; gfx950
 * has no xf32 MFMA): every operand x = hi + lo (two bf16), every product hi*hi + hi*lo + lo*hi on
 * v_mfma_f32_32x32x16_bf16 with fp32 accumulation (<= 3 * 2^-18 relative per product, TF32 2^-11).
 * Same arguments and semantics as tsplat_conv3x3_wino_{,cat_}f32_fwd except w_packed =
 * tsplat_wino_weight_bf16x3(weight): G g G^T split into hi / lo bf16 and packed as
 * [16][cobs][ceil(c_in / 16)][hi, lo][64 lanes][8] (tsplat_wino_weight_bf16x3_bytes bytes). */
size_t tsplat_wino_weight_bf16x3_bytes(int32_t c_out, int32_t c_in);
int tsplat_wino_weight_bf16x3(const float* weight, void* w_packed, int32_t c_out, int32_t c_in, void* stream);
int tsplat_conv3x3_wino_bf16x3_fwd(const float* x, const void* w_packed, const float* bias, float* y, int32_t batch,
                                   int32_t c_in, int32_t height, int32_t width, int32_t c_out, int32_t act,
                                   void* stream);
int tsplat_conv3x3_wino_bf16x3_cat_fwd(const float* const* srcs, const int32_t* chans, int32_t n_src,
                                       const void* w_packed, const float* bias, float* y, int32_t batch,
                                       int32_t height, int32_t width, int32_t c_out, int32_t act, void* stream);
/* The same with the Depth-Anything DPT ResidualConvUnit's glue fused (src/depth_anything_v2/util/
 * blocks.py ResidualConvUnit.forward: conv(relu(x)) ... + x, FeatureFusionBlock's + skip):
 * relu_in != 0 applies ReLU to the input as it is loaded; y = act(conv + bias) + residual +
 * residual2 (each [batch, c_out, height, width] NCHW fp32, or null). */
int tsplat_conv3x3_wino_bf16x3_ex_fwd(const float* const* srcs, const int32_t* chans, int32_t n_src,
                                      const void* w_packed, const float* bias, const float* residual,
                                      const float* residual2, float* y, int32_t batch, int32_t height, int32_t width,
                                      int32_t c_out, int32_t act, int32_t relu_in, void* stream);

/* The same 3x3 / stride-1 / pad-1 convolution (bf16x3 precision, identical arguments except the
 * weight) as a direct implicit GEMM for FEW-channel, full-resolution maps -- the refine U-Net's
 * 32-channel 256^2 / 128^2 levels and the depth heads (depth_predictor_trans.py:138-160, ldm_unet/
 * unet.py at model_channels = 32), where the Winograd form's per-block prologue / epilogue dominate.
 * w_packed = the direct kernels' split-bf16 A operand [ceil(c_out / 32)][9][ceil(c_in / 16)][hi, lo]
 * [64 lanes][8] (as tsplat_conv2d_bf16x3_fwd). Requires width % 4 == 0, 16-B aligned sources,
 * c_out <= 64, c_in <= 128 (else TSPLAT_EINVAL); tsplat_conv3x3_few_form() returns 0 for shapes it
 * does not take and otherwise its launch form (10 * rows per block + 32-channel blocks per workgroup). */
int32_t tsplat_conv3x3_few_form(int32_t batch, int32_t c_in, int32_t height, int32_t width, int32_t c_out);
int tsplat_conv3x3_few_bf16x3_fwd(const float* const* srcs, const int32_t* chans, int32_t n_src,
                                  const void* w_packed, const float* bias, const float* residual,
                                  const float* residual2, float* y, int32_t batch, int32_t height, int32_t width,
                                  int32_t c_out, int32_t act, int32_t relu_in, void* stream);

/* Split-bf16 operands for ONE library bf16 GEMM that computes an fp32 linear layer in bf16x3
 * precision (the nn.Linear layers of the fp32 path -- DINOv2 qkv / proj / fc1 / fc2,
 * src/depth_anything_v2/dinov2_layers/{attention,mlp}.py, the transformer FFN's mlp[0],
 * multiview_transformer.py:327-407 -- in the stand-in for the reference's TF32 matmuls): x [rows, k]
 * fp32 (k % 4 == 0) -> out [rows, 3k] bf16 = [hi | hi | lo] (weight_order = 0, activations) or
 * [hi | lo | hi] (weight_order = 1, weights), hi = bf16(x), lo = bf16(x - hi); then
 * [x_hi | x_hi | x_lo] [W_hi | W_lo | W_hi]^T = x_hi W_hi^T + x_hi W_lo^T + x_lo W_hi^T. */
int tsplat_split_bf16x3(const float* x, void* out, int64_t rows, int32_t k, int32_t weight_order, void* stream);

/* bf16 3x3 / 1x1 convolution (stride 1, padding ksize / 2) for config C3 (bf16 autocast of the same
 * reference nn.Conv2d layers: ldm_unet/unet.py ResBlock in/out convolutions and 1x1 skips
 * unet.py:212-266, Upsample unet.py:105-137, the output blocks' skip concatenation unet.py:1130,
 * the depth predictor's heads depth_predictor_trans.py:110-125), as an implicit GEMM on
 * v_mfma_f32_32x32x16_bf16 with fp32 accumulation: y = act(conv(up(cat(srcs))) + bias) rounded to
 * bf16, act 0 none, 1 SiLU, 2 GELU (erf), 3 ReLU. srcs / src_channels / src_f32 are HOST arrays of
 * n_src (1..4) device pointers [batch, src_channels[s], h_in, w_in] NCHW, their channel counts and
 * dtypes: bf16 (src_f32[s] = 0) or fp32 rounded to bf16 on load (1); (h_in, w_in) = (height, width),
 * or (height / 2, width / 2) with upsample = 1 (nearest 2x, read in place). width a multiple of 8;
 * channel counts free (counts that are not multiples of 8, or mixed dtypes, take a per-channel
 * loader).
 * w_packed = the bf16 weights packed as [ceil(c_out / 32)][ceil(c_in / 16)][ksize^2 taps][64
 * lanes][8] (lane l = c + 32 h holds w[32 b + c][16 k + 8 h + 0..7][tap], zero padded;
 * tsplat_conv2d_bf16_weight_bytes bytes); bias fp32 [c_out] or null; y [batch, c_out, height, width]
 * bf16. */
size_t tsplat_conv2d_bf16_weight_bytes(int32_t c_out, int32_t c_in, int32_t ksize);
int tsplat_conv2d_bf16_fwd(const void* const* srcs, const int32_t* src_channels, int32_t n_src, const int32_t* src_f32,
                           const void* w_packed, const float* bias, void* y, int32_t batch, int32_t height,
                           int32_t width, int32_t c_out, int32_t ksize, int32_t upsample, int32_t act,
                           void* stream);

/* Channels-last form of tsplat_conv2d_f32_fwd for the Depth-Anything DPT head (reference
 * src/depth_anything_v2/util/blocks.py ResidualConvUnit / FeatureFusionBlock.out_conv), whose conv
 * chain runs on channels-last maps: x [batch, height, width, c_in], y and residual
 * [batch, height, width, c_out]; stride 1, padding ksize / 2; y = conv(relu_in ? relu(x) : x) (+ bias)
 * (+ residual). Same packed weights and ksplit as tsplat_conv2d_f32_fwd. */
int tsplat_conv2d_f32_nhwc_fwd(const float* x, int32_t c_in, const float* w_packed, const float* bias,
                               const float* residual, float* y, int32_t batch, int32_t height, int32_t width,
                               int32_t c_out, int32_t ksize, int32_t relu_in, int32_t ksplit, void* stream);

/* y [n, c, height * scale, width * scale] = act(bilinear_upsample(x) + bias[c]) with
 * align_corners = True (reference depth_predictor_trans.py upsampler: Conv2d -> Upsample(bilinear,
 * align_corners=True) -> GELU, with the conv's bias moved past the interpolation); x [n, c, height,
 * width] NCHW fp32, bias may be null; act 0 none, 2 GELU (erf), 3 ReLU; width * scale % 4 == 0. */
int tsplat_upsample_bilinear_act_fwd(const float* x, const float* bias, float* y, int32_t n, int32_t c,
                                     int32_t height, int32_t width, int32_t scale, int32_t act, void* stream);

/* Channels-last bilinear resize with align_corners = True to any output size (the DPT head's
 * F.interpolate calls, reference src/depth_anything_v2/util/blocks.py FeatureFusionBlock.forward and
 * dpt.py DPTHead.forward): x [n, height, width, c], y [n, out_height, out_width, c], c % 4 == 0. */
int tsplat_resize_bilinear_nhwc_fwd(const float* x, float* y, int32_t n, int32_t height, int32_t width, int32_t c,
                                    int32_t out_height, int32_t out_width, void* stream);

/* F.interpolate(x, (out_height, out_width), mode="bilinear", align_corners=True) on an NCHW fp32
 * tensor of `planes` = N * C maps (replaces the PyTorch resizes at the reference's
 * encoder_trans.py DA-V2 input / depth resize and depth_predictor_trans.py DINO-feature resize);
 * torch's arithmetic (source = dst * (in - 1) / (out - 1) in float). */
int tsplat_resize_bilinear_nchw_fwd(const float* x, float* y, int32_t planes, int32_t height, int32_t width,
                                    int32_t out_height, int32_t out_width, void* stream);

/* Split-bf16 ("bf16x3") GEMM for the bf16x3 dense mode's fp32 linears (DINOv2-B/14 qkv / proj /
 * fc1 + GELU / fc2 at M = 650: src/depth_anything_v2/dinov2_layers/attention.py:70-75, mlp.py:33-40;
 * the reference's nn.Linear in TF32, src/main.py:15), replacing the hipBLASLt calls of F.linear.
 * tsplat_gemm_x3_pack splits W [n, k] fp32 (nn.Linear weight) once into its hi / lo bf16 MFMA
 * fragments (tsplat_gemm_x3_pack_bytes(n, k) bytes, 16-B aligned). tsplat_gemm_x3_fwd:
 * out[s, m, n] = sum over split s's share of k of x[m, k] W[n, k] (+ bias[n] in slab 0; act 1 =
 * exact-erf GELU, only with ksplit 1; act 2 = no activation, the output written as hi / lo bf16
 * images [m, n] at out and out + m n bf16 elements, x = hi + lo, only with ksplit 1), x [m, k] fp32 rows
 * contiguous, k % 4 == 0, n % 4 == 0, x /
 * bias / out 16-B aligned, 1 <= ksplit <= ceil(k / 64) with every split non-empty; out holds ksplit
 * slabs [m, n] whose sum is the product (tsplat_residual_ln_slabs_fwd adds them in order). */
size_t tsplat_gemm_x3_pack_bytes(int32_t n, int32_t k);
int tsplat_gemm_x3_pack(const float* w, void* wp, int32_t n, int32_t k, void* stream);
int tsplat_gemm_x3_fwd(const float* x, const void* wp, const float* bias, float* out, int32_t m, int32_t n, int32_t k,
                       int32_t ksplit, int32_t act, void* stream);

/* tsplat_residual_ln_fwd with the sub-layer output y given as nslab partial slabs [nslab, rows, dim]
 * (split-K GEMM output, tsplat_gemm_x3_fwd) summed in slab order before the LayerScale multiply. */
int tsplat_residual_ln_slabs_fwd(const float* x, const float* y, int32_t nslab, const float* ls, const float* ln_w,
                                 const float* ln_b, float ln_eps, float* x_out, float* n_out, int32_t rows,
                                 int32_t dim, void* stream);

/* Diagnostics: write the 100-MHz device wall clock into ((uint64_t*)buf)[slot] when this launch
 * runs on `stream` (stage marks of a captured / replayed step, tools/graph_stages.py). */
int tsplat_timestamp(void* buf, int32_t slot, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* TRANSPLAT_HIP_H */
