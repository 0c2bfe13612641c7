"""Drop-in for the reference's src/model/utils/multi_scale_deformable_attn_function.py: the two
autograd Functions whose forward calls mmcv's `ext_module.ms_deform_attn_forward`, here the gfx950
kernel behind `tsplat_ms_deform_attn_fwd` (kernels.ms_deform_attn). Same call signature
(`Function.apply(value, value_spatial_shapes, value_level_start_index, sampling_locations,
attention_weights, im2col_step)`), same shapes and the same im2col_step divisibility error.

This build covers the inference path (the reference's test_step); the backward
(mmcv ms_deform_attn_backward) is out of scope and raises. TranSplat's own UV layers use one head
and one level and call the tuned single-level kernel (kernels.msda) directly.
"""
import torch
from torch.autograd.function import Function, once_differentiable

from transplat_amd import kernels


class MultiScaleDeformableAttnFunction_fp32(Function):
    """Reference multi_scale_deformable_attn_function.py:83-121 (forward)."""

    @staticmethod
    def forward(ctx, value, value_spatial_shapes, value_level_start_index, sampling_locations, attention_weights,
                im2col_step):
        """value (bs, num_keys, num_heads, embed_dims // num_heads), value_spatial_shapes (num_levels, 2)
        as (h, w), value_level_start_index (num_levels,), sampling_locations (bs, num_queries,
        num_heads, num_levels, num_points, 2) as (x, y), attention_weights (bs, num_queries,
        num_heads, num_levels, num_points) -> (bs, num_queries, embed_dims), fp32."""
        ctx.im2col_step = im2col_step
        return kernels.ms_deform_attn(value.float(), value_spatial_shapes, value_level_start_index,
                                      sampling_locations.float(), attention_weights.float(), im2col_step)

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_output):
        raise NotImplementedError("ms_deform_attn backward (training) is outside this inference build")


class MultiScaleDeformableAttnFunction_fp16(Function):
    """Reference multi_scale_deformable_attn_function.py:8-45 (forward): the inputs are rounded to
    fp16 as the reference's custom_fwd(cast_inputs=torch.float16) does; the sampling and the sum run
    in fp32 and the output is returned as fp16."""

    @staticmethod
    def forward(ctx, value, value_spatial_shapes, value_level_start_index, sampling_locations, attention_weights,
                im2col_step):
        ctx.im2col_step = im2col_step
        h = lambda t: t.half().float()
        return kernels.ms_deform_attn(h(value), value_spatial_shapes, value_level_start_index, h(sampling_locations),
                                      h(attention_weights), im2col_step).half()

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_output):
        raise NotImplementedError("ms_deform_attn backward (training) is outside this inference build")
