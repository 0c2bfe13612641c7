"""usage: op_stacks.py [batch] [fp32|bf16|bf16x3] [attn dtype: auto|bf16|...]
Which Python call sites launch the small PyTorch kernels (copies, elementwise, cat, GELU, clamp ...)
of one e2e step: a TorchDispatchMode records every launching aten op with the innermost repo frame
that called it (torch.profiler's with_stack comes back empty on this build)."""
import collections
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model

# ops that only reshape metadata (no kernel)
VIEWS = {"view", "_unsafe_view", "reshape", "permute", "transpose", "t", "expand", "unsqueeze", "squeeze", "slice",
         "select", "as_strided", "alias", "detach", "split", "split_with_sizes", "chunk", "unbind", "narrow",
         "unflatten", "flatten", "contiguous", "empty", "empty_like", "empty_strided", "new_empty", "lift_fresh",
         "is_same_size", "size", "stride", "movedim", "unfold", "view_as", "diagonal", "_reshape_alias",
         "set_", "resize_", "_local_scalar_dense", "item"}


class Sites(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.agg = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__.split(".")[0]
        if name not in VIEWS:
            frames = [f for f in traceback.extract_stack() if "transplat_amd/" in f.filename]
            where = f"{frames[-1].filename.split('transplat_amd/')[-1]}:{frames[-1].lineno}" if frames else "?"
            if name == "convolution":  # which convolutions stay on MIOpen
                x, w = args[0], args[1]
                where += (f" x{tuple(x.shape)} w{tuple(w.shape)} s{args[3]} bias={args[2] is not None}"
                          f" cl={x.is_contiguous(memory_format=torch.channels_last)}")
            self.agg[(name, where)] += 1
        return func(*args, **(kwargs or {}))


import sys

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 1
dense = sys.argv[2] if len(sys.argv) > 2 else "fp32"
attn = sys.argv[3] if len(sys.argv) > 3 else "auto"
dev = torch.device("cuda:0")
model = build_model(dev, dense, attn_dtype=attn)
data = S.make_batch(batch, image_shape=(256, 256), device=dev)
for _ in range(2):
    model.test_step(data)
torch.cuda.synchronize()
mode = Sites()
with mode:
    model.test_step(data)
torch.cuda.synchronize()
for (name, where), n in mode.agg.most_common(150):
    print(f"{n:4d} {name:24s} {where}")
