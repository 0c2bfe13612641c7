"""Does tsplat_uv_coarse_fwd read outside its inputs? Each input is placed inside a larger buffer whose
margins hold garbage (NaN, then large values); the output must not change. usage: coarse_oob.py [bitmap]"""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests" / "golden"))
if len(sys.argv) > 1 and sys.argv[1] == "bitmap":
    os.environ["TSPLAT_UV_COARSE_BITMAP"] = "1"
from canonical import seeded  # noqa: E402
from test_encoder_ops import _cams, _rotated_cams  # noqa: E402

from transplat_amd import _lib  # noqa: E402
from transplat_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
hw = 64
lib = _lib.load()


def run(feat, cams, disp, out):
    rc = lib.tsplat_uv_coarse_fwd(_lib.ptr(feat), _lib.ptr(cams), _lib.ptr(disp), _lib.ptr(out), 1, hw, hw, 128,
                                  disp.shape[1], _lib.stream_ptr(dev))
    assert rc == 0
    torch.cuda.synchronize()
    return out.clone()


def embed(t, fill, pad=1 << 20):
    buf = torch.full((t.numel() + 2 * pad,), fill, dtype=t.dtype, device=dev)
    buf[pad:pad + t.numel()] = t.reshape(-1)
    return buf[pad:pad + t.numel()].view_as(t)


for name, (intr, pose, disp) in {"synthetic": _cams(1, hw), "rotated": _rotated_cams(1, hw, 3, lambda d: d)}.items():
    feat = seeded((1, 2, hw * hw, 128), 31).to(dev)
    cams = K.pack_cameras(intr.to(dev), pose.to(dev))
    disp = disp.to(dev).contiguous()
    out = torch.zeros((2, hw * hw, disp.shape[1]), device=dev)
    ref = run(feat, cams, disp, out)
    for fill in (float("nan"), 1e30, -7.0):
        res = []
        for which in ("feat", "cams", "disp", "out"):
            f2, c2, d2, o2 = feat, cams, disp, out
            if which == "feat":
                f2 = embed(feat, fill)
            elif which == "cams":
                c2 = embed(cams, fill)
            elif which == "disp":
                d2 = embed(disp, fill)
            else:
                o2 = embed(out, fill)
            r = run(f2, c2, d2, o2)
            res.append(f"{which} {'same' if torch.equal(r, ref) else 'DIFFERS (%d)' % (r != ref).sum().item()}")
        print(f"{name} fill {fill}: " + ", ".join(res), flush=True)
