"""The bench line's precision statement is derived from what a step launched (transplat_amd/routes.py),
not hand-written: the C-ABI hook, the library-op census and the label (CPU), and on the GPU the
routes of the benched C2 step and of C3 as stated -- no library convolution left in either."""
import pytest
import torch

from transplat_amd import _lib, routes
from transplat_amd import synthetic as S


def test_route_hook_and_label():
    r = routes.Routes()
    prev = _lib.ROUTE_HOOK
    _lib.ROUTE_HOOK = r.note
    try:
        _lib.check(0, "tsplat_win_attn_x3_partials_fwd")
        _lib.check(0, "tsplat_linear_f32_fwd", "bf16x3")
        _lib.check(0, "tsplat_linear_f32_fwd", "exact fp32")
        _lib.check(0, "tsplat_conv3x3_wino_bf16x3_fwd")
        _lib.check(0, "tsplat_version")  # not a compute route: ignored
        with pytest.raises(RuntimeError):
            _lib.check(-1, "tsplat_raster_fwd")  # a failed call is not a route
    finally:
        _lib.ROUTE_HOOK = prev
    r.lib("mm", "xf32 (emulated, bf16 MFMA)", [(650, 768), (768, 3072)])
    lab = r.label()
    assert "window attention: bf16x3 (split-bf16 products, fp32 softmax) x1" in lab
    assert "transformer linears (HIP): " in lab and "bf16x3 x1" in lab and "exact fp32 x1" in lab
    assert "library GEMMs (hipBLASLt): xf32 (emulated, bf16 MFMA) x1" in lab
    assert "library convs (MIOpen): none" in lab
    assert "rasterizer" not in lab
    r.lib("convolution", "fp32", [(16, 768, 18, 18), (768, 768, 3, 3)])
    assert "library convs (MIOpen): fp32 x1" in r.label()


def _step_routes(device, dense, batch, attn="auto"):
    from transplat_amd.e2e import build_model

    model = build_model(device, dense, attn_dtype=attn)
    data = S.make_batch(batch, image_shape=(256, 256), device=device)
    with torch.no_grad():
        model.test_step(data)  # warm (weight packing, MIOpen / hipBLASLt choices)
        with routes.record() as r:
            model.test_step(data)
    torch.cuda.synchronize()
    print(r.label())
    return r


@pytest.mark.gpu
def test_c2_step_routes(device):
    """The benched C2 step (b = 1, bf16x3 dense, auto attention): the window attention runs the
    bf16x3 kernel, the 3x3s the bf16x3 Winograd, and no convolution reaches MIOpen."""
    r = _step_routes(device, "bf16x3", 1)
    cats = r.by_category()
    assert set(cats["window attention"]) == {"bf16x3 (split-bf16 products, fp32 softmax)"}
    assert "bf16x3" in cats["3x3 convs (HIP Winograd)"]
    assert "library convs (MIOpen)" not in cats, r.library
    assert cats["rasterizer (HIP)"]["fp32"] == 1


@pytest.mark.gpu
def test_c3_step_routes_library_conv_free(device):
    """C3 as stated (b = 8, bf16x3 dense + bf16 window attention): no MIOpen convolution (round 5
    still ran the DPT's 768 -> 768 stride-2 3x3 and two other 3x3s there)."""
    r = _step_routes(device, "bf16x3", 8, attn="bf16")
    cats = r.by_category()
    assert set(cats["window attention"]) == {"bf16 MFMA, fp32 softmax"}
    convs = [x for x in r.library if x[0] not in routes._GEMMS]
    assert not convs, convs


def test_every_matmul_entry_point_is_censused():
    """Every C-ABI convolution / attention / linear entry point the host code calls has a route
    category, so a new kernel cannot silently drop out of the bench line's precision statement."""
    import re
    from pathlib import Path

    pkg = Path(routes.__file__).parent
    names = set()
    for f in [pkg / "kernels.py", *pkg.glob("model/**/*.py")]:
        names |= set(re.findall(r'check\(\s*\w+,\s*"(tsplat_\w+_fwd)"', f.read_text()))
    hot = {n for n in names if re.search(r"conv|attn|attention|_linear_|mha|raster", n)}
    assert hot, "no entry points found"
    missing = sorted(n for n in hot if n not in routes._HIP)
    assert not missing, missing
