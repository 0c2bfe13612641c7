"""End-to-end TranSplat test_step (encoder -> decoder) on synthetic scenes.

CPU: the full encoder with the oracle ops in place of the HIP kernels (test-only monkeypatch)
produces finite Gaussians. GPU: the real path at 256x256; eager and hipGraph-replayed steps agree
and the output is finite and image-shaped.
"""
import pytest
import torch

from oracle import encoder_ops as E
from transplat_amd import synthetic as S


def test_encoder_cpu_with_oracle_ops(monkeypatch):
    from transplat_amd import kernels
    from transplat_amd.model.encoder import EncoderTrans, EncoderTransCfg

    for n in E.KERNEL_RESTATEMENTS:
        monkeypatch.setattr(kernels, n, getattr(E, n))
    enc = S.init_synthetic_weights(EncoderTrans(EncoderTransCfg()).eval())
    batch = S.make_batch(1, image_shape=(128, 128))
    with torch.no_grad():
        g = enc(batch["context"], 0, deterministic=True)
    assert g.means.shape == (1, 2 * 128 * 128, 3) and g.harmonics.shape == (1, 2 * 128 * 128, 3, 25)
    for t in (g.means, g.covariances, g.harmonics, g.opacities):
        assert torch.isfinite(t).all()


@pytest.mark.gpu
def test_e2e_graph_matches_eager(device):
    """hipBLASLt / MIOpen pick reduction orders per call, so two EAGER steps already differ
    (measured on MI355X: depths ~1e-4 relative, pixels up to ~2.5e-3). The graph must stay within
    that envelope and must actually consume new inputs copied into its static buffers."""
    from transplat_amd.e2e import GraphedStep, build_model

    model = build_model(device)
    data = S.make_batch(1, image_shape=(256, 256), device=device)
    eager = model.test_step(data).color.clone()
    graphed = GraphedStep(model, data)
    out = graphed.run().color.clone()
    torch.cuda.synchronize()
    assert eager.shape == (1, 3, 3, 256, 256)
    assert torch.isfinite(eager).all()
    assert (out - eager).abs().max().item() < 2e-2
    assert (out - eager).abs().mean().item() < 1e-4
    data2 = S.make_batch(1, image_shape=(256, 256), scene_offset=7, device=device)
    eager2 = model.test_step(data2).color.clone()
    out2 = graphed.run(data2).color.clone()
    torch.cuda.synchronize()
    assert (out2 - eager2).abs().mean().item() < 1e-4
    assert (out2 - out).abs().mean().item() > 1e-3  # a different scene really went through the graph


@pytest.mark.gpu
def test_e2e_three_context_views(device):
    """nctx = 3 (the DTU setting at the reference's 256x256): V = 3 window attention (two key
    views), pairwise cost-volume averaging, U-Nets with three frames, 3 x 65,536 Gaussians."""
    from transplat_amd.e2e import build_model

    model = build_model(device, num_context_views=3)
    data = S.make_batch(1, num_context=3, image_shape=(256, 256), device=device)
    with torch.no_grad():
        g = model.encoder(model.data_shim(data)["context"], 0, deterministic=True)
        out = model.test_step(data).color
    torch.cuda.synchronize()
    assert g.means.shape == (1, 3 * 256 * 256, 3)
    assert out.shape == (1, 3, 3, 256, 256) and torch.isfinite(out).all()
