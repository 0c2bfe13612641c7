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
    from transplat_amd.misc.benchmarker import Benchmarker

    enc = S.init_synthetic_weights(EncoderTrans(EncoderTransCfg()).eval())
    batch = S.make_batch(1, image_shape=(128, 128))
    bm = Benchmarker()
    with torch.no_grad():
        g = enc(batch["context"], 0, deterministic=True, benchmarker=bm)
    assert g.means.shape == (1, 2 * 128 * 128, 3) and g.harmonics.shape == (1, 2 * 128 * 128, 3, 25)
    for t in (g.means, g.covariances, g.harmonics, g.opacities):
        assert torch.isfinite(t).all()
    # the reference's stage tags (encoder_trans.py:188-294, depth_predictor_trans.py:320-456)
    tags = set(bm.summary())
    assert {"encoder_1_prep_intrinsics", "encoder_2_backbone", "encoder_3_depth_anything",
            "encoder_4_depth_predictor", "encoder_5_gaussian_adapter", "encoder_4a_prep_features",
            "encoder_4b_cost_volume_matching", "encoder_4c_cost_volume_unet", "encoder_4d_coarse_depth",
            "encoder_4e_depth_refine_unet", "encoder_4f_gaussian_head"} <= tags


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


@pytest.mark.gpu
def test_bf16_weight_precast_keeps_outputs(device):
    """bf16 dense mode stores conv / linear weights in bf16 once (e2e.precast_autocast_weights)
    instead of letting autocast re-cast them each step. The bf16 values are the same (checked
    parameter by parameter); params used outside autocast (norms, HIP kernels, fp32 islands) stay
    fp32. Library algorithm choices differ between the two models, so the rendered views are
    compared through their distance to the fp32 model: the pre-cast model must be as close to it
    as the re-casting one."""
    from transplat_amd import e2e

    data = S.make_batch(1, image_shape=(256, 256), device=device)
    cast = e2e.build_model(device, "bf16")

    def fresh(dtype):
        torch.manual_seed(0)
        cfg = e2e.EncoderTransCfg(dense_dtype=dtype)
        m = e2e.TransplatModel(cfg, e2e.DecoderSplattingHIPCfg(check_overflow=False))
        S.init_synthetic_weights(m.encoder, 0)
        return m.eval().to(device)

    plain, ref = fresh("bf16"), fresh("fp32")
    n_bf16 = sum(p.dtype == torch.bfloat16 for p in cast.parameters())
    # (the convolutions on the HIP bf16 kernel keep fp32 parameters: kernels.conv_bf16_pack_weight
    # rounds them to bf16 once, into its packed operand layout)
    assert n_bf16 > 200
    for (name, p), q in zip(cast.named_parameters(), plain.parameters()):
        if p.dtype == torch.bfloat16:
            assert "norm" not in name.split(".")[-2]
            assert torch.equal(p, q.to(torch.bfloat16))
        else:
            assert torch.equal(p, q)
    with torch.no_grad():
        a = cast.test_step(data).color.float()
        b = plain.test_step(data).color.float()
        r = ref.test_step(data).color.float()
    torch.cuda.synchronize()
    assert torch.isfinite(a).all()
    ea, eb = (a - r).abs().mean().item(), (b - r).abs().mean().item()
    assert ea < 1.5 * eb + 1e-3, (ea, eb)


def _psnr(a, b):
    mse = ((a.clamp(0, 1) - b.clamp(0, 1)) ** 2).flatten(2).mean(-1)
    return (-10 * torch.log10(mse.clamp_min(1e-20))).min().item()


@pytest.mark.gpu
def test_c3_batch8_bf16_step(device):
    """Config C3: 8 scenes per step, bf16 dense layers + bf16-MFMA window attention, fp32
    correlation and fp32 rasterizer, as one replayed hipGraph (the bench's C3 line). Checked
    against the fp32 model on the same weights and inputs: worst view above 30 dB PSNR, mean
    absolute difference < 2e-2 (the bf16 attention kernel alone is held to
    1.5e-2 max abs against the fp32 oracle in test_encoder_ops). Also: the graph replays the eager
    bf16 step, and the batch-8 fp32 step renders each scene as the batch-1 step does."""
    from transplat_amd.e2e import GraphedStep, build_model

    data = S.make_batch(8, image_shape=(256, 256), device=device)
    bf = build_model(device, "bf16")
    graphed = GraphedStep(bf, data)
    out_bf = graphed.run().color.float().clone()
    eager_bf = bf.test_step(data).color.float()
    del graphed, bf
    fp = build_model(device, "fp32")
    out_fp = fp.test_step(data).color.clone()
    one = S.make_batch(1, image_shape=(256, 256), scene_offset=5, device=device)
    out_one = fp.test_step(one).color
    torch.cuda.synchronize()
    assert out_bf.shape == (8, 3, 3, 256, 256) and torch.isfinite(out_bf).all()
    mad = (out_bf - out_fp).abs().mean().item()
    psnr = _psnr(out_bf, out_fp)
    mad_ge = (out_bf - eager_bf).abs().mean().item()
    psnr_ge = _psnr(out_bf, eager_bf)
    mad_one = (out_fp[5] - out_one[0]).abs().mean().item()
    print(f"C3 bf16 vs fp32: mean abs {mad:.3e}, worst-view PSNR {psnr:.2f} dB; graph vs eager bf16: "
          f"{mad_ge:.3e}, {psnr_ge:.2f} dB; fp32 b8[5] vs b1: {mad_one:.3e}")
    # measured on MI355X: 1.27e-2 / 34.6 dB vs fp32, and 1.08e-2 / 36.3 dB between two bf16 runs
    # (graph vs eager pick different library algorithms; bf16 rounding, 2^-8 relative, is
    # amplified by the randomly initialised network): the bf16 step is as close to fp32 as
    # bf16 is to itself
    assert mad < 2e-2 and psnr > 30.0
    assert mad_ge < 2e-2 and psnr_ge > 30.0
    assert mad_one < 1e-4


@pytest.mark.gpu
def test_bf16x3_step_vs_exact_fp32(device):
    """The C2 headline's dense-layer mode (EncoderTransCfg.dense_dtype "bf16x3": split-bf16 Winograd
    convolutions and library GEMMs, the stand-in for the reference's TF32) against the exact-fp32
    model on the same weights and inputs, as one replayed hipGraph. Printed: the Gaussians' and the
    pixels' differences, next to the noise between two exact-fp32 eager steps (library reduction
    orders differ per call). Measured on MI355X (profiles/r4/): means 3.3e-3 relative (two fp32 steps
    1.2e-4: the randomly initialised network amplifies the ~6e-6 per-convolution difference, mostly
    at depth discontinuities), harmonics 2.8e-5, pixels max 1.5e-2 / mean 2.4e-5, worst view 79.7 dB.
    Bounds: 2x the measured means error, and the pixel envelope test_e2e_graph_matches_eager holds
    two fp32 runs to (max 2e-2, mean 1e-4), worst view above 70 dB."""
    from transplat_amd.e2e import GraphedStep, build_model

    data = S.make_batch(1, image_shape=(256, 256), device=device)

    def gauss_and_color(model, graph=False):
        with torch.no_grad():
            g = model.encoder(model.data_shim(data)["context"], 0, deterministic=True)
            out = GraphedStep(model, data).run().color if graph else model.test_step(data).color
        torch.cuda.synchronize()
        return g.means.clone(), g.harmonics.clone(), out.float().clone()

    fp = build_model(device, "fp32")
    ref, ref2 = gauss_and_color(fp), gauss_and_color(fp)
    del fp
    x3 = gauss_and_color(build_model(device, "bf16x3"), graph=True)
    rel = lambda a, b: ((a - b).abs().max() / b.abs().max()).item()
    print(f"bf16x3 vs fp32: means {rel(x3[0], ref[0]):.2e}, harmonics {rel(x3[1], ref[1]):.2e}, pixels max "
          f"{(x3[2] - ref[2]).abs().max().item():.2e} mean {(x3[2] - ref[2]).abs().mean().item():.2e}, PSNR "
          f"{_psnr(x3[2], ref[2]):.1f} dB | two fp32 steps: means {rel(ref2[0], ref[0]):.2e}, pixels max "
          f"{(ref2[2] - ref[2]).abs().max().item():.2e} mean {(ref2[2] - ref[2]).abs().mean().item():.2e}")
    assert torch.isfinite(x3[2]).all()
    assert rel(x3[0], ref[0]) < 7e-3 and rel(x3[1], ref[1]) < 1e-2
    assert _psnr(x3[2], ref[2]) > 70.0
    assert (x3[2] - ref[2]).abs().max().item() < 2e-2
    assert (x3[2] - ref[2]).abs().mean().item() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("dense", ["bf16x3", "fp32"])
def test_graph_replays_equal_eager(device, dense):
    """The bench's timed object is a hipGraph replay of the step with branches on side streams
    (streams.fork); a replay must be the eager step bit for bit, every time. Round 6 found replays
    that were not (1-3 of 4 moved up to 4 % of the pixels, tools/graph_vs_eager.py): a cross-stream
    hazard that eager runs, with their launch gaps, did not show. Six replays against two eager
    steps, with the bench's tuned library GEMMs."""
    from transplat_amd.e2e import GraphedStep, build_model
    from transplat_amd.gemm_tuning import use_tuned_gemms

    use_tuned_gemms(device, dense)
    data = S.make_batch(1, image_shape=(256, 256), device=device)
    model = build_model(device, dense)
    with torch.no_grad():
        e1 = model.test_step(data).color.float().clone()
        e2 = model.test_step(data).color.float().clone()
        g = GraphedStep(model, data)
        diffs = []
        for _ in range(6):
            r = g.run().color.float().clone()
            torch.cuda.synchronize()
            diffs.append((r - e1).abs().max().item())
    print(f"{dense}: eager vs eager {(e2 - e1).abs().max().item():.2e}, replays vs eager {diffs}")
    assert torch.equal(e1, e2)
    assert max(diffs) == 0.0, diffs


@pytest.mark.gpu
def test_c3_stated_bf16_attention_step(device):
    """Config C3 as BASELINE.json states it: batch 8, bf16 window attention (attn_dtype "bf16"),
    fp32-class dense layers (bf16x3), fp32 correlation and raster, one replayed hipGraph; against
    the exact-fp32 model on the same inputs. Floor (written here): worst view above 40 dB PSNR --
    the bf16 attention kernel alone holds 1.5e-2 max abs against the fp32 oracle (test_encoder_ops),
    and the all-bf16 C3 variant sits at ~35 dB (test_c3_batch8_bf16_step)."""
    from transplat_amd.e2e import GraphedStep, build_model

    data = S.make_batch(8, image_shape=(256, 256), device=device)
    m = build_model(device, "bf16x3", attn_dtype="bf16")
    out = GraphedStep(m, data).run().color.float().clone()
    del m
    ref = build_model(device, "fp32").test_step(data).color.float()
    torch.cuda.synchronize()
    psnr, mad = _psnr(out, ref), (out - ref).abs().mean().item()
    print(f"C3 stated (bf16 attention, bf16x3 dense) vs fp32: worst-view PSNR {psnr:.2f} dB, mean abs {mad:.3e}")
    assert out.shape == (8, 3, 3, 256, 256) and torch.isfinite(out).all()
    assert psnr > 40.0


@pytest.mark.gpu
def test_tuned_gemms_keep_outputs(device):
    """The bench step replays the committed TunableOp GEMM choices (transplat_amd/tuned/
    gemms_gfx950.csv, gemm_tuning.use_tuned_gemms). The same eager step with and without them must
    agree within the envelope two eager steps already show (library reduction orders differ per
    call: test_e2e_graph_matches_eager), on the Gaussians and on the rendered views."""
    import torch.cuda.tunable as tun

    from transplat_amd.e2e import build_model
    from transplat_amd.gemm_tuning import use_tuned_gemms

    model = build_model(device)
    data = S.make_batch(1, image_shape=(256, 256), device=device)

    def run():
        with torch.no_grad():
            b = model.data_shim(data)
            g = model.encoder(b["context"], 0, deterministic=True)
            out = model.test_step(data).color
        torch.cuda.synchronize()
        return g.means.clone(), g.harmonics.clone(), out.clone()

    was = tun.is_enabled()
    tun.enable(False)
    try:
        ref = run()
        assert use_tuned_gemms(device), "committed GEMM solutions not loaded (validator mismatch?)"
        assert tun.is_enabled() and not tun.tuning_is_enabled()
        tuned = run()
    finally:
        tun.enable(was)
    rel = lambda a, b: ((a - b).abs().max() / b.abs().max()).item()
    print(f"tuned vs default GEMMs: means {rel(tuned[0], ref[0]):.2e}, harmonics {rel(tuned[1], ref[1]):.2e}, "
          f"pixels max {(tuned[2] - ref[2]).abs().max().item():.2e} mean {(tuned[2] - ref[2]).abs().mean().item():.2e}")
    # measured on MI355X over rounds 3-5 (profiles/r3/pytest_tuned_s3.log, pytest_gpu_s1.log): means
    # 1.3e-4 - 1.6e-4, harmonics 1.1e-6 - 1.2e-6, pixels mean 1.2e-6 - 1.6e-6 (two default fp32 steps
    # alone: pixels max up to 3.4e-3); bounds ~2x the largest measured. The pixel MAX is set by a
    # few blend decisions (alpha >= 1/255, T >= 1e-4) that flip on last-bit differences of the
    # Gaussians: 1.4e-3 - 3.8e-3 in rounds 3-4, one pixel at 1.18e-2 in round 5 (a flipped stop
    # decision moves a pixel by up to ~alpha T ~ 1e-2; the means themselves move by ~1.3e-4), so it
    # is bounded by that size and by how many values move more than 1e-3 (1.5e-4 of them in round 5),
    # not tighter.
    d = (tuned[2] - ref[2]).abs()
    n_big = int((d > 1e-2).sum().item())
    print(f"  values moving > 1e-3: {(d > 1e-3).float().mean().item():.2e} of {d.numel()}; > 1e-2: {n_big}")
    assert rel(tuned[0], ref[0]) < 4e-4 and rel(tuned[1], ref[1]) < 3e-6
    assert d.max().item() < 3e-2 and (d > 1e-3).float().mean().item() < 1e-3
    # a flipped blend decision moves single pixels; a systematic shift would move many past 1e-2
    assert n_big <= 8
    assert d.mean().item() < 3e-6


@pytest.mark.gpu
def test_tuned_gemms_keep_outputs_bf16(device):
    """C3's bf16 library GEMMs replay the allow-list choices of tools/tune_gemms_bf16.py from the same
    file; the bf16 step with and without them must agree within the bf16 envelope that
    test_c3_batch8_bf16_step holds two bf16 runs to (mean abs < 2e-2, worst-view PSNR > 30 dB: a
    different reduction order flips bf16 roundings, 2^-8 relative, which the randomly initialised
    network amplifies -- two default runs whose library algorithms differ read ~36 dB). A warm-up
    step first settles the weight pre-cast and MIOpen's algorithm choices, and the noise between two
    default steps is printed next to the tuned one."""
    import torch.cuda.tunable as tun

    from transplat_amd.e2e import build_model
    from transplat_amd.gemm_tuning import use_tuned_gemms

    model = build_model(device, "bf16")
    data = S.make_batch(2, image_shape=(256, 256), device=device)

    def run():
        with torch.no_grad():
            out = model.test_step(data).color.float()
        torch.cuda.synchronize()
        return out.clone()

    was = tun.is_enabled()
    tun.enable(False)
    try:
        run()
        ref = run()
        ref2 = run()
        assert use_tuned_gemms(device, "bf16")
        tuned = run()
    finally:
        tun.enable(was)
    psnr, noise = _psnr(tuned, ref), _psnr(ref2, ref)
    mad = (tuned - ref).abs().mean().item()
    print(f"bf16 tuned vs default GEMMs: worst-view PSNR {psnr:.1f} dB, mean abs {mad:.2e}; "
          f"two default steps: {noise:.1f} dB")
    assert torch.isfinite(tuned).all()
    assert mad < 2e-2 and psnr > 30.0
