"""End-to-end inference step (reference ModelWrapper.test_step, src/model/model_wrapper.py:185-323):
data shim -> EncoderTrans -> DecoderSplattingHIP for every target view, on synthetic scenes.

Weights are seeded random (no checkpoint is reachable offline); the work per step does not depend
on their values. `build_e2e_workload` is the bench.py workload: one step = B scenes of 2 context
views -> 3 rendered 256x256 target views each.
"""
from __future__ import annotations

import torch

from . import synthetic as S
from .misc.benchmarker import stage
from .model.decoder import DatasetCfgLite, DecoderSplattingHIP, DecoderSplattingHIPCfg
from .model.encoder import EncoderTrans, EncoderTransCfg


class TransplatModel(torch.nn.Module):
    """encoder + decoder pair with the reference ModelWrapper's `encoder.` / `decoder.` names."""

    def __init__(self, encoder_cfg: EncoderTransCfg | None = None, decoder_cfg: DecoderSplattingHIPCfg | None = None,
                 background=(0.0, 0.0, 0.0)):
        super().__init__()
        self.encoder = EncoderTrans(encoder_cfg or EncoderTransCfg())
        self.decoder = DecoderSplattingHIP(decoder_cfg or DecoderSplattingHIPCfg(), DatasetCfgLite(background))
        self.data_shim = self.encoder.get_data_shim()

    @torch.no_grad()
    def test_step(self, batch: dict, global_step: int = 0, benchmarker=None):
        batch = self.data_shim(batch)
        _, _, _, h, w = batch["target"]["image"].shape
        gaussians = self.encoder(batch["context"], global_step, deterministic=True, benchmarker=benchmarker)
        t = batch["target"]
        with stage(benchmarker, "decoder"):  # reference model_wrapper.py:209-218 tags it "decoder"
            return self.decoder(gaussians, t["extrinsics"], t["intrinsics"], t["near"], t["far"], (h, w))

    def load_checkpoint(self, path: str, strict: bool = True):
        """Lightning checkpoint of the reference (`state_dict` with `encoder.` / `decoder.` keys);
        loaded with weights_only=True (nothing in the file is executed)."""
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
        sd = ckpt.get("state_dict", ckpt)
        sd = {k: v for k, v in sd.items() if k.startswith("encoder.")}
        missing, unexpected = self.load_state_dict(sd, strict=False)
        missing = [k for k in missing if k.startswith("encoder.")]
        if strict and (missing or unexpected):
            raise RuntimeError(f"checkpoint mismatch: missing {missing[:5]}..., unexpected {unexpected[:5]}...")
        return missing, unexpected


def build_model(device, dense_dtype: str = "fp32", seed: int = 0, num_context_views: int = 2,
                attn_dtype: str = "auto") -> TransplatModel:
    torch.manual_seed(seed)
    cfg = EncoderTransCfg(dense_dtype=dense_dtype, num_context_views=num_context_views, attn_dtype=attn_dtype)
    model = TransplatModel(cfg, DecoderSplattingHIPCfg(check_overflow=False))
    S.init_synthetic_weights(model.encoder, seed)
    model = model.eval().to(device)
    if dense_dtype == "bf16" and torch.device(device).type == "cuda":
        example = S.make_batch(1, num_context=num_context_views, image_shape=(256, 256), device=device)
        precast_autocast_weights(model, example)
    return model


_AUTOCAST_MATMULS = None


def precast_autocast_weights(model: torch.nn.Module, example: dict) -> int:
    """Store once, in bf16, every parameter whose only uses are conv / linear calls under bf16
    autocast. Autocast would otherwise re-cast those fp32 weights on every step (its cast cache
    lives only as long as one autocast region): ~600 cast kernels per captured step. The values the
    convolutions see are identical (the same round-to-nearest cast, done once). Uses are recorded by
    a TorchFunctionMode over one eager test_step; a parameter used anywhere else (norms, HIP
    kernels, autocast-disabled regions) stays fp32. Returns the number of parameters cast."""
    import torch.nn.functional as F
    from torch.overrides import TorchFunctionMode

    global _AUTOCAST_MATMULS
    if _AUTOCAST_MATMULS is None:
        _AUTOCAST_MATMULS = {F.conv1d, F.conv2d, F.conv3d, F.linear, F.conv_transpose1d, F.conv_transpose2d,
                             torch.conv2d, torch.conv1d, torch.conv_transpose2d}
    params = {id(p): p for p in model.parameters()}
    ok: dict[int, bool] = {}

    class _Record(TorchFunctionMode):
        def __torch_function__(self, func, types, args=(), kwargs=None):
            kwargs = kwargs or {}
            castable = func in _AUTOCAST_MATMULS and torch.is_autocast_enabled("cuda")
            for a in (*args, *kwargs.values()):
                if isinstance(a, (list, tuple)):
                    for x in a:
                        if id(x) in params:
                            ok[id(x)] = False
                elif id(a) in params:
                    ok[id(a)] = ok.get(id(a), True) and castable
            return func(*args, **kwargs)

    with torch.no_grad(), _Record():
        model.test_step(example)
    n = 0
    for pid, good in ok.items():
        p = params[pid]
        if good and p.dtype == torch.float32:
            p.data = p.data.to(torch.bfloat16)
            n += 1
    return n


class GraphedStep:
    """The whole test_step captured once into a hipGraph (torch.cuda.CUDAGraph) and replayed:
    at batch 1 the ~2,500 kernel launches of a step otherwise leave ~30 % of the GPU time idle.
    Inputs live in static buffers: `run(batch)` copies a new batch in (device-to-device) and
    replays; outputs are the graph's static output tensors (valid until the next replay)."""

    def __init__(self, model: TransplatModel, example: dict, warmup: int = 2):
        from . import _lib

        if _lib.debug_enabled():  # its per-launch hipDeviceSynchronize is illegal inside a capture
            raise RuntimeError("tsplat debug mode (TSPLAT_DEBUG=1 / tsplat_set_debug) synchronises after every "
                               "launch and cannot be captured into a hipGraph: run the step eagerly "
                               "(bench.py --no-graph, graph=False)")
        self.model = model
        self.static = _clone_batch(example)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                model.test_step(self.static)
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = model.test_step(self.static)

    def run(self, batch: dict | None = None):
        if batch is not None:
            _copy_batch(self.static, batch)
        self.graph.replay()
        return self.out


def _clone_batch(b):
    if isinstance(b, dict):
        return {k: _clone_batch(v) for k, v in b.items()}
    return b.clone() if torch.is_tensor(b) else b


def _copy_batch(dst, src):
    for k, v in src.items():
        if isinstance(v, dict):
            _copy_batch(dst[k], v)
        elif torch.is_tensor(v):
            dst[k].copy_(v, non_blocking=True)


def precision_label(dense_dtype: str, attn_dtype: str = "auto") -> str:
    """The precision MODES a step runs under (what the model was asked for); route_label() states
    what the step then actually launched."""
    from .kernels import auto_attention

    attn = attn_dtype if attn_dtype != "auto" else auto_attention(dense_dtype)
    dense = {"fp32": "exact fp32", "bf16x3": "bf16x3 (split-bf16 products, fp32 accumulation; >= TF32)",
             "bf16": "bf16 (autocast)"}[dense_dtype]
    return f"dense mode {dense}, window-attention mode {attn}"


def route_label(model, data) -> str:
    """Run one eager step under routes.record() and state what ran in which arithmetic (every HIP
    entry point and every library GEMM / convolution the step reached, with launch counts)."""
    from . import routes

    with torch.no_grad(), routes.record() as r:
        model.test_step(data)
    torch.cuda.synchronize()
    return r.label()


def build_e2e_workload(batch: int, device, scene_offset: int = 0, dense_dtype: str = "fp32", graph: bool = True,
                       attn_dtype: str = "auto"):
    from .gemm_tuning import use_tuned_gemms

    use_tuned_gemms(device, dense_dtype)  # recorded library GEMM solutions (replay only), before any capture
    model = build_model(device, dense_dtype, attn_dtype=attn_dtype)
    data = S.make_batch(batch, image_shape=(256, 256), scene_offset=scene_offset, device=device)
    if graph:
        graphed = GraphedStep(model, data)

        def step():
            return graphed.run()
    else:
        def step():
            return model.test_step(data)

    info = {
        "eager_step": lambda: model.test_step(data),
        "views_per_step": batch * data["target"]["near"].shape[1],
        "workload": f"e2e TranSplat test_step: {batch} scene(s) x (2 ctx -> 3 tgt) 256x256; "
                    + precision_label(dense_dtype, attn_dtype) + "; launched per step: " + route_label(model, data),
    }
    return step, info, model
