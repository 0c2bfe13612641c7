"""Scene-sharded evaluation: rank r of N takes scenes r, r+N, ... of the evaluation
index, runs the reference test_step sequence (encoder -> decoder -> PSNR per target view,
reference src/model/model_wrapper.py:185-323) and the per-scene metrics are gathered once at the
end with ONE all_gather of a fixed-width fp32 tensor [n_local, 4] = (scene_idx, psnr, n_views,
seconds) — RCCL over xGMI on GPUs, gloo on CPU. No collective touches the data path.

With no dataset offline, scenes are synthetic (transplat_amd.synthetic) unless a loader is passed;
the evaluation index (e.g. the reference's assets/evaluation_index_re10k_small.json) supplies the
scene keys and context/target frame indices.

The step the CLI evaluates is the benched one: `GraphedSteps` replays the whole test_step as one
hipGraph per input-shape signature (bench.py's timed region), in the bench's default dense precision
(bf16x3). Per scene the PSNR stays on the device and the step is bracketed by HIP events; the host
synchronises ONCE per shard, after its last scene, then reads the PSNRs and event times.
"""
from __future__ import annotations

import json
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Callable, Optional

import torch
import torch.distributed as dist

from .evaluation.metrics import compute_psnr


@dataclass
class SceneResult:
    scene_idx: int
    psnr: float
    n_views: int
    seconds: float
    capture: bool = False  # the step captured its hipGraph (warmup + capture inside `seconds`)


def load_index(path: str | Path) -> list[tuple[str, dict]]:
    """Non-null entries of an evaluation index, in file order (reference
    ViewSamplerEvaluation, src/dataset/view_sampler/view_sampler_evaluation.py:44-59)."""
    data = json.loads(Path(path).read_text())
    return [(k, v) for k, v in data.items() if v is not None]


def shard(items: list, rank: int, world: int) -> list[tuple[int, object]]:
    """Scenes r, r + N, r + 2N, ... with their global indices."""
    return [(i, items[i]) for i in range(rank, len(items), world)]


def gather_results(local: list[SceneResult], device: torch.device, world: int) -> list[SceneResult]:
    """One all_gather of [n_local_max, 5] fp32 rows (padded with scene_idx = -1)."""
    rows = torch.tensor([[r.scene_idx, r.psnr, r.n_views, r.seconds, float(r.capture)] for r in local],
                        dtype=torch.float32, device=device).reshape(-1, 5)
    if world == 1:
        gathered = [rows]
    else:
        n = torch.tensor([rows.shape[0]], device=device)
        counts = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(counts, n)
        nmax = int(max(c.item() for c in counts))
        pad = torch.full((nmax, 5), -1.0, device=device)
        pad[: rows.shape[0]] = rows
        gathered = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(gathered, pad)
    out = []
    for g in gathered:
        for row in g.cpu().tolist():
            if row[0] >= 0:
                out.append(SceneResult(int(row[0]), row[1], int(row[2]), row[3], row[4] > 0.5))
    return sorted(out, key=lambda r: r.scene_idx)


def _raster_status(device: torch.device) -> None:
    """Raise if any rasterizer call on `device` exceeded its instance capacity (the eval model is
    built with check_overflow=False so its step can be a replayed hipGraph; the flag is sticky)."""
    from .model.decoder.hip_splatting import check_status

    check_status(device)


class GraphedSteps:
    """`step(batch) -> color` as the bench runs it: the model's whole test_step captured once per
    input-shape signature into a replayed hipGraph (e2e.GraphedStep; a new batch is copied into the
    graph's static inputs). The returned color is the graph's static output, valid until the next
    replay -- `_run_scene` reduces it to a PSNR on the same stream before that."""

    def __init__(self, model, max_graphs: int = 4):
        self.model, self.max_graphs, self.graphs = model, max_graphs, {}
        self.last_captured = False  # the last call captured a graph (its time includes warmup + capture)

    @staticmethod
    def signature(batch) -> tuple:
        out = []
        for k in sorted(batch):
            v = batch[k]
            if isinstance(v, dict):
                out.append((k, GraphedSteps.signature(v)))
            elif torch.is_tensor(v):
                out.append((k, tuple(v.shape), v.dtype))
        return tuple(out)

    def __call__(self, batch):
        from .e2e import GraphedStep

        sig = self.signature(batch)
        g = self.graphs.get(sig)
        self.last_captured = g is None
        if g is None:
            if len(self.graphs) >= self.max_graphs:
                self.graphs.pop(next(iter(self.graphs)))
            g = self.graphs[sig] = GraphedStep(self.model, batch)
        return g.run(batch).color


class _Pending:
    """Per-scene results held on the device until the shard's single synchronisation. After each
    scene a device-side copy of the rasterizer's sticky overflow flag is kept, so an overflow found
    at the end names the first scene that raised it."""

    def __init__(self, device: torch.device):
        self.device, self.rows = device, []

    def run(self, idx: int, step, batch: dict) -> None:
        from .model.decoder.hip_splatting import status_tensor

        gt = batch["target"]["image"][0]
        if self.device.type == "cuda":
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            color = step(batch)
            psnr = compute_psnr(gt.to(color.device), color[0]).mean()  # before a replay reuses color
            e1.record()
            st = status_tensor(self.device)
            self.rows.append((idx, psnr, int(color.shape[1]), (e0, e1), getattr(step, "last_captured", False),
                              st.clone() if st is not None else None))
        else:
            t0 = time.perf_counter()
            color = step(batch)
            psnr = compute_psnr(gt.to(color.device), color[0]).mean()
            self.rows.append((idx, psnr, int(color.shape[1]), time.perf_counter() - t0, False, None))

    def results(self) -> list[SceneResult]:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
            # a capacity overflow must not become a silent wrong-image PSNR: name the first scene
            bad = [r[0] for r in self.rows if r[5] is not None and int(r[5].item()) != 0]
            if bad:
                _raster_status(self.device)  # clears the sticky flag and raises
                raise RuntimeError(f"tsplat_raster_fwd: instance capacity exceeded (first at scene {bad[0]})")
            _raster_status(self.device)
        out = []
        for idx, psnr, nv, t, cap, _ in self.rows:
            sec = t[0].elapsed_time(t[1]) / 1e3 if isinstance(t, tuple) else t
            out.append(SceneResult(idx, float(psnr.item()), nv, sec, bool(cap)))
        return out


def evaluate(step: Callable[[dict], torch.Tensor], scenes: list, make_batch: Callable[[int, object], dict],
             device: torch.device, rank: int = 0, world: int = 1) -> list[SceneResult]:
    """`make_batch(scene_idx, entry)` -> batch dict (b = 1); `step(batch)` -> color [1, V, 3, H, W].
    One device synchronisation per shard (after its last scene); `seconds` is each scene's step +
    PSNR time from HIP events on the GPU (host wall time on CPU)."""
    pend = _Pending(device)
    for idx, entry in shard(scenes, rank, world):
        pend.run(idx, step, make_batch(idx, entry))
    return gather_results(pend.results(), device, world)


def evaluate_stream(step: Callable[[dict], torch.Tensor], examples, device: torch.device, rank: int = 0,
                    world: int = 1) -> list[SceneResult]:
    """Like `evaluate`, over an iterable of ready batches (the chunk reader): example i of the
    stream is scene i, and rank r keeps i = r, r + N, ... (every rank decodes the same stream
    order, so the split matches the index-driven one)."""
    pend = _Pending(device)
    for idx, batch in enumerate(examples):
        if idx % world != rank:
            continue
        batch = {k: ({kk: vv.to(device) for kk, vv in v.items()} if isinstance(v, dict) else v)
                 for k, v in batch.items()}
        pend.run(idx, step, batch)
    return gather_results(pend.results(), device, world)


def summarize(results: list[SceneResult]) -> dict:
    """PSNR over every scene; `seconds` over the steady scenes only (a scene whose step captured a
    hipGraph carries the warmup and the capture, reported apart as `capture_seconds`)."""
    n = len(results)
    steady = [r for r in results if not r.capture]
    return {
        "scenes": n,
        "psnr": sum(r.psnr for r in results) / max(n, 1),
        "views": sum(r.n_views for r in results),
        "seconds": sum(r.seconds for r in steady),
        "steady_scenes": len(steady),
        "capture_scenes": n - len(steady),
        "capture_seconds": sum(r.seconds for r in results if r.capture),
    }


def index_batch(idx: int, key: str, entry: dict, image_shape=(256, 256), device="cpu") -> dict:
    """Synthetic stand-in for the re10k chunk reader: the index entry's frame numbers place the
    targets along the context baseline (t = (frame - ctx0) / (ctx1 - ctx0)), the scene index
    seeds the images. Real frames replace this once the dataset is available."""
    from . import synthetic as S

    c0, c1 = entry["context"][0], entry["context"][-1]
    span = max(c1 - c0, 1)
    ts = [(t - c0) / span for t in entry["target"]]
    return S.make_batch(1, num_context=len(entry["context"]), num_target=len(ts), image_shape=image_shape,
                        scene_offset=idx, device=device, target_ts=ts)


def main(argv=None):
    """`python -m transplat_amd.evaluate --index <evaluation_index.json>` (one process per GPU under
    torch.distributed.run; RCCL for the final gather). Prints one JSON summary on rank 0."""
    import argparse
    import os

    ap = argparse.ArgumentParser()
    ap.add_argument("--index", required=True)
    ap.add_argument("--checkpoint", default=None, help="reference Lightning checkpoint (loaded weights_only)")
    ap.add_argument("--dense-dtype", choices=["fp32", "bf16x3", "bf16"], default="bf16x3",
                    help="dense-layer precision; bf16x3 = the bench's default (>= the reference's TF32); "
                         "fp32 = the exact-fp32 parity path the module goldens pin")
    ap.add_argument("--no-graph", action="store_true", help="eager test_step per scene instead of the replayed hipGraph")
    ap.add_argument("--limit", type=int, default=None, help="first N scenes of the index")
    ap.add_argument("--data-root", action="append", default=None,
                    help="dataset root holding test/*.torch chunks (repeatable); real frames instead of synthetic")
    ap.add_argument("--experiment", choices=["re10k", "acid", "dtu"], default="re10k")
    args = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device(f"cuda:{local}")
    torch.cuda.set_device(device)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=device)
    from .e2e import build_model, precision_label

    from .gemm_tuning import use_tuned_gemms

    torch.backends.cudnn.benchmark = True  # bench.py's default MIOpen algorithm search
    use_tuned_gemms(device, args.dense_dtype)  # the bench's recorded library GEMM solutions, before any capture
    model = build_model(device, args.dense_dtype)
    if args.checkpoint:
        model.load_checkpoint(args.checkpoint)
    step = (lambda batch: model.test_step(batch).color) if args.no_graph else GraphedSteps(model)
    if args.data_root:
        from itertools import islice

        from .dataset import EXPERIMENTS, ChunkDatasetCfg, ChunkTestDataset

        cfg = ChunkDatasetCfg(roots=tuple(args.data_root), **EXPERIMENTS[args.experiment])
        ds = ChunkTestDataset.from_index_file(cfg, args.index)
        stream = (ChunkTestDataset.batch(ex) for ex in islice(iter(ds), args.limit))
        results = evaluate_stream(step, stream, device, rank, world)
        data = f"{args.experiment} chunks under {args.data_root}"
    else:
        scenes = load_index(args.index)[: args.limit]
        results = evaluate(step, [(k, v) for k, v in scenes],
                           lambda i, kv: index_batch(i, kv[0], kv[1], device=device), device, rank, world)
        data = "synthetic frames at the index's frame positions"
    if rank == 0:
        summary = summarize(results)
        summary.update({"index": str(args.index), "world": world, "weights": args.checkpoint or "synthetic",
                        "data": data, "dense_dtype": args.dense_dtype, "graph": not args.no_graph,
                        "precision": precision_label(args.dense_dtype)})
        print(json.dumps(summary), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
