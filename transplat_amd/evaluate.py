"""Scene-sharded evaluation: rank r of N takes scenes r, r+N, ... of the evaluation
index, runs the reference test_step sequence (encoder -> decoder -> PSNR per target view,
reference src/model/model_wrapper.py:185-323) and the per-scene metrics are gathered once at the
end with ONE all_gather of a fixed-width fp32 tensor [n_local, 4] = (scene_idx, psnr, n_views,
seconds) — RCCL over xGMI on GPUs, gloo on CPU. No collective touches the data path.

With no dataset offline, scenes are synthetic (transplat_amd.synthetic) unless a loader is passed;
the evaluation index (e.g. the reference's assets/evaluation_index_re10k_small.json) supplies the
scene keys and context/target frame indices.
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


def load_index(path: str | Path) -> list[tuple[str, dict]]:
    """Non-null entries of an evaluation index, in file order (reference
    ViewSamplerEvaluation, src/dataset/view_sampler/view_sampler_evaluation.py:44-59)."""
    data = json.loads(Path(path).read_text())
    return [(k, v) for k, v in data.items() if v is not None]


def shard(items: list, rank: int, world: int) -> list[tuple[int, object]]:
    """Scenes r, r + N, r + 2N, ... with their global indices."""
    return [(i, items[i]) for i in range(rank, len(items), world)]


def gather_results(local: list[SceneResult], device: torch.device, world: int) -> list[SceneResult]:
    """One all_gather of [n_local_max, 4] fp32 rows (padded with scene_idx = -1)."""
    rows = torch.tensor([[r.scene_idx, r.psnr, r.n_views, r.seconds] for r in local], dtype=torch.float32,
                        device=device).reshape(-1, 4)
    if world == 1:
        gathered = [rows]
    else:
        n = torch.tensor([rows.shape[0]], device=device)
        counts = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(counts, n)
        nmax = int(max(c.item() for c in counts))
        pad = torch.full((nmax, 4), -1.0, device=device)
        pad[: rows.shape[0]] = rows
        gathered = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(gathered, pad)
    out = []
    for g in gathered:
        for row in g.cpu().tolist():
            if row[0] >= 0:
                out.append(SceneResult(int(row[0]), row[1], int(row[2]), row[3]))
    return sorted(out, key=lambda r: r.scene_idx)


def evaluate(step: Callable[[dict], torch.Tensor], scenes: list, make_batch: Callable[[int, object], dict],
             device: torch.device, rank: int = 0, world: int = 1) -> list[SceneResult]:
    """`make_batch(scene_idx, entry)` -> batch dict (b = 1); `step(batch)` -> color [1, V, 3, H, W]."""
    local = []
    for idx, entry in shard(scenes, rank, world):
        batch = make_batch(idx, entry)
        t0 = time.perf_counter()
        color = step(batch)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        dt = time.perf_counter() - t0
        gt = batch["target"]["image"][0].to(color.device)
        psnr = compute_psnr(gt, color[0]).mean().item()
        local.append(SceneResult(idx, psnr, int(color.shape[1]), dt))
    return gather_results(local, device, world)


def summarize(results: list[SceneResult]) -> dict:
    n = len(results)
    return {
        "scenes": n,
        "psnr": sum(r.psnr for r in results) / max(n, 1),
        "views": sum(r.n_views for r in results),
        "seconds": sum(r.seconds for r in results),
    }
