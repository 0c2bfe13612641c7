"""Test-stage reader for the pixelSplat-format `.torch` chunks (re10k / ACID / DTU), so the
evaluation CLI can run real frames through the HIP path.

Restates the reference's test-stage iteration, reference `src/dataset/dataset_re10k.py`:
  * chunk discovery: `<root>/test/*.torch`, sorted, every `test_chunk_interval`-th (`:63-79`);
  * per example, `test_times_per_scene` runs; scene key `<key>_<run:02d>` when > 1 (`:121-129`);
  * context / target frame indices from the evaluation index; scenes missing from it are
    skipped (`ViewSamplerEvaluation.sample`, `view_sampler/view_sampler_evaluation.py:44-59`);
  * skip when any frame's field of view exceeds `max_fov` degrees (`:143-145`);
  * JPEG decode -> float [3, h, w] in [0, 1] (`convert_images`, `:228-236`); skip shapes other
    than 3x360x640 when `skip_bad_shape` (`:156-166`);
  * optional baseline normalisation for 2 context views (`make_baseline_1`, `:168-183`);
  * poses: [fx, fy, cx, cy, _, _, w2c 3x4 row-major] -> (c2w, normalised K) (`convert_poses`,
    `:205-226`);
  * near / far from the config (`get_bound`, `:238-245`), divided by the baseline scale when
    `baseline_scale_bounds`;
  * crop shim: LANCZOS rescale through uint8 then centre crop, fx / fy rescaled
    (`shims/crop_shim.py:10-93`).

Chunks are loaded with `torch.load(weights_only=True)`: a chunk is a list of dicts of tensors and
strings, so nothing in the file is executed. Host-side data plumbing only (no GPU work here).
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass
from io import BytesIO
from pathlib import Path
from typing import Iterator

import numpy as np
import torch

from ..geometry.projection import get_fov


@dataclass
class ChunkDatasetCfg:
    """Test-time fields of `DatasetRE10kCfg` (reference dataset_re10k.py:25-41), defaults from
    config/experiment/re10k.yaml:37-43 (near 1, far 100, no baseline rescaling, 256x256)."""

    roots: tuple[str, ...]
    image_shape: tuple[int, int] = (256, 256)
    near: float = 1.0
    far: float = 100.0
    baseline_epsilon: float = 1e-3
    max_fov: float = 100.0
    make_baseline_1: bool = False
    baseline_scale_bounds: bool = False
    skip_bad_shape: bool = True
    test_chunk_interval: int = 1
    test_times_per_scene: int = 1
    test_len: int = -1


# Per-experiment overrides (reference config/experiment/{re10k,acid,dtu}.yaml `dataset:` blocks).
EXPERIMENTS = {
    "re10k": dict(near=1.0, far=100.0),
    "acid": dict(near=1.0, far=100.0),
    "dtu": dict(near=2.125, far=4.525, test_times_per_scene=4, skip_bad_shape=False),
}


def convert_poses(poses: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """[n, 18] camera rows -> (c2w [n, 4, 4], normalised K [n, 3, 3]) (reference :205-226)."""
    n = poses.shape[0]
    poses = poses.float()
    k = torch.eye(3, dtype=torch.float32).repeat(n, 1, 1)
    k[:, 0, 0], k[:, 1, 1], k[:, 0, 2], k[:, 1, 2] = poses[:, 0], poses[:, 1], poses[:, 2], poses[:, 3]
    w2c = torch.eye(4, dtype=torch.float32).repeat(n, 1, 1)
    w2c[:, :3] = poses[:, 6:].reshape(n, 3, 4)
    return w2c.inverse(), k


def decode_images(images: list[torch.Tensor]) -> torch.Tensor:
    """Encoded image byte tensors -> float [n, 3, h, w] in [0, 1] (PIL decode + ToTensor)."""
    from PIL import Image

    out = []
    for im in images:
        pil = Image.open(BytesIO(im.numpy().tobytes())).convert("RGB")
        arr = torch.from_numpy(np.asarray(pil, dtype=np.uint8).copy())
        out.append(arr.permute(2, 0, 1).float().div(255.0))
    return torch.stack(out)


def rescale(image: torch.Tensor, shape: tuple[int, int]) -> torch.Tensor:
    """uint8 truncation -> PIL LANCZOS resize -> /255 (reference crop_shim.py:10-22)."""
    from PIL import Image

    h, w = shape
    u8 = (image * 255).clip(min=0, max=255).to(torch.uint8).permute(1, 2, 0).contiguous().numpy()
    res = np.array(Image.fromarray(u8).resize((w, h), Image.LANCZOS)) / 255
    return torch.tensor(res, dtype=image.dtype).permute(2, 0, 1)


def center_crop(images: torch.Tensor, intrinsics: torch.Tensor, shape: tuple[int, int]):
    """Reference crop_shim.py:25-49 (odd margins give the same half-pixel offset)."""
    *_, h_in, w_in = images.shape
    h_out, w_out = shape
    row, col = (h_in - h_out) // 2, (w_in - w_out) // 2
    images = images[..., :, row:row + h_out, col:col + w_out]
    intrinsics = intrinsics.clone()
    intrinsics[..., 0, 0] *= w_in / w_out
    intrinsics[..., 1, 1] *= h_in / h_out
    return images, intrinsics


def rescale_and_crop(images: torch.Tensor, intrinsics: torch.Tensor, shape: tuple[int, int]):
    """Reference crop_shim.py:52-77."""
    *batch, c, h_in, w_in = images.shape
    h_out, w_out = shape
    if h_out > h_in or w_out > w_in:
        raise ValueError(f"crop shim: target {shape} larger than the image {(h_in, w_in)}")
    s = max(h_out / h_in, w_out / w_in)
    hs, ws = round(h_in * s), round(w_in * s)
    flat = images.reshape(-1, c, h_in, w_in)
    flat = torch.stack([rescale(im, (hs, ws)) for im in flat])
    return center_crop(flat.reshape(*batch, c, hs, ws), intrinsics, shape)


def apply_crop_shim(example: dict, shape: tuple[int, int]) -> dict:
    out = dict(example)
    for part in ("context", "target"):
        views = dict(example[part])
        views["image"], views["intrinsics"] = rescale_and_crop(views["image"], views["intrinsics"], shape)
        out[part] = views
    return out


class ChunkTestDataset:
    """Iterates test examples in the reference's order; each example is the reference's
    un-batched dict (`context`/`target` views with extrinsics, intrinsics, image, near, far,
    index; `scene`). `batch(example)` adds the leading batch axis of the DataLoader."""

    def __init__(self, cfg: ChunkDatasetCfg, index: dict[str, dict | None]):
        self.cfg = cfg
        self.index = index
        self.chunks: list[Path] = []
        for root in cfg.roots:
            d = Path(root) / "test"
            self.chunks.extend(sorted(p for p in d.iterdir() if p.suffix == ".torch"))
        self.chunks = self.chunks[:: cfg.test_chunk_interval]

    @classmethod
    def from_index_file(cls, cfg: ChunkDatasetCfg, index_path: str | Path) -> "ChunkTestDataset":
        return cls(cfg, json.loads(Path(index_path).read_text()))

    def _bound(self, value: float, n: int, scale: float) -> torch.Tensor:
        return torch.full((n,), value, dtype=torch.float32) / scale

    def __iter__(self) -> Iterator[dict]:
        cfg = self.cfg
        produced = 0
        for path in self.chunks:
            chunk = torch.load(path, map_location="cpu", weights_only=True)
            tps = cfg.test_times_per_scene
            for run in range(int(tps * len(chunk))):
                if 0 <= cfg.test_len <= produced:
                    return
                ex = chunk[run // tps]
                ext, intr = convert_poses(ex["cameras"])
                scene = f"{ex['key']}_{run % tps:02d}" if tps > 1 else ex["key"]
                entry = self.index.get(scene)
                if entry is None:
                    continue
                ci = torch.tensor(entry["context"], dtype=torch.int64)
                ti = torch.tensor(entry["target"], dtype=torch.int64)
                if (get_fov(intr).rad2deg() > cfg.max_fov).any():
                    continue
                cimg = decode_images([ex["images"][i] for i in ci.tolist()])
                timg = decode_images([ex["images"][i] for i in ti.tolist()])
                if cfg.skip_bad_shape and (cimg.shape[1:] != (3, 360, 640) or timg.shape[1:] != (3, 360, 640)):
                    continue
                scale = 1.0
                if ci.numel() == 2 and cfg.make_baseline_1:
                    a, b = ext[ci][:, :3, 3]
                    scale = float((a - b).norm())
                    if scale < cfg.baseline_epsilon:
                        continue
                    ext[:, :3, 3] /= scale
                nf = scale if cfg.baseline_scale_bounds else 1.0
                example = {
                    "context": {"extrinsics": ext[ci], "intrinsics": intr[ci], "image": cimg,
                                "near": self._bound(cfg.near, len(ci), nf), "far": self._bound(cfg.far, len(ci), nf),
                                "index": ci},
                    "target": {"extrinsics": ext[ti], "intrinsics": intr[ti], "image": timg,
                               "near": self._bound(cfg.near, len(ti), nf), "far": self._bound(cfg.far, len(ti), nf),
                               "index": ti},
                    "scene": scene,
                }
                produced += 1
                yield apply_crop_shim(example, tuple(cfg.image_shape))

    @staticmethod
    def batch(example: dict, device: torch.device | str = "cpu") -> dict:
        """Leading batch axis of 1 (the test DataLoader's collation), moved to `device`."""
        out = {"scene": [example["scene"]]}
        for part in ("context", "target"):
            out[part] = {k: v.unsqueeze(0).to(device) for k, v in example[part].items()}
        return out


def write_chunk(path: str | Path, examples: list[dict]) -> None:
    """Write a chunk in the reference's format (list of {key, url, timestamps, cameras [n, 18],
    images: list of uint8 JPEG byte tensors}); used by the tests to make fixture chunks."""
    torch.save(examples, path)


def encode_jpeg(image_u8: np.ndarray, quality: int = 95) -> torch.Tensor:
    from PIL import Image

    buf = BytesIO()
    Image.fromarray(image_u8).save(buf, format="JPEG", quality=quality)
    return torch.frombuffer(bytearray(buf.getvalue()), dtype=torch.uint8)


def fov_deg(intrinsics: torch.Tensor) -> torch.Tensor:
    return get_fov(intrinsics) * (180.0 / math.pi)
