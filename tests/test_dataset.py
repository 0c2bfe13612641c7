"""Test-stage chunk reader and shims (host plumbing for the real-data PSNR path).

Crop / patch shims are pinned by reference outputs (tests/golden/crop_shim.npz, made by
tests/golden/gen_golden.py from src/dataset/shims/{crop,patch}_shim.py). The chunk iteration
rules (reference src/dataset/dataset_re10k.py:90-226) are checked on fixture chunks written here
in the reference's on-disk format (no real re10k chunk is reachable offline).
"""
from __future__ import annotations

import math
from pathlib import Path

import numpy as np
import pytest
import torch

from transplat_amd.dataset import ChunkDatasetCfg, ChunkTestDataset, convert_poses
from transplat_amd.dataset.re10k_chunks import apply_crop_shim, encode_jpeg, write_chunk
from transplat_amd.dataset_shims import apply_patch_shim

GOLDEN = Path(__file__).parent / "golden"


def test_crop_shim_matches_reference():
    g = np.load(GOLDEN / "crop_shim.npz")
    ex = {"context": {"image": torch.from_numpy(g["image"]), "intrinsics": torch.from_numpy(g["intrinsics"])},
          "target": {"image": torch.from_numpy(g["image"][:1]), "intrinsics": torch.from_numpy(g["intrinsics"][:1])}}
    out = apply_crop_shim(ex, (64, 64))
    np.testing.assert_array_equal(out["context"]["image"].numpy(), g["out_image"])
    np.testing.assert_array_equal(out["context"]["intrinsics"].numpy(), g["out_intrinsics"])
    assert out["target"]["image"].shape == (1, 3, 64, 64)


def test_patch_shim_matches_reference():
    g = np.load(GOLDEN / "crop_shim.npz")
    views = {"image": torch.from_numpy(g["patch_image"]), "intrinsics": torch.from_numpy(g["patch_intrinsics"])}
    out = apply_patch_shim({"context": views, "target": views}, 14)
    np.testing.assert_array_equal(out["context"]["image"].numpy(), g["patch_out_image"])
    np.testing.assert_array_equal(out["context"]["intrinsics"].numpy(), g["patch_out_intrinsics"])


def _camera_rows(n: int, fx: float = 0.8, seed: int = 0) -> tuple[torch.Tensor, torch.Tensor]:
    """[n, 18] rows (fx, fy, cx, cy, 0, 0, w2c 3x4) and the matching c2w."""
    g = torch.Generator().manual_seed(seed)
    c2w = torch.eye(4).repeat(n, 1, 1)
    for i in range(n):
        a = 0.05 * i
        c2w[i, :3, :3] = torch.tensor([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
        c2w[i, :3, 3] = torch.randn(3, generator=g)
    w2c = c2w.inverse()
    rows = torch.zeros(n, 18)
    rows[:, 0], rows[:, 1], rows[:, 2], rows[:, 3] = fx, fx * 16 / 9, 0.5, 0.5
    rows[:, 6:] = w2c[:, :3].reshape(n, 12)
    return rows, c2w


def _example(key: str, n: int, hw=(360, 640), fx: float = 0.8, seed: int = 0) -> dict:
    rows, _ = _camera_rows(n, fx, seed)
    rng = np.random.default_rng(seed)
    imgs = [encode_jpeg(rng.integers(0, 256, (*hw, 3), dtype=np.uint8)) for _ in range(n)]
    return {"key": key, "url": "", "timestamps": torch.arange(n), "cameras": rows, "images": imgs}


def test_convert_poses_roundtrip():
    rows, c2w = _camera_rows(5)
    ext, k = convert_poses(rows)
    torch.testing.assert_close(ext, c2w, atol=1e-5, rtol=0)
    assert float(k[0, 0, 0]) == pytest.approx(0.8) and float(k[0, 2, 2]) == 1.0


def test_chunk_reader_order_and_skips(tmp_path):
    root = tmp_path / "re10k"
    (root / "test").mkdir(parents=True)
    write_chunk(root / "test" / "000000.torch",
                [_example("sceneA", 6, seed=1), _example("not_indexed", 6, seed=2),
                 _example("bad_shape", 6, hw=(120, 200), seed=3)])
    # fov_x = 2 atan(1 / (2 fx)) > 100 deg for fx = 0.3
    write_chunk(root / "test" / "000001.torch", [_example("wide_fov", 6, fx=0.3, seed=4),
                                                 _example("sceneB", 6, seed=5)])
    index = {"sceneA": {"context": [0, 4], "target": [1, 2, 3]}, "bad_shape": {"context": [0, 4], "target": [2]},
             "wide_fov": {"context": [0, 4], "target": [2]}, "sceneB": {"context": [1, 5], "target": [2, 3, 4]},
             "null_entry": None}
    ds = ChunkTestDataset(ChunkDatasetCfg(roots=(str(root),)), index)
    out = list(ds)
    assert [e["scene"] for e in out] == ["sceneA", "sceneB"]
    a = out[0]
    assert a["context"]["image"].shape == (2, 3, 256, 256) and a["target"]["image"].shape == (3, 3, 256, 256)
    assert a["context"]["index"].tolist() == [0, 4] and a["target"]["index"].tolist() == [1, 2, 3]
    _, c2w = _camera_rows(6, seed=1)
    torch.testing.assert_close(a["context"]["extrinsics"], c2w[[0, 4]], atol=1e-5, rtol=0)
    # 360x640 -> 256x455 -> 256x256: fx scaled by 455/256, fy unchanged
    assert float(a["context"]["intrinsics"][0, 0, 0]) == pytest.approx(0.8 * 455 / 256, rel=1e-6)
    assert float(a["context"]["intrinsics"][0, 1, 1]) == pytest.approx(0.8 * 16 / 9, rel=1e-6)
    assert a["context"]["near"].tolist() == [1.0, 1.0] and a["target"]["far"].tolist() == [100.0] * 3
    b = ChunkTestDataset.batch(a)
    assert b["context"]["image"].shape == (1, 2, 3, 256, 256) and b["scene"] == ["sceneA"]

    # skip_bad_shape off keeps the odd-sized scene; test_len caps the stream
    ds2 = ChunkTestDataset(ChunkDatasetCfg(roots=(str(root),), skip_bad_shape=False, image_shape=(96, 96)), index)
    assert [e["scene"] for e in ds2] == ["sceneA", "bad_shape", "sceneB"]
    ds3 = ChunkTestDataset(ChunkDatasetCfg(roots=(str(root),), test_len=1), index)
    assert len(list(ds3)) == 1


def test_chunk_reader_times_per_scene_and_baseline(tmp_path):
    root = tmp_path / "dtu"
    (root / "test").mkdir(parents=True)
    write_chunk(root / "test" / "000000.torch", [_example("scan1", 5, seed=7)])
    index = {"scan1_00": {"context": [0, 3], "target": [1]}, "scan1_01": {"context": [1, 4], "target": [2]}}
    cfg = ChunkDatasetCfg(roots=(str(root),), test_times_per_scene=2, make_baseline_1=True,
                          baseline_scale_bounds=True, near=2.125, far=4.525)
    out = list(ChunkTestDataset(cfg, index))
    assert [e["scene"] for e in out] == ["scan1_00", "scan1_01"]
    for e in out:
        t = e["context"]["extrinsics"][:, :3, 3]
        assert float((t[0] - t[1]).norm()) == pytest.approx(1.0, rel=1e-5)
        assert float(e["context"]["near"][0]) != pytest.approx(2.125)  # divided by the baseline


def test_evaluate_stream_shards(tmp_path):
    from transplat_amd.evaluate import evaluate_stream

    def batches():
        for i in range(5):
            img = torch.full((1, 3, 3, 8, 8), 0.5)
            yield {"context": {"image": img}, "target": {"image": img}, "scene": [f"s{i}"]}

    step = lambda b: b["target"]["image"] + 0.1
    res = evaluate_stream(step, batches(), torch.device("cpu"))
    assert [r.scene_idx for r in res] == [0, 1, 2, 3, 4]
    assert res[0].psnr == pytest.approx(20.0, abs=1e-3)
