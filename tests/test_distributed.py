"""Scene sharding + the single metric all_gather, world_size 2 over gloo on CPU (the N>1 path of
bench.py / evaluate.py; on GPUs the same code runs over RCCL)."""
import os
import socket
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from transplat_amd import evaluate as ev

INDEX = Path(__file__).resolve().parent / "golden" / "evaluation_index_re10k_small.json"


def test_load_index_small():
    scenes = ev.load_index(INDEX)
    assert [k for k, _ in scenes] == ["5aca87f95a9412c6", "322261824c4a3003"]
    assert all(len(v["context"]) == 2 and len(v["target"]) == 3 for _, v in scenes)


def test_shard_is_partition():
    items = list(range(11))
    parts = [ev.shard(items, r, 4) for r in range(4)]
    flat = sorted(i for p in parts for i, _ in p)
    assert flat == items and [len(p) for p in parts] == [3, 3, 3, 2]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_scenes, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from transplat_amd import synthetic as S

    def make_batch(idx, entry):
        return S.make_batch(1, image_shape=(16, 16), scene_offset=idx)

    def step(batch):  # stand-in renderer: the target images themselves, darkened by the scene idx
        return batch["target"]["image"] * 0.9

    res = ev.evaluate(step, list(range(n_scenes)), make_batch, torch.device("cpu"), rank, world)
    if rank == 0:
        out.put([(r.scene_idx, r.psnr, r.n_views) for r in res])
    dist.destroy_process_group()


def test_gather_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 5, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[0] for r in res] == [0, 1, 2, 3, 4]
    assert all(r[2] == 3 for r in res) and all(r[1] > 15 for r in res)


def test_index_batch_places_targets():
    scenes = ev.load_index(INDEX)
    key, entry = scenes[0]
    b = ev.index_batch(0, key, entry, image_shape=(32, 32))
    assert b["context"]["image"].shape == (1, 2, 3, 32, 32) and b["target"]["image"].shape == (1, 3, 3, 32, 32)
    c0, c1 = entry["context"]
    t = b["target"]["extrinsics"][0, :, 0, 3]  # x translation along the unit baseline
    expect = torch.tensor([(f - c0) / (c1 - c0) for f in entry["target"]], dtype=torch.float32)
    assert torch.allclose(t, expect, atol=1e-6)


@pytest.mark.gpu
def test_evaluate_cli_small_index(device):
    """C1 plumbing on the GPU: the reference's re10k_small evaluation index through the full
    model (synthetic frames and weights), one JSON summary -- by default on the benched step (one
    replayed hipGraph per scene, bf16x3 dense layers, one sync per shard); the eager step of the
    same precision gives the same PSNR."""
    import json
    import subprocess
    import sys

    repo = Path(__file__).resolve().parents[1]
    runs = {}
    for extra in ([], ["--no-graph"]):
        out = subprocess.run([sys.executable, "-m", "transplat_amd.evaluate", "--index", str(INDEX)] + extra,
                             cwd=repo, capture_output=True, text=True, timeout=600)
        assert out.returncode == 0, out.stderr[-2000:]
        summary = json.loads(out.stdout.strip().splitlines()[-1])
        assert summary["scenes"] == 2 and summary["views"] == 6
        assert summary["psnr"] == summary["psnr"]  # finite
        assert summary["dense_dtype"] == "bf16x3" and summary["graph"] == (not extra)
        assert "bf16x3" in summary["precision"]
        # graph capture (warmup + capture) is reported apart from the steady per-scene time
        assert summary["steady_scenes"] + summary["capture_scenes"] == 2
        assert (summary["capture_scenes"] >= 1) == (not extra)
        runs[bool(extra)] = summary
    print(f"evaluate: graphed {runs[False]['psnr']:.4f} dB in {runs[False]['seconds']:.4f} s, "
          f"eager {runs[True]['psnr']:.4f} dB")
    assert abs(runs[False]["psnr"] - runs[True]["psnr"]) < 1e-2


def _bench_worker(rank, world, port, out):
    """bench.py's N > 1 timing path (timed_steps) on gloo: rank r's step sleeps (r + 1) x 20 ms, so
    the max-over-ranks time must be rank 1's and both ranks must report it."""
    import sys
    import time

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    calls = []

    def step():
        calls.append(1)
        time.sleep(0.02 * (rank + 1))

    el = bench.timed_steps(step, 5, world, lambda: None, torch.device("cpu"))
    out.put((rank, len(calls), el))
    dist.destroy_process_group()


def test_bench_timed_steps_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [5, 5]  # exactly `steps` calls per rank
    assert res[0][2] == res[1][2]  # every rank reports the max
    assert 0.2 <= res[1][2] < 0.6  # rank 1: 5 x 40 ms


def _run_bench(*argv, env_extra=None, timeout=240):
    import subprocess
    import sys

    repo = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TSPLAT_DIST_BACKEND="gloo", **(env_extra or {}))
    return subprocess.run([sys.executable, str(repo / "bench.py"), *argv], cwd=repo, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_main_self_launches_world2_gloo():
    """`python bench.py --gpus 2` with no launcher environment starts torch.distributed.run with two
    ranks itself; bench.main() then runs end to end on each rank (CPU selftest step, gloo) and rank 0
    prints one JSON line with n_gpus = 2 and the max-over-ranks time (rank 1 sleeps 20 ms per step,
    rank 0 10 ms)."""
    import json

    out = _run_bench("--gpus", "2", "--workload", "selftest", "--steps", "10", "--warmup", "1")
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == 10
    assert 20.0 <= res["ms_per_step"] < 60.0  # the slower rank's 20 ms steps
    assert abs(res["value"] - 2 * 10 / (res["ms_per_step"] * 10 / 1e3)) < 1e-6 * res["value"]


def test_bench_gpus_must_match_world_size():
    out = _run_bench("--gpus", "2", "--workload", "selftest", "--steps", "1", "--warmup", "0",
                     env_extra={"WORLD_SIZE": "1"})
    assert out.returncode != 0 and "WORLD_SIZE=1" in (out.stderr + out.stdout)
