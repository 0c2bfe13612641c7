"""Side-stream fork / join (transplat_amd/streams.py) and the synchronising debug mode."""
import pytest
import torch

from transplat_amd import streams


def test_tensors_walks_nested_containers():
    a, b, c = torch.zeros(1), torch.ones(2), torch.full((3,), 2.0)
    found = list(streams._tensors((a, [b, {"x": c, "y": 3}], None)))
    assert len(found) == 3 and found[0] is a and found[1] is b and found[2] is c


def test_fork_runs_inline_on_cpu():
    p = streams.fork(torch.device("cpu"), lambda x, d: x + d["y"], torch.ones(2), {"y": torch.ones(2)})
    assert torch.equal(streams.join(p), torch.full((2,), 2.0))


@pytest.mark.gpu
def test_nested_fork_in_capture_raises_and_capture_survives(device):
    """A fork from inside a forked branch during hipGraph capture raises NestedForkError before it
    touches a second side stream (HIP's capture_end crashes on that graph shape); the flat fork's
    capture then ends normally and the graph replays."""
    x = torch.arange(1024, dtype=torch.float32, device=device)
    torch.cuda.synchronize()
    raised = []

    def branch(t):
        try:
            streams.fork(t.device, lambda u: u * 3, t, slot=1)
        except streams.NestedForkError:
            raised.append(True)
        return t * 2

    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device)
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            p = streams.fork(device, branch, x)
            y = streams.join(p) + 1
    torch.cuda.synchronize()
    assert raised == [True]
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y, x * 2 + 1)


@pytest.mark.gpu
def test_raster_debug_mode_matches_and_refuses_capture(device):
    """rasterize(debug=True) (upstream `debug`: sync + check after every launch) renders the same
    image as the normal path, and refuses to run inside hipGraph capture."""
    from transplat_amd import synthetic as S
    from transplat_amd.model.decoder.hip_splatting import prepare_cameras, rasterize

    hw = (64, 64)
    g = {k: v.to(device) for k, v in S.make_gaussians(1, image_shape=hw).items()}
    t = S.make_batch(1, image_shape=hw)["target"]
    cams = prepare_cameras(t["extrinsics"][0], t["intrinsics"][0], t["near"][0], t["far"][0],
                           torch.zeros(3, 3)).to(device)
    args = (g["means"], g["covariances"], g["harmonics"], g["opacities"], cams, hw, 3)
    c0, r0 = rasterize(*args)
    c1, r1 = rasterize(*args, debug=True)
    assert torch.equal(c0, c1) and torch.equal(r0, r1)
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device)
    with torch.cuda.stream(s):
        with pytest.raises(RuntimeError, match="debug"):
            with torch.cuda.graph(graph):
                rasterize(*args, check=False, debug=True)
    torch.cuda.synchronize()
