"""GPU diagnostic: which part of the step misbehaves under graph replay with new inputs."""
import torch

from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model
from transplat_amd.model.decoder.hip_splatting import _STATE, num_rendered, prepare_cameras, rasterize

dev = torch.device("cuda:0")
st = lambda: int(_STATE.status[(dev.type, dev.index)].item())


def capture(fn, *static):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            fn(*static)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn(*static)
    return g, out


# A: rasterizer alone
hw = (256, 256)
batch = S.make_batch(1, image_shape=hw, device=dev)
t = batch["target"]
cams = prepare_cameras(t["extrinsics"][0], t["intrinsics"][0], t["near"][0], t["far"][0],
                       torch.zeros(3, 3, device=dev))
ga = {k: v.to(dev) for k, v in S.make_gaussians(1, image_shape=hw).items()}
gb = {k: v.to(dev) for k, v in S.make_gaussians(1, image_shape=hw, scene_offset=5).items()}
static = {k: v.clone() for k, v in ga.items()}
fn = lambda s: rasterize(s["means"], s["covariances"], s["harmonics"], s["opacities"], cams, hw, 3, check=False)[0]
ea = fn(ga).clone(); eb = fn(gb).clone(); torch.cuda.synchronize()
print("A eager a/b rendered", num_rendered(dev), "status", st(), flush=True)
g, out = capture(fn, static)
g.replay(); torch.cuda.synchronize()
print("A graph a: diff", (out - ea).abs().max().item(), "status", st(), "rendered", num_rendered(dev), flush=True)
for k in static:
    static[k].copy_(gb[k])
g.replay(); torch.cuda.synchronize()
print("A graph b: diff", (out - eb).abs().max().item(), "status", st(), "rendered", num_rendered(dev), flush=True)
for k in static:
    static[k].copy_(ga[k])
g.replay(); torch.cuda.synchronize()
print("A graph a again: diff", (out - ea).abs().max().item(), "status", st(), flush=True)
del g, out

# B: encoder alone
model = build_model(dev)
d1 = S.make_batch(1, image_shape=hw, device=dev)["context"]
d2 = S.make_batch(1, image_shape=hw, scene_offset=7, device=dev)["context"]
enc = lambda c: model.encoder(c, 0, deterministic=True)
with torch.no_grad():
    r1 = enc(d1); r1 = [x.clone() for x in (r1.means, r1.covariances, r1.harmonics, r1.opacities)]
    r2 = enc(d2); r2 = [x.clone() for x in (r2.means, r2.covariances, r2.harmonics, r2.opacities)]
    sc = {k: v.clone() for k, v in d1.items()}
    g, out = capture(enc, sc)
    outs = lambda: [out.means, out.covariances, out.harmonics, out.opacities]
    rel = lambda a, b: [f"{((x - y).abs().max() / y.abs().max()).item():.2e}" for x, y in zip(a, b)]
    g.replay(); torch.cuda.synchronize(); print("B graph d1 vs eager:", rel(outs(), r1), flush=True)
    for k in sc:
        sc[k].copy_(d2[k])
    g.replay(); torch.cuda.synchronize(); print("B graph d2 vs eager:", rel(outs(), r2), flush=True)
    for k in sc:
        sc[k].copy_(d1[k])
    g.replay(); torch.cuda.synchronize(); print("B graph d1 again:", rel(outs(), r1), flush=True)
