"""GPU diagnostic: eager repeatability vs graph replay, at the Gaussian and image level."""
import torch

from transplat_amd import synthetic as S
from transplat_amd.e2e import GraphedStep, build_model

dev = torch.device("cuda:0")
model = build_model(dev)
data = S.make_batch(1, image_shape=(256, 256), device=dev)


def enc(d):
    with torch.no_grad():
        g = model.encoder(model.data_shim(d)["context"], 0, deterministic=True)
    return [t.clone() for t in (g.means, g.covariances, g.harmonics, g.opacities)]


def d(a, b):
    return [f"{(x - y).abs().max().item():.3e}/{x.abs().max().item():.2e}" for x, y in zip(a, b)]


e1, e2 = enc(data), enc(data)
print("encoder eager vs eager:", d(e1, e2))
c1 = model.test_step(data).color.clone()
c2 = model.test_step(data).color.clone()
print("color eager vs eager:", (c1 - c2).abs().max().item())
g = GraphedStep(model, data)
o1 = g.run().color.clone()
o2 = g.run().color.clone()
torch.cuda.synchronize()
print("color graph vs graph:", (o1 - o2).abs().max().item(), " graph vs eager:", (o1 - c1).abs().max().item())
ge = GraphedStep.__new__(GraphedStep)
# encoder-only graph
static = {k: v for k, v in data.items()}
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    enc(static)
torch.cuda.current_stream().wait_stream(side)
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    with torch.no_grad():
        gg = model.encoder(model.data_shim(static)["context"], 0, deterministic=True)
gr.replay()
torch.cuda.synchronize()
print("encoder graph vs eager:", d([gg.means, gg.covariances, gg.harmonics, gg.opacities], e1))
from transplat_amd.model.decoder.hip_splatting import num_rendered  # noqa: E402

model.test_step(data)
print("raster instances (one scene x 3 views):", num_rendered(dev))
