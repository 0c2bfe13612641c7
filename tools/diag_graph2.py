"""GPU diagnostic: graph replay with a second scene copied into the static inputs."""
import torch

from transplat_amd import synthetic as S
from transplat_amd.e2e import GraphedStep, build_model
from transplat_amd.model.decoder.hip_splatting import _STATE, num_rendered

dev = torch.device("cuda:0")
model = build_model(dev)
data = S.make_batch(1, image_shape=(256, 256), device=dev)
data2 = S.make_batch(1, image_shape=(256, 256), scene_offset=7, device=dev)
st = lambda: int(_STATE.status[(dev.type, dev.index)].item())


def report(tag, color):
    torch.cuda.synchronize()
    print(f"{tag}: status={st()} rendered={num_rendered(dev)} mean={color.mean().item():.5f} "
          f"zero_frac={(color == 0).float().mean().item():.4f}", flush=True)


e1 = model.test_step(data).color.clone(); report("eager data ", e1)
e2 = model.test_step(data2).color.clone(); report("eager data2", e2)
g = GraphedStep(model, data)
o1 = g.run().color.clone(); report("graph data ", o1)
o2 = g.run(data2).color.clone(); report("graph data2", o2)
o1b = g.run(data).color.clone(); report("graph data again", o1b)
print("diffs: g1-e1", (o1 - e1).abs().mean().item(), "g2-e2", (o2 - e2).abs().mean().item(),
      "g1b-e1", (o1b - e1).abs().mean().item())
# static buffer contents after copy
print("static ctx image == data2?", torch.equal(g.static["context"]["image"], data["context"]["image"]))
