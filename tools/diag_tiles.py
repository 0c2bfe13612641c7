"""Per-tile instance counts of the e2e synthetic scene (how long are the tile lists?) and the
render time split, to steer rasterizer work."""
import torch

from transplat_amd import _lib, synthetic as S
from transplat_amd.e2e import build_model
from transplat_amd.model.decoder.hip_splatting import _STATE

dev = torch.device("cuda:0")
model = build_model(dev)
data = S.make_batch(1, image_shape=(256, 256), device=dev)
with torch.no_grad():
    model.test_step(data)
torch.cuda.synchronize()
ws, off = _STATE.last[(dev.type, dev.index)]
lib = _lib.load()
G, V, T = 131072, 3, 256
offs = ws[off - 4 * V * T: off + 4].view(torch.int32).cpu().long()
counts = offs[1:] - offs[:-1]
print("instances", int(offs[-1]), "tiles", counts.numel())
q = torch.quantile(counts.float(), torch.tensor([0.0, 0.5, 0.9, 0.99, 1.0]))
print("per-tile count quantiles (0, .5, .9, .99, 1):", [int(x) for x in q])
print("tiles > 4096:", int((counts > 4096).sum()), " > 2048:", int((counts > 2048).sum()))
for name in ("raster_preprocess", "raster_scan", "raster_scatter", "raster_render"):
    _lib.prof_enable(name)
    for _ in range(5):
        with torch.no_grad():
            model.test_step(data)
    ms, n = _lib.prof_read()
    _lib.prof_enable(None)
    print(f"{name}: {ms / n * 1e3:.1f} us")
