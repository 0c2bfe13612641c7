"""Is the graphed bf16x3 step the eager step? Eager color twice, then graph replays, each against the
first eager output (max / mean |d|, fraction > 1e-3). With tuned GEMMs as bench.py runs.
usage: graph_vs_eager.py [dense]"""
import sys

import torch

from transplat_amd import synthetic as S
from transplat_amd.e2e import GraphedStep, build_model
from transplat_amd.gemm_tuning import use_tuned_gemms

dense = sys.argv[1] if len(sys.argv) > 1 else "bf16x3"
nrep = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dev = torch.device("cuda:0")
use_tuned_gemms(dev, dense)
data = S.make_batch(1, image_shape=(256, 256), device=dev)
model = build_model(dev, dense)
with torch.no_grad():
    e = [model.test_step(data).color.float().clone() for _ in range(2)]
    g = GraphedStep(model, data)
    r = []
    for _ in range(nrep):
        r.append(g.run().color.float().clone())
        torch.cuda.synchronize()
    e.append(model.test_step(data).color.float().clone())
torch.cuda.synchronize()


def d(a, b):
    x = (a - b).abs()
    return f"max {x.max().item():.2e} mean {x.mean().item():.2e} frac>1e-3 {(x > 1e-3).float().mean().item():.2e}"


print(f"eager2 vs eager1: {d(e[1], e[0])}; eager3 (after capture) vs eager1: {d(e[2], e[0])}")
bad = [i for i, x in enumerate(r) if not torch.equal(x, e[0])]
print(f"replays differing from eager: {len(bad)} of {len(r)}: {bad}")
for i in bad[:3]:
    print(f"  replay{i} vs eager1: {d(r[i], e[0])}")
