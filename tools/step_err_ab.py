"""bf16x3 C2 step vs the exact-fp32 step on the same weights and inputs (test_bf16x3_step_vs_exact_fp32's
measurement) under the current environment's kernel knobs, optionally with per-stage error prints.
usage: step_err_ab.py [tag]"""
import sys

import torch

from transplat_amd import synthetic as S
from transplat_amd.e2e import GraphedStep, build_model


def psnr(a, b):
    mse = ((a.clamp(0, 1) - b.clamp(0, 1)) ** 2).flatten(2).mean(-1)
    return (-10 * torch.log10(mse.clamp_min(1e-20))).min().item()


dev = torch.device("cuda:0")
if "--tuned" in sys.argv:  # the committed TunableOp GEMM solutions for both steps (what bench.py replays)
    from transplat_amd.gemm_tuning import use_tuned_gemms

    assert use_tuned_gemms(dev)
data = S.make_batch(1, image_shape=(256, 256), device=dev)


def run(model, graph=False):
    with torch.no_grad():
        g = model.encoder(model.data_shim(data)["context"], 0, deterministic=True)
        out = GraphedStep(model, data).run().color if graph else model.test_step(data).color
    torch.cuda.synchronize()
    return g.means.clone(), g.harmonics.clone(), out.float().clone(), g.opacities.clone()


fp = build_model(dev, "fp32")
ref = run(fp)
del fp
x3 = run(build_model(dev, "bf16x3"), graph=True)
rel = lambda a, b: ((a - b).abs().max() / b.abs().max()).item()
d = (x3[2] - ref[2]).abs()
print(f"{sys.argv[1] if len(sys.argv) > 1 else ''}: means {rel(x3[0], ref[0]):.2e} harm {rel(x3[1], ref[1]):.2e} "
      f"opac {rel(x3[3], ref[3]):.2e} px max {d.max().item():.2e} mean {d.mean().item():.2e} "
      f"frac>1e-3 {(d > 1e-3).float().mean().item():.2e} psnr {psnr(x3[2], ref[2]):.1f}", flush=True)
