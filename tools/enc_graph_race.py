"""Encoder-only hipGraph (the C2 step's encoder, branches on side streams) replayed N times against
its eager output: which Gaussian fields differ (a cross-stream race shows up here if it is in the
encoder). usage: enc_graph_race.py [replays]"""
import sys

import torch

from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model
from transplat_amd.gemm_tuning import use_tuned_gemms

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda:0")
use_tuned_gemms(dev, "bf16x3")
data = S.make_batch(1, image_shape=(256, 256), device=dev)
model = build_model(dev, "bf16x3")
ctx = model.data_shim(data)["context"]


def enc():
    g = model.encoder(ctx, 0, deterministic=True)
    return (g.means, g.covariances, g.harmonics, g.opacities)


with torch.no_grad():
    ref = [t.clone() for t in enc()]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            enc()
    torch.cuda.current_stream().wait_stream(side)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        out = enc()
    bad = []
    for i in range(n):
        gr.replay()
        torch.cuda.synchronize()
        d = [(o - r).abs().max().item() for o, r in zip(out, ref)]
        if max(d) > 0:
            bad.append((i, [f"{x:.1e}" for x in d]))
print(f"encoder replays differing: {len(bad)} of {n}: {bad[:4]}  (means, covariances, harmonics, opacities)")
