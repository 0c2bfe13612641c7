"""Run-to-run spread of the whole-encoder error against the reference golden (tests/golden/
encoder_256.npz) in one process: the same encoder and inputs N times per dense precision, each
output's relative error printed per run (nondeterministic reductions show up as a spread).
usage: encoder_repeat.py [N] [--deterministic]  (--deterministic: MIOpen's deterministic solvers)"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))
import test_reference_golden as T  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 4
if "--deterministic" in sys.argv:
    torch.backends.cudnn.deterministic = True
dev = torch.device("cuda:0")
for dense in ("fp32", "bf16x3"):
    from transplat_amd import synthetic as S
    from transplat_amd.model.encoder import EncoderTrans, EncoderTransCfg

    enc = T.canonical_init(EncoderTrans(EncoderTransCfg(dense_dtype=dense)), seed=61).eval().to(dev)
    ctx = {k: t.to(dev) for k, t in S.make_batch(1, image_shape=(256, 256))["context"].items()}
    first = None
    for i in range(n):
        with torch.no_grad():
            gs = enc(ctx, global_step=0, deterministic=True)
        m = gs.means[0].detach().clone()
        same = "" if first is None else f" | max |means - run 0| {(m - first).abs().max().item():.2e}"
        first = m if first is None else first
        try:
            T._check_encoder(gs, 1.0, f" ({dense} run {i}{same})")
        except AssertionError:
            pass
