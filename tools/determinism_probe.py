"""Find where two identical encoder runs diverge: forward hooks record a checksum (float64 sum, sum of
squares, and a strided sample) of every module output in call order, twice; the first modules whose
outputs differ are printed with the size of the difference (a module whose children all match but
whose own output differs did the nondeterministic work itself).
usage: determinism_probe.py [fp32|bf16x3] [cudnn-deterministic 0|1]  (0: bench.py's default MIOpen settings,
cudnn.benchmark on and deterministic off)"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tests"))
import test_reference_golden as T  # noqa: E402
from transplat_amd import synthetic as S  # noqa: E402
from transplat_amd.model.encoder import EncoderTrans, EncoderTransCfg  # noqa: E402

dense = sys.argv[1] if len(sys.argv) > 1 else "fp32"
if len(sys.argv) > 2 and sys.argv[2] == "1":
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
else:
    torch.backends.cudnn.benchmark = True
dev = torch.device("cuda:0")
enc = T.canonical_init(EncoderTrans(EncoderTransCfg(dense_dtype=dense)), seed=61).eval().to(dev)
ctx = {k: t.to(dev) for k, t in S.make_batch(1, image_shape=(256, 256))["context"].items()}
log = []


def first_tensor(o):
    if torch.is_tensor(o):
        return o
    if isinstance(o, (tuple, list)):
        for x in o:
            t = first_tensor(x)
            if t is not None:
                return t
    if isinstance(o, dict):
        for x in o.values():
            t = first_tensor(x)
            if t is not None:
                return t
    return None


def hook(name):
    def f(mod, inp, out):
        t = first_tensor(out)
        if t is None or not t.is_floating_point():
            return
        d = t.detach().double().flatten()
        samp = d[:: max(1, d.numel() // 4096)][:4096].cpu()
        log.append((name, d.sum().item(), (d * d).sum().item(), samp))
    return f


for name, m in enc.named_modules():
    m.register_forward_hook(hook(name or "<encoder>"))
runs = []
for r in range(2):
    log.clear()
    with torch.no_grad():
        gs = enc(ctx, global_step=0, deterministic=True)
    torch.cuda.synchronize()
    runs.append(list(log))
a, b = runs
print(f"{dense}: {len(a)} / {len(b)} module outputs recorded")
shown = 0
for (na, sa, qa, pa), (nb, sb, qb, pb) in zip(a, b):
    if na != nb:
        print("call order differs at", na, nb)
        break
    diff = (pa - pb).abs().max().item()
    if sa != sb or qa != qb or diff > 0:
        print(f"  differs: {na:70s} sum {sa:.9e} vs {sb:.9e}, sample max |d| {diff:.3e}")
        shown += 1
        if shown >= 12:
            break
if shown == 0:
    print("  all module outputs identical")
