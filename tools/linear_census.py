"""Every fused_linear / attention_merge call of one eager C2 step with its shape and GPU time (events
around the call, synchronised), aggregated by shape. Usage: python tools/linear_census.py [dense_dtype] [batch]"""
import collections
import sys

import torch

from transplat_amd import kernels
from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model

dev = torch.device("cuda:0")
dense = sys.argv[1] if len(sys.argv) > 1 else "fp32"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1
model = build_model(dev, dense)
data = S.make_batch(batch, image_shape=(256, 256), device=dev)
for _ in range(2):
    model.test_step(data)
torch.cuda.synchronize()

rec = collections.defaultdict(list)


def timed(name, fn, key_of):
    def wrap(*args, **kw):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = fn(*args, **kw)
        b.record()
        torch.cuda.synchronize()
        rec[(name,) + key_of(*args, **kw)].append(a.elapsed_time(b) * 1000)
        return out
    return wrap


def lin_key(x1, weight, x2=None, **kw):
    flags = ",".join(k for k, v in kw.items() if v is not None and v is not False)
    return (x1.reshape(-1, x1.shape[-1]).shape[0], x1.shape[-1], 0 if x2 is None else x2.shape[-1], weight.shape[0],
            flags)


def merge_key(q, k, v, h, w, num_splits, with_shift, merge_weight, ln, residual=None, kv_shift=0, **kw):
    return (q.shape[0] * q.shape[1], q.shape[2], 0, merge_weight.shape[0], f"splits={num_splits} shift={with_shift}")


kernels.fused_linear = timed("linear", kernels.fused_linear, lin_key)
kernels.attention_merge = timed("attn_merge", kernels.attention_merge, merge_key)
model.test_step(data)
torch.cuda.synchronize()
tot = 0.0
print(f"{'op':10s} {'M':>6s} {'k1':>5s} {'k2':>5s} {'N':>5s} {'calls':>5s} {'avg_us':>7s} {'GB/s':>7s} {'TF/s':>6s}  flags")
for key, ts in sorted(rec.items(), key=lambda kv: -sum(kv[1])):
    name, m, k1, k2, n, flags = key
    avg = sum(ts) / len(ts)
    tot += sum(ts)
    byt = 4.0 * (m * (k1 + k2) + m * n + n * (k1 + k2))
    print(f"{name:10s} {m:6d} {k1:5d} {k2:5d} {n:5d} {len(ts):5d} {avg:7.1f} {byt / avg / 1e3:7.0f} {2.0 * m * (k1 + k2) * n / avg / 1e6:6.1f}  {flags}")
print(f"total {tot:.1f} us (eager, event-bracketed; {dense}, b = {batch})")
