"""Stage boundaries of the REPLAYED C2 step (one hipGraph, concurrent branches as the bench runs them):
TSPLAT_MARKS=1 makes every stage range (the reference's encoder_* / decoder tags plus the diagnostic
backbone_* / da_* sub-stages) launch tsplat_timestamp on its stream; this captures the step with the
marks in it, replays it, and prints each stage's begin / end in microseconds from the step's first
mark, with its stream -- i.e. which branch is the critical path.
usage: graph_stages.py [--dense-dtype bf16x3] [--replays 20]"""
import argparse
import os
import sys
from pathlib import Path

os.environ["TSPLAT_MARKS"] = "1"
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from transplat_amd import synthetic as S  # noqa: E402
from transplat_amd.e2e import build_model  # noqa: E402
from transplat_amd.gemm_tuning import use_tuned_gemms  # noqa: E402
from transplat_amd.misc.benchmarker import MARKS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dense-dtype", default="bf16x3")
ap.add_argument("--replays", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True
use_tuned_gemms(dev, a.dense_dtype)
model = build_model(dev, a.dense_dtype)
data = S.make_batch(1, image_shape=(256, 256), device=dev)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(3):
        model.test_step(data)
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
MARKS.reset()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    model.test_step(data)
for _ in range(a.replays):
    g.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.replays):
    g.replay()
e1.record()
torch.cuda.synchronize()
print(f"replayed step: {e0.elapsed_time(e1) / a.replays * 1e3:.1f} us (with {len(MARKS.slots)} mark launches)")
rows = MARKS.read()
streams = {}
open_ = {}
spans = []
for tag, kind, sid, t in rows:
    streams.setdefault(sid, len(streams))
    if kind == "begin":
        open_[(tag, sid)] = t
    else:
        spans.append((open_.pop((tag, sid), float("nan")), t, tag, streams[sid]))
for t0, t1, tag, s in sorted(spans):
    print(f"{t0 * 1e6:9.1f} -> {t1 * 1e6:9.1f} us  ({(t1 - t0) * 1e6:8.1f})  stream {s}  {tag}")
