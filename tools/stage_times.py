"""Per-stage GPU time of one eager e2e step under the reference's stage tags (Benchmarker with
sync=True: HIP events around each stage, branches serialised so each stage's time is its own).
usage: stage_times.py [batch] [fp32|bf16] [steps]"""
import json
import sys

import torch

from transplat_amd import streams
from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model
from transplat_amd.misc.benchmarker import Benchmarker

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 1
dense = sys.argv[2] if len(sys.argv) > 2 else "fp32"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
torch.backends.cudnn.benchmark = True
dev = torch.device("cuda:0")
model = build_model(dev, dense)
data = S.make_batch(batch, image_shape=(256, 256), device=dev)
for _ in range(3):
    model.test_step(data)
torch.cuda.synchronize()
bm = Benchmarker(sync=True)
with streams.serial():
    for _ in range(steps):
        model.test_step(data, benchmarker=bm)
torch.cuda.synchronize()
summ = bm.summary()
order = ["encoder_1_prep_intrinsics", "encoder_2_backbone", "encoder_3_depth_anything", "encoder_4_depth_predictor",
         "encoder_4a_prep_features", "encoder_4b_cost_volume_matching", "encoder_4c_cost_volume_unet",
         "encoder_4d_coarse_depth", "encoder_4e_depth_refine_unet", "encoder_4f_gaussian_head",
         "encoder_5_gaussian_adapter", "decoder"]
for k in order:
    if k in summ:
        print(f"{k:36s} gpu {summ[k]['gpu_ms']:8.3f} ms   wall {summ[k]['wall_ms']:8.3f} ms")
print(json.dumps({k: round(v["gpu_ms"], 4) for k, v in summ.items()}))
