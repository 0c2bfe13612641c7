"""Tune the e2e step's fp32 library GEMMs with PyTorch TunableOp on the GPU box and write
transplat_amd/tuned/gemms_gfx950.csv (read back, tuning off, by transplat_amd.gemm_tuning):
eager steps of C2 (b = 1) and b = 8, fp32. bf16 (C3) is NOT tuned: during its tuning pass a
candidate library solution faulted the GPU (illegal address); the fp32 passes ran clean.
Usage: python tools/tune_gemms.py [--ms 30]"""
import argparse
import os

import torch
import torch.cuda.tunable as tun

from transplat_amd import synthetic as S
from transplat_amd.e2e import build_model
from transplat_amd.gemm_tuning import TUNED_FILE

ap = argparse.ArgumentParser()
ap.add_argument("--ms", type=int, default=30, help="tuning time budget per GEMM shape (ms)")
args = ap.parse_args()
os.makedirs(TUNED_FILE.parent, exist_ok=True)
tun.enable(True)
tun.tuning_enable(True)
tun.set_max_tuning_duration(args.ms)
tun.set_filename(str(TUNED_FILE))
dev = torch.device("cuda:0")
for dense, batch in (("fp32", 1), ("fp32", 8)):
    model = build_model(dev, dense)
    data = S.make_batch(batch, image_shape=(256, 256), device=dev)
    for _ in range(2):
        model.test_step(data)
    torch.cuda.synchronize()
    print(f"tuned {dense} b={batch}: {len(tun.get_results())} GEMM shapes so far", flush=True)
    del model
# TunableOp writes the results to the set filename when the process exits
print("results go to", TUNED_FILE, "at exit", flush=True)
