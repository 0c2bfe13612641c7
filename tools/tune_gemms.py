"""Tune the e2e step's fp32 library GEMMs with PyTorch TunableOp on the GPU box and write
transplat_amd/tuned/gemms_gfx950.csv (read back, tuning off, by transplat_amd.gemm_tuning):
eager steps of C2 (b = 1) and b = 8, fp32, with TunableOp's numerical check on (round 3). bf16
(C3) is tuned by tools/tune_gemms_bf16.py over an allow-list instead: during a round-2 TunableOp
bf16 pass a candidate library solution faulted the GPU (illegal address).
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
if TUNED_FILE.exists():  # tune from scratch (TunableOp would reuse the file's entries), keep a copy
    TUNED_FILE.replace(TUNED_FILE.with_suffix(".prev.csv"))
tun.enable(True)
tun.tuning_enable(True)
# every candidate's result is compared with the default solution's before it may win (a solution
# that computes garbage is rejected, not recorded); fp32 sums over K <= 3072 differ by ~1e-6
# relative between correct solutions
tun.set_numerical_check_tolerances(True, 1e-3, 1e-3)
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
