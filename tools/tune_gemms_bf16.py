"""Tune the C3 step's bf16 library GEMMs over an ALLOW-LIST: hipBLASLt's own heuristic top-k for each
exact problem (tools/gemm_probe.cpp), never TunableOp's exhaustive search (one of whose candidates
faulted the GPU in round 2). Each candidate's solution index is printed and flushed before it runs.

  1. record: an eager C3 step (batch 8, bf16 dense layers) with TunableOp in record-untuned mode
     lists every GEMM TunableOp sees (op signature, params signature, BLAS signature with strides);
  2. probe: for each BFloat16 GEMM, time the heuristic's top-k solutions (workspace <= 1 MiB, so the
     replay never needs more than torch's hipBLASLt workspace);
  3. write: transplat_amd/tuned/gemms_gfx950.csv keeps its fp32 entries and gains one line per bf16
     GEMM whose best candidate beats the heuristic's first choice by > 3 % (else nothing: torch's
     default path IS that first choice).
Usage (GPU box): python tools/tune_gemms_bf16.py [--topk 8] [--dry]"""
import argparse
import ctypes
import glob
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
if "--record-to" in sys.argv:  # child: TunableOp writes the untuned file when this process exits
    os.environ["PYTORCH_TUNABLEOP_UNTUNED_FILENAME"] = sys.argv[sys.argv.index("--record-to") + 1]

import torch  # noqa: E402
import torch.cuda.tunable as tun  # noqa: E402

from transplat_amd import synthetic as S  # noqa: E402
from transplat_amd.gemm_tuning import TUNED_FILE  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--topk", type=int, default=8)
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--gain", type=float, default=0.03, help="minimum speed-up over the heuristic's first choice")
ap.add_argument("--dry", action="store_true", help="probe and report, do not rewrite the CSV")
ap.add_argument("--record-to", default=None, help=argparse.SUPPRESS)
args = ap.parse_args()

MAX_WS = 1 << 20


def record():
    from transplat_amd.e2e import build_model

    dev = torch.device("cuda:0")
    tun.enable(True)
    tun.tuning_enable(False)
    tun.set_filename(str(Path(tempfile.gettempdir()) / f"tsplat_tunableop_rec_{os.getpid()}.csv"))
    tun.record_untuned_enable(True)
    model = build_model(dev, "bf16")
    data = S.make_batch(8, image_shape=(256, 256), device=dev)
    with torch.no_grad():
        model.test_step(data)
    torch.cuda.synchronize()


def recorded_lines():
    """Run the recording step in a child process (the untuned file is complete when it exits)."""
    out = Path(tempfile.gettempdir()) / f"tsplat_untuned_{os.getpid()}.csv"
    subprocess.run([sys.executable, __file__, "--record-to", str(out)], check=True)
    stem = out.with_suffix("")
    files = glob.glob(str(stem) + "*")
    lines = [l.strip() for f in files for l in open(f) if l.startswith("Gemm")]
    return sorted(set(lines))


def parse(line):
    """-> dict of the hipBLASLt problem, or None for a non-bf16 / unsupported op."""
    parts = line.split(",", 2)
    op_sig, params = parts[0], parts[1]
    blas = parts[2] if len(parts) > 2 else ""
    m = re.match(r"(Gemm|GemmAndBias|GemmStridedBatched)TunableOp_BFloat16_([NT])([NT])$", op_sig)
    if not m:
        return None
    kind = m.group(1)
    p = params.split("_")
    ta, tb = p[0][0], p[0][1]
    mm, nn, kk = int(p[1]), int(p[2]), int(p[3])
    if kind == "GemmStridedBatched":
        batch = int(p[5])
        lda, ldb, ldc = int(p[7]), int(p[8]), int(p[9])
        st = {key: int(v) for key, v in re.findall(r"(stride_[abc]): (\d+)", blas)}
        if len(st) != 3:
            return None
        sa, sb, sc = st["stride_a"], st["stride_b"], st["stride_c"]
    else:
        batch, sa, sb, sc = 1, 0, 0, 0
        lda, ldb, ldc = int(p[5]), int(p[6]), int(p[7])
    return dict(op_sig=op_sig, params=params, ta=ta, tb=tb, m=mm, n=nn, k=kk, lda=lda, ldb=ldb, ldc=ldc,
                batch=batch, sa=sa, sb=sb, sc=sc, bias=int(kind == "GemmAndBias"))


def main():
    lines = recorded_lines()
    print(f"recorded {len(lines)} GEMM signatures", flush=True)
    so = ROOT / "tools" / "_bin" / "libgemm_probe.so"  # hipcc ... -o tools/_bin/libgemm_probe.so (see gemm_probe.cpp)
    lib = ctypes.CDLL(str(so))
    lib.gemm_probe.restype = ctypes.c_int
    lib.gemm_probe.argtypes = [ctypes.c_char, ctypes.c_char] + [ctypes.c_int64] * 6 + [ctypes.c_int32] + \
        [ctypes.c_int64] * 3 + [ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_int32,
                                ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_float)]
    picks = []
    for line in lines:
        g = parse(line)
        if g is None:
            continue
        idx = (ctypes.c_int32 * args.topk)()
        ms = (ctypes.c_float * args.topk)()
        print(f"probe {g['op_sig']},{g['params']} batch {g['batch']}", flush=True)
        got = lib.gemm_probe(g["ta"].encode(), g["tb"].encode(), g["m"], g["n"], g["k"], g["lda"], g["ldb"], g["ldc"],
                             g["batch"], g["sa"], g["sb"], g["sc"], g["bias"], args.topk, MAX_WS, args.iters, idx, ms)
        if got <= 0:
            print("  no candidates", flush=True)
            continue
        best = min(range(got), key=lambda i: ms[i])
        gain = ms[0] / ms[best] - 1.0
        print(f"  first {idx[0]} {ms[0] * 1e3:.1f} us, best {idx[best]} {ms[best] * 1e3:.1f} us (+{100 * gain:.1f} %)",
              flush=True)
        if best != 0 and gain > args.gain:
            picks.append(f"{g['op_sig']},{g['params']},Gemm_Hipblaslt_{idx[best]},{ms[best]:.6f}")
    print(f"{len(picks)} bf16 GEMMs take a non-default solution", flush=True)
    if args.dry or not picks:
        return
    keep = [l.rstrip("\n") for l in open(TUNED_FILE) if "_BFloat16_" not in l]
    TUNED_FILE.write_text("\n".join(keep + picks) + "\n")
    print("wrote", TUNED_FILE, flush=True)


if args.record_to:
    record()
else:
    main()
