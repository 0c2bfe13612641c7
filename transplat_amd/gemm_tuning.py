"""Library GEMM solution choices for the step's hipBLASLt / rocBLAS calls (DINOv2's M = 650 linears,
the transformer's fc1, the correlation-table bmm): PyTorch TunableOp results tuned once on an
MI355X (`tools/tune_gemms.py`) and committed as `tuned/gemms_gfx950.csv`; at run time they are only
READ (tuning off), so every GEMM takes its recorded solution with no search and the hipGraph
capture sees fixed kernels. The file's validator lines (PyTorch / ROCm / hipBLASLt versions, gfx
arch) make TunableOp ignore it on a different stack; TSPLAT_TUNED_GEMMS=0 turns it off (A/B)."""
from __future__ import annotations

import os
import tempfile
from pathlib import Path

import torch

TUNED_FILE = Path(__file__).resolve().parent / "tuned" / "gemms_gfx950.csv"


def use_tuned_gemms(device, dense_dtype: str = "fp32") -> bool:
    """Enable TunableOp in replay-only mode with the committed results; True if they were loaded.
    The file holds fp32 entries (tools/tune_gemms.py) and bf16 ones (tools/tune_gemms_bf16.py: an
    allow-list of hipBLASLt's heuristic top-k per problem); a GEMM with no entry takes TunableOp's
    Default op, i.e. the untuned library path."""
    if os.environ.get("TSPLAT_TUNED_GEMMS", "1") == "0" or torch.device(device).type != "cuda":
        return False
    if not TUNED_FILE.exists():
        return False
    import torch.cuda.tunable as tun

    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(False)
    # anything TunableOp writes back goes to a scratch file, never over the committed results
    # (one file per process: the ranks of a multi-GPU bench all exit at once)
    tun.set_filename(str(Path(tempfile.gettempdir()) / f"tsplat_tunableop_out_{os.getpid()}.csv"))
    return bool(tun.read_file(str(TUNED_FILE)))
