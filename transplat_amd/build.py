"""Build the gfx950 HIP C-ABI library in-tree (no JIT cache: the .so travels with the repo).

`python -m transplat_amd.build` compiles every `csrc/*.hip` with hipcc for gfx950 into
`transplat_amd/libtransplat_hip.so`. Objects are cached under `build/hip/` and rebuilt when a
source or header is newer OR when the compile command (hipcc path, flags, per-file flags) differs
from the one recorded next to the object (`<stem>.cmd`).
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
INCLUDE = PKG.parent / "include"
BUILD = PKG.parent / "build" / "hip"
LIB = PKG / "libtransplat_hip.so"
ARCH = os.environ.get("TSPLAT_ARCH", "gfx950")

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-munsafe-fp-atomics",
    f"-I{INCLUDE}",
]


# raster.hip: the blend loop is scalar fp32 by design (v_pk_fma_f32 runs at v_fma_f32's FLOP rate,
# and the SLP vectoriser's packed form needs operand-pairing register moves: 84 -> 74 cycles per
# (entry, pixel) without it)
FILE_FLAGS = {"raster.hip": ["-fno-slp-vectorize"],
              "upsample.hip": ["-ffp-contract=off"]}  # torch's rounding of the interpolation weights


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: cannot build the transplat HIP library")


def _newest_dep() -> float:
    deps = list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))
    return max((p.stat().st_mtime for p in deps), default=0.0)


def build(verbose: bool = False, jobs: int = 8) -> Path:
    hipcc = _hipcc()
    BUILD.mkdir(parents=True, exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    dep_t = _newest_dep()
    procs = []
    objs = []
    for src in srcs:
        obj = BUILD / (src.stem + ".o")
        stamp = BUILD / (src.stem + ".cmd")
        objs.append(obj)
        cmd = [hipcc, *HIPCC_FLAGS, *FILE_FLAGS.get(src.name, []), "-c", str(src), "-o", str(obj)]
        key = hashlib.sha256("\0".join(cmd).encode()).hexdigest()
        if (obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, dep_t)
                and stamp.exists() and stamp.read_text() == key):
            continue
        stamp.unlink(missing_ok=True)
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT), stamp, key))
        if len(procs) >= jobs:
            _wait(procs.pop(0))
    for pr in procs:
        _wait(pr)
    if not LIB.exists() or LIB.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(LIB)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return LIB


def _wait(item) -> None:
    src, proc, stamp, key = item
    out, _ = proc.communicate()
    if proc.returncode != 0:
        sys.stderr.write(out.decode(errors="replace"))
        raise RuntimeError(f"hipcc failed on {src.name}")
    stamp.write_text(key)


if __name__ == "__main__":
    print(build(verbose=True))
