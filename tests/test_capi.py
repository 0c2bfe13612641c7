"""The C-ABI library loads on the CPU host and exports every symbol include/*.h declares."""
import re
from pathlib import Path

import torch  # noqa: F401  (HIP runtime must come from torch before the library loads)

from transplat_amd import _lib

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        text = h.read_text()
        names |= set(re.findall(r"^\s*(?:int|int32_t|int64_t|size_t|void)\s+\**(tsplat_\w+)\s*\(", text, re.M))
    return sorted(names)


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "tsplat_raster_fwd" in syms and "tsplat_version" in syms


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, f"missing exports: {missing}"


def test_python_signatures_cover_header():
    assert set(declared_symbols()) == set(_lib.SIGNATURES), "ctypes table out of sync with header"


def test_library_reports_version_and_workspace_without_gpu():
    lib = _lib.load()
    assert lib.tsplat_version() >= 1
    nb = lib.tsplat_raster_workspace_bytes(131072, 3, 256, 256, 1 << 20)
    assert nb >= (1 << 20) * 8 + 3 * 131072 * 40
