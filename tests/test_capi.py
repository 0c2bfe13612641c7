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


def test_debug_mode_refuses_graph_capture():
    """TSPLAT_DEBUG=1 / tsplat_set_debug syncs after every launch, which hipGraph capture forbids:
    GraphedStep (bench.py's default) refuses up front instead of failing inside the capture."""
    import pytest

    from transplat_amd.e2e import GraphedStep

    lib = _lib.load()
    was = lib.tsplat_set_debug(1)
    try:
        assert _lib.debug_enabled()
        with pytest.raises(RuntimeError, match="cannot be captured"):
            GraphedStep(None, {})
    finally:
        lib.tsplat_set_debug(was)
    assert _lib.debug_enabled() == bool(was)


def test_package_reads_no_undefined_names():
    """Every name the package's modules read is defined or imported somewhere in them
    (tools/namecheck.py): the GPU dispatch code cannot run in the CPU suite, so a helper an edit
    removed would otherwise surface only on the GPU box."""
    import subprocess
    import sys

    root = Path(__file__).resolve().parents[1]
    files = [str(p) for p in (root / "transplat_amd").rglob("*.py")] + [str(root / "bench.py")]
    out = subprocess.run([sys.executable, str(root / "tools" / "namecheck.py")] + files, capture_output=True,
                         text=True)
    assert out.returncode == 0, out.stdout
