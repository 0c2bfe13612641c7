"""CPU-side ISA check of the shipped library: no instruction touches an MFMA destination inside the
gfx950 wait-state window (tests/isa_hazards.py). Round 5 shipped an inline-asm v_max3_f32 that read
the bf16 v2 attention kernel's score accumulator 0 states after the MFMA issued."""
from pathlib import Path

import pytest

import isa_hazards as H

LIB = Path(__file__).resolve().parents[1] / "transplat_amd" / "libtransplat_hip.so"


def test_scanner_flags_a_hazard():
    # the round-5 sequence (win_attn_bf16_v2_kernel), and the same read after the compiler's pad
    bad = """0000000000001000 <k>:
\tv_mfma_f32_32x32x16_bf16 v[64:79], v[224:227], v[160:163], v[64:79] // 0
\tv_max3_f32 v220, v80, v64, v81 // 8
"""
    good = bad.replace("\tv_max3_f32", "\ts_nop 11\n\tv_max3_f32")
    short = bad.replace("\tv_max3_f32", "\ts_nop 10\n\tv_max3_f32")
    assert len(H.scan_disassembly(bad)[0]) == 1
    assert H.scan_disassembly(good)[0] == []
    assert len(H.scan_disassembly(short)[0]) == 1
    # fp32 SMFMA, 16 passes: 18 states
    f32 = """0000000000001000 <k>:
\tv_mfma_f32_32x32x2_f32 v[2:17], v32, v55, v[2:17]
\ts_nop 7
\ts_nop 7
\ts_nop 0
\tds_write_b32 v19, v2
"""
    assert len(H.scan_disassembly(f32)[0]) == 1
    assert H.scan_disassembly(f32.replace("s_nop 0", "s_nop 1"))[0] == []


@pytest.mark.skipif(not LIB.exists(), reason="library not built (python -m transplat_amd.build)")
def test_no_mfma_read_hazards_in_library():
    viol, mfmas, kernels = H.scan_library(LIB)
    print(f"[isa] {kernels} kernels, {mfmas} MFMAs scanned, {len(viol)} violations")
    assert mfmas > 1000 and kernels > 100
    assert viol == [], "\n".join(viol[:20])
