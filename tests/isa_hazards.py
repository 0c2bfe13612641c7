"""MFMA -> vector-read hazard scan of the shipped gfx950 code objects (CPU only, no GPU).

An XDL MFMA's destination may not be read (or overwritten) by a VALU, LDS or memory instruction
until enough wait states after issue (gfx950: XDL 8-pass -> 12 states; fp32 SMFMA 16-pass -> 18;
LLVM's GCNHazardRecognizer "MFMA write VGPR -> VALU read / VMEM read / WAW" rules, required_states). hipcc pads every read it can
see with s_nop; an inline-asm operand is invisible to it (round 5's v_max3_f32 read its MFMA's
accumulator 0 states after issue). This module disassembles every bundle of the library's
.hip_fatbin section (llvm-objdump --mcpu=gfx950) and walks each kernel linearly:

- an MFMA records its destination registers and pass count;
- every instruction adds one wait state, s_nop N adds N + 1;
- a non-MFMA instruction whose operands touch a pending destination range with fewer states than
  required is a violation (MFMA -> MFMA forwarding is the compiler's own and not checked);
- an unconditional branch or s_endpgm clears the pending set (straight-line paths only: a hazard
  reached only through a taken branch is not seen).

usage: python tests/isa_hazards.py [lib.so]  (prints violations, exit 1 if any)
"""
from __future__ import annotations

import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# passes of the MFMA forms in this build on gfx950 (cycles / 4: 32x32x16 bf16 = 32 cycles, 16x16x32 bf16
# = 16, 16x16x4 f32 = 32, 32x32x2 f32 = 64; 16x16x16 bf16 taken at the 16x16x32 rate, the conservative side)
PASSES = {
    "v_mfma_f32_32x32x16_bf16": 8, "v_mfma_f32_32x32x16_f16": 8,
    "v_mfma_f32_16x16x32_bf16": 4, "v_mfma_f32_16x16x32_f16": 4,
    "v_mfma_f32_16x16x16_bf16": 4, "v_mfma_f32_16x16x16_f16": 4,
    "v_mfma_f32_32x32x8_bf16": 8, "v_mfma_f32_32x32x8_f16": 8,
    "v_mfma_f32_16x16x4_f32": 8, "v_mfma_f32_32x32x2_f32": 16,
    "v_mfma_f32_32x32x1_2b_f32": 16, "v_mfma_f32_16x16x1_4b_f32": 8, "v_mfma_f32_4x4x1_16b_f32": 2,
}
_REG = re.compile(r"\b([va])(?:(\d+)|\[(\d+):(\d+)\])")


def required_states(op: str) -> int:
    """LLVM's gfx940 / gfx950 MFMA-write -> VALU / memory read-or-write wait states: XDL forms (bf16,
    f16, ...) NumPasses + 3, + 1 on gfx950 above 2 passes; the fp32 forms are SMFMA (non-XDL) there:
    NumPasses + 2."""
    passes = PASSES.get(op, 16)
    if "_f32_" in op and op.endswith("f32"):
        return passes + 2
    return passes + 3 + (1 if passes != 2 else 0)


def _regs(text: str) -> set:
    out = set()
    for kind, one, lo, hi in _REG.findall(text):
        if one:
            out.add((kind, int(one)))
        else:
            out.update((kind, r) for r in range(int(lo), int(hi) + 1))
    return out


def code_objects(lib: Path, work: Path) -> list:
    """Every gfx950 code object in lib's .hip_fatbin (one bundle per translation unit)."""
    fat = work / "fatbin"
    subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(lib), str(work / "junk")],
                   check=True, capture_output=True)
    data = fat.read_bytes()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
    cos = []
    for i in range(len(offs) - 1):
        b = work / f"b{i}.bin"
        co = work / f"b{i}.co"
        b.write_bytes(data[offs[i]:offs[i + 1]])
        subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={b}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        cos.append(co)
    return cos


def scan_disassembly(text: str) -> tuple:
    """(violations, number of MFMAs) of one llvm-objdump -d listing."""
    violations, mfmas = [], 0
    kernel = "?"
    pending = []  # [regs, states_left, mnemonic, line]
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            kernel, pending = m.group(1), []
            continue
        s = line.split("//")[0].strip()
        if not s or not line.startswith(("\t", " ")):
            continue
        op, _, args = s.partition(" ")
        if op.startswith("v_mfma") or op.startswith("v_smfmac"):
            mfmas += 1
            dest = _regs(args.split(",")[0])
            # other MFMAs' reads are the compiler's (no inline-asm MFMA here): only age the pending set
            for p in pending:
                p[1] -= 1
            pending = [p for p in pending if p[1] > 0 and not (p[0] & dest and p[0] == dest)]
            pending.append([dest, required_states(op), op, s])
            continue
        # reads and writes alike (VALU / LDS / memory RAW and WAW share the rule)
        touched = _regs(args)
        for p in pending:
            if p[0] & touched:
                need = required_states(p[2])
                got = need - p[1]
                violations.append(f"{kernel}: `{s}` touches the destination of `{p[3]}` {got} wait states "
                                  f"after issue (needs {need})")
        # a touched range is now either a violation (reported once) or safe: drop it either way
        pending = [p for p in pending if not (p[0] & touched)]
        n = int(args.strip() or 0) + 1 if op == "s_nop" else 1
        for p in pending:
            p[1] -= n
        pending = [p for p in pending if p[1] > 0]
        if op in ("s_branch", "s_endpgm", "s_setpc_b64"):
            pending = []
    return violations, mfmas


def scan_library(lib: Path) -> tuple:
    viol, checked, kernels = [], 0, 0
    with tempfile.TemporaryDirectory() as td:
        for co in code_objects(lib, Path(td)):
            text = subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--mcpu=gfx950", str(co)], check=True,
                                  capture_output=True, text=True).stdout
            kernels += len(re.findall(r"^[0-9a-f]+ <\S+>:", text, re.M))
            v, c = scan_disassembly(text)
            viol += v
            checked += c
    return viol, checked, kernels


if __name__ == "__main__":
    lib = Path(sys.argv[1]) if len(sys.argv) > 1 else Path(__file__).resolve().parents[1] / "transplat_amd" / "libtransplat_hip.so"
    v, c, k = scan_library(lib)
    print(f"{k} kernels, {len(v)} violations")
    for x in v:
        print(x)
    sys.exit(1 if v else 0)
