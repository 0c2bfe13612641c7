"""Stage timer with the reference's tags and interface (reference src/misc/benchmarker.py:19-145:
`Benchmarker.time(tag)` pushes an NVTX range and records wall time per tag; the encoder and the
depth predictor wrap their stages in it: encoder_1..5, encoder_4a..4f, decoder).

MI355X form: each range is a roctx range (torch.cuda.nvtx maps to roctx on ROCm), so
`rocprofv3 --marker-trace --kernel-trace` attributes kernels to the reference's stage tags; with
`sync=True` every range also closes with HIP events on the current stream and a synchronise, so
`gpu_times` holds per-stage GPU milliseconds (the reference likewise synchronises around every
stage). Without a Benchmarker the encoder still emits the roctx ranges when TSPLAT_ROCTX=1.
"""
from __future__ import annotations

import json
import os
import time
from collections import defaultdict
from contextlib import contextmanager, nullcontext

import torch


def _nvtx():
    try:
        import torch.cuda.nvtx as nvtx

        return nvtx if torch.cuda.is_available() else None
    except Exception:  # pragma: no cover - torch without nvtx/roctx bindings
        return None


class Benchmarker:
    def __init__(self, sync: bool = False):
        self.execution_times = defaultdict(list)  # wall seconds per tag (reference field name)
        self.gpu_times = defaultdict(list)        # GPU milliseconds per tag (sync mode)
        self.sync = sync
        self._nvtx = _nvtx()

    @contextmanager
    def time(self, tag: str, num_calls: int = 1):
        ev = None
        if self._nvtx is not None:
            self._nvtx.range_push(tag)
        if self.sync and torch.cuda.is_available():
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if ev is not None:
                ev[1].record()
                ev[1].synchronize()
                self.gpu_times[tag].append(ev[0].elapsed_time(ev[1]) / num_calls)
            self.execution_times[tag].append((time.perf_counter() - t0) / num_calls)
            if self._nvtx is not None:
                self._nvtx.range_pop()

    def summary(self) -> dict:
        out = {}
        for tag, ts in self.execution_times.items():
            out[tag] = {"calls": len(ts), "wall_ms": 1e3 * sum(ts) / len(ts)}
            if self.gpu_times.get(tag):
                g = self.gpu_times[tag]
                out[tag]["gpu_ms"] = sum(g) / len(g)
        return out

    def dump(self, path) -> None:
        with open(path, "w") as f:
            json.dump(self.summary(), f, indent=1)

    def clear_history(self) -> None:
        self.execution_times.clear()
        self.gpu_times.clear()


class _RangesOnly:
    """roctx ranges without timing (TSPLAT_ROCTX=1 and no Benchmarker passed)."""

    def __init__(self):
        self._nvtx = _nvtx()

    @contextmanager
    def time(self, tag: str, num_calls: int = 1):
        if self._nvtx is not None:
            self._nvtx.range_push(tag)
        try:
            yield
        finally:
            if self._nvtx is not None:
                self._nvtx.range_pop()


class StageMarks:
    """Device-clock stage marks (TSPLAT_MARKS=1, no Benchmarker passed): entering and leaving a stage
    launches tsplat_timestamp on the current stream, so a captured step replays them in place;
    `read()` returns (tag, "begin" / "end", stream id, seconds since the first mark) per slot, in
    slot order (tools/graph_stages.py)."""

    def __init__(self, capacity: int = 256):
        self.capacity, self.slots, self.buf = capacity, [], None

    def _mark(self, tag: str, kind: str) -> None:
        from .. import _lib

        if not torch.cuda.is_available():
            return
        if self.buf is None:
            self.buf = torch.zeros(self.capacity, dtype=torch.int64, device="cuda")
        if len(self.slots) >= self.capacity:
            return
        s = torch.cuda.current_stream()
        self.slots.append((tag, kind, s.stream_id))
        _lib.check(_lib.load().tsplat_timestamp(_lib.ptr(self.buf), len(self.slots) - 1, _lib.stream_ptr(s.device)),
                   "tsplat_timestamp")

    def reset(self) -> None:
        """Forget the recorded slots (a new capture / eager step records them again)."""
        self.slots = []

    @contextmanager
    def time(self, tag: str, num_calls: int = 1):
        self._mark(tag, "begin")
        try:
            yield
        finally:
            self._mark(tag, "end")

    def read(self) -> list:
        t = self.buf[: len(self.slots)].cpu().tolist()
        t0 = min(t)
        return [(tag, kind, sid, (v - t0) / 1e8) for (tag, kind, sid), v in zip(self.slots, t)]


MARKS = StageMarks() if os.environ.get("TSPLAT_MARKS", "0") == "1" else None
_RANGES = MARKS if MARKS is not None else (_RangesOnly() if os.environ.get("TSPLAT_ROCTX", "0") == "1" else None)


def stage(benchmarker, tag: str):
    """The context a stage runs in: the caller's Benchmarker, else roctx ranges if enabled."""
    b = benchmarker if benchmarker is not None else _RANGES
    return b.time(tag) if b is not None else nullcontext()
