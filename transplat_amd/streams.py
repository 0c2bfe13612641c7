"""Fork / join of independent encoder branches onto side streams (captured into the step's hipGraph
as parallel branches: a stream fork is an event record + wait, which graph capture turns into
graph edges).

At batch 1 most launches of the step are latency-bound chains that occupy a fraction of the 256
CUs (DINOv2's M = 650 GEMMs, the U-Nets' 16^2-64^2 convolutions, 256-workgroup attention
kernels); two independent chains on two streams fill the idle CUs. Which branches are independent
follows the reference's data flow: Depth-Anything and the backbone both read only the context
images (encoder_trans.py:199-228); the depth predictor's full-resolution feature projection reads
only backbone features (depth_predictor_trans.py:448-452) and runs beside the cost volume.

`fork(device, fn, *tensors)` runs fn(*tensors) on a side stream after the current stream's work so
far; `join(pending)` makes the current stream wait for it and returns fn's result. Inputs are
marked as used by the side stream and outputs as used by the current one (record_stream), so the
caching allocator never hands their memory to the other stream while it is still in flight.
`serial()` turns forking off (the reference's serial order), e.g. to time one kernel alone.

Tensors a branch reads must reach it as fork arguments (tuples, lists and dict values are walked)
so that they are marked; a tensor the branch only captures through a closure is not marked and must
stay referenced by the caller until join.

Forks nest only from the current stream: a fork issued while a side stream is current (inside a
forked branch) during hipGraph capture raises. ROCm 7.2's capture_end segfaults on a graph whose
side-stream branch forks onto a second side stream (tools/graph_fork_repro.py nested_once,
profiles/r3/hoist_dbg/); a flat fork from the capturing stream is fine.
"""
from __future__ import annotations

import os
from contextlib import contextmanager

import torch

_ENABLED = os.environ.get("TSPLAT_STREAMS", "1") != "0"  # A/B knob
_SIDE: dict = {}


def enabled(device) -> bool:
    return _ENABLED and torch.device(device).type == "cuda"


@contextmanager
def serial():
    global _ENABLED
    was, _ENABLED = _ENABLED, False
    try:
        yield
    finally:
        _ENABLED = was


def side_stream(device, slot: int = 0) -> torch.cuda.Stream:
    dev = torch.device(device)
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), slot)
    if key not in _SIDE:
        # (a higher-priority side stream made the replayed C2 step 2.6x slower: 184-204 vs 485
        # views/s, profiles/r6/ab_c2_stream_prio.txt)
        _SIDE[key] = torch.cuda.Stream(torch.device("cuda", key[0]))
    return _SIDE[key]


def _tensors(x):
    if torch.is_tensor(x):
        yield x
    elif isinstance(x, (tuple, list)):
        for y in x:
            yield from _tensors(y)
    elif isinstance(x, dict):
        for y in x.values():
            yield from _tensors(y)


class _Pending:
    def __init__(self, out, main=None, side=None):
        self.out, self.main, self.side = out, main, side


class NestedForkError(RuntimeError):
    """A fork from a side stream during hipGraph capture (see the module docstring)."""


def _is_side(stream) -> bool:
    return any(stream == s for s in _SIDE.values())


def fork(device, fn, *args, slot: int = 0) -> _Pending:
    if not enabled(device):
        return _Pending(fn(*args))
    main = torch.cuda.current_stream(device)
    if _is_side(main) and torch.cuda.is_current_stream_capturing():
        raise NestedForkError("streams.fork from a side stream inside hipGraph capture: HIP's capture_end "
                              "crashes on nested side-stream forks (fork from the capturing stream instead)")
    side = side_stream(device, slot)
    side.wait_stream(main)
    for t in _tensors(args):
        t.record_stream(side)
    with torch.cuda.stream(side):
        out = fn(*args)
    return _Pending(out, main, side)


def join(p: _Pending):
    if p.side is not None:
        p.main.wait_stream(p.side)
        for t in _tensors(p.out):
            t.record_stream(p.main)
    return p.out
