"""Per-phase trace ranges (SURVEY §5 tracing: data / fwd / bwd / all-reduce /
optimizer).  `phase(name)` pushes a roctx range (ainp_range_push, the
rocprofiler-sdk marker API) on entry and pops it on exit; `rocprofv3
--marker-trace --kernel-trace` then attributes every kernel to its phase
(tools/phase_table.py).  Off unless AINP_TRACE=1 (or enable()), so the
default path makes no extra host calls."""
from __future__ import annotations

import contextlib
import os

from . import _lib

_ON = os.environ.get("AINP_TRACE", "0") == "1"


def enable(on: bool = True) -> None:
    global _ON
    _ON = bool(on)


def enabled() -> bool:
    return _ON


@contextlib.contextmanager
def phase(name: str):
    if not _ON:
        yield
        return
    _lib.lib.ainp_range_push(name.encode())
    try:
        yield
    finally:
        _lib.lib.ainp_range_pop()


def mark(name: str) -> None:
    if _ON:
        _lib.lib.ainp_mark(name.encode())
