"""Pipeline-stage tracing and metrics.

* ``stage(name)`` -- a context manager around one pipeline stage (parse, H2D,
  localize, pull, forward, backward, push ...). It always accumulates the
  stage's host wall time (cheap: two perf_counter calls); with
  ``WH_TRACE=1`` it also opens a roctx range, so
  ``rocprofv3 --marker-trace --kernel-trace`` shows the stages on the same
  timeline as the kernels (libroctx64 is loaded through ctypes; without it
  the ranges are skipped, never an error).
* ``take()`` -- the accumulated per-stage seconds and call counts since the
  last take (the worker turns them into the reference's "overhead %" line,
  learn/solver/minibatch_solver.h:244-248).
* ``MetricsStream`` -- JSON-lines metrics for benchmark harnesses, enabled by
  ``WH_METRICS=<path>`` (one line per progress report: examples/s and the
  stage breakdown).
* ``timing_on(what)`` -- the profiling aids listed in ``WH_TIMING``
  (comma-separated: ``step``, ``step2``, ``loc``, ``ingest``, ``comm``;
  docs/build.md).
"""
import contextlib
import ctypes
import json
import os
import threading
import time

def timing_on(what):
    """True when ``what`` is listed in WH_TIMING (the C++ side reads the same
    variable: csrc/bind/hip_ops.cc timing_on)."""
    return what in os.environ.get("WH_TIMING", "").split(",")


_lock = threading.Lock()
_acc = {}
_roctx = None
_roctx_tried = False


def _lib():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    if os.environ.get("WH_TRACE", "0") in ("", "0"):
        return None
    root = os.environ.get("ROCM_PATH", "/opt/rocm")
    for name in (os.path.join(root, "lib", "libroctx64.so"), "libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            _roctx = lib
            break
        except OSError:
            continue
    return _roctx


@contextlib.contextmanager
def stage(name):
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    t0 = time.perf_counter()
    try:
        yield
    finally:
        dt = time.perf_counter() - t0
        if lib is not None:
            lib.roctxRangePop()
        with _lock:
            s = _acc.get(name)
            if s is None:
                _acc[name] = [dt, 1]
            else:
                s[0] += dt
                s[1] += 1


def take():
    """{stage: (seconds, calls)} since the last take(), then reset."""
    with _lock:
        out = {k: (v[0], v[1]) for k, v in _acc.items()}
        _acc.clear()
    return out


def overhead_line(stages, wall, n_mb, compute=("process",)):
    """The reference worker's summary: minibatches, time per minibatch and
    the share of wall time NOT spent in compute stages."""
    comp = sum(stages.get(k, (0.0, 0))[0] for k in compute)
    per = wall / max(n_mb, 1)
    ovh = 100.0 * max(wall - comp, 0.0) / wall if wall > 0 else 0.0
    parts = ", ".join("%s %.1f ms" % (k, 1e3 * v[0] / max(n_mb, 1))
                      for k, v in sorted(stages.items()))
    return "done %d minibatches, %.2f ms per minibatch, overhead %.1f%% (%s)" % (
        n_mb, 1e3 * per, ovh, parts)


class MetricsStream:
    """Append-only JSON lines (WH_METRICS=<path>; '{rank}' in the path is
    replaced by the rank)."""

    def __init__(self, rank=0, path=None):
        path = path if path is not None else os.environ.get("WH_METRICS")
        self.f = None
        if path:
            path = path.replace("{rank}", str(rank))
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
            self.f = open(path, "a")
        self.rank = rank

    def write(self, **kw):
        if self.f is None:
            return
        kw.setdefault("t", time.time())
        kw.setdefault("rank", self.rank)
        self.f.write(json.dumps(kw) + "\n")
        self.f.flush()

    def close(self):
        if self.f is not None:
            self.f.close()
            self.f = None


_NULL = contextlib.nullcontext()
ENABLED = os.environ.get("WH_TRACE", "0") not in ("", "0")


def span(name):
    """stage(name) when WH_TRACE is set, else a shared no-op context (the
    learners' inner stages run per minibatch on a sub-millisecond step)."""
    return stage(name) if ENABLED else _NULL
