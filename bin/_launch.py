"""Shared shim of the bin/*.dmlc entry scripts: puts the repo on sys.path;
``run(main, *args)`` runs an app and leaves the process without the
interpreter's teardown."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def run(main, *args):
    """``main(*args)`` -> exit code, then ``os._exit``. A process group
    outlives ``destroy_process_group`` while Python still references it, and a
    gloo worker thread that drops the last reference of a tensor after the
    interpreter began finalising takes the GIL, is ended by the interpreter
    (a forced unwind through a noexcept frame) and aborts the whole process
    with "terminate called without an active exception" once the job is
    already done. Every app has written its files and closed its transport by
    the time ``main`` returns, so the teardown is skipped: stdio (Python's and
    the C library's) is flushed, pending device work is waited for, and the
    process exits with ``main``'s code."""
    import traceback
    try:
        rc = main(*args)
    except SystemExit as e:
        rc = e.code
    except BaseException:  # noqa: BLE001 - reported, then a failing exit code
        traceback.print_exc()
        rc = 1
    if rc is None:
        rc = 0
    elif not isinstance(rc, int):
        print(rc, file=sys.stderr)
        rc = 1
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        torch.cuda.synchronize()
    if os.environ.get("WH_TIMING") and "wormhole_amd._hip" in sys.modules:
        # os._exit skips the native steps' destructors, which print the
        # WH_TIMING=step summaries of runs shorter than 1000 calls
        try:
            sys.modules["wormhole_amd._hip"].timing_flush()
        except Exception:  # noqa: BLE001 - profiling output must not change the exit code
            pass
    for f in (sys.stdout, sys.stderr):
        try:
            f.flush()
        except Exception:  # noqa: BLE001 - a closed pipe must not change the code
            pass
    import ctypes
    ctypes.CDLL(None).fflush(None)
    os._exit(rc)
