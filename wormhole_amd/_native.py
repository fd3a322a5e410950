"""Loader for the in-tree native extensions.

``_hip``  : gfx950 HIP kernels (built by ``build_native.py``)
``_host`` : native C++ host runtime (parsers, config, pool, control plane)

On a machine with a GPU the HIP extension is REQUIRED: ops fail loudly instead
of silently falling back to the PyTorch reference path.
"""
import importlib
import os

_hip = None
_host = None
_err = {}


def _try(name):
    try:
        return importlib.import_module("wormhole_amd." + name)
    except ImportError as e:  # pragma: no cover - reported by require_*()
        _err[name] = e
        return None


def hip():
    """The HIP kernel module; raises if it is not built."""
    global _hip
    if _hip is None:
        import torch  # noqa: F401  (loads libamdhip64 / c10_hip first)
        _hip = _try("_hip")
        if _hip is None:
            raise RuntimeError(
                "wormhole_amd._hip is not built (%s); run `python build_native.py`"
                % _err.get("_hip"))
    return _hip


def host():
    """The native host runtime module; raises if it is not built."""
    global _host
    if _host is None:
        import torch  # noqa: F401
        _host = _try("_host")
        if _host is None:
            raise RuntimeError(
                "wormhole_amd._host is not built (%s); run `python build_native.py`"
                % _err.get("_host"))
    return _host


def have_hip():
    try:
        hip()
        return True
    except RuntimeError:
        return False


def so_paths():
    d = os.path.dirname(os.path.abspath(__file__))
    return [os.path.join(d, f) for f in ("_hip.so", "_host.so")]
