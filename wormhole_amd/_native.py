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
    # WH_AB_HIP=<path to another build's _hip.so>: load that one instead
    # (same-box A/B of two kernel builds in one benchmark call; tools/gpu/ab.sh)
    alt = os.environ.get("WH_AB_HIP") if name == "_hip" else None
    try:
        if alt:
            import importlib.util as ilu
            import sys
            spec = ilu.spec_from_file_location("wormhole_amd._hip", alt)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules["wormhole_amd._hip"] = mod
            return mod
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
