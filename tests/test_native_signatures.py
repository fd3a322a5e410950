"""Every Python call into the native modules matches a pybind signature.

The HIP extension ``wormhole_amd/_hip.so`` loads without a GPU (only its
kernels need one), so its pybind docstrings -- the exact argument lists the
bindings accept -- are readable on the CPU. This test walks every Python file
of the repo, finds the calls that reach a native function or method (directly
as ``X.gbdt_grow(...)`` or through a local alias such as
``grow = hip.gbdt_grow if host else hip.gbdt_grow_dev; grow(...)``) and checks
arity and keyword names against the bindings, so a dropped or renamed argument
fails here instead of first on a GPU box (round 3 lost its whole GPU suite to
a comment that swallowed three arguments of ``gbdt_grow_dev``).
"""
import ast
import inspect
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# attribute names that are also Python-side functions or methods with their
# own signatures: a call is only checked when its receiver is a native module
# handle (``_native.hip()`` / a variable bound to it)
_MODULE_HANDLES = {"hip", "_hip", "host", "_host", "H"}


def _split_params(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _overloads(name, doc, method):
    """[(param names, required names)] from a pybind docstring."""
    sigs = []
    for line in (doc or "").splitlines():
        m = re.match(r"^\s*(?:\d+\.\s*)?" + re.escape(name) + r"\((.*)\)\s*->", line)
        if not m:
            continue
        names, required = [], set()
        for prm in _split_params(m.group(1)):
            if prm in ("*", "/") or prm.startswith("*"):
                continue
            pname = prm.split(":")[0].split("=")[0].strip()
            names.append(pname)
            if "=" not in prm:
                required.add(pname)
        if method and names and names[0] == "self":
            names = names[1:]
            required.discard("self")
        sigs.append((names, required))
    return sigs


def _native_table():
    from wormhole_amd import _native
    table = {}
    for getter in (_native.hip, _native.host):
        mod = getter()
        for name in dir(mod):
            if name.startswith("_"):
                continue
            obj = getattr(mod, name)
            if inspect.isclass(obj):
                sig = _overloads("__init__", obj.__init__.__doc__, True)
                if sig:
                    table.setdefault(name, []).extend(sig)
                for meth in dir(obj):
                    if meth.startswith("_"):
                        continue
                    fn = getattr(obj, meth)
                    if callable(fn) and not isinstance(fn, type):
                        sig = _overloads(meth, getattr(fn, "__doc__", ""), True)
                        if sig:
                            table.setdefault(meth, []).extend(sig)
            elif callable(obj):
                sig = _overloads(name, obj.__doc__, False)
                if sig:
                    table.setdefault(name, []).extend(sig)
    return table


def _py_files():
    skip = {".git", "build", "gpurun_out", "__pycache__", "reference"}
    for d, dirs, files in os.walk(ROOT):
        dirs[:] = [x for x in dirs if x not in skip]
        for f in files:
            if f.endswith(".py"):
                yield os.path.join(d, f)


def _common_attrs():
    """Attribute names of builtin / stdlib / torch types: a call of one of
    these names is most likely not a native one (dict.get, socket.send,
    Tensor.find...), so only handle-receiver calls are checked for them."""
    import io
    import queue
    import socket
    import threading
    import torch
    names = set()
    for t in (dict, list, str, set, bytes, io.IOBase, io.BufferedWriter, socket.socket,
              threading.Thread, threading.Event, queue.Queue, torch.Tensor,
              torch.cuda.Stream, torch.cuda.Event, type(os.environ)):
        names.update(dir(t))
    return names


def _python_defs(paths):
    names = set(_common_attrs())
    for p in paths:
        tree = ast.parse(open(p).read(), p)
        for node in ast.walk(tree):
            if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
                names.add(node.name)
    return names


def _is_handle(expr):
    """``_native.hip()`` / ``_native.host()`` or a name usually bound to one,
    or a native object by its conventional name (``self.store`` is a
    ``KVStore``, ``self._native`` a ``LinearStep``)."""
    if isinstance(expr, ast.Call) and isinstance(expr.func, ast.Attribute):
        return expr.func.attr in ("hip", "host") and not expr.args
    if isinstance(expr, ast.Attribute):
        return expr.attr in ("store", "_native")
    return isinstance(expr, ast.Name) and expr.id in _MODULE_HANDLES | {"store"}


def _matches(call, sig):
    names, required = sig
    npos = len(call.args)
    if npos > len(names):
        return False
    given = set(names[:npos])
    for kw in call.keywords:
        if kw.arg not in names or kw.arg in given:
            return False
        given.add(kw.arg)
    return required <= given


def _calls(table, pydefs):
    """(path, line, native names, call) for each checkable call."""
    for p in _py_files():
        tree = ast.parse(open(p).read(), p)
        scopes = [n for n in ast.walk(tree)
                  if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Module))]
        for scope in scopes:
            alias, kwdicts = {}, {}
            for node in ast.walk(scope):
                # kw = dict(a=..., b=...): the keywords of a later f(**kw)
                if isinstance(node, ast.Assign) and len(node.targets) == 1 and \
                        isinstance(node.targets[0], ast.Name) and \
                        isinstance(node.value, ast.Call) and \
                        isinstance(node.value.func, ast.Name) and node.value.func.id == "dict" \
                        and not node.value.args and all(k.arg for k in node.value.keywords):
                    kwdicts[node.targets[0].id] = [k.arg for k in node.value.keywords]
                # grow = a.gbdt_grow if host else a.gbdt_grow_dev  /  f = a.name
                if isinstance(node, ast.Assign) and len(node.targets) == 1 and \
                        isinstance(node.targets[0], ast.Name):
                    v = node.value
                    cands = [v.body, v.orelse] if isinstance(v, ast.IfExp) else [v]
                    if all(isinstance(c, ast.Attribute) and c.attr in table and
                           (c.attr not in pydefs or _is_handle(c.value)) for c in cands):
                        alias[node.targets[0].id] = [c.attr for c in cands]
            for node in ast.walk(scope):
                if not isinstance(node, ast.Call):
                    continue
                if any(isinstance(a, ast.Starred) for a in node.args):
                    continue
                if any(k.arg is None for k in node.keywords):
                    # f(**kw) with kw a dict(...) of this scope: expand it
                    extra = []
                    for k in node.keywords:
                        if k.arg is None:
                            if not (isinstance(k.value, ast.Name) and k.value.id in kwdicts):
                                extra = None
                                break
                            extra += [ast.keyword(arg=a_, value=k.value)
                                      for a_ in kwdicts[k.value.id]]
                    if extra is None:
                        continue
                    node = ast.Call(func=node.func, args=node.args,
                                    keywords=[k for k in node.keywords if k.arg] + extra,
                                    lineno=node.lineno, col_offset=node.col_offset)
                f = node.func
                if isinstance(f, ast.Attribute) and f.attr in table:
                    if f.attr in pydefs and not _is_handle(f.value):
                        continue
                    yield p, node.lineno, [f.attr], node
                elif isinstance(f, ast.Name) and f.id in alias:
                    yield p, node.lineno, alias[f.id], node


def _load_table():
    so = os.path.join(ROOT, "wormhole_amd", "_hip.so")
    if not os.path.exists(so):
        pytest.skip("native extension not built (python build_native.py)")
    return _native_table()


def test_docstring_parser():
    sig = _overloads("f", "f(self: X, a: int, b: list[tuple[int, int]], c: float = 0.5) -> None",
                     True)
    assert sig == [(["a", "b", "c"], {"a", "b"})]


def test_every_native_call_matches_a_binding():
    table = _load_table()
    pydefs = _python_defs(list(_py_files()))
    bad, seen = [], set()
    for path, line, names, call in _calls(table, pydefs):
        if (path, line, call.col_offset) in seen:  # nested scopes walk a call twice
            continue
        seen.add((path, line, call.col_offset))
        if not any(_matches(call, s) for nm in names for s in table[nm]):
            sigs = "; ".join("%s(%s)" % (nm, ", ".join(s[0])) for nm in names for s in table[nm])
            bad.append("%s:%d: %d positional, keywords %s vs %s" % (
                os.path.relpath(path, ROOT), line, len(call.args),
                [k.arg for k in call.keywords], sigs))
    names = {nm for _, _, nms, _ in _calls(table, pydefs) for nm in nms}
    assert len(seen) > 200, "found only %d native call sites: the scan is broken" % len(seen)
    for must in ("gbdt_grow", "gbdt_grow_dev", "gbdt_hist", "ps_open", "ps_push",
                 "ps_push_linear", "LinearStep", "step"):
        assert must in names, must
    assert not bad, "\n".join(bad)


def test_wide_bindings_have_named_arguments():
    """The bindings with many arguments are called by keyword: they must
    carry py::arg names (unnamed ones show up as arg0, arg1, ...)."""
    table = _load_table()
    for name in ("gbdt_grow", "gbdt_grow_dev", "gbdt_hist", "ps_open", "ps_push",
                 "ps_push_linear", "LinearStep", "step"):
        for names, _ in table[name]:
            assert not any(re.fullmatch(r"arg\d+", x) for x in names), (name, names)


def test_round3_dropped_arguments_are_caught():
    """The round-3 break: a trailing comment swallowed three arguments."""
    table = _load_table()
    src = ("grow = hip.gbdt_grow if host else hip.gbdt_grow_dev\n"
           "out = grow(B, Bc, ridx, gp, qs, valid, nbin, fgroups, mf,\n"
           "           tot,  # device grower: no host wait cv, co, eta,\n"
           "           alpha, lam, mcw, depth, eps, ar)\n")
    call = [n for n in ast.walk(ast.parse(src)) if isinstance(n, ast.Call)][-1]
    assert not any(_matches(call, s) for nm in ("gbdt_grow", "gbdt_grow_dev")
                   for s in table[nm])
    fixed = src.replace("# device grower: no host wait ", "")
    call = [n for n in ast.walk(ast.parse(fixed)) if isinstance(n, ast.Call)][-1]
    assert all(any(_matches(call, s) for s in table[nm]) for nm in ("gbdt_grow", "gbdt_grow_dev"))
