"""Config loading: the native proto-text parser (csrc/host/conf_parser.cc)
produces a key/value tree; this module validates it against the typed
schemas in :mod:`.schema` (unknown keys are fatal, like protobuf TextFormat in
the reference ArgParser, learn/base/arg_parser.h:13-64) and applies argv
overrides ``key=value`` after the file.  ``argv[1] == "none"`` means "no conf
file" (learn/linear/linear.cc:9).
"""
import dataclasses

from .. import _native
from .schema import DifactoConfig, Embedding, LinearConfig  # noqa: F401
from ..utils.fs import open_uri  # noqa: E402

_BOOL = {"true": True, "false": False, "1": True, "0": False, "True": True, "False": False}


def _convert(cls, name, ftype, kind, raw):
    enums = getattr(cls, "ENUMS", {})
    if name in enums:
        table = enums[name]
        if raw in table:
            return table[raw]
        try:
            v = int(raw)
        except ValueError:
            raise ValueError("unknown enum value %r for %s" % (raw, name))
        if v not in table.values():
            raise ValueError("unknown enum value %r for %s" % (raw, name))
        return v
    if ftype in (bool, "bool"):
        if raw not in _BOOL:
            raise ValueError("bad bool %r for %s" % (raw, name))
        return _BOOL[raw]
    if ftype in (int, "int"):
        return int(float(raw)) if ("e" in raw or "." in raw) else int(raw)
    if ftype in (float, "float"):
        return float(raw)
    return raw  # string


def _apply(obj, items):
    cls = type(obj)
    fmap = {f.name: f for f in dataclasses.fields(cls) if not f.name.startswith("_")}
    nested = getattr(cls, "NESTED", {})
    for key, kind, val in items:
        if key not in fmap:
            raise ValueError("unknown configuration key '%s' for %s" % (key, cls.__name__))
        if kind == "m":
            if key not in nested:
                raise ValueError("'%s' is not a message field" % key)
            sub = nested[key]()
            _apply(sub, val)
            getattr(obj, key).append(sub)
        else:
            if key in nested:
                raise ValueError("'%s' must be a message" % key)
            f = fmap[key]
            setattr(obj, key, _convert(cls, key, f.type, kind, val))
        obj._set.add(key)
    return obj


def parse_text(cls, text, base=None):
    obj = base if base is not None else cls()
    return _apply(obj, _native.host().parse_conf(text))


def arg2proto(text):
    """dmlc::Config-format text -> protobuf text (native; the reference's
    alternative front end, learn/base/arg2proto.h:13-20)."""
    return _native.host().arg2proto(text)


def load_dmlc(cls, conf_path):
    """Load a dmlc::Config-style conf (``key = value`` lines, repeated keys
    allowed) into a schema object through :func:`arg2proto`."""
    with open_uri(conf_path) as f:
        return parse_text(cls, arg2proto(f.read()))


def load(cls, conf_path, argv=()):
    """Reference ArgParser: ReadFile(conf) then ReadArgs(argv) (later wins)."""
    obj = cls()
    if conf_path and conf_path != "none":
        with open_uri(conf_path) as f:
            parse_text(cls, f.read(), obj)
    if argv:
        parse_text(cls, "\n".join(argv), obj)
    return obj


def parse_kv_args(argv):
    """``name=value`` arguments of the rabit apps (lbfgs, fm, xgboost):
    returns an ordered list of (name, value)."""
    out = []
    for a in argv:
        if "=" not in a:
            raise ValueError("expected name=value, got %r" % a)
        k, v = a.split("=", 1)
        out.append((k.strip(), v.strip()))
    return out
