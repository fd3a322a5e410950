"""Model shard files of the PS learners.

File name: ``<model_out>[_iter-<k>]_part-<shard>`` (reference IterServer::ModelName,
learn/solver/iter_solver.h:115-119).  Content: for every non-empty entry the
uint64 key followed by the entry payload:

* linear  : f32 w                      (learn/linear/async_sgd.h:59-76; z, n not saved)
* difacto : i32 size, then
            size == 1 -> 8 bytes {f32 w0, 0} + 8 bytes {f32 sqc0, f32 z0}
            size  > 1 -> f32 w[size] (w0, V) + f32 sqc[size + 1] (sqc0, z0, V accumulators)
            (learn/difacto/async_sgd.h:158-193)

Works for the device store (_hip.KVStore) and the host store (CpuKVStore).
"""
import struct

import numpy as np
import torch
from ..utils.fs import open_uri  # noqa: E402


def model_name(base, it, shard):
    name = base
    if it >= 0:
        name += "_iter-%d" % it
    return name + "_part-%d" % shard


def _occupied(store):
    # table order (the device compaction is unordered): identical model
    # files for identical tables
    return store.occupied().long().sort().values


def save_linear(store, path):
    return _write("linear", _numpy(_gather(store, "linear")), 0, path)


def load_linear(store, path):
    raw = np.frombuffer(open_uri(path, "rb").read(), dtype=[("k", "<u8"), ("w", "<f4")])
    keys = torch.from_numpy(raw["k"].view(np.int64).copy())
    w = torch.from_numpy(raw["w"].copy())
    _put(store, keys, {"w": w})
    nnz = int((w != 0).sum())
    store.add_stat(0, nnz)
    return len(raw)


def _rec1():
    return np.dtype([("k", "<u8"), ("size", "<i4"), ("w", "<f4"), ("pad", "<u4"),
                     ("sq", "<f4"), ("z", "<f4")])


def _recv(dim):
    return np.dtype([("k", "<u8"), ("size", "<i4"), ("w", "<f4"), ("V", "<f4", (dim,)),
                     ("sq", "<f4"), ("z", "<f4"), ("VG", "<f4", (dim,))])


def save_difacto(store, path):
    """Vectorised dump: all scalar (size 1) records, then all embedding
    records -- a valid record stream in the reference layout."""
    return _write("difacto", _numpy(_gather(store, "difacto")), int(store.dim), path)


def _gather(store, kind):
    """Snapshot of the occupied entries as tensors on the store's device
    (gathers only: the live table can be updated as soon as they ran).
    z / sq / cnt also feed the resume side file (:func:`write_state`)."""
    slots = _occupied(store)

    def g(t):
        return t[slots.to(t.device)] if t.numel() else t.new_zeros(0)

    snap = {"keys": g(store.keys), "w": g(store.w), "z": g(store.z), "sq": g(store.sq),
            "cnt": g(store.cnt)}
    if kind == "difacto":
        dim = int(store.dim)
        if dim > 0 and slots.numel():
            vrow = g(store.vrow).long()
            has_v = vrow >= 0
            rows = vrow[has_v]
            snap["has_v"] = has_v
            snap["V"] = store.V[rows.to(store.V.device)][:, :dim]
            snap["VG"] = store.VG[rows.to(store.VG.device)][:, :dim]
    return snap


def _numpy(snap):
    return {k: v.cpu().numpy() for k, v in snap.items()}


def _write(kind, snap, dim, path):
    keys = snap["keys"].astype(np.uint64)
    w = snap["w"].astype(np.float32)
    if kind == "linear":
        m = w != 0
        rec = np.empty(int(m.sum()), dtype=[("k", "<u8"), ("w", "<f4")])
        rec["k"] = keys[m]
        rec["w"] = w[m]
        with open_uri(path, "wb") as f:
            f.write(rec.tobytes())
        return len(rec)
    z = snap["z"].astype(np.float32)
    sq = snap["sq"].astype(np.float32)
    has_v = snap.get("has_v")
    if has_v is None:
        has_v = np.zeros(len(keys), dtype=bool)
    one = ~has_v & (w != 0)  # Empty(): w0 == 0 && size == 1
    r1 = np.zeros(int(one.sum()), dtype=_rec1())
    r1["k"], r1["size"], r1["w"], r1["sq"], r1["z"] = keys[one], 1, w[one], sq[one], z[one]
    rv = np.zeros(int(has_v.sum()), dtype=_recv(max(dim, 1)))
    if len(rv):
        rv["k"], rv["size"], rv["w"] = keys[has_v], dim + 1, w[has_v]
        rv["sq"], rv["z"] = sq[has_v], z[has_v]
        rv["V"], rv["VG"] = snap["V"], snap["VG"]
    with open_uri(path, "wb") as f:
        f.write(r1.tobytes())
        f.write(rv.tobytes())
    return len(r1) + len(rv)


# ------------------------------------------------------------ resume state
# The reference shard formats omit optimizer state (linear keeps only w != 0,
# DiFacto keeps no feature counts), so a job restarted from them would not
# continue where it stopped. Next to every shard the worker writes
# ``<shard>.state`` (every occupied entry: key, w, z, sq, count) and, once
# both files are complete, ``<shard>.ok``; a restarted job resumes from the
# newest iteration whose every shard is sealed (apps/ps_app.py).
_STATE = np.dtype([("k", "<u8"), ("w", "<f4"), ("z", "<f4"), ("sq", "<f4"), ("cnt", "<u4")])


def write_state(snap, path):
    rec = np.zeros(len(snap["keys"]), dtype=_STATE)
    rec["k"] = snap["keys"].astype(np.uint64)
    rec["w"], rec["z"], rec["sq"] = snap["w"], snap["z"], snap["sq"]
    rec["cnt"] = snap["cnt"].astype(np.uint32)
    with open_uri(path + ".state", "wb") as f:
        f.write(rec.tobytes())
    with open_uri(path + ".ok", "w") as f:
        f.write("%d\n" % len(rec))


def load_state(store, path):
    """Restore the full optimizer state saved next to a shard (if any)."""
    from ..utils import fs
    if not fs.exists(path + ".state"):
        return 0
    rec = np.frombuffer(open_uri(path + ".state", "rb").read(), dtype=_STATE)
    kt = torch.from_numpy(rec["k"].view(np.int64).copy())
    _put(store, kt, {"w": torch.from_numpy(rec["w"].copy()),
                     "z": torch.from_numpy(rec["z"].copy()),
                     "sq": torch.from_numpy(rec["sq"].copy()),
                     "cnt": torch.from_numpy(rec["cnt"].view(np.int32).copy())})
    return len(rec)


def _write_all(kind, snap, dim, path):
    n = _write(kind, snap, dim, path)
    write_state(snap, path)
    return n


class AsyncSaver:
    """Model-shard saves that do not stall training.

    The occupied entries are gathered on a side stream (the compute stream
    waits only for these gathers, so later updates cannot leak into the
    snapshot), copied device -> pinned host memory asynchronously, and a
    background thread writes the shard file once the copy's event fired.
    ``join()`` waits for every pending write and re-raises its error; the
    worker joins before acknowledging a final save, a load, or exit.
    Host (CPU) stores save synchronously."""

    def __init__(self):
        self._pending = []
        self._stream = None

    def save(self, kind, store, path):
        dev = store.keys.device
        if dev.type != "cuda":
            return _write_all(kind, _numpy(_gather(store, kind)), int(getattr(store, "dim", 0)),
                              path)
        import threading
        main = torch.cuda.current_stream(dev)
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=dev)
        side = self._stream
        side.wait_stream(main)
        with torch.cuda.stream(side):
            snap = _gather(store, kind)
            gathered = torch.cuda.Event()
            gathered.record(side)
            host = {}
            for k, v in snap.items():
                h = torch.empty(v.shape, dtype=v.dtype, pin_memory=True)
                h.copy_(v, non_blocking=True)
                host[k] = h
            copied = torch.cuda.Event()
            copied.record(side)
        main.wait_event(gathered)
        dim = int(getattr(store, "dim", 0))
        box = {}

        def finish():
            try:
                copied.synchronize()
                box["n"] = _write_all(kind, {k: v.numpy() for k, v in host.items()}, dim, path)
            except BaseException as e:  # surfaced by join()
                box["err"] = e

        t = threading.Thread(target=finish, name="wh-save", daemon=True)
        t.start()
        self._pending.append((t, box, snap))
        return None

    def join(self):
        pending, self._pending = self._pending, []
        n = 0
        for t, box, _ in pending:
            t.join()
            if "err" in box:
                raise box["err"]
            n += box.get("n", 0)
        return n


def _parse_difacto(data, dim):
    """(keys, w, z, sq, vkeys, V, VG). Fast path for files laid out as all
    scalar records then all embedding records (what save_difacto writes);
    interleaved files (e.g. written by the reference) take the record walk."""
    d1, dv = _rec1(), _recv(max(dim, 1))
    n = len(data)
    # find the prefix of scalar records
    n1 = 0
    if n >= d1.itemsize:
        cand = np.frombuffer(data[: (n // d1.itemsize) * d1.itemsize], dtype=d1)
        bad = np.nonzero(cand["size"] != 1)[0]
        n1 = int(bad[0]) if len(bad) else len(cand)
    rest = n - n1 * d1.itemsize
    if dim > 0 and rest % dv.itemsize == 0:
        rv = np.frombuffer(data, dtype=dv, offset=n1 * d1.itemsize)
        if bool((rv["size"] == dim + 1).all()):
            r1 = np.frombuffer(data, dtype=d1, count=n1)
            return (np.concatenate([r1["k"], rv["k"]]), np.concatenate([r1["w"], rv["w"]]),
                    np.concatenate([r1["z"], rv["z"]]), np.concatenate([r1["sq"], rv["sq"]]),
                    rv["k"], rv["V"], rv["VG"])
    if rest == 0:
        r1 = np.frombuffer(data, dtype=d1, count=n1)
        e = np.zeros(0, dtype=np.float32)
        return r1["k"], r1["w"], r1["z"], r1["sq"], np.zeros(0, np.uint64), e, e
    # interleaved: walk the records
    pos = 0
    keys, w, z, sq, vk, vv, vg = [], [], [], [], [], [], []
    while pos < n:
        k, size = struct.unpack_from("<Qi", data, pos)
        pos += 12
        if size == 1:
            w0, _, s0, z0 = struct.unpack_from("<fIff", data, pos)
            pos += 16
            keys.append(k), w.append(w0), sq.append(s0), z.append(z0)
        else:
            if size - 1 != dim:
                raise ValueError("model embedding dim %d != configured dim %d" % (size - 1, dim))
            arr = np.frombuffer(data, dtype="<f4", count=size, offset=pos)
            pos += 4 * size
            acc = np.frombuffer(data, dtype="<f4", count=size + 1, offset=pos)
            pos += 4 * (size + 1)
            keys.append(k), w.append(arr[0]), sq.append(acc[0]), z.append(acc[1])
            vk.append(k), vv.append(arr[1:]), vg.append(acc[2:])
    f32 = np.float32
    return (np.array(keys, dtype=np.uint64), np.array(w, f32), np.array(z, f32),
            np.array(sq, f32), np.array(vk, dtype=np.uint64),
            np.stack(vv) if vv else np.zeros((0, dim), f32),
            np.stack(vg) if vg else np.zeros((0, dim), f32))


def load_difacto(store, path):
    data = open_uri(path, "rb").read()
    dim = int(store.dim)
    keys, w, z, sq, vk, V, VG = _parse_difacto(data, dim)
    if len(vk) and V.shape[1] != dim:
        raise ValueError("model embedding dim %d != configured dim %d" % (V.shape[1], dim))
    kt = torch.from_numpy(np.ascontiguousarray(keys).view(np.int64).copy())
    _put(store, kt, {"w": torch.from_numpy(np.array(w, dtype=np.float32)),
                     "z": torch.from_numpy(np.array(z, dtype=np.float32)),
                     "sq": torch.from_numpy(np.array(sq, dtype=np.float32))})
    if len(vk):
        _put_v(store, torch.from_numpy(np.ascontiguousarray(vk).view(np.int64).copy()),
               torch.from_numpy(np.array(V, dtype=np.float32)),
               torch.from_numpy(np.array(VG, dtype=np.float32)))
    store.add_stat(0, int((np.asarray(w) != 0).sum()))
    store.add_stat(1, len(vk) * dim)
    return len(keys)


def _put(store, keys, cols):
    if hasattr(store, "load_entries"):
        store.load_entries(keys, cols)
        return
    dev = store.w.device
    slots = store.find(keys.to(dev), True).long()
    if bool((slots < 0).any()):
        raise RuntimeError("parameter table full while loading the model")
    for name, val in cols.items():
        getattr(store, name).index_put_((slots,), val.to(dev))


def _put_v(store, keys, V, VG):
    if hasattr(store, "load_v"):
        store.load_v(keys, V, VG)
        return
    dev = store.w.device
    slots = store.find(keys.to(dev), True).long()
    m = keys.numel()
    start = int(store.vnext.item())
    if start + m > store.vcap:
        raise RuntimeError("embedding slab too small for the model (%d rows)" % (start + m))
    rows = torch.arange(start, start + m, device=dev, dtype=torch.int64)
    store.vnext.fill_(start + m)
    store.vrow.index_put_((slots,), rows.to(torch.int32))
    vs = store.vstride
    pad = torch.zeros(m, vs, dtype=torch.float32)
    pad[:, : V.shape[1]] = V
    store.V.index_put_((rows,), pad.to(dev))
    pad.zero_()
    pad[:, : VG.shape[1]] = VG
    store.VG.index_put_((rows,), pad.to(dev))
