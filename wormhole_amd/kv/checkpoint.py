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


def model_name(base, it, shard):
    name = base
    if it >= 0:
        name += "_iter-%d" % it
    return name + "_part-%d" % shard


def _occupied(store):
    slots = store.occupied().long()
    return slots


def _arr(t, slots):
    return t[slots.to(t.device)].cpu().numpy() if t.numel() else np.zeros(0)


def save_linear(store, path):
    slots = _occupied(store)
    keys = _arr(store.keys, slots).astype(np.uint64)
    w = _arr(store.w, slots).astype(np.float32)
    m = w != 0
    rec = np.empty(int(m.sum()), dtype=[("k", "<u8"), ("w", "<f4")])
    rec["k"] = keys[m]
    rec["w"] = w[m]
    with open(path, "wb") as f:
        f.write(rec.tobytes())
    return len(rec)


def load_linear(store, path):
    raw = np.fromfile(path, dtype=[("k", "<u8"), ("w", "<f4")])
    keys = torch.from_numpy(raw["k"].view(np.int64).copy())
    w = torch.from_numpy(raw["w"].copy())
    _put(store, keys, {"w": w})
    nnz = int((w != 0).sum())
    store.stats[0] += nnz
    return len(raw)


def save_difacto(store, path):
    slots = _occupied(store)
    keys = _arr(store.keys, slots).astype(np.uint64)
    w = _arr(store.w, slots).astype(np.float32)
    z = _arr(store.z, slots).astype(np.float32)
    sq = _arr(store.sq, slots).astype(np.float32)
    dim = int(store.dim)
    has_v = np.zeros(len(keys), dtype=bool)
    V = VG = None
    if dim > 0:
        vrow = _arr(store.vrow, slots).astype(np.int64)
        has_v = vrow >= 0
        if has_v.any():
            rows = torch.from_numpy(vrow[has_v])
            V = store.V[rows.to(store.V.device)].cpu().numpy()[:, :dim]
            VG = store.VG[rows.to(store.VG.device)].cpu().numpy()[:, :dim]
    out = bytearray()
    vi = 0
    n = 0
    for i in range(len(keys)):
        if not has_v[i]:
            if w[i] == 0:
                continue  # Empty(): w0 == 0 && size == 1
            out += struct.pack("<Qi", int(keys[i]), 1)
            out += struct.pack("<fIff", float(w[i]), 0, float(sq[i]), float(z[i]))
        else:
            size = dim + 1
            out += struct.pack("<Qi", int(keys[i]), size)
            out += np.concatenate([[w[i]], V[vi]]).astype("<f4").tobytes()
            out += np.concatenate([[sq[i], z[i]], VG[vi]]).astype("<f4").tobytes()
            vi += 1
        n += 1
    if dim > 0 and has_v.any():
        assert vi == int(has_v.sum())
    with open(path, "wb") as f:
        f.write(bytes(out))
    return n


def load_difacto(store, path):
    data = open(path, "rb").read()
    pos = 0
    keys, w, z, sq, vk, vv, vg = [], [], [], [], [], [], []
    dim = int(store.dim)
    while pos < len(data):
        k, size = struct.unpack_from("<Qi", data, pos)
        pos += 12
        if size == 1:
            w0, _, s0, z0 = struct.unpack_from("<fIff", data, pos)
            pos += 16
            keys.append(k), w.append(w0), sq.append(s0), z.append(z0)
        else:
            arr = np.frombuffer(data, dtype="<f4", count=size, offset=pos)
            pos += 4 * size
            acc = np.frombuffer(data, dtype="<f4", count=size + 1, offset=pos)
            pos += 4 * (size + 1)
            if size - 1 != dim:
                raise ValueError("model embedding dim %d != configured dim %d" % (size - 1, dim))
            keys.append(k), w.append(arr[0]), sq.append(acc[0]), z.append(acc[1])
            vk.append(k), vv.append(arr[1:]), vg.append(acc[2:])
    kt = torch.tensor(np.array(keys, dtype=np.uint64).view(np.int64))
    _put(store, kt, {"w": torch.tensor(w, dtype=torch.float32),
                     "z": torch.tensor(z, dtype=torch.float32),
                     "sq": torch.tensor(sq, dtype=torch.float32)})
    if vk:
        _put_v(store, torch.tensor(np.array(vk, dtype=np.uint64).view(np.int64)),
               torch.tensor(np.stack(vv)), torch.tensor(np.stack(vg)))
    store.stats[0] += int((torch.tensor(w) != 0).sum())
    store.stats[1] += len(vk) * dim
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
