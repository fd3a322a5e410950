"""bin/xgboost.dmlc: ``<conf> [name=value ...]`` -- distributed GBDT with the
xgboost CLI surface the reference drives (learn/xgboost/mushroom.hadoop.conf,
learn/xgboost/run_yarn.sh; SURVEY §2.2 "xgboost"):

tasks ``train | pred | dump | eval``; parameters booster, objective, eta,
gamma, min_child_weight, max_depth, lambda, alpha, base_score, max_bin,
subsample, colsample_bytree, seed, eval_metric, num_round, save_period,
eval_train, eval[name]=path, data, test:data, model_in, model_out, model_dir,
fmap, name_dump, name_pred, dump_stats, dsplit=row, dsparse (keep the rows CSR:
wide libsvm data; default when num_feature > 4096), nthread (ignored),
num_feature.  Output: ``[r]\\t<set>-<metric>:<value>`` lines per round.
"""
import os
import sys

import torch

from .ps_app import _device
from ..utils.fs import open_uri  # noqa: E402


def _strip(v):
    v = v.strip()
    if len(v) >= 2 and v[0] == v[-1] and v[0] in "\"'":
        return v[1:-1]
    return v


def parse_args(argv):
    from .. import _native
    items = []
    if argv and argv[0] != "none" and "=" not in argv[0]:
        for key, kind, val in _native.host().parse_conf(open_uri(argv[0]).read()):
            if kind == "m":
                raise ValueError("nested messages are not valid in an xgboost conf")
            items.append((key, val))
        argv = argv[1:]
    for a in argv:
        if "=" not in a:
            raise ValueError("expected name=value, got %r" % a)
        k, v = a.split("=", 1)
        items.append((k.strip(), _strip(v)))
    return items


def main(argv):
    from .. import _native
    from ..models import gbdt as G
    from ..parallel.bsp import BSP, fault_point

    dev = _device()
    bsp = BSP(dev, job="xgboost")
    if not argv:
        bsp.tracker_print("Usage: xgboost.dmlc <conf> [name=value ...]")
        return 0
    param = G.GBDTParam()
    task, data, test_data = "train", None, None
    model_in, model_out, model_dir = None, None, "./"
    num_round, save_period, eval_train = 10, 0, 0
    fmap, name_dump, name_pred, dump_stats = None, "dump.txt", "pred.txt", 0
    num_feature = 0
    dsparse = None  # dsparse=1|0: keep the data CSR / dense (default: by width)
    evals = []
    for k, v in parse_args(argv):
        if param.set(k, v):
            continue
        if k == "task":
            task = v
        elif k == "data":
            data = v
        elif k == "test:data":
            test_data = v
        elif k.startswith("eval[") and k.endswith("]"):
            # a later setting of the same eval set (command line after the
            # conf) replaces the earlier one, like any other parameter
            evals = [(n, p) for n, p in evals if n != k[5:-1]] + [(k[5:-1], v)]
        elif k == "model_in":
            model_in = None if v == "NULL" else v
        elif k == "model_out":
            model_out = v
        elif k == "model_dir":
            model_dir = v
        elif k == "num_round":
            num_round = int(v)
        elif k == "save_period":
            save_period = int(v)
        elif k == "eval_train":
            eval_train = int(v)
        elif k == "fmap":
            fmap = v
        elif k == "name_dump":
            name_dump = v
        elif k == "name_pred":
            name_pred = v
        elif k in ("dump_stats", "with_stats"):
            dump_stats = int(v)
        elif k == "num_feature":
            num_feature = int(v)
        elif k == "dsparse":
            dsparse = bool(int(v))
        elif k in ("dsplit",):
            if v not in ("row", "auto"):
                raise SystemExit("only dsplit=row is supported")
        elif k in ("nthread", "tree_method", "updater", "silent", "use_buffer"):
            pass
        else:
            bsp.tracker_print("Warning: unknown parameter %s=%s ignored" % (k, v))
    if param.booster != "gbtree":
        raise SystemExit("only booster=gbtree is supported")
    host = _native.host()

    def load(path):
        # xgboost external-memory syntax "data#name.cache": the first run parses
        # the text split and writes this rank's rows as a binary CRB page
        # (RecordIO + LZ4, the reference's compressed row block) next to the
        # cache name; later runs load the page instead of re-parsing. The
        # matrix itself is then binned into HBM (288 GB per GPU holds any
        # split this tool is pointed at).
        cache = None
        if "#" in path:
            path, cache = path.split("#", 1)
        if cache:
            cpath = "%s.r%dof%d.crb" % (cache, bsp.rank, bsp.world)
            if host.file_size(cpath) > 0:
                return host.load_split(cpath, 0, 1, "crb")
        blk = host.load_split(path, bsp.rank, bsp.world, "libsvm")
        if cache:
            keys, off, val, lab, wt = blk
            w = host.RecordIOWriter(cpath)
            n = lab.numel()
            for r0 in range(0, max(n, 1), 1 << 18):  # records stay far below 2^29 bytes
                r1 = min(n, r0 + (1 << 18))
                a, b = int(off[r0]), int(off[r1])
                w.write(host.crb_encode(keys[a:b].contiguous(), (off[r0:r1 + 1] - a).contiguous(),
                                        val[a:b].contiguous() if val is not None and val.numel() else None,
                                        lab[r0:r1].contiguous(),
                                        wt[r0:r1].contiguous() if wt is not None and wt.numel() else None))
            w.close()
        return blk

    if task == "dump":
        if bsp.rank == 0:
            b = G.Booster.load(model_in, param)
            fm = G.load_fmap(fmap) if fmap else None
            with open_uri(name_dump, "w") as f:
                f.write(b.dump(fm, bool(dump_stats)))
        bsp.finalize()
        return 0

    if task in ("pred", "eval"):
        b = G.Booster.load(model_in, param)
        path = test_data or data
        raw = load(path)
        dm = G.make_dmatrix(*raw, ncol=b.num_feature, device=dev, sparse=dsparse)
        pred = b.obj.pred(b.predict_margin(dm))
        if task == "eval":
            metrics = param.eval_metric or [b.obj.default_metric()]
            s = "".join("\ttest-%s:%f" % (m, G.eval_metric(m, pred, dm.label, dm.weight, bsp))
                        for m in metrics)
            bsp.tracker_print(s.lstrip("\t"))
        else:
            parts = bsp.comm.allgather_object(pred.float().cpu().tolist())
            if bsp.rank == 0:
                with open_uri(name_pred, "w") as f:
                    for part in parts:
                        f.write("".join("%g\n" % p for p in part))
        bsp.finalize()
        return 0

    if task != "train":
        raise SystemExit("unknown task " + task)
    if data is None:
        raise SystemExit("need data=<path> for task=train")
    train_raw = load(data)
    eval_raw = [(name, load(path)) for name, path in evals]
    ncol = max([int(r[0].max().item()) + 1 if r[0].numel() else 0
                for r in [train_raw] + [e[1] for e in eval_raw]] + [num_feature])
    ncol = int(bsp.allreduce_scalar(ncol, "max", torch.int64))
    dtrain = G.make_dmatrix(*train_raw, ncol=ncol, device=dev, sparse=dsparse)
    deval = [(name, G.make_dmatrix(*r, ncol=ncol, device=dev, sparse=dsparse))
             for name, r in eval_raw]
    booster = G.Booster.load(model_in, param) if model_in else G.Booster(param, ncol)
    start = len(booster.trees)
    version, gstate, _ = bsp.load_checkpoint()
    if version > 0:
        booster = _booster_from_state(G, gstate, param)
        start = len(booster.trees)
        print("restart from version=%d (round %d)" % (version, start), flush=True)
    margin = booster.predict_margin(dtrain)
    # hessian-weighted sketch: weights at the starting margin
    hess = booster.obj.gpair(margin, dtrain.label, None)[:, 1] if dtrain.n else None
    cuts = G.Cuts.build(dtrain, param.max_bin, bsp, hess=hess)
    B = cuts.bin(dtrain)
    builder = G.make_builder(param, bsp, dtrain, cuts, B)
    emargins = [booster.predict_margin(d) for _, d in deval]
    metrics = param.eval_metric or [booster.obj.default_metric()]
    gen = torch.Generator().manual_seed(param.seed + 17 * bsp.rank)
    fgen = torch.Generator().manual_seed(param.seed)
    for r in range(start, num_round):
        gp = booster.obj.gpair(margin, dtrain.label, dtrain.weight)
        if param.subsample < 1.0:
            keep = (torch.rand(dtrain.n, generator=gen) < param.subsample).to(dev)
            gp = gp * keep[:, None].float()
        builder.sample_features(fgen)
        tree = builder.build(gp, margin)
        booster.trees.append(tree)
        msg = "[%d]" % r
        for (name, d), em in zip(deval, emargins):
            d.predict_tree(tree, em)
            p = booster.obj.pred(em)
            for m in metrics:
                msg += "\t%s-%s:%f" % (name, m, G.eval_metric(m, p, d.label, d.weight, bsp))
        if eval_train:
            p = booster.obj.pred(margin)
            for m in metrics:
                msg += "\ttrain-%s:%f" % (m, G.eval_metric(m, p, dtrain.label, dtrain.weight, bsp))
        bsp.tracker_print(msg)
        if save_period and (r + 1) % save_period == 0 and bsp.rank == 0:
            booster.save(os.path.join(model_dir, "%04d.model" % (r + 1)))
        v = bsp.checkpoint(_booster_state(booster))
        fault_point(bsp.rank, v)
    if bsp.rank == 0:
        out = model_out or os.path.join(model_dir, "%04d.model" % num_round)
        booster.save(out)
    bsp.finalize()
    return 0


def _booster_state(b):
    trees = []
    for t in b.trees:
        trees.append({k: torch.tensor(getattr(t, k), dtype=torch.float64)
                      for k in ("feat", "cond", "left", "right", "defl", "leaf", "gain", "cover")})
    return {"num_feature": b.num_feature, "trees": trees}


def _booster_from_state(G, s, param):
    b = G.Booster(param, int(s["num_feature"]))
    for d in s["trees"]:
        t = G.RegTree()
        n = d["feat"].numel()
        for k in ("feat", "left", "right", "defl"):
            setattr(t, k, [int(x) for x in d[k].tolist()])
        for k in ("cond", "leaf", "gain", "cover"):
            setattr(t, k, [float(x) for x in d[k].tolist()])
        t.parent = [-1] * n
        t.bin = [0] * n
        t.base_weight = [0.0] * n
        b.trees.append(t)
    return b


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
