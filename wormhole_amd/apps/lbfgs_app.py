"""bin/lbfgs.dmlc and bin/fm.dmlc: ``<bin> <data_uri> [name=value ...]``
(reference learn/lbfgs-linear/lbfgs.cc:218-246, learn/lbfgs-fm/fm.cc:270-298).

Parameters (SetParam): objective={linear,logistic}, base_score,
num_feature, reg_L2, reg_L1, lbfgs_stop_tol, max_lbfgs_iter, min_lbfgs_iter,
max_linesearch_iter, linesearch_c1, linesearch_backoff, size_memory,
nthread, task={train,pred}, model_in, model_out, name_pred;
FM adds nfactor, reg_L2_V, fm_random.
"""
import sys

import torch

from .ps_app import _device
from ..utils.fs import open_uri  # noqa: E402


def main(kind, argv):
    from .. import _native
    from ..config import parse_kv_args
    from ..models.lbfgs_models import FMObjective, LinearObjective, _SplitData
    from ..parallel.bsp import BSP
    from ..solver.lbfgs import LBFGSSolver

    dev = _device()
    bsp = BSP(dev, job=kind)
    if len(argv) < 1:
        bsp.tracker_print("Usage: <data_in> param=val")
        return 0
    kv = parse_kv_args(argv[1:])
    keys, off, val, label, _w = _native.host().load_split(argv[0], bsp.rank, bsp.world, "libsvm")
    data = _SplitData(keys, off, val, label, dev)
    obj = (FMObjective if kind == "fm" else LinearObjective)(bsp, data, dev)
    solver = LBFGSSolver(bsp, obj)
    task, model_in, model_out, name_pred = "train", "NULL", "final.model", "pred.txt"
    for k, v in kv:
        obj.set_param(k, v)
        solver.set_param(k, v)
        if k == "task":
            task = v
        elif k == "model_in":
            model_in = v
        elif k == "model_out":
            model_out = v
        elif k == "name_pred":
            name_pred = v
    if model_in != "NULL":
        obj.load_model(model_in)
    if task == "train":
        w = solver.run()
        if bsp.rank == 0:
            obj.save_model(model_out, w)
    elif task == "pred":
        if model_in == "NULL":
            raise SystemExit("must set model_in for task=pred")
        w = obj.loaded.to(dev)
        pred = obj.predict(w).float().cpu()
        parts = bsp.comm.allgather_object(pred.tolist())
        if bsp.rank == 0:
            with open_uri(name_pred, "w") as f:
                for part in parts:
                    f.write("".join("%g\n" % p for p in part))
            print("Finishing writing to %s" % name_pred, flush=True)
    else:
        raise SystemExit("unknown task " + task)
    bsp.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2:]))
