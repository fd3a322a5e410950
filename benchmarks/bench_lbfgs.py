#!/usr/bin/env python3
"""L-BFGS benchmark: logistic regression with OWL-QN (L1) on Criteo-shaped
sparse data, device-resident CSR, one GPU (or N ranks, data-parallel).

The reference runs the same solver over a libsvm split on each rabit rank
(learn/lbfgs-linear/lbfgs.cc:131-207 objective, learn/solver/lbfgs.h:168-196
iteration: one gradient pass, the two-loop direction, a backtracking line
search of >= 1 objective passes, a checkpoint). Here every rank generates its
split on the device (13 integer + 26 categorical fields, Criteo-1TB value
cardinalities, power law), hashes the keys into ``--features`` columns (the
libsvm form of the data: feature ids < num_feature), localizes it ONCE, and
then every objective / gradient pass is SpMV / SpMV^T over that resident CSR.

Reports ms per L-BFGS iteration (timed over ``--iters`` after ``--warmup``),
line-search objective evaluations per iteration and the time of one
objective and one gradient pass.

    python benchmarks/bench_lbfgs.py [--rows 4000000] [--features 16777216] [--iters 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from wormhole_amd.data.synthetic import CRITEO_TB_CARD, criteo_batch  # noqa: E402
from wormhole_amd.models.lbfgs_models import LinearObjective, _SplitData  # noqa: E402
from wormhole_amd.parallel.bsp import BSP  # noqa: E402
from wormhole_amd.parallel.comm import env_local_rank  # noqa: E402
from wormhole_amd.solver.lbfgs import LBFGSSolver  # noqa: E402


def split(rows, features, rank, device, chunk=1_000_000):
    """This rank's rows: Criteo-shaped keys hashed into [0, features)."""
    ks, ls, offs, base = [], [], [], 0
    for i, a in enumerate(range(0, rows, chunk)):
        n = min(chunk, rows - a)
        keys, label, off = criteo_batch(n, 4242 + rank, i, device, CRITEO_TB_CARD)
        ks.append(torch.remainder(keys, features))
        ls.append(label)
        offs.append(off[:-1] + base)
        base += int(off[-1])
    offs.append(torch.tensor([base], dtype=torch.int64, device=device))
    return torch.cat(ks), torch.cat(offs), torch.cat(ls)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_000_000, help="rows per rank")
    ap.add_argument("--features", type=int, default=1 << 24)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reg-l1", type=float, default=1.0)
    ap.add_argument("--memory", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", env_local_rank()) if torch.cuda.is_available() else \
        torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    bsp = BSP(dev, job="bench_lbfgs")
    t0 = time.perf_counter()
    keys, off, label = split(args.rows, args.features, bsp.rank, dev)
    data = _SplitData(keys, off, None, label, dev)
    del keys
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    sync()
    t_load = time.perf_counter() - t0
    obj = LinearObjective(bsp, data, dev)
    obj.set_param("objective", "logistic")
    obj.set_param("num_feature", str(args.features))
    solver = LBFGSSolver(bsp, obj)
    solver.silent = True
    for k, v in (("reg_L1", args.reg_l1), ("size_memory", args.memory),
                 ("lbfgs_stop_tol", 0.0), ("min_lbfgs_iter", 1 << 30),
                 ("max_lbfgs_iter", args.warmup + args.iters)):
        solver.set_param(k, str(v))
    # count the objective passes (line-search trials)
    evals = [0]
    inner = obj.eval

    def counted(w):
        evals[0] += 1
        return inner(w)
    obj.eval = counted
    solver.init()
    # the objective after every iteration (pins the trajectory: a change to
    # the solver or the kernels that moves the iterates shows here)
    traj = [float(solver.old_objval)]
    for _ in range(args.warmup):
        solver.update_one_iter()
        traj.append(float(solver.old_objval))
    sync()
    bsp.barrier()
    e0, it0 = evals[0], solver.num_iteration
    t1 = time.perf_counter()
    for _ in range(args.iters):
        solver.update_one_iter()
        traj.append(float(solver.old_objval))  # (a host float the solver already holds)
    sync()
    bsp.barrier()
    dt = time.perf_counter() - t1
    n_it = solver.num_iteration - it0
    # one objective and one gradient pass alone
    w = solver.weight
    reps = 5
    sync()
    ta = time.perf_counter()
    for _ in range(reps):
        inner(w)
    sync()
    t_eval = (time.perf_counter() - ta) / reps
    ta = time.perf_counter()
    for _ in range(reps):
        obj.calc_grad(w)
    sync()
    t_grad = (time.perf_counter() - ta) / reps
    if bsp.rank == 0:
        print(json.dumps({
            "bench": "lbfgs-logistic-owlqn", "n_ranks": bsp.world, "rows_per_rank": args.rows,
            "nnz_per_rank": int(off[-1]), "num_feature": args.features,
            "uniq_features_per_rank": int(data.uniq.numel()), "size_memory": args.memory,
            "reg_L1": args.reg_l1, "iters": n_it, "ms_per_iter": 1000.0 * dt / n_it,
            "objective_evals_per_iter": (evals[0] - e0) / n_it,
            "ms_objective_pass": 1000.0 * t_eval, "ms_gradient_pass": 1000.0 * t_grad,
            "objval": float(solver.old_objval), "objval_per_iter": traj, "load_s": t_load,
            "data": "synthetic Criteo-1TB-shaped (13 int + 26 cat fields, power law), "
                    "keys hashed into num_feature columns; device-resident CSR",
        }), flush=True)
    bsp.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
