"""bin/kmeans.dmlc: ``<data_path> <num_cluster> <max_iter> <out_model>``
(reference learn/kmeans/kmeans.cc:132-220)."""
import sys

import torch

from .ps_app import _device


def main(argv):
    from .. import _native
    from ..models.kmeans import KMeans, KMeansCSR, densify, use_sparse
    from ..parallel.bsp import BSP, fault_point

    dev = _device()
    bsp = BSP(dev, job="kmeans")
    if len(argv) < 4:
        bsp.tracker_print("Usage: <data_path> num_cluster max_iter <out_model>")
        return 0
    k, max_iter, out = int(argv[1]), int(argv[2]), argv[3]
    keys, off, val, _lab, _w = _native.host().load_split(argv[0], bsp.rank, bsp.world, "libsvm")
    version, g, _ = bsp.load_checkpoint()
    if version == 0:
        fdim = int(keys.max().item()) + 1 if keys.numel() else 0
        fdim = int(bsp.allreduce_scalar(fdim, "max", torch.int64))
    else:
        fdim = int(g["centroids"].shape[1])
    nrows = off.numel() - 1
    # sparse or dense, decided together (every rank must run the same path)
    sparse = bsp.allreduce_scalar(1.0 if use_sparse(nrows, fdim, keys.numel()) else 0.0,
                                  "max") > 0
    if sparse:
        km = KMeansCSR(bsp, keys, off, val, fdim, k, dev)
    else:
        km = KMeans(bsp, densify(keys, off, val, nrows, fdim, dev), k)
    if version == 0:
        km.init_centroids(0)
    else:
        km.C = g["centroids"].to(dev)
    for r in range(version, max_iter):
        km.step()
        km.flush_warnings()  # this iteration's empty-cluster warning, in order
        v = bsp.lazy_checkpoint({"centroids": km.C.cpu()})
        fault_point(bsp.rank, v)
        bsp.tracker_print("Finish %d-th iteration" % r)
    if bsp.rank == 0:
        km.save_text(out)
        bsp.tracker_print("All iteration finished, centroids saved to %s" % out)
    bsp.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
