"""wormhole_amd: an MI355X-native distributed classic-ML toolkit with the
capabilities of DMLC wormhole (linear async SGD/FTRL, DiFacto FM, L-BFGS,
k-means, GBDT) on PyTorch-ROCm tensors, hand-written gfx950 HIP kernels and
RCCL over xGMI."""
__version__ = "0.1.0"

import os as _os

# Kernel arguments in device memory (a HIP runtime switch, read when the
# runtime initialises, so it is set here, before the first GPU call): the
# launch-bound small-minibatch steps gain 8-28 % (the reference tutorial's
# dim 16 / minibatch 1000: 6.7 -> 7.3-8.6 M ex/s), the headline 0.2-0.7 %
# (profiles/round6_small_minibatch_host.txt). An explicit setting wins.
_os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
