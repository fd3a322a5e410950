"""wormhole_amd: an MI355X-native distributed classic-ML toolkit with the
capabilities of DMLC wormhole (linear async SGD/FTRL, DiFacto FM, L-BFGS,
k-means, GBDT) on PyTorch-ROCm tensors, hand-written gfx950 HIP kernels and
RCCL over xGMI."""
__version__ = "0.1.0"
