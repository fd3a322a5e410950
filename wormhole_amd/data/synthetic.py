"""Synthetic data shapes used by benchmarks and tests.

CRITEO_TB_CARD: per-field value cardinalities of the Criteo 1TB click log
(13 integer fields bucketised + the 26 categorical fields' well-known counts).
"""
import torch

from .. import _native

CRITEO_INT_CARD = [64, 3000, 2000, 500, 200000, 10000, 3000, 500, 6000, 20, 200, 1000, 600]
CRITEO_CAT_CARD = [39884406, 39043, 17289, 7420, 20263, 3, 7120, 1543, 63, 38532951,
                   2953546, 403346, 10, 2208, 11938, 155, 4, 976, 14, 39979771, 25641295,
                   39664984, 585935, 12972, 108, 36]
CRITEO_TB_CARD = CRITEO_INT_CARD + CRITEO_CAT_CARD


def criteo_batch(nrows, seed, step, device, card=None):
    """(keys int64[nrows*39], label f32[nrows], offset int64[nrows+1]) on device."""
    card_t = torch.tensor(card or CRITEO_TB_CARD, dtype=torch.int64, device=device)
    if card_t.is_cuda:
        return _native.hip().synth_criteo(nrows, seed, step, card_t)
    return criteo_batch_cpu(nrows, seed, step, card or CRITEO_TB_CARD)


def criteo_batch_cpu(nrows, seed, step, card):
    """CPU twin of the device generator (same distribution, numpy RNG)."""
    import numpy as np
    rng = np.random.default_rng([seed, step])
    nf = len(card)
    u = rng.random((nrows, nf))
    c = np.array(card, dtype=np.float64)
    rank = np.clip(np.exp(np.log(c) * u).astype(np.int64) - 1, 0, c.astype(np.int64) - 1)
    f = np.arange(nf, dtype=np.uint64)
    with np.errstate(over="ignore"):
        tok = (rank.astype(np.uint64) * np.uint64(0x9e3779b97f4a7c15)) ^ (f << np.uint64(40))
        keys = (tok >> np.uint64(10)) | (f << np.uint64(54))
    th = ((rank * 2654435761 + np.arange(nf) * 97) % 1000) / 1000.0 - 0.5
    logit = -1.2 + 0.9 * th.sum(1)
    label = (rng.random(nrows) < 1 / (1 + np.exp(-logit))).astype(np.float32)
    offset = np.arange(nrows + 1, dtype=np.int64) * nf
    return (torch.from_numpy(keys.reshape(-1).view(np.int64).copy()), torch.from_numpy(label),
            torch.from_numpy(offset))
