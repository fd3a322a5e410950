"""Minibatches of Criteo / libsvm text parsed on the GPU.

The reference worker parses every line on the host (learn/base/
criteo_parser.h:64-86, dmlc LibSVMParser) and draws minibatches through a
shuffle buffer with negative down-sampling (learn/base/minibatch_iter.h).
Here the host only reads file bytes: ``_host.TextBatches`` cuts the file part
into whole-line blocks in pinned memory (memchr, no parsing), and each block
is copied to the GPU and tokenized + hashed there (csrc/hip/ingest.hip:
newline scan, wave-per-line tokenizer, CityHash64) into a CSR block whose
keys are bit-identical to the host parsers' (tests/test_ingest.py).

With a shuffle buffer (``rand_shuffle`` > 0) a buffer holds
``minibatch * rand_shuffle`` lines, as the host iterator's does: their text
batches are copied into one device buffer and parsed at once, the rows are
permuted on the device (``torch.randperm`` with a seeded device generator),
negatives are kept with probability ``neg_sampling``, and the permuted rows
are gathered into one CSR block (``k_csr_gather``) whose consecutive slices
are the minibatches -- spanning buffer boundaries like the host iterator's.
Without a shuffle buffer, text batches are minibatches.

All device work runs on a per-device side stream: its host reads (the key
count of a block, the size of a gather) wait for that stream only, not for
the training step in flight on the main stream, which waits for the batch
when it is handed over (``DeviceBatch.to_main``).
"""
import os

import torch

from .. import _native

_STREAMS = {}


def _side(dev):
    s = _STREAMS.get(dev)
    if s is None:
        s = _STREAMS[dev] = torch.cuda.Stream(dev)
    return s


def applies(fmt, path, device):
    """Device parsing is used for plain Criteo / libsvm files on a GPU worker
    (``WH_DEVICE_PARSE=0`` keeps the host parsers)."""
    return (fmt in ("criteo", "criteo_test", "libsvm") and device.type == "cuda"
            and os.environ.get("WH_DEVICE_PARSE", "1") != "0"
            and not path.endswith((".gz", ".crb", ".rec"))
            and "://" not in path.replace("file://", ""))


def parse_block(text, lines, fmt):
    """Device text bytes of ``lines`` whole lines -> (keys, off, val, label)."""
    hip = _native.hip()
    if fmt == "libsvm":
        keys, label, off, val, _w = hip.parse_libsvm(text, int(lines))
        return keys, off, val, label
    keys, label, off = hip.parse_criteo(text, int(lines), fmt == "criteo")
    return keys, off, None, label


class DeviceBatch:
    """A minibatch produced on the side stream; ``to_main`` hands it to the
    current stream."""

    __slots__ = ("args", "text", "lines", "fmt")

    def __init__(self, args=None, text=None, lines=0, fmt=None):
        self.args, self.text, self.lines, self.fmt = args, text, lines, fmt

    def to_main(self, dev):
        side = _side(dev)
        if self.args is None:  # an unshuffled block: parsed when handed over
            with torch.cuda.stream(side):
                self.args = parse_block(self.text.to(dev, non_blocking=True), self.lines,
                                        self.fmt)
        main = torch.cuda.current_stream(dev)
        main.wait_stream(side)
        for x in self.args:
            if x is not None:
                x.record_stream(main)
        return self.args


def concat_blocks(parts):
    """CSR blocks (keys, off, val, label) -> one block."""
    if len(parts) == 1:
        return parts[0]
    keys = torch.cat([p[0] for p in parts])
    offs, base = [parts[0][1]], parts[0][1][-1:]
    for p in parts[1:]:
        offs.append(p[1][1:] + base)
        base = offs[-1][-1:]
    vals = None
    if any(p[2] is not None for p in parts):
        vals = torch.cat([p[2] if p[2] is not None else torch.ones_like(p[0], dtype=torch.float32)
                          for p in parts])
    return keys, torch.cat(offs), vals, torch.cat([p[3] for p in parts])


class DeviceTextIter:
    """Minibatches of one file part, parsed on the device (the
    ``_host.MinibatchIter`` contract: ``next()`` -> batch or None)."""

    def __init__(self, host, path, part, nparts, fmt, mb, shuf, neg, seed, device):
        self.fmt, self.mb, self.neg, self.dev = fmt, mb, neg, device
        # a shuffle buffer is needed for negative sampling too (as on the host)
        self.shuffled = shuf > 0 or neg < 1.0
        # host reads stay minibatch-sized (pinned buffers are reused); a
        # shuffle buffer is assembled from several parsed blocks on the device
        self.per_block = max(1, -(-max(shuf, mb + 1) // mb)) if self.shuffled else 1
        self.tb = host.TextBatches(path, part, nparts, mb, True)
        self.gen = None
        if self.shuffled:
            self.gen = torch.Generator(device=device)
            self.gen.manual_seed(int(seed) & 0x7FFFFFFFFFFFFFFF)
        self.cur = None  # (block, sel, pos)

    def _next_block(self, first):
        """Read, parse and permute the next shuffle buffer; ``first`` rows
        complete the minibatch begun in the previous buffer. Three host
        reads per buffer (key count, rows kept, minibatch boundaries)."""
        texts, lines = [], 0
        for _ in range(self.per_block):
            b = self.tb.next()
            if b is None:
                break
            texts.append(b[0])
            lines += int(b[1])
        if not texts:
            return False
        # the text batches go into one device buffer: one parse per buffer
        text = torch.empty(sum(t.numel() for t in texts), dtype=torch.uint8, device=self.dev)
        o = 0
        for t in texts:
            text[o:o + t.numel()].copy_(t, non_blocking=True)
            o += t.numel()
        keys, off, val, label = parse_block(text, lines, self.fmt)
        del text
        sel = torch.randperm(lines, generator=self.gen, device=self.dev)
        if self.neg < 1.0:
            r = torch.rand(lines, generator=self.gen, device=self.dev)
            keep = (label.index_select(0, sel) > 0) | (r <= self.neg)
            sel = sel[keep]
        n = sel.numel()
        # the permuted buffer as one CSR block: minibatches are slices of it
        noff = torch.zeros(n + 1, dtype=torch.int64, device=self.dev)
        torch.cumsum((off[1:] - off[:-1]).index_select(0, sel), 0, out=noff[1:])
        cuts = [0] + list(range(min(first, n), n, self.mb)) + [n]
        cuts = sorted(set(cuts))
        at = noff.index_select(0, torch.tensor(cuts, device=self.dev)).cpu().tolist()
        pk, pv, pl = _native.hip().csr_gather(keys, off, val, label, sel, noff, int(at[-1]))
        self.cur = [pk, noff, pv, pl, dict(zip(cuts, at)), 0, n]
        return True

    def _slice(self, take):
        pk, noff, pv, pl, at, pos, n = self.cur
        a, b = at[pos], at[pos + take]
        self.cur[5] = pos + take
        return (pk[a:b], noff[pos:pos + take + 1] - a, pv[a:b] if pv is not None else None,
                pl[pos:pos + take])

    def next(self):
        if not self.shuffled:
            b = self.tb.next()
            return None if b is None else DeviceBatch(text=b[0], lines=b[1], fmt=self.fmt)
        with torch.cuda.stream(_side(self.dev)):
            parts, need = [], self.mb
            while need > 0:
                if self.cur is None or self.cur[5] == self.cur[6]:
                    if not self._next_block(need):
                        break
                    continue
                take = min(need, self.cur[6] - self.cur[5])
                parts.append(self._slice(take))
                need -= take
            if not parts:
                return None
            return DeviceBatch(args=concat_blocks(parts))
