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

A producer thread per file part does the reading, copying and parsing on
its own stream, a block or two ahead: the ingest ops release the GIL during
their single device read each, so the training loop keeps enqueueing work
meanwhile, and the main stream waits for a batch (event) only when it is
handed over (``DeviceBatch.to_main``).
"""
import os

import torch

from .. import _native
from ..utils import trace

def applies(fmt, path, device):
    """Device parsing is used for plain Criteo / libsvm files on a GPU worker,
    and CRB records (decoded on the host's reader threads) are shuffled and
    sliced into minibatches on the device (``WH_DEVICE_PARSE=0`` keeps the
    host path for both)."""
    if device.type != "cuda" or os.environ.get("WH_DEVICE_PARSE", "1") == "0":
        return False
    if fmt == "crb":
        return True
    return (fmt in ("criteo", "criteo_test", "libsvm")
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
    """A minibatch produced on a producer stream; ``to_main`` makes the
    current stream wait for it (event) and hands the tensors over."""

    __slots__ = ("args", "event")

    def __init__(self, args, event=None):
        self.args, self.event = args, event

    def to_main(self, dev):
        main = torch.cuda.current_stream(dev)
        if self.event is not None:
            main.wait_event(self.event)
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


_STREAM_POOL = {}


def _producer_stream(dev):
    """Producer streams, a small pool per device (one per live iterator in
    the usual prefetch depth)."""
    pool = _STREAM_POOL.setdefault(dev, [[], 0])
    if len(pool[0]) < 4:
        pool[0].append(torch.cuda.Stream(dev))
    pool[1] = (pool[1] + 1) % len(pool[0])
    return pool[0][pool[1]]


class DeviceTextIter:
    """Minibatches of one file part, parsed on the device (the
    ``_host.MinibatchIter`` contract: ``next()`` -> batch or None).

    A producer thread reads the part's text batches, copies them to the
    device and parses (and, with a shuffle buffer, permutes and gathers)
    them on its own stream, ``depth`` blocks ahead of the consumer; the
    parse ops release the GIL while they wait for their one device read, so
    ingest overlaps the training loop instead of running between its steps.
    """

    def __init__(self, host, path, part, nparts, fmt, mb, shuf, neg, seed, device, depth=2):
        import queue
        import threading
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.fmt, self.mb, self.neg, self.dev = fmt, mb, neg, device
        # a shuffle buffer is needed for negative sampling too (as on the host)
        self.shuffled = shuf > 0 or neg < 1.0
        # host reads stay minibatch-sized (pinned buffers are reused); a
        # shuffle buffer is assembled from several text batches on the device
        self.per_block = max(1, -(-max(shuf, mb + 1) // mb)) if self.shuffled else 1
        # CRB (binary records, LZ4 sections): the host's reader threads decode
        # the records in parallel (csrc/host/parsers.cc ThreadedReader) and a
        # copy pool assembles pinned CSR blocks of per_block minibatches, in
        # file order (csrc/host/registry.cc BlockIter); the
        # shuffle buffer, negative sampling and minibatch slicing then run on
        # the device exactly as for parsed text (the host shuffle was the
        # single-threaded bottleneck of CRB input: 4.9 M rows/s)
        # blocks go straight from the decoded records into pinned tensors,
        # copied by a thread pool (host.BlockIter; one copy per byte)
        self.blocks = fmt == "crb"
        if self.blocks:
            self.tb = host.BlockIter(path, part, nparts, fmt, int(mb * self.per_block), True)
        else:
            # several readers over line-aligned sub-ranges of the part, taken
            # round-robin in a fixed order (one reader thread copies ~7 GB/s
            # of page cache into pinned buffers: ~22 M Criteo rows/s). Only
            # behind a shuffle buffer: without one, the reference trains on
            # the part's rows in file order, mb rows per minibatch
            # (learn/base/minibatch_iter.h:75-121), and interleaved
            # sub-ranges would reorder them and cut a short minibatch at
            # every sub-range end.
            nsub = max(1, int(os.environ.get("WH_TEXT_READERS", "4"))) if self.shuffled else 1
            self.tbs = [host.TextBatches(path, part * nsub + j, nparts * nsub, mb, True)
                        for j in range(nsub)]
            self.tb_i = 0
        self.gen = None
        if self.shuffled:
            self.gen = torch.Generator(device=device)
            self.gen.manual_seed(int(seed) & 0x7FFFFFFFFFFFFFFF)
        self.stream = _producer_stream(device)
        self.q = queue.Queue(maxsize=max(1, depth))
        self.stop = False
        self.done = False
        self.cur = None  # shuffled: [keys, noff, val, label, cuts->offset, pos, n]
        self.th = threading.Thread(target=self._produce, daemon=True)
        self.th.start()

    # ---------------------------------------------------------- producer
    def _put(self, item):
        import queue
        while not self.stop:
            try:
                self.q.put(item, timeout=0.5)
                return True
            except queue.Full:
                continue
        return False

    def _produce(self):
        # WH_TIMING=ingest: the producer's seconds waiting for the readers,
        # working (copy / parse / shuffle), and blocked on a full queue
        timing = trace.timing_on("ingest")
        self.t_read = self.t_work = self.t_put = 0.0
        try:
            import time
            torch.cuda.set_device(self.dev)
            with torch.cuda.stream(self.stream):
                while not self.stop:
                    t0 = time.perf_counter()
                    self.t_read_blk = 0.0
                    item = self._block() if self.shuffled else self._minibatch()
                    t1 = time.perf_counter()
                    if item is None:
                        break
                    if not self._put(item):
                        return
                    self.t_read += self.t_read_blk
                    self.t_work += t1 - t0 - self.t_read_blk
                    self.t_put += time.perf_counter() - t1
        except BaseException as e:  # surfaced by the consumer
            self._put(e)
            return
        if timing:
            import sys
            print("[ingest] part producer: read wait %.3f s, work %.3f s, queue full %.3f s"
                  % (self.t_read, self.t_work, self.t_put), file=sys.stderr)
        self._put(None)

    def _csr_block(self, b):
        """A decoded host CSR block (pinned) -> device (keys, off, val, label)."""
        dev = self.dev
        keys, off, val, label = b[0], b[1], b[2], b[3]
        return (keys.to(dev, non_blocking=True), off.to(dev, non_blocking=True),
                val.to(dev, non_blocking=True) if val is not None and val.numel() else None,
                label.to(dev, non_blocking=True))

    def _text_next(self):
        """The next text batch from the sub-range readers, round-robin;
        None once all are exhausted."""
        import time
        t0 = time.perf_counter()
        try:
            return self._text_next_()
        finally:
            self.t_read_blk += time.perf_counter() - t0

    def _text_next_(self):
        while self.tbs:
            i = self.tb_i % len(self.tbs)
            b = self.tbs[i].next()
            if b is not None:
                self.tb_i = i + 1
                return b
            del self.tbs[i]
        return None

    def _minibatch(self):
        b = self.tb.next() if self.blocks else self._text_next()
        if b is None:
            return None
        if self.blocks:
            args = self._csr_block(b)
            ev = torch.cuda.Event()
            ev.record(self.stream)
            return DeviceBatch(args, ev)
        args = parse_block(b[0].to(self.dev, non_blocking=True), b[1], self.fmt)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return DeviceBatch(args, ev)

    def _block(self):
        """The next shuffle buffer: parsed, permuted and gathered into one CSR
        block whose consecutive slices are minibatches; host reads: the key
        count, the rows kept (negative sampling), the slice boundaries."""
        if self.blocks:  # one decoded block = one shuffle buffer
            b = self.tb.next()
            if b is None:
                return None
            keys, off, val, label = self._csr_block(b)
            lines = int(label.numel())
        else:
            texts, lines = [], 0
            for _ in range(self.per_block):
                b = self._text_next()
                if b is None:
                    break
                texts.append(b[0])
                lines += int(b[1])
            if not texts:
                return None
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
        noff = torch.zeros(n + 1, dtype=torch.int64, device=self.dev)
        torch.cumsum((off[1:] - off[:-1]).index_select(0, sel), 0, out=noff[1:])
        # the row offsets come to the host once (8 bytes per row): they size
        # the gather, and slices of any length are then views plus one
        # subtraction (the event wait releases the GIL)
        hoff = torch.empty(n + 1, dtype=torch.int64, pin_memory=True)
        hoff.copy_(noff, non_blocking=True)
        e0 = torch.cuda.Event()
        e0.record(self.stream)
        e0.synchronize()
        # (hoff stays a pinned tensor: a Python list of a shuffle buffer's
        # million offsets took the producer tens of ms under the GIL)
        pk, pv, pl = _native.hip().csr_gather(keys, off, val, label, sel, noff, int(hoff[n]))
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return [pk, noff, pv, pl, hoff, n, ev]

    # ---------------------------------------------------------- consumer
    def _get(self):
        if self.done:  # the producer's end marker was taken already
            return None
        item = self.q.get()
        if isinstance(item, BaseException):
            raise item
        if item is None:
            self.done = True
        return item

    def _slice(self, take):
        pk, noff, pv, pl, hoff, pos, n = self.cur
        a, b = int(hoff[pos]), int(hoff[pos + take])
        self.cur[5] = pos + take
        return (pk[a:b], noff[pos:pos + take + 1] - a, pv[a:b] if pv is not None else None,
                pl[pos:pos + take])

    def next(self):
        if not self.shuffled:
            return self._get()
        parts, need = [], self.mb
        while need > 0:
            if self.cur is None or self.cur[5] == self.cur[6]:
                blk = self._get()
                if blk is None:
                    self.cur = None
                    break
                main = torch.cuda.current_stream(self.dev)
                main.wait_event(blk[6])
                for x in blk[:4]:
                    if x is not None:
                        x.record_stream(main)
                self.cur = [blk[0], blk[1], blk[2], blk[3], blk[4], 0, blk[5]]
                continue
            take = min(need, self.cur[6] - self.cur[5])
            parts.append(self._slice(take))
            need -= take
        if not parts:
            return None
        return DeviceBatch(concat_blocks(parts))

    def close(self):
        self.stop = True

    def __del__(self):
        self.stop = True
