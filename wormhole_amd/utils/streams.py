"""Cheap stream switching for the per-minibatch host path.

``torch.cuda.current_stream(dev)`` / ``torch.cuda.stream(s)`` /
``Stream.wait_stream`` each resolve the device through several Python layers
(environment lookups included) or create a fresh event; a multi-shard step
made ~30 such calls, ~100 us of host time per minibatch. These helpers call
the C entry points directly and reuse events from a ring.
"""
import torch

_get = torch._C._cuda_getCurrentStream
_set = torch._C._cuda_setStream
_getdev = torch._C._cuda_getDevice


def current_id(device_index):
    """Id of the current stream of a device (compare with ``Stream.stream_id``);
    ``None``: the current device."""
    if device_index is None:
        device_index = torch.cuda.current_device()
    return _get(device_index)[0]


class on:
    """``with on(stream):`` -- make ``stream`` current, restore the previous
    current stream of its device on exit. Setting a stream also makes its
    device current; like ``torch.cuda.stream``, the caller's current device
    is restored too when it was a different one (one device per process is
    the usual case, where this costs one integer compare)."""

    __slots__ = ("s", "prev", "dev")

    def __init__(self, s):
        self.s = s
        self.prev = None
        self.dev = None

    def __enter__(self):
        s = self.s
        cur = _getdev()
        self.dev = cur if cur != s.device_index else None
        self.prev = _get(s.device_index)
        _set(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type)
        return s

    def __exit__(self, *exc):
        p = self.prev
        _set(stream_id=p[0], device_index=p[1], device_type=p[2])
        if self.dev is not None:
            torch.cuda.set_device(self.dev)
        return False


class EventRing:
    """Reusable events: an event may be re-recorded once the stream waits on
    its previous record are enqueued (they capture the record they saw)."""

    __slots__ = ("ev", "i")

    def __init__(self, n=32):
        self.ev = [torch.cuda.Event() for _ in range(n)]
        self.i = 0

    def record(self, stream):
        ev = self.ev[self.i]
        self.i = (self.i + 1) % len(self.ev)
        ev.record(stream)
        return ev

    def wait(self, waiter, producer):
        """``waiter`` waits for everything queued on ``producer`` so far."""
        waiter.wait_event(self.record(producer))
