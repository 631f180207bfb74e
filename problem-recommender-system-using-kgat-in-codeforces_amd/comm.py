"""The library's own RCCL transport (kgat_comm_* in include/kgat_hip.h).

``RcclComm`` is a drop-in for ``sharded.Comm`` (the all-peer row gather ``gather_v``, the
refresh's ``all_to_all_v``, ``all_reduce_``, ``all_gather``, the ring ``exchange``) plus the
row-block ``reduce_scatter_rows`` / ``all_gather_rows`` of the data-parallel exchange, with
every collective issued by libkgat_hip.so on an RCCL communicator it owns -- the path a host
without torch.distributed uses.  The reference has
no counterpart (single device, src/model/KGAT/main.py:239).

Overlap: each collective runs on the communicator's own HIP stream, ordered after the work
already queued on the caller's stream (event), and ``wait()`` makes the caller's stream wait
for it -- so the ring's next-shard transfer proceeds under the current block's SpMM, as with
torch's RCCL backend.  The process holds one RCCL instance: the library binds torch's bundled
RCCL when there is one (kgat_comm_load), else the system's librccl.so.1.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

from . import _lib

_LOADED = False


class WireLog:
    """Bytes this rank puts on the wire, by phase (the row-sharded CF step sets ``phase`` to "forward" /
    "backward"; everything else counts as "other").  Counted per collective from its shapes, the same rule
    for every transport: a row gather sends this rank's rows to each of the G-1 peers, a ring all-reduce
    2 (G-1) / G of the buffer, an all-gather (G-1) copies of this rank's part, an all-to-all the blocks
    addressed to peers.  The bench reports it as ``wire_bytes_per_step``."""

    def __init__(self):
        self.phase = "other"
        self.bytes: dict[str, int] = {}

    def add(self, nbytes: int) -> None:
        if nbytes > 0:
            self.bytes[self.phase] = self.bytes.get(self.phase, 0) + int(nbytes)

    def reset(self) -> None:
        self.bytes = {}


def wire(comm) -> WireLog:
    """The comm object's WireLog (created on first use)."""
    w = comm.__dict__.get("_wire")
    if w is None:
        w = comm.__dict__["_wire"] = WireLog()
    return w


def count_gather(comm, out: torch.Tensor, n_own: int) -> None:
    """A row gather / block post: this rank's n_own rows of ``out`` to each of the G-1 peers."""
    if comm.world > 1 or getattr(comm, "counts_as", 0) > 1:
        g = max(comm.world, getattr(comm, "counts_as", 0))
        wire(comm).add(int(n_own) * out.stride(0) * out.element_size() * (g - 1))


def count_all_reduce(comm, t: torch.Tensor) -> None:
    g = max(comm.world, getattr(comm, "counts_as", 0))
    if g > 1:
        wire(comm).add(2 * (g - 1) * t.numel() * t.element_size() // g)


def count_all_gather(comm, t: torch.Tensor) -> None:
    g = max(comm.world, getattr(comm, "counts_as", 0))
    if g > 1:
        wire(comm).add((g - 1) * t.numel() * t.element_size())


def _load_rccl() -> None:
    global _LOADED
    if _LOADED:
        return
    bundled = Path(torch.__file__).resolve().parent / "lib" / "librccl.so"
    path = os.environ.get("KGAT_RCCL_LIB") or (str(bundled) if bundled.exists() else None)
    _lib.call("kgat_comm_load", path.encode() if path else None)
    _LOADED = True


def unique_id() -> bytes:
    _load_rccl()
    buf = (ctypes.c_uint8 * _lib.KGAT_COMM_ID_BYTES)()
    _lib.call("kgat_comm_unique_id", buf)
    return bytes(buf)


class _Done:
    def __init__(self, event: torch.cuda.Event, device: torch.device):
        self._event, self._device = event, device

    def wait(self) -> None:
        """The caller's stream waits for the collective (no host synchronisation)."""
        torch.cuda.current_stream(self._device).wait_event(self._event)


class RcclComm:
    """A communicator of ``world`` ranks (one per GPU) made by kgat_comm_init."""

    def __init__(self, rank: int, world: int, uid: bytes, device: torch.device | int, force: bool = False):
        """``uid``: rank 0's unique_id(), shared out of band (``from_process_group`` uses the
        torch.distributed store).  ``force``: collectives run even on a world of one rank."""
        _load_rccl()
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.rank, self.world = int(rank), int(world)
        self.force = bool(force)
        self.host = False
        self.group = None
        self.next = (self.rank + 1) % self.world
        self.prev = (self.rank - 1) % self.world
        if len(uid) != _lib.KGAT_COMM_ID_BYTES:
            raise ValueError("uid must be unique_id()'s bytes")
        handle = ctypes.c_void_p()
        idbuf = (ctypes.c_uint8 * _lib.KGAT_COMM_ID_BYTES).from_buffer_copy(uid)
        _lib.call("kgat_comm_init", self.rank, self.world, idbuf, self.device.index or 0, ctypes.byref(handle))
        self._h = handle
        self._side = torch.cuda.Stream(device=self.device)

    @classmethod
    def from_process_group(cls, device, group=None, force: bool = False) -> "RcclComm":
        """One communicator over the ranks of a torch.distributed group (the id travels by broadcast)."""
        import torch.distributed as dist

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        box = [unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                       group=group)
        return cls(rank, world, box[0], device, force=force)

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            torch.cuda.synchronize(self.device)
            _lib.call("kgat_comm_destroy", self._h)
            self._h = None

    def __del__(self):  # noqa: D105
        try:
            self.close()
        except Exception:  # noqa: BLE001  (interpreter teardown)
            pass

    # ---------------------------------------------------------------- plumbing
    def _begin(self, *tensors: torch.Tensor) -> int:
        """Order the side stream after the caller's queued work; return its handle."""
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._side.wait_event(ev)
        for t in tensors:
            if t.is_cuda:
                t.record_stream(self._side)
        return self._side.cuda_stream

    def _end(self) -> _Done:
        ev = torch.cuda.Event()
        ev.record(self._side)
        return _Done(ev, self.device)

    @staticmethod
    def _check(t: torch.Tensor, name: str) -> None:
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError(f"{name}: a contiguous GPU tensor is required")

    @property
    def active(self) -> bool:
        """Collectives move data (more than one rank, or forced at world 1)."""
        return self.world > 1 or self.force

    # ------------------------------------------------------------ collectives
    def gather_v(self, send: torch.Tensor, out: torch.Tensor, bounds) -> _Done:
        """All-peer row gather (kgat_comm_allgatherv): rank r's rows land in out[bounds[r]:bounds[r+1]];
        ``send`` = this rank's rows (may be that slice of ``out``).  wait() orders the caller after it."""
        self._check(out, "out")
        self._check(send, "send")
        row = out.stride(0) * out.element_size()
        offs = (ctypes.c_int64 * (self.world + 1))(*[int(b) * row for b in bounds])
        count_gather(self, out, int(bounds[self.rank + 1]) - int(bounds[self.rank]))
        st = self._begin(send, out)
        _lib.call("kgat_comm_allgatherv", self._h, send.data_ptr(), out.data_ptr(), offs, st)
        return self._end()

    def gather_at(self, send: torch.Tensor, out: torch.Tensor, starts, sizes) -> _Done:
        """Rank r's ``sizes[r]`` rows land in out[starts[r]:starts[r] + sizes[r]] (kgat_comm_gather_at);
        ``send`` = this rank's rows.  The pipelined row-sharded forward's block post."""
        self._check(out, "out")
        row = out.stride(0) * out.element_size()
        offs = (ctypes.c_int64 * self.world)(*[int(a) * row for a in starts])
        nb = (ctypes.c_int64 * self.world)(*[int(z) * row for z in sizes])
        if int(sizes[self.rank]):
            self._check(send, "send")
        count_gather(self, out, int(sizes[self.rank]))
        st = self._begin(send, out)
        _lib.call("kgat_comm_gather_at", self._h, send.data_ptr() if int(sizes[self.rank]) else None, out.data_ptr(),
                  offs, nb, st)
        return self._end()

    def all_to_all_v(self, send: torch.Tensor, send_off, recv: torch.Tensor, recv_off) -> None:
        """send[send_off[p]:send_off[p+1]] -> rank p, rank p's block -> recv[recv_off[p]:...] (1-D,
        element offsets; kgat_comm_alltoallv); the caller's stream is ordered after it."""
        self._check(send, "send")
        self._check(recv, "recv")
        es = send.element_size()
        so = (ctypes.c_int64 * (self.world + 1))(*[int(x) * es for x in send_off])
        ro = (ctypes.c_int64 * (self.world + 1))(*[int(x) * es for x in recv_off])
        wire(self).add(es * (int(send_off[-1]) - int(send_off[0]) - (int(send_off[self.rank + 1]) -
                                                                      int(send_off[self.rank]))))
        st = self._begin(send, recv)
        _lib.call("kgat_comm_alltoallv", self._h, send.data_ptr(), so, recv.data_ptr(), ro, st)
        self._end().wait()

    def exchange(self, send: torch.Tensor, recv: torch.Tensor) -> _Done:
        """Start: send -> next rank, prev rank -> recv (kgat_comm_ring_exchange).  wait() completes both."""
        self._check(send, "send")
        self._check(recv, "recv")
        nbytes = send.numel() * send.element_size()
        if recv.numel() * recv.element_size() != nbytes:
            raise ValueError("exchange: send and recv sizes differ")
        wire(self).add(nbytes)
        st = self._begin(send, recv)
        _lib.call("kgat_comm_ring_exchange", self._h, send.data_ptr(), recv.data_ptr(), nbytes, st)
        return self._end()

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over ranks (fp32)."""
        if self.world == 1 and not self.force:
            return t
        self._check(t, "t")
        if t.dtype != torch.float32:
            raise ValueError("all_reduce_: fp32 only")
        count_all_reduce(self, t)
        st = self._begin(t)
        _lib.call("kgat_comm_allreduce_sum_f32", self._h, t.data_ptr(), t.data_ptr(), t.numel(), st)
        self._end().wait()
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape], rank order."""
        if self.world == 1 and not self.force:
            return t.unsqueeze(0)
        t = t.contiguous()
        self._check(t, "t")
        out = torch.empty((self.world, *t.shape), dtype=t.dtype, device=t.device)
        count_all_gather(self, t)
        st = self._begin(t, out)
        _lib.call("kgat_comm_allgather_rows", self._h, t.data_ptr(), out.data_ptr(), t.numel() * t.element_size(), st)
        self._end().wait()
        return out

    def all_gather_rows_(self, full: torch.Tensor) -> torch.Tensor:
        """In place: rank k's block full[k*s:(k+1)*s] (s = rows // world) to every rank."""
        self._check(full, "full")
        s = full.shape[0] // self.world
        own = full[self.rank * s:(self.rank + 1) * s]
        st = self._begin(full)
        _lib.call("kgat_comm_allgather_rows", self._h, own.data_ptr(), full.data_ptr(),
                  own.numel() * own.element_size(), st)
        self._end().wait()
        return full

    def reduce_scatter_rows(self, full: torch.Tensor) -> torch.Tensor:
        """The sum over ranks of block k of ``full`` (fp32, rows // world rows), on rank k, in place."""
        self._check(full, "full")
        if full.dtype != torch.float32:
            raise ValueError("reduce_scatter_rows: fp32 only")
        s = full.shape[0] // self.world
        own = full[self.rank * s:(self.rank + 1) * s]
        st = self._begin(full)
        _lib.call("kgat_comm_reduce_scatter_rows_f32", self._h, full.data_ptr(), own.data_ptr(), own.numel(), st)
        self._end().wait()
        return own
