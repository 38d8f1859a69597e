"""A direct RCCL communicator for the step's gradient collective.

torch.distributed's ProcessGroupNCCL launches every collective on an internal stream of its own: the
caller's stream records an event, the internal stream waits for it, RCCL runs, and the caller's
stream waits back.  In the pipelined language step (langsplat_amd.pipeline) that round trip sits on
the critical stream between the backward and the update: measured on one rank at C3, ~10 us of idle
stream before the collective and ~13 us after it (profiles/r06_direct_rccl.txt), plus ~70 us of host
time per call.

Communicator builds an RCCL communicator over the ranks of a torch.distributed group (the unique id
goes through the group once, at construction) and enqueues ncclAllReduce on the CALLER's stream: the
reduce then follows the backward's last kernel as any other launch on that stream.  It is the same
RCCL library torch links (torch/lib/librccl.so, found through torch's own load), over the same xGMI
links; torch.distributed stays the bootstrap and the barrier.  Inside a HIP graph capture the
launch is captured on the capturing stream itself (no fork / join branch).

The step's reductions use it by default when the group's backend is "nccl" (distributed.GradBucket;
LSR_DIRECT_RCCL=0 keeps torch.distributed.all_reduce).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import torch
import torch.distributed as dist

_NCCL_FLOAT32 = 7          # ncclFloat32 (rccl.h ncclDataType_t)
_OPS = {"sum": 0, "max": 2, "avg": 4}  # ncclSum, ncclMax, ncclAvg (rccl.h ncclRedOp_t)


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]  # NCCL_UNIQUE_ID_BYTES


_lib = None


def _load():
    """torch's own librccl.so (already mapped by its HIP backend): one RCCL in the process."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    if not os.path.exists(path):
        path = "librccl.so"
    lib = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
    lib.ncclCommInitRank.argtypes = [ctypes.POINTER(vp), ctypes.c_int, _UniqueId, ctypes.c_int]
    lib.ncclAllReduce.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, vp, vp]
    lib.ncclCommDestroy.argtypes = [vp]
    lib.ncclGetErrorString.argtypes = [ctypes.c_int]
    lib.ncclGetErrorString.restype = ctypes.c_char_p
    for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclCommDestroy", "ncclGroupStart",
              "ncclGroupEnd"):
        getattr(lib, f).restype = ctypes.c_int
    _lib = lib
    return lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = _load().ncclGetErrorString(rc)
        raise RuntimeError(f"RCCL {what} failed: {msg.decode() if msg else rc}")


class Communicator:
    """An RCCL communicator over the ranks of `group` (default: the world), on the current device.
    Collective over the group: every rank constructs it at the same point."""

    def __init__(self, group=None, device: Optional[torch.device] = None):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("rccl.Communicator: torch.distributed is not initialised")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        lib = _load()
        uid = _UniqueId()
        if self.rank == 0:
            _check(lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        box = [ctypes.string_at(ctypes.byref(uid), 128) if self.rank == 0 else None]  # all 128 bytes (NULs too)
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        uid = _UniqueId()
        ctypes.memmove(ctypes.byref(uid), box[0], 128)
        self._comm = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _check(lib.ncclCommInitRank(ctypes.byref(self._comm), self.world, uid, self.rank), "ncclCommInitRank")

    def all_reduce(self, tensors: Sequence[torch.Tensor], op: str = "sum", stream=None):
        """In place, one RCCL group over the tensors (contiguous fp32 on this device), on `stream`
        (default: the current stream)."""
        if self._comm is None:
            raise RuntimeError("rccl.Communicator: destroyed")
        lib = _load()
        s = torch.cuda.current_stream(self.device) if stream is None else stream
        for t in tensors:
            if t.dtype != torch.float32 or not t.is_contiguous() or t.device != self.device:
                raise ValueError("rccl.Communicator.all_reduce: contiguous fp32 tensors on the communicator's device")
        _check(lib.ncclGroupStart(), "ncclGroupStart")
        try:
            for t in tensors:
                _check(lib.ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), _NCCL_FLOAT32, _OPS[op], self._comm,
                                         s.cuda_stream), "ncclAllReduce")
        finally:
            _check(lib.ncclGroupEnd(), "ncclGroupEnd")

    def destroy(self):
        """Free the communicator (after the device finished its collectives: call after a synchronize)."""
        if self._comm is not None and self._comm.value:
            _load().ncclCommDestroy(self._comm)
        self._comm = None


_default: Optional[Communicator] = None
_failed: Optional[str] = None  # why the direct communicator could not be built (then torch's path is used)


def direct_enabled(group=None) -> bool:
    """The direct communicator is used for a group whose backend is "nccl" unless LSR_DIRECT_RCCL=0
    (or it failed to build on this process)."""
    return (_failed is None and os.environ.get("LSR_DIRECT_RCCL", "1") != "0" and dist.is_available()
            and dist.is_initialized() and dist.get_backend(group) == "nccl")


def default_communicator() -> Optional[Communicator]:
    """The world's direct communicator, built on first use (a collective: every rank's first
    GradBucket reduction happens at the same point of the step).  None if it could not be built
    (e.g. the library lacks a symbol: every rank fails alike and keeps torch.distributed's path)."""
    global _default, _failed
    if _default is None and _failed is None:
        try:
            _default = Communicator()
        except (OSError, AttributeError, RuntimeError) as e:  # noqa: PERF203
            _failed = f"{type(e).__name__}: {e}"
    return _default


def destroy_default():
    global _default
    if _default is not None:
        _default.destroy()
        _default = None
