"""Autograd over the native Engine: the data-parallel NT-Xent with a C++ host path.

``parallel.symmetric`` / ``parallel.distributed`` drive the stage kernels from Python and
exchange rows through ``torch.distributed``: every step issues dozens of Python-level calls
(tensor slicing, ``batch_isend_irecv`` op lists, per-step allocations). On the round-5 one-GPU
RCCL rehearsals that cost 1.4 ms of host time per step at W = 2 and 4.9 ms at W = 8 for the
symmetric mode (``profiles/r5/w8_full``), against a GPU step of ~1-3 ms: the step could be
host-bound on the node. The native ``ntxent::Engine`` (``csrc/runtime/engine*.cpp``) runs the
same launch sequence, the same tile lists and the same point-to-point exchanges from C++ (one
``ncclGroupStart/End`` per exchange, all buffers in one arena sized once), so a step is two
Python calls.

This module puts that engine behind ``torch.autograd``:

* one :class:`~ntxent_amd._C.RcclCommunicator` per (process group, device), bootstrapped once
  through the group (rank 0's RCCL unique id broadcast with ``broadcast_object_list``) and shared
  by the engines of every shape;
* one engine per (rows, dim, temperature, dtype, compute, negatives, keep_cos) on that
  communicator, cached;
* :class:`EngineNTXentFunction`: forward = ``engine.forward(h)`` (the global mean loss), backward
  = ``engine.backward(grad_out)`` (the gradient of the global loss w.r.t. this rank's rows), the
  same value and gradient as :func:`parallel.distributed.dist_ntxent_loss`.

An engine holds the state of ONE forward (its cosines, LSE and partials live in its arena), so a
second forward through the same engine before the first one's backward makes that backward
raise instead of returning a wrong gradient (generation check).

No reference counterpart: the reference links MPI / NCCL in CMake and never calls them
(``/root/reference/CMakeLists.txt:13-14,41-47,115-121``).
"""
from __future__ import annotations

import threading
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops import _ext

_DT = {torch.float32: "fp32", torch.float16: "fp16", torch.bfloat16: "bf16"}
_lock = threading.Lock()
_COMMS: Dict[tuple, object] = {}
_ENGINES: Dict[tuple, "_Slot"] = {}


def _group_key(group) -> tuple:
    ranks = tuple(dist.get_process_group_ranks(group)) if group is not None else tuple(range(dist.get_world_size()))
    return (id(group) if group is not None else None, ranks)


def group_communicator(group=None, device: Optional[int] = None):
    """The process group's shared RCCL communicator on ``device`` (created on first use: a
    collective call, every rank of the group must make it)."""
    C = _ext.load()
    dev = torch.cuda.current_device() if device is None else int(device)
    key = (_group_key(group), dev)
    with _lock:
        comm = _COMMS.get(key)
    if comm is not None:
        return comm
    W, r = dist.get_world_size(group), dist.get_rank(group)
    obj = [C.rccl_unique_id() if r == 0 else None]
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast_object_list(obj, src=src, group=group)
    comm = C.RcclCommunicator(r, W, obj[0], dev)
    with _lock:
        _COMMS[key] = comm
    return comm


class _Slot:
    """An engine plus the generation of the forward whose state it holds."""

    __slots__ = ("engine", "gen")

    def __init__(self, engine):
        self.engine = engine
        self.gen = 0


def engine_for(rows: int, dim: int, temperature: float, dtype: torch.dtype, compute: str, negatives: str,
               keep_cos: bool, group=None, device: Optional[int] = None, comm_reserve_cus: int = 8) -> _Slot:
    """The cached engine slot for this shape on the group's communicator."""
    if dtype not in _DT:
        raise TypeError(f"engine path: dtype must be one of {list(_DT)}")
    C = _ext.load()
    dev = torch.cuda.current_device() if device is None else int(device)
    key = (_group_key(group), dev, int(rows), int(dim), float(temperature), dtype, compute, negatives, bool(keep_cos),
           int(comm_reserve_cus))
    with _lock:
        slot = _ENGINES.get(key)
    if slot is not None:
        return slot
    comm = group_communicator(group, dev)
    eng = C.NativeEngine(int(rows), int(dim), float(temperature), _DT[dtype], compute, negatives, comm.rank, comm.world,
                         b"", dev, bool(keep_cos), int(comm_reserve_cus), comm)
    slot = _Slot(eng)
    with _lock:
        _ENGINES[key] = slot
    return slot


def release_engines() -> None:
    """Drop every cached engine and communicator (frees their arenas; call before
    ``destroy_process_group`` to tear RCCL down in order)."""
    with _lock:
        _ENGINES.clear()
        _COMMS.clear()


def cached_engine_bytes() -> int:
    """Device bytes held by the cached engines' arenas (outside torch's allocator)."""
    with _lock:
        return sum(s.engine.device_bytes for s in _ENGINES.values())


class EngineNTXentFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h: torch.Tensor, slot: _Slot):
        slot.gen += 1
        slot.engine.forward(h)
        ctx.slot, ctx.gen = slot, slot.gen
        ctx.mark_non_differentiable()
        return slot.engine.loss_tensor()

    @staticmethod
    def backward(ctx, grad_out: torch.Tensor):
        slot = ctx.slot
        if slot.gen != ctx.gen:
            raise RuntimeError("engine NT-Xent: another forward of the same shape ran on this engine before this "
                               "backward (an engine holds one forward's state); call backward first, or use "
                               "dist_ntxent_loss(..., impl='torch')")
        return slot.engine.backward(grad_out), None


def engine_eligible(h: torch.Tensor, group, negatives: str, backward_mode: str = "symmetric",
                    overlap: bool = True) -> Tuple[bool, str]:
    """(ok, reason): whether :func:`engine_ntxent_loss` can run this call."""
    if not h.is_cuda:
        return False, "CPU tensor"
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) < 2:
        return False, "world size 1"
    if dist.get_backend(group) != "nccl":
        return False, f"backend {dist.get_backend(group)} (the engine talks RCCL)"
    if negatives not in ("symmetric", "allgather"):
        return False, f"negatives={negatives}"
    if backward_mode != "symmetric":
        return False, f"backward_mode={backward_mode}"
    if not overlap:
        return False, "overlap=False"
    if h.dtype not in _DT or h.dim() != 2:
        return False, f"dtype {h.dtype}"
    return True, ""


def engine_ntxent_loss(h_local: torch.Tensor, temperature: float, *, group=None, compute: str = "fp16",
                       negatives: str = "symmetric", keep_logits: bool = True, comm_reserve_cus: int = 8) -> torch.Tensor:
    """Global NT-Xent over ``group`` on the native engine (see the module docstring);
    ``compute`` is a resolved compute dtype (``ops.ntxent.resolve_compute``)."""
    h = h_local.contiguous()
    slot = engine_for(h.shape[0], h.shape[1], temperature, h.dtype, compute, negatives, keep_logits, group,
                      h.device.index, comm_reserve_cus)
    return EngineNTXentFunction.apply(h, slot)
