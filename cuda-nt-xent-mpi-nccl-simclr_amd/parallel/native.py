"""The native C++ runtime (``ntxent::Engine`` + ``ntxent::RcclComm``) driven from Python.

``csrc/include/ntxent/engine.h`` is the libtorch-free runtime behind ``build/bin/ntxent_bench``
and the C++ tests. It uses one arena allocation per shape and a fixed launch sequence, so a
whole fwd+bwd step can be captured in a hipGraph. At world size > 1 it does data parallelism
through its own RCCL communicator, in the symmetric or all-gather negatives mode. This module
exposes it to torch users:

* ``NativeNTXent(rows, dim)``: one GPU. ``step(h)`` returns ``(loss, dh)`` for the
  ``[view1; view2]`` rows ``h``. ``capture(h)`` / ``replay()`` replays a step from a hipGraph.
* ``NativeNTXent.from_process_group(rows, dim)``: one rank per process. The RCCL unique id is
  made on rank 0 and broadcast through the torch.distributed store. The
  engine then runs its own RCCL communicator, outside torch's ProcessGroup.

Unlike ``ntxent_loss`` this path has no autograd graph: ``dh`` is the gradient of the global mean
loss w.r.t. this rank's rows (times ``grad_out`` if given). Replaces the reference's
``ntxent_forward_cuda`` / ``ntxent_backward_cuda`` host functions
(``/root/reference/src/ntxent_kernel.cu:138-239``) for C++-style callers.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ..ops import _ext

_DT = {torch.float32: "fp32", torch.float16: "fp16", torch.bfloat16: "bf16"}


class NativeNTXent:
    """Fused NT-Xent forward + backward on the native Engine (see module docstring)."""

    def __init__(self, rows: int, dim: int, temperature: float = 0.07, *, dtype: torch.dtype = torch.bfloat16,
                 compute: str = "auto", negatives: str = "symmetric", device: Optional[int] = None,
                 keep_cos: bool = True, comm_reserve_cus: int = 8, rank: int = 0, world: int = 1,
                 uid: bytes = b""):
        if dtype not in _DT:
            raise TypeError(f"dtype must be one of {list(_DT)}")
        C = _ext.load()
        dev = torch.cuda.current_device() if device is None else int(device)
        self.rows, self.dim, self.temperature, self.dtype = int(rows), int(dim), float(temperature), dtype
        self.device = torch.device("cuda", dev)
        self._e = C.NativeEngine(self.rows, self.dim, self.temperature, _DT[dtype], compute, negatives, int(rank),
                                 int(world), uid, dev, bool(keep_cos), int(comm_reserve_cus))

    @classmethod
    def from_process_group(cls, rows: int, dim: int, temperature: float = 0.07, *, group=None, **kw) -> "NativeNTXent":
        """One engine per rank of ``group``, each with an RCCL communicator of its own over the same
        ranks (bootstrapped through the torch.distributed store)."""
        import torch.distributed as dist

        W = dist.get_world_size(group)
        r = dist.get_rank(group)
        if W == 1:
            return cls(rows, dim, temperature, **kw)
        obj = [_ext.load().rccl_unique_id() if r == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=group)
        return cls(rows, dim, temperature, rank=r, world=W, uid=obj[0], **kw)

    def _check(self, h: torch.Tensor) -> torch.Tensor:
        if h.dtype != self.dtype or tuple(h.shape) != (self.rows, self.dim) or h.device != self.device:
            raise ValueError(f"h must be {self.dtype} [{self.rows}, {self.dim}] on {self.device}, got "
                             f"{h.dtype} {list(h.shape)} on {h.device}")
        return h.contiguous()

    def forward(self, h: torch.Tensor) -> torch.Tensor:
        """Global mean loss (0-d fp32 tensor, stream-ordered)."""
        self._h = self._check(h)
        self._e.forward(self._h)
        return self._e.loss_tensor()

    def backward(self, grad_out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """d loss / d h for the preceding forward (times ``grad_out``)."""
        return self._e.backward(grad_out)

    def step(self, h: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        self._h = self._check(h)
        return self._e.step(self._h)

    def capture(self, h: torch.Tensor) -> torch.Tensor:
        """Capture one step for this ``h`` into a hipGraph; returns the ``dh`` buffer every
        ``replay()`` rewrites (single process only)."""
        self._h = self._check(h)
        return self._e.capture(self._h)

    def replay(self) -> torch.Tensor:
        self._e.replay()
        return self._e.loss_tensor()

    @property
    def device_bytes(self) -> int:
        return self._e.device_bytes

    @property
    def symmetric(self) -> bool:
        return self._e.symmetric

    @property
    def small(self) -> bool:
        return self._e.small
