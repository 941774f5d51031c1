"""Per-rank communication-wait accounting for the data-parallel paths.

Every place where a data-parallel forward/backward makes the compute stream depend on a
collective (``work.wait()`` on an RCCL work handle, or a synchronous collective) is wrapped
in :func:`span`. When enabled, a span records a HIP event on the current stream before and
after the dependency: the elapsed time between the two is how long the compute stream stood
still waiting for communication (zero when the transfer was already hidden under earlier
kernels). Nothing is recorded (and nothing synchronises) when accounting is disabled, which is
the default; ``bench.py`` enables it around its timed steps and reports the per-step sum.

On the gloo rehearsal backend the collectives are host-staged and synchronous, so a span
brackets the whole host-side transfer.
"""
from __future__ import annotations

import contextlib
from collections import defaultdict
from typing import Dict, List, Tuple

import torch

_enabled = False
_spans: List[Tuple[str, object, object]] = []


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = bool(on)
    _spans.clear()


def enabled() -> bool:
    return _enabled


@contextlib.contextmanager
def span(name: str, device=None):
    """Bracket a dependency of the current stream on communication (no-op when disabled or
    on CPU tensors)."""
    if not _enabled or not torch.cuda.is_available():
        yield
        return
    s = torch.cuda.current_stream(device)
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record(s)
    try:
        yield
    finally:
        b.record(s)
        _spans.append((name, a, b))


def collect(reset: bool = True) -> Dict[str, float]:
    """Sum of the recorded spans in ms, by name (synchronises on the recorded events)."""
    out: Dict[str, float] = defaultdict(float)
    for name, a, b in _spans:
        b.synchronize()
        out[name] += a.elapsed_time(b)
    if reset:
        _spans.clear()
    return dict(out)


def comm_reserve_cus(backend: str = "nccl") -> int:
    """CUs a GEMM leaves free while an RCCL transfer it overlaps is in flight.

    The similarity GEMMs are persistent (one 512-thread block per CU holding 128 KiB of LDS and
    the whole register file), so without a reserve the RCCL kernels of an overlapped P2P /
    all-gather cannot be scheduled until the GEMM ends. ``NTXENT_COMM_RESERVE_CUS`` overrides
    the default of 8 (one per XCD: 3 % of the chip); gloo transfers are host-staged and complete
    before the GEMM is launched, so they reserve nothing. The value is passed per launch
    (``reserve_cus=`` of the stage ops): no process-wide state, so GEMMs on concurrent streams
    each keep their own reserve."""
    if backend == "gloo":
        return 0
    import os

    return max(0, int(os.environ.get("NTXENT_COMM_RESERVE_CUS", "8")))


def rccl_shared_gpu_env(rank: int) -> Dict[str, str]:
    """Environment for rehearsing W RCCL ranks on ONE GPU (call before init_process_group).

    RCCL refuses two ranks of one host on one device ("Duplicate GPU detected"). A distinct
    ``NCCL_HOSTID`` per rank makes each rank its own host for RCCL's topology, so the ranks
    connect over RCCL's socket transport on loopback instead of xGMI P2P: the same RCCL
    collectives, grouped send/recv, proxy threads and communicator streams run as on an 8-GPU
    node, only the wire differs (and so the timing means nothing). Existing settings win."""
    import os

    env = {"NCCL_HOSTID": f"ntxent-shared-gpu-rank{int(rank)}", "NCCL_SOCKET_IFNAME": "lo",
           "NCCL_IB_DISABLE": "1"}
    for k, v in env.items():
        os.environ.setdefault(k, v)
    return {k: os.environ[k] for k in env}


def use_compute_stream(device=None, priority: str = "high"):
    """Make a new (high-priority by default) stream the current stream of `device` and return
    it. Data-parallel steps should not run on the device's default stream: there the RCCL
    kernels of the transfers they overlap shared its hardware queue and ran only between the
    compute kernels (profiles/r3/overlap: no RCCL kernel time inside the GEMM spans on the
    default stream, ~1.1 ms of 1.7 ms on a new high-priority stream). bench.py and the SimCLR
    trainer call this; call it once per process after torch.cuda.set_device."""
    import torch

    if priority not in ("high", "normal"):
        raise ValueError("priority must be 'high' or 'normal'")
    s = torch.cuda.Stream(device=device, priority=-1 if priority == "high" else 0)
    torch.cuda.set_stream(s)
    return s
