"""Checkpoint / resume for the SimCLR trainer (the loss op itself is stateless: SURVEY.md §5).

* Atomic: written to ``<path>.tmp`` then ``os.replace``d, so a crash mid-write never leaves a
  truncated checkpoint behind.
* Safe load: ``torch.load(..., weights_only=True)`` only — no pickled code is executed.
* Rank-aware: only rank 0 writes; every rank can load (the state is replicated under DDP).
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Any, Dict, Optional

import torch


def save_checkpoint(path: str | Path, *, model: torch.nn.Module, optimizer: Optional[torch.optim.Optimizer] = None,
                    step: int = 0, extra: Optional[Dict[str, Any]] = None, rank: int = 0) -> Optional[Path]:
    if rank != 0:
        return None
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    m = model.module if hasattr(model, "module") else model
    state = {"model": m.state_dict(), "step": int(step), "extra": extra or {}}
    if optimizer is not None:
        state["optimizer"] = optimizer.state_dict()
    tmp = path.with_suffix(path.suffix + ".tmp")
    torch.save(state, tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(path: str | Path, *, model: torch.nn.Module, optimizer: Optional[torch.optim.Optimizer] = None,
                    map_location: Any = "cpu") -> Dict[str, Any]:
    state = torch.load(Path(path), map_location=map_location, weights_only=True)
    m = model.module if hasattr(model, "module") else model
    m.load_state_dict(state["model"])
    if optimizer is not None and "optimizer" in state:
        optimizer.load_state_dict(state["optimizer"])
    return {"step": int(state.get("step", 0)), "extra": state.get("extra", {})}


def latest_checkpoint(directory: str | Path, prefix: str = "ckpt_") -> Optional[Path]:
    d = Path(directory)
    if not d.is_dir():
        return None
    cands = sorted(d.glob(f"{prefix}*.pt"), key=lambda p: int(p.stem[len(prefix):]) if p.stem[len(prefix):].isdigit() else -1)
    return cands[-1] if cands else None
