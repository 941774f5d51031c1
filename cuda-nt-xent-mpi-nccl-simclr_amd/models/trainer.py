"""SimCLR training loop: DDP over RCCL, global-batch NT-Xent, LARS, bf16 autocast, checkpoints.

One process per GPU (``torchrun``); the contrastive loss gathers every rank's embeddings
(``NTXentLoss(distributed=True)`` -> RCCL all-gather over xGMI), so each rank's negatives are
the whole global batch — the "MPI-NCCL SimCLR" the reference's name promises but never
implements.

Gradient scaling: the distributed loss is already the *global* mean, and the gradient it
returns for this rank's rows is this rank's share of d(global loss); DDP then AVERAGES
parameter gradients over ranks, so the loss is multiplied by the world size before
``backward`` to end with the exact gradient of the global loss.

Data is synthetic (no datasets on this box): images drawn around ``num_classes`` random
prototypes, so two augmented views of the same image share content and the loss can fall.
"""
from __future__ import annotations

import json
import math
import os
import time
from dataclasses import asdict, dataclass, field
from pathlib import Path
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..ops.ntxent import NTXentLoss
from ..utils.checkpoint import latest_checkpoint, load_checkpoint, save_checkpoint
from ..utils.memory import GPUMemoryTracker
from ..utils.trace import trace_range
from .augment import AugmentConfig, two_views
from .lars import LARS
from .simclr import MLPEncoder, SimCLR, param_groups_for_lars, resnet18


@dataclass
class TrainConfig:
    steps: int = 100
    batch: int = 256                 # images per GPU (pairs per GPU)
    image_size: int = 32
    encoder: str = "resnet18"        # resnet18 | mlp
    width: int = 64
    proj_hidden: int = 2048
    proj_out: int = 128
    temperature: float = 0.5
    lr: float = 0.3                  # base LR, scaled by global batch / 256
    weight_decay: float = 1e-6
    warmup_steps: int = 10
    optimizer: str = "lars"          # lars | sgd | adamw
    amp: bool = True                 # bf16 autocast on the GPU
    # GPU: run the step on a new high-priority stream ("high"), a new stream ("new") or the
    # default stream ("default"). On the default stream RCCL kernels (DDP's bucket all-reduces,
    # the NT-Xent transfers) shared its hardware queue and ran only between compute kernels
    # (profiles/r3/overlap).
    compute_stream: str = "high"
    compute: str = "auto"            # loss compute dtype
    negatives: str = "symmetric"     # multi-GPU negatives: symmetric | allgather | ring
    sync_bn: bool = True             # global BN statistics (SimCLR)
    num_classes: int = 100
    seed: int = 0
    ckpt_dir: Optional[str] = None
    ckpt_every: int = 0
    resume: bool = True
    log_every: int = 10
    metrics_path: Optional[str] = None


def _dist():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


class SyntheticImages:
    """Deterministic per-(rank, step) batches: prototype image + per-image noise."""

    def __init__(self, cfg: TrainConfig, device: torch.device, rank: int):
        g = torch.Generator().manual_seed(cfg.seed)
        self.protos = torch.rand(cfg.num_classes, 3, cfg.image_size, cfg.image_size, generator=g).to(device)
        self.cfg, self.device, self.rank = cfg, device, rank

    def batch(self, step: int) -> torch.Tensor:
        g = torch.Generator(device=self.device).manual_seed(self.cfg.seed * 1_000_003 + step * 997 + self.rank)
        idx = torch.randint(0, self.cfg.num_classes, (self.cfg.batch,), generator=g, device=self.device)
        noise = 0.1 * torch.randn(self.cfg.batch, 3, self.cfg.image_size, self.cfg.image_size, generator=g,
                                  device=self.device)
        return (self.protos[idx] + noise).clamp(0, 1)


def build_model(cfg: TrainConfig) -> SimCLR:
    if cfg.encoder == "mlp":
        enc = MLPEncoder(3 * cfg.image_size * cfg.image_size, 512, 256)
    else:
        enc = resnet18(cfg.width, cifar_stem=cfg.image_size <= 64)
    return SimCLR(enc, cfg.proj_hidden, cfg.proj_out)


def build_optimizer(cfg: TrainConfig, model: torch.nn.Module, world: int) -> torch.optim.Optimizer:
    lr = cfg.lr * cfg.batch * world / 256.0
    if cfg.optimizer == "lars":
        return LARS(list(param_groups_for_lars(model, cfg.weight_decay)), lr=lr)
    if cfg.optimizer == "adamw":
        return torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=cfg.weight_decay)
    return torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=cfg.weight_decay)


def lr_at(step: int, cfg: TrainConfig, base: float) -> float:
    if step < cfg.warmup_steps:
        return base * (step + 1) / cfg.warmup_steps
    t = (step - cfg.warmup_steps) / max(1, cfg.steps - cfg.warmup_steps)
    return base * 0.5 * (1 + math.cos(math.pi * min(1.0, t)))


class SimCLRTrainer:
    def __init__(self, cfg: TrainConfig, device: Optional[torch.device] = None):
        self.cfg = cfg
        self.world, self.rank = _dist()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        self.device = device
        # Data-parallel steps run on their own (high-priority) stream, entered per step: the RCCL
        # kernels of overlapped transfers then do not share the compute stream's hardware queue
        # (commstats.use_compute_stream). Kept on self and entered in train_step(), so the caller's
        # current stream is never switched; each step is ordered after the caller's queued work.
        self.stream = None
        if device.type == "cuda" and cfg.compute_stream != "default":
            self.stream = torch.cuda.Stream(device=device, priority=-1 if cfg.compute_stream == "high" else 0)
        torch.manual_seed(cfg.seed)
        model = build_model(cfg).to(device)
        if device.type == "cuda":
            model = model.to(memory_format=torch.channels_last)
        if self.world > 1 and cfg.sync_bn and device.type == "cuda":  # SyncBN needs GPU tensors
            model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
        self.model = model
        if self.world > 1:
            self.model = torch.nn.parallel.DistributedDataParallel(
                model, device_ids=[device.index] if device.type == "cuda" else None, bucket_cap_mb=64)
        self.opt = build_optimizer(cfg, self.model, self.world)
        self.base_lrs = [g["lr"] for g in self.opt.param_groups]
        self.loss_fn = NTXentLoss(cfg.temperature, compute=cfg.compute, distributed=self.world > 1,
                                  negatives=cfg.negatives)
        self.data = SyntheticImages(cfg, device, self.rank)
        self.aug = AugmentConfig(out_size=cfg.image_size)
        self.mem = GPUMemoryTracker() if device.type == "cuda" else None
        self.step = 0
        self.history: List[Dict] = []
        if cfg.ckpt_dir and cfg.resume:
            last = latest_checkpoint(cfg.ckpt_dir)
            if last is not None:
                st = load_checkpoint(last, model=self.model, optimizer=self.opt, map_location=device)
                self.step = st["step"]

    def train_step(self) -> Dict:
        if self.stream is None:
            return self._train_step()
        caller = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(caller)
        with torch.cuda.stream(self.stream):
            rec = self._train_step()
        caller.wait_stream(self.stream)
        return rec

    def _train_step(self) -> Dict:
        cfg = self.cfg
        for g, base in zip(self.opt.param_groups, self.base_lrs):
            g["lr"] = lr_at(self.step, cfg, base)
        t0 = time.perf_counter()
        with trace_range("simclr.data"):
            x = self.data.batch(self.step)
            gen = torch.Generator(device=self.device).manual_seed(cfg.seed + 7919 * self.step + self.rank)
            v1, v2 = two_views(x, self.aug, gen)
            if self.device.type == "cuda":
                v1 = v1.contiguous(memory_format=torch.channels_last)
                v2 = v2.contiguous(memory_format=torch.channels_last)
        use_amp = cfg.amp and self.device.type == "cuda"
        with trace_range("simclr.forward"), torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=use_amp):
            z = self.model(v1, v2)
        with trace_range("simclr.loss"):
            loss = self.loss_fn(z)
        with trace_range("simclr.backward"):
            self.opt.zero_grad(set_to_none=True)
            (loss * self.world).backward()
        with trace_range("simclr.optimizer"):
            self.opt.step()
        lv = float(loss.detach())
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rec = {"step": self.step, "loss": lv, "lr": self.opt.param_groups[0]["lr"], "step_ms": dt * 1e3,
               "images_per_s": cfg.batch * self.world / dt}
        if not math.isfinite(lv):
            raise FloatingPointError(f"non-finite loss at step {self.step}")
        self.step += 1
        if cfg.ckpt_dir and cfg.ckpt_every and self.step % cfg.ckpt_every == 0:
            save_checkpoint(Path(cfg.ckpt_dir) / f"ckpt_{self.step}.pt", model=self.model, optimizer=self.opt,
                            step=self.step, extra={"config": asdict(cfg)}, rank=self.rank)
        return rec

    def fit(self, steps: Optional[int] = None) -> List[Dict]:
        end = self.cfg.steps if steps is None else self.step + steps
        while self.step < end:
            rec = self.train_step()
            self.history.append(rec)
            if self.mem is not None and (rec["step"] % max(1, self.cfg.log_every) == 0):
                self.mem.log(f"step {rec['step']}")
            if self.rank == 0 and self.cfg.log_every and rec["step"] % self.cfg.log_every == 0:
                print(json.dumps(rec), flush=True)
        if self.rank == 0 and self.cfg.metrics_path:
            Path(self.cfg.metrics_path).parent.mkdir(parents=True, exist_ok=True)
            with open(self.cfg.metrics_path, "w") as f:
                for r in self.history:
                    f.write(json.dumps(r) + "\n")
        return self.history
