"""CLI: SimCLR pre-training on synthetic images, one process per GPU.

  python -m ntxent_amd.models.train --steps 50 --batch 256
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
      -m ntxent_amd.models.train --steps 200 --batch 512 --ckpt-dir ckpt/ --ckpt-every 50
"""
from __future__ import annotations

import argparse
import dataclasses
import os
from datetime import timedelta

import torch
import torch.distributed as dist

from .trainer import SimCLRTrainer, TrainConfig


def main(argv=None):
    ap = argparse.ArgumentParser()
    for f in dataclasses.fields(TrainConfig):
        name = "--" + f.name.replace("_", "-")
        if f.type in ("bool", bool):
            ap.add_argument(name, type=lambda s: s.lower() in ("1", "true", "yes"), default=f.default)
        elif f.type in ("int", int):
            ap.add_argument(name, type=int, default=f.default)
        elif f.type in ("float", float):
            ap.add_argument(name, type=float, default=f.default)
        else:
            ap.add_argument(name, default=f.default)
    ap.add_argument("--pg-timeout", type=float, default=600.0,
                    help="process-group timeout (s): a rank stuck in a collective fails the job instead of hanging")
    args = ap.parse_args(argv)
    cfg = TrainConfig(**{f.name: getattr(args, f.name) for f in dataclasses.fields(TrainConfig)})
    pg_timeout = timedelta(seconds=args.pg_timeout)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not dist.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=pg_timeout)
        else:
            dist.init_process_group("gloo", timeout=pg_timeout)
    try:
        SimCLRTrainer(cfg).fit()
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
