"""CPU checks of the shared-GPU RCCL rehearsal environment (parallel/commstats.py)."""
import os

from ntxent_amd.parallel.commstats import comm_reserve_cus, rccl_shared_gpu_env


def test_rccl_shared_gpu_env_sets_per_rank_host(monkeypatch):
    for k in ("NCCL_HOSTID", "NCCL_SOCKET_IFNAME", "NCCL_IB_DISABLE"):
        monkeypatch.delenv(k, raising=False)
    env = rccl_shared_gpu_env(3)
    assert env["NCCL_HOSTID"].endswith("rank3") and os.environ["NCCL_HOSTID"] == env["NCCL_HOSTID"]
    assert env["NCCL_SOCKET_IFNAME"] == "lo" and env["NCCL_IB_DISABLE"] == "1"


def test_rccl_shared_gpu_env_keeps_existing(monkeypatch):
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "eth9")
    monkeypatch.delenv("NCCL_HOSTID", raising=False)
    assert rccl_shared_gpu_env(0)["NCCL_SOCKET_IFNAME"] == "eth9"


def test_comm_reserve_defaults(monkeypatch):
    monkeypatch.delenv("NTXENT_COMM_RESERVE_CUS", raising=False)
    assert comm_reserve_cus("gloo") == 0
    assert comm_reserve_cus("nccl") == 8
    monkeypatch.setenv("NTXENT_COMM_RESERVE_CUS", "16")
    assert comm_reserve_cus("nccl") == 16


def test_native_engine_rejects_bad_dtype_before_loading():
    import pytest
    import torch

    from ntxent_amd.parallel.native import NativeNTXent

    with pytest.raises(TypeError):
        NativeNTXent(64, 32, dtype=torch.int8)
