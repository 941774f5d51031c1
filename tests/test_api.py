"""API-surface tests (CPU): reference names/kwargs, op registration, autograd routing.

Reference surface: pybind ``forward/backward/check_tensor_core_support``
(src/binding_new.cpp:4-21) and ``torch.ops.ntxent_cuda.*`` (python/test.py:137).
"""
import inspect

import pytest
import torch

import ntxent_amd
from ntxent_amd.ops import _ext, reference


def test_package_exports():
    for name in ("ntxent_loss", "NTXentLoss", "NTXentFunction", "forward", "backward", "forward_with_stats",
                 "check_tensor_core_support", "check_matrix_core_support"):
        assert hasattr(ntxent_amd, name), name
    assert ntxent_amd.__version__


def test_reference_signatures():
    sig = inspect.signature(ntxent_amd.forward)
    assert list(sig.parameters) == ["z", "T", "use_mixed_precision"]
    assert sig.parameters["use_mixed_precision"].default is False
    sig = inspect.signature(ntxent_amd.backward)
    # the reference's five parameters first; the opt-in debug output after them
    assert list(sig.parameters)[:5] == ["z", "softmax", "grad_out", "T", "use_mixed_precision"]
    assert sig.parameters["want_grad_logits"].default is False


def test_extension_loads_and_registers_ops():
    C = _ext.load()
    for name in ("forward", "backward", "forward_with_stats", "check_tensor_core_support",
                 "check_matrix_core_support", "fused_forward", "fused_backward", "get_optimal_block_size"):
        assert hasattr(C, name), name
    assert hasattr(torch.ops.ntxent_cuda, "forward")
    assert hasattr(torch.ops.ntxent_cuda, "backward")
    assert hasattr(torch.ops.ntxent, "forward_with_stats")
    schema = str(torch.ops.ntxent_cuda.forward.default._schema)
    assert "use_mixed_precision=False" in schema
    assert "want_grad_logits=False" in str(torch.ops.ntxent_cuda.backward.default._schema)


def test_cpu_tensors_use_oracle_with_autograd():
    h = torch.randn(16, 8, dtype=torch.float64, requires_grad=True)
    loss = ntxent_amd.ntxent_loss(h, 0.1)
    loss.backward()
    torch.testing.assert_close(h.grad, reference.ntxent_backward_analytic(h.detach(), 0.1))


def test_module_front_end():
    m = ntxent_amd.NTXentLoss(temperature=0.2)
    z1, z2 = torch.randn(4, 6, dtype=torch.float64), torch.randn(4, 6, dtype=torch.float64)
    torch.testing.assert_close(m(z1, z2), reference.ntxent_loss_pair(z1, z2, 0.2))
    assert "temperature=0.2" in repr(m)


def test_compute_policy():
    from ntxent_amd.ops import resolve_compute

    assert resolve_compute(torch.float32) == "fp32"
    assert resolve_compute(torch.float32, use_mixed_precision=True) == "fp16"
    assert resolve_compute(torch.bfloat16) == "fp16"
    assert resolve_compute(torch.bfloat16, compute="bf16") == "bf16"
    with pytest.raises(ValueError):
        resolve_compute(torch.float32, compute="int8")
    C = _ext.load()
    assert C.choose_compute("float32", False, "auto") == "fp32"
    assert C.choose_compute("bfloat16", False, "auto") == "fp16"


def test_cuda_op_rejects_cpu_tensor():
    C = _ext.load()
    with pytest.raises(Exception):
        C.forward(torch.randn(8, 4), 0.07, False)


def test_block_size_heuristic():
    C = _ext.load()
    assert C.get_optimal_block_size(1) >= 64
    assert C.get_optimal_block_size(1 << 20) % 64 == 0
