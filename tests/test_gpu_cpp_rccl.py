"""Native RcclComm at world size > 1 on the 1-GPU box: ntxent_bench as W processes over RCCL
(per-rank NCCL_HOSTID, socket transport), every rank's loss against the in-process ThreadComm
run of the same seeds (tools/cpp_rccl_procs.py)."""
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("W,negatives", [(2, "symmetric"), (2, "allgather"), (3, "symmetric"),
                                        (8, "symmetric"), (8, "allgather")])  # W = 8: the scaling run
def test_native_rccl_processes_match_emulated(W, negatives):
    bench = ROOT / "build" / "bin" / "ntxent_bench"
    assert bench.exists(), "build/bin/ntxent_bench missing: run tools/build_ext.py"
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "cpp_rccl_procs.py"), "--gpus", str(W), "--negatives",
                        negatives, "--batch", "512", "--dim", "128", "--shared-gpu", "--timeout", "90"],
                       capture_output=True, text=True, timeout=200)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
