"""The C++ test suite (tests/cpp/ntxent_tests.cpp, registered with ctest by CMakeLists.txt) inside
the driver's ``pytest -m gpu`` run, so the C++ API is covered by the round-end GPU tests too.

The reference registers its GTests with ctest (/root/reference/tests/CMakeLists.txt:8-21;
tests/test_forward.cpp, tests/test_backward.cpp). Here the executable checks the raw C++ API
(Engine, launchers, communicators, fault injection) against a host fp64 oracle; this test runs it
once, fails on any ``[ FAIL ]`` line or a non-zero exit, and refuses a binary built from other
sources than the tree's (a stale build would test yesterday's code): tools/build_ext.py records a
sha256 of the sources next to the binary, compared here by content, not by file mtimes (a fresh
checkout resets those). Without a built binary the test skips on a CPU-only checkout and fails on a GPU box.
"""
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
import build_ext  # noqa: E402


def test_cpp_suite_passes():
    exe = ROOT / "build" / "bin" / "ntxent_tests"
    if not exe.exists():
        msg = "build/bin/ntxent_tests not built: run tools/build_ext.py (or __graft_entry__.build())"
        # on a GPU box (or a tools/gpu_check.sh run) a missing binary is a failure, not a skip: the
        # C++ API suite must not silently drop out of a green GPU run
        import torch

        if torch.cuda.is_available() or os.environ.get("NTXENT_GPU_CHECK"):
            pytest.fail(msg)
        pytest.skip(msg)
    rec = build_ext.TESTS_HASH.read_text().strip() if build_ext.TESTS_HASH.exists() else None
    cur = build_ext.source_hash(build_ext.cpp_test_sources())
    assert rec == cur, "build/bin/ntxent_tests was built from other sources: rebuild (tools/build_ext.py)"
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, cwd=str(ROOT))
    out = r.stdout + r.stderr
    print(out[-4000:])
    fails = [ln for ln in out.splitlines() if ln.startswith("[ FAIL ]")]
    assert not fails, "\n".join(fails)
    assert r.returncode == 0, out[-3000:]
    passed = [ln for ln in out.splitlines() if ln.startswith("[ PASS ]")]
    assert len(passed) >= 20, f"only {len(passed)} C++ tests ran"
