"""Launch the native bench as N RCCL ranks in N processes (``ntxent_bench --proc-rank``) and
check every rank's loss against the in-process ThreadComm run of the same seeds (--emulate).

With --shared-gpu all ranks use GPU 0 and each gets its own NCCL_HOSTID, so RCCL connects them
over its socket transport (the RcclComm all-gather / grouped send_recv code runs as on an 8-GPU
node; the wire is not xGMI). The parent never touches the GPU: it only starts children.

usage: python tools/cpp_rccl_procs.py --gpus 2 [--shared-gpu] [--negatives symmetric|allgather]
       [--batch 1024 --dim 256]"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

BENCH = Path(__file__).resolve().parents[1] / "build" / "bin" / "ntxent_bench"
LOSS = re.compile(r"loss (-?[0-9.]+(?:e[-+]?\d+)?)")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--negatives", default="symmetric", choices=["symmetric", "allgather"])
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--shared-gpu", action="store_true")
    ap.add_argument("--timeout", type=int, default=120)
    ap.add_argument("--rtol", type=float, default=1e-4)
    a = ap.parse_args()
    common = ["--gpus", str(a.gpus), "--batch", str(a.batch), "--dim", str(a.dim), "--negatives", a.negatives,
              "--iters", str(a.iters), "--warmup", "1"]
    emu = subprocess.run([str(BENCH), *common, "--emulate"], capture_output=True, text=True, timeout=a.timeout)
    print(emu.stdout.strip().splitlines()[-1] if emu.stdout.strip() else emu.stderr[-2000:])
    if emu.returncode != 0:
        return 1
    ref = float(LOSS.findall(emu.stdout)[-1])
    with tempfile.TemporaryDirectory() as td:
        uid = os.path.join(td, "rccl_uid")
        procs = []
        for r in range(a.gpus):
            env = dict(os.environ)
            if a.shared_gpu:
                env.setdefault("NCCL_SOCKET_IFNAME", "lo")
                env.setdefault("NCCL_IB_DISABLE", "1")
                env["NCCL_HOSTID"] = f"ntxent-cpp-rank{r}"
            cmd = [str(BENCH), *common, "--proc-rank", str(r), "--uid-file", uid] + (["--shared-gpu"] if a.shared_gpu else [])
            procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
        ok = True
        for r, p in enumerate(procs):
            try:
                out, _ = p.communicate(timeout=a.timeout)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                print(f"rank {r}: timed out")
                return 1
            lines = [ln for ln in out.splitlines() if ln.startswith("proc rank")]
            print(lines[-1] if lines else f"rank {r} rc={p.returncode}: {out[-2000:]}")
            if p.returncode != 0 or not lines:
                ok = False
                continue
            loss = float(LOSS.findall(lines[-1])[-1])
            if abs(loss - ref) > a.rtol * max(1.0, abs(ref)):
                print(f"rank {r}: loss {loss} != emulated {ref}")
                ok = False
    print(f"{'PASS' if ok else 'FAIL'}: {a.gpus} RCCL processes ({a.negatives}) vs emulated loss {ref:.6f}")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
