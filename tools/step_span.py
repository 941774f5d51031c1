"""Per-step span from a rocprofv3 kernel trace: first kernel start of each step (a kernel whose
name matches --first) to the end of the last kernel before the next step starts; prints mean /
min over the steps and the mean duration of each kernel (overlapped kernels counted whole)."""
import csv
import sys
from collections import defaultdict


def main(path, first="prep"):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], None
    for r in rows:
        if first in r["Kernel_Name"]:
            if cur:
                steps.append(cur)
            cur = []
        if cur is not None:
            cur.append(r)
    if cur:
        steps.append(cur)
    steps = steps[2:]  # skip the first (cold) steps
    spans = [(max(int(r["End_Timestamp"]) for r in s) - int(s[0]["Start_Timestamp"])) / 1e3 for s in steps]
    print(f"{path}: {len(spans)} steps, span mean {sum(spans) / len(spans):.1f} us, min {min(spans):.1f} us")


if __name__ == "__main__":
    main(*sys.argv[1:])
