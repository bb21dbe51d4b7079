"""Per-dispatch PMC counters per kernel from tools/gpu_pmc.sh output dirs.

Counter rows are per dispatch (and per XCD / SE instance for some blocks):
values are summed per (pass, dispatch) and then averaged over the dispatches
of each kernel, so every figure is "per launch".

    python tools/summarize_pmc.py gpurun_out/pmc [kernel-substring ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root, keys):
    per = defaultdict(lambda: defaultdict(float))     # (kernel, counter, pass, dispatch) sums
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        pas = os.path.relpath(f, root).split(os.sep)[0]
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:80]
            if keys and not any(s in k for s in keys):
                continue
            d = r.get("Dispatch_Id") or r.get("Correlation_Id") or "0"
            per[(k, r["Counter_Name"])][(pas, d)] += float(r["Counter_Value"])
    kern = defaultdict(dict)
    for (k, c), v in per.items():
        kern[k][c] = (sum(v.values()) / len(v), len(v))
    for k in sorted(kern):
        print(k)
        for c in sorted(kern[k]):
            m, n = kern[k][c]
            print("   %-32s %14.6g   (%d dispatches)" % (c, m, n))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
