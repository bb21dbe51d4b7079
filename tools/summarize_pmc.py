"""Average PMC counters per kernel from tools/gpu_pmc.sh output dirs."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    tot = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            k = k[:70]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]] += 1
    # counter rows are per dispatch (and per XCD/SE instance for some); report the
    # per-dispatch total = sum / number of dispatches of that kernel
    for k in sorted(tot):
        print(k)
        for c in sorted(tot[k]):
            print("   %-32s %.4g" % (c, tot[k][c]))


if __name__ == "__main__":
    main(sys.argv[1])
