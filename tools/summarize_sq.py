"""Summarise the SQ pipe-utilisation passes of tools/gpu_pmc_sq.sh: per
kernel, the mean over dispatches of each counter, and the derived fractions
(per wave-cycle: VALU / LDS / VMEM issue, waits; MFMA busy per GRBM cycle)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?").split("(")[0].split("<")[0].replace("void ", "")
            k = k.split("::")[-1]
            acc[k][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, m in sorted(acc.items()):
        per = defaultdict(list)
        for (disp, name), vals in m.items():
            per[name].append(sum(vals))   # summed over the dimensions of one dispatch
        mean = {n: sum(v) / len(v) for n, v in per.items()}
        print(k)
        for n in sorted(mean):
            print("  %-28s %.4g" % (n, mean[n]))
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM",
                      "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                if n in mean:
                    print("  %-28s %.3f of wave-cycles" % (n, mean[n] / wc))
        g = mean.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
            print("  MFMA busy / (GRBM x 256 CU x 4 SIMD)   %.3f"
                  % (mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 256 * 4)))
        if g and "SQ_LDS_IDX_ACTIVE" in mean:
            print("  LDS active / (GRBM x 256 CU)           %.3f"
                  % (mean["SQ_LDS_IDX_ACTIVE"] / (g / 8 * 256)))


if __name__ == "__main__":
    main(sys.argv[1])
