"""Summarise a rocprofv3 run of bench.py (tools/gpu_prof.sh) into profiles/.

Reads <dir>/trace/run_kernel_stats.csv and the FETCH_SIZE / WRITE_SIZE PMC
passes and writes a JSON + text summary.  HBM bytes per launch follow
MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so it is
doubled (hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024).

    python tools/summarize_prof.py gpurun_out/prof_r1 profiles/r1_bench
"""
import collections
import csv
import json
import os
import re
import sys


def short(name):
    m = re.search(r"fasst::k_estep<\d+, \d+, \d+, (\d), \d+>", name)
    if m:
        return "k_estep_part%s" % m.group(1)
    if "fasst::k_estep_mx<" in name:
        return "k_estep"
    if name.startswith("Cijk"):
        return "rocblas_" + name[:12]
    m = re.search(r"fasst::(k_\w+)", name)
    return m.group(1) if m else name[:40]


def main(src, dst):
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    kernels = collections.OrderedDict()
    for r in stats:
        k = short(r["Name"])
        e = kernels.setdefault(k, {"calls": 0, "total_ns": 0.0})
        e["calls"] += int(r["Calls"])
        e["total_ns"] += float(r["TotalDurationNs"])
    for k, e in kernels.items():
        e["avg_us"] = round(e["total_ns"] / e["calls"] / 1e3, 3)
    # steady-clock average: the second half of each kernel's launches (the
    # first iterations of a run execute while the GPU clock ramps up)
    tpath = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(tpath):
        durs = collections.defaultdict(list)
        for r in csv.DictReader(open(tpath)):
            durs[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, d in durs.items():
            if k in kernels and len(d) >= 2:
                tail = d[len(d) // 2:]
                kernels[k]["avg_us_2nd_half"] = round(sum(tail) / len(tail) / 1e3, 3)
    pmc =collections.defaultdict(lambda: collections.defaultdict(list))
    for sub, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        path = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == counter:
                pmc[short(r["Kernel_Name"])][counter].append(float(r["Counter_Value"]))
    for k, c in pmc.items():
        e = kernels.setdefault(k, {})
        f = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"]) if c["FETCH_SIZE"] else None
        w = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"]) if c["WRITE_SIZE"] else None
        e["FETCH_SIZE_KiB"] = f
        e["WRITE_SIZE_KiB"] = w
        if f is not None and w is not None:
            e["hbm_bytes_per_launch"] = (2.0 * f + w) * 1024.0
            t = e.get("avg_us_2nd_half") or e.get("avg_us")
            if t:
                e["hbm_GBps"] = round(e["hbm_bytes_per_launch"] / (t * 1e-6) / 1e9, 1)
                e["hbm_frac_of_8TBps"] = round(e["hbm_GBps"] / 8000.0, 3)
    out = {"source": src, "kernels": kernels,
           "note": "avg_us from rocprofv3 --kernel-trace --stats; hbm bytes = (2*FETCH_SIZE + "
                   "WRITE_SIZE)*1024 per launch (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md)"}
    with open(dst + ".json", "w") as fh:
        json.dump(out, fh, indent=1)
    with open(dst + ".txt", "w") as fh:
        fh.write("# rocprofv3 summary of %s\n" % src)
        fh.write("%-16s %7s %12s %12s %14s %14s %16s %9s %6s\n" % (
            "kernel", "calls", "avg_us", "avg_us_2h", "FETCH_KiB", "WRITE_KiB", "hbm_B/launch",
            "GB/s", "frac"))
        for k, e in sorted(kernels.items(), key=lambda kv: -kv[1].get("total_ns", 0)):
            fh.write("%-16s %7s %12s %12s %14s %14s %16s %9s %6s\n" % (
                k, e.get("calls", ""), e.get("avg_us", ""), e.get("avg_us_2nd_half", ""),
                "%.0f" % e["FETCH_SIZE_KiB"] if e.get("FETCH_SIZE_KiB") is not None else "",
                "%.0f" % e["WRITE_SIZE_KiB"] if e.get("WRITE_SIZE_KiB") is not None else "",
                "%.3e" % e["hbm_bytes_per_launch"] if e.get("hbm_bytes_per_launch") else "",
                e.get("hbm_GBps", ""), e.get("hbm_frac_of_8TBps", "")))
    print(open(dst + ".txt").read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
