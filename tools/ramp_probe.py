"""Per-iteration GEM time over the first iterations of a process (the clock
ramp behind the driver's short-warm-up bench figure).  Diagnostic only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

m = bench.build_model(seed=0, device=0)
eng = m._engine
m._upload()
rows = bench.psd_schedule(m, 80)
out = []
t_start = time.perf_counter()
for i in range(80):
    t0 = time.perf_counter()
    eng.run(rows[i:i + 1], m.nmfUpdateCoeff)
    out.append((time.perf_counter() - t0) * 1e3)
print("per-iteration ms (host, synced each):")
for i in range(0, 80, 10):
    print(i, " ".join("%.3f" % x for x in out[i:i + 10]))
print("elapsed %.1f ms" % ((time.perf_counter() - t_start) * 1e3))
