"""One step of a rocprofv3 trace (kernel + HIP API + memory copies) as a merged timeline (tools
only): device work (kernels, copies) and the host's HIP calls in start order, each with its start
offset, duration and -- for device work -- the idle gap before it; then per-category totals.

  python tools/e2e_timeline.py <trace dir> <first-kernel-of-step substring> [step index from end]

Categories: host calls (HIP runtime: launches, copies issued, synchronisations -- a synchronisation
that waits on the device is a host round trip), device kernels, device copies."""
import csv
import glob
import sys
from collections import defaultdict


def load(d, pat):
    f = glob.glob(f"{d}/**/*{pat}", recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    d, first = sys.argv[1], sys.argv[2]
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    ker = sorted(load(d, "kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    marks = [int(r["Start_Timestamp"]) for r in ker if first in r["Kernel_Name"]]
    t0, t1 = marks[-back], marks[-back + 1]
    ev = []
    for r in ker:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 - 2_000_000 <= s < t1:
            ev.append((s, e, "K", r["Kernel_Name"]))
    for r in load(d, "memory_copy_trace.csv"):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 - 2_000_000 <= s < t1:
            ev.append((s, e, "C", f"{r.get('Direction', '')} {r.get('Size', '')} B"))
    api = []
    for r in load(d, "hip_api_trace.csv"):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 - 2_000_000 <= s < t1:
            api.append((s, e, "H", r["Function"]))
    # the step starts at the host call that precedes the step's first device op (its launch)
    dev = sorted(x for x in ev if x[0] >= t0)
    prev_step_dev_end = max([x[1] for x in ev if x[0] < t0] or [t0])
    api = [a for a in api if a[0] >= prev_step_dev_end]
    start = min([a[0] for a in api] + [t0])
    tot = defaultdict(float)
    prev = start
    print(f"{'start_us':>9} {'dur_us':>8} {'gap_us':>7}  kind  name")
    for s, e, k, n in sorted(dev + api):
        gap = (s - prev) / 1000 if k != "H" else 0.0
        print(f"{(s - start) / 1000:9.1f} {(e - s) / 1000:8.1f} {gap:7.1f}  {k}     {n[:90]}")
        if k != "H":
            prev = max(prev, e)
        tot[k] += (e - s) / 1000
    span = (t1 - start) / 1000
    print(f"step span {span:.1f} us; device kernels {tot['K']:.1f} us, device copies {tot['C']:.1f} us, "
          f"host HIP calls {tot['H']:.1f} us (incl. synchronisation waits)")


if __name__ == "__main__":
    main()
