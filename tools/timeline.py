"""Print one step of a rocprofv3 kernel trace (tools only): kernels in start order with their
durations and the idle gaps between them.
  python tools/timeline.py <k_kernel_trace.csv> <first-kernel-of-step substring> [step index from end]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"]]
back = int(sys.argv[3]) if len(sys.argv) > 3 else 3
i0, i1 = marks[-back], marks[-back + 1]
t0 = prev = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1000:8.1f} +{(e - s) / 1000:7.1f} gap {(s - prev) / 1000:6.1f}  "
          f"{r['Kernel_Name'][:80]}")
    prev = e
print("step span us", (int(rows[i1]["Start_Timestamp"]) - t0) / 1000)
