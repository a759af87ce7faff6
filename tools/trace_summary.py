#!/usr/bin/env python3
"""Per-kernel durations and gaps of the last search step in a rocprofv3 kernel trace: the step is
the run of kernels ending at the last `knn` kernel, starting at the last query-prep kernel (or,
when the query prep runs inside the int8 scan, at the last knn_i8_scan_kernel)."""
import csv, sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
starts = [i for i, n in enumerate(names) if "prep" in n or "query" in n]
last = max(starts) if starts else max(i for i, n in enumerate(names) if "knn_i8_scan" in n)
# the step starts at the last query-prep kernel that begins a chain (walk back over i8 query)
start = last
while start > 0 and ("prep" in names[start - 1] or "query" in names[start - 1]):
    start -= 1
t0 = int(rows[start]["Start_Timestamp"])
prev_end = t0
for r in rows[start:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"gap {(s - prev_end) / 1e3:7.1f} us  dur {(e - s) / 1e3:7.1f} us  {r['Kernel_Name'][:100]}")
    prev_end = e
print(f"step span {(prev_end - t0) / 1e3:.1f} us")
