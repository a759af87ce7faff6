"""Idle gaps between consecutive kernels in a rocprofv3 kernel trace (run_kernel_trace.csv):
for the longest run of back-to-back searches (the bench's timed region), the average per search
of each kernel's duration and of the gap before it.  Usage: python tools/trace_gaps.py <csv> [first_kernel_regex]"""
import csv
import re
import sys
from collections import defaultdict


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    first = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"knn_b16w_tile_kernel")
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:70]) for r in rows]
    # split into searches at each occurrence of the first kernel
    idx = [i for i, e in enumerate(ev) if first.search(e[2])]
    dur, gap, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
    spans = []
    for a, b in zip(idx, idx[1:]):
        span = ev[b][0] - ev[a][0]
        spans.append((span, a, b))
    spans.sort()
    med = spans[len(spans) // 2][0]
    use = [s for s in spans if s[0] < 1.5 * med]
    for _, a, b in use:
        for i in range(a, b):
            name = ev[i][2]
            dur[name] += ev[i][1] - ev[i][0]
            gap[name] += ev[i][0] - (ev[i - 1][1] if i > 0 else ev[i][0])
            cnt[name] += 1
    n = len(use)
    print(f"searches {n}, median span {med / 1e3:.1f} us")
    tot_d = tot_g = 0.0
    for name in sorted(dur, key=lambda k: -dur[k]):
        print(f"{name:72s} x{cnt[name] / n:.2f}  dur {dur[name] / n / 1e3:8.2f} us  gap before {gap[name] / n / 1e3:7.2f} us")
        tot_d += dur[name] / n
        tot_g += gap[name] / n
    print(f"total per search: kernels {tot_d / 1e3:.1f} us, gaps {tot_g / 1e3:.1f} us")


if __name__ == "__main__":
    main()
