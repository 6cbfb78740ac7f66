"""Diagnostic: a rocprofv3 kernel_trace.csv summarised per (kernel, grid size): launches and average
duration in microseconds, sorted by total time. Usage: trace_by_grid.py TRACE.csv [TOP]."""
import collections
import csv
import sys


def main(path, top=40):
    acc = collections.defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0][:70]
            grid = f"{r.get('Grid_Size_X', r.get('Grid_Size', '?'))}x{r.get('Grid_Size_Y', '')}x{r.get('Grid_Size_Z', '')}"
            a = acc[(name, grid)]
            a[0] += 1
            a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    rows = sorted(acc.items(), key=lambda kv: -kv[1][1])[:top]
    for (name, grid), (n, tot) in rows:
        print(f"{tot / 1e3:9.2f} ms  {n:7d} x {tot / n:8.2f} us  {grid:>16}  {name}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
