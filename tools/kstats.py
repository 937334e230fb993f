#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time with calls, average and share.
usage: python3 tools/kstats.py <run_kernel_stats.csv> [n]"""
import csv
import sys


def main(path, n=14):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
        print(f"{r['Name'][:88]:88s} calls={r['Calls']:>7} avg={float(r['AverageNs']) / 1000:8.2f}us "
              f"share={100 * float(r['TotalDurationNs']) / tot:5.1f}%")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 14)
