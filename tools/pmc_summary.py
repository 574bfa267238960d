#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch).

usage: python tools/pmc_summary.py DIR [DIR...]   (each DIR holds run_counter_collection.csv)
"""
import csv
import sys
from collections import defaultdict


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        k = r["Kernel_Name"].split("(")[0][:48]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    try:
        for r in csv.DictReader(open(d + "/run_kernel_trace.csv")):
            k = r["Kernel_Name"].split("(")[0][:48]
            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    except FileNotFoundError:
        pass
    return acc, dur


def main():
    tot = defaultdict(dict)
    durs = defaultdict(list)
    for d in sys.argv[1:]:
        acc, dur = load(d)
        for k, cs in acc.items():
            for c, v in cs.items():
                tot[k][c] = sum(v) / len(v)
        for k, v in dur.items():
            durs[k] += v
    for k in sorted(tot, key=lambda k: -(sum(durs[k]) / max(1, len(durs[k])))):
        d = sum(durs[k]) / max(1, len(durs[k]))
        print("== %s  (mean %.1f us)" % (k, d / 1e3))
        for c, v in sorted(tot[k].items()):
            print("   %-24s %16.0f" % (c, v))


if __name__ == "__main__":
    main()
