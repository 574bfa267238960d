#!/usr/bin/env python3
"""GPU timeline of a rocprofv3 kernel trace: busy time vs wall, the gaps
between dispatches, and per-kernel totals inside a window.

    python tools/timeline.py kernel_trace.csv [--split KERNEL] [--skip N]

--split KERNEL: cut the trace into segments at each dispatch of KERNEL (e.g.
k_stream_buckets, the first kernel of a stream batch) and report every
segment's wall span, busy time, dispatch count and largest gaps; --skip N
drops the first N segments (warmup).
"""
import argparse
import csv
import collections


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def busy(rows):
    """Union of the dispatch intervals (ns)."""
    t, end = 0, None
    for s, e, _ in rows:
        if end is None or s > end:
            t += e - s
            end = e
        elif e > end:
            t += e - end
            end = e
    return t


def short(name):
    return name.split("(")[0].replace("void ", "")[:48]


def report(rows, label):
    span = rows[-1][1] - rows[0][0]
    b = busy(rows)
    gaps = []
    end = rows[0][1]
    for (s, e, n), prev in zip(rows[1:], rows[:-1]):
        if s > end:
            gaps.append((s - end, short(prev[2]), short(n)))
        end = max(end, e)
    gaps.sort(reverse=True)
    per = collections.defaultdict(lambda: [0, 0])
    for s, e, n in rows:
        per[short(n)][0] += 1
        per[short(n)][1] += e - s
    print("%s: span %.1f us, busy %.1f us (%.0f%%), %d dispatches, gaps %.1f us" %
          (label, span / 1e3, b / 1e3, 100.0 * b / span, len(rows), sum(g[0] for g in gaps) / 1e3))
    for g, a, n in gaps[:6]:
        print("   gap %7.1f us  after %-40s before %s" % (g / 1e3, a, n))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--split", default=None)
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    rows = load(a.trace)
    if not a.split:
        per = report(rows, "all")
    else:
        cuts = [i for i, r in enumerate(rows) if r[2].startswith(a.split) or short(r[2]) == a.split]
        segs = [rows[i:j] for i, j in zip(cuts, cuts[1:] + [len(rows)])][a.skip:]
        per = collections.defaultdict(lambda: [0, 0])
        for k, seg in enumerate(segs):
            p = report(seg, "segment %d" % k)
            for n, (c, t) in p.items():
                per[n][0] += c
                per[n][1] += t
        for n in per:
            per[n][0] /= max(len(segs), 1)
            per[n][1] /= max(len(segs), 1)
    print("kernel totals (per segment when split): count, us")
    for n, (c, t) in sorted(per.items(), key=lambda x: -x[1][1])[:a.top]:
        print("   %-48s %6.1f %9.1f" % (n, c, t / 1e3))


if __name__ == "__main__":
    main()
