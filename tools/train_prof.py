#!/usr/bin/env python3
"""Per-step kernel breakdown of a bench_train.py kernel trace: the dispatches
between consecutive adamw_kernel launches are one training step.
    python tools/train_prof.py <run_kernel_trace.csv> [--skip 3]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--skip', type=int, default=3, help='warmup steps to drop')
    ap.add_argument('--top', type=int, default=40)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if 'adamw' in r['Kernel_Name']]
    steps = list(zip(ends[a.skip:-1], ends[a.skip + 1:]))
    agg = collections.defaultdict(lambda: [0.0, 0])
    wall = 0.0
    for lo, hi in steps:
        wall += (int(rows[hi]['End_Timestamp']) - int(rows[lo]['End_Timestamp'])) / 1e3
        for r in rows[lo + 1:hi + 1]:
            k = r['Kernel_Name'].split('(')[0][:90]
            agg[k][0] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
            agg[k][1] += 1
    n = len(steps)
    busy = sum(v[0] for v in agg.values()) / n
    print(f'{n} steps: wall {wall / n:.1f} us/step, kernel busy {busy:.1f} us/step')
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f'{t / n:9.1f} us {100 * t / n / busy:5.1f}%  x{c / n:5.1f}  {k}')


if __name__ == '__main__':
    main()
