#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel trace + optional PMC passes) into a
markdown table: per kernel shape, launches/step, avg duration, ms/step, share,
and HBM bytes per launch from FETCH_SIZE (x2, gfx950 wide-read correction,
MI355X_MICROARCH.md "HBM") and WRITE_SIZE.

  python tools/profsum.py --trace gpurun_out/prof3 --fetch gpurun_out/pmc_fetch \
      --write gpurun_out/pmc_write --steps 4 > profiles/r01_bench_kernels.md
"""
import argparse
import collections
import csv
import os


def load_trace(d):
    rows = list(csv.DictReader(open(os.path.join(d, 'run_kernel_trace.csv'))))
    agg = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        k = (r['Kernel_Name'].split('(')[0].replace('void ', ''), int(r['Grid_Size_X']) * int(r['Grid_Size_Y']))
        agg[k][0] += 1
        agg[k][1] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    return agg


def load_pmc(d, name):
    if not d:
        return {}
    rows = list(csv.DictReader(open(os.path.join(d, 'run_counter_collection.csv'))))
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        if r['Counter_Name'] != name:
            continue
        k = (r['Kernel_Name'].split('(')[0].replace('void ', ''), int(r['Grid_Size']))
        agg[k][0] += 1
        agg[k][1] += float(r['Counter_Value'])
    return {k: v[1] / v[0] for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--trace', required=True)
    ap.add_argument('--fetch')
    ap.add_argument('--write')
    ap.add_argument('--steps', type=int, required=True, help='steps in the traced run (warmup + timed)')
    ap.add_argument('--json', help='also write {kernel: {avg_us, hbm_read_bytes, hbm_write_bytes}} here '
                                   '(bench.py reads it for roofline.traffic)')
    a = ap.parse_args()
    tr = load_trace(a.trace)
    fe = load_pmc(a.fetch, 'FETCH_SIZE')
    wr = load_pmc(a.write, 'WRITE_SIZE')
    tot = sum(v[1] for v in tr.values()) / a.steps
    if a.json:
        import json
        out = {}
        for k, (n, t) in tr.items():
            f, w = fe.get(k), wr.get(k)
            out[f'{k[0]}|{k[1]}'] = {'avg_us': t / n / 1e3, 'launches_per_step': n / a.steps,
                                     'hbm_read_bytes': None if f is None else 2 * f * 1024,
                                     'hbm_write_bytes': None if w is None else w * 1024}
        json.dump(out, open(a.json, 'w'), indent=1)
    print('| kernel | grid (threads) | launches/step | avg us | ms/step | share | HBM read MB/launch (2xFETCH) | HBM write MB/launch |')
    print('|---|---|---|---|---|---|---|---|')
    for k, (n, t) in sorted(tr.items(), key=lambda x: -x[1][1]):
        ms = t / a.steps / 1e6
        if ms < 0.005:
            continue
        f = fe.get(k)
        w = wr.get(k)
        print(f'| `{k[0]}` | {k[1]} | {n / a.steps:g} | {t / n / 1e3:.1f} | {ms:.2f} | {100 * ms * 1e6 / tot:.1f}% | '
              f'{"" if f is None else f"{2 * f / 1024:.1f}"} | {"" if w is None else f"{w / 1024:.1f}"} |')
    print(f'\nTotal GPU kernel time per step: {tot / 1e6:.2f} ms')


if __name__ == '__main__':
    main()
