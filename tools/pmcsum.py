#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc (+ --kernel-trace) directory: per kernel
(template name with 'unsigned short' -> u16, grid size) the mean of each counter
per launch, the mean duration, and for GRBM_GUI_ACTIVE the effective clock
(counter / 8 XCDs / duration)."""
import collections
import csv
import glob
import sys


def short(name):
    return name.split('(')[0].replace('void ', '').replace('unsigned short', 'u16').replace('sad::', '')


def main(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in glob.glob(d + '/**/run_counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = (short(r['Kernel_Name']), int(r['Grid_Size']))
            agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
    for f in glob.glob(d + '/**/run_kernel_trace.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = (short(r['Kernel_Name']), int(r['Grid_Size_X']) * int(r['Grid_Size_Y']) * int(r.get('Grid_Size_Z', 1)))
            dur[k].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    names = sorted({n for v in agg.values() for n in v})
    hdr = ['kernel', 'grid', 'n', 'avg us'] + names + (['clock GHz'] if 'GRBM_GUI_ACTIVE' in names else [])
    print('| ' + ' | '.join(hdr) + ' |')
    print('|' + '---|' * len(hdr))
    rows = []
    for k, v in agg.items():
        n = max(len(x) for x in v.values())
        us = sum(dur[k]) / len(dur[k]) / 1e3 if dur.get(k) else float('nan')
        cells = [f'`{k[0]}`', str(k[1]), str(n), f'{us:.1f}']
        for c in names:
            cells.append(f'{sum(v[c]) / len(v[c]):.4g}' if v.get(c) else '')
        if 'GRBM_GUI_ACTIVE' in names and v.get('GRBM_GUI_ACTIVE') and dur.get(k):
            cells.append(f'{sum(v["GRBM_GUI_ACTIVE"]) / len(v["GRBM_GUI_ACTIVE"]) / 8 / (us * 1e3):.3f}')
        rows.append((us * n if us == us else 0, cells))
    for _, cells in sorted(rows, key=lambda r: -r[0]):
        print('| ' + ' | '.join(cells) + ' |')


if __name__ == '__main__':
    main(sys.argv[1])
