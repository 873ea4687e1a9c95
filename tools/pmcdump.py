#!/usr/bin/env python3
"""Average every PMC counter per kernel over the passes under a rocprofv3
output directory (tools/pmc_conv.sh) and print one table per kernel.

    python tools/pmcdump.py gpurun_out/pmc_conv
"""
import collections
import csv
import glob
import os
import sys


def main(root):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, '*', '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0].replace('void ', '')
            agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, cs in sorted(agg.items()):
        print(f'## {k}')
        for c, v in sorted(cs.items()):
            print(f'  {c:36s} {sum(v) / len(v):16.4g}   (n={len(v)})')


if __name__ == '__main__':
    main(sys.argv[1])
