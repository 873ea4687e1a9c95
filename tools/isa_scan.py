#!/usr/bin/env python3
"""Scan the gfx950 code objects embedded in a shared library for instructions:
the clang offload bundles of every translation unit are carved out of the
.so, disassembled with llvm-objdump, and counted per kernel.

  python tools/isa_scan.py synthetic-audio-detection_amd/sad/libsad.so 'v_pk_(fma|mul|add)_f32'

Round 6: packed-FP32 VALU instructions returned wrong values
when MFMA instructions of another wave ran on the same CU (the front end beside
the stem, or beside a kernel of bare MFMA chains: tools/fe_concurrency.py);
libsad is built without them (csrc/Makefile NOPK), and tests/test_isa_scan.py
checks the build."""
import collections
import os
import re
import struct
import subprocess
import sys
import tempfile

OBJDUMP = '/opt/rocm/lib/llvm/bin/llvm-objdump'


def code_objects(path: str, arch: str = 'gfx950'):
    """The `arch` code objects of every clang offload bundle in `path`."""
    data = open(path, 'rb').read()
    out, start = [], 0
    while True:
        i = data.find(b'__CLANG_OFFLOAD_BUNDLE__', start)
        if i < 0:
            return out
        n = struct.unpack_from('<Q', data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from('<QQQ', data, p)
            triple = data[p + 24:p + 24 + tl].decode(errors='replace')
            p += 24 + tl
            if arch in triple:
                out.append(data[i + off:i + off + size])
        start = i + 24


def scan(path: str, pattern: str):
    """{kernel symbol: count of instructions matching `pattern`}, and the number
    of code objects scanned."""
    rx = re.compile(pattern)
    counts = collections.Counter()
    cos = code_objects(path)
    with tempfile.TemporaryDirectory() as d:
        for k, co in enumerate(cos):
            f = os.path.join(d, f'co{k}.o')
            open(f, 'wb').write(co)
            dis = subprocess.run([OBJDUMP, '-d', f], capture_output=True, text=True, check=True).stdout
            cur = None
            for line in dis.splitlines():
                m = re.match(r'^[0-9a-f]+ <(.+)>:', line)
                if m:
                    cur = m.group(1)
                elif rx.search(line):
                    counts[cur] += 1
    return counts, len(cos)


def main(argv):
    counts, n = scan(argv[0], argv[1])
    for k, c in counts.most_common():
        print(f'{c:6d}  {k}')
    print(f'{sum(counts.values())} matches in {len(counts)} kernels ({n} code objects)')
    return 1 if counts else 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1:]))
