#!/usr/bin/env python3
"""Audit of the inline-asm MFMA kernels' generated code: hipcc's
hazard recognizer does not see MFMAs written as inline asm (the resident-weight
kernels l1block.hip / l2conv.hip use them for their AGPR weight operands), so a
compiler instruction that reads or overwrites an MFMA's destination too soon
after it -- e.g. a register copy the allocator inserts -- reads a stale
accumulator silently.  The 8-pass XDL result needs 12 wait states before any
reader other than the next MFMA taking it whole as C
(/opt/skills/guides/cdna_hip_programming.md, inline-asm rule 2).

Scans every kernel of the given sources (hipcc -S for gfx950) linearly: for each
inline-asm v_mfma (between ;;#ASMSTART / ;;#ASMEND; hipcc pads its own), the
instructions in the following 12 wait states (one per instruction, N + 1 per
s_nop N, 4 per intervening MFMA -- the wave cannot issue it before the XDL pipe
frees, >= 16 cycles) must not read or write its destination registers, except
an MFMA whose C and D are exactly that range (an accumulation chain).  Prints the
violations; exit status 1 if any.

    python tools/asm_hazards.py synthetic-audio-detection_amd/csrc/l1block.hip ...
"""
import os
import re
import subprocess
import sys
import tempfile

HIPCC = '/opt/rocm/bin/hipcc'
FLAGS = ['-O3', '-std=c++17', '-fPIC', '--offload-arch=gfx950', '-munsafe-fp-atomics', '--cuda-device-only', '-S']
STATES = 12

_RANGE = re.compile(r'\bv\[(\d+):(\d+)\]|\bv(\d+)\b')


def regs(text):
    out = set()
    for m in _RANGE.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def instructions(asm, name):
    """(kernel, [instruction lines]) for every kernel in the .s text"""
    kernels = {}
    for m in re.finditer(r'^(_Z\w+):\s*(?:;.*)?$', asm, re.M):
        k = m.group(1)
        end = asm.find('.Lfunc_end', m.end())
        body, in_asm = [], False
        for raw in asm[m.end():end].split('\n'):
            if ';;#ASMSTART' in raw:
                in_asm = True
            if ';;#ASMEND' in raw:
                in_asm = False
            line = raw.split(';')[0].strip()
            if not line or line.startswith('.') or line.endswith(':'):
                continue
            # inline-asm MFMAs are marked: the compiler pads only its own
            body.append(line + (' ;asm' if in_asm and line.startswith('v_mfma') else ''))
        kernels[k] = body
    return kernels


def audit(body):
    bad = []
    for i, ins in enumerate(body):
        if not (ins.startswith('v_mfma') and ins.endswith(';asm')):
            continue
        ops = [o.strip() for o in ins[:-4].split(None, 1)[1].split(',')]
        dst = regs(ops[0])
        if not dst:
            continue  # AGPR destination: not used here
        states = 0
        for j in range(i + 1, len(body)):
            nxt = body[j]
            op = nxt.split()[0]
            if op == 's_nop':
                states += int(nxt.split()[1], 0) + 1
                if states >= STATES:
                    break
                continue
            if op.startswith(('s_', 'buffer_', 'global_', 'ds_')) and not regs(nxt):
                states += 1
                if states >= STATES:
                    break
                continue
            if op.startswith('v_mfma'):
                o2 = [o.strip() for o in nxt.replace(' ;asm', '').split(None, 1)[1].split(',')]
                d2, a2, b2, c2 = regs(o2[0]), regs(o2[1]), regs(o2[2]), regs(o2[3]) if len(o2) > 3 else set()
                if (a2 | b2) & dst or ((c2 & dst) and not (c2 == dst and d2 == dst)) or ((d2 & dst) and d2 != dst):
                    bad.append((i, ins, nxt, states))
                # an intervening MFMA holds the wave >= 16 cycles (the XDL pipe
                # is busy with the one before it): counted as 4 wait states
                states += 4
                if states >= STATES:
                    break
                continue
            elif regs(nxt) & dst:
                bad.append((i, ins, nxt, states))
            states += 1
            if states >= STATES:
                break
    return bad


def main(paths):
    total = 0
    for p in paths:
        with tempfile.TemporaryDirectory() as d:
            out = os.path.join(d, 'k.s')
            subprocess.run([HIPCC, *FLAGS, p, '-o', out], check=True, capture_output=True)
            asm = open(out).read()
        for k, body in instructions(asm, p).items():
            if not any(l.startswith('v_mfma') for l in body):
                continue
            bad = audit(body)
            total += len(bad)
            print(f'{os.path.basename(p)} {k[:70]}: {len(bad)} MFMA-result hazards')
            for i, a, b, st in bad[:6]:
                print(f'    [{i}] {a}\n        -> after {st} states: {b}')
    return 1 if total else 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1:]))
