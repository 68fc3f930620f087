#!/usr/bin/env python3
"""Static VALU / SALU instruction counts of the kernels in a gfx950 assembly file
(`hipcc --cuda-device-only -S`) whose mangled name contains a pattern.
usage: isa_count.py FILE.s PATTERN"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    pat = sys.argv[2]
    for m in re.finditer(r'^(_Z[^:\s]*):', s, re.M):
        name = m.group(1)
        if pat not in name:
            continue
        body = s[m.end():]
        body = body[:body.index('.Lfunc_end')]
        ins = [ln.strip() for ln in body.split('\n')]
        ins = [ln for ln in ins if ln[:2] in ('v_', 's_')]
        print(name[:100], 'VALU', sum(ln.startswith('v_') for ln in ins), 'SALU', sum(ln.startswith('s_') for ln in ins))


if __name__ == '__main__':
    main()
