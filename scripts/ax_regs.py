#!/usr/bin/env python3
"""Registers, scratch and occupancy of every k_scan_ax instantiation from a hipcc -Rpass-analysis=kernel-resource-usage
log: python scripts/ax_regs.py build.log"""
import re
import sys

log = open(sys.argv[1]).read()
for b in re.split(r'remark: [^\n]*Function Name: ', log)[1:]:
    name = b.split('\n')[0]
    if 'k_scan_ax' not in name:
        continue

    def g(k):
        m = re.search(k + r': (\d+)', b)
        return m.group(1) if m else '?'
    args = re.search(r'k_scan_axIL(.*)EEEv', name)
    scratch, occ = g(r'ScratchSize \[bytes/lane\]'), g(r'Occupancy \[waves/SIMD\]')
    print(f"{args.group(1) if args else name:40s} VGPR {g('VGPRs'):>4} AGPR {g('AGPRs'):>3} scratch {scratch:>4} occ {occ}")
