#!/usr/bin/env python3
"""Instruction mix per kernel of a hipcc -S (device-only) assembly file.
   tools/isa_count.py file.s [name-regex]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
flt = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
pat = r"^\s+(ds_\w+|global_\w+|v_min\w*|v_max\w*|s_waitcnt|v_cndmask\w*|scratch_\w+|buffer_\w+|s_barrier|v_mov_b32_dpp|v_perm\w*)"
for m in re.finditer(r"^(_Z\S*):\s*;.*?\n(.*?)s_endpgm", s, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if not flt.search(name):
        continue
    c = collections.Counter(re.findall(pat, body, re.M))
    total = len(re.findall(r"^\s+[sv]_\w+|^\s+ds_\w+|^\s+global_\w+", body, re.M))
    print(name[:100], "instrs=%d" % total)
    print("   ", dict(sorted(c.items())))
