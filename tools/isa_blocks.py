#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a hipcc -S (gfx950) listing.
usage: isa_blocks.py file.s kernel_substring"""
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r"^(\S*%s\S*):" % re.escape(sys.argv[2]), s, re.M)
start = m.end()
body = s[start:s.index(".Lfunc_end", start)]
blk, order, cnt = "entry", ["entry"], {"entry": [0, 0, 0, 0, ""]}
for l in body.split("\n"):
    t = l.strip()
    if re.match(r"^\.LBB\S+:", t):
        blk = t.split(":")[0]
        order.append(blk)
        cnt[blk] = [0, 0, 0, 0, ""]
        continue
    if not t or t.startswith(";") or t.startswith("."):
        continue
    op = t.split()[0]
    c = cnt[blk]
    if op.startswith("v_"):
        c[0] += 1
    elif op.startswith("ds_"):
        c[1] += 1
    elif op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"):
        c[2] += 1
    else:
        c[3] += 1
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        c[4] = t
for b in order:
    c = cnt[b]
    print("%-14s valu %4d ds %3d vmem %3d other %4d  %s" % (b, c[0], c[1], c[2], c[3], c[4]))
