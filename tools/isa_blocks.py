#!/usr/bin/env python3
"""Per-basic-block instruction counts of one kernel in a device assembly file
(hipcc --cuda-device-only -S): scratch, DPP FMAs, LDS, VALU, SALU, waitcnt.
usage: python tools/isa_blocks.py FILE.s KERNEL_SYMBOL_SUBSTRING"""
import re
import sys

src = open(sys.argv[1]).read()
key = sys.argv[2]
m = re.search(r"^(\S*" + re.escape(key) + r"\S*):", src, re.M)
if not m:
    sys.exit("kernel not found")
i = m.end()
j = src.index(".Lfunc_end", i)
blk, order, cnt = "entry", ["entry"], {"entry": [0] * 6}
for line in src[i:j].split("\n"):
    lm = re.match(r"^(\.LBB\d+_\d+):", line)
    if lm:
        blk = lm.group(1)
        order.append(blk)
        cnt[blk] = [0] * 6
        continue
    t = line.strip()
    c = cnt[blk]
    if t.startswith("scratch_") or t.startswith("buffer_"):
        c[0] += 1
    if t.startswith("v_fmac_f64_dpp"):
        c[1] += 1
    if t.startswith("ds_"):
        c[2] += 1
    if t.startswith("v_"):
        c[3] += 1
    if t.startswith("s_") and not t.startswith("s_waitcnt") and not t.startswith("s_nop"):
        c[4] += 1
    if t.startswith("s_waitcnt"):
        c[5] += 1
print(f"{'block':14s} scratch   dpp    ds  valu  salu  wait")
for b in order:
    print(f"{b:14s} " + " ".join(f"{v:5d}" for v in cnt[b]))
