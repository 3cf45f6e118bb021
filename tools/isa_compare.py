#!/usr/bin/env python3
"""Per-kernel resource use and instruction count of two device assembly files (hipcc
--cuda-device-only -S): the check that a change leaves an unrelated configuration's kernels alone.
    python tools/isa_compare.py old.s new.s"""
import re
import sys


def kernels(path):
    txt = open(path).read()
    meta = {}
    for blk in re.split(r"\n\s+- \.", txt.split("amdhsa.kernels:", 1)[1].split("amdhsa.target", 1)[0]):
        name = re.search(r"\.name:\s+(\S+)", blk)
        if not name:
            continue
        g = lambda k: (re.search(r"\.%s:\s+(\d+)" % k, blk) or [None, "?"])[1]
        meta[name.group(1)] = {k: g(k) for k in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count",
                                                  "sgpr_spill_count", "private_segment_fixed_size")}
    for name in meta:
        m = re.search(r"^%s:.*?\n(.*?)^\s*s_endpgm" % re.escape(name), txt, re.S | re.M)
        body = m.group(1).splitlines() if m else []
        meta[name]["insts"] = sum(1 for l in body if l.strip() and not l.strip().startswith((".", ";", "//"))
                                  and not l.rstrip().endswith(":"))
    return meta


a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
for k in sorted(set(a) | set(b)):
    short = re.sub(r"_Z\d+", "", k)[:60]
    print(short, a.get(k), "\n" + " " * len(short), b.get(k), "" if a.get(k) == b.get(k) else "  <-- differs")
