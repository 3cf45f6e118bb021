"""Static per-source-line instruction / spill counts of the rmsc03 run kernel (or of the kernel
whose mangled name starts with $MXA_ISA_KERNEL, e.g. _Z15mxa_step_kernelILi3ELb0ELb1E).
usage: python tools/isa_lines.py [extra hipcc flags]   (device-only compile with line tables)"""
import collections
import os
import re
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(R, "marl-optimal-execution_amd/csrc/mxa_api.hip")
out = "/tmp/isa_lines.s"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-ffp-contract=off", "-fno-fast-math", "-mllvm", "-structurizecfg-skip-uniform-regions",
       "-DMXA_ONLY_RMSC03", "--cuda-device-only", "-S", "-gline-tables-only",
       "-I" + os.path.join(R, "marl-optimal-execution_amd/csrc"), "-I" + os.path.join(R, "include"), src, "-o", out] + sys.argv[1:]
subprocess.check_call(cmd, stderr=subprocess.DEVNULL)
s = open(out).read()
files = {m.group(1): m.group(3) for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', s)}
i = s.find(":\n", s.find("\n" + os.environ.get("MXA_ISA_KERNEL", "_Z14mxa_run_kernel")))
body = s[i:s.find(".Lfunc_end", i)]
cur = None
ins = collections.Counter()
spl = collections.Counter()
sal = collections.Counter()
for l in body.splitlines():
    l = l.strip()
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        cur = (os.path.basename(files.get(m.group(1), m.group(1))), int(m.group(2)))
        continue
    if not l or l[0] in ".;_" or l.endswith(":"):
        continue
    ins[cur] += 1
    if l.startswith("s_") and not l.startswith(("s_waitcnt", "s_cbranch", "s_branch", "s_nop", "s_load", "s_buffer")):
        sal[cur] += 1
    if l.startswith("scratch_"):
        spl[cur] += 1
print("total", sum(ins.values()), "scratch", sum(spl.values()))
srcs = {}
def text(f, n):
    p = os.path.join(R, "marl-optimal-execution_amd/csrc", f)
    if p not in srcs:
        srcs[p] = open(p).read().splitlines() if os.path.exists(p) else []
    return srcs[p][n - 1].strip()[:70] if 0 < n <= len(srcs[p]) else ""
print("-- top lines by scratch ops")
for k, v in spl.most_common(25):
    print("%5d %6d %s:%d  %s" % (v, ins[k], k[0], k[1], text(*k)))
print("-- top lines by instructions (scratch, all, SALU)")
for k, v in ins.most_common(40):
    print("%5d %6d %5d %s:%d  %s" % (spl[k], v, sal[k], k[0], k[1], text(*k)))
print("-- top lines by SALU")
for k, v in sal.most_common(40):
    print("%5d %6d %5d %s:%d  %s" % (spl[k], ins[k], v, k[0], k[1], text(*k)))
