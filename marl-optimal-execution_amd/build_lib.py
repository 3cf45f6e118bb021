"""Build libmxa.so (HIP, gfx950) in-tree: marl-optimal-execution_amd/lib/libmxa.so.

The C-ABI (csrc/mxa_api.hip) and each configuration's engine (csrc/mxa_inst.hip with
-DMXA_INST_CFG=<id>) are separate translation units compiled in parallel, then linked."""
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "mxa_api.hip")
INST = os.path.join(HERE, "csrc", "mxa_inst.hip")
OUT = os.path.join(HERE, "lib", "libmxa.so")
OBJ = os.path.join(HERE, "build")
N_CONFIGS = 18  # csrc/mxa_entry.h MXA_N_CONFIGS
DEPS = ["mxa_api.hip", "mxa_inst.hip", "mxa_entry.h", "mxa_kernels.hip", "mxa_layout.h", "mxa_config.h", "glibc_math.h",
        "glibc_math_tables.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -structurizecfg-skip-uniform-regions: branches on wave-uniform conditions stay plain scalar
# branches instead of being structurized into exec-mask regions (saveexec / restore pairs and
# flow blocks on the event loop's paths).  The CU's one scalar unit is what bounds the run kernel
# (instruction issue); same per-env digests, r05: rmsc03 x4096 41.0 -> 38.3 ms,
# sparse_zi_1000 x1024 720.5 -> 607.8 ms (profiles/r05/ab_mr/ab_flags.txt)
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++20", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
         "-Wno-unused-result", "-Wno-unused-value", "-mllvm", "-structurizecfg-skip-uniform-regions"]

# per-configuration backend options (config id -> extra flags of its translation unit).  The
# max-ILP scheduler, same digests (profiles/r05/ab_mr/ab_sched.txt): the ABIDESEnv replay step
# kernel (config 3, one wave per SIMD on a serial chain) IBM x512 0.3229 -> 0.3177 ms and GOOG
# 0.4656 -> 0.4575 ms per step; sparse_zi_100 (1) 105.3 -> 103.9 ms.  It cost sparse_zi_1000
# 1.5 %, rmsc03 1.8 %, rmsc01 2.5 %, random_fund_* 0.5-1 %, rmsc02 neutral: those keep the default.
# A/B variant builds (tools/build_variants.sh) pass it themselves.
# Without SLP vectorisation, sparse_zi_1000's run kernel (config 2) 607 -> 596 ms, same digests; it
# cost rmsc01 7 % and value_noise 3.5 %, and left rmsc02, sparse_zi_100, random_fund_value and the
# replay unchanged (profiles/r06/ab/ab19_noslp_*.txt): config 2 only.
CFG_FLAGS = {1: ["-mllvm", "-amdgpu-sched-strategy=max-ilp"], 2: ["-fno-slp-vectorize"],
             3: ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]}


def sources():
    return [os.path.join(HERE, "csrc", d) for d in DEPS] + [os.path.join(ROOT, "include", "mxa.h")]


def build_id(extra=()):
    """hash of the kernel sources and compile flags (mxa_build_id()): profile records name the
    build they were measured on"""
    h = hashlib.sha256()
    for s in sources():
        with open(s, "rb") as f:
            h.update(f.read())
    h.update(" ".join(FLAGS + list(extra)).encode())
    h.update(repr(sorted(CFG_FLAGS.items())).encode())
    return h.hexdigest()[:16]


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(s) <= t for s in sources() + [os.path.abspath(__file__)])


def build(force=False, verbose=True, jobs=None):
    if not force and up_to_date():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    os.makedirs(OBJ, exist_ok=True)
    inc = ["-I" + os.path.join(HERE, "csrc"), "-I" + os.path.join(ROOT, "include")]
    cflags = [f for f in FLAGS if f != "-shared"] + ["-c"]
    # the compile line of the runtime compositions' specialisations (mxa_config_compile) is this one
    jit = ['-DMXA_JIT_FLAGS="%s"' % " ".join(FLAGS),
           '-DMXA_JIT_CFG_FLAGS="%s"' % ";".join("%d:%s" % (c, " ".join(f)) for c, f in sorted(CFG_FLAGS.items()))]
    units = [([HIPCC] + cflags + ['-DMXA_BUILD_ID="%s"' % build_id()] + jit + inc + [SRC, "-o", os.path.join(OBJ, "mxa_api.o")])]
    for c in range(N_CONFIGS):
        units.append([HIPCC] + cflags + CFG_FLAGS.get(c, []) + ["-DMXA_INST_CFG=%d" % c] + inc +
                     [INST, "-o", os.path.join(OBJ, "mxa_inst_%d.o" % c)])
    if verbose:
        for u in units:
            print(" ".join(u), flush=True)
    jobs = jobs or min(len(units), max(1, min(16, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        for f in [ex.submit(subprocess.check_call, u) for u in units]:
            f.result()
    link = [HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared"] + [u[-1] for u in units] + ["-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(link), flush=True)
    subprocess.check_call(link)
    os.replace(OUT + ".tmp", OUT)
    return OUT


DDQN_SRC = os.path.join(HERE, "csrc", "ddqn_period.hip")
DDQN_OUT = os.path.join(HERE, "lib", "libmxa_ddqn.so")


def build_ddqn(force=False, verbose=True):
    """libmxa_ddqn.so: the DDQN learner's per-period bookkeeping kernel (mxabides.ddqn run_episode);
    a library of its own, outside the engine's build id"""
    if not force and os.path.exists(DDQN_OUT) and os.path.getmtime(DDQN_OUT) >= max(
            os.path.getmtime(DDQN_SRC), os.path.getmtime(os.path.abspath(__file__))):
        return DDQN_OUT
    os.makedirs(os.path.dirname(DDQN_OUT), exist_ok=True)
    cmd = [HIPCC] + FLAGS + [DDQN_SRC, "-o", DDQN_OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(DDQN_OUT + ".tmp", DDQN_OUT)
    return DDQN_OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_ddqn(force="--force" in sys.argv)
