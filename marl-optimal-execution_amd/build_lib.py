"""Build libmxa.so (HIP, gfx950) in-tree: marl-optimal-execution_amd/lib/libmxa.so."""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "mxa_api.hip")
OUT = os.path.join(HERE, "lib", "libmxa.so")
DEPS = ["mxa_api.hip", "mxa_kernels.hip", "mxa_layout.h", "mxa_config.h", "glibc_math.h", "glibc_math_tables.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++20", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
         "-Wno-unused-result", "-Wno-unused-value"]


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
    return h.hexdigest()[:16]


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(s) <= t for s in sources())


def build(force=False, verbose=True):
    if not force and up_to_date():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [HIPCC] + FLAGS + ['-DMXA_BUILD_ID="%s"' % build_id(), "-I" + os.path.join(HERE, "csrc"),
                            "-I" + os.path.join(ROOT, "include"), SRC, "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
