"""Build the gfx950 HIP library behind the C ABI (include/kdpc.h).

    python kd-pointcloud_amd/build_native.py        # -> kd-pointcloud_amd/lib/libkdpc_hip.so

Plain hipcc (no torch headers): each csrc/*.hip is compiled to an object in parallel and
linked into one shared library.  Objects are rebuilt only when a source or header is newer.
"""
import concurrent.futures
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "lib", "libkdpc_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("KDPC_ARCH", "gfx950")

CFLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    "-ffp-contract=off",            # every fma the parity contract needs is explicit
    "-fvisibility=hidden",          # only KDPC_API symbols are exported
    "-Wall", "-Wno-unused-result",
    "-I", os.path.join(ROOT, "include"), "-I", CSRC,
]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    deps = [src] + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(ROOT, "include", "kdpc.h")]
    if _newer(obj, deps):
        cmd = [HIPCC] + CFLAGS + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    if _newer(LIB, objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    try:
        build()
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
