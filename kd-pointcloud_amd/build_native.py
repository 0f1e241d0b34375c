"""Build the gfx950 HIP library behind the C ABI (include/kdpc.h).

    python kd-pointcloud_amd/build_native.py        # -> kd-pointcloud_amd/lib/libkdpc_hip.so

Plain hipcc (no torch headers): each csrc/*.hip is compiled to an object in parallel and
linked into one shared library.  Objects are keyed by a hash of everything that determines
them (the source, every header, the flags and the hipcc version), never by file times, so a
build reuses an object only if it would compile to the same thing.  The library exports
kdpc_build_id() = "<source hash>+<flags hash>+<tool hash>": the sources it was built from
(source_id()), the target arch and compile flags (flags_id()) and the hipcc version
(tool_id()).  kdpc_native refuses to load a library whose source or flags part does not match
the tree next to it (KDPC_ARCH included), and build() relinks unless all three match, so a run
can never use a stale binary or one built for another arch / with other flags.
"""
import concurrent.futures
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "lib", "libkdpc_hip.so")
TORCH_OPS_SRC = os.path.join(HERE, "torch_ops", "kdpc_torch_ops.cpp")
TORCH_OPS_LIB = os.path.join(HERE, "lib", "libkdpc_torch.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("KDPC_ARCH", "gfx950")

CFLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    "-ffp-contract=off",            # every fma the parity contract needs is explicit
    # no packed f32 VALU (v_pk_fma/mul/add_f32, which the SLP and loop vectorisers form from
    # pairs of scalar ops): on the MI355X their results were occasionally wrong while another
    # kernel's waves ran beside them (tools/knn_race.py);
    # tests/test_native_lib.py checks the built library holds none
    "-fno-slp-vectorize", "-fno-vectorize",
    "-fvisibility=hidden",          # only KDPC_API symbols are exported
    "-Wall", "-Wno-unused-result",
    "-I", os.path.join(ROOT, "include"), "-I", CSRC,
]


# per-source extra flags (none at present; SLP packing, off everywhere, also forced the
# cost-volume backward's LDS operands into adjacent registers: 182 -> >256 VGPRs)
# Adam's update is compiled the way torch compiles its fused Adam (clang's default HIP
# contraction; adam_fastdiv.hip also with fast f32 division / sqrt), see csrc/adam_math.h
EXTRA_FLAGS = {
    "adam.hip": ["-ffp-contract=fast-honor-pragmas"],
    "adam_fastdiv.hip": ["-ffp-contract=fast-honor-pragmas",
                         "-fno-hip-fp32-correctly-rounded-divide-sqrt"],
}


def source_files(csrc=CSRC, root=ROOT):
    """Every file the library is built from, in a fixed order."""
    return (sorted(glob.glob(os.path.join(csrc, "*.hip"))) +
            sorted(glob.glob(os.path.join(csrc, "*.h"))) + [os.path.join(root, "include", "kdpc.h")])


def source_id(csrc=CSRC, root=ROOT):
    """sha256 over the names and contents of the library's sources (what kdpc_build_id()
    of a library built from them returns)."""
    h = hashlib.sha256()
    for p in source_files(csrc, root):
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


def _hipcc_version():
    r = subprocess.run([HIPCC, "--version"], capture_output=True, text=True)
    return r.stdout


def flags_id():
    """Hash of the target arch and every compile flag (per-source extras included); the tree's
    own include paths enter relative to it (the GPU box runs a copy at another path)."""
    h = hashlib.sha256()
    flags = [f.replace(ROOT, "<root>") for f in CFLAGS]
    h.update(ARCH.encode() + b"\0" + " ".join(flags).encode())
    for k in sorted(EXTRA_FLAGS):
        h.update(b"\0" + k.encode() + b"=" + " ".join(EXTRA_FLAGS[k]).encode())
    return h.hexdigest()[:16]


def tool_id(tool=None):
    """Hash of the hipcc version text."""
    return hashlib.sha256((tool if tool is not None else _hipcc_version()).encode()).hexdigest()[:16]


def build_id(sid=None, tool=None):
    """The string a library built now from this tree embeds as kdpc_build_id()."""
    return f"{sid or source_id()}+{flags_id()}+{tool_id(tool)}"


def _compile(src, headers_digest, tool):
    h = hashlib.sha256()
    with open(src, "rb") as f:
        h.update(f.read())
    h.update(headers_digest.encode())
    flags = CFLAGS + EXTRA_FLAGS.get(os.path.basename(src), [])
    h.update(" ".join(flags).encode())
    h.update(tool.encode())
    obj = os.path.join(OBJ, f"{os.path.basename(src)}.{h.hexdigest()[:16]}.o")
    if not os.path.exists(obj):
        tmp = obj + ".tmp"
        r = subprocess.run([HIPCC] + flags + ["-c", src, "-o", tmp], capture_output=True,
                           text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        os.replace(tmp, obj)
    return obj


def _torch_flags():
    """Compile / link flags for a host-only op library against this torch-ROCm install."""
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api",
                                                       "include")]
    abi = int(torch.compiled_with_cxx11_abi())
    cflags = ["-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall",
              "-Wno-unused-variable", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
              f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", os.path.join(ROOT, "include"),
              "-I", "/opt/rocm/include"] + [f for i in inc for f in ("-isystem", i)]
    ldflags = ["-shared", "-L", os.path.join(tdir, "lib"), "-lc10", "-lc10_hip", "-ltorch",
               "-ltorch_cpu", "-ltorch_hip", "-lamdhip64",
               "-L", os.path.dirname(LIB), "-lkdpc_hip",
               "-Wl,-rpath,$ORIGIN", "-Wl,-rpath," + os.path.join(tdir, "lib")]
    return cflags, ldflags, torch.__version__


def build_torch_ops(verbose=True):
    """torch.ops.kdpc (torch_ops/kdpc_torch_ops.cpp) -> lib/libkdpc_torch.so, linked to
    libkdpc_hip.so.  Rebuilt when the op source, the C ABI header, the flags, the torch
    version or the HIP library's sources change."""
    cflags, ldflags, tv = _torch_flags()
    h = hashlib.sha256()
    for p in (TORCH_OPS_SRC, os.path.join(ROOT, "include", "kdpc.h")):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(cflags + ldflags).encode() + tv.encode() + source_id().encode())
    key = h.hexdigest()
    stamp = TORCH_OPS_LIB + ".inputs"
    if os.path.exists(TORCH_OPS_LIB) and os.path.exists(stamp) and open(stamp).read() == key:
        return TORCH_OPS_LIB
    tmp = TORCH_OPS_LIB + ".tmp"
    r = subprocess.run(["g++"] + cflags + [TORCH_OPS_SRC, "-o", tmp] + ldflags,
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"torch op library failed to build:\n{r.stderr[-6000:]}")
    os.replace(tmp, TORCH_OPS_LIB)
    with open(stamp, "w") as f:
        f.write(key)
    if verbose:
        print(f"built {TORCH_OPS_LIB}")
    return TORCH_OPS_LIB


def _lib_current(bid):
    """The shipped library was linked from exactly these sources, for this arch, with these
    flags and this hipcc (its kdpc_build_id string is embedded in the binary): nothing to
    compile.  The GPU box receives lib/ with the tree (the
    driver runs the GPU tests there without building) but not build/, so without this check a
    build() there would recompile every object only to find the link up to date."""
    try:
        with open(LIB, "rb") as f:
            return bid.encode() in f.read()
    except OSError:
        return False


def build(verbose=True):
    sid = source_id()
    tool = _hipcc_version()
    bid = build_id(sid, tool)
    if _lib_current(bid):
        if verbose:
            print(f"{LIB} is current (sources {sid[:12]})")
        build_torch_ops(verbose)
        return LIB
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hd = hashlib.sha256()
    for p in source_files()[len(srcs):]:
        with open(p, "rb") as f:
            hd.update(f.read())
    with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, hd.hexdigest(), tool), srcs))
    # the build id: a one-function host object naming the sources' hash
    idsrc = os.path.join(OBJ, "kdpc_build_id.cpp")
    with open(idsrc, "w") as f:
        f.write('extern "C" __attribute__((visibility("default"))) const char* '
                f'kdpc_build_id(void) {{ return "{bid}"; }}\n')
    idobj = _compile(idsrc, hd.hexdigest(), tool)
    stamp = LIB + ".inputs"
    link_key = "\n".join(objs + [idobj])
    old = open(stamp).read() if os.path.exists(stamp) else None
    if old != link_key or not os.path.exists(LIB):
        tmp = LIB + ".tmp"
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", tmp] + objs + [idobj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, LIB)
        with open(stamp, "w") as f:
            f.write(link_key)
    for o in glob.glob(os.path.join(OBJ, "*.o")):  # objects of superseded sources
        if o not in objs and o != idobj:
            os.remove(o)
    if verbose:
        print(f"built {LIB} (sources {sid[:12]})")
    build_torch_ops(verbose)
    return LIB


if __name__ == "__main__":
    try:
        build()
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
