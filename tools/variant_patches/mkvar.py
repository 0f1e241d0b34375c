"""Diagnostic library variants (never committed): copy the package to /tmp/var_<name>, apply
text replacements, build, and copy the libs to ab/<name>/ (run with KDPC_LIB=ab/<name>/libkdpc_hip.so).
    python tools/variant_patches/mkvar.py <name> <patchfile.py>  (VAR_OUT=tools/variants/out to ship to the GPU box)
patchfile defines REPL = [(relpath under kd-pointcloud_amd, old, new), ...]"""
import os, shutil, subprocess, sys, runpy
name, pf = sys.argv[1], sys.argv[2]
root = "/root/repo"
dst = f"/tmp/var_{name}"
shutil.rmtree(dst, ignore_errors=True)
os.makedirs(dst)
shutil.copytree(f"{root}/kd-pointcloud_amd", f"{dst}/kd-pointcloud_amd", ignore=shutil.ignore_patterns("__pycache__"))
shutil.copytree(f"{root}/include", f"{dst}/include")
for rel, old, new in runpy.run_path(pf)["REPL"]:
    p = f"{dst}/kd-pointcloud_amd/{rel}"
    s = open(p).read()
    assert s.count(old) >= 1, (rel, old[:80])
    s = s.replace(old, new)
    open(p, "w").write(s)
subprocess.check_call([sys.executable, f"{dst}/kd-pointcloud_amd/build_native.py"])
out = os.environ.get("VAR_OUT", f"{root}/ab")  # ab/ stays off GPU snapshots; tools/variants/out travels
os.makedirs(f"{out}/{name}", exist_ok=True)
for f in ("libkdpc_hip.so", "libkdpc_torch.so"):
    shutil.copy(f"{dst}/kd-pointcloud_amd/lib/{f}", f"{out}/{name}/{f}")
print("ok", name)
