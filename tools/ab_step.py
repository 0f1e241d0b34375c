"""Whole-step A/B without touching the package: set module attributes, then run bench.py.

    python tools/ab_step.py wgrad.enabled=0 wgrad._NSTREAMS=1 -- --sections train --steps 20

Each `module.attr=value` (int / float / True / False) is set after importing the module from
kd-pointcloud_amd; everything after `--` goes to bench.main().
"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kd-pointcloud_amd"))


def parse(v):
    if v in ("True", "False"):
        return v == "True"
    try:
        return int(v)
    except ValueError:
        return float(v)


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    for a in argv[:cut]:
        key, val = a.split("=")
        mod, attr = key.rsplit(".", 1)
        m = importlib.import_module(mod)
        assert hasattr(m, attr), key
        setattr(m, attr, parse(val))
        print(f"set {key} = {getattr(m, attr)!r}", flush=True)
    import bench
    bench.main(argv[cut + 1:])


if __name__ == "__main__":
    main()
