"""Build the in-tree HIP extension ``fairify_amd/_C*.so`` for gfx950 with hipcc.

No hipify, no torch C++ headers: the kernels are plain HIP, the bindings plain pybind11, and
everything is compiled by ``hipcc --offload-arch=gfx950`` (cross-compiles without a GPU).
Objects are cached under ``build/`` and rebuilt when a source or header is newer.

    python -m fairify_amd.csrc.build            # or: python setup.py build_ext --inplace
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_C" + suffix)


def _flags(debug: bool):
    import pybind11

    inc = [f"-I{HERE}", f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    opt = ["-O0", "-g"] if debug else ["-O3"]
    # FAIRIFY_HIPCC_DEFINES="A=1 B=2": extra -D flags (occupancy A/B builds, tools/variants)
    defs = ["-D" + d for d in os.environ.get("FAIRIFY_HIPCC_DEFINES", "").split() if d]
    # loops bounded by a template tile count but exited early at the layer's width ("if (t >= tin)
    # break") unroll only up to LLVM's upper-bound limit of 8 trips: the 10-tile kernels (BM-4's
    # 150-wide layer) kept their operand arrays in scratch (points 656 B/lane, refine 336 B/lane)
    unroll = ["-mllvm", "-unroll-max-upperbound=16"]
    return inc + opt + defs + unroll + ["-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result"]


def _newer(src: str, obj: str, headers) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or any(os.path.getmtime(h) > t for h in headers)


def build(debug: bool = False, verbose: bool = False, jobs: int = 4, out: str = None, tag: str = "") -> str:
    out = out or ext_path()
    bdir = os.path.join(ROOT, "build", "hip-" + ARCH + ("-dbg" if debug else "") + (("-" + tag) if tag else ""))
    os.makedirs(bdir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(HERE, "*.hip"))) + sorted(glob.glob(os.path.join(HERE, "*.cpp")))
    headers = glob.glob(os.path.join(HERE, "*.h"))
    flags = _flags(debug)
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(bdir, os.path.basename(s) + ".o")
        objs.append(o)
        if _newer(s, o, headers):
            todo.append((s, o))

    def compile_one(so):
        s, o = so
        cmd = [HIPCC] + flags + ["-c", s, "-o", o]
        if s.endswith(".cpp"):
            cmd = [HIPCC] + [f for f in flags if not f.startswith("--offload-arch")] + ["-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {s}:\n{r.stderr}")
        return o

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(compile_one, todo))
    if todo or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + objs + ["-o", out]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    return out


if __name__ == "__main__":
    # python -m fairify_amd.csrc.build [--debug] [--out PATH --tag NAME]  (variant builds go to PATH)
    argv = sys.argv[1:]
    kw = {}
    if "--out" in argv:
        kw["out"] = argv[argv.index("--out") + 1]
    if "--tag" in argv:
        kw["tag"] = argv[argv.index("--tag") + 1]
    print(build(debug="--debug" in argv, verbose=True, **kw))
