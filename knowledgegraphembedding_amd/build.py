"""Build recipe for the HIP shared library (gfx950 only).

    python knowledgegraphembedding_amd/build.py          # incremental
    python knowledgegraphembedding_amd/build.py --clean  # full rebuild

(run as a file it does not import the package, whose __init__ loads the
libraries being replaced; `python -m knowledgegraphembedding_amd.build` works
while the existing libraries still load)

Every csrc/*.hip translation unit is compiled with hipcc for
--offload-arch=gfx950 in parallel and linked into
knowledgegraphembedding_amd/libkge_hip.so, in-tree, so the library travels
with the repository snapshot to the GPU box.  -ffp-contract=off keeps the
per-element arithmetic rounding like the reference's separate ATen ops.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
INCLUDE = PKG.parent / "include"
BUILD = PKG / "_build"
LIB = PKG / "libkge_hip.so"
ARCH = "gfx950"

CFLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-ffp-contract=off",
    "-Wall",
    "-Wno-unused-function",
    f"-I{INCLUDE}",
]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain (ROCm) is required to build knowledgegraphembedding_amd")


def _deps() -> list[Path]:
    return sorted(CSRC.glob("*.h")) + sorted(CSRC.glob("*.inc")) + sorted(INCLUDE.glob("*.h"))


def _stale(obj: Path, src: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(p.stat().st_mtime > t for p in [src, *deps])


def _compile(hipcc: str, src: Path, obj: Path) -> tuple[Path, str]:
    cmd = [hipcc, *CFLAGS, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    return src, r.stderr


TORCH_SRC = CSRC / "torch" / "kge_torch_ops.cpp"
TORCH_LIB = PKG / "libkge_torch.so"


def build_torch_ops(verbose: bool = False) -> Path:
    """libkge_torch.so: the `kge` operator library (TORCH_LIBRARY, csrc/torch/),
    host C++ against libtorch and libkge_hip.so — loaded by torch_ops.py with
    torch.ops.load_library, or linked by a libtorch C++ caller."""
    import torch
    import torch.utils.cpp_extension as cx
    deps = [TORCH_SRC, INCLUDE / "kge_hip.h", LIB]
    if TORCH_LIB.exists() and all(p.stat().st_mtime <= TORCH_LIB.stat().st_mtime for p in deps):
        return TORCH_LIB
    tlib = cx.library_paths()[0]
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-unused-parameter",
           "-Wno-return-type", f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=kge_torch",
           *[f"-I{p}" for p in cx.include_paths()], "-I/opt/rocm/include", f"-I{INCLUDE}",
           str(TORCH_SRC), "-o", str(TORCH_LIB.with_suffix(".so.tmp")),
           f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", f"-Wl,-rpath,{tlib}",
           f"-L{PKG}", "-lkge_hip", "-Wl,-rpath,$ORIGIN", "-L/opt/rocm/lib", "-lamdhip64"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"libkge_torch.so build failed:\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr, file=sys.stderr)
    os.replace(TORCH_LIB.with_suffix(".so.tmp"), TORCH_LIB)
    return TORCH_LIB


def build(clean: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    hipcc = _hipcc()
    if clean and BUILD.exists():
        shutil.rmtree(BUILD)
    BUILD.mkdir(exist_ok=True)
    deps = _deps()
    srcs = sorted(CSRC.glob("*.hip"))
    objs = [BUILD / (s.stem + ".o") for s in srcs]
    todo = [(s, o) for s, o in zip(srcs, objs) if _stale(o, s, deps)]
    jobs = jobs or min(len(todo) or 1, max(1, min(16, os.cpu_count() or 1)))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for src, err in ex.map(lambda so: _compile(hipcc, *so), todo):
                if verbose:
                    print(f"[build] {src.name}", file=sys.stderr)
                    if err.strip():
                        print(err, file=sys.stderr)
    if todo or not LIB.exists() or any(o.stat().st_mtime > LIB.stat().st_mtime for o in objs):
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
    if clean and TORCH_LIB.exists():
        TORCH_LIB.unlink()
    build_torch_ops(verbose=verbose)
    return LIB


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    print(build(clean=a.clean, jobs=a.jobs, verbose=a.verbose))


if __name__ == "__main__":
    main()
