"""Native build for butterfly_amd: explicit hipcc / g++ invocations, no hipify, no JIT.

Products (in-tree, so they travel to the GPU box with the repo snapshot):
  butterfly_amd/_C.so       HIP/CDNA4 kernels (csrc/kernels/*.hip, --offload-arch=gfx950) +
                            torch.ops.bfly registrations (csrc/bindings/*.cpp), including the
                            native RCCL communicator (rccl_comm.cpp, linked to torch's RCCL).
  butterfly_amd/_native.so  Host C++ runtime (csrc/runtime/*.cpp): paged-KV block allocator,
                            partition cut-point search, request scheduler core. pybind11,
                            no torch / HIP dependency, so it loads and is tested on CPU.

Usage:  python -m butterfly_amd._build [--force] [--jobs N]
Objects are cached under build/obj keyed by a hash of (source, included headers, flags).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "butterfly_amd"
CSRC = ROOT / "csrc"
OBJ = ROOT / "build" / "obj"
ARCH = os.environ.get("BFLY_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch  # noqa: WPS433 (import inside: only the kernel library needs torch)

    base = Path(torch.__file__).resolve().parent
    return base / "include", base / "lib"


def _headers() -> list[Path]:
    return (sorted((CSRC / "include").glob("*.h")) + sorted((CSRC / "runtime").glob("*.h"))
            + sorted((CSRC / "kernels").glob("*.inc")))


def _digest(src: Path, flags: list[str]) -> str:
    h = hashlib.sha256()
    h.update(src.read_bytes())
    for hdr in _headers():
        h.update(hdr.read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def _compile(cmd: list[str], src: Path, obj: Path, force: bool) -> tuple[Path, bool]:
    stamp = obj.with_suffix(".sha")
    dig = _digest(src, cmd)
    if not force and obj.exists() and stamp.exists() and stamp.read_text() == dig:
        return obj, False
    obj.parent.mkdir(parents=True, exist_ok=True)
    full = cmd + ["-c", str(src), "-o", str(obj)]
    res = subprocess.run(full, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(full)}\n{res.stdout}\n{res.stderr}")
    stamp.write_text(dig)
    return obj, True


def _link(cmd: list[str], out: Path) -> None:
    tmp = out.with_suffix(".so.tmp")
    res = subprocess.run(cmd + ["-o", str(tmp)], capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    os.replace(tmp, out)


def build_kernels(force: bool = False, jobs: int = 8, verbose: bool = True) -> Path:
    tinc, tlib = _torch_paths()
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{CSRC / 'include'}", "-Wno-unused-result",
              "-D__HIP_PLATFORM_AMD__=1"]
    # fast-math for contraction / reassociation, but infinities stay meaningful: the attention
    # kernels use -inf as the empty-score sentinel
    kflags = [HIPCC, f"--offload-arch={ARCH}", "-ffast-math", "-fno-finite-math-only", "-fno-gpu-rdc", *common]
    # Host-only C++ for the bindings: ROCm's clang (x86 __bf16 support, libstdc++ ABI).
    hostcxx = os.environ.get("BFLY_HOST_CXX", "/opt/rocm/lib/llvm/bin/clang++")
    bflags = [hostcxx, "-x", "c++", *common, "-I/opt/rocm/include", f"-I{tinc}", f"-I{tinc / 'torch/csrc/api/include'}",
              "-DUSE_ROCM=1", "-D_GLIBCXX_USE_CXX11_ABI=1", "-Wno-deprecated-declarations"]
    jobs_list = []
    for src in sorted((CSRC / "kernels").glob("*.hip")):
        jobs_list.append((kflags, src, OBJ / "kernels" / (src.stem + ".o")))
    for src in sorted((CSRC / "bindings").glob("*.cpp")):
        jobs_list.append((bflags, src, OBJ / "bindings" / (src.stem + ".o")))
    objs, rebuilt = [], False
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, f, s, o, force) for f, s, o in jobs_list]
        for fut in futs:
            obj, did = fut.result()
            objs.append(obj)
            rebuilt |= did
            if did and verbose:
                print(f"[bfly-build] compiled {obj.relative_to(ROOT)}", flush=True)
    out = PKG / "_C.so"
    if rebuilt or force or not out.exists():
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs),
                f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
                "-lrccl",   # torch's own librccl.so (csrc/bindings/rccl_comm.cpp)
                f"-Wl,-rpath,{tlib}"]
        _link(link, out)
        if verbose:
            print(f"[bfly-build] linked {out.relative_to(ROOT)}", flush=True)
    return out


def build_native(force: bool = False, jobs: int = 8, verbose: bool = True) -> Path:
    import pybind11

    cxx = os.environ.get("CXX", shutil.which("g++") or "c++")
    pyinc = sysconfig.get_paths()["include"]
    flags = [cxx, "-O2", "-fPIC", "-std=c++17", "-Wall", "-fvisibility=hidden",
             f"-I{CSRC / 'include'}", f"-I{pybind11.get_include()}", f"-I{pyinc}"]
    srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    objs, rebuilt = [], False
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, flags, s, OBJ / "runtime" / (s.stem + ".o"), force) for s in srcs]
        for fut in futs:
            obj, did = fut.result()
            objs.append(obj)
            rebuilt |= did
            if did and verbose:
                print(f"[bfly-build] compiled {obj.relative_to(ROOT)}", flush=True)
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    out = PKG / f"_native{suffix}"
    if rebuilt or force or not out.exists():
        _link([cxx, "-shared", "-fPIC", *map(str, objs)], out)
        if verbose:
            print(f"[bfly-build] linked {out.relative_to(ROOT)}", flush=True)
    return out


def build_all(force: bool = False, jobs: int | None = None, verbose: bool = True) -> None:
    jobs = jobs or min(8, os.cpu_count() or 4)
    if list((CSRC / "runtime").glob("*.cpp")):
        build_native(force, jobs, verbose)
    build_kernels(force, jobs, verbose)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    build_all(a.force, a.jobs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
