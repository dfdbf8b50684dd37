"""In-tree build of the native extensions (``python -m ps_amd._build``).

Two shared objects are produced next to the Python sources, so they travel with the repo
snapshot to the GPU box (``gpurun``) and are what the tests import:

* ``ps_amd/_C*.so``       -- HIP kernels for gfx950 (csrc/kernels/*.hip, compiled by hipcc
  with ``--offload-arch=gfx950``) + torch bindings (csrc/bindings.cpp, host compiler).
* ``ps_amd/_native*.so``  -- CPU runtime in C++ (csrc/runtime/*.cpp): the TCP parameter
  server / client, the threaded batch loader and the key router.  No torch dependency.

The build is driven by a generated ``build.ninja`` (ninja is in the image), so rebuilds are
incremental and kernel TUs compile in parallel.  No hipify, no torch JIT cache: explicit
hipcc / g++ command lines only.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "ps_amd"
BUILD = ROOT / "build"
ARCH = os.environ.get("PS_AMD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_paths():
    import torch

    base = Path(torch.__file__).resolve().parent
    return base / "include", base / "lib", int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _ninja_bin() -> str:
    exe = shutil.which("ninja")
    if exe:
        return exe
    try:
        import ninja  # type: ignore

        return str(Path(ninja.BIN_DIR) / "ninja")
    except Exception as e:  # pragma: no cover
        raise RuntimeError("ninja not found") from e


def _write_ninja() -> Path:
    tinc, tlib, abi = _torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    ext = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    import pybind11

    hip_srcs = sorted((ROOT / "csrc" / "kernels").glob("*.hip"))
    rt_srcs = sorted((ROOT / "csrc" / "runtime").glob("*.cpp"))
    hipcc = f"{ROCM}/bin/hipcc"
    cxx = os.environ.get("CXX", "g++")
    lines = [
        "ninja_required_version = 1.3",
        f"hipcc = {hipcc}",
        f"cxx = {cxx}",
        f"hipflags = -O3 -std=c++17 -fPIC --offload-arch={ARCH} -I{ROOT}/csrc/include "
        f"-Wno-unused-result -ffp-contract=fast",
        f"bindflags = -O2 -std=c++17 -fPIC -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 "
        f"-DTORCH_EXTENSION_NAME=_C -DTORCH_API_INCLUDE_EXTENSION_H -D_GLIBCXX_USE_CXX11_ABI={abi} "
        f"-I{tinc} -I{tinc}/torch/csrc/api/include -I{pyinc} -I{ROCM}/include -I{ROOT}/csrc/include "
        f"-Wno-deprecated-declarations -Wno-unused-parameter",
        f"rtflags = -O3 -std=c++17 -fPIC -pthread -DPS_NATIVE_EXTENSION_NAME=_native "
        f"-I{pybind11.get_include()} -I{pyinc} -I{ROOT}/csrc/include -Wall -Wno-unused-parameter",
        f"ldflags = -shared -fPIC --offload-arch={ARCH} -L{tlib} -lc10 -lc10_hip -ltorch -ltorch_cpu "
        f"-ltorch_hip -ltorch_python -Wl,-rpath,{tlib}",
        "rule hip",
        "  command = $hipcc $hipflags -c $in -o $out -MD -MF $out.d",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC $in",
        "rule bind",
        "  command = $cxx $bindflags -c $in -o $out -MD -MF $out.d",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule rt",
        "  command = $cxx $rtflags -c $in -o $out -MD -MF $out.d",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule link",
        "  command = $hipcc $in -o $out $ldflags",
        "  description = LINK $out",
        "rule linkrt",
        "  command = $cxx -shared -fPIC -pthread $in -o $out",
        "  description = LINK $out",
    ]
    objs = []
    for s in hip_srcs:
        o = BUILD / (s.stem + ".hip.o")
        objs.append(o)
        lines.append(f"build {o}: hip {s}")
    for src in sorted((ROOT / "csrc").glob("*.cpp")):  # bindings.cpp + host-side GPU runtime (async PS)
        bo = BUILD / (src.stem + ".o")
        lines.append(f"build {bo}: bind {src}")
        objs.append(bo)
    out_c = PKG / f"_C{ext}"
    lines.append(f"build {out_c}: link " + " ".join(str(o) for o in objs))
    targets = [str(out_c)]
    if rt_srcs:
        rt_objs = []
        for s in rt_srcs:
            o = BUILD / (s.stem + ".rt.o")
            rt_objs.append(o)
            lines.append(f"build {o}: rt {s}")
        out_n = PKG / f"_native{ext}"
        lines.append(f"build {out_n}: linkrt " + " ".join(str(o) for o in rt_objs))
        targets.append(str(out_n))
    lines.append("default " + " ".join(targets))
    BUILD.mkdir(exist_ok=True)
    nf = BUILD / "build.ninja"
    text = "\n".join(lines) + "\n"
    if not nf.exists() or nf.read_text() != text:
        nf.write_text(text)
    return nf


def build(verbose: bool = False, jobs: int | None = None) -> None:
    nf = _write_ninja()
    j = jobs or int(os.environ.get("MAX_JOBS", min(8, os.cpu_count() or 4)))
    j = max(1, min(j, 16))
    cmd = [_ninja_bin(), "-f", str(nf), f"-j{j}"]
    if verbose:
        cmd.append("-v")
    r = subprocess.run(cmd, cwd=str(BUILD), capture_output=not verbose, text=True)  # .ninja_log in build/
    if r.returncode != 0:
        sys.stderr.write((r.stdout or "") + (r.stderr or ""))
        raise RuntimeError("ps_amd native build failed")


if __name__ == "__main__":
    build(verbose="-v" in sys.argv)
    print("ps_amd: native build OK")
