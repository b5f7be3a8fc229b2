"""In-tree build of the native HIP/C++ extension(s) for gfx950.

Builds ``spark_druid_olap_amd/ops/_sdo_native*.so`` with ``hipcc --offload-arch=gfx950``.  No
torch headers are needed (device pointers cross the boundary as integers), so a rebuild takes a
few seconds.  The .so is git-ignored but travels to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path
from typing import Optional

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
ARCH = "gfx950"

SOURCES = ["olap_scan.hip", "post_scan.hip", "sketch.hip", "partition.hip", "p2p.hip", "bindings.cpp"]


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def target_path() -> Path:
    return HERE / ("_sdo_native" + _ext_suffix())


def _source_hash() -> str:
    h = hashlib.sha256()
    for f in sorted(CSRC.iterdir()):
        if f.suffix in (".hip", ".cpp", ".h"):
            h.update(f.name.encode())
            h.update(f.read_bytes())
    h.update(ARCH.encode())
    return h.hexdigest()[:16]


def _stamp_path() -> Path:
    return HERE / "_sdo_native.stamp"


def is_fresh() -> bool:
    t = target_path()
    s = _stamp_path()
    return t.exists() and s.exists() and s.read_text().strip() == _source_hash()


def build(force: bool = False, verbose: bool = False) -> Path:
    target = target_path()
    if not force and is_fresh():
        return target
    import pybind11

    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    py_inc = sysconfig.get_paths()["include"]
    objs = []
    builddir = HERE / "build"
    builddir.mkdir(exist_ok=True)
    common = [
        f"--offload-arch={ARCH}",
        "-O3",
        "-fPIC",
        "-std=c++17",
        "-munsafe-fp-atomics",
        f"-I{CSRC}",
        f"-I{py_inc}",
        f"-I{pybind11.get_include()}",
        "-DNDEBUG",
    ]
    for src in SOURCES:
        obj = builddir / (Path(src).stem + ".o")
        cmd = [hipcc, *common, "-c", str(CSRC / src), "-o", str(obj)]
        if src.endswith(".cpp"):
            cmd.insert(1, "-xhip")
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        objs.append(str(obj))
    tmp = target.with_suffix(".tmp.so")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", str(tmp), "-lhiprtc"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, target)
    _stamp_path().write_text(_source_hash())
    return target


# ------------------------------------------------------------------ native HiveServer2 gateway
# Host-only C++ (sockets, threads, Thrift binary protocol): built with g++, no HIP toolchain needed.
GW_SRC = HERE.parent / "server" / "csrc" / "hs2_gateway.cpp"


def gateway_path() -> Path:
    return HERE.parent / "server" / ("_sdo_gateway" + _ext_suffix())


def _gateway_hash() -> str:
    return hashlib.sha256(GW_SRC.read_bytes()).hexdigest()[:16]


def build_gateway(force: bool = False, verbose: bool = False, extra_flags=(), out: Optional[Path] = None) -> Path:
    """``extra_flags`` + ``out``: an instrumented variant (e.g. the host ASan build) written beside,
    never over, the in-tree module."""
    target = Path(out) if out is not None else gateway_path()
    stamp = target.parent / "_sdo_gateway.stamp"
    if not force and not extra_flags and out is None and target.exists() and stamp.exists() and \
            stamp.read_text().strip() == _gateway_hash():
        return target
    import pybind11

    cxx = os.environ.get("CXX", "g++")
    tmp = target.with_suffix(".tmp.so")
    cmd = [cxx, "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wextra", *extra_flags,
           f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}", str(GW_SRC), "-o", str(tmp),
           "-lpthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, target)
    if not extra_flags and out is None:
        stamp.write_text(_gateway_hash())
    return target


if __name__ == "__main__":
    p = build(force="--force" in sys.argv, verbose=True)
    print(p)
    print(build_gateway(force="--force" in sys.argv, verbose=True))
