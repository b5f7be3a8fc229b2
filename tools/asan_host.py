"""Host-side AddressSanitizer/UBSan run of the native code, on the CPU box.

GPU ASan / XNACK builds are not available on the MI355X pool, so the sanitizer covers the HOST
code paths of both native modules:

* ``server/csrc/hs2_gateway.cpp`` (sockets, SASL, Thrift binary codec, statement batching, result
  paging -- all host C++): built with g++ ``-fsanitize=address,undefined`` and driven by the
  native-gateway tests plus a malformed-frame fuzz pass (``tests/test_asan_host.py``), with GCC's
  libasan preloaded into the Python process.
* ``ops/csrc/bindings.cpp`` (descriptor layout, hipRTC JIT compile wrapper): built by hipcc with
  ``-Xarch_host -fsanitize=address`` (device code is not instrumented) and exercised by compiling
  the per-query JIT kernels of the TPC-H bench queries through hipRTC, with clang's ASan runtime
  preloaded.

Usage: ``python tools/asan_host.py [outdir]`` -- builds both, runs both drivers, exits non-zero on
any sanitizer report.  The instrumented modules are written under ``outdir`` (default
/tmp/sdo_asan), never over the in-tree builds.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g", "-O1"]


def _suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def build_gateway_asan(out: Path) -> Path:
    from spark_druid_olap_amd.ops import build as B

    return B.build_gateway(force=True, extra_flags=SAN, out=out / ("_sdo_gateway" + _suffix()))


def build_native_asan(out: Path) -> Path:
    import pybind11

    from spark_druid_olap_amd.ops import build as B

    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    inc = [f"-I{B.CSRC}", f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]
    common = [f"--offload-arch={B.ARCH}", "-O1", "-g", "-fPIC", "-std=c++17", "-munsafe-fp-atomics", *inc]
    host_san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]
    objs = []
    for src in B.SOURCES:
        obj = out / (Path(src).stem + ".o")
        cmd = [hipcc, *common, "-c", str(B.CSRC / src), "-o", str(obj)]
        if src.endswith(".cpp"):
            cmd[1:1] = ["-xhip", *host_san]
        subprocess.run(cmd, check=True)
        objs.append(str(obj))
    target = out / ("_sdo_native" + _suffix())
    subprocess.run([hipcc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *host_san, *objs, "-o", str(target),
                    "-lhiprtc"], check=True)
    return target


def gcc_asan_runtime() -> str:
    """libasan plus libstdc++: preloaded into a C main program (python) ASan must see libstdc++ at
    start-up to intercept ``__cxa_throw`` (the gateway throws ProtocolError on bad frames)."""
    p = [subprocess.run(["gcc", f"-print-file-name={lib}"], capture_output=True, text=True, check=True).stdout.strip()
         for lib in ("libasan.so", "libstdc++.so")]
    return " ".join(p)


def clang_asan_runtime() -> str:
    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    if not hits:
        raise FileNotFoundError("clang ASan runtime not found under /opt/rocm/lib/llvm")
    return hits[-1]


def san_env(runtime: str, **extra) -> dict:
    env = dict(os.environ)
    env.update(LD_PRELOAD=runtime, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", PYTHONPATH=str(ROOT), **extra)
    return env


def jit_compile_driver() -> None:
    """Runs INSIDE the sanitized process: lower the bench queries on a CPU shard, generate their
    JIT kernel sources and compile every one through the instrumented hipRTC wrapper."""
    import torch  # noqa: F401

    from spark_druid_olap_amd.engine.executor import Engine
    from spark_druid_olap_amd.models import tpch
    from spark_druid_olap_amd.models.bench_queries import DRUID_JSON
    from spark_druid_olap_amd.ops import desc as D
    from spark_druid_olap_amd.ops import jit, native
    from spark_druid_olap_amd.query.spec import query_from_json

    m = native.load()
    assert m.__file__ == os.environ["SDO_NATIVE_SO"], m.__file__
    assert m.layout() == D.layout() and m.desc_size() == D.SCANDESC.itemsize
    os.environ.setdefault("SDO_JIT_CACHE", "/tmp/sdo_asan/jitcache")
    ds = tpch.to_datasource(tpch.generate_flat(0.002, "cpu"), profile="bench")
    eng = Engine(use_native=False)
    n = 0
    for name, js in DRUID_JSON.items():
        prog = eng.prepare(query_from_json(js), ds).scans[0][1]
        if prog.empty:
            continue
        try:
            k = jit.JitScan(prog, D.M_DENSE_LDS, 4, prog.nhll > 0, 1 << prog.hll_p, True, load=False)
        except ValueError:  # table too large for LDS: the HBM-table kernel variant
            k = jit.JitScan(prog, D.M_DENSE_GLOBAL, 4, False, 1 << prog.hll_p, True, load=False)
        assert k.src and k.name.startswith("sdo_jit_")
        n += 1
    # a compile error must surface as a Python exception, not a crash
    try:
        m.rtc_compile("this is not C++", "bad", jit.OPTS)
        raise AssertionError("bad source compiled")
    except RuntimeError:
        pass
    print(f"asan: compiled {n} JIT kernels through the instrumented hipRTC wrapper")


def main() -> int:
    if "--jit-driver" in sys.argv:
        jit_compile_driver()
        return 0
    out = Path(sys.argv[1] if len(sys.argv) > 1 else "/tmp/sdo_asan")
    out.mkdir(parents=True, exist_ok=True)
    gw = build_gateway_asan(out)
    nat = build_native_asan(out)
    r1 = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                         str(ROOT / "tests" / "test_thrift_server.py"), str(ROOT / "tests" / "test_asan_host.py"),
                         "-k", "native or fuzz"],
                        env=san_env(gcc_asan_runtime(), SDO_GATEWAY_SO=str(gw), SDO_ASAN_CHILD="1"), cwd=str(ROOT))
    r2 = subprocess.run([sys.executable, str(Path(__file__).resolve()), "--jit-driver"],
                        env=san_env(clang_asan_runtime(), SDO_NATIVE_SO=str(nat), SDO_JIT_CACHE=str(out / "jit")),
                        cwd="/tmp")
    print(f"asan gateway rc={r1.returncode} native rc={r2.returncode}")
    return r1.returncode or r2.returncode


if __name__ == "__main__":
    sys.exit(main())
