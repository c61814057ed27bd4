"""In-tree build of the native core (``_C.so``) for gfx950.

Kernels (``csrc/*.hip``) are compiled by ``hipcc --offload-arch=gfx950`` without torch headers
(fast, a few seconds each); host C++ (``csrc/*.cpp``) and the pybind11/torch binding TU are
compiled by ``hipcc`` as host code. Objects are cached by a content hash of the source plus
every header in ``csrc/``, so an unchanged tree rebuilds nothing. The shared object links
against the HIP runtime that torch itself loads (same soname ``libamdhip64.so.7``), so the
extension never brings a second HIP runtime into the process.

Usage: ``python -m fraud_detection_spark_kafka_llm_amd._build [--force] [-j N]``.
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

PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
BUILD = REPO / "build" / "native"
TARGET = PKG_DIR / "_C.so"
ARCH = os.environ.get("FDX_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the native core)")


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce

    inc = [Path(p) for p in ce.include_paths()]
    lib = Path(ce.library_paths()[0])
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _headers_digest() -> str:
    h = hashlib.sha256()
    for p in sorted(CSRC.glob("*.h")):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def _obj_for(src: Path, flags: list[str], hdr: str) -> Path:
    h = hashlib.sha256()
    h.update(src.read_bytes())
    h.update(hdr.encode())
    h.update(" ".join(flags).encode())
    return BUILD / f"{src.stem}.{src.suffix[1:]}.{h.hexdigest()[:16]}.o"


def _run(cmd: list[str]) -> None:
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"native build failed:\n{' '.join(cmd)}\n{res.stdout}\n{res.stderr}")


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    hipcc = _hipcc()
    inc, lib, abi = _torch_paths()
    BUILD.mkdir(parents=True, exist_ok=True)
    hdr = _headers_digest()
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{CSRC}", "-I/opt/rocm/include", "-Wno-unused-result", "-Wno-deprecated-declarations"]
    # No -ffast-math: reassociation would break the bitwise host/device agreement of the fp64
    # reductions (and Spark parity); kernels opt into fast paths explicitly where it is safe.
    kernel_flags = common + ["-x", "hip", f"--offload-arch={ARCH}", "-ffp-contract=off"]
    # host C++ (CPU path): no GPU code, plain optimisation.
    host_flags = common + ["-x", "c++", "-D__HIP_PLATFORM_AMD__=1", "-march=x86-64-v2", "-pthread",
                           "-ffp-contract=off"]
    py_inc = sysconfig.get_paths()["include"]
    bind_flags = common + ["-x", "c++", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C",
                           "-DTORCH_API_INCLUDE_EXTENSION_H", f"-I{py_inc}"] + [f"-I{p}" for p in inc]
    jobs_list = []
    for src in sorted(CSRC.glob("*.hip")):
        jobs_list.append((src, kernel_flags))
    for src in sorted(CSRC.glob("*.cpp")):
        jobs_list.append((src, bind_flags if src.name.startswith("bindings") else host_flags))

    objs: list[Path] = []
    todo = []
    for src, fl in jobs_list:
        obj = _obj_for(src, fl, hdr)
        objs.append(obj)
        if force or not obj.exists():
            todo.append((src, fl, obj))

    def compile_one(item):
        src, fl, obj = item
        tmp = obj.with_suffix(".tmp.o")
        cmd = [hipcc, *fl, "-c", str(src), "-o", str(tmp)]
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
        tmp.replace(obj)
        return src.name

    if todo:
        n = jobs or min(len(todo), max(1, (os.cpu_count() or 4)))
        with cf.ThreadPoolExecutor(n) as ex:
            for name in ex.map(compile_one, todo):
                if verbose:
                    print(f"[fdx-build] compiled {name}", flush=True)

    link_key = hashlib.sha256("".join(str(o) for o in objs).encode()).hexdigest()[:16]
    stamp = BUILD / "link.stamp"
    if force or not TARGET.exists() or not stamp.exists() or stamp.read_text() != link_key:
        tmp = TARGET.with_suffix(".tmp.so")
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp),
               f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
               f"-Wl,-rpath,{lib}", "-pthread"]
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
        tmp.replace(TARGET)
        stamp.write_text(link_key)
        # drop stale objects of older source revisions
        keep = {o.name for o in objs}
        for o in BUILD.glob("*.o"):
            if o.name not in keep:
                o.unlink(missing_ok=True)
    return TARGET


# identical private string literals that libstdc++ headers instantiate in several TUs trip ASan's
# ODR check (false positive); every other check stays on, and UBSan findings abort.
SELFTEST_ENV = {"ASAN_OPTIONS": "detect_odr_violation=0:abort_on_error=1:detect_leaks=1",
                "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}
HOST_SOURCES = ("text_cpu.cpp", "sparse_cpu.cpp", "tree_cpu.cpp", "json_text.cpp", "json_encode.cpp")


def build_host_selftest(sanitize: bool = True, out: Path | None = None) -> Path:
    """Debug target of SURVEY §5.2: the host (CPU) implementations + ``csrc/tests/host_selftest.cpp``
    as a standalone executable, built with AddressSanitizer + UndefinedBehaviorSanitizer (host
    code only: no device code is compiled into it)."""
    hipcc = _hipcc()
    out = out or (BUILD / ("host_selftest_asan" if sanitize else "host_selftest"))
    out.parent.mkdir(parents=True, exist_ok=True)
    flags = ["-O1", "-g", "-std=c++17", f"-I{CSRC}", "-I/opt/rocm/include", "-x", "c++", "-D__HIP_PLATFORM_AMD__=1",
             "-pthread", "-ffp-contract=off", "-fno-omit-frame-pointer"]
    if sanitize:
        flags += ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-gpu-sanitize",
                  ]
    # one translation unit (unity build): inline functions of libstdc++ then exist once, so ASan
    # does not see the same COMDAT string literal registered by several objects (false ODR report)
    unity = out.parent / "host_selftest_unity.cpp"
    unity.write_text("".join(f'#include "{CSRC / s}"\n' for s in HOST_SOURCES)
                     + f'#include "{CSRC / "tests" / "host_selftest.cpp"}"\n')
    link = ["-fsanitize=address,undefined"] if sanitize else []
    _run([hipcc, *flags, str(unity), "-o", str(out), "-pthread", *link])
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--host-selftest", action="store_true", help="build + run the ASan/UBSan host self-test")
    args = ap.parse_args(argv)
    if args.host_selftest:
        exe = build_host_selftest()
        return subprocess.run([str(exe)], env={**os.environ, **SELFTEST_ENV}).returncode
    path = build(force=args.force, jobs=args.jobs, verbose=args.verbose)
    print(f"built {path}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
