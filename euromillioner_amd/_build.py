"""Native build driver: compiles every ``csrc/*.hip`` / ``csrc/*.cpp`` for gfx950.

The reference reaches native code only through dependency binaries (XGBoost4J's
``libxgboost`` via JNI at ``Main.java:110-141``; the declared-but-unused ND4J
natives behind DL4J, ``pom.xml:62-66``).  Here every native piece is our own
source, compiled in-tree with ``hipcc --offload-arch=gfx950`` into ONE shared
library ``euromillioner_amd/lib/libem_native.so`` exposing a plain C ABI.

Design notes (MI355X-first):
  * No torch headers in the native code: kernels and the C++ runtime (CSV
    loader, tree drivers) compile in seconds and never go through hipify.
  * The library is loaded with ``ctypes`` *after* ``import torch``; both the
    torch wheel's HIP runtime and ours carry SONAME ``libamdhip64.so.7``, so
    the dynamic linker binds our library to the runtime torch already mapped
    (one HIP runtime per process, shared streams / device pointers).
  * Objects are rebuilt incrementally (mtime vs. source + every header).
"""
from __future__ import annotations

import concurrent.futures as _cf
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OBJDIR = os.path.join(ROOT, "build", "obj")
LIBDIR = os.path.join(ROOT, "euromillioner_amd", "lib")
LIBNAME = "libem_native.so"
HOST_LIBNAME = "libem_host.so"  # pure C++ (no device code): data generator, CSV loader, tree oracles
ARCH = os.environ.get("EUROM_OFFLOAD_ARCH", "gfx950")


def lib_path() -> str:
    return os.path.join(LIBDIR, LIBNAME)


def host_lib_path() -> str:
    return os.path.join(LIBDIR, HOST_LIBNAME)


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (need ROCm at /opt/rocm)")


COMMON_FLAGS = [
    "-O3",
    "-fPIC",
    "-std=c++17",
    f"--offload-arch={ARCH}",
    "-Wno-unused-result",
    "-Wno-unused-command-line-argument",
    "-munsafe-fp-atomics",
]


def _sources():
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip"))) + sorted(glob.glob(os.path.join(CSRC, "*.cpp")))
    headers = sorted(glob.glob(os.path.join(CSRC, "*.h")))
    return srcs, headers


def _obj_for(src: str) -> str:
    base = os.path.basename(src)
    return os.path.join(OBJDIR, base + ".o")


def _needs_build(src: str, obj: str, headers) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    if os.path.getmtime(src) > t:
        return True
    return any(os.path.getmtime(h) > t for h in headers)


def _file_flags(src: str) -> list[str]:
    """Per-file flags from a ``// EM_BUILD_FLAGS: ...`` line in the first 40 lines."""
    out: list[str] = []
    with open(src, encoding="utf-8", errors="replace") as f:
        for i, line in enumerate(f):
            if i > 40:
                break
            if "EM_BUILD_FLAGS:" in line:
                out += line.split("EM_BUILD_FLAGS:", 1)[1].split()
    return out


def _compile(src: str, obj: str, extra=()):
    cmd = [_hipcc()] + COMMON_FLAGS + _file_flags(src) + list(extra) + ["-I", CSRC]
    if src.endswith(".hip"):
        cmd += ["-x", "hip"]
    cmd += ["-c", src, "-o", obj]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{p.stdout}")
    return p.stdout


HOST_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-march=x86-64-v2", "-Wall", "-Wno-unused-function", "-pthread"]


def build_host(force: bool = False, verbose: bool = False, extra_flags=()) -> str:
    """g++ build of csrc/host/*.cpp -> libem_host.so (loads without any GPU/HIP runtime)."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    headers = sorted(glob.glob(os.path.join(CSRC, "host", "*.h")))
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        raise RuntimeError("g++ not found")
    objs = []
    for src in srcs:
        obj = os.path.join(OBJDIR, "host_" + os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _needs_build(src, obj, headers):
            cmd = [cxx] + HOST_FLAGS + list(extra_flags) + ["-I", os.path.join(CSRC, "host"), "-c", src, "-o", obj]
            p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
            if p.returncode != 0:
                raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{p.stdout}")
            if verbose:
                print(f"[build] host/{os.path.basename(src)}", file=sys.stderr)
    lib = host_lib_path()
    if objs and (force or not os.path.exists(lib) or any(os.path.getmtime(o) > os.path.getmtime(lib) for o in objs)):
        tmp = lib + ".tmp"
        cmd = [cxx, "-shared", "-fPIC", "-pthread"] + list(extra_flags) + ["-o", tmp] + objs
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{p.stdout}")
        os.replace(tmp, lib)
    return lib


def build_all(force: bool = False, verbose: bool = False) -> tuple[str, str]:
    return build_host(force=force, verbose=verbose), build(force=force, verbose=verbose)


def build(force: bool = False, jobs: int | None = None, verbose: bool = False, extra_flags=()) -> str:
    """Compile + link the HIP library; returns its path."""
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    srcs, headers = _sources()
    if not srcs:
        raise RuntimeError(f"no native sources under {CSRC}")
    todo = [(s, _obj_for(s)) for s in srcs if force or _needs_build(s, _obj_for(s), headers)]
    jobs = jobs or min(8, max(1, (os.cpu_count() or 2)))
    if todo:
        with _cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = {ex.submit(_compile, s, o, extra_flags): s for s, o in todo}
            for f in _cf.as_completed(futs):
                out = f.result()
                if verbose:
                    print(f"[build] {os.path.basename(futs[f])}", file=sys.stderr)
                    if out.strip():
                        print(out, file=sys.stderr)
    lib = lib_path()
    objs = [_obj_for(s) for s in srcs]
    if todo or not os.path.exists(lib) or any(os.path.getmtime(o) > os.path.getmtime(lib) for o in objs):
        tmp = lib + ".tmp"
        cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + ["-lpthread"]
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{p.stdout}")
        os.replace(tmp, lib)
    return lib


def resource_usage(src_name: str) -> str:
    """Compile one source with ``-Rpass-analysis=kernel-resource-usage`` (VGPR/AGPR/LDS report)."""
    src = os.path.join(CSRC, src_name)
    cmd = [_hipcc()] + COMMON_FLAGS + _file_flags(src) + ["-I", CSRC, "-x", "hip", "-Rpass-analysis=kernel-resource-usage",
                                       "--cuda-device-only", "-c", src, "-o", "/dev/null"]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    return p.stdout


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--usage", default=None, help="print kernel resource usage for one csrc file")
    ap.add_argument("--debug", action="store_true",
                    help="debug build (-g, device asserts kept; run with HIP_LAUNCH_BLOCKING=1 to localise a fault); "
                         "forces a rebuild -- rebuild without --debug afterwards")
    ap.add_argument("--define", action="append", default=[], metavar="NAME=VALUE",
                    help="extra -D for the HIP sources (kernel tuning sweeps); forces a rebuild")
    ap.add_argument("--host-sanitize", action="store_true",
                    help="host-only ASan/UBSan build of the C++ host library (GPU sanitizers are unavailable)")
    a = ap.parse_args()
    if a.usage:
        print(resource_usage(a.usage))
    else:
        host_flags = ("-fsanitize=address,undefined", "-fno-omit-frame-pointer") if a.host_sanitize else ()
        print(build_host(force=a.force or a.host_sanitize, verbose=a.verbose, extra_flags=host_flags))
        dbg = ("-g", "-O1") if a.debug else ()
        defs = tuple("-D" + d for d in a.define)
        print(build(force=a.force or a.debug or bool(defs), jobs=a.jobs, verbose=a.verbose, extra_flags=dbg + defs))
