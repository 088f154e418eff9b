"""In-tree build of the gfx950 extension (``_C``) with hipcc.

Each ``csrc/kernels/*.hip`` file is a standalone HIP translation unit (no PyTorch headers,
seconds to compile) exposing C-ABI launchers; ``csrc/binding.cpp`` is the only file that
includes the PyTorch headers. Objects are rebuilt only when their source or a shared header
is newer, compiled in parallel, and linked into
``pytorch_distributed_training_example_amd/_C.<abi>.so`` next to this file, so the built
library travels with the repository snapshot to the GPU box (no JIT cache).

Usage: ``python -m pytorch_distributed_training_example_amd._build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "build")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path() -> str:
    return os.path.join(PKG, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _torch_dirs():
    import torch
    base = os.path.dirname(torch.__file__)
    inc = [os.path.join(base, "include"), os.path.join(base, "include", "torch", "csrc", "api", "include")]
    return base, inc, os.path.join(base, "lib")


def _headers() -> list[str]:
    return glob.glob(os.path.join(CSRC, "*.h"))


def _stale(obj: str, src: str, deps: list[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src] + deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    torch_base, torch_inc, torch_lib = _torch_dirs()
    py_inc = sysconfig.get_paths()["include"]
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-D__HIP_PLATFORM_AMD__",
              "-Wno-unused-result", "-I", CSRC]
    hdrs = _headers()
    jobs_list: list[tuple[str, list[str]]] = []
    objs: list[str] = []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, src, hdrs):
            jobs_list.append((obj, [HIPCC, *common, "-c", src, "-o", obj]))
    bsrc = os.path.join(CSRC, "binding.cpp")
    bobj = os.path.join(BUILD, "binding.o")
    objs.append(bobj)
    if force or _stale(bobj, bsrc, []):
        inc = sum([["-I", d] for d in torch_inc + [py_inc]], [])
        jobs_list.append((bobj, [HIPCC, *common, *inc, "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
                                 "-D_GLIBCXX_USE_CXX11_ABI=1", "-DUSE_ROCM=1", "-c", bsrc, "-o", bobj]))
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = {ex.submit(_run, cmd): obj for obj, cmd in jobs_list}
        for f in cf.as_completed(futs):
            f.result()
            if verbose:
                print("built", os.path.basename(futs[f]), flush=True)
    out = ext_path()
    if force or jobs_list or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        tmp = out + ".tmp"
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp, "-L", torch_lib,
              "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
              f"-Wl,-rpath,{torch_lib}"])
        os.replace(tmp, out)
    return out


def build_host_selftest(out: str | None = None) -> str:
    """The host-logic self-test (csrc/host/host_selftest.cpp) under AddressSanitizer +
    UndefinedBehaviorSanitizer. The sanitizers apply to the HOST half only (-Xarch_host): GPU
    sanitizer runs are not available on this pool, and the binary makes no HIP runtime call, so it
    runs on a CPU-only machine. Returns the executable path."""
    src = os.path.join(CSRC, "host", "host_selftest.cpp")
    out = out or os.path.join(BUILD, "host_selftest_asan")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    deps = _headers() + glob.glob(os.path.join(CSRC, "kernels", "*.hip"))
    if _stale(out, src, deps):
        _run([HIPCC, "-x", "hip", "-std=c++17", "-O1", "-g", f"--offload-arch={ARCH}",
              "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
              "-Xarch_host", "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer",
              src, "-o", out])
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--host-selftest", action="store_true",
                    help="build and run the ASan/UBSan host-logic self-test instead")
    a = ap.parse_args(argv)
    if a.host_selftest:
        exe = build_host_selftest()
        return subprocess.run([exe]).returncode
    print(build(force=a.force, jobs=a.jobs, verbose=True))
    return 0


if __name__ == "__main__":
    sys.exit(main())
