"""Build the native pieces in-tree (no cmake; hipcc/g++ directly).

* ``emqx_amd/libemqx_gpu_match.so`` — the C-ABI + gfx950 kernels (product)
* ``emqx_amd/libegm_synth.so``      — synthetic workload generator (bench/tests)
* ``oracle/liboracle_trie.so``      — C++ oracle restatement (tests/bench CPU leg only)

Rebuilds only when a source is newer than its output.  ``python -m emqx_amd.build``.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("EGM_OFFLOAD_ARCH", "gfx950")

LIB = os.path.join(HERE, "libemqx_gpu_match.so")
SYNTH = os.path.join(HERE, "libegm_synth.so")
ORACLE = os.path.join(ROOT, "oracle", "liboracle_trie.so")

HEADERS = [os.path.join(CSRC, f) for f in ("egm_common.h", "egm_table.h", "egm_kernels.h", "egm_dma.h", "egm_pack.h")] + [
    os.path.join(ROOT, "include", "emqx_gpu_match.h")]


def _hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    return p


def _stale(out: str, srcs) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {' '.join(cmd[:3])} ...")
    return r


def build_lib(verbose=False, force=False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    objs = []
    for name in ("egm_kernels.hip", "egm_pack.hip"):
        hip_src = os.path.join(CSRC, name)
        o = os.path.join(BUILD, name.replace(".hip", ".o"))
        if force or _stale(o, [hip_src] + HEADERS):
            _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-result",
                  "-Wno-unused-value", "-c", hip_src, "-o", o], verbose)
        objs.append(o)
    for name in ("egm_table.cpp", "egm_bulk.cpp", "egm_capi.cpp", "egm_retain.cpp", "egm_dma.cpp"):
        src = os.path.join(CSRC, name)
        o = os.path.join(BUILD, name.replace(".cpp", ".o"))
        if force or _stale(o, [src] + HEADERS):
            _run(["g++", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-result", "-Wno-unused-value", "-pthread", "-D__HIP_PLATFORM_AMD__",
                  f"-I{ROCM}/include", "-c", src, "-o", o], verbose)
        objs.append(o)
    if force or _stale(LIB, objs + [os.path.abspath(__file__)]):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", LIB] + objs +
             [f"-L{ROCM}/lib", "-lhsa-runtime64"], verbose)
    return LIB


def build_synth(verbose=False, force=False) -> str:
    src = os.path.join(CSRC, "egm_synth.cpp")
    if force or _stale(SYNTH, [src]):
        _run(["g++", "-O3", "-fPIC", "-shared", "-std=c++17", "-o", SYNTH, src], verbose)
    return SYNTH


def build_oracle(verbose=False, force=False) -> str:
    srcs = [os.path.join(ROOT, "oracle", f) for f in ("trie_oracle.cpp", "retainer_scan.cpp")]
    if force or _stale(ORACLE, srcs):
        _run(["g++", "-O3", "-fPIC", "-shared", "-std=c++17", "-pthread", "-o", ORACLE] + srcs, verbose)
    return ORACLE


def build_all(verbose=False, force=False):
    return build_lib(verbose, force), build_synth(verbose, force), build_oracle(verbose, force)


if __name__ == "__main__":
    print(build_all(verbose=True, force="--force" in sys.argv))
