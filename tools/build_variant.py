"""Build an A/B variant of the library with extra -D flags (tuning only).

    python tools/build_variant.py TAG -DEGM_WALK_STACK=320 ...
      -> emqx_amd/libemqx_gpu_match_TAG.so   (select it with EGM_LIB=<path>)

Every source — the kernels AND the host table builder — is compiled with the
flags, so a flag that changes a layout or hash shared by both (egm_common.h)
stays consistent inside the variant.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import build as B  # noqa: E402

tag, flags = sys.argv[1], sys.argv[2:]
out = os.path.join(B.HERE, f"libemqx_gpu_match_{tag}.so")
bdir = f"/tmp/egm_var_{tag}"
os.makedirs(bdir, exist_ok=True)
objs = []
for name in ("egm_kernels.hip", "egm_pack.hip"):
    objs.append(os.path.join(bdir, name.replace(".hip", ".o")))
    B._run([B._hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result",
            "-Wno-unused-value", *flags, "-c", os.path.join(B.CSRC, name), "-o", objs[-1]], True)
for name in ("egm_table.cpp", "egm_bulk.cpp", "egm_capi.cpp", "egm_retain.cpp", "egm_dma.cpp"):
    o = os.path.join(bdir, name.replace(".cpp", ".o"))
    B._run(["g++", "-O3", "-fPIC", "-std=c++17", "-pthread", "-D__HIP_PLATFORM_AMD__", f"-I{B.ROCM}/include", *flags,
            "-c", os.path.join(B.CSRC, name), "-o", o], True)
    objs.append(o)
B._run([B._hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-pthread", "-o", out] + objs +
       [f"-L{B.ROCM}/lib", "-lhsa-runtime64"], True)
print(out)
