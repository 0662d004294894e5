"""Build an A/B variant of the library with extra -D flags (tuning only).

    python tools/build_variant.py TAG -DEGM_WALK_STACK=320 ...
      -> emqx_amd/libemqx_gpu_match_TAG.so   (select it with EGM_LIB=<path>)
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import build as B  # noqa: E402

tag, flags = sys.argv[1], sys.argv[2:]
out = os.path.join(B.HERE, f"libemqx_gpu_match_{tag}.so")
obj = f"/tmp/egm_kernels_{tag}.o"
B._run([B._hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-fPIC", "-std=c++17", *flags, "-c",
        os.path.join(B.CSRC, "egm_kernels.hip"), "-o", obj], True)
B.build_lib()
objs = [obj] + [os.path.join(B.BUILD, n) for n in ("egm_table.o", "egm_bulk.o", "egm_capi.o", "egm_retain.o")]
B._run([B._hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-pthread", "-o", out] + objs, True)
print(out)
