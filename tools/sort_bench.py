"""Walk-order sort alone (egm_debug_walk_sort) on 10M pairs shaped like the
walk key (a Zipf-skewed top level, hashed lower levels): run under
`rocprofv3 --kernel-trace --stats` and read k_sort_pass / k_sort_hist; with
EGM_LIB=<variant .so> for A/B (tools/build_variant.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from emqx_amd.engine import GpuMatcher  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rng = np.random.default_rng(1)
top = np.minimum(rng.zipf(1.1, n), 16).astype(np.uint32) - 1
keys = (top << np.uint32(28)) | (rng.integers(0, 1 << 20, n, dtype=np.uint32) << np.uint32(8))
vals = np.arange(n, dtype=np.uint64)
dev = torch.device("cuda:0")
dk = torch.from_numpy(keys.view(np.int32)).to(dev)
dv = torch.from_numpy(vals.view(np.int64)).to(dev)
out = torch.empty(n, dtype=torch.int64, device=dev)
gm = GpuMatcher(0)
for _ in range(reps):
    gm.debug_walk_sort(dk.data_ptr(), dv.data_ptr(), n, 24, out.data_ptr())
torch.cuda.synchronize()
o = out.cpu().numpy().view(np.uint64)
assert np.array_equal(o, vals[np.argsort(keys >> np.uint32(8), kind="stable")])
print("ok", n, reps)
gm.close()
