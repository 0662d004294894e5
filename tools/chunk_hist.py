"""Distribution of the ids per walk chunk (64 consecutive rows of the walk
order) at C2: what an LDS-staged compaction window must hold.  Untimed
diagnostic; prints one JSON line."""
import json

import numpy as np
import torch

from emqx_amd import _lib as L
from emqx_amd import synth
from emqx_amd.engine import GpuMatcher


def main():
    f, t = synth.config("c2")
    gm = GpuMatcher(0, max_batch=t.n)
    gm.build(f.blob, f.off)
    dev = torch.device("cuda:0")
    n, cap = t.n, 60 * t.n
    d_blob = torch.from_numpy(t.blob).to(dev)
    d_off = torch.from_numpy(t.off.view(np.int32)).to(dev)
    d_row = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    d_top = torch.zeros(n, dtype=torch.int32, device=dev)
    d_ids = torch.zeros(cap, dtype=torch.int32, device=dev)
    gm.match_device_ordered(d_blob.data_ptr(), int(t.off[-1]), d_off.data_ptr(), n, L.EGM_MODE_ROUTES, 0,
                            d_row.data_ptr(), d_top.data_ptr(), d_ids.data_ptr(), cap)
    torch.cuda.synchronize()
    row = d_row.cpu().numpy()
    ch = row[np.minimum(np.arange(0, n + 64, 64), n)]
    tot = np.diff(ch)
    qs = [50, 75, 90, 95, 99, 99.9, 100]
    out = {"chunks": int(len(tot)), "ids": int(row[-1]), "mean": float(tot.mean()),
           "pct": {str(q): float(np.percentile(tot, q)) for q in qs}}
    for lim in (2048, 3072, 4096, 6144, 8192):
        m = tot > lim
        out[f"over_{lim}"] = {"chunks": float(m.mean()), "ids": float(tot[m].sum() / row[-1])}
    print(json.dumps(out))
    gm.close()


if __name__ == "__main__":
    main()
