import numpy as np, sys
sys.path.insert(0, '.')
from emqx_amd import _lib as L
from emqx_amd.engine import GpuMatcher
import ctypes as C
gm = GpuMatcher(0)
gm.build_strings([b'sensor/1/metric/2', b'sensor/+/#', b'sensor/#'])
for topics in ([b'sensor'], [b'sensor/1'], [b'a'] * 100):
    res = C.POINTER(L.egm_result)()
    from emqx_amd.engine import pack_strings
    blob, off = pack_strings(topics)
    rc = gm.lib.egm_match_batch(gm.ctx, C.c_void_p(blob.ctypes.data), C.c_void_p(off.ctypes.data), len(topics), 0, C.byref(res))
    print('rc', rc, gm.lib.egm_last_error(gm.ctx), gm.last_stats(), gm.walk_counters(), flush=True)
