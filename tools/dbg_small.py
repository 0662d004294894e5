"""Debug helper: test_deep_and_long's batch, topic by topic or whole, with stats."""
import sys
import time
sys.path.insert(0, '.')
from emqx_amd.engine import GpuMatcher  # noqa: E402

gm = GpuMatcher(0)
T = b"a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q/r/s/t/u/v/w/x/y/z"
deep = b"/".join(b"l%d" % i for i in range(300))
filters = [b"#", T + b"/#", T + b"/+", b"/".join([b"+"] * 26) + b"/#",
           b"a/+/c/+/e/+/g/+/i/+/k/+/m/+/o/+/q/+/s/+/u/+/w/+/y/+/#", deep, deep + b"/#",
           b"/".join([b"+"] * 299) + b"/+", b"x" * 5000 + b"/+"]
gm.build_strings(filters)
topics = [T, T + b"/1", deep, deep + b"/more", b"x" * 5000 + b"/y", b"/".join([b"q"] * 300)]
which = sys.argv[1] if len(sys.argv) > 1 else "each"
sets = [[t] for t in topics] if which == "each" else [topics]
for mode in (0, 1):
    for ts in sets:
        t0 = time.time()
        print("mode", mode, "topic", ts[0][:20], len(ts), flush=True)
        r = gm.match(*__import__("emqx_amd.engine", fromlist=["pack_strings"]).pack_strings(ts), mode,
                     allow_error=True) if False else None
        try:
            r = gm.match_strings(ts, mode)
            print("  ok", time.time() - t0, r.row_ptr[-1], gm.last_stats(), gm.walk_counters(), flush=True)
        except Exception as e:  # noqa: BLE001
            print("  error", e, gm.last_stats(), flush=True)
