"""emqx_amd — MI355X-native publish-time route lookup for EMQX.

Hot path: emqx_trie:match/1 + emqx_router:match_routes/1 +
emqx_broker dispatch fan-out, as gfx950 HIP kernels behind the C-ABI in
include/emqx_gpu_match.h (libemqx_gpu_match.so).  The Python modules mirror the
reference's Erlang interfaces for that path:

* ``emqx_amd.topic``  — emqx_topic (words/wildcard/join/validate/parse; host utilities)
* ``emqx_amd.trie``   — emqx_trie (insert/delete/match/empty) on the GPU table
* ``emqx_amd.router`` — emqx_router (add/delete route, match_routes)
* ``emqx_amd.broker`` — emqx_broker publish/dispatch fan-out + emqx_shared_sub picks
* ``emqx_amd.engine`` — GpuMatcher, the ctypes handle on one device context
"""
__version__ = "0.1.0"
