"""Per-row order-independent checksums of CSR match results.

A row's checksum is the sum (mod 2^64) of a 64-bit mix of each filter id in
it, so two rows with the same id SET have the same checksum whatever their
order (the reference's results are order-free sets:
apps/emqx/test/emqx_trie_SUITE.erl:82,101,118).  The C++ oracle computes the
same mix per row (oracle/trie_oracle.cpp ot_match_sums), which lets every row
of a full-size batch be compared as a set without moving its ids; the sum is
additive over disjoint filter shards.
"""
import numpy as np


def id_mix(ids):
    x = ids.astype(np.uint64)
    x ^= x >> np.uint64(16)
    x *= np.uint64(0x9E3779B97F4A7C15)
    x ^= x >> np.uint64(29)
    return x


def row_checksums(row, ids):
    """Per-row order-independent checksum: sum of a 64-bit mix of each id."""
    x = id_mix(ids[: int(row[-1])] if len(ids) > int(row[-1]) else ids)
    cnt = np.diff(row).astype(np.int64)
    out = np.zeros(len(cnt), np.uint64)
    nz = np.nonzero(cnt)[0]
    if len(nz):
        out[nz] = np.add.reduceat(x, row[:-1].astype(np.int64)[nz])
    return out
