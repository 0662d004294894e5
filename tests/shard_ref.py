"""Reference merge of filter-shard CSRs (numpy, test-side checker for
egm_shard_merge and ShardExchange): per topic, shard 0's ids, then shard 1's."""
import numpy as np


def merge_shard_results(parts):
    rows = [np.asarray(r, dtype=np.uint64) for r, _ in parts]
    n = len(rows[0]) - 1
    cnts = np.stack([np.diff(r).astype(np.int64) for r in rows])          # [G, n]
    tot = cnts.sum(axis=0)
    row = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(tot, out=row[1:])
    before = np.cumsum(cnts, axis=0) - cnts                                 # ids of earlier shards per topic
    ids = np.zeros(int(row[-1]), dtype=np.uint32)
    for g, (r, gi) in enumerate(parts):
        c = cnts[g]
        if c.sum() == 0:
            continue
        tpos = np.repeat(np.arange(n, dtype=np.int64), c)
        k = np.arange(len(gi), dtype=np.int64) - np.repeat(rows[g][:-1].astype(np.int64), c)
        ids[row[:-1].astype(np.int64)[tpos] + before[g][tpos] + k] = gi
    return row, ids
