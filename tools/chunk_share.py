"""How much of a 64-topic walk chunk's memory traffic is shared inside the chunk?

CPU analysis of the C2 workload (measurement tool, not a product path): the
table image is built on the host (egm_image_build), the 10M-topic batch is
tokenised and put in walk order (the a86 key of k_tokenise, stable sort),
and sampled chunks of 64 consecutive topics are walked state by state the way
k_walk does (signature-gated literal probes, '+' record reads).  Per chunk it
counts the reads the 64 topics make and how many distinct lines they touch:
literal bucket probes keyed (node, word) and '+' record reads keyed by node.

    python tools/chunk_share.py [n_filters] [n_topics] [n_chunks]
"""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from emqx_amd import synth  # noqa: E402
from emqx_amd.engine import TableImage  # noqa: E402

NONE = 0xFFFFFFFF
WID_NONE, WID_MAX = 0xFFFFFFFF, 0xFFFFFFF0
F_LIT, F_PLUS, F_HASH, F_TERM = 1, 2, 4, 8
M64 = (1 << 64) - 1
FNV_BASIS, FNV_PRIME = 0xcbf29ce484222325, 0x100000001b3


def mix64(x):
    x ^= x >> 33
    x = (x * 0xff51afd7ed558ccd) & M64
    x ^= x >> 33
    x = (x * 0xc4ceb9fe1a85ec53) & M64
    x ^= x >> 33
    return x


def sig_bit(w):
    h = mix64(0x9E3779B97F4A7C15 ^ w) >> 32
    return 1 << (4 + ((h * 28) >> 32))


def walk_key(w, shape=0xA86):
    h, k, used = FNV_BASIS, 0, 0
    for l in range(4):
        bl = (shape >> (4 * l)) & 0xF
        h = mix64(((h ^ (w[l] if l < len(w) else 0)) * FNV_PRIME) & M64)
        b = (h >> (64 - bl)) if (l < len(w) and bl) else 0
        if bl:
            k = (k << bl) | b
        used += bl
    return k << (32 - used) if used < 32 else k


def main():
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    nt = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_000
    nch = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    t0 = time.time()
    f, t = synth.config("c2", n_filters=nf, n_topics=nt)
    img = TableImage()
    img.bulk_build(f.blob, f.off, threads=8)
    a = img.arrays()
    print(f"built {time.time() - t0:.0f}s nodes={len(a['nodes'])} edge slots={len(a['edges'])}", flush=True)
    blob, doff = a["dict_blob"].tobytes(), a["dict_off"]
    vocab = {blob[int(doff[i]):int(doff[i + 1])]: i for i in range(len(doff) - 1)}
    topics = t.to_list()
    wids = [[vocab.get(w, WID_NONE) for w in s.split(b"/")] for s in topics]
    keys = np.array([walk_key(w) if b"+" not in s and b"#" not in s else 0xFFFFFFFF
                     for s, w in zip(topics, wids)], dtype=np.uint64)
    order = np.argsort(keys, kind="stable")
    print(f"tokenised + sorted {time.time() - t0:.0f}s", flush=True)
    nodes, edges, emask = a["nodes"], a["edges"], a["edge_mask"]

    def edge(node, w):
        b = img.edge_bucket(node, w, emask)
        nk = len(edges) // (int(emask) + 1)   # slots per bucket
        probes = 0
        while True:
            for k in range(nk):
                s = edges[b * nk + k]
                if int(s[0]) == node and int(s[1]) == w:
                    return int(s[2]), int(s[3]), int(s[4]), b
                if int(s[0]) == NONE:
                    return NONE, 0, 0, b
            b = (b + 1) & emask
            probes += 1

    rng = np.random.default_rng(1)
    starts = rng.choice(nt // 64, nch, replace=False) * 64

    # The same chunks walked by prefix groups: the chunk's topics in
    # lexicographic order of their word ids, a state carries the range of
    # topics that share its prefix, so a '+' read or a literal probe is made
    # once per (state, group) / (state, distinct next word) and an emit covers
    # a range of topics.
    grp = dict(lit=0, plus=0, emits=0, ids=0)
    for s0 in starts:
        ch = [ti for ti in order[s0:s0 + 64] if b"+" not in topics[ti] and b"#" not in topics[ti]]
        ch.sort(key=lambda ti: wids[ti])
        W = [wids[ti] for ti in ch]
        dol = [topics[ti][:1] == b"$" for ti in ch]
        # root: one group per (dollar, w0) split is enough; groups = runs of equal prefixes
        r = nodes[0]
        stack = [(0, 0, int(r[3]), int(r[0]), 0, len(ch))]
        while stack:
            node, lvl, fl, plus, lo, hi = stack.pop()
            # emits: '#' for the whole group (not at a '$' root), terminal for topics ending here
            if fl & F_HASH:
                cov = sum(1 for j in range(lo, hi) if len(W[j]) >= lvl and not (lvl == 0 and dol[j]))
                if cov:
                    grp["emits"] += 1
                    grp["ids"] += cov
            live = [j for j in range(lo, hi) if len(W[j]) > lvl]
            if (fl & F_TERM) and any(len(W[j]) == lvl for j in range(lo, hi)):
                grp["emits"] += 1
            if not live:
                continue
            # literal: one probe per run of equal words at this level among the
            # live topics (shorter topics inside the range are skipped over)
            i = 0
            while i < len(live):
                k = i
                while k < len(live) and W[live[k]][lvl] == W[live[i]][lvl]:
                    k += 1
                wd = W[live[i]][lvl]
                if (fl & F_LIT) and wd < WID_MAX and (fl & sig_bit(wd)):
                    grp["lit"] += 1
                    c, cfl, cplus, b = edge(node, wd)
                    if c != NONE:
                        stack.append((c, lvl + 1, cfl, cplus, live[i], live[k - 1] + 1))
                i = k
            nd = [j for j in live if not (lvl == 0 and dol[j])]
            if (fl & F_PLUS) and nd:
                grp["plus"] += 1
                pr = nodes[plus]
                # the non-'$' live topics are contiguous only if '$' words sort together; count it as one read
                stack.append((plus, lvl + 1, int(pr[3]), int(pr[0]), nd[0], nd[-1] + 1))
    n = nch * 64
    for cn in (0, 32, 64, 128, 256):
        tot_it = tot_r = tot_l = tot_h = 0
        for s0 in starts[:100]:
            ch = [ti for ti in order[s0:s0 + 64] if b"+" not in topics[ti] and b"#" not in topics[ti]]
            W = [wids[ti] for ti in ch]
            dol = [topics[ti][:1] == b"$" for ti in ch]
            i_, r_, l_, h_ = emulate_wave(nodes, edge, W, dol, cache_n=cn)
            tot_it += i_; tot_r += r_; tot_l += l_; tot_h += h_
            tot_x = globals().get("TOT_X", 0) + EXACT
            globals()["TOT_X"] = tot_x
        print(f"per-topic walk, cache {cn}: iterations/chunk {tot_it / 100:.1f}, reads/topic {tot_r / 6400:.1f}, "
              f"lines after merging/topic {tot_l / 6400:.1f} (same address only {globals().get('TOT_X', 0) / 6400:.1f}), "
              f"cache hits/topic {tot_h / 6400:.1f}", flush=True)
        globals()["TOT_X"] = 0
        break
    print(f"prefix-group walk per topic: literal probes {grp['lit'] / n:.2f}, '+' reads {grp['plus'] / n:.2f}, "
          f"range emits {grp['emits'] / n:.2f} covering {grp['ids'] / n:.1f} ids")
    tot = dict(lit=0, lit_lines=0, plus=0, plus_lines=0, states=0, lit_fail=0, lit_keys=0, plus_keys=0)
    by_level = {}
    for s0 in starts:
        lines_b, keys_b, lines_p = set(), set(), set()
        for ti in order[s0:s0 + 64]:
            s, w = topics[ti], wids[ti]
            if b"+" in s or b"#" in s:
                continue
            D, dollar = len(w), s[:1] == b"$"
            r = nodes[0]
            fl = int(r[3])
            stack = [(0, 0, fl, int(r[0]))]
            while stack:
                node, lvl, fl, plus = stack.pop()
                tot["states"] += 1
                if lvl == D:
                    continue
                rootd = lvl == 0 and dollar
                wd = w[lvl]
                if (fl & F_LIT) and wd < WID_MAX and (fl & sig_bit(wd)):
                    c, cfl, cplus, b = edge(node, wd)
                    tot["lit"] += 1
                    lines_b.add(b)
                    keys_b.add((node, wd))
                    by_level.setdefault(lvl, [0, 0, 0])[0] += 1
                    if c != NONE:
                        stack.append((c, lvl + 1, cfl, cplus))
                    else:
                        tot["lit_fail"] += 1
                        by_level[lvl][2] += 1
                if (fl & F_PLUS) and not rootd:
                    pr = nodes[plus]
                    tot["plus"] += 1
                    lines_p.add(plus >> 2)   # 16-B records, 64-B lines
                    by_level.setdefault(lvl, [0, 0, 0])[1] += 1
                    stack.append((plus, lvl + 1, int(pr[3]), int(pr[0])))
        tot["lit_lines"] += len(lines_b)
        tot["lit_keys"] += len(keys_b)
        tot["plus_lines"] += len(lines_p)
    n = nch * 64
    print(f"per topic: states {tot['states'] / n:.1f}, literal probes {tot['lit'] / n:.1f} "
          f"(fail {tot['lit_fail'] / n:.1f}), '+' reads {tot['plus'] / n:.1f}")
    print(f"distinct per chunk / reads: bucket lines {tot['lit_lines'] / max(1, tot['lit']):.3f} "
          f"(keys {tot['lit_keys'] / max(1, tot['lit']):.3f}), '+' record lines {tot['plus_lines'] / max(1, tot['plus']):.3f}")
    print("level: [literal probes, '+' reads, failed probes] per topic")
    for l in sorted(by_level):
        print(l, [round(x / n, 2) for x in by_level[l]])



def emulate_wave(nodes, edge_fn, W, dollar, S=32, stack_cap=320, cache_n=0):
    """The per-topic walk of k_walk (round 2) over one chunk, iteration by
    iteration: sub-chunks of S topics admitted at once, up to 64 items popped
    LIFO (bounded by room - dmax), literal children pushed before '+'
    children.  Returns (iterations, lane reads, distinct lines per iteration
    summed (what the CU's merging leaves), reads a direct-mapped per-wave cache
    of cache_n entries would have served)."""
    dmax = max(len(w) for w in W)
    it = reads = lines = hits = 0
    global EXACT
    EXACT = 0
    cache = {}
    for s0 in range(0, len(W), S):
        stack = []
        for j in range(s0, min(s0 + S, len(W))):
            r = nodes[0]
            stack.append((0, 0, int(r[3]), int(r[0]), j))
        while stack:
            room = stack_cap - len(stack)
            take = min(64, len(stack), room - dmax if room > dmax else 1)
            pop = stack[len(stack) - take:]
            del stack[len(stack) - take:]
            it += 1
            ln = set()
            ex = set()
            c0, c1 = [], []
            for (node, lvl, fl, plus, j) in pop:
                w = W[j]
                if lvl == len(w):
                    continue
                rootd = lvl == 0 and dollar[j]
                wd = w[lvl]
                for kind, key in ((0, (node, wd)), (1, plus)):
                    if kind == 0 and not ((fl & F_LIT) and wd < WID_MAX and (fl & sig_bit(wd))):
                        continue
                    if kind == 1 and not ((fl & F_PLUS) and not rootd):
                        continue
                    reads += 1
                    line = ("b", key) if kind == 0 else ("p", key >> 2)
                    if cache_n:
                        slot = hash(line) % cache_n
                        if cache.get(slot) == line and line not in ln:
                            hits += 1
                        cache[slot] = line
                    ln.add(line)
                    ex.add((kind, key))
                    if kind == 0:
                        c, cfl, cplus, _ = edge_fn(node, wd)
                        if c != NONE and lvl + 1 < len(w) + 1:
                            c0.append((c, lvl + 1, cfl, cplus, j))
                    else:
                        pr = nodes[key]
                        c1.append((key, lvl + 1, int(pr[3]), int(pr[0]), j))
            lines += len(ln)
            EXACT += len(ex)

            def go(x):   # pushed only with a transition left to take (finish())
                node, lvl, fl, plus, j = x
                if lvl >= len(W[j]):
                    return False
                wd = W[j][lvl]
                return bool((fl & F_PLUS) or ((fl & F_LIT) and wd < WID_MAX and (fl & sig_bit(wd))))
            stack.extend(x for x in c0 if go(x))
            stack.extend(x for x in c1 if go(x))
    return it, reads, lines, hits


if __name__ == "__main__":
    main()
