"""Test-side emulation of the kernels' NFA walk over a host-built table image.

Used only to check, on a machine without a GPU, that the HBM image produced by
the host table builder (egm_table.cpp, exposed through TableImage) encodes the
filter set: tokenise -> byte-exact dictionary probe -> edge bucket probe ->
frontier expansion, exactly as egm_kernels.hip does it (items carry their
node's record; a literal edge slot carries a copy of its child's record).
Not a product path.
"""
NONE = 0xFFFFFFFF
WID_NONE, WID_PLUS, WID_HASH, WID_MAX = 0xFFFFFFFF, 0xFFFFFFFD, 0xFFFFFFFC, 0xFFFFFFF0
F_LIT, F_PLUS, F_HASH, F_TERM = 1, 2, 4, 8


class Emul:
    def __init__(self, img, arrays):
        self.img = img
        self.a = arrays
        self.blob = arrays["dict_blob"].tobytes()

    def word_id(self, w: bytes) -> int:
        a = self.a
        h = self.img.word_hash(w)
        i = h & a["dict_mask"]
        while True:
            s = a["dict"][i]
            wid = int(s[2])
            if wid == NONE:
                return WID_NONE
            sh = int(s[0]) | (int(s[1]) << 32)
            if sh == h and int(s[3]) == len(w):
                o0, o1 = int(a["dict_off"][wid]), int(a["dict_off"][wid + 1])
                if self.blob[o0:o1] == w:
                    return wid
            i = (i + 1) & a["dict_mask"]

    def edge(self, node, w):
        """-> (child, record tuple (plus, hash, term, flags)) or (NONE, None)."""
        a = self.a
        b = self.img.edge_bucket(node, w, a["edge_mask"])
        nk = len(a["edges"]) // (int(a["edge_mask"]) + 1)   # slots per bucket
        while True:
            for k in range(nk):
                s = a["edges"][b * nk + k]
                if int(s[0]) == node and int(s[1]) == w:
                    c = int(s[2])
                    rec = (int(s[4]), int(s[5]), int(s[6]), int(s[3]))
                    assert rec == self.rec(c), "edge slot's copy of the child record is stale"
                    pc = rec[0]   # the slot also carries the flags of the child's '+' child (the walk's skip)
                    assert int(s[7]) == (self.rec(pc)[3] if pc != NONE else 0), "edge slot's '+' child flags are stale"
                    return c, rec
                if int(s[0]) == NONE:
                    return NONE, None
            b = (b + 1) & a["edge_mask"]

    def rec(self, node):
        r = self.a["nodes"][node]
        return int(r[0]), int(r[1]), int(r[2]), int(r[3])

    def match(self, topic: bytes, mode: int = 0):
        a = self.a
        ws = topic.split(b"/")
        wids = []
        wild = False
        for w in ws:
            if w == b"+":
                wids.append(WID_PLUS); wild = True
            elif w == b"#":
                wids.append(WID_HASH); wild = True
            else:
                wids.append(self.word_id(w))
        dollar = topic[:1] == b"$"
        D = len(ws)
        out = []
        self.states = 0
        if wild:
            if mode == 0:
                return out
            node = 0
            for l in range(D):
                w = wids[l]
                if w == WID_PLUS:
                    node = self.rec(node)[0]
                elif w == WID_HASH:
                    node = int(a["hash_child"][node])
                elif w < WID_MAX:
                    node = self.edge(node, w)[0]
                else:
                    node = NONE
                if node == NONE:
                    return out
            plus, hsh, term, fl = self.rec(node)
            if fl & F_TERM:
                out.append(term)
            return out
        stack = [(0, 0, self.rec(0), 0)]
        self.states = 0   # states created (the kernels' `visited`, SURVEY §8d V_t)
        while stack:
            node, level, (plus, hsh, term, fl), wc = stack.pop()
            self.states += 1
            atend = level == D
            rootd = level == 0 and dollar
            if (fl & F_HASH) and not rootd:
                out.append(hsh)
            if atend and (fl & F_TERM) and (mode == 1 or wc or (D == 1 and dollar)):
                out.append(term)
            if atend:
                continue
            if (fl & F_LIT) and wids[level] < WID_MAX:
                c, r = self.edge(node, wids[level])
                if c != NONE:
                    stack.append((c, level + 1, r, wc))
            if (fl & F_PLUS) and not rootd:
                stack.append((plus, level + 1, self.rec(plus), 1))
        return out
