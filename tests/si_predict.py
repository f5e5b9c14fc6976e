"""Which tree docids the reference's second pass fails to find (test-side
restatement, used only to check where the GPU path declines).

The second pass (Posdb.cpp:6195-6241) looks each tree docid up in every
shrunk sublist with getWordPosList (Posdb.h:873-956).  shrinkSubLists
(Posdb.cpp:5334-5428) rewrote each sublist in place as the runs of the vote
buffer's docids; past the shrunk end the buffer still holds the list's own
bytes.  The search may miss a docid that is there."""


def image(lst: bytes) -> bytes:
    """The list as PosdbTable reads it: the first 18-byte key cut to 12
    bytes with the half bit set (Posdb.cpp:5671-5703)."""
    if not lst:
        return b""
    b = bytearray(lst[:12])
    b[0] |= 0x02
    return bytes(b) + lst[18:]


def runs(img: bytes):
    out, p = [], 0
    while p < len(img):
        q = p + 12
        while q < len(img) and img[q] & 0x04:
            q += 6
        out.append((int.from_bytes(img[p + 7:p + 12], "little") >> 2, p, q))
        p = q
    return out


def word_pos_list(buf: bytes, size: int, doc: int):
    """getWordPosList over buf[0:size] (reads past it as the reference does)."""
    def g(i):
        return buf[i] if 0 <= i < len(buf) else 0
    step = (size // 12) * 6
    p, count = step, 0
    for _ in range(256):
        origp = p
        while p > 0 and (g(p + 1) & 0x02):
            p -= 6
        p -= 6
        d = int.from_bytes(bytes(g(p + 7 + k) for k in range(5)), "little") >> 2
        if d == doc:
            return p
        step >>= 1
        step -= step % 6
        if step <= 0:
            step = 6
            count += 1
            if count >= 3:
                return None
        if d < doc:
            p = origp + step
            if p > size:
                p = size - 6
        else:
            p = max(0, origp - step)
    return None


def shrink(buf: bytearray, end: int, votes) -> int:
    """shrinkSubLists on one sublist, in place over buf[0:end] (Posdb.cpp:
    5334-5428); returns the new end.  A list shared by several groups is
    shrunk once per use, the later passes over the earlier one's output and
    the stale bytes after it (end stays the list's own)."""
    def kd(p):
        return int.from_bytes(bytes(buf[p + 7:p + 12]), "little") >> 2
    rec = dst = vi = 0
    nv = len(votes)
    if end <= 0:
        return 0
    while True:
        while True:
            if vi >= nv:
                return dst
            v, k = votes[vi], kd(rec)
            if v > k:
                break
            if v < k:
                vi += 1
                continue
            buf[dst:dst + 12] = buf[rec:rec + 12]
            dst += 12
            rec += 12
            while True:
                if rec >= end:
                    return dst
                if not (buf[rec] & 0x04):
                    break
                buf[dst:dst + 6] = buf[rec:rec + 6]
                dst += 6
                rec += 6
            vi += 1
        rec += 12
        while True:
            if rec >= end:
                return dst
            if not (buf[rec] & 0x04):
                break
            rec += 6


def misses(lists, votes, docids):
    """(list index, docid) pairs where a docid with a run in the list is
    not found at that run, in the list's first-use view or (a superset for
    lists shared by groups) its re-shrunk view."""
    vs = sorted(int(v) for v in votes)
    vset = set(vs)
    out = []
    for li, lst in enumerate(lists):
        img = image(lst)
        own, off = {}, 0
        for d, p, q in runs(img):
            if d in vset:
                own[d] = off
                off += q - p
        buf = bytearray(img)
        s1 = shrink(buf, len(img), vs)
        s2 = shrink(buf, len(img), vs)
        for d in docids:
            d = int(d)
            if d not in own:
                continue
            if any(word_pos_list(buf, s, d) != own[d] for s in {s1, s2}):
                out.append((li, d))
    return out
