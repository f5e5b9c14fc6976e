"""Independent numpy decoder of posdb termlists (Posdb.h:3-25 layout), used
by the tests to recompute docid sets without going through either C path."""
import numpy as np


def key_size(b0):
    return 6 if b0 & 0x04 else (12 if b0 & 0x02 else 18)


def decode_runs(data: bytes):
    """Serial walk (RdbList::getRecSize semantics): [(docid, start_off, nkeys)]"""
    out = []
    off = 0
    n = len(data)
    while off < n:
        ks = key_size(data[off])
        if ks != 6:
            d = (int.from_bytes(data[off + 7:off + 12], "little") >> 2)
            out.append([d, off, 1])
        else:
            out[-1][2] += 1
        off += ks
    return out


def docids(data: bytes) -> np.ndarray:
    return np.array([r[0] for r in decode_runs(data)], dtype=np.int64)


def decode_keys(data: bytes):
    """All keys as dicts with the getter fields (Posdb.h:291-380)."""
    keys = []
    off = 0
    cur = None
    while off < len(data):
        b = data[off:off + 18]
        ks = key_size(b[0])
        if ks == 18:
            cur = bytes(b[6:18])
        elif ks == 12:
            cur = bytes(b[6:12]) + cur[6:12]
        full = bytes(data[off:off + 6]) + cur
        u16_0 = full[0] | full[1] << 8
        u32_2 = int.from_bytes(full[2:6], "little")
        n1 = int.from_bytes(full[2:10], "little")
        keys.append(dict(
            termid=int.from_bytes(full[12:18], "little"),
            docid=int.from_bytes(full[7:12], "little") >> 2,
            siterank=(n1 >> 37) & 0xf,
            langid=((n1 >> 32) & 0x1f) | (0x20 if full[0] & 0x08 else 0),
            wordpos=u32_2 >> 14,
            hashgroup=(full[3] >> 2) & 0xf,
            wordspam=((full[2] | full[3] << 8) >> 6) & 0xf,
            diversity=(full[2] >> 2) & 0xf,
            syn=full[2] & 3,
            density=(u16_0 >> 11) & 0x1f,
            multiplier=(u16_0 >> 4) & 0xf,
            shard_by_termid=full[1] & 1,
            positive=full[0] & 1,
            size=ks,
        ))
        off += ks
    return keys


def full_keys(data: bytes):
    """The list's keys as whole 18-byte keys, compression bits cleared."""
    out, off, hi, lo = [], 0, b"", b""
    while off < len(data):
        ks = key_size(data[off])
        if ks == 18:
            hi = bytes(data[off + 12:off + 18])
        if ks >= 12:
            lo = bytes(data[off + 6:off + 12])
        k = bytearray(bytes(data[off:off + 6]) + lo + hi)
        k[0] &= 0xf9
        out.append(bytes(k))
        off += ks
    return out


def encode_keys(keys) -> bytes:
    """RdbList::addRecord's posdb compression (RdbList.cpp:282-327) of sorted
    whole keys: same bytes 6..17 -> 6 bytes, same 12..17 -> 12, else 18."""
    out, prev = bytearray(), None
    for k in keys:
        k = bytearray(k)
        if prev is not None and prev[6:18] == k[6:18]:
            k[0] |= 0x06
            out += k[:6]
        elif prev is not None and prev[12:18] == k[12:18]:
            k[0] |= 0x02
            out += k[:12]
        else:
            out += k
        prev = bytes(k)
    return bytes(out)


def with_docid(k: bytes, d: int) -> bytes:
    """Key k with its docid (bytes 7..11 >> 2, Posdb.h:295) replaced."""
    k = bytearray(k)
    v = (int.from_bytes(k[7:12], "little") & 0x3) | (d << 2)
    k[7:12] = v.to_bytes(5, "little")
    return bytes(k)


def remap_docids(lists, new_docids):
    """Relabel the union of the lists' docids, in order, with the sorted
    new_docids (at least as many): every list keeps its key order."""
    ks = [full_keys(l) for l in lists]
    old = sorted({int.from_bytes(k[7:12], "little") >> 2 for kl in ks for k in kl})
    new = sorted(new_docids)[:len(old)]
    assert len(new) == len(old)
    m = dict(zip(old, new))
    return [encode_keys([with_docid(k, m[int.from_bytes(k[7:12], "little") >> 2]) for k in kl]) for kl in ks]


def site_lists(lists, nsites=2, frac=0.3, seed=5, flip_frac=0.05, multi_frac=0.0):
    """Whitelist ("&sites=") termlists for a query's lists: each of nsites
    site terms holds a random fraction of the query's docids, one key per doc
    (18 then 12 bytes) carrying the doc's own siteRank, so byte 7 (docid low
    bits + siteRank's top bit) matches the query keys -- except a flip_frac
    share whose siteRank top bit is flipped, which the reference's 5-byte
    table compare rejects.  multi_frac docs get 2-3 keys (6-byte keys inside
    a list; never the last key)."""
    import gbgpu
    rng = np.random.default_rng(seed)
    docs = {}
    for l in lists:
        for k in decode_keys(l):
            docs.setdefault(k["docid"], (k["siterank"], k["langid"]))
    ids = np.array(sorted(docs), dtype=np.int64)
    out = []
    for s in range(nsites):
        tid = (0x5173 + 977 * s + (seed << 20)) & ((1 << 48) - 1)
        pick = ids[rng.random(len(ids)) < frac]
        keys = []
        for j, d in enumerate(pick):
            sr, lang = docs[int(d)]
            if rng.random() < flip_frac:
                sr ^= 0x8
            npos = 1 if (j == len(pick) - 1 or rng.random() >= multi_frac) else int(rng.integers(2, 4))
            for w in range(npos):
                keys.append(gbgpu.make_key(tid, int(d), 5 + 7 * w, 20, 15, 15, sr, 7, lang & 0x3f))
        out.append(gbgpu.compress(b"".join(keys)))
    return out
