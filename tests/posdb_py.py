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
