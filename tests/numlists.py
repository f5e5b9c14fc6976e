"""Numeric posdb termlists for gbsortby:/gbmin:/gbmax:/gbequal: terms (synthetic)."""
import numpy as np


def number_list(lists, frac, seed, termid=0x3C3C3C3C3C3, kmax=1, ints=False):
    """A numeric termlist of 1..kmax keys per docid for a `frac` share of
    the query's docids: a float (or int32) in bytes 2..5 of each key."""
    import struct
    import posdb_py
    rng = np.random.default_rng(seed)
    first = {}
    for l in lists:
        for k in posdb_py.full_keys(l):
            first.setdefault(int.from_bytes(k[7:12], "little") >> 2, k)
    keys = []
    for d in sorted(first):
        if rng.random() >= frac:
            continue
        vals = set()
        for _ in range(int(rng.integers(1, kmax + 1))):
            vals.add(struct.pack("<i", int(rng.integers(-20, 200))) if ints else
                     struct.pack("<f", float(rng.integers(0, 400)) / 4.0))
        run = []
        for v in vals:
            k = bytearray(first[d])
            k[2:6] = v
            k[12:18] = termid.to_bytes(6, "little")
            run.append(bytes(k))
        keys += sorted(run, key=lambda k: int.from_bytes(k[0:6], "little"))
    return posdb_py.encode_keys(keys)
