"""Posdb key codec, list compression and the synthetic generator.

The known-answer test is the reference's own (Posdb::init, Posdb.cpp:24-86):
the only fixture the reference holds that pins posdb bits."""
import numpy as np
import pytest

import gbgpu
import posdb_py

MAXWORDPOS = 0x3FFFF


def test_posdb_kat():
    # Posdb.cpp:26-52 values
    k = gbgpu.make_key(123456789, 34567292222, MAXWORDPOS - 1, 10, 15 - 1, 15 - 1, 13, 1, 59, 13,
                       syn=1, delkey=0, shard_by_termid=1)
    (d,) = posdb_py.decode_keys(k)
    assert d["termid"] == 123456789
    assert d["docid"] == 34567292222
    assert d["hashgroup"] == 1
    assert d["wordpos"] == MAXWORDPOS - 1
    assert d["density"] == 10
    assert d["diversity"] == 14
    assert d["wordspam"] == 14
    assert d["siterank"] == 13
    assert d["langid"] == 59
    assert d["multiplier"] == 13
    assert d["syn"] == 1
    assert d["shard_by_termid"] == 1
    assert d["positive"] == 1
    assert d["size"] == 18


def test_kat_alignment_bits():
    # every key start carries byte1 bit 0x02; byte 7 bit 0x02 is the zero bit
    k = gbgpu.make_key(987654321, (1 << 38) - 1, 777, 31, 15, 15, 15, 15, 63, 15)
    assert k[1] & 0x02
    assert not (k[7] & 0x02)


def _py_compress(keys):
    # RdbList::addRecord posdb branch (RdbList.cpp:282-327)
    out = bytearray()
    hi = lo = None
    for k in keys:
        if hi is not None and hi == k[12:18]:
            if lo == k[6:12]:
                b = bytearray(k[:6]); b[0] |= 0x06; out += b
                continue
            b = bytearray(k[:12]); b[0] |= 0x02; out += b
            lo = k[6:12]
            continue
        out += k
        lo, hi = k[6:12], k[12:18]
    return bytes(out)


def test_compress_matches_restatement():
    rng = np.random.default_rng(7)
    keys = []
    for t in (5, 9):
        for d in sorted(rng.choice(1 << 30, 40, replace=False)):
            for p in sorted(rng.choice(5000, int(rng.integers(1, 5)), replace=False)):
                keys.append(gbgpu.make_key(t, int(d), int(p), int(rng.integers(32)), 15, 15, 3, 0, 1))
    keys.sort(key=lambda k: (k[12:18][::-1], k[6:12][::-1], k[:6][::-1]))
    blob = b"".join(keys)
    assert gbgpu.compress(blob) == _py_compress(keys)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_synth_lists_wellformed(seed):
    specs = [gbgpu.TermSpec(1111, 0.3), gbgpu.TermSpec(2222, 0.2),
             gbgpu.TermSpec(3333, 0.6, gbgpu.SYNTH_BIGRAM, 0, 1, -1, 50)]
    lists = gbgpu.synth_lists(5000, specs, seed=seed)
    for l, sp in zip(lists, specs):
        keys = posdb_py.decode_keys(l)
        assert keys[0]["size"] == 18
        assert all(k["termid"] == sp.term_id for k in keys)
        # sorted by full key order and docids strictly increasing per run
        runs = posdb_py.decode_runs(l)
        ds = [r[0] for r in runs]
        assert ds == sorted(ds) and len(set(ds)) == len(ds)
        # unit classifier (alignment bit) == serial walk, on the swapped list
        sw = bytearray(l[:12]); sw[0] |= 0x02
        sw = bytes(sw) + l[18:]
        u = np.frombuffer(sw, np.uint8).reshape(-1, 6)
        starts = np.nonzero(((u[:, 1] & 2) != 0) & ((u[:, 0] & 4) == 0))[0]
        serial = [0]
        off = 12
        while off < len(sw):
            ks = posdb_py.key_size(sw[off])
            if ks != 6:
                serial.append(off // 6)
            off += ks
        assert list(starts) == serial
    # bigram docs are a subset of docs having both component words
    a, b, bg = (set(posdb_py.docids(x)) for x in lists)
    assert bg <= (a & b)


def test_synth_sharding_concatenates():
    specs = [gbgpu.TermSpec(42, 0.25), gbgpu.TermSpec(43, 0.1, gbgpu.SYNTH_SYNONYM, -1, -1, -1, 50)]
    full = gbgpu.synth_lists(200000, specs)
    parts = [gbgpu.synth_lists(200000, specs, doc_begin=a, doc_end=b)
             for a, b in ((0, 70000), (70000, 130000), (130000, 200000))]
    for t in range(2):
        ks = sum((posdb_py.decode_keys(p[t]) for p in parts), [])
        kf = posdb_py.decode_keys(full[t])
        assert [(k["docid"], k["wordpos"]) for k in ks] == [(k["docid"], k["wordpos"]) for k in kf]
