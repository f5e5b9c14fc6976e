"""Synthetic tiered posdb runs for the list merge (config 5, BASELINE.json):
n sorted posdb files ("runs") of relative sizes 1:2:4:..., a fraction of keys
repeated across runs (a newer copy overrides an older one) and a fraction of
delete keys, exactly what RdbList::posdbMerge_r (RdbList.cpp:3065-3568)
consumes when Msg5/RdbMerge merge posdb files oldest-first.

Keys are packed with numpy following Posdb::makeKey (Posdb.cpp:374-460); the
layout is the one csrc/posdb_key.h documents.  Runs are ordered by the
bfcmpPosdb compare (RdbList.h:620-641: the 18-byte key as a big integer with
the low 3 bits -- delete bit and compression bits -- ignored) and compressed
with gbgpu.compress (RdbList::addRecord, RdbList.cpp:282-327)."""
from __future__ import annotations

from typing import List

import numpy as np

import gbgpu

DOCID_BITS = 38


def pack_keys(term, docid, wordpos, density, diversity, spam, siterank, hashgroup, langid, syn, positive):
    """(n0 u16, n1 u64, n2 u64) arrays of Posdb::makeKey."""
    term = term.astype(np.uint64)
    docid = docid.astype(np.uint64)
    n2 = (term << np.uint64(16)) | (docid >> np.uint64(22))
    n1 = ((docid & np.uint64(0x3FFFFF)) << np.uint64(42)) \
        | (siterank.astype(np.uint64) << np.uint64(37)) \
        | ((langid.astype(np.uint64) & np.uint64(0x1F)) << np.uint64(32)) \
        | (wordpos.astype(np.uint64) << np.uint64(14)) \
        | (hashgroup.astype(np.uint64) << np.uint64(10)) \
        | (spam.astype(np.uint64) << np.uint64(6)) \
        | (diversity.astype(np.uint64) << np.uint64(2)) \
        | syn.astype(np.uint64)
    n0 = (density.astype(np.uint32) << 11) | (1 << 9) | (((langid.astype(np.uint32) >> 5) & 1) << 3) \
        | positive.astype(np.uint32)
    return n0.astype(np.uint16), n1, n2


def to_bytes(n0, n1, n2) -> bytes:
    rec = np.zeros(len(n0), dtype=[("n0", "<u2"), ("n1", "<u8"), ("n2", "<u8")])
    rec["n0"], rec["n1"], rec["n2"] = n0, n1, n2
    return rec.tobytes()


def _order(n0, n1, n2):
    # bfcmpPosdb order: n2, n1, then n0 with the low 3 bits ignored
    return np.lexsort(((n0 | 7), n1, n2))


def tiered_runs(total_keys: int, nruns: int = 8, seed: int = 5, dup_frac: float = 0.05,
                neg_frac: float = 0.01, nterms: int = 200) -> List[bytes]:
    """nruns compressed posdb runs, oldest first, sizes ~1:2:...:2^(nruns-1)."""
    rng = np.random.default_rng(seed)
    n = int(total_keys)
    # Zipf-ish term mix; docids uniform 38-bit; fields as SURVEY.md §8(d)
    tids = (rng.integers(1, 1 << 47, size=nterms, dtype=np.int64)).astype(np.uint64)
    w = 1.0 / np.arange(1, nterms + 1)
    term = tids[rng.choice(nterms, size=n, p=w / w.sum())]
    docid = rng.integers(0, 1 << DOCID_BITS, size=n, dtype=np.int64).astype(np.uint64)
    wordpos = rng.integers(0, 1 << 18, size=n)
    density = rng.integers(0, 32, size=n)
    diversity = np.full(n, 15)
    spam = np.where(rng.random(n) < 0.8, 15, rng.integers(0, 16, size=n))
    siterank = rng.integers(0, 16, size=n)
    hashgroup = rng.choice(11, size=n, p=[0.80, 0.05, 0.04, 0.03, 0.02, 0.04, 0, 0, 0, 0.02, 0])
    langid = np.where(rng.random(n) < 0.9, 1, rng.integers(0, 64, size=n))
    syn = (rng.random(n) < 0.05).astype(np.uint64)
    positive = np.ones(n, np.uint32)
    n0, n1, n2 = pack_keys(term, docid, wordpos, density, diversity, spam, siterank, hashgroup, langid,
                           syn, positive)
    # unique keys under the merge compare
    o = _order(n0, n1, n2)
    n0, n1, n2 = n0[o], n1[o], n2[o]
    keep = np.ones(len(n0), bool)
    keep[1:] = ~((n2[1:] == n2[:-1]) & (n1[1:] == n1[:-1]) & ((n0[1:] | 7) == (n0[:-1] | 7)))
    n0, n1, n2 = n0[keep], n1[keep], n2[keep]
    n = len(n0)
    wts = 2.0 ** np.arange(nruns)
    run = rng.choice(nruns, size=n, p=wts / wts.sum())
    # duplicates: a copy of the key in another run (its delete bit may flip)
    dup = np.nonzero(rng.random(n) < dup_frac)[0]
    drun = rng.integers(0, nruns, size=len(dup))
    drun = np.where(drun == run[dup], (drun + 1) % nruns, drun)
    dn0 = n0[dup].copy()
    flip = rng.random(len(dup)) < 0.5
    dn0[flip] ^= 1
    # delete keys
    neg = rng.random(n) < neg_frac
    n0 = n0.copy()
    n0[neg] &= np.uint16(0xFFFE)
    all0 = np.concatenate([n0, dn0])
    all1 = np.concatenate([n1, n1[dup]])
    all2 = np.concatenate([n2, n2[dup]])
    allr = np.concatenate([run, drun])
    out = []
    for r in range(nruns):
        sel = np.nonzero(allr == r)[0]
        a0, a1, a2 = all0[sel], all1[sel], all2[sel]
        o = _order(a0, a1, a2)
        out.append(gbgpu.compress(to_bytes(a0[o], a1[o], a2[o])))
    return out
