"""Shard-reply sets for the Msg3a::mergeLists fixtures (tests/golden/x_*.npz,
made by make_golden.py from the reference's own mergeLists) and for the
seeded checks of the device / host merges against the oracle.

A reply is what one shard's Msg39 sends (Msg39.cpp:1633-1684): docids with
double scores -- a float TopNode::m_score widened, or (double)m_intScore for
gbsortby int queries -- best first (TopTree high -> low: score desc, docid
asc).  Some sets break that order on purpose: Msg3a's loop only compares the
shard heads, so it is defined for any reply order."""
import numpy as np

MAXD = 1 << 38


def _sorted(d, s):
    o = np.lexsort((d, -s))
    return d[o], s[o]


def partitioned(rng, nshards, per, k_levels, int_scores=False):
    """Docid-range shards: disjoint docids, many score ties."""
    out = []
    for r in range(nshards):
        n = int(rng.integers(0, per + 1))
        lo, hi = r * (MAXD // nshards), (r + 1) * (MAXD // nshards)
        d = rng.choice(np.arange(lo, min(hi, lo + 50 * per + 1)), size=n, replace=False).astype(np.int64)
        if int_scores:
            s = rng.integers(-k_levels, k_levels, size=n).astype(np.int32).astype(np.float64)
        else:
            s = (rng.integers(1, k_levels + 1, size=n).astype(np.float32) * np.float32(1.5)).astype(np.float64)
        out.append(_sorted(d, s))
    return out


def cases():
    """[(name, shards, docs_to_get)]"""
    rng = np.random.default_rng(0x3A)
    c = []
    c.append(("sorted8_ties", partitioned(rng, 8, 100, 20), 100))
    c.append(("sorted8_ties_k10", partitioned(rng, 8, 100, 5), 10))
    # twin replicas: the same docids with the same scores on two shards
    base = partitioned(rng, 2, 60, 8)
    c.append(("twins", [base[0], base[1], base[0], base[1]], 50))
    # the same docid on several shards with different scores: the first one
    # merged (the best) is kept, the rest are passed over
    d = rng.choice(1000, size=40, replace=False).astype(np.int64)
    sh = []
    for r in range(3):
        s = rng.integers(1, 6, size=40).astype(np.float64)
        sh.append(_sorted(d.copy(), s))
    c.append(("dup_diff_scores", sh, 30))
    c.append(("k_gt_union", partitioned(rng, 3, 7, 4), 100))
    p = partitioned(rng, 5, 40, 6)
    p[1] = (np.zeros(0, np.int64), np.zeros(0))
    p[3] = (np.zeros(0, np.int64), np.zeros(0))
    c.append(("empty_some", p, 30))
    c.append(("empty_all", [(np.zeros(0, np.int64), np.zeros(0))] * 4, 10))
    c.append(("one_shard", partitioned(rng, 1, 80, 10), 50))
    # replies out of order: the loop compares heads only
    un = []
    for r in range(4):
        n = int(rng.integers(5, 30))
        un.append((rng.choice(5000, size=n, replace=False).astype(np.int64),
                   rng.integers(1, 4, size=n).astype(np.float64)))
    c.append(("unsorted", un, 40))
    c.append(("int_scores", partitioned(rng, 6, 80, 30, int_scores=True), 100))
    # -0.0 and +0.0 compare equal as doubles: the lower docid goes first
    z = []
    for r in range(3):
        d = np.sort(rng.choice(np.arange(r * 1000, r * 1000 + 500), size=6, replace=False)).astype(np.int64)
        s = np.array([1.0, 1.0, 0.0, -0.0, 0.0, -0.0])
        if r == 1:
            s = np.array([1.0, -0.0, -0.0, 0.0, 0.0, -1.0])
        z.append((d, s))
    c.append(("signed_zero", z, 20))
    c.append(("many64", partitioned(rng, 64, 60, 40), 1000))
    c.append(("k1", partitioned(rng, 4, 10, 2), 1))
    return c


# ---------------------------------------------------------------- full replies
# Msg39Replies with cluster records and facet lists (Msg39.cpp:1346-1684) for
# the whole Msg3a::mergeLists: the <=2-per-site cap (Msg3a.cpp:1342-1379),
# the facet-table merge (1089-1240) and the facet doc counts (794-802).
FACET_STR, FACET_INT, FACET_FLOAT = 63, 64, 65
FE = np.dtype([("key", "<i4"), ("count", "<i4"), ("outside", "<i4"), ("docid", "<i8"), ("sum", "<i8"),
               ("max", "<i4"), ("min", "<i4")])  # i32 key + Posdb.h:401-413's FacetEntry: 36 bytes
assert FE.itemsize == 36


def cluster_rec(docid, site, adult=False, lang=0):
    """Clusterdb::makeClusterRecKey (Clusterdb.cpp:775-803) as 12 bytes
    (key_t n0 then n1): docid at n0 >> 35 | n1 << 29, the family bit at 34,
    the language at 28, the 26-bit site hash at 2, a positive key."""
    n1 = (docid >> 29) & 0x1FF
    n0 = ((docid << 35) & 0xFFFFFFFFFFFFFFFF) | (int(adult) << 34) | ((lang & 0x3F) << 28) | ((site & 0x3FFFFFF) << 2) | 1
    return np.array([n0], "<u8").tobytes() + np.array([n1], "<u4").tobytes()


def facet_section(rng, term_id, fcode, keys, docids):
    """One query term's facet list as Msg39 serializes its m_facetHashTable
    (Msg39.cpp:1513-1550): i64 termid, i32 n, n x (i32 key, FacetEntry), in
    hash-slot order (here shuffled)."""
    e = np.zeros(len(keys), FE)
    e["key"] = keys
    e["count"] = rng.integers(0, 6, len(keys))
    e["count"][rng.random(len(keys)) < 0.15] = 0  # a range entry never voted into
    e["outside"] = e["count"] + rng.integers(0, 40, len(keys))
    e["docid"] = rng.choice(docids, len(keys)) if len(docids) else 0
    if fcode == FACET_FLOAT:
        vals = (rng.standard_normal((len(keys), 2)) * 1e3).astype(np.float32)
        e["min"] = np.minimum(vals[:, 0], vals[:, 1]).view(np.int32)
        e["max"] = np.maximum(vals[:, 0], vals[:, 1]).view(np.int32)
        e["sum"] = (rng.standard_normal(len(keys)) * 1e4 + 0.1).astype(np.float64).view(np.int64)
    else:
        a = rng.integers(-10**6, 10**6, (len(keys), 2)).astype(np.int32)
        e["min"] = a.min(1)
        e["max"] = a.max(1)
        e["sum"] = rng.integers(-10**12, 10**12, len(keys))
    e = e[rng.permutation(len(keys))]
    return np.array([term_id], "<i8").tobytes() + np.array([len(keys)], "<i4").tobytes() + e.tobytes()


def full_reply(rng, lo, hi, n, nsites, fterms, key_pool, rec_kinds=True, int_scores=False):
    """One shard: n docids of [lo, hi) best first, with cluster records over
    nsites site hashes and facet lists for fterms = [(term_id, fcode)]."""
    d = rng.choice(np.arange(lo, hi), size=n, replace=False).astype(np.int64) if n else np.zeros(0, np.int64)
    if int_scores:
        s = rng.integers(-20, 20, n).astype(np.float64)
    else:
        s = (rng.integers(1, 12, n).astype(np.float32) * np.float32(1.25)).astype(np.float64)
    d, s = _sorted(d, s)
    recs = []
    for x in d:
        k = rng.random() if rec_kinds else 1.0
        if k < 0.08:
            recs.append(bytes(12))  # not found in clusterdb: passes the cap (Msg3a.cpp:1343-1347)
        elif k < 0.14:
            recs.append(cluster_rec(int(x), int(rng.integers(0, nsites)), adult=True))
        elif k < 0.20:
            recs.append(cluster_rec(int(x), 0))  # site hash 0: counted, never capped
        else:
            recs.append(cluster_rec(int(x), int(rng.integers(1, nsites + 1)), lang=int(rng.integers(0, 5))))
    fl = b"".join(facet_section(rng, tid, fc, np.sort(rng.choice(key_pool, size=int(rng.integers(0, len(key_pool) + 1)),
                                                                   replace=False)).astype(np.int32), d)
                  for tid, fc in fterms)
    return dict(docids=d, scores=s, recs=b"".join(recs), hits=int(rng.integers(n, n + 5000)), facets=fl)


def full_cases():
    """[(name, req, shards)]: req = dict(docs_to_get, clus, hide, family,
    tids, fcs); shards = [dict(docids, scores, recs (bytes or None), hits,
    facets (bytes), fcounts (int64[nqt] or None))]"""
    rng = np.random.default_rng(0x3A3)
    out = []

    def req(dtg, clus=1, hide=0, family=0, fcs=(0, FACET_INT, FACET_FLOAT, FACET_STR)):
        tids = [1000003 * (i + 1) for i in range(len(fcs))]
        return dict(docs_to_get=dtg, clus=clus, hide=hide, family=family, tids=tids, fcs=list(fcs))

    def shards(r, ns, per, nsites, key_pool, lohi=None, **kw):
        fterms = [(t, f) for t, f in zip(r["tids"], r["fcs"]) if f in (FACET_STR, FACET_INT, FACET_FLOAT)]
        sh = []
        for j in range(ns):
            lo, hi = lohi(j) if lohi else (j * (MAXD // ns) + (1 << 30), j * (MAXD // ns) + (1 << 30) + 40 * per)
            x = full_reply(rng, lo, hi, int(rng.integers(per // 2, per + 1)), nsites, fterms, key_pool, **kw)
            x["fcounts"] = rng.integers(0, 10**6, len(r["tids"])).astype(np.int64)
            sh.append(x)
        return sh

    keys = np.arange(-40, 40, 3)
    r = req(20)
    out.append(("clus3_sites6", r, shards(r, 3, 30, 6, keys)))
    r = req(50)
    out.append(("clus4_sites3", r, shards(r, 4, 40, 3, keys)))
    r = req(30, hide=1)
    out.append(("clus3_hideall", r, shards(r, 3, 30, 5, keys)))
    r = req(30, family=1)
    out.append(("clus3_family", r, shards(r, 3, 30, 5, keys)))
    r = req(100, clus=0)
    out.append(("noclus3_facets", r, shards(r, 3, 60, 5, keys)))
    r = req(10)
    out.append(("clus8_k10", r, shards(r, 8, 25, 4, keys)))
    # docids below 2^29: n1 = 0, so the cap passes them (Msg3a.cpp:1346-1347)
    r = req(25)
    out.append(("clus3_low_docids", r, shards(r, 3, 20, 3, keys, lohi=lambda j: (j * 4000 + 1, j * 4000 + 3000))))
    # twin replicas: the same docids and records on two shards (counted
    # against the site before the docid is found merged, Msg3a.cpp:1342-1385)
    r = req(40)
    a = shards(r, 2, 40, 4, keys)
    out.append(("clus_twins", r, [a[0], a[1], a[0], a[1]]))
    # int scores (gbsortby int: (double)m_intScore) and one float facet only
    r = req(40, fcs=(0, FACET_FLOAT))
    out.append(("clus3_int_scores", r, shards(r, 3, 40, 5, keys, int_scores=True)))
    # a facet list naming a termid the query lacks ends the walk over the
    # replies, its own and every later reply's lists (the `break` of
    # Msg3a.cpp:1156-1162 leaves the loop over j); a termid held by two
    # terms goes to the first
    r = req(30, fcs=(0, FACET_INT, FACET_INT))
    r["tids"][2] = r["tids"][1]
    sh = shards(r, 3, 30, 5, keys)
    sh[1]["facets"] = (facet_section(rng, 999, FACET_INT, np.arange(3, dtype=np.int32), sh[1]["docids"]) +
                       sh[1]["facets"])
    sh[2]["facets"] = sh[2]["facets"] + facet_section(rng, 999, FACET_INT, np.arange(2, dtype=np.int32),
                                                      sh[2]["docids"])
    out.append(("clus3_facet_termids", r, sh))
    r = req(30, fcs=(0, FACET_INT, FACET_STR))
    sh = shards(r, 4, 30, 5, keys)
    sh[2]["facets"] = sh[2]["facets"] + facet_section(rng, 999, FACET_INT, np.arange(2, dtype=np.int32),
                                                      sh[2]["docids"])
    out.append(("clus4_facet_termid_last", r, sh))
    # empty replies, a shard with no facet list and no counts, no facet terms
    r = req(20)
    sh = shards(r, 4, 20, 4, keys)
    sh[1] = dict(docids=np.zeros(0, np.int64), scores=np.zeros(0), recs=b"", hits=0, facets=b"", fcounts=None)
    sh[3]["facets"] = b""
    out.append(("clus4_empty_some", r, sh))
    r = req(20, fcs=(0, 0))
    out.append(("clus5_no_facets", r, shards(r, 5, 30, 4, keys)))
    r = req(200)
    out.append(("clus8_k200_big_facets", r, shards(r, 8, 150, 20, np.arange(-3000, 3000, 7))))
    return out


def save_full(path, name, req, shards, exp=None):
    """one full-reply case (+ the reference's merge) as an .npz of plain arrays"""
    ns = len(shards)
    nqt = len(req["tids"])
    z = dict(req=np.array([ns, req["docs_to_get"], req["clus"], req["hide"], req["family"], nqt], np.int32),
             tids=np.array(req["tids"], np.int64), fcs=np.array(req["fcs"], np.int32),
             counts=np.array([len(s["docids"]) for s in shards], np.int32),
             docids=np.concatenate([s["docids"] for s in shards] + [np.zeros(0, np.int64)]),
             scores=np.concatenate([s["scores"] for s in shards] + [np.zeros(0)]),
             has_recs=np.array([s["recs"] is not None for s in shards], np.int32),
             recs=np.frombuffer(b"".join(s["recs"] or b"" for s in shards), np.uint8),
             hits=np.array([s["hits"] for s in shards], np.int32),
             fsizes=np.array([len(s["facets"]) for s in shards], np.int32),
             fblob=np.frombuffer(b"".join(s["facets"] for s in shards), np.uint8),
             has_fc=np.array([s["fcounts"] is not None for s in shards], np.int32),
             fcounts=np.concatenate([s["fcounts"] if s["fcounts"] is not None else np.zeros(nqt, np.int64)
                                     for s in shards] + [np.zeros(0, np.int64)]))
    if exp is not None:
        z.update(exp_docids=exp["docids"], exp_scores=exp["scores"],
                 exp_recs=np.frombuffer(exp["recs"] or b"", np.uint8), exp_has_recs=np.int32(exp["recs"] is not None),
                 exp_hits=np.int64(exp["hits"]), exp_fdocs=exp["fdocs"],
                 exp_tcounts=np.array([len(t) for t in exp["tables"]], np.int32),
                 exp_tables=np.concatenate(exp["tables"] + [np.zeros(0, FE)]).view(np.uint8))
    np.savez_compressed(path, **z)


def load_full(path):
    """-> (name, req, shards, exp) as save_full took them"""
    import os
    z = np.load(path, allow_pickle=False)
    ns, dtg, clus, hide, family, nqt = (int(x) for x in z["req"])
    req = dict(docs_to_get=dtg, clus=clus, hide=hide, family=family, tids=list(z["tids"]), fcs=list(z["fcs"]))
    shards, o, ro, fo = [], 0, 0, 0
    for j in range(ns):
        n = int(z["counts"][j])
        hr = bool(z["has_recs"][j])
        fs = int(z["fsizes"][j])
        shards.append(dict(docids=z["docids"][o:o + n], scores=z["scores"][o:o + n],
                           recs=z["recs"][ro:ro + 12 * n].tobytes() if hr else None, hits=int(z["hits"][j]),
                           facets=z["fblob"][fo:fo + fs].tobytes(),
                           fcounts=z["fcounts"][j * nqt:(j + 1) * nqt] if z["has_fc"][j] else None))
        o += n
        ro += 12 * n if hr else 0
        fo += fs
    exp = None
    if "exp_docids" in z:
        tabs, t, k = [], z["exp_tables"].view(FE), 0
        for c in z["exp_tcounts"]:
            tabs.append(t[k:k + c])
            k += c
        exp = dict(docids=z["exp_docids"], scores=z["exp_scores"],
                   recs=z["exp_recs"].tobytes() if int(z["exp_has_recs"]) else None, hits=int(z["exp_hits"]),
                   fdocs=z["exp_fdocs"], tables=tabs)
    return os.path.basename(path)[:-4], req, shards, exp


def facet_contributions(req, shards):
    """{(term, key): [docid of every entry merged into it, in merge order]}:
    the reference keeps one of them at random (Msg3a.cpp:1232-1233)"""
    tid_term = {}
    for i, t in enumerate(req["tids"]):
        tid_term.setdefault(int(t), i)
    out = {}
    for s in shards:
        b, p = s["facets"], 0
        while p < len(b):
            tid = int(np.frombuffer(b, "<i8", 1, p)[0])
            nh = int(np.frombuffer(b, "<i4", 1, p + 8)[0])
            p += 12
            if tid not in tid_term:
                return out
            e = np.frombuffer(b, FE, nh, p)
            p += 36 * nh
            for x in e:
                out.setdefault((tid_term[tid], int(x["key"])), []).append(int(x["docid"]))
    return out
