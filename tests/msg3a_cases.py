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
