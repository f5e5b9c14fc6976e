"""RdbList::posdbMerge_r (RdbList.cpp:3065-3568) on the GPU -- config 5.

Parity bar: the merged output BYTES are identical to the reference's
(tests/golden/m_*.npz, made by the reference's own RdbList::merge_r) and to the
oracle restatement (oracle/posdb_merge_oracle.c) on seeded tiered runs, for
removeNegKeys on/off and minRecSizes cuts; the cases the reference's loop
distinguishes are covered: cross-run duplicates (newest wins, delete bit
included), delete keys, keys equal within one run, empty runs, a single run,
many runs, a first key that is not 18 bytes (EINVAL) and cuts that land on
every key size.  CPU tests pin the config-5 generator (csrc/synth.cpp) to the
oracle; GPU tests go through the C ABI (gbgpu_merge_posdb)."""
import ctypes

import numpy as np
import pytest

import gbgpu
import oracle_binding as orc
from mergegen import tiered_runs
from test_golden import MCASES, orc_merge, split_blob


def orc_merge_rc(runs, rm, mrs, cap):
    keep, ptrs, sizes = orc._lists(runs)
    out = ctypes.create_string_buffer(max(cap, 1))
    n = orc.lib().orc_posdb_merge(ptrs, sizes, len(runs), rm, mrs, out, cap)
    return (n, b"") if n < 0 else (0, out.raw[:n])


def key_stream(blob):
    """Decompress a posdb list into 18-byte keys (hi, lo, base as ints)."""
    out, i, hi, lo = [], 0, None, None
    while i < len(blob):
        b0 = blob[i]
        ks = 6 if b0 & 4 else (12 if b0 & 2 else 18)
        base = int.from_bytes(blob[i:i + 6], "little")
        if ks >= 12:
            lo = int.from_bytes(blob[i + 6:i + 12], "little")
        if ks == 18:
            hi = int.from_bytes(blob[i + 12:i + 18], "little")
        out.append((hi, lo, base))
        i += ks
    return out


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("seed", [1, 2])
def test_generator_runs_are_canonical_sorted_lists(seed):
    runs = gbgpu.synth_merge_runs(60000, nruns=8, seed=seed, nterms=300)
    sizes = [len(r) for r in runs]
    assert all(s % 6 == 0 for s in sizes) and sizes[-1] > 20 * sizes[0]
    for r in runs:
        # a single sorted canonical run merges to itself
        assert orc_merge([r], 0, -1) == r
        ks = [(h, l, b | 7) for h, l, b in key_stream(r)]
        assert ks == sorted(ks) and len(set(ks)) == len(ks)


def test_generator_is_thread_count_independent():
    a = gbgpu.synth_merge_runs(50000, nruns=4, seed=7, nterms=100, nthreads=1)
    b = gbgpu.synth_merge_runs(50000, nruns=4, seed=7, nterms=100, nthreads=5)
    assert a == b


def test_oracle_dedup_rule_newest_wins():
    # same key in runs 0 and 2 (delete bit differs): run 2's copy survives
    k = gbgpu.make_key(77, 123456, 100, 3, 15, 15, 2, 0, 1, 0, 0, 0, 0)
    neg = bytes([k[0] & 0xFE]) + k[1:]
    other = gbgpu.make_key(78, 5, 9, 3, 15, 15, 2, 0, 1, 0, 0, 0, 0)
    runs = [k, other, neg]
    assert orc_merge(runs, 0, -1) == gbgpu.compress(neg + other)
    assert orc_merge(runs, 1, -1) == gbgpu.compress(other)


# ------------------------------------------------------------------ GPU
def gpu_vs_oracle(engine, runs, rm, mrs, cap=None):
    cap = sum(map(len, runs)) + 64 if cap is None else cap
    rc, want = orc_merge_rc(runs, rm, mrs, cap)
    if rc < 0:
        with pytest.raises(gbgpu.GbgpuError) as ei:
            engine.merge_posdb(runs, rm, mrs, cap)
        assert ei.value.code == -rc
        return
    got = engine.merge_posdb(runs, rm, mrs, cap)
    assert got == want, (len(got), len(want), rm, mrs)
    lk = engine.merge_last_key()
    if not want:
        assert lk is None
    else:
        h, l, b = key_stream(want)[-1]
        assert lk == (b & ~0x06).to_bytes(6, "little") + l.to_bytes(6, "little") + h.to_bytes(6, "little")


@pytest.mark.gpu
@pytest.mark.parametrize("path", MCASES, ids=[p.rsplit("/", 1)[1][2:-4] for p in MCASES])
def test_gpu_merge_vs_reference(engine, path):
    z = np.load(path, allow_pickle=False)
    runs = split_blob(z["run_sizes"], z["run_blob"])
    outs = split_blob(z["out_sizes"], z["out_blob"])
    for rm, mrs, want in zip(z["remove_neg"], z["min_rec_sizes"], outs):
        assert engine.merge_posdb(runs, bool(rm), int(mrs)) == want, (int(rm), int(mrs))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12, 13])
@pytest.mark.parametrize("rm", [0, 1])
def test_gpu_merge_tiered_runs(engine, merge_path, seed, rm):
    runs = tiered_runs(20000, nruns=8, seed=seed, dup_frac=0.1, neg_frac=0.05, nterms=50)
    total = sum(map(len, runs))
    for mrs in (-1, 1, 6, 100, 4099, total // 3, total - 7, total + 100):
        gpu_vs_oracle(engine, runs, rm, mrs)


@pytest.mark.gpu
@pytest.mark.parametrize("nruns", [1, 2, 3, 5, 20, 64])
def test_gpu_merge_run_counts(engine, merge_path, nruns):
    runs = tiered_runs(6000, nruns=nruns, seed=20 + nruns, dup_frac=0.3, neg_frac=0.1, nterms=20)
    for rm in (0, 1):
        gpu_vs_oracle(engine, runs, rm, -1)
        gpu_vs_oracle(engine, runs, rm, sum(map(len, runs)) // 2)


@pytest.mark.gpu
def test_gpu_merge_heavy_duplicates(engine, merge_path):
    # half the keys repeated across runs: long tie chains, flipped delete bits
    runs = tiered_runs(30000, nruns=6, seed=3, dup_frac=0.5, neg_frac=0.2, nterms=5)
    for rm in (0, 1):
        gpu_vs_oracle(engine, runs, rm, -1)


@pytest.mark.gpu
def test_gpu_merge_generator_runs(engine, merge_path):
    runs = gbgpu.synth_merge_runs(400000, nruns=8, seed=9, nterms=2000)
    for rm in (0, 1):
        gpu_vs_oracle(engine, runs, rm, -1)
    gpu_vs_oracle(engine, runs, 1, 1 << 20)


@pytest.mark.gpu
def test_gpu_merge_edge_cases(engine, merge_path):
    k1 = gbgpu.make_key(5, 1000, 10, 1, 15, 15, 3, 0, 1, 0, 0, 0, 0)
    k2 = gbgpu.make_key(5, 1000, 20, 1, 15, 15, 3, 0, 1, 0, 0, 0, 0)
    k3 = gbgpu.make_key(5, 2000, 30, 1, 15, 15, 3, 0, 1, 0, 0, 0, 0)
    k4 = gbgpu.make_key(6, 5, 30, 1, 15, 15, 3, 0, 1, 0, 0, 0, 0)
    one = gbgpu.compress(k1)
    assert engine.merge_posdb([], 0, -1) == b""
    assert engine.merge_posdb([b"", b""], 0, -1) == b""
    assert engine.merge_posdb([one], 0, 0) == b""           # minRecSizes 0: nothing
    gpu_vs_oracle(engine, [one], 0, -1)
    gpu_vs_oracle(engine, [b"", one, b""], 1, -1)
    # interleaved runs: 6-byte keys become 12/18 bytes in the output
    gpu_vs_oracle(engine, [gbgpu.compress(k1 + k3), gbgpu.compress(k2 + k4)], 0, -1)
    # the same key three times in one run (not canonical) and once in an older run
    dup3 = gbgpu.compress(k1) + (bytes([k1[0] | 0x06]) + k1[1:6]) * 2
    gpu_vs_oracle(engine, [gbgpu.compress(k1 + k2), dup3], 0, -1)
    gpu_vs_oracle(engine, [dup3, gbgpu.compress(k1 + k2)], 0, -1)
    # a run whose first key is not 18 bytes: EINVAL as in the oracle
    bad = bytes([k1[0] | 0x02]) + k1[1:12]
    gpu_vs_oracle(engine, [one, bad], 0, -1)
    # every cut position, small and large capacity
    runs = [gbgpu.compress(k1 + k3), gbgpu.compress(k2 + k4)]
    for mrs in range(1, 80, 5):
        gpu_vs_oracle(engine, runs, 0, mrs)
    for cap in (0, 5, 18, 30, 40, 200):
        gpu_vs_oracle(engine, runs, 0, -1, cap=cap)


@pytest.mark.gpu
def test_gpu_merge_large_vs_oracle_and_properties(engine):
    # ~25 M keys (~250 MB of runs): bit-exact against the oracle, and the
    # size-independent properties: idempotent (merging the output alone
    # returns it) and every key survives exactly once
    m = gbgpu.MergeRuns(25_000_000, nruns=8, seed=21, nterms=20000)
    try:
        runs = m.as_bytes()
    finally:
        m.free()
    got = engine.merge_posdb(runs, False, -1)
    _, want = orc_merge_rc(runs, 0, -1, sum(map(len, runs)) + 64)
    assert got == want
    assert engine.merge_posdb([got], False, -1) == got
    got1 = engine.merge_posdb(runs, True, -1)
    assert engine.merge_posdb([got1], True, -1) == got1
    _, nk, nt = engine.merge_timings()
    assert nk > 0 and nt > 0


@pytest.fixture
def merge_path():
    """The merge pipeline every merge runs (gbgpu_merge_path): 2, the decoded
    keys (the tile pipeline, 1, was retired in round 4: DESIGN.md §3b)."""
    return 2


@pytest.mark.gpu
def test_gpu_merge_paths_agree(engine, merge_path):
    # 8 and 40 runs: the oracle's bytes, and the pipeline reported
    runs = tiered_runs(30000, nruns=8, seed=31, dup_frac=0.2, neg_frac=0.05, nterms=30)
    total = sum(map(len, runs))
    for rm in (0, 1):
        gpu_vs_oracle(engine, runs, rm, -1)
        assert engine.merge_path() == merge_path
    gpu_vs_oracle(engine, runs, 0, total // 3)
    many = tiered_runs(8000, nruns=40, seed=32, dup_frac=0.2, neg_frac=0.05, nterms=30)
    gpu_vs_oracle(engine, many, 0, -1)
    assert engine.merge_path() == 2


def _run(term, docid, wordpos):
    from mergegen import pack_keys, to_bytes, _order
    n = len(docid)
    z = np.zeros(n, dtype=np.uint32)
    n0, n1, n2 = pack_keys(np.full(n, term, dtype=np.uint64), np.asarray(docid, dtype=np.uint64),
                           np.asarray(wordpos, dtype=np.uint32), z + 3, z + 15, z + 15, z + 2, z, z + 1, z, z + 1)
    o = _order(n0, n1, n2)
    return gbgpu.compress(to_bytes(n0[o], n1[o], n2[o]))


@pytest.mark.gpu
def test_gpu_merge_long_carries(engine, merge_path):
    # one docid with 30000 positions: 6-byte keys whose lo and hi units lie
    # thousands of units back (the decode inherits them through the chunk
    # carries of k_mscan); a newer run interleaves docids around it and
    # repeats some of its keys
    d = 1 << 30
    a = _run(77, np.full(30000, d), np.arange(30000))
    b = _run(77, np.concatenate([np.arange(d - 3000, d + 3000), np.full(500, d)]),
             np.concatenate([np.full(6000, 7), np.arange(0, 30000, 60)]))
    c = _run(78, np.arange(1, 4000), np.full(3999, 1))
    for runs in ([a, b, c], [c, a, b], [a]):
        for rm in (0, 1):
            gpu_vs_oracle(engine, runs, rm, -1)
            assert engine.merge_path() == merge_path
        gpu_vs_oracle(engine, runs, 0, sum(map(len, runs)) // 2)
