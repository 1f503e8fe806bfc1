"""Parity of the MI355X product (libsyzsig.so, through its C-ABI) with the
oracle and the reference's own known answers.  Bit-exact everywhere: this path
is integer / index work only."""
import numpy as np
import pytest

from oracle import pyoracle as O
from tests import refmodel as R

pytestmark = pytest.mark.gpu

SENT = 0xFFFFFFFF


@pytest.fixture(scope="module")
def C(ctx):
    from syzkaller_amd import cover

    return cover


def zipf_batch(rng, nprog, calls, pcs, s=1.1, nranks=1 << 16, ragged=False):
    """Synthetic Zipf traces -> per-call signal through the executor restatement."""
    lens = (rng.integers(0, 2 * pcs, size=nprog * calls) if ragged else np.full(nprog * calls, pcs)).astype(np.uint64)
    call_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    ranks = np.minimum(rng.zipf(s, size=int(call_off[-1])), nranks) - 1
    trace = (0x81000000 + 16 * ranks).astype(np.uint32)
    prog_off = (np.arange(nprog + 1) * calls).astype(np.uint64)
    return O.exec_signal(trace, call_off, prog_off)


# ---- pkg/cover KATs through the product (cover_test.go) -------------------------
OPS = {"TestDifference": "Difference", "TestSymmetricDifference": "SymmetricDifference", "TestUnion": "Union",
       "TestIntersection": "Intersection"}


def _cases(t):
    cases = [(c["v0"], c["v1"], c["r"]) for c in t["cases"]]
    if t["symmetric"]:
        cases += [(b, a, r) for a, b, r in cases]
    cases.append(([], [], []))
    return cases


@pytest.mark.parametrize("name", sorted(OPS))
def test_kat_ops(C, kats, name):
    f = getattr(C, OPS[name])
    for v0, v1, r in _cases(kats[name]):
        res = f(np.array(v0, np.uint32), np.array(v1, np.uint32))
        assert list(res) == r
        assert list(res) == sorted(res)


def test_kat_canonicalize(C, kats):
    for v0, _, r in _cases(kats["TestCanonicalize"]):
        assert list(C.Canonicalize(np.array(v0, np.uint32))) == r


def test_kat_minimize(C, kats):
    for case in kats["TestMinimize"]["cases"]:
        assert C.Minimize([np.array(c, np.uint32) for c in case["inp"]]) == case["out"]


# ---- random parity with the oracle ---------------------------------------------
def test_ops_random_vs_oracle(C):
    rng = np.random.default_rng(100)
    for it in range(300):
        n0, n1 = (int(x) for x in rng.integers(0, 40, size=2))
        hi = [4, 64, 1 << 32][it % 3]
        a = np.sort(rng.integers(0, hi, size=n0, dtype=np.uint64)).astype(np.uint32)
        b = np.sort(rng.integers(0, hi, size=n1, dtype=np.uint64)).astype(np.uint32)
        if it % 5 == 0:
            a = np.sort(np.concatenate([a, np.full(int(rng.integers(1, 3)), SENT, np.uint32)]))
        if it % 7 == 0:
            b = np.sort(np.concatenate([b, np.full(1, SENT, np.uint32)]))
        for op, f in enumerate([C.Difference, C.SymmetricDifference, C.Union, C.Intersection]):
            assert np.array_equal(f(a, b), O.foreach(op, a, b)), (op, a, b)
        assert C.HasDifference(a, b) == O.has_difference(a, b)


def test_ops_large_multiset(C):
    rng = np.random.default_rng(101)
    for n0, n1, hi in [(100000, 3000, 5000), (4096, 1 << 20, 1 << 22), (70000, 70000, 1 << 30)]:
        a = np.sort(rng.integers(0, hi, size=n0)).astype(np.uint32)
        b = np.sort(rng.integers(0, hi, size=n1)).astype(np.uint32)
        for op, f in enumerate([C.Difference, C.SymmetricDifference, C.Union, C.Intersection]):
            assert np.array_equal(f(a, b), O.foreach(op, a, b)), (op, n0, n1)
        assert C.HasDifference(a, b) == O.has_difference(a, b)
        assert C.HasDifference(b, a) == O.has_difference(b, a)


def test_has_difference_batch_vs_oracle(C):
    """sg_has_difference_batch against the oracle's HasDifference per pair:
    empty sides, duplicates (the t-th copy against b's count), sentinels, equal
    lists, a shared b, and pairs longer than a workgroup's stride."""
    from syzkaller_amd import cover as cv

    rng = np.random.default_rng(131)
    pairs = [(np.zeros(0, np.uint32), np.zeros(0, np.uint32)), (np.array([5], np.uint32), np.zeros(0, np.uint32)),
             (np.zeros(0, np.uint32), np.array([5], np.uint32)), (np.array([3, 3], np.uint32), np.array([3], np.uint32)),
             (np.array([3], np.uint32), np.array([3, 3], np.uint32)),
             (np.array([SENT], np.uint32), np.array([SENT], np.uint32)), (np.array([1, SENT], np.uint32), np.array([1], np.uint32))]
    shared = np.sort(rng.integers(0, 3000, size=20000)).astype(np.uint32)
    for it in range(200):
        n0 = int(rng.integers(0, 3000 if it % 10 == 0 else 40))
        hi = [4, 64, 3000, 1 << 32][it % 4]
        a = np.sort(rng.integers(0, hi, size=n0, dtype=np.uint64)).astype(np.uint32)
        if it % 3 == 0:
            b = shared
        elif it % 3 == 1:
            b = a.copy() if it % 2 else np.sort(rng.integers(0, hi, size=int(rng.integers(0, 40)), dtype=np.uint64)).astype(np.uint32)
        else:
            b = np.sort(np.concatenate([a, rng.integers(0, hi, size=5, dtype=np.uint64).astype(np.uint32)]))
        pairs.append((a, b))
    av = np.concatenate([p[0] for p in pairs])
    al = np.array([p[0].size for p in pairs], np.uint64)
    ab = np.concatenate([[0], np.cumsum(al)[:-1]]).astype(np.uint64)
    bl = np.array([p[1].size for p in pairs], np.uint64)
    bv = np.concatenate([p[1] for p in pairs])
    bb = np.concatenate([[0], np.cumsum(bl)[:-1]]).astype(np.uint64)
    got = cv.has_difference_batch(av, ab, al, bv, bb, bl)
    want = np.array([O.has_difference(a, b) for a, b in pairs])
    assert np.array_equal(got, want)
    assert 0 < want.sum() < len(pairs)


def test_merge_batch_small_side_multisets(C):
    """The one-small-side merge (sg_merge.hip k_merge_small): pairs whose
    small list fits in LDS against large lists with long runs of one value
    (across its 4096-element tiles), sentinels on both sides, either side
    small, and a mix with a pair too large for it (generic path); then
    Difference / Intersection with every first list small (k_diff_small)."""
    rng = np.random.default_rng(115)
    lists = []
    for it in range(24):
        ns = int(rng.integers(0, 4097))
        nl = int(rng.integers(0, 30000))
        hi = [8, 300, 1 << 20, 1 << 32][it % 4]
        small = np.sort(rng.integers(0, hi, size=ns, dtype=np.uint64)).astype(np.uint32)
        large = rng.integers(0, hi, size=nl, dtype=np.uint64)
        if it % 3 == 0 and nl:  # a run of one value over several tiles
            large[: nl // 2] = large[0]
        large = np.sort(large).astype(np.uint32)
        if it % 5 == 0:
            small = np.sort(np.concatenate([small, np.full(2, SENT, np.uint32)]))
        if it % 4 == 1:
            large = np.sort(np.concatenate([large, np.full(3, SENT, np.uint32)]))
        lists.append((small, large) if it % 2 else (large, small))
    # and every first list small (Difference / Intersection: k_diff_small)
    firsts = [(x, y) if x.size <= y.size else (y, x) for x, y in lists]
    for op, pairs in [(op, lists) for op in range(4)] + [(0, firsts), (3, firsts)]:
        a = np.concatenate([x for x, _ in pairs])
        b = np.concatenate([y for _, y in pairs])
        al = np.array([x.size for x, _ in pairs], np.uint64)
        bl = np.array([y.size for _, y in pairs], np.uint64)
        ab = np.concatenate([[0], np.cumsum(al)[:-1]]).astype(np.uint64)
        bb = np.concatenate([[0], np.cumsum(bl)[:-1]]).astype(np.uint64)
        outs = C.merge_batch(op, a, ab, al, b, bb, bl)
        for k, (x, y) in enumerate(pairs):
            assert np.array_equal(outs[k], O.foreach(op, x, y)), (op, k, x.size, y.size)


def test_has_difference_property(C):
    # cover_test.go:210-221
    rng = np.random.default_rng(102)
    for _ in range(200):
        a = C.Canonicalize(rng.integers(0, 100, size=rng.integers(0, 20)).astype(np.uint32))
        b = C.Canonicalize(rng.integers(0, 100, size=rng.integers(0, 20)).astype(np.uint32))
        assert C.HasDifference(a, b) == (C.Difference(a, b).size != 0)


def test_merge_batch_shared_corpus(C):
    # C1 shape in miniature: many traces vs one corpus signal, Union and Difference
    rng = np.random.default_rng(103)
    corpus = np.unique(rng.integers(0, 1 << 24, size=200000)).astype(np.uint32)
    traces = [np.sort(rng.integers(0, 1 << 24, size=int(rng.integers(0, 3000)))).astype(np.uint32) for _ in range(64)]
    a = np.concatenate(traces)
    a_len = np.array([t.size for t in traces], np.uint64)
    a_beg = np.concatenate([[0], np.cumsum(a_len)[:-1]]).astype(np.uint64)
    b_beg = np.zeros(64, np.uint64)
    b_len = np.full(64, corpus.size, np.uint64)
    for op in range(4):
        res = C.merge_batch(op, a, a_beg, a_len, corpus, b_beg, b_len)
        for k, t in enumerate(traces):
            assert np.array_equal(res[k], O.foreach(op, t, corpus)), (op, k)


def test_canonicalize_random_vs_oracle(C):
    rng = np.random.default_rng(104)
    for n in [0, 1, 2, 63, 64, 100, 4095, 4096, 4097, 8193, 20000, 70000, 300000]:
        for hi in [3, 1000, 1 << 32]:
            v = rng.integers(0, hi, size=n, dtype=np.uint64).astype(np.uint32)
            if n and hi == 3:
                v[rng.integers(0, n)] = SENT
            exp, m = O.canonicalize(v)
            got = v.copy()
            res = C.Canonicalize(got)
            assert res.size == m and np.array_equal(res, exp[:m]), (n, hi)
            assert np.array_equal(got, exp), (n, hi)  # whole slice, stale tail included


def test_canonicalize_batch_ragged(C):
    rng = np.random.default_rng(105)
    lens = [0, 5, 4096, 1, 0, 9000, 33, 70000, 4097, 2, 16384]
    segs = [rng.integers(0, [10, 1 << 32][k % 2], size=L, dtype=np.uint64).astype(np.uint32) for k, L in enumerate(lens)]
    segs[3][:] = SENT
    vals = np.concatenate(segs)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    got = vals.copy()
    out_len = C.canonicalize_batch(got, off)
    for k in range(len(lens)):
        exp, m = O.canonicalize(segs[k])
        assert out_len[k] == m
        assert np.array_equal(got[off[k]:off[k + 1]], exp)


def test_canonicalize_batch_tile_segments(C):
    """Every segment <= 4096 (the one-pass sort + unique in LDS): empty
    segments, sentinel-only and sentinel-tailed ones, all-equal values, full
    4096-element segments, and many short lists."""
    rng = np.random.default_rng(132)
    lens = [0, 1, 4096, 0, 3, 4095, 64, 65, 2] + [int(x) for x in rng.integers(0, 300, size=400)] + [0]
    # the wave-per-list sizes (<= 1024: 64-1024-slot networks) and their edges
    lens += [127, 128, 129, 255, 256, 257, 511, 512, 513, 1023, 1024, 1025, 2048]
    lens += [int(x) for x in rng.integers(0, 1100, size=200)]
    segs = []
    for k, L in enumerate(lens):
        v = rng.integers(0, [4, 1000, 1 << 32][k % 3], size=L, dtype=np.uint64).astype(np.uint32)
        if k % 7 == 1 and L:
            v[:] = SENT
        elif k % 7 == 2 and L:
            v[rng.integers(0, L)] = SENT
        elif k % 7 == 3:
            v[:] = 9
        segs.append(v)
    vals = np.concatenate(segs)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    got = vals.copy()
    out_len = C.canonicalize_batch(got, off)
    for k in range(len(lens)):
        exp, m = O.canonicalize(segs[k])
        assert out_len[k] == m, k
        assert np.array_equal(got[off[k]:off[k + 1]], exp), k


def test_minimize_vs_oracle(C):
    rng = np.random.default_rng(106)
    for n, hi in [(1, 5), (7, 20), (50, 100), (2000, 5000), (20000, 1 << 16)]:
        covs = [C.Canonicalize(rng.integers(0, hi, size=int(rng.integers(0, 60))).astype(np.uint32)) for _ in range(n)]
        vals, off = C.to_csr(covs)
        assert np.array_equal(C.minimize_csr(vals, off), O.minimize(vals, off)), n
        order = rng.permutation(n).astype(np.uint32)
        assert np.array_equal(C.minimize_csr(vals, off, order), O.minimize(vals, off, order)), n
        # non-canonical covers with duplicates and sentinels are processed the same way
        raw = [rng.integers(0, 8, size=int(rng.integers(0, 6))).astype(np.uint32) for _ in range(n)]
        rv, ro = C.to_csr(raw)
        rv[rv == 7] = SENT
        assert np.array_equal(C.minimize_csr(rv, ro, order), O.minimize(rv, ro, order)), n


def test_minimize_filtered_claim(C, ctx_option):
    """Minimize's filtered claim (sg_triage.hip k_min_claim_f): the values
    common to the first inputs in processing order fill an LDS set, and later
    elements found in it skip the owner table.  Phase A (the inputs claimed
    one workgroup each) is the first 4 inputs, or more
    (option minimize_filter_ranks); Zipf values (most later elements held),
    sentinels, empty inputs, inputs longer than a claim window, any
    processing order, and the unfiltered path (option minimize_filter 0)."""
    rng = np.random.default_rng(108)

    def corpus(n, med, hi, s=1.1):
        lens = np.clip(np.exp(rng.normal(np.log(med), 1.0, size=n)), 0, 20000).astype(np.int64)
        lens[rng.integers(0, n, size=n // 20)] = 0
        covs = []
        for L in lens:
            v = (np.minimum(rng.zipf(s, size=int(L)), hi) - 1).astype(np.uint64)
            v = (0x81000000 + 16 * v).astype(np.uint32)
            if rng.random() < 0.05 and L:
                v[0] = SENT
            covs.append(C.Canonicalize(v))
        return C.to_csr(covs)

    for n, med, hi, budget in [(3000, 40, 5000, "4"), (5000, 300, 1 << 20, "60"), (2500, 3000, 1 << 16, "1")]:
        vals, off = corpus(n, med, hi)
        dc = C.default_context()
        ctx_option(dc, "minimize_filter_ranks", int(budget))
        order = C.minimize_order(off)
        got = C.minimize_csr(vals, off, order)
        dc.set_option("minimize_filter_ranks", 0)
        assert np.array_equal(got, O.minimize(vals, off, order)), (n, budget)
        perm = rng.permutation(n).astype(np.uint32)
        dc.set_option("minimize_filter_ranks", int(budget))
        got = C.minimize_csr(vals, off, perm)
        dc.set_option("minimize_filter_ranks", 0)
        assert np.array_equal(got, O.minimize(vals, off, perm)), (n, budget)
    # just past phase A: one or two inputs left, empty inputs, all-sentinel inputs
    for covs in ([[1, 2, 3], [2, 3], [3], [3, 4], [4, 5]], [[7, 8], [], [8], [], [SENT], [8, 9], []],
                 [[SENT], [SENT], [SENT], [SENT], [SENT, 1], [1]]):
        v, o = C.to_csr([np.array(c, np.uint32) for c in covs])
        for order in (C.minimize_order(o), np.arange(len(covs), dtype=np.uint32)[::-1].copy()):
            assert np.array_equal(C.minimize_csr(v, o, order), O.minimize(v, o, order)), covs
    vals, off = corpus(12000, 200, 1 << 22)  # the default phase A
    order = C.minimize_order(off)
    assert np.array_equal(C.minimize_csr(vals, off, order), O.minimize(vals, off, order))
    ctx_option(C.default_context(), "minimize_filter", 0)
    assert np.array_equal(C.minimize_csr(vals, off, order), O.minimize(vals, off, order))


# ---- signal sets (map replacements) --------------------------------------------
def test_signal_set_ops(C):
    rng = np.random.default_rng(107)
    s = C.SignalSet()
    o = O.OSet()
    for it in range(20):
        add = rng.integers(0, 1 << 32, size=int(rng.integers(0, 5000)), dtype=np.uint64).astype(np.uint32)
        if it % 3 == 0:
            add = np.concatenate([add, np.array([0, SENT, 1, 0], np.uint32)])
        C.SignalAdd(s, add)
        o.add(add)
        probe = np.concatenate([add[: add.size // 2], rng.integers(0, 1 << 32, size=300, dtype=np.uint64).astype(np.uint32)])
        assert C.SignalNew(s, probe) == O.signal_new(o, probe)
        assert C.SignalNew(s, add) is False
        assert np.array_equal(C.SignalDiff(s, probe), O.signal_diff(o, probe))
    assert len(s) == len(o)
    assert np.array_equal(s.export(), o.export())
    s.clear()
    assert len(s) == 0 and s.export().size == 0


# ---- the hot path: batched new-signal triage (fuzzer.go:645-693) ----------------
class TwoPaths:
    """The same sets kept twice: one pair driven through the ordered-output
    path (the diff CSR from the bucket stage's first owners, sg_triage.hip
    owned_outputs), one through the flags-only partitioned path."""

    def __init__(self, C, ctx=None):
        self.C = C
        self.d = (C.SignalSet(ctx), C.SignalSet(ctx))
        self.f = (C.SignalSet(ctx), C.SignalSet(ctx))

    def add(self, vals):
        self.C.SignalAdd(self.d[0], vals)
        self.C.SignalAdd(self.f[0], vals)

    def clear(self):
        for s in self.d + self.f:
            s.clear()

    def triage(self, vals, off):
        flags, dv, do = self.C.triage_batch(self.d[0], self.d[1], vals, off)
        fflags, _, _ = self.C.triage_batch(self.f[0], self.f[1], vals, off, want_diff=False)
        assert np.array_equal(flags, fflags), "flags-only path disagrees with the ordered-output path"
        return flags, dv, do

    def exports(self):
        m, n = self.d[0].export(), self.d[1].export()
        assert np.array_equal(m, self.f[0].export()) and np.array_equal(n, self.f[1].export())
        return m, n


def _check_triage(P, osets, vals, off):
    om, on = osets
    flags, dv, do = P.triage(vals, off)
    ef, ev, eo = O.triage_batch(om, on, vals, off)
    assert np.array_equal(flags, ef)
    assert np.array_equal(do, eo)
    assert np.array_equal(dv, ev)
    return flags


def test_triage_small_vs_python(C):
    rng = np.random.default_rng(108)
    P = TwoPaths(C)
    for it in range(60):
        P.clear()
        nrec = int(rng.integers(0, 40))
        recs = [[int(x) for x in rng.integers(0, 80, size=rng.integers(0, 14))] for _ in range(nrec)]
        if it % 4 == 0 and nrec:
            recs[0] += [0, SENT, SENT]
        if it % 3 == 0:  # spread over many partition buckets
            recs = [[(x * 0x9E3779B1) & 0xFFFFFFFF for x in r] for r in recs]
        m0 = sorted(set(int(x) for x in rng.integers(0, 80, size=rng.integers(0, 50))))
        if it % 3 == 0:
            m0 = sorted(set((x * 0x9E3779B1) & 0xFFFFFFFF for x in m0))
        P.add(np.array(m0, np.uint32))
        vals = np.array([x for r in recs for x in r], dtype=np.uint32)
        off = np.concatenate([[0], np.cumsum([len(r) for r in recs])]).astype(np.uint64)
        flags, dv, do = P.triage(vals, off)
        pm, pn = set(m0), set()
        pf, pd = R.triage(pm, pn, recs)
        assert list(flags) == pf
        assert [list(dv[int(do[r]):int(do[r + 1])]) for r in range(nrec)] == pd
        m, n = P.exports()
        assert set(m.tolist()) == pm and set(n.tolist()) == pn


def test_triage_zipf_sequence_vs_oracle(C):
    """Several consecutive batches against the same sets (the fuzzer's steady
    state): exercises the decreasing owner-key generations."""
    rng = np.random.default_rng(109)
    P = TwoPaths(C)
    om, on = O.OSet(), O.OSet()
    warm, _ = zipf_batch(rng, 64, 8, 256)
    P.add(warm)
    om.add(warm)
    for b in range(6):
        vals, off = zipf_batch(rng, 128, 8, 512, ragged=(b % 2 == 1))
        flags = _check_triage(P, (om, on), vals, off)
        assert flags.sum() > 0
    m, n = P.exports()
    assert np.array_equal(m, om.export())
    assert np.array_equal(n, on.export())


def test_triage_edge_cases(C):
    P = TwoPaths(C)
    om, on = O.OSet(), O.OSet()
    cases = [
        (np.array([], np.uint32), np.array([0], np.uint64)),                  # no records
        (np.array([], np.uint32), np.array([0, 0, 0], np.uint64)),            # only empty records
        (np.array([0, SENT, 0, SENT], np.uint32), np.array([0, 2, 2, 4], np.uint64)),
        (np.array([7] * 5000, np.uint32), np.array([0, 2500, 5000], np.uint64)),  # dups within a record
        (np.arange(10000, dtype=np.uint32), np.array([0, 1, 1, 1, 4096, 4097, 8191, 10000], np.uint64)),
        (np.arange(10000, dtype=np.uint32), np.array([0, 10000], np.uint64)),  # everything already known
    ]
    for vals, off in cases:
        _check_triage(P, (om, on), vals, off)
    # many empty records around tile boundaries (record window > LDS window)
    rng = np.random.default_rng(110)
    lens = np.where(rng.random(20000) < 0.9, 0, rng.integers(1, 30, size=20000)).astype(np.uint64)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    vals = rng.integers(0, 1 << 20, size=int(off[-1])).astype(np.uint32)
    _check_triage(P, (om, on), vals, off)
    # records longer than a tile, unaligned lengths, one of them reaching every partition bucket
    lens = rng.integers(4000, 70000, size=12).astype(np.uint64)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    vals = rng.integers(0, 1 << 21, size=int(off[-1])).astype(np.uint32)
    vals[: int(lens[0])] = rng.integers(0, 1 << 32, size=int(lens[0]), dtype=np.uint64).astype(np.uint32)
    _check_triage(P, (om, on), vals, off)
    # a skewed batch: every value in one 32768-signal bucket, heavily repeated
    vals = (0xABC00000 + rng.integers(0, 32768, size=300000)).astype(np.uint32)
    off = np.concatenate([[0], np.sort(rng.integers(0, vals.size, size=999)), [vals.size]]).astype(np.uint64)
    _check_triage(P, (om, on), vals, off)
    # one coarse slice (s >> 23) spanning many partition tiles beside hundreds of
    # tiny ones, and a bucket whose distinct candidates nearly fill the LDS map
    big = (0x12000000 + rng.integers(0, 1 << 23, size=50000)).astype(np.uint32)
    tiny = ((rng.integers(0, 512, size=700) << 23) | rng.integers(0, 1 << 23, size=700)).astype(np.uint32)
    dense = (0x77700000 + rng.permutation(32768)[:3000]).astype(np.uint32)
    vals = np.concatenate([tiny[:300], big, dense, tiny[300:], dense[::-1], big[:999]])
    off = np.concatenate([[0], np.sort(rng.integers(0, vals.size, size=300)), [vals.size]]).astype(np.uint64)
    _check_triage(P, (om, on), vals, off)
    m, n = P.exports()
    assert np.array_equal(m, om.export()) and np.array_equal(n, on.export())


def test_triage_partition_geometry(C):
    """Inputs aimed at the partitioned path's tables (sg_bucket.hip): tiles cut
    by the 64-record cap (kRecCap), runs of >= 64 empty records (coinciding
    cuts), record counts around multiples of 64, several pass-2 groups of 1020
    tiles (kGroupTiles), one slice holding the whole batch, and a 2^16-signal
    bucket with more distinct candidates than its LDS map."""
    P = TwoPaths(C)
    om, on = O.OSet(), O.OSet()
    rng = np.random.default_rng(113)

    def run(vals, lens):
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        assert int(off[-1]) == vals.size
        _check_triage(P, (om, on), vals.astype(np.uint32), off)

    # tiny records: every tile hits the record cap long before 8192 entries
    lens = rng.integers(0, 4, size=40000)
    run(rng.integers(0, 1 << 32, size=int(lens.sum()), dtype=np.uint64), lens)
    # ~3200 tiles: four pass-2 groups, the last one partial
    lens = rng.integers(0, 3, size=200000)
    run(rng.integers(0, 1 << 32, size=int(lens.sum()), dtype=np.uint64), lens)
    # >= 64 consecutive empty records, at and around cap boundaries
    for nrec in (63, 64, 65, 127, 128, 129, 255, 256, 257, 1024):
        lens = np.zeros(nrec, np.int64)
        lens[rng.integers(0, nrec, size=5)] = rng.integers(1, 3000, size=5)
        lens[-1] += 7
        run(rng.integers(0, 1 << 32, size=int(lens.sum()), dtype=np.uint64), lens)
    lens = np.concatenate([np.full(300, 0), [9000], np.full(700, 0), [20000], np.full(64, 0), [3], np.full(130, 0), [5]])
    run(rng.integers(0, 1 << 32, size=int(lens.sum()), dtype=np.uint64), lens)
    # one top byte (slice) for everything: long runs, many chunks in one slice
    n = 3_000_000
    vals = (0x5A000000 | rng.integers(0, 1 << 24, size=n)).astype(np.uint64)
    lens = np.diff(np.concatenate([[0], np.sort(rng.integers(0, n, size=2999)), [n]]))
    run(vals, lens)
    # a bucket with ~20k distinct candidates (overflows the 8192-slot map), repeated
    base = 0x3C7A0000
    vals = base + rng.permutation(65536)[:20000].astype(np.uint64)
    vals = np.concatenate([vals, vals[::-1], rng.integers(0, 1 << 32, size=5000, dtype=np.uint64)])
    lens = np.diff(np.concatenate([[0], np.sort(rng.integers(0, vals.size, size=99)), [vals.size]]))
    run(vals, lens)
    m, nn = P.exports()
    assert np.array_equal(m, om.export()) and np.array_equal(nn, on.export())


@pytest.mark.slow
def test_triage_slice_over_lds_run_window(C):
    """A slice with more pass-2 chunks than the bucket kernel keeps in LDS
    (> 2048 chunks: > 16.7M entries sharing a top byte): the global run-search
    branch."""
    P = TwoPaths(C)
    om, on = O.OSet(), O.OSet()
    rng = np.random.default_rng(114)
    n = 18_000_000
    vals = (0xC3000000 | rng.integers(0, 1 << 24, size=n)).astype(np.uint32)
    off = np.concatenate([[0], np.sort(rng.integers(0, n, size=40000)), [n]]).astype(np.uint64)
    _check_triage(P, (om, on), vals, off)


def test_triage_flags_only_matches(C):
    rng = np.random.default_rng(111)
    ms, om = C.SignalSet(), O.OSet()
    vals, off = zipf_batch(rng, 64, 4, 300)
    flags, dv, do = C.triage_batch(ms, None, vals, off, want_diff=False)
    assert dv is None and do is None
    assert np.array_equal(flags, O.triage_flags_only(om, None, vals, off))
    assert np.array_equal(ms.export(), om.export())


# ---- manager / fuzzer merges ------------------------------------------------------
def test_add_inputs_vs_oracle(C):
    rng = np.random.default_rng(112)
    cs, ms = C.SignalSet(), C.SignalSet()
    oc, om = O.OSet(), O.OSet()
    m0 = rng.integers(0, 5000, size=3000).astype(np.uint32)
    C.SignalAdd(ms, m0)
    om.add(m0)
    for _ in range(3):
        inputs = [rng.integers(0, 8000, size=int(rng.integers(0, 200))).astype(np.uint32) for _ in range(100)]
        vals, off = C.to_csr(inputs)
        C.add_inputs(cs, ms, vals, off)
        O.add_inputs(oc, om, vals, off)
        assert np.array_equal(cs.export(), oc.export())
        assert np.array_equal(ms.export(), om.export())


def test_accept_batch_vs_oracle(C):
    rng = np.random.default_rng(113)
    cs, cc = C.SignalSet(), C.SignalSet()
    oc, ov = O.OSet(), O.OSet()
    for _ in range(3):
        sig = [C.Canonicalize(rng.integers(0, 3000, size=int(rng.integers(0, 100))).astype(np.uint32))
               for _ in range(300)]
        cov = [C.Canonicalize(rng.integers(0, 1 << 30, size=int(rng.integers(0, 50))).astype(np.uint32))
               for _ in range(300)]
        sv, so = C.to_csr(sig)
        cv, co = C.to_csr(cov)
        acc = C.accept_batch(cs, cc, sv, so, cv, co)
        eacc = O.accept_batch(oc, ov, sv, so, cv, co)
        assert np.array_equal(acc, eacc)
        assert np.array_equal(cs.export(), oc.export())
        assert np.array_equal(cc.export(), ov.export())


def test_accept_batch_groups_and_empty(C):
    """sg_accept_batch runs the partitioned path: > 2^16 inputs (two record
    groups), empty inputs, an all-empty batch, no coverage."""
    rng = np.random.default_rng(115)
    cs, oc = C.SignalSet(), O.OSet()
    lens = rng.integers(0, 6, size=70_000)
    lens[rng.integers(0, lens.size, size=5000)] = 0
    so = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    sv = rng.integers(0, 1 << 18, size=int(so[-1])).astype(np.uint32)
    sv[-1] = 0xFFFFFFFF
    sums = []
    for v, o in ((sv, so), (np.zeros(0, np.uint32), np.zeros(9, np.uint64)), (sv, so)):
        acc = C.accept_batch(cs, None, v, o)
        eacc = O.accept_batch(oc, None, v, o)
        assert np.array_equal(acc, eacc)
        assert np.array_equal(cs.export(), oc.export())
        sums.append(int(eacc.sum()))
    assert 0 < sums[0] < 70_000 and sums[1:] == [0, 0]


def test_merge_poll_vs_oracle(C):
    rng = np.random.default_rng(114)
    mm, om = C.SignalSet(), O.OSet()
    for _ in range(4):
        polls = [np.unique(rng.integers(0, 20000, size=int(rng.integers(0, 2000)))).astype(np.uint32)
                 for _ in range(20)]
        polls = [rng.permutation(p) for p in polls]  # map iteration order
        polls.append(np.array([5, 5, 6, 5], np.uint32))  # duplicates: first occurrence only
        # a poll owning more than the per-wave set (k_own_big) and one past a
        # piece of it, both with repeats; the 0xFFFFFFFF signal
        big = rng.integers(0, 1 << 24, size=30000).astype(np.uint32)
        polls.append(np.concatenate([big[:3000], big[:1500], big[2000:12000], [0xFFFFFFFF], big[500:9000]]))
        polls.append(np.concatenate([big[12000:], [0xFFFFFFFF, 0xFFFFFFFF], big[12000:20000]]))
        polls.append(np.array([0xFFFFFFFF, 9, 0xFFFFFFFF], np.uint32))
        av, ao = C.to_csr(polls)
        nv, no = C.merge_poll(mm, av, ao)
        ev, eo = O.merge_poll(om, av, ao)
        assert np.array_equal(no, eo) and np.array_equal(nv, ev)
    assert np.array_equal(mm.export(), om.export())


# ---- executor edge signal (executor.h:389-401, :497-526) --------------------------
def test_exec_signal_vs_reference_golden(C, exec_golden):
    g = exec_golden
    sig, off = C.exec_signal(g["pcs"], g["call_off"], g["prog_off"])
    assert np.array_equal(off, g["sig_off"])
    assert np.array_equal(sig, g["sig"])


def test_exec_signal_random_vs_oracle(C):
    rng = np.random.default_rng(115)
    for nprog, calls, pcs in [(1, 1, 1), (3, 5, 10), (40, 16, 1024), (4, 2, 30000)]:
        lens = rng.integers(0, 2 * pcs, size=nprog * calls).astype(np.uint64)
        call_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        trace = (0x81000000 + 16 * (np.minimum(rng.zipf(1.1, size=int(call_off[-1])), 1 << 18) - 1)).astype(np.uint32)
        prog_off = (np.arange(nprog + 1) * calls).astype(np.uint64)
        a = C.exec_signal(trace, call_off, prog_off)
        b = O.exec_signal(trace, call_off, prog_off)
        assert np.array_equal(a[1], b[1]) and np.array_equal(a[0], b[0])


def _exec_hash(a):  # executor.h:497-505
    a = (a ^ 61) ^ (a >> 16)
    a = (a + (a << 3)) & 0xFFFFFFFF
    a = a ^ (a >> 4)
    a = (a * 0x27D4EB2D) & 0xFFFFFFFF
    return a ^ (a >> 15)


def _trace_for_signals(sigs, call_off):
    """PCs whose edge signals (pc ^ hash(prev pc), prev = 0 at call start) are `sigs`."""
    pcs = np.zeros(len(sigs), np.uint32)
    for c in range(len(call_off) - 1):
        prev = 0
        for i in range(int(call_off[c]), int(call_off[c + 1])):
            pc = int(sigs[i]) ^ prev
            pcs[i] = pc
            prev = _exec_hash(pc)
    return pcs


def test_exec_signal_region_boundaries_vs_oracle(C):
    """Signals crowded onto the slots where the slot-region kernel's lanes meet
    (home % 128 in 124..127 and 0..3, table wrap-around 8189..8191 -> 0..2), a
    few distinct high parts so probe windows fill and home slots get
    overwritten, the zero signal, repeats, empty calls, high parts up to
    0xFFFFE000 (the table keeps 22-bit slot codes): every window's decisions
    in program order, as executor.h:507-526 takes them."""
    rng = np.random.default_rng(117)
    homes = np.array([(r * 128 + d) % 8192 for r in (0, 1, 2, 31, 63) for d in range(-4, 4)], np.uint64)
    for nprog, calls, pcs, nhigh, top in [(2, 3, 700, 3, False), (6, 4, 1500, 6, False), (3, 2, 5000, 40, False),
                                          (4, 3, 1500, 5, True)]:
        lens = rng.integers(1, 2 * pcs, size=nprog * calls).astype(np.uint64)
        lens[rng.random(lens.size) < 0.2] = 0  # empty calls between full ones
        call_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        n = int(call_off[-1])
        hi = rng.integers(0, nhigh, size=n).astype(np.uint64) * 8192 + 8192 * 977
        if top:  # the largest high parts (s >> 13 near 2^19: the 22-bit slot codes' top values)
            hi = ((1 << 19) - 1 - rng.integers(0, nhigh, size=n).astype(np.uint64)) * 8192
        sigs = (hi + rng.choice(homes, size=n)) & 0xFFFFFFFF
        sigs[rng.random(n) < 0.02] = 0
        far = rng.random(n) < 0.3  # anywhere in the table
        sigs[far] = rng.integers(0, 1 << 32, size=int(far.sum()), dtype=np.uint64)
        trace = _trace_for_signals(sigs.astype(np.uint32), call_off)
        prog_off = (np.arange(nprog + 1) * calls).astype(np.uint64)
        a = C.exec_signal(trace, call_off, prog_off)
        b = O.exec_signal(trace, call_off, prog_off)
        assert np.array_equal(a[1], b[1]) and np.array_equal(a[0], b[0])


# ---- cover report (syz-manager/cover.go:257-307) ------------------------------------
def _symtab(rng, nsym, base=0xffffffff81000000):
    starts = base + 16 * np.sort(rng.choice(nsym * 8, size=nsym, replace=False)).astype(np.uint64)
    sizes = 16 * rng.integers(1, 8, size=nsym).astype(np.uint64)
    nxt = np.append(starts[1:], starts[-1] + sizes[-1])
    ends = np.minimum(starts + sizes, nxt)
    sites = np.unique(np.concatenate([s + 5 + 16 * np.arange(int((e - s) // 16) + 1, dtype=np.uint64)
                                      for s, e in zip(starts, ends)]))
    return starts, ends, sites


def test_cover_uncovered_vs_oracle(C):
    rng = np.random.default_rng(116)
    for nsym, nq in [(1, 1), (10, 50), (500, 4000), (5000, 100000)]:
        starts, ends, sites = _symtab(rng, nsym)
        q = rng.choice(sites, size=nq) + 5 - 0xffffffff00000000
        q = np.concatenate([q, rng.integers(0, 1 << 32, size=nq // 10, dtype=np.uint64)]).astype(np.uint32)
        got = C.cover_uncovered(q, 0xffffffff, starts, ends, sites)
        exp = O.cover_uncovered(q, 0xffffffff, starts, ends, sites)
        assert np.array_equal(got, exp), nsym


def test_triage_dev_unaligned_input(C):
    """sg_triage_batch_dev on caller buffers that are not 16-B aligned (the
    pass-1 histogram then takes its scalar-load kernel): flags and set
    updates equal the oracle's."""
    import torch
    from syzkaller_amd._lib import call

    rng = np.random.default_rng(121)
    lens = rng.integers(0, 3000, size=700)
    n = int(lens.sum())
    vals = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    vals[rng.integers(0, n, size=n // 3)] = vals[rng.integers(0, n, size=n // 3)]  # cross-record repeats
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    m0 = np.unique(vals[rng.integers(0, n, size=n // 4)])
    for shift in (1, 2, 3):
        ms, ns = C.SignalSet(), C.SignalSet()
        C.SignalAdd(ms, m0)
        om, on = O.OSet(m0), O.OSet()
        buf = torch.zeros(n + 4, dtype=torch.int32, device="cuda")
        buf[shift:shift + n] = torch.from_numpy(vals.view(np.int32)).cuda()
        dv = buf[shift:shift + n]
        assert dv.data_ptr() % 16 != 0
        doff = torch.from_numpy(off.view(np.int64)).cuda()
        flags = torch.zeros(lens.size, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # the library queues on its own stream
        call("sg_triage_batch_dev", ms.ctx.h, ms.h, ns.h, dv.data_ptr(), doff.data_ptr(), n, lens.size,
             flags.data_ptr(), None, None)
        ms.ctx.sync()
        ef, _, _ = O.triage_batch(om, on, vals, off)
        assert np.array_equal(flags.cpu().numpy().astype(bool), np.asarray(ef).astype(bool))
        assert np.array_equal(ms.export(), om.export())
        assert np.array_equal(ns.export(), on.export())


def test_triage_record_slices(C):
    """Batches above the per-launch record limit run as consecutive record
    slices (sg_bucket.hip bucket_triage); the limit is lowered here so that
    slices start mid-batch, at empty records and at group boundaries.  The
    cuts come from the device (k_slice_cuts): up to 64 slices read with their
    count, more in a second read (3, 300), and past 4096 the host's own walk
    (1, 5000)."""
    rng = np.random.default_rng(131)
    for limit, nrec in ((1000, 4321), (100000, 240000), (7, 50), (3, 300), (1, 5000)):
        ctx = C.Context(0)
        ctx.set_option("max_launch_records", limit)
        assert ctx.counter("max_launch_records") == limit
        P = TwoPaths(C, ctx)
        om, on = O.OSet(), O.OSet()
        lens = rng.integers(0, 40, size=nrec)
        lens[rng.integers(0, nrec, size=nrec // 5)] = 0
        vals = rng.integers(0, 1 << 22, size=int(lens.sum()), dtype=np.uint64).astype(np.uint32)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        m0 = np.unique(vals[rng.integers(0, vals.size, size=vals.size // 3)])
        P.add(m0)
        om.add(m0)
        _check_triage(P, (om, on), vals, off)
        m, n = P.exports()
        assert np.array_equal(m, om.export()) and np.array_equal(n, on.export())
        del P
        ctx.close()


def test_owner_key_generation_reset(C):
    """The first-owner table (sg_ctx.hip owner_keys) hands out decreasing keys
    and starts a fresh generation (a full reset of the table) when the key
    space runs out.  The key space is lowered here so that rank-keyed
    Minimize crosses several resets, between triage batches and Poll merges
    (which take their owners from the bucket stage, not the table); every
    result still equals the oracle's."""
    ctx = C.Context(0)
    ctx.set_option("owner_key_space", 1500)
    assert ctx.counter("owner_key_space") == 1500
    rng = np.random.default_rng(151)
    ms, ns, mm = C.SignalSet(ctx), C.SignalSet(ctx), C.SignalSet(ctx)
    om, on, omm = O.OSet(), O.OSet(), O.OSet()
    for it in range(9):
        nrec = int(rng.integers(1000, 2500))
        lens = rng.integers(0, 12, size=nrec)
        vals = rng.integers(0, 1 << 16, size=int(lens.sum())).astype(np.uint32)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        flags, dv, do = C.triage_batch(ms, ns, vals, off)  # the ordered outputs
        ef, ev, eo = O.triage_batch(om, on, vals, off)
        assert np.array_equal(flags, ef) and np.array_equal(dv, ev) and np.array_equal(do, eo), it
        polls = [rng.permutation(np.unique(rng.integers(0, 1 << 17, size=int(rng.integers(0, 900)))).astype(np.uint32))
                 for _ in range(4)]
        av, ao = C.to_csr(polls)
        nv, no = C.merge_poll(mm, av, ao, ctx=ctx)
        ev2, eo2 = O.merge_poll(omm, av, ao)
        assert np.array_equal(nv, ev2) and np.array_equal(no, eo2), it
        covs = [C.Canonicalize(rng.integers(0, 3000, size=int(rng.integers(0, 40))).astype(np.uint32), ctx=ctx)
                for _ in range(700)]
        cv, co = C.to_csr(covs)
        assert np.array_equal(C.minimize_csr(cv, co, ctx=ctx), O.minimize(cv, co)), it  # rank keys
    assert ctx.counter("owner_resets") >= 3
    assert np.array_equal(ms.export(), om.export()) and np.array_equal(ns.export(), on.export())
    assert np.array_equal(mm.export(), omm.export())
    del ms, ns, mm
    ctx.close()


def test_cover_uncovered_radix_edges(C):
    """The report's radix indexes (sg_report.hip): symbol tables with gaps
    spanning many index buckets (filled by the search pass), clusters far
    apart, tables ending at the top of the u64 range, queries below the first
    and above the last symbol, and base 0 with PCs that wrap below zero."""
    rng = np.random.default_rng(141)
    cases = []
    # two clusters 2^40 apart: most buckets empty, one huge gap
    s1, e1, p1 = _symtab(rng, 300, base=0x1000000)
    far = np.uint64(1 << 40)
    cases.append((np.concatenate([s1, s1 + far]), np.concatenate([e1, e1 + far]), np.concatenate([p1, p1 + far]), 0))
    # a table ending at 2^64 - 1
    s2, e2, p2 = _symtab(rng, 200)
    top = np.uint64(0xffffffffffffffff) - max(e2[-1], p2[-1])
    cases.append((s2 + top, e2 + top, p2 + top, 0xffffffff))
    for starts, ends, sites, base in cases:
        hi32 = np.uint64(base) << np.uint64(32)
        q = (rng.choice(sites, size=20000) + np.uint64(5) - hi32).astype(np.uint32)
        q = np.concatenate([q, rng.integers(0, 1 << 32, size=3000, dtype=np.uint64).astype(np.uint32),
                            np.array([0, 1, 4, 5, 0xffffffff], np.uint32)])
        got = C.cover_uncovered(q, base, starts, ends, sites)
        exp = O.cover_uncovered(q, base, starts, ends, sites)
        assert np.array_equal(got, exp)
    # base 0: PCs below 5 wrap to the top of the range (Go uint64 arithmetic)
    s3, e3, p3 = _symtab(rng, 100)
    q = np.array([0, 3, 4, 5, 6, 100], np.uint32)
    got = C.cover_uncovered(q, 0, s3, e3, p3)
    exp = O.cover_uncovered(q, 0, s3, e3, p3)
    assert np.array_equal(got, exp)


def test_cover_uncovered_chunk_edges(C, ctx_option):
    """The chunked query path (sg_report.hip k_q_*): a chunk whose PC range
    spans more symbols than it holds in LDS (many site-less symbols: global
    symbol search), queries below the first and above the last call site,
    site counts at and around the 4096-site chunk size; the same queries in
    PC order (no regrouping), and through the direct per-query passes of the
    > 16M-site regime (option report_direct 1)."""
    rng = np.random.default_rng(143)
    hi32 = np.uint64(0xffffffff) << np.uint64(32)
    base = np.uint64(0xffffffff81000000)
    # 6000 adjacent 16-byte symbols, a call site in every 5th: chunk 0 spans all of them
    starts = base + 16 * np.arange(6000, dtype=np.uint64)
    ends = starts + np.uint64(16)
    sites = starts[::5] + np.uint64(5)
    cases = [(starts, ends, sites)]
    for nsites in (4095, 4096, 4097, 8192 + 3):
        s, e, p = _symtab(rng, 3 * nsites)
        cases.append((s, e, p[:nsites]))
    for starts, ends, sites in cases:
        q = (rng.choice(sites, size=30000) + np.uint64(5) - hi32).astype(np.uint32)
        lo = int(starts[0] + np.uint64(5) - hi32)
        q = np.concatenate([q, rng.integers(0, 1 << 32, size=2000, dtype=np.uint64).astype(np.uint32),
                            np.arange(lo - 40, lo + 40, dtype=np.uint32),
                            (np.uint32(int(ends[-1] + np.uint64(5) - hi32)) + np.arange(20, dtype=np.uint32))])
        exp = O.cover_uncovered(q, 0xffffffff, starts, ends, sites)
        got = C.cover_uncovered(q, 0xffffffff, starts, ends, sites)
        assert np.array_equal(got, exp), sites.size
        # in PC order (a canonical cover, as html.go passes): no regrouping
        qs = np.sort(q)
        assert np.array_equal(C.cover_uncovered(qs, 0xffffffff, starts, ends, sites),
                              O.cover_uncovered(qs, 0xffffffff, starts, ends, sites)), sites.size
        ctx_option(C.default_context(), "report_direct", 1)
        got = C.cover_uncovered(q, 0xffffffff, starts, ends, sites)
        C.default_context().set_option("report_direct", 0)
        assert np.array_equal(got, exp), sites.size


def test_cover_uncovered_symbol_past_last_site(C):
    """Queries above the last call site but inside a symbol (the symbol holding
    the last site reaches past it, and later symbols hold no site), with a site
    count that is not a multiple of the 4096-site chunk: such a query lands in
    the past-the-end chunk, whose symbol range starts at the last site's symbol
    (syz-manager/cover.go:278-299 marks that symbol's sites and later ones find
    none)."""
    rng = np.random.default_rng(797)
    hi32 = np.uint64(0xffffffff) << np.uint64(32)
    for nsites in (1, 4095, 4097, 4100, 8195):
        starts, ends, allsites = _symtab(rng, nsites + 64)
        # keep the sites of the leading symbols only, cut inside a symbol (the
        # first cut at or below nsites that is not a multiple of 4096), so that
        # symbol reaches past the last kept site
        while True:
            sites = allsites[:nsites]
            last = sites[-1]
            k = int(np.searchsorted(ends, last, side="right"))
            if starts[k] <= last < ends[k] - np.uint64(1) and nsites % 4096:
                break
            nsites -= 1
        gap = np.arange(int(last) + 1, int(ends[k]), dtype=np.uint64)
        later = np.concatenate([starts[k + 1:], ends[k + 1:] - np.uint64(1)])
        pcs = np.concatenate([gap, later, rng.choice(sites, size=3000)])
        q = (pcs + np.uint64(5) - hi32).astype(np.uint32)
        exp = O.cover_uncovered(q, 0xffffffff, starts, ends, sites)
        got = C.cover_uncovered(q, 0xffffffff, starts, ends, sites)
        assert np.array_equal(got, exp), nsites
        qs = np.sort(q)
        assert np.array_equal(C.cover_uncovered(qs, 0xffffffff, starts, ends, sites),
                              O.cover_uncovered(qs, 0xffffffff, starts, ends, sites)), nsites


def test_cover_uncovered_partial_functions(C):
    """A non-degenerate report (C5's shape, scaled down): 10% of the functions
    are touched, each on about half of its call sites, so the result holds
    every untouched site of every touched function (syz-manager/cover.go:288-299
    marks the function's whole range, then the covered PCs leave it)."""
    rng = np.random.default_rng(142)
    starts, ends, sites = _symtab(rng, 20000)
    fn = np.searchsorted(starts, sites, side="right") - 1
    touched = rng.random(starts.size) < 0.10
    pool = sites[touched[fn] & (rng.random(sites.size) < 0.5)]
    q = (rng.choice(pool, size=2_000_000) + np.uint64(5) - (np.uint64(0xffffffff) << np.uint64(32))).astype(np.uint32)
    got = C.cover_uncovered(q, 0xffffffff, starts, ends, sites)
    exp = O.cover_uncovered(q, 0xffffffff, starts, ends, sites)
    assert np.array_equal(got, exp)
    assert exp.size > 0.2 * pool.size  # about half of the touched functions' sites stay uncovered
