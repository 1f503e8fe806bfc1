"""The manager's cover.Union folds (SURVEY.md §8(f) row 2:
syz-manager/html.go:84/:94/:184/:306, manager.go:916-917) as one batched
k-way tree of Unions (sg_union_fold) against the oracle's left fold of
cover.go:63-70, bit-exact: multiset max-count semantics, 0xFFFFFFFF dropped."""
import numpy as np
import pytest

from oracle import pyoracle as O
from tests import refmodel as R


def _corpus(rng, n, universe, maxlen, multiset=False):
    covs = []
    for k in range(n):
        m = int(rng.integers(0, maxlen)) if k % 11 else 0
        v = np.sort(rng.choice(universe, size=m, replace=multiset)).astype(np.uint32)
        if k % 13 == 1 and m:
            v[-1] = 0xFFFFFFFF  # cover.go:97 drops it in every Union
        covs.append(v)
    return covs


def test_oracle_fold_vs_counts():
    rng = np.random.default_rng(51)
    uni = (0x81000000 + 16 * np.arange(5000)).astype(np.uint32)
    for multiset in (False, True):
        covs = _corpus(rng, 40, uni, 300, multiset)
        vals, off = O._csr(covs)
        fv, fo = O.union_fold(vals, off)
        acc = []
        for c in covs:
            acc = R.foreach_counts(2, acc, [int(x) for x in c])
        assert list(fv) == acc


@pytest.mark.gpu
@pytest.mark.parametrize("multiset", [False, True])
def test_union_fold_vs_oracle(ctx, multiset):
    from syzkaller_amd import cover as C

    rng = np.random.default_rng(52 + multiset)
    uni = (0x81000000 + 16 * np.arange(1 << 16)).astype(np.uint32)
    # html.go:84 (grouped by call), :306 (everything)
    covs = _corpus(rng, 3000, uni, 2000, multiset)
    vals, off = C.to_csr(covs)
    calls = rng.integers(0, 37, size=len(covs)).astype(np.uint32)
    calls[:5] = 36  # a group with several lists up front
    gv, go = C.union_fold(vals, off, calls, 40, ctx=ctx)  # groups 37..39 stay empty
    ev, eo = O.union_fold(vals, off, calls, 40)
    assert np.array_equal(go, eo) and np.array_equal(gv, ev)
    gv, go = C.union_fold(vals, off, ctx=ctx)
    ev, eo = O.union_fold(vals, off)
    assert np.array_equal(go, eo) and np.array_equal(gv, ev)
    # html.go:94: the per-call covers folded again
    gv2, go2 = C.union_fold(*C.union_fold(vals, off, calls, 40, ctx=ctx), ctx=ctx)
    assert np.array_equal(gv2, ev)
    # manager.go:916-917: Union of two
    a, b = covs[3], covs[4]
    gv, go = C.union_fold(*C.to_csr([a, b]), ctx=ctx)
    assert np.array_equal(gv, O.foreach(O.UNION, a, b))
    # a single list: Union(nil, c) -- the sentinel goes
    c = np.array([5, 7, 7, 0xFFFFFFFF], np.uint32)
    gv, _ = C.union_fold(*C.to_csr([c]), ctx=ctx)
    assert list(gv) == [5, 7, 7]
    # nothing at all
    gv, go = C.union_fold(np.zeros(0, np.uint32), np.zeros(3, np.uint64), ctx=ctx)
    assert gv.size == 0 and not go.any()


@pytest.mark.gpu
def test_union_fold_key_width_edges(ctx):
    """The sort path packs (group, value, copy index) into 64 bits: 2^20
    groups (20 bits) with a value repeated 4096 times (copy index 4095: 12
    bits) fill them exactly; 8192 repeats need 13 bits, so that fold takes the
    merge-tree path.  Both equal the oracle's left fold."""
    from syzkaller_amd import cover as C

    rng = np.random.default_rng(55)
    ng = 1 << 20
    for reps in (4096, 8192):
        covs = [np.sort(rng.integers(0, 1 << 32, size=int(rng.integers(0, 50)), dtype=np.uint64).astype(np.uint32))
                for _ in range(300)]
        covs[7] = np.concatenate([covs[7][:3], np.full(reps, 0xC0FFEE, np.uint32)])
        covs[7].sort()
        covs[9] = np.array([0xC0FFEE] * 5 + [0xFFFFFFFF] * 3, np.uint32)
        vals, off = C.to_csr(covs)
        grp = rng.integers(0, ng, size=len(covs)).astype(np.uint32)
        grp[9] = grp[7]
        grp[10] = ng - 1
        gv, go = C.union_fold(vals, off, grp, ng, ctx=ctx)
        ev, eo = O.union_fold(vals, off, grp, ng)
        assert np.array_equal(go, eo) and np.array_equal(gv, ev), reps


@pytest.mark.gpu
def test_union_fold_zipf_corpus(ctx):
    """A bench-like corpus (canonical Zipf covers, many groups) against the
    oracle: values sharing their top byte, so the sort skips digits."""
    from syzkaller_amd import cover as C

    rng = np.random.default_rng(56)
    n = 4000
    lens = np.clip(np.exp(rng.normal(np.log(300), 0.8, size=n)), 1, 4000).astype(np.int64)
    ranks = np.minimum(rng.zipf(1.05, size=int(lens.sum())), 1 << 21) - 1
    raw = (0x81000000 + 16 * ranks).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(lens)])
    covs = [np.unique(raw[off[k]:off[k + 1]]) for k in range(n)]
    vals, off = C.to_csr(covs)
    for grp, ng in ((rng.integers(0, 300, size=n).astype(np.uint32), 300), (None, 1)):
        gv, go = C.union_fold(vals, off, grp, ng, ctx=ctx)
        ev, eo = O.union_fold(vals, off, grp, ng)
        assert np.array_equal(go, eo) and np.array_equal(gv, ev)


@pytest.mark.gpu
def test_union_fold_byte_map_edges(ctx, ctx_option):
    """One group of canonical lists takes the byte map over [AND, OR] of the
    values: value 0, spans just under and over 2^28 (the latter sorts), the
    sentinel (dropped; its presence widens the span, so the fold sorts), lists
    sharing most values, a wide span over few values (too sparse for the map:
    sorts); each equal to the oracle and to the sort (option fold_map 0)."""
    from syzkaller_amd import cover as C

    rng = np.random.default_rng(57)
    for span in (1, 4096, 1 << 24, (1 << 28) - 5, (1 << 28) + 5, 1 << 32):
        lo = int(rng.integers(0, (1 << 32) - min(span, 1 << 32) + 1))
        covs = []
        for k in range(60):
            m = int(rng.integers(0, 400))
            v = lo + rng.integers(0, span, size=m, dtype=np.uint64)
            covs.append(np.unique(v.astype(np.uint32)))
        covs[0] = np.array([lo, min(lo + span - 1, 0xFFFFFFFF)], np.uint32)
        if span in ((1 << 28) - 5, (1 << 28) + 5):  # dense enough for the map (range <= 16 N)
            covs[2] = np.arange(lo, lo + span, 15, dtype=np.uint64).astype(np.uint32)
        if span == 1 << 32:
            covs[1] = np.array([0, 0xFFFFFFFF], np.uint32)
        vals, off = C.to_csr(covs)
        ev, eo = O.union_fold(vals, off)
        gv, go = C.union_fold(vals, off, ctx=ctx)
        assert np.array_equal(go, eo) and np.array_equal(gv, ev), span
        ctx_option(ctx, "fold_map", 0)
        sv, so = C.union_fold(vals, off, ctx=ctx)
        ctx.set_option("fold_map", -1)
        assert np.array_equal(so, eo) and np.array_equal(sv, ev), span


@pytest.mark.gpu
def test_union_fold_lds_groups(ctx):
    """Many groups of canonical lists: a workgroup sorts each group in LDS
    (sg_fold.hip k_fold_lds, groups of <= 32768 values in three forms), the
    bigger groups fold beside them by the key sort (k_fold_bigkeys /
    k_fold_bigmove).
    Groups at and around that size, several big ones (one holding the
    sentinel, one of a single repeated value spread over many lists), empty
    groups, one-value groups, constant groups (no digit pass), values over the
    whole 32-bit range (four passes), the sentinel at the ends of lists."""
    from syzkaller_amd import cover as C

    rng = np.random.default_rng(57)
    for top, extra in ((16384, []), (16385, []), (16385, [70000, 20000, 40000, 32768, 32769])):
        covs, calls = [], []
        sizes = [top, 16000, 1, 0, 5, 300, 8191, 8192, 2, 2] + extra
        for gi, sz in enumerate(sizes):
            left = sz
            while left > 0:  # a group's values over several lists, repeats across lists
                m = int(min(left, rng.integers(1, 3000)))
                if gi == 4:
                    v = np.full(1, 0x12345678, np.uint32)  # a constant group
                    m = 1
                elif gi in (5, 12):
                    v = np.unique(rng.integers(0, 1 << 32, size=m, dtype=np.uint64)).astype(np.uint32)
                elif gi == 11:
                    v = np.full(1, 0xABCD, np.uint32)  # a big group of one value
                else:
                    v = (0x81000000 + 16 * rng.choice(1 << 20, size=m, replace=False)).astype(np.uint32)
                if gi == 9:
                    v = np.array([7, 0xFFFFFFFF], np.uint32)
                if gi == 12 and left == sz:
                    v = np.unique(np.append(v, 0xFFFFFFFF).astype(np.uint32))
                covs.append(np.sort(v))
                calls.append(gi)
                left -= max(1, v.size)
        calls = np.array(calls, np.uint32)
        vals, off = C.to_csr(covs)
        ng = len(sizes) + 2  # two empty groups past the last
        gv, go = C.union_fold(vals, off, calls, ng, ctx=ctx)
        ev, eo = O.union_fold(vals, off, calls, ng)
        assert np.array_equal(go, eo) and np.array_equal(gv, ev), top
