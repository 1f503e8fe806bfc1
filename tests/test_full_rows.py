"""Full-size parity of the secondary rows (SURVEY.md §8 configs C1, C4, C5 and
row f2), each against the oracle over the whole workload -- not a sample:

  C1  pkg/cover Union / Difference (cover.go:42-102): all 1000 canonical
      traces x 4096 PCs against the 1M-PC corpus signal.
  C4  cover.Minimize + minimizeCorpus (cover.go:120-146, manager.go:769-784):
      the 500k-input corpus (lognormal lengths, median 1k, clipped to
      [1, 16k]; Zipf values) in the Go sort.Sort order.
  C5  uncoveredPcsInFuncs (syz-manager/cover.go:257-307): 100M queries against
      5M call sites in 50k functions, in random order and in PC order.
  f2  the manager's cover.Union folds (html.go:84/:94/:306): the 50k-input
      corpus folded per syscall (4000 groups) and over everything.

Inputs come from the same recipes as bench_rows.py (GPU-generated Zipf PCs
where numpy would dominate the run time).  Bit-exact."""
import numpy as np
import pytest
import torch

from oracle import pyoracle as O

pytestmark = pytest.mark.gpu

UNIVERSE_SEED = 0x5A17C0DE


@pytest.fixture(scope="module")
def C(ctx):
    from syzkaller_amd import cover

    return cover


def _gpu_zipf(ctx, n, seed, s=1.1, nranks=1 << 22):
    """n Zipf(s) PCs over nranks ranks (pc = 0x81000000 + 16 perm(rank)), by the
    bench's counter-based generator, to the host."""
    from syzkaller_amd._lib import call

    t = torch.empty(n, dtype=torch.int32, device="cuda")
    call("sg_gen_zipf_traces_dev", ctx.h, UNIVERSE_SEED, seed, s, nranks, 0, 1, 1, n, t.data_ptr())
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.timeout(180)
def test_c1_full_union_difference(C, ctx):
    rng = np.random.default_rng(8101)
    corpus = (0x81000000 + 16 * np.sort(rng.choice(1 << 22, size=1_000_000, replace=False))).astype(np.uint32)
    raw = _gpu_zipf(ctx, 1000 * 6000, 8102, s=1.05)
    traces = [np.unique(raw[k * 6000:(k + 1) * 6000])[:4096] for k in range(1000)]
    a = np.concatenate(traces)
    a_len = np.array([t.size for t in traces], np.uint64)
    a_beg = np.concatenate([[0], np.cumsum(a_len)[:-1]]).astype(np.uint64)
    b_beg = np.zeros(1000, np.uint64)
    b_len = np.full(1000, corpus.size, np.uint64)
    for op in (2, 0):  # Union, Difference
        out = C.merge_batch(op, a, a_beg, a_len, corpus, b_beg, b_len, ctx=ctx)
        for k in range(1000):
            assert np.array_equal(out[k], O.foreach(op, traces[k], corpus)), (op, k)


@pytest.mark.timeout(180)
def test_c4_full_minimize(C, ctx):
    rng = np.random.default_rng(8401)
    n = 500_000
    lens = np.clip(np.exp(rng.normal(np.log(1000), 1.0, size=n)), 1, 16384).astype(np.int64)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    vals = _gpu_zipf(ctx, int(off[-1]), 8402)
    order = C.minimize_order(off)
    assert np.array_equal(order, O.minimize_order(off))  # the Go sort.Sort permutation
    got = C.minimize_csr(vals, off, order, ctx=ctx)
    exp = O.minimize(vals, off, order)
    assert 0 < exp.size < n
    assert np.array_equal(got, exp)


def _c5_table(rng, nsym=50_000, nsites=5_000_000):
    base = 0xffffffff81000000
    sizes = 16 * (1 + rng.integers(0, 2 * nsites // nsym, size=nsym)).astype(np.uint64)
    starts = base + np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    ends = starts + sizes
    per = (sizes // 16).astype(np.int64)
    fn = np.repeat(np.arange(nsym), per)
    first = np.repeat(starts, per)
    k = np.arange(per.sum()) - np.repeat(np.cumsum(per) - per, per)
    sites = (first + 5 + 16 * k.astype(np.uint64))[:nsites]
    return starts, ends, sites, fn[:nsites]


@pytest.mark.timeout(300)
def test_c5_full_report_random_and_pc_order(C):
    """C5 at its configured size: 100M queries against the 5M-site table, in
    random order (the GPU regroups them by call-site chunk) and in PC order
    (a canonical cover, html.go:177-189: no regrouping).  The report depends
    on the queries as a multiset only (per symbol the first covering query,
    per site the last deleting one: syz-manager/cover.go:257-307 folds them
    with no order-dependent state), so the oracle runs once, on the sorted
    queries (the random-order oracle loop misses cache on every query: ~90 s
    at this size); the order independence itself is checked on a 2M prefix."""
    rng = np.random.default_rng(8501)
    starts, ends, sites, fn = _c5_table(rng)
    touched = rng.random(starts.size) < 0.10
    pool = sites[touched[fn] & (rng.random(sites.size) < 0.5)]
    nq = 100_000_000
    q = (rng.choice(pool, size=nq) + 5 - (np.uint64(0xffffffff) << np.uint64(32))).astype(np.uint32)
    # a few queries off every site and outside every symbol
    q[:: 997] = rng.integers(0, 1 << 32, size=q[:: 997].size, dtype=np.uint64).astype(np.uint32)
    p = q[:2_000_000]
    assert np.array_equal(O.cover_uncovered(p, 0xffffffff, starts, ends, sites),
                          O.cover_uncovered(np.sort(p), 0xffffffff, starts, ends, sites))
    qs = np.sort(q)  # PC order
    exp = O.cover_uncovered(qs, 0xffffffff, starts, ends, sites)
    assert exp.size > 0
    got = C.cover_uncovered(q, 0xffffffff, starts, ends, sites)
    assert np.array_equal(got, exp)
    assert np.array_equal(C.cover_uncovered(qs, 0xffffffff, starts, ends, sites), exp)


def _fold_vectorized(vals, off, group, ngroups):
    """The left fold of cover.Union over each group's inputs (cover.go:63-70
    via foreach: a value's multiplicity is the max over the inputs, the
    sentinel 0xFFFFFFFF dropped), computed without the O(inputs x |cov|)
    loop: max multiplicity of every (group, value) over the inputs.
    Cross-checked against the oracle's literal fold on a prefix below."""
    n = off.size - 1
    lens = np.diff(off.astype(np.int64))
    inp = np.repeat(np.arange(n, dtype=np.int64), lens)
    g = np.zeros(n, np.int64) if group is None else group.astype(np.int64)
    keep = vals != 0xFFFFFFFF
    key = (g[inp] << 48) | (inp << 32) | vals.astype(np.int64)  # n < 2^16, ngroups < 2^15
    key = key[keep]
    u, cnt = np.unique(key, return_counts=True)  # multiplicity per (group, input, value)
    gv = ((u >> 48) << 32) | (u & 0xFFFFFFFF)
    order = np.lexsort((cnt, gv))  # by (group, value), then count
    gv, cnt = gv[order], cnt[order]
    last = np.r_[gv[1:] != gv[:-1], True]  # the max count of each (group, value)
    gv, cnt = gv[last], cnt[last]
    out = np.repeat(gv & 0xFFFFFFFF, cnt).astype(np.uint32)
    og = np.repeat(gv >> 32, cnt)
    fo = np.searchsorted(og, np.arange(ngroups + 1)).astype(np.uint64)
    return out, fo


@pytest.mark.timeout(240)
def test_f2_full_union_folds(C, ctx):
    rng = np.random.default_rng(8201)
    n, ncalls = 50_000, 4000
    lens = np.clip(np.exp(rng.normal(np.log(1000), 0.8, size=n)), 1, 16384).astype(np.int64)
    roff = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    raw = _gpu_zipf(ctx, int(roff[-1]), 8202, s=1.05, nranks=1 << 21)
    # executor-deduped covers: per input sorted and unique, as html.go folds them
    inp = np.repeat(np.arange(n, dtype=np.int64), lens)
    u = np.unique((inp << 32) | raw.astype(np.int64))
    vals = (u & 0xFFFFFFFF).astype(np.uint32)
    off = np.searchsorted(u >> 32, np.arange(n + 1)).astype(np.uint64)
    calls = rng.integers(0, ncalls, size=n).astype(np.uint32)
    # the vectorized fold equals the oracle's literal left fold on a prefix
    m = 1500
    for grp, ng in ((calls[:m], ncalls), (None, 1)):
        ev, eo = O.union_fold(vals[: off[m]], off[: m + 1], grp, ng)
        vv, vo = _fold_vectorized(vals[: off[m]], off[: m + 1], grp, ng)
        assert np.array_equal(vv, ev) and np.array_equal(vo, eo)
    for grp, ng in ((calls, ncalls), (None, 1)):
        fv, fo = C.union_fold(vals, off, grp, ng, ctx=ctx)
        ev, eo = _fold_vectorized(vals, off, grp, ng)
        assert np.array_equal(fo, eo)
        assert np.array_equal(fv, ev)
