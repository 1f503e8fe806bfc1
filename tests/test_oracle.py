"""Pins the CPU oracle (oracle/sigoracle.c) before it is trusted as the checker:
against the reference's own known-answer tables (pkg/cover/cover_test.go),
the reference's properties, the reference executor compiled from its sources
(tests/golden/exec_signal_golden.npz), and tiny line-by-line restatements.
CPU only."""
import numpy as np
import pytest

from oracle import pyoracle as O
from tests import refmodel as R

OPS = {"TestDifference": O.DIFF, "TestSymmetricDifference": O.SYMDIFF, "TestUnion": O.UNION,
       "TestIntersection": O.INTER}


def _cases(t):
    """runTest (cover_test.go:31-38): mirrored cases for symmetric ops + empty case."""
    cases = [(c["v0"], c["v1"], c["r"]) for c in t["cases"]]
    if t["symmetric"]:
        cases += [(b, a, r) for a, b, r in cases]
    cases.append(([], [], []))
    return cases


@pytest.mark.parametrize("name", sorted(OPS))
def test_kat_foreach(kats, name):
    for v0, v1, r in _cases(kats[name]):
        assert list(O.foreach(OPS[name], v0, v1)) == r, (name, v0, v1)


def test_kat_canonicalize(kats):
    for v0, _, r in _cases(kats["TestCanonicalize"]):
        a, n = O.canonicalize(v0)
        assert list(a[:n]) == r


def test_kat_minimize(kats):
    # cover_test.go:104-157 through the restated Go sort.Sort order
    for case in kats["TestMinimize"]["cases"]:
        lens = [len(c) for c in case["inp"]]
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        vals = np.concatenate([np.array(c, dtype=np.uint32) for c in case["inp"]])
        assert list(O.minimize(vals, off)) == case["out"]


def test_foreach_vs_loop_and_counts():
    rng = np.random.default_rng(1)
    for it in range(3000):
        n0, n1 = rng.integers(0, 12, size=2)
        hi = [5, 50, 0xFFFFFFFF][it % 3]
        a = sorted(int(x) for x in rng.integers(0, hi, size=n0, endpoint=True))
        b = sorted(int(x) for x in rng.integers(0, hi, size=n1, endpoint=True))
        if it % 7 == 0:  # force sentinels in
            a = sorted(a + [R.SENT] * int(rng.integers(1, 3)))
        for op in range(4):
            got = list(O.foreach(op, a, b))
            assert got == R.foreach_loop(op, a, b) == R.foreach_counts(op, a, b), (op, a, b)


def test_canonicalize_sentinel_rule():
    # cover.go:31: `last` starts at sent -> 0xFFFFFFFF survives unless it is the smallest value
    a, n = O.canonicalize([R.SENT, 3, 3, 1])
    assert list(a[:n]) == [1, 3, R.SENT]
    a, n = O.canonicalize([R.SENT, R.SENT])
    assert n == 0
    rng = np.random.default_rng(2)
    for _ in range(2000):
        v = [int(x) for x in rng.integers(0, 8, size=rng.integers(0, 20))]
        v = [R.SENT if x == 7 else x for x in v]
        a, n = O.canonicalize(v)
        assert list(a[:n]) == R.canonicalize(v)
        # in place like Go: the tail beyond n keeps the sorted values
        assert list(a[n:]) == sorted(v)[n:] and set(a) == set(v)


def test_has_difference_property():
    # cover_test.go:210-221: HasDifference(a, b) == (len(Difference(a, b)) != 0)
    rng = np.random.default_rng(3)
    for _ in range(5000):
        a, na = O.canonicalize(rng.integers(0, 100, size=rng.integers(0, 20)))
        b, nb = O.canonicalize(rng.integers(0, 100, size=rng.integers(0, 20)))
        assert O.has_difference(a[:na], b[:nb]) == (O.foreach(O.DIFF, a[:na], b[:nb]).size != 0)


def test_minimize_random_property():
    # cover_test.go:178-208: union of the selected covers == union of all
    rng = np.random.default_rng(4)
    for _ in range(1000):
        n = int(rng.integers(0, 20))
        covs = []
        for _ in range(n):
            a, k = O.canonicalize(rng.integers(0, 100, size=rng.integers(0, 10)))
            covs.append(list(a[:k]))
        lens = [len(c) for c in covs]
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) if n else np.zeros(1, np.uint64)
        vals = np.array([x for c in covs for x in c], dtype=np.uint32)
        sel = O.minimize(vals, off)
        total = set().union(*map(set, covs)) if covs else set()
        got = set().union(*[set(covs[i]) for i in sel]) if sel.size else set()
        assert got == total
        order = O.minimize_order(off)
        assert list(sel) == R.minimize(covs, list(order))


def test_go_sort_small_is_stable():
    # for n <= 6 Go's sort.Sort is insertion sort, i.e. stable (SURVEY.md §0 finding 4)
    rng = np.random.default_rng(5)
    for _ in range(500):
        n = int(rng.integers(0, 7))
        lens = rng.integers(0, 4, size=n)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        order = O.minimize_order(off)
        assert list(order) == sorted(range(n), key=lambda i: (-lens[i], i))


def test_go_sort_is_permutation():
    rng = np.random.default_rng(6)
    for n in [13, 41, 100, 1000, 5000]:
        lens = rng.integers(0, 5, size=n)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        order = O.minimize_order(off)
        assert sorted(order) == list(range(n))
        assert all(lens[order[i]] >= lens[order[i + 1]] for i in range(n - 1))


def test_triage_vs_python():
    rng = np.random.default_rng(7)
    for it in range(200):
        nrec = int(rng.integers(0, 30))
        recs = [[int(x) for x in rng.integers(0, 60, size=rng.integers(0, 12))] for _ in range(nrec)]
        m0 = set(int(x) for x in rng.integers(0, 60, size=rng.integers(0, 40)))
        vals = np.array([x for r in recs for x in r], dtype=np.uint32)
        off = np.concatenate([[0], np.cumsum([len(r) for r in recs])]).astype(np.uint64)
        ms, ns = O.OSet(sorted(m0)), O.OSet()
        flags, dv, do = O.triage_batch(ms, ns, vals, off)
        pm, pn = set(m0), set()
        pf, pd = R.triage(pm, pn, recs)
        assert list(flags) == pf
        assert [list(dv[int(do[r]):int(do[r + 1])]) for r in range(nrec)] == pd
        assert set(ms.export().tolist()) == pm and set(ns.export().tolist()) == pn


def test_exec_hash_matches_reference(exec_golden):
    for a, h in zip(exec_golden["hash_in"], exec_golden["hash_out"]):
        assert O.exec_hash(int(a)) == int(h)


def test_exec_signal_matches_reference(exec_golden):
    g = exec_golden
    sig, off = O.exec_signal(g["pcs"], g["call_off"], g["prog_off"])
    assert np.array_equal(off, g["sig_off"])
    assert np.array_equal(sig, g["sig"])


def test_exec_signal_vs_compiled_reference():
    if O.ref_executor() is None:
        pytest.skip("reference executor not built here (no reference checkout)")
    rng = np.random.default_rng(8)
    pcs = (0x81000000 + 16 * (np.minimum(rng.zipf(1.2, size=30000), 1 << 14) - 1)).astype(np.uint32)
    call_off = np.array([0, 100, 100, 9000, 9001, 30000], dtype=np.uint64)
    prog_off = np.array([0, 2, 5], dtype=np.uint64)
    a = O.exec_signal(pcs, call_off, prog_off)
    b = O.ref_exec_signal(pcs, call_off, prog_off)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_exec_signal_crafted_vs_compiled_reference():
    """Signals crowded onto a few home slots (full probe windows, home-slot
    overwrites) and the zero signal, whose overwrite empties slot 0: the
    oracle against the reference's own dedup loop on the same traces."""
    if O.ref_executor() is None:
        pytest.skip("reference executor not built here (no reference checkout)")
    from tests.test_gpu_parity import _trace_for_signals
    rng = np.random.default_rng(117)
    homes = np.array([(r * 128 + d) % 8192 for r in (0, 1, 63) for d in range(-4, 4)], np.uint64)
    call_off = np.array([0, 700, 1900, 1900, 5000], np.uint64)
    n = int(call_off[-1])
    sigs = (rng.integers(0, 6, size=n).astype(np.uint64) * 8192 + 8192 * 977 + rng.choice(homes, size=n)) & 0xFFFFFFFF
    sigs[rng.random(n) < 0.03] = 0
    trace = _trace_for_signals(sigs.astype(np.uint32), call_off)
    prog_off = np.array([0, 2, 4], np.uint64)
    a = O.exec_signal(trace, call_off, prog_off)
    b = O.ref_exec_signal(trace, call_off, prog_off)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert (a[0] == 0).any()  # a zero signal did overwrite


def test_merge_poll_and_accept_vs_python():
    rng = np.random.default_rng(9)
    for _ in range(100):
        polls = [[int(x) for x in rng.integers(0, 50, size=rng.integers(0, 10))] for _ in range(rng.integers(0, 8))]
        av = np.array([x for p in polls for x in p], dtype=np.uint32)
        ao = np.concatenate([[0], np.cumsum([len(p) for p in polls])]).astype(np.uint64)
        m0 = [int(x) for x in rng.integers(0, 50, size=10)]
        nv, no = O.merge_poll(O.OSet(m0), av, ao)
        mx, exp = set(m0), []
        for p in polls:
            cur = []
            for s in p:
                if s in mx:
                    continue
                mx.add(s)
                cur.append(s)
            exp.append(cur)
        assert [list(nv[int(no[k]):int(no[k + 1])]) for k in range(len(polls))] == exp
        acc = O.accept_batch(O.OSet(m0), None, av, ao)
        cs, exp_acc = set(m0), []
        for p in polls:
            ok = any(s not in cs for s in p)
            exp_acc.append(int(ok))
            if ok:
                cs.update(p)
        assert list(acc) == exp_acc


def test_cover_uncovered_vs_python():
    rng = np.random.default_rng(10)
    for _ in range(100):
        nsym = int(rng.integers(1, 30))
        starts = np.sort(rng.choice(np.arange(0xffffffff81000000, 0xffffffff81000000 + 4096 * 16, 16, dtype=np.uint64),
                                    nsym, replace=False))
        sizes = rng.integers(1, 6, size=nsym).astype(np.uint64) * 16
        ends = np.minimum(starts + sizes, np.append(starts[1:], starts[-1] + sizes[-1]))
        allpcs = np.unique(np.concatenate([s + 5 + 16 * np.arange(int((e - s) // 16) + 1, dtype=np.uint64)
                                           for s, e in zip(starts, ends)]))
        cov = (rng.choice(allpcs, size=int(rng.integers(0, 40))) + 5 - 0xffffffff00000000).astype(np.uint32)
        got = O.cover_uncovered(cov, 0xffffffff, starts, ends, allpcs)
        # direct restatement of syz-manager/cover.go:277-301
        handled, unc = set(), set()
        for c in cov:
            pc = (0xffffffff << 32) + int(c) - 5
            idx = int(np.searchsorted(ends, pc, side="right"))
            if idx == nsym or pc < starts[idx] or pc > ends[idx]:
                continue
            if int(starts[idx]) not in handled:
                handled.add(int(starts[idx]))
                lo = np.searchsorted(allpcs, starts[idx], side="left")
                hi = np.searchsorted(allpcs, ends[idx], side="right")
                unc.update(int(x) for x in allpcs[lo:hi])
            unc.discard(pc)
        assert list(got) == sorted(unc)
