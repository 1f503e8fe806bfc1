"""Randomised batches through the ordered outputs (sg_triage.hip
owned_outputs): sg_triage_batch with the diff CSR, sg_merge_poll and
sg_accept_batch against the oracle's sequential loops (fuzzer.go:645-693,
manager.go:907-912, 949-956), over
seeds that put record counts across the 2^16-record group boundaries, records
past the sweep's chunk and set caps, empty records, repeats, the sentinel and
maxSignal overlap from none to most."""
import numpy as np
import pytest

from oracle import pyoracle as O

SENT = 0xFFFFFFFF


@pytest.fixture(scope="module")
def C(ctx):
    from syzkaller_amd import cover

    return cover


def _batch(rng):
    nrec = int(rng.choice([1, 37, 4096, 65535, 65536, 65537, 131073, 200000]))
    lens = rng.integers(0, 24, size=nrec)
    for _ in range(int(rng.integers(0, 6))):  # a few long records
        lens[rng.integers(0, nrec)] = int(rng.choice([2047, 2049, 4097, 20000, 70000]))
    lens[rng.integers(0, nrec, size=nrec // 7 + 1)] = 0
    n = int(lens.sum())
    hi = int(rng.choice([1 << 12, 1 << 20, 1 << 32]))
    vals = rng.integers(0, hi, size=n, dtype=np.uint64).astype(np.uint32)
    if rng.random() < 0.3 and n:
        vals[rng.integers(0, n, size=max(1, n // 1000))] = SENT
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    m0 = np.unique(vals[rng.integers(0, n, size=int(n * rng.random()))]) if n else np.zeros(0, np.uint32)
    return vals, off, m0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(24))
def test_ordered_outputs_random_batches(C, seed):
    rng = np.random.default_rng(1000 + seed)
    vals, off, m0 = _batch(rng)
    ms, ns = C.SignalSet(), C.SignalSet()
    C.SignalAdd(ms, m0)
    om, on = O.OSet(m0), O.OSet()
    f, dv, do = C.triage_batch(ms, ns, vals, off)
    ef, ev, eo = O.triage_batch(om, on, vals, off)
    assert np.array_equal(f, ef)
    assert np.array_equal(do, eo) and np.array_equal(dv, ev)
    for a, b in ((ms, om), (ns, on)):
        assert np.array_equal(np.sort(a.export()), np.sort(b.export()))
    mp = C.SignalSet()
    C.SignalAdd(mp, m0)
    pv, po = C.merge_poll(mp, vals, off)
    qv, qo = O.merge_poll(O.OSet(m0), vals, off)
    assert np.array_equal(po, qo) and np.array_equal(pv, qv)
    # NewInput over the same batch as RPCs (manager.go:907-912), with cover
    cl = rng.integers(0, 8, size=off.size - 1)
    co = np.concatenate([[0], np.cumsum(cl)]).astype(np.uint64)
    cv = rng.integers(0, 1 << 30, size=int(co[-1]), dtype=np.uint64).astype(np.uint32)
    cs, cc = C.SignalSet(), C.SignalSet()
    C.SignalAdd(cs, m0)
    os_, oc = O.OSet(m0), O.OSet()
    acc = C.accept_batch(cs, cc, vals, off, cv, co)
    assert np.array_equal(acc, O.accept_batch(os_, oc, vals, off, cv, co))
    for a, b in ((cs, os_), (cc, oc)):
        assert np.array_equal(np.sort(a.export()), np.sort(b.export()))
    for s in (ms, ns, mp, cs, cc):
        s.close()
