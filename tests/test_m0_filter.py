"""The M0 filter (sg_bucket.hip k_m0_index / k_m0_filter and the tail): the
flags path's regime for low-novelty batches, between the two partition
passes.  Forced on (context option m0_filter 1) every batch must give the
sequential loop's flags, maxSignal and newSignal (syz-fuzzer/fuzzer.go:645-693,
oracle/sigoracle.c) -- through the filter's own tail when the survivors fit,
through pass 2 and the bucket stage when they overflow -- and auto must pick
the regime from the last slices.  The edge cases are the filter's own: no
survivors, every entry a survivor, a slice holding more maxSignal signals than
its LDS index (kFCap: the rest are re-checked against the bitmap), signals 0
and 0xFFFFFFFF, repeats of a new signal across records (first owner), record
slices, and raw traces (the set-exact trace path runs the same filter)."""
import numpy as np
import pytest

from oracle import pyoracle as O

pytestmark = pytest.mark.gpu

SENT = 0xFFFFFFFF


@pytest.fixture(scope="module")
def C(ctx):
    from syzkaller_amd import cover

    return cover


def _batch(rng, nrec, m0, novelty, maxlen=60, hi=1 << 32):
    lens = rng.integers(0, maxlen, size=nrec)
    lens[rng.integers(0, nrec, size=nrec // 6)] = 0
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    n = int(off[-1])
    vals = m0[rng.integers(0, m0.size, size=n)] if m0.size else np.zeros(n, np.uint32)
    fresh = rng.random(n) < novelty
    vals[fresh] = rng.integers(0, hi, size=int(fresh.sum()), dtype=np.uint64).astype(np.uint32)
    return vals.astype(np.uint32), off


def _check(C, ctx, m0, vals, off, mode, expect):
    """One batch through sg_triage_batch with option m0_filter = mode against
    the oracle; expect: "used" (the filter's tail produced the results),
    "fallback" (its survivors overflowed), "skip" (not tried), None (any)."""
    ctx.set_option("m0_filter", mode)
    u0, f0 = ctx.counter("m0_filter_used"), ctx.counter("m0_filter_fallback")
    ms, ns = C.SignalSet(ctx), C.SignalSet(ctx)
    if m0.size:
        C.SignalAdd(ms, m0)
    got, _, _ = C.triage_batch(ms, ns, vals, off, want_diff=False, ctx=ctx)
    du, df = ctx.counter("m0_filter_used") - u0, ctx.counter("m0_filter_fallback") - f0
    om, on = O.OSet(m0), O.OSet()
    exp = O.triage_flags_only(om, on, vals, off)
    assert np.array_equal(got, exp)
    assert np.array_equal(ms.export(), om.export())
    assert np.array_equal(ns.export(), on.export())
    ms.close()
    ns.close()
    if expect == "used":
        assert du >= 1 and df == 0, (du, df)
    elif expect == "fallback":
        assert df >= 1 and du == 0, (du, df)
    elif expect == "skip":
        assert du == 0 and df == 0, (du, df)
    return exp


@pytest.mark.parametrize("halves", [0, 1, 2])
def test_m0_filter_low_novelty_and_edges(C, ctx, ctx_option, halves):
    """Also with the index in 2 and 4 parts per slice (option m0_filter_halves):
    each entry tested by exactly one part."""
    ctx_option(ctx, "m0_filter", 1)
    ctx_option(ctx, "m0_filter_halves", halves)
    rng = np.random.default_rng(6001)
    m0 = np.unique(rng.integers(0, 1 << 32, size=300_000, dtype=np.uint64).astype(np.uint32))
    m0 = np.unique(np.concatenate([m0, np.array([0, SENT], np.uint32)]))
    for nov in (1e-3, 0.0, 0.02):  # low novelty, no survivor at all, more of them
        vals, off = _batch(rng, 20_000, m0, nov)
        vals[:5] = [0, SENT, 0, SENT, m0[7]]
        exp = _check(C, ctx, m0, vals, off, 1, "used")
        assert (exp.sum() == 0) == (nov == 0.0)
    # a new signal repeated over many records: its first owner only
    vals, off = _batch(rng, 5_000, m0, 0.0)
    rep = np.uint32(0x12345679)
    assert rep not in set(m0.tolist())
    vals[rng.integers(0, vals.size, size=200)] = rep
    _check(C, ctx, m0, vals, off, 1, "used")
    # empty maxSignal: every entry survives (fewer than the cap)
    vals, off = _batch(rng, 4_000, np.zeros(0, np.uint32), 1.0)
    _check(C, ctx, np.zeros(0, np.uint32), vals, off, 1, "used")
    # ... all of them in one pass-1 slice (b2 = 0): past the regions of its
    # 8 filter workgroups (2048 each), so the partition goes on (with the index
    # in parts, a slice's values all sit in the first part: past its workgroups')
    vals, off = _batch(rng, 4_000, np.zeros(0, np.uint32), 1.0, hi=1 << 16)
    assert vals.size > 8 * 2048 + 1000
    _check(C, ctx, np.zeros(0, np.uint32), vals, off, 1, "fallback")
    # empty records only / a batch without entries
    _check(C, ctx, m0, np.zeros(0, np.uint32), np.zeros(9, np.uint64), 1, None)


def test_m0_filter_index_cap_and_overflow(C, ctx, ctx_option):
    """A pass-1 slice holding 100K maxSignal signals (past the index's 61,440):
    the bucket prefixes past the cap leave signals unproven, which the tail
    re-checks against the bitmap; and a fresh batch whose survivors overflow
    the 2^20 cap goes on through pass 2 and the bucket stage."""
    ctx_option(ctx, "m0_filter", 1)
    rng = np.random.default_rng(6002)
    # signals of pass-1 slice 5: b2 (bits 16..23) = 5
    low = rng.choice(1 << 24, size=100_000, replace=False).astype(np.uint64)
    dense = np.unique(((low >> np.uint64(16)) << np.uint64(24)) | (np.uint64(5) << np.uint64(16))
                      | (low & np.uint64(0xFFFF))).astype(np.uint32)
    other = np.unique(rng.integers(0, 1 << 32, size=50_000, dtype=np.uint64).astype(np.uint32))
    m0 = np.unique(np.concatenate([dense, other]))
    vals, off = _batch(rng, 30_000, other, 1e-3)
    hot = rng.random(vals.size) < 0.02  # ~15K entries in the dense slice: ~1/3 of them unproven by its index
    vals[hot] = dense[rng.integers(0, dense.size, size=int(hot.sum()))]
    _check(C, ctx, m0, vals, off, 1, "used")
    # a few buckets past 15 values (their rest in the slice's spill list):
    # entries on the spilled positions are proven there, not survivors
    base = np.uint64(9) << np.uint64(16)  # slice 9
    spilled = []
    for j in range(12):
        vs = np.sort(rng.choice(1 << 11, size=30, replace=False)).astype(np.uint64)
        pos = (np.uint64(j * 37) << np.uint64(11)) | vs  # 24-bit position in the slice: b1 b3 b0
        sig = ((pos >> np.uint64(16)) << np.uint64(8)) | ((pos >> np.uint64(8) & np.uint64(255)) << np.uint64(24)) \
            | (pos & np.uint64(255)) | base
        spilled.append(sig[15:].astype(np.uint32))
    spilled = np.concatenate(spilled)
    m0s = np.unique(np.concatenate([other, spilled]))
    assert np.isin(spilled, m0s).all()
    vals, off = _batch(rng, 20_000, other, 0.0)
    hot = rng.random(vals.size) < 0.05
    vals[hot] = spilled[rng.integers(0, spilled.size, size=int(hot.sum()))]
    assert hot.sum() > 10_000
    _check(C, ctx, m0s, vals, off, 1, "used")
    assert ctx.counter("m0_filter_survivors") == 0
    # fresh: ~1.6M survivors > the cap
    vals, off = _batch(rng, 50_000, m0, 1.0, maxlen=80)
    assert vals.size > (1 << 20) + 200_000
    _check(C, ctx, m0, vals, off, 1, "fallback")


def test_m0_filter_auto_regime_and_record_slices(C, ctx_option):
    """auto: tried after a slice it filtered; after a partitioned slice only
    when that slice queued under a quarter of its records (a fresh batch queues
    nearly all: the next one is partitioned, and its own low queued fraction
    brings the filter back); after a fallback not for 1, 2, 4 .. slices;
    record slices (a lowered per-launch record limit) are filtered one by one,
    each against the maxSignal the slices before it left."""
    ctx = C.Context(0)
    try:
        rng = np.random.default_rng(6003)
        m0 = np.unique(rng.integers(0, 1 << 32, size=200_000, dtype=np.uint64).astype(np.uint32))
        vals, off = _batch(rng, 12_000, m0, 2e-3)
        ctx.set_option("max_launch_records", 1000)  # 12 slices
        _check(C, ctx, m0, vals, off, 1, "used")
        assert ctx.counter("m0_filter_used") >= 12
        ctx.set_option("max_launch_records", 0)
        fresh, foff = _batch(rng, 50_000, m0, 1.0, maxlen=80)
        _check(C, ctx, m0, fresh, foff, -1, "fallback")  # (tried: the last slice was filtered)
        _check(C, ctx, m0, vals, off, -1, "skip")  # the fresh batch queued ~83 % of its records
        _check(C, ctx, m0, vals, off, -1, "used")  # ... this one a few percent
        assert ctx.counter("m0_filter_queued_milli") < 250
        _check(C, ctx, m0, vals, off, 0, "skip")  # never
        _check(C, ctx, m0, fresh, foff, -1, "fallback")
        # after a fallback auto backs off: 1 slice, then (another fallback) 2,
        # then a filtered slice resets it -- a maxSignal past the index's
        # capacity falls back on every slice it tries
        _check(C, ctx, m0, vals, off, -1, "skip")
        _check(C, ctx, m0, fresh, foff, -1, "fallback")
        _check(C, ctx, m0, vals, off, -1, "skip")
        _check(C, ctx, m0, vals, off, -1, "skip")
        _check(C, ctx, m0, vals, off, -1, "used")
        _check(C, ctx, m0, fresh, foff, -1, "fallback")
        _check(C, ctx, m0, vals, off, -1, "skip")
        _check(C, ctx, m0, vals, off, -1, "used")
    finally:
        ctx.close()


def test_m0_filter_index_parts_auto(C):
    """A slice whose maxSignal signals overflow one index part (its hot
    entries then overflow the survivor regions): auto falls back once, takes
    the index in two parts, and filters the same batch the next time."""
    ctx = C.Context(0)
    try:
        rng = np.random.default_rng(6005)
        low = rng.choice(1 << 24, size=100_000, replace=False).astype(np.uint64)  # slice 5, λ ≈ 12 per bucket
        dense = np.unique(((low >> np.uint64(16)) << np.uint64(24)) | (np.uint64(5) << np.uint64(16))
                          | (low & np.uint64(0xFFFF))).astype(np.uint32)
        other = np.unique(rng.integers(0, 1 << 32, size=50_000, dtype=np.uint64).astype(np.uint32))
        m0 = np.unique(np.concatenate([dense, other]))
        vals, off = _batch(rng, 40_000, other, 1e-4)
        hot = rng.random(vals.size) < 0.12  # ~140K entries in the dense slice, a third of them past one part
        vals[hot] = dense[rng.integers(0, dense.size, size=int(hot.sum()))]
        assert ctx.counter("m0_filter_halves_log") == 0
        _check(C, ctx, m0, vals, off, 1, "fallback")
        assert ctx.counter("m0_filter_halves_log") == 1
        _check(C, ctx, m0, vals, off, 1, "used")
        ctx.set_option("m0_filter_halves", 0)  # forced back to one part: the same fallback
        _check(C, ctx, m0, vals, off, 1, "fallback")
    finally:
        ctx.close()


def test_m0_filter_traces(C, ctx, ctx_option):
    """The set-exact trace path (sg_triage_traces: the edge signal computed in
    pass 1's loads) through the filter, against the oracle's executor signal
    and loop."""
    ctx_option(ctx, "m0_filter", 1)
    rng = np.random.default_rng(6004)
    ncalls = 6000
    lens = rng.integers(0, 200, size=ncalls)
    call_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    pcs = (0x81000000 + 16 * (np.minimum(rng.zipf(1.1, size=int(call_off[-1])), 1 << 14) - 1)).astype(np.uint32)
    prog_off = np.arange(ncalls + 1, dtype=np.uint64)
    sig, soff = O.exec_signal(pcs, call_off, prog_off)
    m0 = np.unique(sig[: int(soff[ncalls * 9 // 10])])  # most of the batch's edges already known
    om, on = O.OSet(m0), O.OSet()
    exp = O.triage_flags_only(om, on, sig, soff)
    u0 = ctx.counter("m0_filter_used")
    ms, ns = C.SignalSet(ctx), C.SignalSet(ctx)
    C.SignalAdd(ms, m0)
    got = C.triage_traces(ms, ns, pcs, call_off, ctx=ctx)
    assert ctx.counter("m0_filter_used") > u0
    assert 0 < exp.sum() < ncalls
    assert np.array_equal(got, exp)
    assert np.array_equal(ms.export(), om.export()) and np.array_equal(ns.export(), on.export())
    ms.close()
    ns.close()
