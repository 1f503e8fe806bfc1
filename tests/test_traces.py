"""Set-exact trace triage (sg_triage_traces[_dev]): raw per-call PC traces in,
edge signal computed in the partition's loads (sg_bucket.hip k_hist_trace /
k_p1_scatter<trace>), zero edges dropped.  The claim under test
(include/syzsig.h): the per-call flags and the maxSignal / newSignal updates
equal those of the executor-exact signal (executor/executor.h:389-401,
:497-526 -- the oracle's exec_signal, itself pinned to the compiled reference
executor by tests/golden/exec_signal_golden.npz) followed by the sequential
new-signal loop (syz-fuzzer/fuzzer.go:645-693, the oracle's triage).  Bit-exact."""
import numpy as np
import pytest

from oracle import pyoracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C(ctx):
    from syzkaller_amd import cover

    return cover


def _expected(m0, pcs, call_off, prog_off):
    sig, off = O.exec_signal(pcs, call_off, prog_off)
    om, on = O.OSet(m0), O.OSet()
    flags = O.triage_flags_only(om, on, sig, off)
    return flags, om.export(), on.export()


def _check(C, m0, pcs, call_off, prog_off=None):
    call_off = np.asarray(call_off, np.uint64)
    if prog_off is None:  # one program per call (the dedup table is per program)
        prog_off = np.arange(call_off.size, dtype=np.uint64)
    ef, em, en = _expected(m0, pcs, call_off, prog_off)
    ms, ns = C.SignalSet(), C.SignalSet()
    if len(m0):
        C.SignalAdd(ms, np.asarray(m0, np.uint32))
    got = C.triage_traces(ms, ns, pcs, call_off)
    assert np.array_equal(got, ef)
    assert np.array_equal(ms.export(), em)
    assert np.array_equal(ns.export(), en)
    ms.close()
    ns.close()
    return got


def _zipf_pcs(rng, n, nranks=1 << 16):
    return (0x81000000 + 16 * (np.minimum(rng.zipf(1.1, size=n), nranks) - 1)).astype(np.uint32)


def test_traces_small_and_zero_edges(C):
    """Tiny batches, empty calls, and every way an edge is 0: a call's first
    PC equal to 0, and a PC equal to hash(previous PC)."""
    rng = np.random.default_rng(701)
    h = np.vectorize(O.exec_hash, otypes=[np.uint64])
    for it in range(40):
        ncalls = int(rng.integers(1, 30))
        lens = rng.integers(0, 12, size=ncalls)
        lens[rng.integers(0, ncalls, size=ncalls // 4)] = 0
        n = int(lens.sum())
        pcs = rng.integers(0, 64, size=n).astype(np.uint32)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        starts = off[:-1][lens > 0].astype(np.int64)
        if it % 3 == 0 and starts.size:
            pcs[starts[0]] = 0  # sig = 0 ^ 0
        if it % 2 == 0 and n > 2:  # sig = hash(prev) ^ hash(prev) = 0 inside a call
            for j in rng.integers(1, n, size=3):
                if j not in set(starts.tolist()):
                    pcs[j] = np.uint32(h(pcs[j - 1]))
        m0 = np.unique(rng.integers(0, 64, size=int(rng.integers(0, 20)))).astype(np.uint32)
        _check(C, m0, pcs, off)


def test_traces_programs_and_evictions(C):
    """Programs of many calls whose traces repeat edges often enough that the
    executor's 8192-slot table evicts and re-emits them (multiplicity differs
    from the raw edges, flags and sets may not)."""
    rng = np.random.default_rng(702)
    for nprog, calls, pcs in [(1, 1, 1), (3, 5, 10), (40, 16, 1024), (4, 2, 30000), (8, 40, 3000)]:
        lens = rng.integers(0, 2 * pcs, size=nprog * calls).astype(np.uint64)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        tr = _zipf_pcs(rng, int(off[-1]), 1 << 18)
        prog_off = (np.arange(nprog + 1) * calls).astype(np.uint64)
        sig, _ = O.exec_signal(tr, off, prog_off)
        m0 = np.unique(sig[rng.integers(0, max(1, sig.size), size=sig.size // 5)]) if sig.size else sig
        _check(C, m0, tr, off, prog_off)


def test_traces_reference_golden(C, exec_golden):
    """The traces behind the compiled reference executor's golden vectors."""
    g = exec_golden
    _check(C, np.zeros(0, np.uint32), g["pcs"], g["call_off"], g["prog_off"])


def test_traces_tile_geometry(C):
    """Calls longer than a pass-1 tile, tiles cut by the record cap, and a call
    starting exactly at a tile cut (16384-entry steps)."""
    rng = np.random.default_rng(703)
    for lens in ([16384, 16384, 1, 16383, 70000], [1] * 3000 + [40000], [0, 0, 16384, 0, 5, 16379, 16385],
                 list(rng.integers(0, 4, size=30000))):
        lens = np.asarray(lens, np.int64)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        tr = rng.integers(0, 1 << 32, size=int(off[-1]), dtype=np.uint64).astype(np.uint32)
        tr[rng.integers(0, tr.size, size=tr.size // 3)] = tr[rng.integers(0, tr.size, size=tr.size // 3)]
        _check(C, np.zeros(0, np.uint32), tr, off)


def test_traces_equal_exec_then_triage_on_gpu(C):
    """A larger Zipf batch (4096 programs x 16 calls x 1024 PCs, generated on
    the GPU): sg_triage_traces_dev equals sg_exec_signal_dev followed by the
    flags-only sg_triage_batch_dev, in flags and in both sets."""
    import torch
    from syzkaller_amd._lib import call

    nprog, calls, pcs = 4096, 16, 1024
    ctx = C.default_context()
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        ncalls, npcs = nprog * calls, nprog * calls * pcs
        tr = torch.empty(npcs, dtype=torch.int32, device="cuda")
        call_off = torch.arange(0, npcs + 1, pcs, dtype=torch.int64, device="cuda")
        prog_off = torch.arange(0, ncalls + 1, calls, dtype=torch.int64, device="cuda")
        sig = torch.empty(npcs, dtype=torch.int32, device="cuda")
        soff = torch.empty(ncalls + 1, dtype=torch.int64, device="cuda")
        sets = [C.SignalSet(ctx) for _ in range(4)]
        # the starting maxSignal of both paths: a population of 256 programs'
        # signal; the batch: population members re-executed with flaky
        # coverage (mixed flags; a fresh Zipf batch flags every call)
        npop = 256
        call("sg_gen_zipf_traces_dev", ctx.h, 0x5A17C0DE, 77, 1.1, 1 << 20, 0, npop, calls, pcs, tr.data_ptr())
        warm_flags = torch.zeros(npop * calls, dtype=torch.uint8, device="cuda")
        call("sg_triage_traces_dev", ctx.h, sets[0].h, None, tr.data_ptr(), call_off.data_ptr(), npop * calls * pcs,
             npop * calls, warm_flags.data_ptr())
        call("sg_set_copy", sets[2].h, sets[0].h)
        call("sg_gen_population_traces_dev", ctx.h, 0x5A17C0DE, 77, npop, 78, 2e-4, 1.1, 1 << 20, 0, nprog, calls, pcs,
             tr.data_ptr())
        fa = torch.zeros(ncalls, dtype=torch.uint8, device="cuda")
        fb = torch.zeros(ncalls, dtype=torch.uint8, device="cuda")
        call("sg_triage_traces_dev", ctx.h, sets[0].h, sets[1].h, tr.data_ptr(), call_off.data_ptr(), npcs, ncalls,
             fa.data_ptr())
        call("sg_exec_signal_dev", ctx.h, tr.data_ptr(), call_off.data_ptr(), prog_off.data_ptr(), nprog, ncalls, npcs,
             sig.data_ptr(), soff.data_ptr())
        torch.cuda.synchronize()
        nv = int(soff[-1].item())
        call("sg_triage_batch_dev", ctx.h, sets[2].h, sets[3].h, sig.data_ptr(), soff.data_ptr(), nv, ncalls,
             fb.data_ptr(), None, None)
        torch.cuda.synchronize()
        a, b = fa.cpu().numpy(), fb.cpu().numpy()
        assert 0 < a.sum() < a.size
        assert np.array_equal(a, b)
        assert np.array_equal(sets[0].export(), sets[2].export())
        assert np.array_equal(sets[1].export(), sets[3].export())
        for s_ in sets:
            s_.close()
    finally:
        ctx.reset_stream()


def test_traces_record_slices(C):
    """Trace batches above the per-launch record limit (lowered here) run as
    record slices; each slice starts at a call start."""
    rng = np.random.default_rng(704)
    ctx = C.Context(0)
    ctx.set_option("max_launch_records", 500)
    try:
        lens = rng.integers(0, 60, size=3000)
        lens[rng.integers(0, lens.size, size=600)] = 0
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        tr = _zipf_pcs(rng, int(off[-1]))
        ef, em, en = _expected(np.zeros(0, np.uint32), tr, off, np.arange(off.size, dtype=np.uint64))
        ms, ns = C.SignalSet(ctx), C.SignalSet(ctx)
        got = C.triage_traces(ms, ns, tr, off, ctx=ctx)
        assert np.array_equal(got, ef)
        assert np.array_equal(ms.export(), em) and np.array_equal(ns.export(), en)
        ms.close()
        ns.close()
    finally:
        ctx.close()


def test_exec_signal_queued_lists(C, ctx):
    """sg_exec_signal_queued_dev after a set-exact trace triage: each queued
    call's list equals the executor-exact list (sg_exec_signal_dev, pinned to
    the compiled reference executor), every other call's list is empty
    (fuzzer.go:678-683 copies the signal of queued records only).  A steady
    population batch, so programs hold queued calls at any position, none,
    or several; then the oracle on a small ragged batch."""
    import torch

    from syzkaller_amd._lib import call

    nprog, calls, pcs, npop = 4096, 16, 1024, 512
    n, ncalls = nprog * calls * pcs, nprog * calls
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    tr = torch.empty(n, dtype=torch.int32, device="cuda")
    call("sg_gen_zipf_traces_dev", ctx.h, 0x5A17C0DE, 0x9091A7E5, 1.1, 1 << 20, 0, npop, calls, pcs, tr.data_ptr())
    co = torch.arange(0, n + 1, pcs, dtype=torch.int64, device="cuda")
    po = torch.arange(0, ncalls + 1, calls, dtype=torch.int64, device="cuda")
    sig = torch.empty(n, dtype=torch.int32, device="cuda")
    so = torch.empty(ncalls + 1, dtype=torch.int64, device="cuda")
    call("sg_exec_signal_dev", ctx.h, tr.data_ptr(), co.data_ptr(), po.data_ptr(), npop, npop * calls, npop * calls * pcs,
         sig.data_ptr(), so.data_ptr())
    torch.cuda.synchronize()
    m0 = np.unique(sig[: int(so[npop * calls].item())].cpu().numpy().view(np.uint32))
    call("sg_gen_population_traces_dev", ctx.h, 0x5A17C0DE, 0x9091A7E5, npop, 6_001, 2e-4, 1.1, 1 << 20, 0, nprog,
         calls, pcs, tr.data_ptr())
    ms, ns = C.SignalSet(ctx), C.SignalSet(ctx)
    C.SignalAdd(ms, m0)
    flags = torch.zeros(ncalls, dtype=torch.uint8, device="cuda")
    call("sg_triage_traces_dev", ctx.h, ms.h, ns.h, tr.data_ptr(), co.data_ptr(), n, ncalls, flags.data_ptr())
    call("sg_exec_signal_dev", ctx.h, tr.data_ptr(), co.data_ptr(), po.data_ptr(), nprog, ncalls, n, sig.data_ptr(),
         so.data_ptr())
    qsig = torch.empty(n, dtype=torch.int32, device="cuda")
    qso = torch.empty(ncalls + 1, dtype=torch.int64, device="cuda")
    call("sg_exec_signal_queued_dev", ctx.h, tr.data_ptr(), co.data_ptr(), po.data_ptr(), nprog, ncalls, n,
         flags.data_ptr(), qsig.data_ptr(), qso.data_ptr())
    torch.cuda.synchronize()
    f = flags.cpu().numpy().astype(bool)
    assert 0.01 < f.mean() < 0.9
    fp = f.reshape(nprog, calls)
    assert fp.any(1).mean() < 1.0 and (fp.sum(1) > 1).any()  # programs with none / several queued calls
    full_off, q_off = so.cpu().numpy(), qso.cpu().numpy()
    full_len, q_len = np.diff(full_off), np.diff(q_off)
    assert np.array_equal(q_len, np.where(f, full_len, 0))
    fv, qv = sig.cpu().numpy(), qsig.cpu().numpy()
    idx = np.flatnonzero(f)
    src = np.concatenate([np.arange(full_off[c], full_off[c + 1]) for c in idx])
    assert np.array_equal(qv[: q_off[-1]], fv[src])
    ms.close()
    ns.close()
    # the oracle, a small ragged batch with arbitrary flags
    rng = np.random.default_rng(707)
    lens = rng.integers(0, 300, size=48)
    call_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    prog_off = np.array([0, 5, 5, 17, 30, 48], np.uint64)
    p = _zipf_pcs(rng, int(call_off[-1]), nranks=1 << 10)
    es, eo = O.exec_signal(p, call_off, prog_off)
    fl = (rng.random(48) < 0.3).astype(np.uint8)
    # (device copies held in names: a temporary's memory could be reused
    # before the kernel reads it)
    dp, dco, dpo = (torch.from_numpy(a.view(t)).cuda() for a, t in ((p, np.int32), (call_off, np.int64),
                                                                     (prog_off, np.int64)))
    dfl = torch.from_numpy(fl).cuda()
    dq = torch.empty(max(int(call_off[-1]), 1), dtype=torch.int32, device="cuda")
    dqo = torch.empty(49, dtype=torch.int64, device="cuda")
    call("sg_exec_signal_queued_dev", ctx.h, dp.data_ptr(), dco.data_ptr(), dpo.data_ptr(), 5, 48, int(call_off[-1]),
         dfl.data_ptr(), dq.data_ptr(), dqo.data_ptr())
    torch.cuda.synchronize()
    got_off, got = dqo.cpu().numpy().view(np.uint64), dq.cpu().numpy().view(np.uint32)
    for c in range(48):
        want = es[eo[c]:eo[c + 1]] if fl[c] else np.zeros(0, np.uint32)
        assert np.array_equal(got[got_off[c]:got_off[c + 1]], want), c


def test_triage_traces_queued_host(C, ctx):
    """sg_triage_traces_queued: host traces in, the fuzzer's flags, both set
    updates and the queued calls' executor-exact lists out, against the
    oracle (executor.h:389-401 lists, then the loop of fuzzer.go:645-693 over
    them, which the set-exact triage of the traces equals); three batches in
    a row on the same sets, with empty calls and an empty program."""
    rng = np.random.default_rng(909)
    ms, ns = C.SignalSet(ctx), C.SignalSet(ctx)
    om, on = O.OSet(), O.OSet()
    m0 = _zipf_pcs(rng, 3000, nranks=1 << 12)
    C.SignalAdd(ms, m0)
    om.add(m0)
    for b in range(3):
        lens = rng.integers(0, 400, size=60)
        lens[rng.integers(0, 60, size=8)] = 0
        call_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        prog_off = np.array([0, 7, 7, 20, 33, 41, 60], np.uint64)
        p = _zipf_pcs(rng, int(call_off[-1]), nranks=1 << 12)
        es, eo = O.exec_signal(p, call_off, prog_off)
        ef = O.triage_flags_only(om, on, es, eo)
        flags, vals, off = C.triage_traces_queued(ms, ns, p, call_off, prog_off, ctx=ctx)
        assert np.array_equal(flags, ef), b
        assert 0 < ef.sum() < 60
        for c in range(60):
            want = es[eo[c]:eo[c + 1]] if ef[c] else np.zeros(0, np.uint32)
            assert np.array_equal(vals[off[c]:off[c + 1]], want), (b, c)
        assert np.array_equal(ms.export(), om.export()) and np.array_equal(ns.export(), on.export())
    ms.close()
    ns.close()
