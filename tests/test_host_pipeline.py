"""The host entry points' pipelined ingest (sg_host.hip): a batch in host
memory goes through pinned double-buffered staging in record slices, each
slice's copies overlapping the previous slice's triage.  Cutting the batch
between records is exact (the sequential loop of syz-fuzzer/fuzzer.go:665 sees
the same maxSignal at every record), so the flags and both set updates must
equal the device entry point's on the same batch, whatever the slice size --
including slices of one record, and records longer than a slice."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

UNIVERSE_SEED = 0x5A17C0DE


POP_SEED = 0x9091A7E5


def _batch(ctx, nprog, calls, pcs, seed, npop=None):
    """Zipf programs (trace seed `seed`), or with npop: programs drawn from a
    population of npop, re-executed with flaky coverage (mixed flags against
    the population's signal)."""
    from syzkaller_amd._lib import call

    n = nprog * calls * pcs
    trace = torch.empty(n, dtype=torch.int32, device="cuda")
    if npop:
        call("sg_gen_population_traces_dev", ctx.h, UNIVERSE_SEED, POP_SEED, npop, seed, 2e-4, 1.1, 1 << 20, 0, nprog,
             calls, pcs, trace.data_ptr())
    else:
        call("sg_gen_zipf_traces_dev", ctx.h, UNIVERSE_SEED, seed, 1.1, 1 << 20, 0, nprog, calls, pcs,
             trace.data_ptr())
    call_off = torch.arange(0, n + 1, pcs, dtype=torch.int64, device="cuda")
    prog_off = torch.arange(0, nprog * calls + 1, calls, dtype=torch.int64, device="cuda")
    sig = torch.empty(n, dtype=torch.int32, device="cuda")
    off = torch.empty(nprog * calls + 1, dtype=torch.int64, device="cuda")
    call("sg_exec_signal_dev", ctx.h, trace.data_ptr(), call_off.data_ptr(), prog_off.data_ptr(), nprog, nprog * calls,
         n, sig.data_ptr(), off.data_ptr())
    torch.cuda.synchronize()
    nv = int(off[-1].item())
    return trace, call_off, sig[:nv].clone(), off


def _dev_reference(ctx, m0, d_vals, d_off, trace):
    from syzkaller_amd._lib import call
    from syzkaller_amd.cover import SignalSet

    ms, ns = SignalSet(ctx), SignalSet(ctx)
    dm0 = torch.from_numpy(m0.view(np.int32)).cuda()  # (held until the kernel has read it)
    call("sg_set_add_dev", ms.h, dm0.data_ptr(), m0.size)
    nrec = d_off.numel() - 1
    flags = torch.zeros(nrec, dtype=torch.uint8, device="cuda")
    if trace:
        call("sg_triage_traces_dev", ctx.h, ms.h, ns.h, d_vals.data_ptr(), d_off.data_ptr(), d_vals.numel(), nrec,
             flags.data_ptr())
    else:
        call("sg_triage_batch_dev", ctx.h, ms.h, ns.h, d_vals.data_ptr(), d_off.data_ptr(), d_vals.numel(), nrec,
             flags.data_ptr(), None, None)
    torch.cuda.synchronize()
    out = flags.cpu().numpy(), ms.export(), ns.export()
    ms.close()
    ns.close()
    return out


@pytest.mark.parametrize("trace", [False, True])
def test_host_pipeline_slices_equal_device_path(ctx, ctx_option, trace):
    from syzkaller_amd import cover as C

    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    npop = 256
    tr, call_off, sig, off = _batch(ctx, 512, 16, 1024, 4_401, npop=npop)
    _, _, warm, _ = _batch(ctx, npop, 16, 1024, POP_SEED)  # the population's own signal
    m0 = np.unique(warm.cpu().numpy().view(np.uint32))
    d_vals, d_off = (tr, call_off) if trace else (sig, off)
    exp = _dev_reference(ctx, m0, d_vals, d_off, trace)
    assert 0.05 < exp[0].mean() < 0.999
    h_vals = d_vals.cpu().numpy().view(np.uint32)
    h_off = d_off.cpu().numpy().view(np.uint64)
    # default slices (one slice here), many slices, slices of about one record,
    # and slices smaller than a record (each record then is a slice of its own);
    # the M0 filter on its auto regime, and forced on / off for the first two
    for slice_entries, mode in ((None, -1), (1 << 19, -1), (1000, -1), (300, -1), (None, 1), (1 << 19, 1),
                                (1 << 19, 0)):
        ctx_option(ctx, "host_slice", slice_entries or 0)
        ctx_option(ctx, "m0_filter", mode)
        u0 = ctx.counter("m0_filter_used")
        ms, ns = C.SignalSet(ctx), C.SignalSet(ctx)
        C.SignalAdd(ms, m0)
        if trace:
            got = C.triage_traces(ms, ns, h_vals, h_off, ctx=ctx)
        else:
            got, _, _ = C.triage_batch(ms, ns, h_vals, h_off, want_diff=False, ctx=ctx)
        assert np.array_equal(got, exp[0]), (slice_entries, mode)
        assert np.array_equal(ms.export(), exp[1]), (slice_entries, mode)
        assert np.array_equal(ns.export(), exp[2]), (slice_entries, mode)
        if (slice_entries, mode) == (1 << 19, 1):  # low-novelty slices: the filter's own tail ran
            assert ctx.counter("m0_filter_used") > u0
        if mode == 0:
            assert ctx.counter("m0_filter_used") == u0
        ms.close()
        ns.close()


def test_host_pipeline_copy_threads_and_empty_records(ctx, ctx_option):
    """Empty records at slice edges, one copy thread or many, and a batch of
    only empty records."""
    from syzkaller_amd import cover as C

    rng = np.random.default_rng(4403)
    lens = rng.integers(0, 400, size=5000)
    lens[rng.integers(0, lens.size, size=800)] = 0
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    vals = (rng.zipf(1.2, size=int(off[-1])) * 2654435761 % (1 << 32)).astype(np.uint32)
    d_vals = torch.from_numpy(vals.view(np.int32)).cuda()
    d_off = torch.from_numpy(off.view(np.int64)).cuda()
    m0 = np.unique(vals[: vals.size // 3])
    exp = _dev_reference(ctx, m0, d_vals, d_off, False)
    for thr, sl in ((1, 777), (16, 5000), (3, 1 << 26)):
        ctx_option(ctx, "host_copy_threads", thr)
        ctx_option(ctx, "host_slice", sl)
        ms, ns = C.SignalSet(ctx), C.SignalSet(ctx)
        C.SignalAdd(ms, m0)
        got, _, _ = C.triage_batch(ms, ns, vals, off, want_diff=False, ctx=ctx)
        assert np.array_equal(got, exp[0]), (thr, sl)
        assert np.array_equal(ms.export(), exp[1])
        assert np.array_equal(ns.export(), exp[2])
        ms.close()
        ns.close()
    ms = C.SignalSet(ctx)
    got, _, _ = C.triage_batch(ms, None, np.zeros(0, np.uint32), np.zeros(7, np.uint64), want_diff=False, ctx=ctx)
    assert not got.any() and got.size == 6 and len(ms.export()) == 0
    ms.close()
