"""Full-size C2 parity (BASELINE.json configs[1]: 64Ki programs x 16 calls x
1024 PCs): one whole batch through the product's device path
(sg_triage_batch_dev, the partitioned kernels the bench times) against the
oracle's sequential loop (oracle/sigoracle.c, restating
syz-fuzzer/fuzzer.go:645-693) on the same batch, bit-exact in the per-record
flags and in both sets afterwards -- and the same batch again through the
ordered-output path (the diff CSR of fuzzer.go:669, sg_triage.hip
owned_outputs) from the same starting sets, bit-exact in the flags, every
record's diff list and both sets.

The batch is the fuzzer's steady state (bench.py "steady"): programs drawn
from a fixed population with flaky coverage, against maxSignal = the
population's signal, so the flags are mixed (the fresh-Zipf C2 batch flags
every record: each one carries some never-seen edge)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import pyoracle as O

pytestmark = pytest.mark.gpu

UNIVERSE_SEED = 0x5A17C0DE
POP_SEED = 0x9091A7E5


def _signal(call, ctx, trace, nprog, calls, pcs):
    ncalls, npcs = nprog * calls, nprog * calls * pcs
    call_off = torch.arange(0, npcs + 1, pcs, dtype=torch.int64, device="cuda")
    prog_off = torch.arange(0, ncalls + 1, calls, dtype=torch.int64, device="cuda")
    sig = torch.empty(npcs, dtype=torch.int32, device="cuda")
    off = torch.empty(ncalls + 1, dtype=torch.int64, device="cuda")
    call("sg_exec_signal_dev", ctx.h, trace.data_ptr(), call_off.data_ptr(), prog_off.data_ptr(), nprog, ncalls, npcs,
         sig.data_ptr(), off.data_ptr())
    torch.cuda.synchronize()
    n = int(off[-1].item())
    return sig[:n], off


def _diff_path(call, ctx, m0, sig, off, ef, ev, eo, em, en):
    """The batch through sg_triage_batch_dev with the diff CSR, from maxSignal
    = m0 and an empty newSignal; everything against the oracle's loop."""
    from syzkaller_amd.cover import SignalSet

    nvals, nrec = sig.numel(), off.numel() - 1
    ms, ns = SignalSet(ctx), SignalSet(ctx)
    dm0 = torch.from_numpy(m0.view(np.int32)).cuda()
    call("sg_set_add_dev", ms.h, dm0.data_ptr(), m0.size)
    rec_new = torch.zeros(nrec, dtype=torch.uint8, device="cuda")
    dv = torch.empty(nvals, dtype=torch.int32, device="cuda")
    do = torch.empty(nrec + 1, dtype=torch.int64, device="cuda")
    call("sg_triage_batch_dev", ctx.h, ms.h, ns.h, sig.data_ptr(), off.data_ptr(), nvals, nrec, rec_new.data_ptr(),
         dv.data_ptr(), do.data_ptr())
    torch.cuda.synchronize()
    del dm0
    assert np.array_equal(rec_new.cpu().numpy(), ef)
    got_o = do.cpu().numpy().view(np.uint64)
    assert np.array_equal(got_o, eo)
    nd = int(got_o[-1])
    assert nd == ev.size
    assert np.array_equal(dv[:nd].cpu().numpy().view(np.uint32), ev)
    del dv, do, rec_new
    assert np.array_equal(ns.export(), en)
    assert np.array_equal(ms.export(), em)
    ns.close()
    ms.close()


@pytest.mark.timeout(600)
def test_c2_full_batch_steady_state_vs_oracle(ctx):
    from syzkaller_amd._lib import call
    from syzkaller_amd.cover import SignalSet

    nprog, calls, pcs, npop = 65536, 16, 1024, 2048
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    trace = torch.empty(nprog * calls * pcs, dtype=torch.int32, device="cuda")
    # maxSignal = every population member's signal
    call("sg_gen_zipf_traces_dev", ctx.h, UNIVERSE_SEED, POP_SEED, 1.1, 1 << 20, 0, npop, calls, pcs, trace.data_ptr())
    msig, moff = _signal(call, ctx, trace, npop, calls, pcs)
    m0 = np.unique(msig.cpu().numpy().view(np.uint32))
    # the batch: population programs re-executed with flaky coverage
    call("sg_gen_population_traces_dev", ctx.h, UNIVERSE_SEED, POP_SEED, npop, 5_001, 2e-4, 1.1, 1 << 20, 0, nprog,
         calls, pcs, trace.data_ptr())
    sig, off = _signal(call, ctx, trace, nprog, calls, pcs)
    del trace
    nvals, nrec = sig.numel(), off.numel() - 1
    assert nrec == nprog * calls and nvals > 800_000_000  # the C2 shape
    # the oracle's sequential loop over the same batch
    om, on = O.OSet(m0), O.OSet()
    exp, ev, eo = O.triage_batch(om, on, sig.cpu().numpy().view(np.uint32), off.cpu().numpy().view(np.uint64))
    frac = float(exp.mean())
    assert 0.05 < frac < 0.95, frac  # mixed flags: the attribution is really tested
    em, en = om.export(), on.export()
    del om, on
    # the flags path with the M0 filter forced (its tail makes the results:
    # ~139K survivors), in its auto regime (which takes it here), and without it
    dm0 = torch.from_numpy(m0.view(np.int32)).cuda()  # (held until the kernels have read it)
    rec_new = torch.zeros(nrec, dtype=torch.uint8, device="cuda")
    for mode in (1, -1, 0):
        ctx.set_option("m0_filter", mode)
        used = ctx.counter("m0_filter_used")
        ms, ns = SignalSet(ctx), SignalSet(ctx)
        call("sg_set_add_dev", ms.h, dm0.data_ptr(), m0.size)
        call("sg_triage_batch_dev", ctx.h, ms.h, ns.h, sig.data_ptr(), off.data_ptr(), nvals, nrec, rec_new.data_ptr(),
             None, None)
        torch.cuda.synchronize()
        assert (ctx.counter("m0_filter_used") > used) == (mode != 0), mode
        assert np.array_equal(rec_new.cpu().numpy(), exp), mode
        assert np.array_equal(ns.export(), en), mode
        assert np.array_equal(ms.export(), em), mode
        ns.close()
        ms.close()
    ctx.set_option("m0_filter", -1)
    del dm0
    _diff_path(call, ctx, m0, sig, off, exp, ev, eo, em, en)
    call("sg_ctx_reset_stream", ctx.h)


@pytest.mark.timeout(900)
def test_c2_full_fresh_batch_sets_vs_oracle(ctx):
    """The headline configuration itself (bench.py's recipe): a fresh Zipf
    batch of 64Ki programs x 16 calls x 1024 PCs against a >= 16M-entry
    maxSignal taken from a warm batch's first programs.  Every record is
    queued (each carries a never-seen edge), so the check that matters is the
    ~200M new signals: maxSignal and newSignal after the batch, exported and
    compared whole with the oracle's sequential loop, plus the flags; then
    the ~208M-element diff CSR of the ordered-output path."""
    from syzkaller_amd._lib import call
    from syzkaller_amd.cover import SignalSet

    nprog, calls, pcs = 65536, 16, 1024
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    trace = torch.empty(nprog * calls * pcs, dtype=torch.int32, device="cuda")
    # maxSignal: the warm batch's (seed 2_000_000) first 4608 programs
    nwarm = 4608
    call("sg_gen_zipf_traces_dev", ctx.h, UNIVERSE_SEED, 2_000_000, 1.1, 1 << 20, 0, nwarm, calls, pcs, trace.data_ptr())
    wsig, woff = _signal(call, ctx, trace, nwarm, calls, pcs)
    m0 = np.unique(wsig.cpu().numpy().view(np.uint32))
    del wsig, woff
    assert m0.size >= 16 << 20
    # the bench's first timed batch (seed 1000 + warmup 2)
    call("sg_gen_zipf_traces_dev", ctx.h, UNIVERSE_SEED, 1_002, 1.1, 1 << 20, 0, nprog, calls, pcs, trace.data_ptr())
    sig, off = _signal(call, ctx, trace, nprog, calls, pcs)
    del trace
    nvals, nrec = sig.numel(), off.numel() - 1
    ms, ns = SignalSet(ctx), SignalSet(ctx)
    dm0 = torch.from_numpy(m0.view(np.int32)).cuda()  # (held until the kernel has read it)
    call("sg_set_add_dev", ms.h, dm0.data_ptr(), m0.size)
    rec_new = torch.zeros(nrec, dtype=torch.uint8, device="cuda")
    # the M0 filter forced: its survivors (~326M) overflow, and pass 2 and the
    # bucket stage go on from the same pass-1 output
    ctx.set_option("m0_filter", 1)
    fb = ctx.counter("m0_filter_fallback")
    call("sg_triage_batch_dev", ctx.h, ms.h, ns.h, sig.data_ptr(), off.data_ptr(), nvals, nrec, rec_new.data_ptr(),
         None, None)
    torch.cuda.synchronize()
    ctx.set_option("m0_filter", -1)
    assert ctx.counter("m0_filter_fallback") == fb + 1
    got = rec_new.cpu().numpy()
    om, on = O.OSet(m0), O.OSet()
    exp, ev, eo = O.triage_batch(om, on, sig.cpu().numpy().view(np.uint32), off.cpu().numpy().view(np.uint64))
    assert np.array_equal(got, exp)
    em, en = om.export(), on.export()
    del om, on
    gn = ns.export()
    assert gn.size > 100_000_000 and gn.size == en.size  # ~208M new signals
    assert np.array_equal(gn, en)
    del gn
    assert np.array_equal(ms.export(), em)
    ns.close()
    ms.close()
    _diff_path(call, ctx, m0, sig, off, exp, ev, eo, em, en)
    call("sg_ctx_reset_stream", ctx.h)
