"""The two-stage pipelined fuzzer loop (syzkaller_amd/pipeline.py): batch i+1's
partition on one stream beside batch i's bucket stage on another, the bucket
stages in batch order.  Over a run of batches sharing one maxSignal (the loop
of syz-fuzzer/fuzzer.go:645-693 across batches), the flags of every batch and
the final maxSignal / newSignal must equal sg_triage_batch_dev's, batch by
batch -- including empty batches and a slot reused while the other holds a
batch."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

UNIVERSE_SEED = 0x5A17C0DE
POP_SEED = 0x70A1B0C5


def _batch(ctx, nprog, calls, pcs, seed, npop=None):
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
    return sig[:nv].clone(), off


def _batches(ctx):
    out = [_batch(ctx, 96, 16, 256, 11)]  # fresh
    out += [_batch(ctx, 128, 16, 256, 20 + k, npop=64) for k in range(3)]  # re-executions: mixed flags
    out.append((torch.empty(0, dtype=torch.int32, device="cuda"), torch.zeros(1, dtype=torch.int64, device="cuda")))
    out.append((torch.empty(0, dtype=torch.int32, device="cuda"), torch.zeros(33, dtype=torch.int64, device="cuda")))
    out += [_batch(ctx, 64, 16, 512, 40), _batch(ctx, 160, 16, 128, 41, npop=64)]
    return out


@pytest.mark.timeout(120)
def test_pipelined_equals_sequential(ctx):
    from syzkaller_amd._lib import call
    from syzkaller_amd.cover import SignalSet
    from syzkaller_amd.pipeline import PipelinedTriage

    m0_vals, m0_off = _batch(ctx, 64, 16, 256, 7, npop=64)
    batches = _batches(ctx)
    sets = {}
    for name in ("seq", "pipe"):
        ms, ns = SignalSet(ctx), SignalSet(ctx)
        call("sg_set_add_dev", ms.h, m0_vals.data_ptr(), m0_vals.numel())
        sets[name] = (ms, ns)
    torch.cuda.synchronize()
    ms, ns = sets["seq"]
    exp = []
    for v, o in batches:
        nrec = o.numel() - 1
        f = torch.zeros(max(nrec, 1), dtype=torch.uint8, device="cuda")
        call("sg_triage_batch_dev", ctx.h, ms.h, ns.h, v.data_ptr() if v.numel() else None, o.data_ptr(), v.numel(),
             nrec, f.data_ptr() if nrec else None, None, None)
        exp.append(f)
    torch.cuda.synchronize()
    ms, ns = sets["pipe"]
    pt = PipelinedTriage(ctx)
    got = []
    for v, o in batches:
        nrec = o.numel() - 1
        f = torch.full((max(nrec, 1),), 7, dtype=torch.uint8, device="cuda")
        pt.submit(ms, ns, v, o, v.numel(), nrec, f)
        got.append(f)
    pt.close()
    torch.cuda.synchronize()
    mixed = 0
    for k, (v, o) in enumerate(batches):
        nrec = o.numel() - 1
        e, g = exp[k][:nrec].cpu().numpy(), got[k][:nrec].cpu().numpy()
        assert np.array_equal(e, g), k
        mixed += int(0 < e.sum() < nrec)
    assert mixed >= 2  # the re-executed batches have queued and dropped records
    for a, b in zip(sets["seq"], sets["pipe"]):
        assert np.array_equal(a.export(), b.export())
    for s in sets["seq"] + sets["pipe"]:
        s.close()


def test_partition_form_arguments(ctx):
    """Form 2 takes neither set (nor a novelty counter); forms 0/1 need both."""
    from syzkaller_amd._lib import SyzSigError, call
    from syzkaller_amd.cover import SignalSet

    v, o = _batch(ctx, 4, 4, 64, 3)
    a, b = SignalSet(ctx), SignalSet(ctx)
    nc = torch.zeros(1, dtype=torch.int64, device="cuda")
    for args in ((2, a.h, b.h, None), (2, None, None, nc.data_ptr()), (1, None, None, None), (3, None, None, None)):
        with pytest.raises(SyzSigError):
            call("sg_prefix_begin_form_dev", ctx.h, 0, args[0], args[1], args[2], v.data_ptr(), o.data_ptr(),
                 v.numel(), o.numel() - 1, args[3])
    a.close()
    b.close()
