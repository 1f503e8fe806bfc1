"""The sharded triage's stage kernels (sg_shard.hip) against their numpy
restatements, and the whole protocol (syzkaller_amd/shard.py) on the GPU
against the oracle's sequential loop (syz-fuzzer/fuzzer.go:645-693): one rank,
and two ranks sharing the one GPU of the test box over gloo (host-staged
exchanges; RCCL needs one GPU per rank)."""
import os
import socket

import numpy as np
import pytest
import torch

from oracle import pyoracle as O
from tests.test_shard import NumpyStages, NpSet, shard_of

pytestmark = pytest.mark.gpu


def _batch(seed, nrec, hi=1 << 22, maxlen=60):
    if nrec == 0:
        return np.zeros(0, np.uint32), np.zeros(1, np.uint64)
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, maxlen, size=nrec)
    lens[rng.integers(0, nrec, size=max(1, nrec // 5))] = 0
    vals = rng.integers(0, hi, size=int(lens.sum())).astype(np.uint32)
    vals[rng.integers(0, vals.size, size=vals.size // 3)] = vals[rng.integers(0, vals.size, size=vals.size // 3)]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    return vals, off


def _dev(a, dt):
    return torch.from_numpy(np.ascontiguousarray(a).view(dt)).cuda()


def _pairs_by_shard(pairs, shard_off, g):
    p = pairs.view(-1, 2)
    return [p[shard_off[k]:shard_off[k + 1]] for k in range(g)]


@pytest.mark.parametrize("g", [1, 3, 8])
def test_shard_candidates_vs_numpy(ctx, g):
    from syzkaller_amd.cover import SignalSet
    from syzkaller_amd.shard import HipStages

    vals, off = _batch(200 + g, 30000)
    m0 = np.unique(vals[:: 3])
    snap = SignalSet(ctx)
    from syzkaller_amd import cover as C
    C.SignalAdd(snap, m0)
    st = HipStages(ctx)
    pairs = torch.empty(2 * vals.size, dtype=torch.int32, device="cuda")
    so = st.candidates(snap, _dev(vals, np.int32), _dev(off, np.int64), vals.size, off.size - 1, 1000, g, pairs)
    exp_pairs = torch.zeros(2 * vals.size, dtype=torch.int32)
    eso = NumpyStages().candidates(NpSet(m0), torch.from_numpy(vals.view(np.int32)),
                                   torch.from_numpy(off.view(np.int64)), vals.size, off.size - 1, 1000, g, exp_pairs)
    assert so == eso
    got = pairs.cpu().numpy().view(np.uint32)
    exp = exp_pairs.numpy().view(np.uint32)
    for k in range(g):
        a = got[2 * so[k]: 2 * so[k + 1]].reshape(-1, 2)
        b = exp[2 * eso[k]: 2 * eso[k + 1]].reshape(-1, 2)
        a = a[np.lexsort((a[:, 1], a[:, 0]))]
        assert np.array_equal(a, b), k
        assert (shard_of(a[:, 0], g) == k).all()
    # the snapshot is only read
    assert np.array_equal(snap.export(), m0)


def test_shard_candidates_record_slices(C):
    """Record slices of the local stage (a lowered per-launch record limit):
    a signal may come once per slice; its smallest record is the first one."""
    from syzkaller_amd.shard import HipStages

    ctx2 = C.Context(0)
    ctx2.set_option("max_launch_records", 777)
    vals, off = _batch(301, 5000, hi=1 << 16)
    snap = C.SignalSet(ctx2)
    st = HipStages(ctx2)
    pairs = torch.empty(2 * vals.size, dtype=torch.int32, device="cuda")
    so = st.candidates(snap, _dev(vals, np.int32), _dev(off, np.int64), vals.size, off.size - 1, 0, 4, pairs)
    exp_pairs = torch.zeros(2 * vals.size, dtype=torch.int32)
    eso = NumpyStages().candidates(NpSet(), torch.from_numpy(vals.view(np.int32)), torch.from_numpy(off.view(np.int64)),
                                   vals.size, off.size - 1, 0, 4, exp_pairs)
    got = pairs.cpu().numpy().view(np.uint32)[: 2 * so[-1]].reshape(-1, 2)
    exp = exp_pairs.numpy().view(np.uint32)[: 2 * eso[-1]].reshape(-1, 2)
    exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))]  # the restatement's pairs are grouped by shard
    srt = got[np.lexsort((got[:, 1], got[:, 0]))]
    u, first = np.unique(srt[:, 0], return_index=True)
    assert np.array_equal(srt[first], exp)
    assert (shard_of(got[:, 0], 4) == np.repeat(np.arange(4), np.diff(so))).all()  # grouped by owning shard
    del snap
    ctx2.close()


class _Words:
    """A set's device words as the prefix argument of sg_prefix_end_dev."""

    def __init__(self, s):
        self.s = s

    def data_ptr(self):
        return self.s.device_words()


@pytest.mark.parametrize("pairs", [False, True])
@pytest.mark.parametrize("as_prefix", [False, True])
def test_prefix_begin_end_equals_triage(C, as_prefix, pairs):
    """sg_prefix_begin_dev / sg_prefix_end_dev (the partitions kept between
    the two calls, or with option prefix_pairs the first-owner pairs; several
    record slices via a lowered per-launch record limit) against the oracle: the
    marks are the batch's signal not in the base set, and the flags after end
    are the sequential loop's against maxsig | prefix.  Without a prefix
    maxsig / newsig end as the loop's; with one, maxsig ends between M0 ∪ new
    and M0 ∪ prefix ∪ new, and is the loop's after the prefix is ORed in."""
    from syzkaller_amd.shard import HipStages

    ctx2 = C.Context(0)
    ctx2.set_option("max_launch_records", 777)
    if pairs:
        ctx2.set_option("prefix_pairs", 1)
    st = HipStages(ctx2)
    vals, off = _batch(305, 5000, hi=1 << 18)
    m0 = np.unique(np.random.default_rng(306).integers(0, 1 << 18, size=20000)).astype(np.uint32)
    extra = np.unique(np.random.default_rng(307).integers(0, 1 << 18, size=5000)).astype(np.uint32)
    base, marks, ms, ns = C.SignalSet(ctx2), C.SignalSet(ctx2), C.SignalSet(ctx2), C.SignalSet(ctx2)
    C.SignalAdd(base, m0)
    pre = C.SignalSet(ctx2)
    if as_prefix:  # end runs against ms | pre = base | extra
        C.SignalAdd(ms, m0)
        C.SignalAdd(pre, extra)
    else:
        C.SignalAdd(ms, np.union1d(m0, extra))
    v, o = _dev(vals, np.int32), _dev(off, np.int64)
    nrec = off.size - 1
    rec_new = torch.zeros(nrec, dtype=torch.uint8, device="cuda")
    C.SignalAdd(marks, extra[::3])  # begin overwrites the marks
    st.prefix_begin(base, marks, v, o, vals.size, nrec, slot=1)
    st.prefix_end(ms, _Words(pre) if as_prefix else None, ns, rec_new, slot=1)
    torch.cuda.synchronize()
    assert np.array_equal(marks.export(), np.setdiff1d(np.unique(vals), m0))
    om, on = O.OSet(np.union1d(m0, extra)), O.OSet()
    ef = O.triage_flags_only(om, on, vals, off)
    assert np.array_equal(rec_new.cpu().numpy(), ef)
    assert 0 < ef.sum() < nrec
    assert np.array_equal(ns.export(), on.export())
    got = ms.export()
    if as_prefix:
        new = on.export()
        assert np.isin(np.union1d(m0, new), got).all() and np.isin(got, np.union1d(om.export(), extra)).all()
        ms.or_device(pre.device_words())
        got = ms.export()
    assert np.array_equal(got, om.export())
    # sg_prefix_flags_dev: the same flags; maxsig gains at most marks | prefix
    ms0 = m0 if as_prefix else np.union1d(m0, extra)
    ms2 = C.SignalSet(ctx2)
    C.SignalAdd(ms2, ms0)
    rec2 = torch.full((nrec,), 7, dtype=torch.uint8, device="cuda")
    C.SignalAdd(marks, extra)  # (begin overwrites marks: include/syzsig.h)
    st.prefix_begin(base, marks, v, o, vals.size, nrec, slot=0)
    st.prefix_flags(ms2, _Words(pre) if as_prefix else None, rec2, slot=0)
    torch.cuda.synchronize()
    assert np.array_equal(rec2.cpu().numpy(), ef)
    got2 = ms2.export()
    assert np.isin(ms0, got2).all()
    assert np.isin(got2, np.union1d(np.union1d(ms0, marks.export()), extra if as_prefix else ms0)).all()
    del ms2
    del base, marks, ms, ns, pre
    ctx2.close()


@pytest.fixture(scope="module")
def C(ctx):
    from syzkaller_amd import cover

    return cover


def test_shard_owners_and_flags_vs_numpy(ctx):
    from syzkaller_amd.shard import HipStages

    rng = np.random.default_rng(7)
    nrec_total = 100000
    parts = []
    for r in range(5):  # five senders: distinct s per sender
        s = np.unique(rng.integers(0, 1 << 18, size=20000)).astype(np.uint32)
        rec = rng.integers(0, nrec_total, size=s.size).astype(np.uint32)
        parts.append(np.stack([s, rec], axis=1))
    p = np.concatenate(parts).reshape(-1)
    npairs = p.size // 2
    st = HipStages(ctx)
    bits = torch.empty((nrec_total + 31) // 32, dtype=torch.int32, device="cuda")
    new = torch.empty(npairs, dtype=torch.int32, device="cuda")
    nnew = st.owners(_dev(p, np.int32), npairs, nrec_total, bits, new)
    ebits = torch.zeros((nrec_total + 31) // 32, dtype=torch.int32)
    enew = torch.zeros(npairs, dtype=torch.int32)
    ennew = NumpyStages().owners(torch.from_numpy(p.view(np.int32)), npairs, nrec_total, ebits, enew)
    assert nnew == ennew
    assert np.array_equal(bits.cpu().numpy(), ebits.numpy())
    assert np.array_equal(np.sort(new[:nnew].cpu().numpy().view(np.uint32)), np.sort(enew[:ennew].numpy().view(np.uint32)))
    # flags: three parts of one rank's word range, odd record bounds
    for rec_lo, nrec in ((0, 64), (37, 1000), (96, 5), (12345, 54321)):
        wpp = ((rec_lo + nrec + 31) >> 5) - (rec_lo >> 5)
        b = rng.integers(-(1 << 31), (1 << 31) - 1, size=3 * wpp).astype(np.int32)
        got = torch.zeros(nrec, dtype=torch.uint8, device="cuda")
        st.flags(_dev(b, np.int32), 3, wpp, rec_lo, nrec, got)
        exp = torch.zeros(nrec, dtype=torch.uint8)
        NumpyStages().flags(torch.from_numpy(b), 3, wpp, rec_lo, nrec, exp)
        assert np.array_equal(got.cpu().numpy(), exp.numpy()), (rec_lo, nrec)


def _run_protocol(ctx_dev, world, rank, batches, m0, proto="pairs", collectives=False, form="auto"):
    from syzkaller_amd import cover as C
    from syzkaller_amd.shard import Comm, HipStages, PrefixTriage, ShardedTriage
    from tests.test_shard import split

    ctx = C.Context(ctx_dev)
    side_ctx = None
    exchange = "auto"
    if proto.endswith("_sparse"):  # the candidate-list exchange from the first batch on
        proto, exchange = proto[: -len("_sparse")], "sparse"
    if proto == "prefix_pipelined":
        # the PrefixTriage the bench runs at N > 1: batches overlapped through
        # the two slots, the prefix-OR on a side stream (here also at one rank;
        # the all-to-all form -- plain "prefix" at two ranks is gather mode)
        side = torch.cuda.Stream()
        side_ctx = C.Context(ctx_dev)
        with torch.cuda.stream(side):
            side_st = HipStages(side_ctx)
        tri = PrefixTriage(HipStages(ctx), Comm(collectives=collectives), two_phase_at_one=True, side_stages=side_st,
                           side_stream=side, gather=False, form=form, exchange=exchange)
    elif proto == "prefix":
        tri = PrefixTriage(HipStages(ctx), Comm(collectives=collectives),
                           two_phase_at_one=collectives or exchange == "sparse", form=form, exchange=exchange)
    else:
        tri = ShardedTriage(HipStages(ctx), Comm(collectives=collectives))
    ms, ns = C.SignalSet(ctx), C.SignalSet(ctx)
    C.SignalAdd(ms, m0)
    out, pend = [], None
    for seed, nrec in batches:
        vals, off = _batch(seed, nrec)
        r0, r1 = split(nrec, world, seed)[rank] if world > 1 else (0, nrec)
        e0, e1 = int(off[r0]), int(off[r1])
        v = _dev(vals[e0:e1] if e1 > e0 else np.zeros(1, np.uint32), np.int32)
        o = _dev((off[r0:r1 + 1] - off[r0]).astype(np.uint64), np.int64)
        rec_new = torch.zeros(max(r1 - r0, 1), dtype=torch.uint8, device="cuda")
        out.append((r0, r1, rec_new))
        if side_ctx is None:
            tri.step(ms, ns, v, o, e1 - e0, r1 - r0, r0, rec_new)
            continue
        p = tri.start(ms, ns, v, o, e1 - e0, r1 - r0, r0, rec_new, nrec_total=nrec)
        if pend is not None:
            assert tri.finish(pend[0]) == pend[1]
        pend = (p, nrec, v, o)  # (the batch's buffers live until its finish)
    if pend is not None:
        assert tri.finish(pend[0]) == pend[1]
    torch.cuda.synchronize()
    out = [(r0, fl[: r1 - r0].cpu().tolist()) for r0, r1, fl in out]
    res = (out, ms.export().tolist(), ns.export().tolist())
    del ms, ns, tri, pend
    ctx.close()
    if side_ctx is not None:
        side_ctx.close()
    return res


BATCHES = [(401, 4000), (402, 3000), (403, 0), (404, 5000)]
M0 = np.unique(np.random.default_rng(400).integers(0, 1 << 22, size=50000)).astype(np.uint32)


def _expected():
    om, on = O.OSet(M0), O.OSet()
    flags = []
    for seed, nrec in BATCHES:
        vals, off = _batch(seed, nrec)
        flags.append(O.triage_flags_only(om, on, vals, off))
    return flags, om.export().tolist(), on.export().tolist()


@pytest.mark.parametrize("proto,form", [("pairs", "auto"), ("prefix", "auto"), ("prefix_pipelined", "auto"),
                                        ("prefix_pipelined", "pairs"), ("prefix_pipelined", "kept"),
                                        ("prefix_sparse", "auto"), ("prefix_pipelined_sparse", "auto")])
def test_sharded_protocol_one_rank_vs_oracle(ctx, proto, form):
    """form: PrefixTriage's per-batch step-1 form (auto by the last counted
    batch's novelty, or forced) -- the same flags and sets whichever runs."""
    out, m, n = _run_protocol(0, 1, 0, BATCHES, M0, proto, form=form)
    ef, em, en = _expected()
    for b, (r0, fl) in enumerate(out):
        assert np.array_equal(np.array(fl, np.uint8), ef[b]), b
        if BATCHES[b][1] > 100:
            assert 0 < ef[b].sum() < BATCHES[b][1]
    assert m == em and n == en


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, proto, backend="gloo"):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":  # RCCL: one rank on the box's one GPU, its collectives forced on
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _run_protocol(0, world, rank, BATCHES, M0, proto, collectives=backend == "nccl")))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("proto", ["pairs", "prefix", "prefix_pipelined", "prefix_sparse", "prefix_pipelined_sparse"])
def test_sharded_protocol_two_ranks_one_gpu(proto):
    import torch.multiprocessing as mp

    world = 2
    port = _free_port()
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    procs = [mctx.Process(target=_worker, args=(r, world, port, q, proto)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, v = q.get(timeout=280)
        res[r] = v
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ef, em, en = _expected()
    for b, (seed, nrec) in enumerate(BATCHES):
        got = np.zeros(nrec, np.uint8)
        for r in range(world):
            r0, fl = res[r][0][b]
            got[r0:r0 + len(fl)] = fl
        assert np.array_equal(got, ef[b]), b
    for r in range(world):
        assert res[r][1] == em and res[r][2] == en


@pytest.mark.timeout(300)
@pytest.mark.parametrize("proto", ["pairs", "prefix", "prefix_pipelined", "prefix_sparse"])
def test_sharded_protocol_rccl_one_rank(proto):
    """The RCCL branch of Comm (syzkaller_amd/shard.py): a one-rank "nccl"
    group with the collectives forced on, so the device-tensor
    all_to_all_single / all_gather_into_tensor run through RCCL, the async
    handles are waited on, and (prefix_pipelined) the prefix-OR runs on the
    side stream between them; flags and sets equal the oracle's sequential
    loop.  (Two or more RCCL ranks need one GPU each: the driver's multi-GPU
    runs.)"""
    import torch.multiprocessing as mp

    port = _free_port()
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    p = mctx.Process(target=_worker, args=(0, 1, port, q, proto, "nccl"))
    p.start()
    r, (out, m, n) = q.get(timeout=280)
    p.join(timeout=60)
    assert p.exitcode == 0
    ef, em, en = _expected()
    for b, (r0, fl) in enumerate(out):
        assert np.array_equal(np.array(fl, np.uint8), ef[b]), b
    assert m == em and n == en
