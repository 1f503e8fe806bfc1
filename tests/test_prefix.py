"""The bitmap-prefix one-batch triage protocol (syzkaller_amd/shard.py
PrefixTriage) on CPU: world size 2 and 4 over gloo, with the stages restated
in numpy from their contracts (sg_triage_batch_dev, sg_prefix_begin_dev /
sg_prefix_end_dev / sg_prefix_flags_dev, sg_set_clear / or_dev, sg_bitmap_prefix_or_dev) over
a 2^20-signal bitmap (the protocol is word-wise, so a smaller signal space
exercises it fully; the full 2^32 space runs on the GPU in
tests/test_shard_gpu.py).  The flags of every record and the final
maxSignal / newSignal must equal the single-rank oracle's sequential loop
(syz-fuzzer/fuzzer.go:645-693) over the whole batch in record order."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.test_shard import _free_port, split

BITS = 20
WORDS = 1 << (BITS - 5)


class BitSet:
    """A signal set as a bitmap of WORDS uint32 words (bit s & 31 of word s >> 5)."""

    def __init__(self, w=None):
        self.w = np.zeros(WORDS, np.uint32) if w is None else w

    def has(self, s):
        s = np.asarray(s, dtype=np.uint64)
        return ((self.w[s >> np.uint64(5)] >> (s & np.uint64(31)).astype(np.uint32)) & 1).astype(bool)

    def add(self, s):
        s = np.asarray(s, dtype=np.uint64)
        np.bitwise_or.at(self.w, s >> np.uint64(5), (np.uint32(1) << (s & np.uint64(31)).astype(np.uint32)))

    def export(self):
        i = np.nonzero(np.unpackbits(self.w.view(np.uint8), bitorder="little"))[0]
        return i.astype(np.uint32).tolist()


class NumpyPrefixStages:
    words = WORDS

    def __init__(self):
        self.kept = {}
        self.forms = []  # the forms begin was asked for (both restate the same contract)

    def new_set(self):
        return BitSet()

    def wrap(self, t):
        return BitSet(t.numpy().view(np.uint32)[:WORDS])

    def copy(self, dst, src):
        dst.w[:] = src.w

    def clear(self, s):
        s.w[:] = 0

    def or_words(self, s, t):
        s.w |= t.numpy().view(np.uint32)[:WORDS]

    def or_new_words(self, s, t, exclude):
        s.w |= t.numpy().view(np.uint32)[:WORDS] & ~exclude.w

    def prefix_or(self, parts, nparts, words, prefix, total):
        p = parts.numpy().view(np.uint32)[: nparts * words].reshape(nparts, words)
        pre = prefix.numpy().view(np.uint32)[: nparts * words].reshape(nparts, words)
        acc = np.zeros(words, np.uint32)
        for k in range(nparts):
            pre[k] = acc
            acc = acc | p[k]
        total.numpy().view(np.uint32)[:words] = acc

    def prefix_or_rank(self, parts, nparts, words, rank, prefix, total):
        p = parts.numpy().view(np.uint32)[: nparts * words].reshape(nparts, words)
        if prefix is not None:
            acc = np.zeros(words, np.uint32)
            for k in range(rank):
                acc |= p[k]
            prefix.numpy().view(np.uint32)[:words] = acc
        total.numpy().view(np.uint32)[:words] = np.bitwise_or.reduce(p, axis=0)

    def or_new_or(self, newset, s, t):
        w = t.numpy().view(np.uint32)[:WORDS]
        if newset is not None:
            newset.w |= w & ~s.w
        s.w |= w

    def add(self, sset, vals, n):
        if n:
            sset.add(vals[:n].numpy().view(np.uint32))

    def add_new(self, newset, sset, vals, n):
        """sset |= vals[:n]; newset gains those sset lacked (sg_set_add_new_dev)."""
        if n:
            v = vals[:n].numpy().view(np.uint32)
            if newset is not None:
                newset.add(v[~sset.has(v)])
            sset.add(v)

    def delete(self, sset, vals, n):
        if n:
            v = vals[:n].numpy().view(np.uint32).astype(np.uint64)
            np.bitwise_and.at(sset.w, v >> np.uint64(5), ~(np.uint32(1) << (v & np.uint64(31)).astype(np.uint32)))

    def prefix_cands(self, out, cap, slot=0):
        """The slot's batch signal not in base, once each (sg_prefix_cands_dev)."""
        m = np.array(self.kept[slot][4].export(), np.uint32)[:cap]
        out.numpy().view(np.uint32)[: m.size] = m

    def prefix_begin(self, base, marks, vals, off, nvals, nrec, slot=0, form=None, ncand=None):
        v = vals[:nvals].numpy().view(np.uint32)
        marks.w[:] = 0  # (marks = the batch's signal not in base)
        if v.size:
            marks.add(v[~base.has(v)])
        self.kept[slot] = (vals, off, nvals, nrec, marks)
        self.forms.append(form)
        if ncand is not None:  # the batch's distinct signals not in base
            ncand[0] = int(np.unpackbits(marks.w.view(np.uint8)).sum())

    def prefix_flags(self, maxset, prefix, rec_new, slot=0):
        """The loop's flags against maxset | prefix (include/syzsig.h)."""
        vals, off, nvals, nrec, _ = self.kept.pop(slot)
        start = maxset.w | (prefix.numpy().view(np.uint32)[:WORDS] if prefix is not None else 0)
        self.triage(BitSet(start.copy()), None, vals, off, nvals, nrec, rec_new)

    def prefix_end(self, maxset, prefix, newset, rec_new, slot=0):
        """The flags; newset gains marks minus maxset | prefix, maxset |= marks."""
        marks = self.kept[slot][4]
        pre = prefix.numpy().view(np.uint32)[:WORDS] if prefix is not None else 0
        if newset is not None:
            newset.w |= marks.w & ~(maxset.w | pre)
        self.prefix_flags(maxset, prefix, rec_new, slot)
        maxset.w |= marks.w

    def triage(self, maxset, newset, vals, off, nvals, nrec, rec_new):
        """The sequential loop (fuzzer.go:665-690) restated over bitmaps."""
        v = vals[:nvals].numpy().view(np.uint32)
        o = off.numpy().astype(np.int64)
        for r in range(nrec):
            sig = v[o[r]:o[r + 1]]
            new = sig[~maxset.has(sig)] if sig.size else sig
            rec_new[r] = 1 if new.size else 0
            if new.size:
                maxset.add(new)
                if newset is not None:
                    newset.add(new)


def batch(seed, nrec):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 30, size=nrec)
    lens[rng.integers(0, nrec, size=nrec // 4)] = 0
    vals = rng.integers(0, 3000, size=int(lens.sum())).astype(np.uint32)
    if vals.size > 10:
        vals[rng.integers(0, vals.size, size=5)] = (1 << BITS) - 1
        vals[rng.integers(0, vals.size, size=5)] = 0
        vals[-3:] = rng.integers(0, 1 << BITS, size=3).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    return vals, off


M0 = np.arange(0, 3000, 5, dtype=np.uint32)
BATCHES = [(21, 700), (22, 1), (23, 900), (24, 0), (25, 600)]


def _worker(rank, world, port, q, pipelined, gather, drain=False, pairs_below=0.05, exchange="auto", sparse_below=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from syzkaller_amd.shard import Comm, PrefixTriage

        stages = NumpyPrefixStages()
        tri = PrefixTriage(stages, Comm(), device="cpu", gather=gather, pairs_below=pairs_below, exchange=exchange,
                           sparse_below=sparse_below)
        xforms = []  # each started batch's exchange form
        xbytes = []
        models = []  # non-pipelined: tri.exchange_model() agrees with the bytes sent
        ms, ns = BitSet(), BitSet()
        ms.add(M0)
        out = []
        drained = []  # drain: newSignal after each batch's finish, then cleared (the Poll, fuzzer.go:358-364)
        pend = None

        def finish(pd):
            xforms.append(pd[0]["last"]["exchange"])
            xbytes.append(pd[0]["last"]["exchange_bytes"])
            assert tri.finish(pd[0]) == pd[1]
            if drain:
                drained.append(ns.export())
                ns.w[:] = 0

        for seed, nrec in BATCHES:
            vals, off = batch(seed, nrec)
            r0, r1 = split(nrec, world, seed)[rank]
            e0, e1 = int(off[r0]), int(off[r1])
            v = torch.from_numpy(vals[e0:e1].view(np.int32).copy())
            o = torch.from_numpy((off[r0:r1 + 1] - off[r0]).astype(np.int64))
            rec_new = torch.zeros(max(r1 - r0, 1), dtype=torch.uint8)
            out.append((r0, r1, rec_new))
            if not pipelined:
                assert tri.step(ms, ns, v, o, e1 - e0, r1 - r0, r0, rec_new) == nrec
                xforms.append(tri.last["exchange"])
                xbytes.append(tri.last["exchange_bytes"])
                # the batch's exchange in both forms: the one it took is what it sent
                model = tri.exchange_model()
                if exchange == "dense":  # (forced dense: no counts are gathered, no model)
                    models.append(model is None)
                else:
                    models.append(model is not None and model[tri.last["exchange"]] == tri.last["exchange_bytes"]
                                  and model["sparse"] == (4 * model["candidates_max"] + 16) * (world - 1))
                continue
            # the next batch started (marked against the maxSignal that still
            # lacks this batch's total) before the previous one is finished
            p = tri.start(ms, ns, v, o, e1 - e0, r1 - r0, r0, rec_new, nrec_total=nrec)
            if pend is not None:
                finish(pend)
            pend = (p, nrec)
        if pend is not None:
            finish(pend)
        q.put((rank, [(r0, fl[: r1 - r0].tolist()) for r0, r1, fl in out], ms.export(),
               drained if drain else ns.export(), stages.forms, xforms, xbytes, models))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,pipelined,gather,drain,pairs_below",
                         [(2, False, False, False, 0.05), (4, False, False, False, 0.05),
                          (2, True, False, False, 0.05), (4, True, False, False, 0.05),
                          (2, True, True, False, 0.05), (4, False, True, False, 0.05),
                          (2, True, False, True, 0.05), (4, True, True, True, 0.05),
                          (2, False, False, False, 2.0), (4, True, False, True, 2.0),
                          (2, True, True, False, -1.0),
                          # G = 8, the C3 node: the prefix-OR over 7 predecessors,
                          # gather mode's 8 bitmaps per rank
                          (8, False, False, False, 0.05), (8, True, True, True, 0.05),
                          (8, True, False, False, 2.0)])
def test_prefix_triage_equals_sequential_loop(world, pipelined, gather, drain, pairs_below):
    _run_and_check(world, pipelined, gather, drain, pairs_below, "auto", None, None)


def _run_and_check(world, pipelined, gather, drain, pairs_below, exchange, sparse_below, expect_x):
    """drain: newSignal is read and cleared after every finish() while the next
    batch is already started -- each drained set must be exactly that batch's
    new signal (fuzzer.go:674: only what maxSignal lacked), not a re-report of
    the previous batch's."""
    from oracle import pyoracle as O

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, pipelined, gather, drain, pairs_below, exchange,
                                               sparse_below)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    xall = []
    for _ in range(world):
        r, out, m, n, forms, xforms, xbytes, models = q.get(timeout=240)
        assert all(models), models
        if expect_x is None:  # (the default sparse_below, 0.05, is below the novelty here)
            assert set(xforms) == {"dense"}, xforms
        else:
            if expect_x == "any":
                xall.append(xforms)
            else:
                assert xforms == expect_x, xforms
            for f, b in zip(xforms, xbytes):  # a list of candidates against whole bitmaps
                assert (b < 4 * (1 << 20)) if f == "sparse" else (b >= (1 << 15)), (f, b)
        res[r] = (out, m, n)
        # the form of each batch from the novelty of the last counted one: kept
        # first (no count yet); pairs_below 2.0 (above any novelty): pairs after
        if expect_x is not None:  # the sparse exchange takes the pairs form
            assert all(f == 1 for f, x in zip(forms, expect_x) if x == "sparse"), forms
        elif pairs_below > 1.0:  # kept until a non-empty batch has been counted, pairs after
            assert forms[-1] == 1 and forms == sorted(forms), forms
        elif pairs_below < 0:
            assert set(forms) == {0}, forms
        if expect_x is None or expect_x[0] == "dense":
            assert forms[0] == 0, forms
        else:  # by each rank's novelty (later batches overlap the earlier ones' signal)
            assert set(forms) <= {0, 1}, forms
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(x == xall[0] for x in xall), xall  # every rank took the same forms
    om, on = O.OSet(M0), O.OSet()
    per_batch_new = []
    for b, (seed, nrec) in enumerate(BATCHES):
        vals, off = batch(seed, nrec)
        if drain:
            on = O.OSet()
        ef = O.triage_flags_only(om, on, vals, off)
        per_batch_new.append(on.export().tolist())
        got = np.zeros(nrec, np.uint8)
        for r in range(world):
            r0, fl = res[r][0][b]
            got[r0:r0 + len(fl)] = fl
        assert np.array_equal(got, ef), (world, seed)
        if nrec > 100:
            assert 0 < ef.sum() < nrec  # mixed flags
    for r in range(world):  # the replicated state is the sequential loop's on every rank
        assert res[r][1] == om.export().tolist()
        if drain:
            assert res[r][2] == per_batch_new
        else:
            assert res[r][2] == on.export().tolist()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,pipelined,gather,drain,exchange,sparse_below,expect",
                         [(2, False, True, False, "auto", 2.0, ["dense", "dense", "sparse", "sparse", "sparse"]),
                          (4, True, False, True, "auto", 2.0, ["dense", "dense", "sparse", "sparse", "sparse"]),
                          (4, False, False, False, "sparse", None, ["sparse"] * 5),
                          (2, True, True, True, "sparse", None, ["sparse"] * 5),
                          (4, True, True, False, "auto", 0.2, None),
                          # G = 8: the count agreement over 8 ranks, dense / sparse / auto,
                          # gather and all-to-all modes
                          (8, True, False, True, "auto", 2.0, ["dense", "dense", "sparse", "sparse", "sparse"]),
                          (8, False, True, False, "sparse", None, ["sparse"] * 5),
                          (8, True, False, False, "auto", 0.2, None),
                          (8, True, True, False, "dense", None, ["dense"] * 5)])
def test_prefix_sparse_exchange_equals_sequential_loop(world, pipelined, gather, drain, exchange, sparse_below, expect):
    """The candidate-list exchange: forced from the first
    batch, and mixed with the bitmap exchange within one run (the form agreed
    from the counts two batches back; sparse_below 2.0 is above any novelty,
    0.2 lets the batches decide), pipelined or not, in gather and all-to-all
    mode, with newSignal drained between batches.  Flags and both sets equal
    the sequential loop's; the sparse steps move a few KB per rank."""
    if expect is None:  # the forms depend on the batches: any mix, the same on every rank
        _run_and_check(world, pipelined, gather, drain, 0.05, exchange, sparse_below, "any")
    else:
        _run_and_check(world, pipelined, gather, drain, 0.05, exchange, sparse_below, expect)


def test_exchange_time_model():
    """The per-rank exchange time model that the C3 line
    reports as predicted_exchange_ms: no exchange at one rank; the dense
    all-to-all form moves 3 slices of 512 MiB / G per link (G = 8: ~1.3 ms of
    link time at 153 GB/s per direction); the gather form the whole bitmap per
    link; the sparse form only the candidate lists."""
    from syzkaller_amd.shard import XGMI_LINK_GBS, exchange_time_model

    assert exchange_time_model(1) == {"dense": 0.0, "sparse": None}
    m8 = exchange_time_model(8, cand_max=100_000)
    link8 = 3 * (512 << 20) / 8 / (XGMI_LINK_GBS * 1e6)
    assert link8 < m8["dense"] < link8 + 0.5
    assert exchange_time_model(2)["dense"] > exchange_time_model(4)["dense"] > m8["dense"]
    assert exchange_time_model(8, gather=True)["dense"] > m8["dense"]
    assert m8["sparse"] < 0.2 and exchange_time_model(8, cand_max=10 ** 8)["sparse"] > m8["sparse"]
