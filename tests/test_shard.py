"""The hash-sharded one-batch triage protocol (syzkaller_amd/shard.py) on CPU:
world size 2 and 4 over gloo, with the stages restated in numpy from their
contracts in include/syzsig.h (sg_shard_candidates_dev, sg_shard_owners_dev,
sg_shard_flags_dev, sg_set_add_dev).  The flags of every record and the final
maxSignal / newSignal must equal the single-rank oracle's sequential loop
(syz-fuzzer/fuzzer.go:645-693) over the whole batch in record order -- across
consecutive batches, with empty records, ranks holding no records, signal
shared between ranks, and the values 0 and 0xFFFFFFFF."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

SENT = 0xFFFFFFFF


def fmix32(s):
    """sg_shard_of's hash: the murmur3 finaliser (uint32 numpy arithmetic)."""
    s = np.asarray(s, dtype=np.uint32).copy()
    s ^= s >> np.uint32(16)
    s *= np.uint32(0x85EBCA6B)
    s ^= s >> np.uint32(13)
    s *= np.uint32(0xC2B2AE35)
    s ^= s >> np.uint32(16)
    return s


def shard_of(s, g):
    return ((fmix32(s).astype(np.uint64) * np.uint64(g)) >> np.uint64(32)).astype(np.int64)


class NpSet:
    """map[uint32]struct{} as a sorted unique array."""

    def __init__(self, vals=()):
        self.v = np.unique(np.asarray(vals, dtype=np.uint32))

    def has(self, x):
        return np.isin(np.asarray(x, dtype=np.uint32), self.v)

    def add(self, x):
        self.v = np.union1d(self.v, np.asarray(x, dtype=np.uint32)).astype(np.uint32)


class NumpyStages:
    """The stage contracts of include/syzsig.h restated in numpy."""

    def candidates(self, snapshot, vals, off, nvals, nrec, rec_base, nshards, pairs):
        v = vals[:nvals].numpy().view(np.uint32)
        o = off.numpy().astype(np.int64)
        rec = np.repeat(np.arange(nrec, dtype=np.int64), np.diff(o))
        m = ~snapshot.has(v)
        s, r = v[m], rec[m]
        us, first = np.unique(s, return_index=True)  # first occurrence = first record
        fr = r[first] + rec_base
        sh = shard_of(us, nshards)
        order = np.argsort(sh, kind="stable")
        out = np.stack([us[order], fr[order].astype(np.uint32)], axis=1).reshape(-1)
        pairs[: out.size] = torch.from_numpy(out.view(np.int32).copy())
        cnt = np.bincount(sh, minlength=nshards)
        return [0] + np.cumsum(cnt).tolist()

    def owners(self, pairs, npairs, nrec_total, rec_bits, new_vals):
        p = pairs[: 2 * npairs].numpy().view(np.uint32).reshape(-1, 2)
        nw = (nrec_total + 31) // 32
        bits = np.zeros(nw, dtype=np.uint32)
        if npairs == 0:
            rec_bits[:nw] = torch.from_numpy(bits.view(np.int32))
            return 0
        order = np.lexsort((p[:, 1], p[:, 0]))  # by s, then record
        ps = p[order]
        firsts = np.concatenate([[True], ps[1:, 0] != ps[:-1, 0]])
        own = ps[firsts]
        np.bitwise_or.at(bits, own[:, 1] >> 5, np.uint32(1) << (own[:, 1] & 31))
        rec_bits[:nw] = torch.from_numpy(bits.view(np.int32))
        new_vals[: own.shape[0]] = torch.from_numpy(own[:, 0].view(np.int32).copy())
        return int(own.shape[0])

    def flags(self, bits, nparts, wpp, rec_lo, nrec, rec_new):
        b = bits[: nparts * wpp].numpy().view(np.uint32).reshape(nparts, wpp)
        orb = np.bitwise_or.reduce(b, axis=0) if nparts else np.zeros(wpp, np.uint32)
        r = rec_lo + np.arange(nrec, dtype=np.int64)
        w = (r >> 5) - (rec_lo >> 5)
        rec_new[:nrec] = torch.from_numpy(((orb[w] >> (r & 31).astype(np.uint32)) & 1).astype(np.uint8))

    def add(self, sset, vals, n):
        if n:
            sset.add(vals[:n].numpy().view(np.uint32))


def batch(seed, nrec):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 30, size=nrec)
    lens[rng.integers(0, nrec, size=nrec // 4)] = 0
    vals = rng.integers(0, 3000, size=int(lens.sum())).astype(np.uint32)
    if vals.size > 10:
        vals[rng.integers(0, vals.size, size=5)] = SENT
        vals[rng.integers(0, vals.size, size=5)] = 0
        vals[-3:] = rng.integers(0, 1 << 32, size=3, dtype=np.uint64).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    return vals, off


def split(nrec, world, seed):
    """Contiguous record ranges per rank; some ranks may get none."""
    rng = np.random.default_rng(seed)
    cuts = np.sort(rng.integers(0, nrec + 1, size=world - 1))
    if seed % 3 == 0:
        cuts[0] = 0  # rank 0 empty
    b = np.concatenate([[0], cuts, [nrec]]).astype(np.int64)
    return [(int(b[k]), int(b[k + 1])) for k in range(world)]


M0 = np.arange(0, 3000, 5, dtype=np.uint32)
BATCHES = [(11, 700), (12, 1), (13, 900), (14, 0)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from syzkaller_amd.shard import Comm, ShardedTriage

        tri = ShardedTriage(NumpyStages(), Comm(), device="cpu")
        ms, ns = NpSet(M0), NpSet()
        out = []
        for seed, nrec in BATCHES:
            vals, off = batch(seed, nrec)
            r0, r1 = split(nrec, world, seed)[rank]
            e0, e1 = int(off[r0]), int(off[r1])
            v = torch.from_numpy(vals[e0:e1].view(np.int32).copy())
            o = torch.from_numpy((off[r0:r1 + 1] - off[r0]).astype(np.int64))
            rec_new = torch.zeros(max(r1 - r0, 1), dtype=torch.uint8)
            total = tri.step(ms, ns, v, o, e1 - e0, r1 - r0, r0, rec_new)
            assert total == nrec
            out.append((r0, rec_new[: r1 - r0].tolist(), tri.last))
        q.put((rank, out, ms.v.tolist(), ns.v.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4, 8])  # 8: the C3 node (manager.go:957-962 fans out to every fuzzer)
def test_sharded_triage_equals_sequential_loop(world):
    from oracle import pyoracle as O

    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, out, m, n = q.get(timeout=240)
        res[r] = (out, m, n)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    om, on = O.OSet(M0), O.OSet()
    for b, (seed, nrec) in enumerate(BATCHES):
        vals, off = batch(seed, nrec)
        ef = O.triage_flags_only(om, on, vals, off)
        got = np.zeros(nrec, np.uint8)
        for r in range(world):
            r0, fl, _ = res[r][0][b]
            got[r0:r0 + len(fl)] = fl
        assert np.array_equal(got, ef), (world, seed)
        if nrec > 100:
            assert 0 < ef.sum() < nrec  # mixed flags
            assert sum(res[r][0][b][2]["pairs_sent"] for r in range(world)) >= res[0][0][b][2]["new_signal"]
    for r in range(world):  # the replicated state is the sequential loop's on every rank
        assert res[r][1] == om.export().tolist()
        assert res[r][2] == on.export().tolist()


def test_shard_hash_matches_library():
    """The numpy restatement of sg_shard_of equals the library's (a pure
    function: callable without a GPU)."""
    from syzkaller_amd._lib import lib

    rng = np.random.default_rng(5)
    s = np.concatenate([rng.integers(0, 1 << 32, size=2000, dtype=np.uint64), [0, 1, SENT]]).astype(np.uint32)
    for g in (1, 2, 3, 4, 7, 8, 64):
        exp = shard_of(s, g)
        got = np.array([lib.sg_shard_of(int(x), g) for x in s])
        assert np.array_equal(got, exp), g
        assert exp.min() >= 0 and exp.max() < g
    assert lib.sg_shard_of(5, 0) == -1
