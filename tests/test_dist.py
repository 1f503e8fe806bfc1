"""Multi-rank plumbing on CPU (gloo, world size 2): the newSignal OR-exchange
that implements the manager's Poll merge (syzkaller_amd/dist.py), checked
against a sequential replay of the reference protocol (fuzzer.go:358-364,
manager.go:949-962, fuzzer.go:392-398) with the oracle as each fuzzer's
local triage."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORDS = 1 << 15  # a 2^20-signal space keeps the CPU test small (the product uses 2^27 words)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bits_to_values(words):
    w = words.numpy().view(np.uint32)
    idx = np.nonzero(w)[0]
    out = [int(i) * 32 + b for i in idx for b in range(32) if (int(w[i]) >> b) & 1]
    return np.array(out, dtype=np.uint32)


def _values_to_bits(vals):
    w = np.zeros(WORDS, dtype=np.uint32)
    for v in np.asarray(vals, dtype=np.uint64):
        w[int(v) >> 5] |= np.uint32(1 << (int(v) & 31))
    return torch.from_numpy(w.view(np.int32).copy())


def _batch(seed):
    rng = np.random.default_rng(seed)
    recs = [rng.integers(0, 1 << 20, size=int(rng.integers(0, 40))).astype(np.uint32) for _ in range(200)]
    off = np.concatenate([[0], np.cumsum([r.size for r in recs])]).astype(np.uint64)
    return np.concatenate(recs), off


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pyoracle as O
        from syzkaller_amd.dist import OrExchange, or_allreduce

        # 1. plain OR all-reduce
        g = torch.Generator().manual_seed(rank)
        w = torch.randint(-(1 << 31), (1 << 31) - 1, (WORDS,), dtype=torch.int32, generator=g)
        allw = [torch.empty_like(w) for _ in range(world)]
        dist.all_gather(allw, w)
        exp = allw[0].clone()
        for x in allw[1:]:
            exp |= x
        assert torch.equal(or_allreduce(w), exp)
        # 2. one fuzzer per rank: local triage (oracle), then Poll as OR-exchange
        m0 = np.arange(0, 1 << 20, 7, dtype=np.uint32)
        ms, ns = O.OSet(m0), O.OSet()
        vals, off = _batch(100 + rank)
        flags, _, _ = O.triage_batch(ms, ns, vals, off)
        ex = OrExchange(torch.zeros(WORDS, dtype=torch.int32))
        merged = ex(_values_to_bits(ns.export()))
        ms.add(_bits_to_values(merged))
        q.put((rank, ms.export().tolist(), ns.export().tolist(), flags.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_poll_or_exchange_world2():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, m, n, f = q.get(timeout=240)
        res[r] = (set(m), set(n), f)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # sequential replay of the reference protocol
    from oracle import pyoracle as O

    m0 = np.arange(0, 1 << 20, 7, dtype=np.uint32)
    mgr = O.OSet(m0)
    fuzz = []
    for r in range(world):
        ms, ns = O.OSet(m0), O.OSet()
        vals, off = _batch(100 + r)
        flags, _, _ = O.triage_batch(ms, ns, vals, off)
        assert list(flags) == res[r][2]
        fuzz.append((ms, ns))
    # every fuzzer polls (manager.go:949-962); then every fuzzer polls again and
    # receives what the others added (fuzzer.go:392-398)
    queues = {r: [] for r in range(world)}
    for r in range(world):
        drained = fuzz[r][1].export()
        newmax, _ = O.merge_poll(mgr, drained, np.array([0, drained.size], np.uint64))
        for r1 in range(world):
            if r1 != r:
                queues[r1].extend(newmax.tolist())
    for r in range(world):
        fuzz[r][0].add(np.array(queues[r], dtype=np.uint32))
        assert set(fuzz[r][0].export().tolist()) == res[r][0]
        assert set(fuzz[r][1].export().tolist()) == res[r][1]
    assert set(mgr.export().tolist()) == res[0][0] == res[1][0]
