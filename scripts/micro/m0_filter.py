#!/usr/bin/env python3
"""Microbenchmark: can an exact M0 pre-filter beat the partition in the steady state?

Builds bench.py's steady-state workload (maxSignal = a 2048-program population's
signal, a batch of 64Ki programs re-executed from it with flaky coverage), puts
maxSignal's signals into a compact hash table (full 32-bit values, 4-slot 16-B
buckets) and times one pass over the batch's 880M entries (non-temporal loads)
that probes the table per entry (m0_filter.hip).  Prints one JSON line per
variant: ms, G probes/s, the fraction of entries the table proves to be in M0.

Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o scripts/micro/libm0filter.so scripts/micro/m0_filter.hip
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from syzkaller_amd.cover import Context, SignalSet  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
mf = ctypes.CDLL(os.path.join(HERE, "libm0filter.so"))
mf.mf_build.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                        ctypes.c_void_p]
mf.mf_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32,
                        ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]


def out(**kw):
    print(json.dumps(kw), flush=True)


def table(vals, log2):
    t = torch.zeros(4 << log2, dtype=torch.int32, device="cuda")
    d = torch.zeros(1, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    assert mf.mf_build(t.data_ptr(), log2, vals.data_ptr(), vals.numel(), d.data_ptr(), st) == 0
    torch.cuda.synchronize()
    return t, int(d.item())


def probe(mode, vals, tab, log2, hot=None, hlog2=0, reps=5, blocks=4096):
    st = torch.cuda.current_stream().cuda_stream
    hits = torch.zeros(1, dtype=torch.int64, device="cuda")
    hp = hot.data_ptr() if hot is not None else tab.data_ptr()
    n = vals.numel() & ~3
    assert mf.mf_probe(mode, vals.data_ptr(), n, tab.data_ptr(), log2, hp, hlog2, hits.data_ptr(), blocks, st) == 0
    ts = []
    for _ in range(reps):
        hits.zero_()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        assert mf.mf_probe(mode, vals.data_ptr(), n, tab.data_ptr(), log2, hp, hlog2, hits.data_ptr(), blocks,
                           st) == 0
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ms = float(np.median(ts))
    return ms, n / ms / 1e6, int(hits.item()) / n


def main():
    torch.cuda.set_device(0)
    ctx = Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    cfg = {"programs": 65536, "calls": 16, "pcs_per_call": 1024, "zipf_s": 1.1, "ranks": 1 << 20}
    npop, noise = 2048, 2e-4
    g = bench.Gen(cfg)
    m0set = SignalSet(ctx)
    rec_new = torch.empty(cfg["programs"] * cfg["calls"], dtype=torch.uint8, device="cuda")
    t0 = time.perf_counter()
    b = g.members(ctx, cfg, 0, npop)
    bench.triage(ctx, m0set, None, b, rec_new)
    torch.cuda.synchronize()
    del b
    m0 = torch.from_numpy(m0set.export().view(np.int32)).cuda()
    prev = g.population(ctx, cfg, 5_000, npop, noise)
    cur = g.population(ctx, cfg, 5_001, npop, noise)
    out(what="setup", m0=int(m0.numel()), entries=int(cur.nvals), s=round(time.perf_counter() - t0, 1))

    # frequency profile of the previous batch: coverage of the current batch by its top-K signals
    u, c = torch.unique(prev.vals, return_counts=True)
    order = torch.argsort(c, descending=True)
    hot_sorted = u[order]
    cs = torch.cumsum(c[order], 0).double() / prev.nvals
    cov = {str(k): round(float(cs[min(k, cs.numel()) - 1]), 4) for k in (1 << 14, 1 << 16, 1 << 17, 1 << 18, 1 << 20,
                                                                        1 << 22) if cs.numel()}
    out(what="prev-batch coverage by its top-K signals", distinct=int(u.numel()), coverage=cov)
    del u, c, order, cs

    ms, rate, frac = probe(0, cur.vals, m0, 0)
    out(what="stream only (NT read of the entries)", ms=ms, gb_s=cur.nvals * 4 / ms / 1e6)
    for log2 in (21, 22, 23, 24):
        tab, dropped = table(m0, log2)
        ms, rate, frac = probe(1, cur.vals, tab, log2)
        out(what="one table", table_mib=(16 << log2) >> 20, load=m0.numel() / (4 << log2), dropped=dropped,
            ms=ms, g_probes_s=rate, hit_frac=frac)
        if log2 in (22, 23):
            for hl in (14, 16, 18):
                k = min(hot_sorted.numel(), (4 << hl) // 2)
                hot, hd = table(hot_sorted[:k].contiguous(), hl)
                ms, rate, frac = probe(2, cur.vals, tab, log2, hot, hl)
                out(what="hot table, then big table", table_mib=(16 << log2) >> 20, hot_kib=(16 << hl) >> 10,
                    hot_signals=k, hot_dropped=hd, ms=ms, g_probes_s=rate, hit_frac=frac)
                del hot
        del tab
    # uniform random members of M0: no skew
    idx = torch.randint(0, m0.numel(), (cur.nvals,), device="cuda")
    uni = m0[idx]
    del idx
    for log2 in (22, 23):
        tab, _ = table(m0, log2)
        ms, rate, frac = probe(1, uni, tab, log2)
        out(what="one table, uniform M0 members", table_mib=(16 << log2) >> 20, ms=ms, g_probes_s=rate, hit_frac=frac)
        del tab


if __name__ == "__main__":
    main()
