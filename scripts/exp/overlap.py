#!/usr/bin/env python3
"""Experiment: do two C2 triages on two HIP streams overlap?  Sequential (one
context) vs concurrent (two contexts, each its own stream and workspace) over
the same batches, each against its own copy of the 16M-entry maxSignal.
Measurement only (the concurrent runs are independent triages, not one loop)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import Gen, build_m0, triage, Context, SignalSet, call  # noqa: E402
from syzkaller_amd.shard import _WrappedSet  # noqa: E402

NB = int(os.environ.get("NB", "4"))
cfg = {"programs": 65536, "calls": 16, "pcs_per_call": 1024, "zipf_s": 1.1, "ranks": 1 << 20}
sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
ctxA, ctxB = Context(0), Context(0)
ctxA.set_stream(sA.cuda_stream)
ctxB.set_stream(sB.cuda_stream)
g = Gen(cfg)
warm = g.zipf(ctxA, cfg, 2_000_000)
bs = [g.zipf(ctxA, cfg, 3000 + k) for k in range(NB)]
del g
rec = [torch.empty(bs[0].nrec, dtype=torch.uint8, device="cuda") for _ in range(2)]
m0 = SignalSet(ctxA)
build_m0(ctxA, m0, warm, cfg["calls"], 16 << 20, rec[0])
del warm
W = 1 << 27
m0t = torch.empty(W, dtype=torch.int32, device="cuda")
m0w = _WrappedSet(ctxA, m0t)
call("sg_set_copy", m0w.h, m0.h)
torch.cuda.synchronize()
stt = [torch.empty(W, dtype=torch.int32, device="cuda") for _ in range(NB)]
nwt = [torch.zeros(W, dtype=torch.int32, device="cuda") for _ in range(2)]
wrapped = {}


def wset(ctx, t):
    k = (id(ctx), t.data_ptr())
    if k not in wrapped:
        wrapped[k] = _WrappedSet(ctx, t)
    return wrapped[k]


def reset():
    for t in stt:
        t.copy_(m0t)
    torch.cuda.synchronize()


def run(ctxs):
    reset()
    t = time.perf_counter()
    for i, b in enumerate(bs):
        k = i % len(ctxs)
        triage(ctxs[k], wset(ctxs[k], stt[i]), wset(ctxs[k], nwt[k]), b, rec[k])
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3 / NB


for rep in range(3):
    a = run([ctxA])
    b = run([ctxA, ctxB])
    print(f"rep {rep}: sequential {a:.3f} ms/batch, two streams {b:.3f} ms/batch", flush=True)
