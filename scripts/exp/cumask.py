#!/usr/bin/env python3
"""Experiment: the pipelined loop (syzkaller_amd/pipeline.py) with batch i's
bucket stage and batch i+1's partition on disjoint CU sets
(hipExtStreamCreateWithCUMask).  The bucket kernel fills every CU's LDS, so on
shared CUs nothing of the partition runs beside it; on disjoint sets the
latency-bound bucket kernel and the HBM-bound partition passes run together.

  BUCKET_CUS=none|lo:N|even   (lo:N = CUs 0..N-1, even = the even CUs; the
                               partition stream gets the complement)
Each step triages its batch against its own copy of the 16M-entry maxSignal
(bench.py's C2 recipe); every batch's flags are checked against the unmasked
sequential path.  Measurement only."""
import ctypes
import json
import os
import sys
import time

spec = os.environ.get("BUCKET_CUS", "none")
NCU = 256
if spec == "none":
    bcus = None
elif spec == "even":
    bcus = list(range(0, NCU, 2))
elif spec == "odd8":  # whole XCDs if CUs are numbered XCD-interleaved: CUs c with c % 8 < 4
    bcus = [c for c in range(NCU) if c % 8 < 4]
else:
    bcus = list(range(int(spec.split(":")[1])))
if bcus is not None:
    os.environ["SG_BUCKET_BLOCKS"] = str(3 * len(bcus))  # (read once, at the first bucket launch)

import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from bench import Gen, build_m0, triage, Context, SignalSet, call, kernel_table, STEP_KERNELS  # noqa: E402
from syzkaller_amd.pipeline import PipelinedTriage  # noqa: E402

NB = int(os.environ.get("NB", "8"))


def cu_stream(cus):
    hip = ctypes.CDLL("libamdhip64.so")
    mask = (ctypes.c_uint32 * (NCU // 32))()
    for c in cus:
        mask[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(NCU // 32), mask)
    assert rc == 0, rc
    got = (ctypes.c_uint32 * (NCU // 32))()
    hip.hipExtStreamGetCUMask(s, ctypes.c_uint32(NCU // 32), got)
    return torch.cuda.ExternalStream(s.value), [int(x) for x in got]


cfg = {"programs": 65536, "calls": 16, "pcs_per_call": 1024, "zipf_s": 1.1, "ranks": 1 << 20}
ctx = Context(0)
ctx.set_stream(torch.cuda.current_stream().cuda_stream)
g = Gen(cfg)
warm = g.zipf(ctx, cfg, 2_000_000)
bs = [g.zipf(ctx, cfg, 1000 + k) for k in range(NB)]
del g
rec = torch.empty(bs[0].nrec, dtype=torch.uint8, device="cuda")
m0 = SignalSet(ctx)
build_m0(ctx, m0, warm, cfg["calls"], 16 << 20, rec)
del warm
ns = SignalSet(ctx)
states = [SignalSet(ctx) for _ in bs]
# the sequential unmasked flags, per batch
exp = []
for b in bs:
    call("sg_set_copy", states[0].h, m0.h)
    triage(ctx, states[0], None, b, rec)
    exp.append(rec[: b.nrec].clone())
torch.cuda.synchronize()
if bcus is None:
    sp, sb, masks = torch.cuda.Stream(), torch.cuda.current_stream(), None
else:
    pcus = [c for c in range(NCU) if c not in set(bcus)]
    sb, mb = cu_stream(bcus)
    sp, mp_ = cu_stream(pcus)
    masks = {"bucket": [hex(x) for x in mb], "partition": [hex(x) for x in mp_]}
flags = [torch.empty(b.nrec, dtype=torch.uint8, device="cuda") for b in bs]
res = {"bucket_cus": spec, "masks": masks, "reps": []}
for rep in range(3):
    for st in states:
        call("sg_set_copy", st.h, m0.h)
    torch.cuda.synchronize()
    pt = PipelinedTriage(ctx, part_stream=sp, bucket_stream=sb)
    if rep == 2:
        ctx.timing(True)
    t0 = time.perf_counter()
    for st, b, f in zip(states, bs, flags):
        pt.submit(st, ns, b.vals, b.off, b.nvals, b.nrec, f)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / NB
    pt.close()
    ok = all(torch.equal(f, e) for f, e in zip(flags, exp))
    res["reps"].append({"ms_per_batch": round(ms, 3), "flags_equal": ok})
    print(f"rep {rep}: {spec} pipelined {ms:.3f} ms/batch flags_equal={ok}", flush=True)
res["kernels"] = {k: round(v["avg_ms"], 3) for k, v in kernel_table(ctx, STEP_KERNELS, NB).items()}
ctx.timing(False)
ctx.set_stream(torch.cuda.current_stream().cuda_stream)
print(json.dumps(res), flush=True)
