#!/usr/bin/env python3
"""A few steady-state C2 triage steps (bench.py's steady workload: maxSignal =
a 2048-program population's signal, a batch of 64Ki programs re-executed from
it with flaky coverage), for kernel traces and PMC passes of the flags path
with the M0 filter (option m0_filter: argv[1], default -1 auto).  Prints the
HIP-event time of each step."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from bench import call  # noqa: E402
from syzkaller_amd.cover import Context, SignalSet  # noqa: E402


def main():
    mode = int(sys.argv[1]) if len(sys.argv) > 1 else -1
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    torch.cuda.set_device(0)
    ctx = Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.set_option("m0_filter", mode)
    cfg = {"programs": 65536, "calls": 16, "pcs_per_call": 1024, "zipf_s": 1.1, "ranks": 1 << 20}
    g = bench.Gen(cfg)
    m0 = SignalSet(ctx)
    rec_new = torch.zeros(g.ncalls, dtype=torch.uint8, device="cuda")
    b = g.members(ctx, cfg, 0, 2048)
    bench.triage(ctx, m0, None, b, rec_new)
    del b
    batch = g.population(ctx, cfg, 5_000, 2048, 2e-4)
    states = [SignalSet(ctx) for _ in range(steps + 1)]
    for st in states:
        call("sg_set_copy", st.h, m0.h)
    bench.triage(ctx, states[0], None, batch, rec_new)  # warm-up
    torch.cuda.synchronize()
    call("sg_ctx_marker", ctx.h, 0, 9)
    ctx.timing(True)
    for st in states[1:]:
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        bench.triage(ctx, st, None, batch, rec_new)
        e.record()
        torch.cuda.synchronize()
        print(f"step {a.elapsed_time(e):.3f} ms, queued {int(rec_new.sum())}, "
              f"filtered slices {ctx.counter('m0_filter_used')}, survivors {ctx.counter('m0_filter_survivors')}", flush=True)
    call("sg_ctx_marker", ctx.h, 1, 9)
    kt = {}
    for name in ("p1_hist", "p1_scatter", "m0_index", "m0_filter", "m0_tail", "p2_hist", "p2_scatter", "bucket_triage"):
        ms, n = ctx.kernel_time(name)
        if n:
            kt[name] = round(ms / n, 3)
    print("kernels (ms per launch):", kt, flush=True)


if __name__ == "__main__":
    main()
