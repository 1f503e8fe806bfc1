#!/usr/bin/env python3
"""Per-program cycle breakdown of the executor-exact kernel (k_exec_region2,
sg_exec.hip) with the context's debug_part option: the steady state's queued
lists (bench.py steady_state.from_traces: triage of the traces, then
sg_exec_signal_queued_dev), every list of the same traces, and the a0 row's
fresh Zipf programs.  The library prints one "[exec dbg]" line per launch on
stderr; this script adds the HIP-event time of each launch on stdout."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from bench import POP_SEED, UNIVERSE_SEED, call  # noqa: E402
from syzkaller_amd.cover import Context, SignalSet  # noqa: E402


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b)


def main():
    torch.cuda.set_device(0)
    ctx = Context(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    cfg = {"programs": 65536, "calls": 16, "pcs_per_call": 1024, "zipf_s": 1.1, "ranks": 1 << 20}
    npop, noise = 2048, 2e-4
    g = bench.Gen(cfg)
    m0 = SignalSet(ctx)
    rec_new = torch.zeros(g.ncalls, dtype=torch.uint8, device="cuda")
    b = g.members(ctx, cfg, 0, npop)
    bench.triage(ctx, m0, None, b, rec_new)
    torch.cuda.synchronize()
    del b
    call("sg_gen_population_traces_dev", ctx.h, UNIVERSE_SEED, POP_SEED, npop, 5_000, noise, cfg["zipf_s"],
         cfg["ranks"], 0, cfg["programs"], cfg["calls"], cfg["pcs_per_call"], g.trace.data_ptr())
    so = torch.empty(g.ncalls + 1, dtype=torch.int64, device="cuda")
    ms = SignalSet(ctx)
    call("sg_set_copy", ms.h, m0.h)
    t_flags = timed(lambda: call("sg_triage_traces_dev", ctx.h, ms.h, None, g.trace.data_ptr(), g.call_off.data_ptr(),
                                 g.npcs, g.ncalls, rec_new.data_ptr()))
    print(f"steady flags from traces: {t_flags:.2f} ms, queued records {int(rec_new.sum())}", flush=True)

    def queued():
        call("sg_exec_signal_queued_dev", ctx.h, g.trace.data_ptr(), g.call_off.data_ptr(), g.prog_off.data_ptr(),
             cfg["programs"], g.ncalls, g.npcs, rec_new.data_ptr(), g.sig.data_ptr(), so.data_ptr())

    def every():
        call("sg_exec_signal_dev", ctx.h, g.trace.data_ptr(), g.call_off.data_ptr(), g.prog_off.data_ptr(),
             cfg["programs"], g.ncalls, g.npcs, g.sig.data_ptr(), so.data_ptr())

    for name, fn in (("queued lists", queued), ("every list", every)):
        fn()  # warm (code load)
        t = timed(fn)
        ctx.set_option("debug_part", 1)
        print(f"{name}: {t:.2f} ms (plain launch); breakdown launch follows on stderr", flush=True)
        fn()
        torch.cuda.synchronize()
        ctx.set_option("debug_part", 0)
    # the a0 row: 8192 fresh Zipf programs
    a0 = dict(cfg, programs=8192)
    call("sg_gen_zipf_traces_dev", ctx.h, UNIVERSE_SEED, 77, a0["zipf_s"], a0["ranks"], 0, a0["programs"], a0["calls"],
         a0["pcs_per_call"], g.trace.data_ptr())
    nc = a0["programs"] * a0["calls"]

    def row():
        call("sg_exec_signal_dev", ctx.h, g.trace.data_ptr(), g.call_off.data_ptr(), g.prog_off.data_ptr(),
             a0["programs"], nc, nc * a0["pcs_per_call"], g.sig.data_ptr(), so.data_ptr())

    row()
    t = timed(row)
    print(f"a0 row (8192 fresh programs): {t:.2f} ms (plain launch)", flush=True)
    ctx.set_option("debug_part", 1)
    row()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
