#!/usr/bin/env python3
"""bench.py -- coverage PCs triaged per second on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): per GPU, batches of 64Ki programs x
16 calls x 1024 PCs of synthetic Zipf(1.1) traces over 2^20 PC ranks
(pc = 0x81000000 + 16*perm(rank)), turned into per-call signal by the
executor-exact edge/dedup kernel (executor/executor.h:389-401, :497-526), then
triaged against a maxSignal bitmap that starts with >=16M entries (built from a
warm-up batch of another seed).  All inputs are generated on the GPU and stay
resident in HBM before the timed region starts.

One step = one pass of the hot path over one batch: syz-fuzzer/fuzzer.go:645-693
execute() for every call record of the batch (new-signal test, per-record
attribution, the ordered diffs, maxSignal/newSignal update), followed by the
Poll drain of newSignal (fuzzer.go:358-364; with N>1 the manager merge of
manager.go:949-962 and fuzzer.go:392-398 as an RCCL OR-exchange of the
newSignal bitmaps).  Each step triages a fresh batch (the fuzzer's steady
state); value = all signal entries triaged by all ranks / max-over-ranks time.

Run:  python bench.py [--gpus N --steps K --warmup W]
      (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from syzkaller_amd import _lib  # noqa: E402  (fails loudly without libsyzsig.so)
from syzkaller_amd._lib import call, lib  # noqa: E402
from syzkaller_amd.cover import Context, SignalSet  # noqa: E402

METRIC = "coverage PCs triaged/sec vs corpus signal (+ % HBM roofline), 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
U32_WORDS = 1 << 27     # 2^32-bit signal bitmap


class Batch:
    def __init__(self, vals, off, nvals, nrec, seed):
        self.vals, self.off, self.nvals, self.nrec, self.seed = vals, off, nvals, nrec, seed


def gen_batch(ctx, cfg, seed, trace_buf, sig_cap, call_off, prog_off):
    """Zipf traces -> executor signal (CSR), resident on the GPU."""
    nprog, calls, pcs = cfg["programs"], cfg["calls"], cfg["pcs_per_call"]
    ncalls, npcs = nprog * calls, nprog * calls * pcs
    call("sg_gen_zipf_traces_dev", ctx.h, cfg["universe_seed"], seed, cfg["zipf_s"], cfg["ranks"], 0, nprog, calls,
         pcs, trace_buf.data_ptr())
    sig_off = torch.empty(ncalls + 1, dtype=torch.int64, device="cuda")
    call("sg_exec_signal_dev", ctx.h, trace_buf.data_ptr(), call_off.data_ptr(), prog_off.data_ptr(), nprog, ncalls,
         npcs, sig_cap.data_ptr(), sig_off.data_ptr())
    torch.cuda.synchronize()
    nvals = int(sig_off[-1].item())
    vals = sig_cap[:nvals].clone()
    return Batch(vals, sig_off, nvals, ncalls, seed)


class Poll:
    """newSignal drain + manager merge (fuzzer.go:358-364, manager.go:949-962,
    fuzzer.go:392-398): every rank's maxSignal gains every other rank's new
    signal.  Bitmaps are OR-reduced with an all-to-all of 1/N shards, a local
    OR, and an all-gather (RCCL has no bitwise-OR reduction).

    The reference polls on its own timer (every 10 s or when candidates run
    low, fuzzer.go:331-346): triage never waits for a Poll, and other fuzzers'
    signal reaches maxSignal at arbitrary points.  So the exchange runs one
    step behind, on a stream of its own:
      step k triages into newSignal buffer k % 2;
      that buffer is exchanged while step k + 1 triages into the other one;
      before step k + 2 the merged bits are OR-ed into maxSignal and the buffer
      is cleared (the drain).
    drain() finishes every pending exchange (inside the timed region).  At N=1
    there is no exchange and the buffer is just drained each step, unless
    `selftest` runs the same streams and events with an identity exchange."""

    def __init__(self, ctx, world, selftest=False):
        from syzkaller_amd.dist import OrExchange

        self.world = world
        self.bufs = [torch.zeros(U32_WORDS, dtype=torch.int32, device="cuda") for _ in range(2)]
        self.sets = []
        for buf in self.bufs:
            h = ctypes_void_p()
            call("sg_set_wrap_dev", ctx.h, buf.data_ptr(), ctypes_byref(h))
            self.sets.append(_Wrapped(h))
        self.active = world > 1 or selftest
        self.k = 0
        if self.active:
            self.comm = torch.cuda.Stream()
            self.ex = [OrExchange(buf) if world > 1 else None for buf in self.bufs]
            self.merged = [None, None]
            self.done = [None, None]

    def newsig(self):
        """The newSignal set step k triages into."""
        return self.sets[self.k % 2]

    def after_triage(self, maxsig):
        """Call once step k's triage is queued on the compute stream."""
        slot = self.k % 2
        self.k += 1
        if not self.active:
            self.bufs[slot].zero_()  # drained (fuzzer.go:358-364)
            return
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(ev)
            merged = self.ex[slot](self.bufs[slot]) if self.ex[slot] is not None else self.bufs[slot]
            done = torch.cuda.Event()
            done.record(self.comm)
        self.merged[slot], self.done[slot] = merged, done
        self._apply(self.k % 2, maxsig)  # the slot the next step triages into

    def _apply(self, slot, maxsig):
        if not self.active or self.done[slot] is None:
            return
        torch.cuda.current_stream().wait_event(self.done[slot])
        call("sg_set_or_dev", maxsig.h, self.merged[slot].data_ptr())  # fuzzer.go:392-398
        self.bufs[slot].zero_()
        self.done[slot] = None

    def drain(self, maxsig):
        for d in (1, 0):  # the older pending exchange first
            self._apply((self.k + d) % 2, maxsig)


def triage_step(ctx, maxsig, newsig, b, rec_new, diff_vals, diff_off):
    """fuzzer.go:645-693 over one batch.  With diff buffers the claim/resolve
    path also emits the ordered diff lists; without, the partitioned path
    computes the same flags and set updates (the diff is a transient of the
    reference loop, fuzzer.go:669-674)."""
    call("sg_triage_batch_dev", ctx.h, maxsig.h, newsig.h, b.vals.data_ptr(), b.off.data_ptr(), b.nvals, b.nrec,
         rec_new.data_ptr(), diff_vals.data_ptr() if diff_vals is not None else None,
         diff_off.data_ptr() if diff_off is not None else None)


KERNELS = ["p1_hist", "p1_scatter", "p2_hist", "p2_scatter", "bucket_triage", "bucket_spill", "scan",
           "triage_claim", "triage_resolve", "emit"]


def part_geometry(n_in, n_rec):
    """Tile / chunk counts of the partitioned path (sg_bucket.hip BucketPlan):
    pass-1 tiles (16384 entries / 256 records each), and pass-2 chunks (about
    one per non-empty (slice, 2^16-record group) pair beyond the full ones)."""
    na = -(-int(n_in) // 16384)
    t = na + (int(n_rec) - 1) // 256
    ng = (int(n_rec) - 1) // 65536 + 1
    return t, na + 256 * ng // 2


def algo_bytes(n_in, n_cand, n_diff, n_rec, n_newwords):
    """Algorithmic bytes per launch of each kernel.  n_cand =
    values not in maxSignal at batch start.  Partition passes move 4 B per
    entry each way plus their [digit][tile] offset tables."""
    t, g2 = part_geometry(n_in, n_rec)
    mbits = 4 * (1 << 27)  # the maxSignal bitmap, read once slice by slice
    return {
        "p1_hist": 4 * n_in + 256 * t * 4,
        "p1_scatter": 4 * n_in + 4 * n_in + 256 * t * 4,
        "p2_hist": 4 * n_in + 256 * g2 * 4,
        "p2_scatter": 4 * n_in + 4 * n_in + 256 * g2 * 4,
        # entries + the maxSignal and newSignal slices + the two new-word stores + one owner-key flag each
        "bucket_triage": 4 * n_in + 2 * mbits + 8 * n_newwords + n_diff,
        "triage_claim": 4 * n_in + 4 * n_in + 8 * n_cand + n_in / 8,
        "triage_resolve": n_in / 8 + 4 * n_cand + 4 * n_cand + 16 * n_diff + n_rec + n_in / 8 + n_in / 64,
    }


def set_count(s):
    return len(s)


def cpu_baseline(m0_values, batch, cfg, gpu_flags, budget_s):
    """The oracle (C restatement of fuzzer.go:645-693 with Go-map-like hash
    sets) on a bounded prefix of the first batch, single-threaded, plus a
    prefix parity check against the GPU's flags for the same records."""
    from oracle import pyoracle as O

    calls = cfg["calls"]
    off = batch.off.cpu().numpy().astype(np.uint64)
    vals_all = None
    t0 = time.perf_counter()
    ms = O.OSet(m0_values)
    build_s = time.perf_counter() - t0
    done_prog, elapsed, nel = 0, 0.0, 0
    flags = []
    chunk = 16
    while done_prog < cfg["programs"] and elapsed < budget_s:
        p1 = min(cfg["programs"], done_prog + chunk)
        r0, r1 = done_prog * calls, p1 * calls
        e0, e1 = int(off[r0]), int(off[r1])
        v = batch.vals[e0:e1].cpu().numpy().view(np.uint32)
        o = (off[r0:r1 + 1] - off[r0]).astype(np.uint64)
        t = time.perf_counter()
        f, dv, do = O.triage_batch(ms, None, v, o)
        elapsed += time.perf_counter() - t
        flags.append(f)
        nel += e1 - e0
        done_prog = p1
        if elapsed > 0:
            chunk = max(16, int(done_prog * (budget_s / elapsed) - done_prog) // 4)
    flags = np.concatenate(flags) if flags else np.zeros(0, np.uint8)
    parity = None
    if gpu_flags is not None:
        parity = bool(np.array_equal(flags, gpu_flags[: flags.size]))
    return {
        "value": nel / elapsed if elapsed else None,
        "unit": "PCs/s",
        "cores": 1,
        "kind": "port",
        "sample": f"first {done_prog} programs ({done_prog * calls} call records, {nel} signal entries) of the first "
                  f"batch vs the same {len(m0_values)}-entry maxSignal; C restatement of the Go reference "
                  f"(oracle/sigoracle.c, Go maps mirrored by open-addressing hash sets), not Go; set build "
                  f"{build_s:.1f}s excluded",
        "prefix_parity_vs_gpu": parity,
    }


def load_traffic(kernel):
    """HBM bytes per launch from the PMC summary committed under profiles/
    (FETCH_SIZE/WRITE_SIZE passes, gfx950-corrected), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("kernels", {}).get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--programs", type=int, default=65536)
    ap.add_argument("--calls", type=int, default=16)
    ap.add_argument("--pcs", type=int, default=1024)
    ap.add_argument("--m0", type=int, default=16 << 20, help="entries in the starting maxSignal")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU baseline work")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-account", action="store_true", help="skip the byte-accounting replay")
    ap.add_argument("--diff", action="store_true", help="also emit the ordered diff lists (claim/resolve path)")
    ap.add_argument("--poll-selftest", action="store_true",
                    help="N=1: run the pipelined Poll's streams and events with an identity exchange")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE={world}"

    cfg = {"programs": args.programs, "calls": args.calls, "pcs_per_call": args.pcs, "zipf_s": 1.1,
           "ranks": 1 << 20, "universe_seed": 0x5A17C0DE}
    ctx = Context(local)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)

    nprog, calls, pcs = cfg["programs"], cfg["calls"], cfg["pcs_per_call"]
    ncalls, npcs = nprog * calls, nprog * calls * pcs
    trace_buf = torch.empty(npcs, dtype=torch.int32, device="cuda")
    sig_cap = torch.empty(npcs, dtype=torch.int32, device="cuda")
    call_off = torch.arange(0, npcs + 1, pcs, dtype=torch.int64, device="cuda")
    prog_off = torch.arange(0, ncalls + 1, calls, dtype=torch.int64, device="cuda")

    t_gen = time.perf_counter()
    # warm-up corpus signal (seed 2 family) and the step batches (distinct seeds per rank and step)
    warm = gen_batch(ctx, cfg, 2_000_000 + rank, trace_buf, sig_cap, call_off, prog_off)
    batches = [gen_batch(ctx, cfg, 1_000 + 100_000 * rank + k, trace_buf, sig_cap, call_off, prog_off)
               for k in range(args.warmup + args.steps)]
    del trace_buf, sig_cap
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t_gen

    maxsig = SignalSet(ctx)
    poll = Poll(ctx, world, selftest=args.poll_selftest)

    # M0: triage the warm batch program-chunk by program-chunk until >= --m0 entries
    maxnrec = max(b.nrec for b in batches)
    maxnvals = max([b.nvals for b in batches] + [warm.nvals])
    rec_new = torch.empty(maxnrec, dtype=torch.uint8, device="cuda")
    diff_vals = torch.empty(maxnvals, dtype=torch.int32, device="cuda")
    diff_off = torch.empty(maxnrec + 1, dtype=torch.int64, device="cuda")
    chunk_prog = 256
    woff = warm.off.cpu().numpy()
    p = 0
    while p < nprog and len(maxsig) < args.m0:
        p1 = min(nprog, p + chunk_prog)
        r0, r1 = p * calls, p1 * calls
        e0, e1 = int(woff[r0]), int(woff[r1])
        sub_off = (warm.off[r0:r1 + 1] - e0).contiguous()
        sub_vals = warm.vals[e0:e1].contiguous()
        call("sg_triage_batch_dev", ctx.h, maxsig.h, None, sub_vals.data_ptr(), sub_off.data_ptr(), e1 - e0, r1 - r0,
             rec_new.data_ptr(), None, None)
        p = p1
    torch.cuda.synchronize()
    m0_count = len(maxsig)
    m0_values = maxsig.export() if (rank == 0 and world == 1 and not args.no_cpu) else None
    del warm

    # warm-up steps (untimed)
    gpu_flags0 = None
    dv_t, do_t = (diff_vals, diff_off) if args.diff else (None, None)
    for k in range(args.warmup):
        triage_step(ctx, maxsig, poll.newsig(), batches[k], rec_new, dv_t, do_t)
        if k == 0:
            gpu_flags0 = rec_new[: batches[0].nrec].cpu().numpy()
        poll.after_triage(maxsig)
    poll.drain(maxsig)
    torch.cuda.synchronize()

    # snapshot the state for the byte-accounting replay
    backup = None
    if not args.no_account:
        backup = SignalSet(ctx)
        call("sg_set_copy", backup.h, maxsig.h)
        torch.cuda.synchronize()
    m_start = len(maxsig)

    # ---- timed region ----
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.timing(True)
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        triage_step(ctx, maxsig, poll.newsig(), batches[k], rec_new, dv_t, do_t)
        poll.after_triage(maxsig)
    poll.drain(maxsig)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernels = {}
    for name in KERNELS:
        ms, n = ctx.kernel_time(name)
        if n:
            kernels[name] = {"ms_total": ms, "launches": n}
    ctx.timing(False)
    m_end = len(maxsig)

    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    units = torch.tensor([sum(b.nvals for b in batches[args.warmup:])], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(units, op=dist.ReduceOp.SUM)
    elapsed = float(t.item())
    total_units = float(units.item())

    # ---- byte accounting replay (outside the timed region) ----
    acct = None
    if backup is not None:
        call("sg_set_copy", maxsig.h, backup.h)
        for buf in poll.bufs:
            buf.zero_()
        torch.cuda.synchronize()
        n_in = n_cand = n_diff = n_rec = n_new = n_queued = 0
        for k in range(args.warmup, args.warmup + args.steps):
            b = batches[k]
            c = ctypes_u64()
            call("sg_set_count_missing_dev", maxsig.h, b.vals.data_ptr(), b.nvals, ctypes_byref(c))
            m_before = len(maxsig)
            # the diff path here, so the diff element count is known too
            triage_step(ctx, maxsig, poll.newsig(), b, rec_new, diff_vals, diff_off)
            torch.cuda.synchronize()
            n_diff += int(diff_off[b.nrec].item())
            n_queued += int(rec_new[: b.nrec].sum().item())
            n_new += len(maxsig) - m_before
            n_in += b.nvals
            n_cand += c.value
            n_rec += b.nrec
            poll.after_triage(maxsig)
        poll.drain(maxsig)
        torch.cuda.synchronize()
        acct = {"n_in": n_in, "n_cand": n_cand, "n_diff": n_diff, "n_rec": n_rec, "n_new_signal": n_new,
                "n_queued": n_queued}

    result = None
    if rank == 0:
        ms_step = elapsed * 1e3 / args.steps
        roof = None
        pipeline = None
        if acct and kernels:
            L = args.steps
            n_in, n_cand, n_diff, n_rec, n_new = (acct[x] / L for x in ("n_in", "n_cand", "n_diff", "n_rec",
                                                                         "n_new_signal"))
            per = algo_bytes(n_in, n_cand, n_diff, n_rec, min(n_new, 1 << 27))
            for kname, b in per.items():
                if kname in kernels:
                    avg_s = kernels[kname]["ms_total"] / kernels[kname]["launches"] / 1e3
                    kernels[kname]["avg_ms"] = avg_s * 1e3
                    kernels[kname]["algo_bytes_per_launch"] = b
                    kernels[kname]["achieved_GBs"] = b / avg_s / 1e9
            dom = max((k for k in per if k in kernels), key=lambda k: kernels[k]["ms_total"])
            ach = kernels[dom]["achieved_GBs"]
            roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": load_traffic(dom)}
            # whole-step view with SURVEY.md §8(d)'s C2 formula (N_uniq taken as N_in)
            b_step = 4 * n_in + 4 * n_in + 8 * n_cand + 4 * n_cand + 4 * n_diff + n_rec / 8
            pipeline = {"algo_bytes_per_step": b_step, "achieved_GBs": b_step / (ms_step / 1e3) / 1e9,
                        "frac": b_step / (ms_step / 1e3) / 1e9 / HBM_PEAK_GBS,
                        "formula": "4N_in + 4N_uniq + 8N_cand + 4N_cand + 4N_out + N_rec/8 (N_uniq=N_in)"}
        cpu = None
        if world == 1 and not args.no_cpu and m0_values is not None:
            cpu = cpu_baseline(m0_values, batches[0], cfg, gpu_flags0, args.cpu_budget)
        per_step_new = (m_end - m_start) / args.steps
        result = {
            "metric": METRIC,
            "value": total_units / elapsed,
            "unit": "PCs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (Zipf(1.1) PC traces generated on the GPU, counter-based PRNG)",
            "config": {
                "workload": "C2: per GPU 64Ki programs x 16 calls x 1024 Zipf PCs -> executor signal -> "
                            "batched new-signal triage vs a >=16M-entry maxSignal bitmap",
                "programs_per_gpu": nprog, "calls": calls, "pcs_per_call": pcs,
                "signal_per_step_per_gpu": total_units / args.steps / world,
                "maxsignal_start": m0_count, "maxsignal_at_timing": m_start,
                "new_signal_per_step": per_step_new,
                "parallelism": f"one fuzzer per GPU x{world}, newSignal OR-exchange (RCCL all-to-all + all-gather) "
                               f"per step, pipelined one step behind" if world > 1 else "single GPU",
            },
            "roofline": roof,
            "cpu_baseline": cpu,
            "kernels": kernels,
            "pipeline_roofline": pipeline,
            "path": "claim/resolve + ordered diff" if args.diff else "partitioned (flags + set updates)",
            "accounting": acct,
            "gen_s": round(t_gen, 2),
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


# small ctypes helpers kept local to the bench
import ctypes  # noqa: E402


def ctypes_void_p():
    return ctypes.c_void_p()


def ctypes_u64():
    return ctypes.c_uint64()


def ctypes_byref(x):
    return ctypes.byref(x)


class _Wrapped:
    """A sg_set handle wrapping caller memory (freed by its owner tensor)."""

    def __init__(self, h):
        self.h = h

    def __del__(self):
        try:
            lib.sg_set_destroy(self.h)
        except Exception:
            pass


if __name__ == "__main__":
    main()
