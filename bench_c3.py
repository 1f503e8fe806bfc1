"""bench.py's multi-GPU workloads (one process per GPU, RCCL over xGMI).

C3 (BASELINE.json configs[2]): ONE batch of N x 128Ki programs (16 calls x
1024 Zipf PCs each, the C2 recipe; N=8 is C3's 1Mi-program batch), its records
split contiguously over the N ranks, triaged as the single sequential loop of
syz-fuzzer/fuzzer.go:645-693 by the hash-sharded protocol of
syzkaller_amd/shard.py against a replicated 16M-entry maxSignal snapshot
(each timed step against its own copy of it, made before the timed region, as at N=1).  Weak scaling: 128Ki programs per GPU.

fuzzers: one independent fuzzer per GPU, each triaging its own batches, with
the Poll merge (fuzzer.go:358-364, manager.go:949-962, fuzzer.go:392-398) as an
RCCL OR-exchange of the newSignal bitmaps (syzkaller_amd/dist.py).
"""
import time

import numpy as np
import torch
import torch.distributed as dist

from bench import (METRIC, STEP_KERNELS, Gen, build_m0, call, cpu_baseline, kernel_table, n_uniq, pmc_bytes_per_step,
                   step_bytes, triage, HBM_PEAK_GBS, Context, SignalSet, U32_WORDS, StepTimer)
from syzkaller_amd.shard import Comm, HipStages, PrefixTriage, ShardedTriage, exchange_time_model

SHARD_KERNELS = STEP_KERNELS + ["shard_local", "shard_route", "shard_owner", "shard_resolve", "shard_flags",
                                "set_add", "prefix_or", "bucket_mark", "prefix_flags", "prefix_merge", "set_or", "set_or_new_or",
                                "set_or_new"]


def _cdev():
    """Device of small collective tensors: host ones under gloo (rehearsals)."""
    return "cuda" if not dist.is_initialized() or dist.get_backend() == "nccl" else "cpu"


def _max_over_ranks(x, world):
    t = torch.tensor([x], dtype=torch.float64, device=_cdev())
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _sum_over_ranks(x, world):
    t = torch.tensor([x], dtype=torch.float64, device=_cdev())
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def run_c3(ctx, args, cfg, rank, world):
    calls, nprog = cfg["calls"], cfg["programs"]
    g = Gen(cfg)
    t_gen = time.perf_counter()
    # the replicated snapshot: every rank builds the same 16M-entry maxSignal
    # from the same warm batch (deterministic, so no broadcast is needed)
    steady = getattr(args, "c3_steady", False)
    maxsig, newsig, m0set = SignalSet(ctx), SignalSet(ctx), SignalSet(ctx)
    if steady:
        # the low-novelty steady state (bench.py run_steady's recipe): maxSignal
        # = the population's signal, batches of population programs re-executed
        # with flaky coverage
        rec_new = torch.empty(nprog * calls, dtype=torch.uint8, device="cuda")
        step = max(1, min(nprog, args.npop))
        for m in range(0, args.npop, step):
            mb = g.members(ctx, cfg, m, min(args.npop, m + step))
            triage(ctx, m0set, None, mb, rec_new)
            torch.cuda.synchronize()
            del mb
        batches = [g.population(ctx, cfg, 5_000 + k, args.npop, args.noise, prog_base=rank * nprog)
                   for k in range(args.warmup + args.steps)]
    else:
        warm = g.zipf(ctx, dict(cfg, programs=nprog), 2_000_000, prog_base=0)
        batches = [g.zipf(ctx, cfg, 3_000 + k, prog_base=rank * nprog) for k in range(args.warmup + args.steps)]
        rec_new = torch.empty(max(b.nrec for b in batches), dtype=torch.uint8, device="cuda")
        build_m0(ctx, m0set, warm, calls, args.m0, rec_new)
        del warm
    del g
    t_gen = time.perf_counter() - t_gen
    m0_count = len(m0set)
    if world > 1:
        counts = [torch.zeros(1, dtype=torch.int64, device=_cdev()) for _ in range(world)]
        dist.all_gather(counts, torch.tensor([m0_count], dtype=torch.int64, device=_cdev()))
        assert len({int(c.item()) for c in counts}) == 1, "maxSignal snapshots differ between ranks"
    prefix = getattr(args, "c3_proto", "prefix") == "prefix"
    two_phase = getattr(args, "c3_two_phase", False)
    # the prefix protocol's exchange: batches overlapped through PrefixTriage's
    # two slots (batch i's bitmaps travel while batch i+1 is partitioned), the
    # prefix-OR on a side stream of a second context
    pipelined = prefix and (world > 1 or two_phase)
    side_ctx = None
    if prefix:
        side_st = side = None
        if pipelined:
            side = torch.cuda.Stream()
            side_ctx = Context(ctx.device)
            with torch.cuda.stream(side):
                side_st = HipStages(side_ctx)
        tri = PrefixTriage(HipStages(ctx), Comm(), two_phase_at_one=two_phase, side_stages=side_st, side_stream=side,
                           form=getattr(args, "c3_form", "auto"), exchange=getattr(args, "c3_exchange", "auto"))
    else:
        tri = ShardedTriage(HipStages(ctx), Comm())
    forms = []  # the prefix protocol's step-1 form per batch
    xchg = []   # its exchange form and bytes per rank, per batch (warm-up batches included)
    rec_base = rank * nprog * calls
    nrec_total = world * nprog * calls
    # every step runs against the restored snapshot: overlapped steps use a
    # maxSignal (and flag buffer) each
    maxsigs = [maxsig, SignalSet(ctx)] if pipelined else [maxsig]
    rec_news = [rec_new, torch.empty_like(rec_new)] if pipelined else [rec_new]

    def run(bs, states=None):
        pend = None
        for i, b in enumerate(bs):
            if states is None:
                ms = maxsigs[i % len(maxsigs)]
                call("sg_set_copy", ms.h, m0set.h)
            else:
                ms = states[i]
            if not pipelined:
                tri.step(ms, newsig, b.vals, b.off, b.nvals, b.nrec, rec_base, rec_new)
                if prefix:
                    xchg.append((tri.last.get("exchange", "local"), tri.last.get("exchange_bytes", 0)))
                continue
            p = tri.start(ms, newsig, b.vals, b.off, b.nvals, b.nrec, rec_base, rec_news[i % 2], nrec_total)
            if prefix:
                forms.append(p["last"].get("form"))
                xchg.append((p["last"].get("exchange", "local"), p["last"].get("exchange_bytes", 0)))
            if pend is not None:
                tri.finish(pend)
            pend = p
        if pend is not None:
            tri.finish(pend)

    run(batches[: args.warmup])
    torch.cuda.synchronize()
    timed = batches[args.warmup:]
    # each timed step against its own copy of the snapshot, made before the
    # timed region (the state reset is not part of the reference's step)
    states = [maxsig] + [SignalSet(ctx) for _ in timed[1:]]
    for st in states:
        call("sg_set_copy", st.h, m0set.h)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.timing(True)
    if side_ctx is not None:
        side_ctx.timing(True)
    call("sg_ctx_marker", ctx.h, 0, 4)  # the timed region, for kernel traces / PMC passes (workload "c3")
    t0 = time.perf_counter()
    run(timed, states)
    call("sg_ctx_marker", ctx.h, 1, 4)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    for st in states[1:]:
        st.close()
    kernels = kernel_table(ctx, SHARD_KERNELS, args.steps)
    if side_ctx is not None:
        side_kernels = kernel_table(side_ctx, ["prefix_or"], args.steps)
        if "prefix_or" in side_kernels:
            kernels["prefix_or"] = side_kernels["prefix_or"]
        side_ctx.timing(False)
    ctx.timing(False)
    wall = _max_over_ranks(wall, world)
    units = _sum_over_ranks(sum(b.nvals for b in timed), world)
    # accounting, outside the timed region: first timed batch
    b = timed[0]
    call("sg_set_copy", maxsig.h, m0set.h)
    import ctypes
    c = ctypes.c_uint64()
    call("sg_set_count_missing_dev", maxsig.h, b.vals.data_ptr(), b.nvals, ctypes.byref(c))
    tri.step(maxsig, None, b.vals, b.off, b.nvals, b.nrec, rec_base, rec_new)
    torch.cuda.synchronize()
    last = dict(tri.last)
    # the same batch's exchange in both forms (the one it took and the other),
    # from the counts every rank gathered with it
    xmodel = tri.exchange_model() if prefix else None
    queued = int(rec_new[: b.nrec].sum().item())
    acct_rank = {"n_in": b.nvals, "n_uniq": n_uniq(b, calls), "n_cand": c.value, "n_rec": b.nrec,
                 "n_queued": queued, "pairs_sent": last.get("pairs_sent", 0),
                 "pairs_received": last.get("pairs_received", 0)}
    acct = {k: _sum_over_ranks(v, world) for k, v in acct_rank.items()}
    after = len(maxsig)
    new_signal = last["new_signal"] if "new_signal" in last else after - m0_count
    acct["n_new_signal"] = new_signal
    acct["n_diff"] = new_signal  # diff multiplicity not emitted by the sharded path
    acct["queued_frac"] = acct["n_queued"] / acct["n_rec"] if acct["n_rec"] else None
    acct["maxsignal_after"] = after
    acct["consistent"] = after == m0_count + new_signal
    ms_step = wall * 1e3 / args.steps
    # roofline: whole-job step bytes over all ranks / step time / aggregate peak
    bpr = step_bytes(acct) / world
    # HBM bytes of one rank's step: the PMC section of the per-rank work (the
    # two-phase prefix step measured at one rank, profiles/pmc_traffic.json "c3")
    pmc_names = [k for k in kernels if k not in ("scan", "bucket_spill", "set_add")]
    # (measured at the default 128Ki programs per rank: another size has no section)
    traffic, ttag = pmc_bytes_per_step(pmc_names, "c3") if prefix and nprog == 131072 else (None, None)
    roof = {"bound": "hbm", "achieved": round(bpr / (ms_step / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(bpr / (ms_step / 1e3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
            "scope": "whole sharded step per GPU (wall clock, max over ranks; exchanges included)",
            "algo_bytes_per_step_per_gpu": bpr,
            "formula": "SURVEY.md §8(d) C2/C3 bytes over all ranks / N (N_out taken as the new-signal count)",
            "traffic_source": (f"profiles/pmc_traffic.json ({ttag}): FETCH_SIZE/WRITE_SIZE of one rank's two-phase "
                               f"prefix step (bench.py --mode c3 --c3-two-phase at one rank, 128Ki programs), summed "
                               f"over its kernels; RCCL traffic not included" if traffic is not None else None),
            "traffic_over_algo": round(traffic / bpr, 3) if traffic else None}
    cpu = None
    if not getattr(args, "no_cpu", False):
        # rank 0's records come first in the batch's record order: its flags
        # are the sequential loop's over its own slice against the snapshot,
        # which the oracle reproduces on a bounded prefix of that slice
        if rank == 0:
            gpu_flags = rec_new[: b.nrec].cpu().numpy()
            cpu = cpu_baseline(m0set.export(), b, calls, gpu_flags, args.cpu_budget / 2, args.cpu_threads)
            cpu["sample"] = "rank 0's slice: " + cpu["sample"]
        if world > 1:
            dist.barrier()
    if prefix:
        # per exchange form, the mean bytes a rank sent per step (dense: bitmaps
        # whatever the novelty; sparse: the candidate lists)
        by = {}
        for f, nb in xchg:
            by.setdefault(f, []).append(nb)
        xgmi = {f: sum(v) / len(v) for f, v in by.items()}
    else:
        xgmi = 8 * acct["pairs_sent"] / world + 4 * (acct["n_rec"] / 32) / world + 4 * last["new_signal"]
    if rank != 0:
        return None
    return {
        "metric": METRIC,
        "value": units / wall,
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
            "workload": f"C3 recipe: one batch of {world} x {nprog} programs x {calls} calls x {cfg['pcs_per_call']} "
                        f"Zipf PCs (N=8: C3's 1Mi programs), records split contiguously, {nprog} programs "
                        f"({nprog * calls} call records) per rank; one sequential triage loop over the whole batch, "
                        + ("by bitmap prefixes (local new signal, RCCL all-to-all of bitmap slices and exclusive "
                           "prefix-OR, local triage against maxSignal | prefix)" if prefix else
                           "hash-sharded by signal (RCCL all-to-all of candidates, OR of record-flag slices, "
                           "all-gather of new signal)")
                        + f" vs a replicated {m0_count}-entry maxSignal (each step against its own copy of it)",
            "programs_per_gpu": nprog, "batch_programs": world * nprog, "calls": calls,
            "pcs_per_call": cfg["pcs_per_call"], "signal_per_step": units / args.steps,
            "maxsignal_start": m0_count, "queued_frac": acct["queued_frac"],
            "parallelism": (f"record-sliced x{world}, bitmap-prefix exchange"
                            + (" overlapped with the next batch's partition" if pipelined else "") if prefix else
                            f"signal-sharded x{world}") + " (one rank per GPU, RCCL)",
        },
        "roofline": roof,
        "cpu_baseline": cpu,
        "kernels": kernels,
        "accounting": acct,
        "exchange_bytes_per_rank_per_step": xgmi,
        "exchange_bytes_by_form_first_batch": xmodel,
        # the exchange time model of DESIGN.md §5 at this world size and at G = 8
        # (the node the driver's scaling run uses), for checking measured N > 1 steps
        "predicted_exchange_ms": ({str(g): exchange_time_model(g, gather=tri.gather if g == world else None,
                                                               cand_max=(xmodel or {}).get("candidates_max"))
                                   for g in sorted({world, 8})} if prefix else None),
        "prefix_forms": forms[-args.steps:] if prefix and forms else None,
        "exchange_forms": [f for f, _ in xchg[-args.steps:]] if prefix else None,
        "path": ("prefix (syzkaller_amd/shard.py PrefixTriage)" if prefix else
                 "sharded (syzkaller_amd/shard.py ShardedTriage + sg_shard.hip)"),
        "gen_s": round(t_gen, 2),
    }


class Poll:
    """newSignal drain + manager merge (fuzzer.go:358-364, manager.go:949-962,
    fuzzer.go:392-398) between independent per-GPU fuzzers: every rank's
    maxSignal gains every other rank's new signal, as an OR-exchange of the
    newSignal bitmaps (syzkaller_amd/dist.py), one step behind on its own
    stream (the reference polls asynchronously, fuzzer.go:331-346)."""

    def __init__(self, ctx, world):
        import ctypes
        from syzkaller_amd.dist import OrExchange
        from syzkaller_amd._lib import lib

        self.lib = lib
        self.bufs = [torch.zeros(U32_WORDS, dtype=torch.int32, device="cuda") for _ in range(2)]
        self.sets = []
        for buf in self.bufs:
            h = ctypes.c_void_p()
            call("sg_set_wrap_dev", ctx.h, buf.data_ptr(), ctypes.byref(h))
            self.sets.append(h)
        self.k = 0
        self.comm = torch.cuda.Stream()
        self.ex = [OrExchange(buf) for buf in self.bufs]
        self.merged = [None, None]
        self.done = [None, None]

    def newsig(self):
        class _H:
            pass
        h = _H()
        h.h = self.sets[self.k % 2]
        return h

    def after_triage(self, maxsig):
        slot = self.k % 2
        self.k += 1
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(ev)
            merged = self.ex[slot](self.bufs[slot])
            done = torch.cuda.Event()
            done.record(self.comm)
        self.merged[slot], self.done[slot] = merged, done
        self._apply(self.k % 2, maxsig)

    def _apply(self, slot, maxsig):
        if self.done[slot] is None:
            return
        torch.cuda.current_stream().wait_event(self.done[slot])
        call("sg_set_or_dev", maxsig.h, self.merged[slot].data_ptr())  # fuzzer.go:392-398
        self.bufs[slot].zero_()
        self.done[slot] = None

    def drain(self, maxsig):
        for d in (1, 0):
            self._apply((self.k + d) % 2, maxsig)

    def close(self):
        for h in self.sets:
            self.lib.sg_set_destroy(h)


def run_fuzzers(ctx, args, cfg, rank, world):
    calls = cfg["calls"]
    g = Gen(cfg)
    warm = g.zipf(ctx, cfg, 2_000_000 + rank)
    batches = [g.zipf(ctx, cfg, 1_000 + 100_000 * rank + k) for k in range(args.warmup + args.steps)]
    del g
    rec_new = torch.empty(max(b.nrec for b in batches), dtype=torch.uint8, device="cuda")
    maxsig = SignalSet(ctx)
    build_m0(ctx, maxsig, warm, calls, args.m0, rec_new)
    del warm
    poll = Poll(ctx, world)
    for b in batches[: args.warmup]:
        triage(ctx, maxsig, poll.newsig(), b, rec_new)
        poll.after_triage(maxsig)
    poll.drain(maxsig)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for b in batches[args.warmup:]:
        triage(ctx, maxsig, poll.newsig(), b, rec_new)
        poll.after_triage(maxsig)
    poll.drain(maxsig)
    torch.cuda.synchronize()
    dist.barrier()
    wall = _max_over_ranks(time.perf_counter() - t0, world)
    units = _sum_over_ranks(sum(b.nvals for b in batches[args.warmup:]), world)
    poll.close()
    if rank != 0:
        return None
    return {"metric": METRIC, "value": units / wall, "unit": "PCs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": wall * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": "fuzzers: one independent C2 fuzzer per GPU, Poll as an RCCL OR-exchange of "
                                   "newSignal bitmaps (maxSignal grows across steps)",
                       "programs_per_gpu": cfg["programs"], "parallelism": f"independent fuzzers x{world}"},
            "roofline": None, "cpu_baseline": None, "path": "partitioned per rank + OR-exchange"}
