#!/usr/bin/env python3
"""bench.py -- coverage PCs triaged per second on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch: syz-fuzzer/fuzzer.go:645-693
execute() for every call record of the batch (the new-signal test, per-record
attribution, the maxSignal / newSignal update), against a maxSignal that holds
the configuration's starting signal.

Workloads (BASELINE.json configs):
  C2 (default at N=1, the metric's configuration): per GPU 64Ki programs x 16
     calls x 1024 synthetic Zipf(1.1) PCs over 2^20 ranks (pc = 0x81000000 +
     16*perm(rank)), turned into per-call signal by the executor-exact edge /
     dedup kernel (executor/executor.h:389-401, :497-526), triaged against a
     16M-entry maxSignal bitmap.  Every timed step triages against its own
     copy of the 16M-entry state, made before the timed region (the state
     reset is not part of the reference's step), so every timed step runs
     against the stated maxSignal.  Each step triages a fresh batch.
  from traces (N=1, reported under "from_traces"): C2 end to end -- the timed
     step also runs the executor signal kernels over the batch's raw PC traces
     (resident in HBM), then triages what they produce.
  steady (N=1, reported under "steady_state"): the fuzzer's low-novelty steady
     state -- programs drawn from a fixed population of --npop programs,
     re-executed with flaky coverage (each PC replaced by a fresh draw with
     probability --noise), against maxSignal = the population's signal.  The
     flags path runs in its default auto regime, which takes these batches
     through the M0 filter ("m0_filter" counts the slices).
  C3 (default at N>1): one batch of 128Ki programs per rank (the C2 recipe;
     N=8 is C3's 1Mi-program batch) triaged as ONE sequential loop over the
     whole batch, hash-sharded by signal across the ranks (syzkaller_amd/shard.py:
     replicated maxSignal snapshot, candidates routed to their owning shard
     with RCCL all-to-all, first owners there, record flags OR-reduced back).
  fuzzers (--mode fuzzers): one independent fuzzer per GPU with the Poll
     merge as an RCCL OR-exchange of newSignal bitmaps (the round-1 mode).

All inputs are generated on the GPU and resident in HBM before the timed
region.  value = all signal entries triaged by all ranks / max-over-ranks time.

Run:  python bench.py [--gpus N --steps K --warmup W]
      N>1 either under a launcher that sets RANK / LOCAL_RANK / WORLD_SIZE /
      MASTER_* (python -m torch.distributed.run --nproc-per-node N ... bench.py
      --gpus N), or plain: without WORLD_SIZE, `--gpus N` starts the N rank
      processes itself (spawn_ranks: the parent makes no GPU call, prints rank
      0's line and exits non-zero when any rank fails).
"""
import argparse
import ctypes
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _gpus_arg(argv):
    """--gpus N / --gpus=N from argv (1 when absent)."""
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            return int(argv[i + 1])
        if a.startswith("--gpus="):
            return int(a.split("=", 1)[1])
    return 1


def spawn_ranks(n, argv, poll_s=0.2, script=None):
    """`bench.py --gpus N` without a launcher: start N fresh rank processes of
    this script (RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1,
    a free MASTER_PORT), as children, never by exec.  This process touches no
    GPU (it has imported neither torch nor the library).  Rank 0's stdout is
    this process's stdout: it prints the one JSON line.  When a rank fails the
    others are stopped (they would wait in a collective) and its exit status is
    returned; 0 when all succeed."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    try:
        while any([p.poll() is None for p in procs]):  # (a list: poll every rank)
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            time.sleep(poll_s)
        else:
            bad = [p.returncode for p in procs if p.returncode != 0]
            rc = bad[0] if bad else 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if rc:
        print(f"bench.py: a rank failed (exit status {rc})", file=sys.stderr)
    return rc if rc > 0 else (1 if rc else 0)


if __name__ == "__main__" and "WORLD_SIZE" not in os.environ and _gpus_arg(sys.argv[1:]) > 1:
    sys.exit(spawn_ranks(_gpus_arg(sys.argv[1:]), sys.argv[1:]))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from syzkaller_amd import _lib  # noqa: E402,F401  (fails loudly without libsyzsig.so)
from syzkaller_amd._lib import call, lib  # noqa: E402
from syzkaller_amd.cover import Context, SignalSet  # noqa: E402

METRIC = "coverage PCs triaged/sec vs corpus signal (+ % HBM roofline), 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
U32_WORDS = 1 << 27     # 2^32-bit signal bitmap
UNIVERSE_SEED = 0x5A17C0DE
POP_SEED = 0x9091A7E5

# kernels of one partitioned triage step (sg_bucket.hip), for the per-kernel table
STEP_KERNELS = ["p1_hist", "p1_scatter", "p2_hist", "p2_scatter", "bucket_triage", "bucket_spill", "scan",
                "m0_index", "m0_filter", "m0_tail"]
ORDERED_KERNELS = ["owned_sort", "owned_sweep", "emit"]
OTHER_KERNELS = ["emit", "shard_local", "shard_route", "shard_owner",
                 "shard_resolve", "shard_flags", "set_add"]


class Batch:
    def __init__(self, vals, off, nvals, nrec, seed):
        self.vals, self.off, self.nvals, self.nrec, self.seed = vals, off, nvals, nrec, seed


class Gen:
    """Trace generation buffers (freed once the batches exist)."""

    def __init__(self, cfg):
        nprog, calls, pcs = cfg["programs"], cfg["calls"], cfg["pcs_per_call"]
        self.ncalls, self.npcs = nprog * calls, nprog * calls * pcs
        self.trace = torch.empty(self.npcs, dtype=torch.int32, device="cuda")
        self.sig = torch.empty(self.npcs, dtype=torch.int32, device="cuda")
        self.call_off = torch.arange(0, self.npcs + 1, pcs, dtype=torch.int64, device="cuda")
        self.prog_off = torch.arange(0, self.ncalls + 1, calls, dtype=torch.int64, device="cuda")

    def signal(self, ctx, cfg, seed):
        """traces in self.trace -> executor signal (CSR), a resident Batch."""
        sig_off = torch.empty(self.ncalls + 1, dtype=torch.int64, device="cuda")
        call("sg_exec_signal_dev", ctx.h, self.trace.data_ptr(), self.call_off.data_ptr(), self.prog_off.data_ptr(),
             cfg["programs"], self.ncalls, self.npcs, self.sig.data_ptr(), sig_off.data_ptr())
        torch.cuda.synchronize()
        nvals = int(sig_off[-1].item())
        return Batch(self.sig[:nvals].clone(), sig_off, nvals, self.ncalls, seed)

    def zipf(self, ctx, cfg, seed, prog_base=0):
        """Programs prog_base .. prog_base + programs - 1 of the batch `seed`."""
        call("sg_gen_zipf_traces_dev", ctx.h, UNIVERSE_SEED, seed, cfg["zipf_s"], cfg["ranks"], prog_base,
             cfg["programs"], cfg["calls"], cfg["pcs_per_call"], self.trace.data_ptr())
        return self.signal(ctx, cfg, seed)

    def population(self, ctx, cfg, seed, npop, noise, prog_base=0):
        call("sg_gen_population_traces_dev", ctx.h, UNIVERSE_SEED, POP_SEED, npop, seed, noise, cfg["zipf_s"],
             cfg["ranks"], prog_base, cfg["programs"], cfg["calls"], cfg["pcs_per_call"], self.trace.data_ptr())
        return self.signal(ctx, cfg, seed)

    def members(self, ctx, cfg, m0, m1):
        """Population members m0 .. m1-1 executed exactly (no noise)."""
        sub = dict(cfg, programs=m1 - m0)
        call("sg_gen_zipf_traces_dev", ctx.h, UNIVERSE_SEED, POP_SEED, cfg["zipf_s"], cfg["ranks"], m0, m1 - m0,
             cfg["calls"], cfg["pcs_per_call"], self.trace.data_ptr())
        ncalls, npcs = sub["programs"] * cfg["calls"], sub["programs"] * cfg["calls"] * cfg["pcs_per_call"]
        sig_off = torch.empty(ncalls + 1, dtype=torch.int64, device="cuda")
        call("sg_exec_signal_dev", ctx.h, self.trace.data_ptr(), self.call_off.data_ptr(), self.prog_off.data_ptr(),
             sub["programs"], ncalls, npcs, self.sig.data_ptr(), sig_off.data_ptr())
        torch.cuda.synchronize()
        nvals = int(sig_off[-1].item())
        return Batch(self.sig[:nvals], sig_off, nvals, ncalls, None)


def triage(ctx, maxsig, newsig, b, rec_new, diff_vals=None, diff_off=None, rec0=0, rec1=None, e0=0, e1=None):
    """fuzzer.go:645-693 over one batch (or records [rec0, rec1) of it).
    Without diff buffers: the partitioned path (flags + set updates); with:
    the ordered-output path, which also emits the diff lists (fuzzer.go:669)."""
    if rec1 is None:
        rec1, e1 = b.nrec, b.nvals
        vals, off = b.vals, b.off
    else:
        vals, off = b.vals[e0:e1], (b.off[rec0:rec1 + 1] - e0).contiguous()
    call("sg_triage_batch_dev", ctx.h, maxsig.h, newsig.h if newsig is not None else None, vals.data_ptr(),
         off.data_ptr(), e1 - e0, rec1 - rec0, rec_new.data_ptr(),
         diff_vals.data_ptr() if diff_vals is not None else None, diff_off.data_ptr() if diff_off is not None else None)


def build_m0(ctx, maxsig, batch, calls, target, rec_new, chunk_prog=256):
    """maxSignal <- the warm batch's signal, program chunk by program chunk,
    until it holds >= target entries."""
    off = batch.off.cpu().numpy()
    nprog = batch.nrec // calls
    p = 0
    while p < nprog and len(maxsig) < target:
        p1 = min(nprog, p + chunk_prog)
        triage(ctx, maxsig, None, batch, rec_new, rec0=p * calls, rec1=p1 * calls, e0=int(off[p * calls]),
               e1=int(off[p1 * calls]))
        p = p1
    torch.cuda.synchronize()


def n_uniq(batch, calls, chunk_prog=4096):
    """N_uniq of SURVEY.md §8(d): program-distinct signal entries (one bitmap
    probe per distinct signal of a program), counted exactly on the GPU."""
    off = batch.off
    nprog = batch.nrec // calls
    total = 0
    prog_of_rec = torch.arange(batch.nrec, device="cuda", dtype=torch.int64) // calls
    lens = off[1:] - off[:-1]
    for p0 in range(0, nprog, chunk_prog):
        p1 = min(nprog, p0 + chunk_prog)
        r0, r1 = p0 * calls, p1 * calls
        e0, e1 = int(off[r0].item()), int(off[r1].item())
        if e1 == e0:
            continue
        pid = torch.repeat_interleave(prog_of_rec[r0:r1], lens[r0:r1], output_size=e1 - e0)
        keys = (pid << 32) | (batch.vals[e0:e1].to(torch.int64) & 0xFFFFFFFF)
        total += int(torch.unique(keys).numel())
    return total


def step_bytes(a):
    """SURVEY.md §8(d) algorithmic bytes of one C2/C3 step: 4 N_in (signal read)
    + 4 N_uniq (a bitmap-word probe per program-distinct signal) + 8 N_cand
    (first-owner RMW for s not in maxSignal) + 4 N_cand (owner re-read) + 4 N_out
    (diff elements) + N_rec / 8 (flag bits)."""
    return 4 * a["n_in"] + 4 * a["n_uniq"] + 12 * a["n_cand"] + 4 * a["n_diff"] + a["n_rec"] / 8


def pmc_bytes_per_step(kernels, workload, minor=()):
    """HBM bytes per step of `workload` ("c2", "steady", "from_traces") from the
    PMC summary committed under profiles/ (separate FETCH_SIZE / WRITE_SIZE
    passes over that workload's own timed launches, gfx950-corrected), summed
    over the step's kernels, or None when the summary holds no measurement of
    this workload or of another kernel set.  `minor`: kernels that ran in the
    timed steps but under 5 % of their time (the M0 filter's probe of a fresh
    batch, one record slice in 16), skipped when the summary lacks them."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            d = json.load(f)
    except Exception:
        return None, None
    w = d.get("workloads", {}).get(workload)
    if not w:
        return None, None
    per = w.get("kernels", {})
    tot, seen = 0.0, []
    for k in kernels:
        if k in per and per[k].get("hbm_bytes_per_launch") is not None:
            tot += per[k]["hbm_bytes_per_launch"] * per[k].get("launches_per_step", 1)
            seen.append(k)
        elif k not in ("scan", "bucket_spill") and k not in minor:  # a summary of another kernel set: stale
            return None, None
    return (tot if seen else None), f"{w.get('tag', d.get('tag'))}/{workload}"


class StepTimer:
    """HIP events on the launch stream around each step's triage."""

    def __init__(self):
        self.ev = []

    def mark(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.ev.append(e)

    def spans(self):
        torch.cuda.synchronize()
        return [self.ev[i].elapsed_time(self.ev[i + 1]) for i in range(len(self.ev) - 1)]


def cpu_quota():
    """CPUs the cgroup lets this process use (cpu.max quota / period), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        return None


def cpu_info():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return model, os.cpu_count(), avail


def cpu_baseline(m0_values, batch, calls, gpu_flags, budget_s, threads, threads_nproc=None):
    """The oracle on a bounded prefix of one batch, from the same starting
    maxSignal: (i) single-threaded, the reference's per-exec structure
    (fuzzer.go:661-691 under signalMu), with a parity check against the GPU's
    flags for the same records; (ii) `threads` procs sharing the maps under a
    reader-writer lock (fuzzer.go:248-327, :661-676).  C restatement of the Go
    reference (oracle/sigoracle.c, Go maps mirrored by open-addressing hash
    sets), not Go: no Go toolchain exists in this image."""
    from oracle import pyoracle as O

    off = batch.off.cpu().numpy().astype(np.uint64)
    nprog = batch.nrec // calls
    t0 = time.perf_counter()
    ms = O.OSet(m0_values)
    build_s = time.perf_counter() - t0
    done_prog, elapsed, nel = 0, 0.0, 0
    flags = []
    chunk = 16
    while done_prog < nprog and elapsed < budget_s:
        p1 = min(nprog, done_prog + chunk)
        r0, r1 = done_prog * calls, p1 * calls
        e0, e1 = int(off[r0]), int(off[r1])
        v = batch.vals[e0:e1].cpu().numpy().view(np.uint32)
        o = (off[r0:r1 + 1] - off[r0]).astype(np.uint64)
        t = time.perf_counter()
        f = O.triage_flags_only(ms, None, v, o)
        elapsed += time.perf_counter() - t
        flags.append(f)
        nel += e1 - e0
        done_prog = p1
        if elapsed > 0:
            chunk = max(16, int(done_prog * (budget_s / elapsed) - done_prog) // 4)
    flags = np.concatenate(flags) if flags else np.zeros(0, np.uint8)
    parity = bool(np.array_equal(flags, gpu_flags[: flags.size])) if gpu_flags is not None else None
    queued_frac = float(flags.mean()) if flags.size else None
    del ms
    # (ii) the same prefix with P procs under the reader-writer lock: P =
    # `threads` (the box's CPU share) and P = nproc (SURVEY.md §8(d) leg (ii))
    e1 = int(off[done_prog * calls])
    v = batch.vals[:e1].cpu().numpy().view(np.uint32)
    o = off[: done_prog * calls + 1].astype(np.uint64)
    pr = np.arange(0, done_prog * calls + 1, calls, dtype=np.uint64)

    def procs_leg(p):
        ms_ = O.OSet(m0_values)
        t_ = time.perf_counter()
        _, used_ = O.triage_procs(ms_, None, v, o, pr, p)
        return time.perf_counter() - t_, used_

    mt_s, used = procs_leg(threads)
    legs_n = procs_leg(threads_nproc) if threads_nproc and threads_nproc != threads else None
    model, ncpu, avail = cpu_info()
    structure = ("procs taking whole programs, maps under one pthread rwlock with the RLock->Lock upgrade of "
                 "fuzzer.go:671-676 (racy, as the reference)")
    sample = (f"first {done_prog} programs ({done_prog * calls} call records, {nel} signal entries) of the first "
              f"timed batch vs the same {len(m0_values)}-entry maxSignal; C restatement of the Go reference "
              f"(oracle/sigoracle.c, Go maps mirrored by open-addressing hash sets), not Go; set build "
              f"{build_s:.1f}s excluded")
    return {
        "value": nel / elapsed if elapsed else None,
        "unit": "PCs/s",
        "cores": 1,
        "kind": "port",
        "sample": sample,
        "prefix_parity_vs_gpu": parity,
        "prefix_queued_frac": queued_frac,
        "all_cores": {"value": nel / mt_s if mt_s else None, "unit": "PCs/s", "cores": used,
                      "threads_used": used, "structure": structure},
        "all_cores_nproc": ({"value": nel / legs_n[0] if legs_n[0] else None, "unit": "PCs/s", "cores": legs_n[1],
                             "threads_used": legs_n[1], "structure": structure,
                             "note": "P = nproc threads; the cgroup CPU quota (host.cpu_quota) bounds how many run "
                                     "at once"} if legs_n else None),
        "host": {"cpu_model": model, "nproc": ncpu, "cpus_available": avail, "cpu_quota": cpu_quota()},
    }


def account(ctx, maxsig, m0set, newsig, batches, calls, rec_new, diff_vals, diff_off):
    """Outside the timed region: replay the timed steps from the same state,
    on the ordered-output path (so the diff element count is known), with the
    candidate and program-distinct counts measured."""
    tot = dict(n_in=0, n_uniq=0, n_cand=0, n_diff=0, n_rec=0, n_new_signal=0, n_queued=0)
    flags_eq = True
    for b in batches:
        call("sg_set_copy", maxsig.h, m0set.h)
        c = ctypes.c_uint64()
        call("sg_set_count_missing_dev", maxsig.h, b.vals.data_ptr(), b.nvals, ctypes.byref(c))
        m_before = len(maxsig)
        triage(ctx, maxsig, newsig, b, rec_new)
        torch.cuda.synchronize()
        fl = rec_new[: b.nrec].clone()
        call("sg_set_copy", maxsig.h, m0set.h)
        triage(ctx, maxsig, newsig, b, rec_new, diff_vals, diff_off)
        torch.cuda.synchronize()
        flags_eq &= bool(torch.equal(fl, rec_new[: b.nrec]))
        tot["n_diff"] += int(diff_off[b.nrec].item())
        tot["n_queued"] += int(rec_new[: b.nrec].sum().item())
        tot["n_new_signal"] += len(maxsig) - m_before
        tot["n_in"] += b.nvals
        tot["n_uniq"] += n_uniq(b, calls)
        tot["n_cand"] += c.value
        tot["n_rec"] += b.nrec
    L = len(batches)
    per = {k: v / L for k, v in tot.items()}
    per["queued_frac"] = tot["n_queued"] / tot["n_rec"] if tot["n_rec"] else None
    per["paths_agree"] = flags_eq  # flags-only path == ordered-output path's flags on every timed batch
    return per


def timed_steps(ctx, maxsig, m0set, newsig, batches, rec_new, world, tag=1):
    """K steps, each triaging its batch against its own copy of the starting
    maxSignal (made before the timed region: the state reset is not part of
    the reference's step, fuzzer.go:645-693).  maxsig ends as step 0's copy
    after step 0.  Returns (wall seconds, per-step triage ms)."""
    tm = StepTimer()
    states = [maxsig] + [SignalSet(ctx) for _ in batches[1:]]
    for st in states:
        call("sg_set_copy", st.h, m0set.h)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.timing(True)
    call("sg_ctx_marker", ctx.h, 0, tag)  # the timed region, for kernel traces (scripts/trace_summary.py, pmc_summary.py)
    t0 = time.perf_counter()
    for st, b in zip(states, batches):
        tm.mark()
        triage(ctx, st, newsig, b, rec_new)
        tm.mark()
    call("sg_ctx_marker", ctx.h, 1, tag)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    tri = [tm.ev[i].elapsed_time(tm.ev[i + 1]) for i in range(0, len(tm.ev), 2)]
    for st in states[1:]:
        st.close()
    return wall, tri


def timed_steps_pipelined(ctx, m0set, newsig, batches, flags0):
    """The timed steps through syzkaller_amd/pipeline.py: step i+1's partition
    on a second stream beside step i's bucket stage (bucket stages in step
    order, each step against its own copy of the starting maxSignal, as in
    timed_steps).  Every step's flags are checked against the sequential path
    outside the timed region; flags0 = step 0's from timed_steps."""
    from syzkaller_amd.pipeline import PipelinedTriage

    states = [SignalSet(ctx) for _ in batches]
    for st in states:
        call("sg_set_copy", st.h, m0set.h)
    flags = [torch.empty(b.nrec, dtype=torch.uint8, device="cuda") for b in batches]
    pt = PipelinedTriage(ctx)
    for st, b, f in zip(states[:2], batches[:2], flags[:2]):  # warm: both slots' workspaces
        pt.submit(st, newsig, b.vals, b.off, b.nvals, b.nrec, f)
    for st in states[:2]:
        call("sg_set_copy", st.h, m0set.h)
    torch.cuda.synchronize()
    call("sg_ctx_marker", ctx.h, 0, 5)
    t0 = time.perf_counter()
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for st, b, f in zip(states, batches, flags):
        pt.submit(st, newsig, b.vals, b.off, b.nvals, b.nrec, f)
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record()
    call("sg_ctx_marker", ctx.h, 1, 5)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    pt.close()
    ok = bool(np.array_equal(flags[0].cpu().numpy(), flags0))
    rec_new = torch.empty(max(b.nrec for b in batches), dtype=torch.uint8, device="cuda")
    for b, f in zip(batches[1:], flags[1:]):  # the sequential path, outside the timed region
        call("sg_set_copy", states[0].h, m0set.h)
        triage(ctx, states[0], None, b, rec_new)
        ok = ok and bool(torch.equal(rec_new[: b.nrec], f))
    counts = {len(st) for st in states[1:]}
    for st in states:
        st.close()
    ms = e0.elapsed_time(e1) / len(batches)
    return {"ms_per_step": round(ms, 4), "wall_ms_per_step": round(wall * 1e3 / len(batches), 4),
            "flags_equal_sequential": ok, "steps": len(batches),
            "how": "syzkaller_amd/pipeline.py: step i+1's partition (sg_prefix_begin_form_dev form 2) on a second "
                   "stream beside step i's bucket stage (sg_prefix_end_dev), the bucket stages in step order",
            "state_sizes_after": sorted(counts)}


def timed_ordered(ctx, maxsig, m0set, newsig, batches, rec_new, diff_vals, diff_off, flags_ms):
    """The C2 step with the ordered outputs (the per-record diff CSR of
    fuzzer.go:669 besides flags and set updates, sg_triage.hip
    owned_outputs), timed like timed_steps over the same batches from the
    same state, one untimed step first (its workspace)."""
    call("sg_set_copy", maxsig.h, m0set.h)
    triage(ctx, maxsig, newsig, batches[0], rec_new, diff_vals, diff_off)
    states = [maxsig] + [SignalSet(ctx) for _ in batches[1:]]
    for st in states:
        call("sg_set_copy", st.h, m0set.h)
    torch.cuda.synchronize()
    ctx.timing(True)
    tm = StepTimer()
    call("sg_ctx_marker", ctx.h, 0, 6)
    t0 = time.perf_counter()
    for st, b in zip(states, batches):
        tm.mark()
        triage(ctx, st, newsig, b, rec_new, diff_vals, diff_off)
        tm.mark()
    call("sg_ctx_marker", ctx.h, 1, 6)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kernels = kernel_table(ctx, STEP_KERNELS + ORDERED_KERNELS, len(batches))
    ctx.timing(False)
    tri = [tm.ev[i].elapsed_time(tm.ev[i + 1]) for i in range(0, len(tm.ev), 2)]
    for st in states[1:]:
        st.close()
    ms = float(np.mean(tri))
    return {"ms_per_step": round(ms, 4), "wall_ms_per_step": round(wall * 1e3 / len(batches), 4),
            "over_flags": round(ms / flags_ms, 3), "diff_elements_last_step": int(diff_off[batches[-1].nrec].item()),
            "kernels": kernels,
            "how": "sg_triage_batch_dev with diff_vals/diff_off: partition + update-emitting bucket stage (each new "
                   "signal with its first record), pairs radix-sorted by record, one wave per record sweeping S_r "
                   "against its owned signals into ballot masks, ordered compaction"}


def kernel_table(ctx, names, steps):
    out = {}
    for name in names:
        ms, n = ctx.kernel_time(name)
        if n:
            out[name] = {"ms_total": ms, "launches": n, "avg_ms": ms / n, "ms_per_step": ms / steps}
    return out


def roofline(acct, step_ms, kernels, workload="c2"):
    b = step_bytes(acct)
    ach = b / (step_ms / 1e3) / 1e9
    ran = [k for k in kernels if k in STEP_KERNELS] or STEP_KERNELS
    minor = [k for k in ran if kernels.get(k, {}).get("ms_per_step", 0) < 0.05 * step_ms]
    traffic, tag = pmc_bytes_per_step(ran, workload, minor)
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
            "scope": "whole triage step (all its kernels, HIP events on the launch stream)",
            "algo_bytes_per_step": b, "step_ms_events": step_ms,
            "formula": "4N_in + 4N_uniq + 8N_cand + 4N_cand + 4N_out + N_rec/8 (SURVEY.md §8(d), N_uniq measured)",
            "traffic_source": f"profiles/pmc_traffic.json ({tag}): FETCH_SIZE/WRITE_SIZE of this workload's timed "
                              f"launches, summed over the step's kernels" if traffic is not None else None,
            "traffic_over_algo": round(traffic / b, 3) if traffic else None}


def run_c2(ctx, args, cfg, rank):
    """C2 (and its steady-state companion) on one GPU."""
    calls = cfg["calls"]
    g = Gen(cfg)
    t_gen = time.perf_counter()
    warm = g.zipf(ctx, cfg, 2_000_000 + rank)
    batches = [g.zipf(ctx, cfg, 1_000 + 100_000 * rank + k) for k in range(args.warmup + args.steps)]
    t_gen = time.perf_counter() - t_gen
    maxnrec = max(b.nrec for b in batches)
    maxnvals = max(b.nvals for b in batches)
    rec_new = torch.empty(maxnrec, dtype=torch.uint8, device="cuda")
    maxsig, newsig, m0set = SignalSet(ctx), SignalSet(ctx), SignalSet(ctx)
    build_m0(ctx, m0set, warm, calls, args.m0, rec_new)
    m0_count = len(m0set)
    del warm
    for b in batches[: args.warmup]:  # untimed warm-up steps, same state
        call("sg_set_copy", maxsig.h, m0set.h)
        triage(ctx, maxsig, newsig, b, rec_new)
    torch.cuda.synchronize()
    gpu_flags0 = None
    timed = batches[args.warmup:]
    wall, tri = timed_steps(ctx, maxsig, m0set, newsig, timed, rec_new, 1)
    kernels = kernel_table(ctx, STEP_KERNELS + OTHER_KERNELS, args.steps)
    ctx.timing(False)
    call("sg_set_copy", maxsig.h, m0set.h)
    triage(ctx, maxsig, None, timed[0], rec_new)
    torch.cuda.synchronize()
    gpu_flags0 = rec_new[: timed[0].nrec].cpu().numpy()
    res = {"wall_s": wall, "triage_ms": float(np.mean(tri)),
           "m0": m0_count, "units": sum(b.nvals for b in timed), "kernels": kernels, "gen_s": round(t_gen, 2)}
    if not args.no_account:
        diff_vals = torch.empty(maxnvals, dtype=torch.int32, device="cuda")
        diff_off = torch.empty(maxnrec + 1, dtype=torch.int64, device="cuda")
        res["acct"] = account(ctx, maxsig, m0set, newsig, timed, calls, rec_new, diff_vals, diff_off)
        if args.ordered:
            res["ordered"] = timed_ordered(ctx, maxsig, m0set, newsig, timed, rec_new, diff_vals, diff_off,
                                           float(np.mean(tri)))
        del diff_vals, diff_off
    if not args.no_cpu:
        m0_values = m0set.export()
        res["cpu"] = cpu_baseline(m0_values, timed[0], calls, gpu_flags0, args.cpu_budget, args.cpu_threads,
                                  os.cpu_count())
    if args.pipeline:
        res["pipelined"] = timed_steps_pipelined(ctx, m0set, newsig, timed, gpu_flags0)
    if args.host_api:
        res["host_api"] = run_host_api(ctx, timed[0], maxsig, newsig, m0set, gpu_flags0)
    del batches, timed
    torch.cuda.empty_cache()
    if args.from_traces:
        res["from_traces"] = run_from_traces(ctx, args, cfg, g, maxsig, newsig, m0set, rec_new,
                                             min(args.steps, 4))
    if args.steady:
        res["steady"] = run_steady(ctx, args, cfg, g, maxsig, newsig, m0set, rec_new)
    return res


def pinned_h2d_gbs(nbytes=1 << 30, reps=3):
    """The box's host -> device DMA rate from pinned memory (the bound of any
    host entry point)."""
    src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    src.fill_(1)
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    best = 0.0
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, nbytes / (time.perf_counter() - t) / 1e9)
    del src, dst
    return best


def run_host_api(ctx, b, maxsig, newsig, m0set, gpu_flags, reps=3):
    """The drop-in host entry point (sg_triage_batch, flags + set updates) on
    one C2 batch handed over in pageable host memory, as the Go adapter hands
    it (the signal is born in host shm, pkg/ipc/ipc_linux.go:247): the
    pipelined ingest of sg_host.hip.  End to end, PCIe included; never `value`.
    The call's own stage rates come from the context's counters: the
    pageable -> pinned copies (GB/s over the copy threads' wall time) and the
    time the host waited for a staging slot's DMA; the default thread count
    (half the CPU quota) is timed beside 4 and 16 threads."""
    vals = b.vals.cpu().numpy().view(np.uint32).copy()
    off = b.off.cpu().numpy().view(np.uint64).copy()
    flags = np.zeros(b.nrec, dtype=np.uint8)
    nbytes = vals.nbytes + off.nbytes
    pinned = pinned_h2d_gbs()
    ok = True

    def leg(threads):
        nonlocal ok
        ctx.set_option("host_copy_threads", threads)
        best = None
        for _ in range(reps):
            call("sg_set_copy", maxsig.h, m0set.h)
            torch.cuda.synchronize()
            t = time.perf_counter()
            call("sg_triage_batch", ctx.h, maxsig.h, newsig.h, vals.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                 off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), b.nrec,
                 flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), None, None, None)
            t = time.perf_counter() - t
            ok &= bool(np.array_equal(flags, gpu_flags))
            c = {k: ctx.counter(k) for k in ("host_copy_bytes", "host_copy_ns", "host_wait_ns", "host_copy_threads")}
            if best is None or t < best[0]:
                best = (t, c)
        t, c = best
        return {"ms_per_batch": t * 1e3, "h2d_gbs": nbytes / t / 1e9, "frac_of_pinned_h2d": nbytes / t / 1e9 / pinned,
                "copy_threads": c["host_copy_threads"],
                "pageable_to_pinned_gbs": c["host_copy_bytes"] / max(c["host_copy_ns"], 1),
                "host_copy_ms": c["host_copy_ns"] / 1e6, "host_wait_dma_ms": c["host_wait_ns"] / 1e6}

    dflt = leg(0)
    sweep = {str(k): leg(k) for k in (4, 16) if k != dflt["copy_threads"]}
    ctx.set_option("host_copy_threads", 0)
    out = {"workload": f"C2 batch in pageable host memory ({b.nvals} signal entries, {nbytes / 1e9:.2f} GB with the "
                       "record offsets) through sg_triage_batch: record slices through pinned double-buffered "
                       "staging, each slice's copies overlapping the previous slice's triage (sg_host.hip)",
           "value": b.nvals / (dflt["ms_per_batch"] / 1e3), "unit": "PCs/s (PCIe-inclusive)"}
    out.update(dflt)
    out.update({"pinned_h2d_gbs": pinned, "cpu_quota": ctx.counter("cpu_quota_milli") / 1000.0,
                "flags_equal_device_path": ok, "reps": reps, "threads_sweep": sweep})
    return out


def run_from_traces(ctx, args, cfg, g, maxsig, newsig, m0set, rec_new, steps):
    """End to end from executor traces (C2's seeds, so the triage work is the
    timed C2 batches'): each timed step triages the batch's raw PC traces,
    resident in HBM, with sg_triage_traces_dev -- the set-exact front stage
    (edge signal computed in the partition's loads, executor.h:389-401) whose
    flags and set updates equal the executor-exact signal's (include/syzsig.h,
    tests/test_traces.py).  For comparison, the same steps through the
    executor-exact kernels (A0, executor.h:389-401 + :497-526) and then the
    triage of the signal they produce ("executor_exact")."""
    traces, offs = [], []
    for k in range(steps):
        call("sg_gen_zipf_traces_dev", ctx.h, UNIVERSE_SEED, 1_000 + args.warmup + k, cfg["zipf_s"], cfg["ranks"], 0,
             cfg["programs"], cfg["calls"], cfg["pcs_per_call"], g.trace.data_ptr())
        traces.append(g.trace.clone())
        offs.append(torch.empty(g.ncalls + 1, dtype=torch.int64, device="cuda"))
    torch.cuda.synchronize()
    ev = []

    def mark():
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.append(e)

    def step_set_exact(tr, st):
        mark()
        call("sg_triage_traces_dev", ctx.h, st.h, newsig.h, tr.data_ptr(), g.call_off.data_ptr(), g.npcs, g.ncalls,
             rec_new.data_ptr())
        mark()

    def step_exact(tr, so):
        call("sg_set_copy", maxsig.h, m0set.h)
        mark()
        call("sg_exec_signal_dev", ctx.h, tr.data_ptr(), g.call_off.data_ptr(), g.prog_off.data_ptr(),
             cfg["programs"], g.ncalls, g.npcs, g.sig.data_ptr(), so.data_ptr())
        mark()
        n = int(so[-1].item())  # the signal count, for the triage launch (8 bytes to the host)
        call("sg_triage_batch_dev", ctx.h, maxsig.h, newsig.h, g.sig.data_ptr(), so.data_ptr(), n, g.ncalls,
             rec_new.data_ptr(), None, None)
        mark()
        return n

    # set-exact (the product's trace path); each timed step against its own
    # copy of the starting maxSignal, made before the timed region (as C2's)
    call("sg_set_copy", maxsig.h, m0set.h)
    step_set_exact(traces[0], maxsig)  # warm-up
    states = [SignalSet(ctx) for _ in traces]
    for st in states:
        call("sg_set_copy", st.h, m0set.h)
    torch.cuda.synchronize()
    ev.clear()
    ctx.timing(True)
    torch.cuda.synchronize()
    call("sg_ctx_marker", ctx.h, 0, 3)
    t0 = time.perf_counter()
    for tr, st in zip(traces, states):
        step_set_exact(tr, st)
    call("sg_ctx_marker", ctx.h, 1, 3)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kernels = kernel_table(ctx, STEP_KERNELS, steps)
    ctx.timing(False)
    tri = [ev[i].elapsed_time(ev[i + 1]) for i in range(0, len(ev), 2)]
    for st in states:
        st.close()
    # executor-exact, for comparison
    ev.clear()
    step_exact(traces[0], offs[0])
    torch.cuda.synchronize()
    ev.clear()
    t1 = time.perf_counter()
    units = sum(step_exact(tr, so) for tr, so in zip(traces, offs))
    torch.cuda.synchronize()
    wall_x = time.perf_counter() - t1
    ex = [ev[i].elapsed_time(ev[i + 1]) for i in range(0, len(ev), 3)]
    tx = [ev[i + 1].elapsed_time(ev[i + 2]) for i in range(0, len(ev), 3)]
    roof, acct = None, None
    if not args.no_account:
        # the §8(d) bytes of the timed steps, with N_in = the raw PCs read: the
        # set-exact step's flags and set updates are the executor-exact
        # signal's, so N_uniq / N_cand / N_out are counted on that signal
        # (outside the timed region, each trace against the starting state)
        diff_vals = torch.empty(g.npcs, dtype=torch.int32, device="cuda")
        diff_off = torch.empty(g.ncalls + 1, dtype=torch.int64, device="cuda")
        per = []
        for tr, so in zip(traces, offs):
            call("sg_exec_signal_dev", ctx.h, tr.data_ptr(), g.call_off.data_ptr(), g.prog_off.data_ptr(),
                 cfg["programs"], g.ncalls, g.npcs, g.sig.data_ptr(), so.data_ptr())
            torch.cuda.synchronize()
            n = int(so[-1].item())
            b = Batch(g.sig[:n], so, n, g.ncalls, None)
            per.append(account(ctx, maxsig, m0set, newsig, [b], cfg["calls"], rec_new, diff_vals, diff_off))
        del diff_vals, diff_off
        acct = {k: float(np.mean([a[k] for a in per])) for k in per[0] if isinstance(per[0][k], (int, float))}
        acct["paths_agree"] = all(a["paths_agree"] for a in per)
        acct["n_signal"] = acct["n_in"]
        acct["n_in"] = float(g.npcs)  # the trace read: 4 bytes per raw PC
        roof = roofline(acct, float(np.mean(tri)), kernels, "from_traces")
        roof["formula"] = ("4N_in (raw PCs) + 4N_uniq + 8N_cand + 4N_cand + 4N_out + N_rec/8 (SURVEY.md §8(d); "
                           "N_uniq, N_cand, N_out counted on the executor-exact signal of the same traces)")
    del traces, offs
    torch.cuda.empty_cache()
    return {"workload": "C2 from traces: the timed step triages the batch's "
                        f"{g.npcs} resident raw PCs (sg_triage_traces_dev, set-exact edge signal in the partition's "
                        "loads), each step against its own copy of the starting maxSignal made before the timed "
                        "region",
            "value": g.npcs * steps / wall, "unit": "raw PCs/s", "ms_per_step": wall * 1e3 / steps, "steps": steps,
            "triage_ms_events": float(np.mean(tri)), "kernels": kernels, "roofline": roof, "accounting": acct,
            "executor_exact": {"value": g.npcs * steps / wall_x, "unit": "raw PCs/s",
                               "ms_per_step": wall_x * 1e3 / steps, "signal_per_step": units / steps,
                               "exec_ms_events": float(np.mean(ex)), "triage_ms_events": float(np.mean(tx)),
                               "path": "sg_exec_signal_dev (executor-exact per-call lists) + sg_triage_batch_dev"}}


def run_steady(ctx, args, cfg, g, maxsig, newsig, m0set, rec_new):
    """The low-novelty steady state: a fixed population re-executed with flaky
    coverage, against maxSignal = the population's signal."""
    calls = cfg["calls"]
    t_gen = time.perf_counter()
    m0set.clear()
    newsig.clear()
    step = max(1, min(cfg["programs"], args.npop))
    for m in range(0, args.npop, step):  # maxSignal <- every member's signal
        b = g.members(ctx, cfg, m, min(args.npop, m + step))
        triage(ctx, m0set, None, b, rec_new)
        torch.cuda.synchronize()
        del b
    m0_count = len(m0set)
    batches = [g.population(ctx, cfg, 5_000 + k, args.npop, args.noise) for k in range(args.warmup + args.steps)]
    t_gen = time.perf_counter() - t_gen
    maxnrec = max(b.nrec for b in batches)
    maxnvals = max(b.nvals for b in batches)
    for b in batches[: args.warmup]:
        call("sg_set_copy", maxsig.h, m0set.h)
        triage(ctx, maxsig, newsig, b, rec_new)
    timed = batches[args.warmup:]
    f0 = {k: ctx.counter("m0_filter_" + k) for k in ("used", "fallback")}
    wall, tri = timed_steps(ctx, maxsig, m0set, newsig, timed, rec_new, 1, tag=2)
    m0f = {k: ctx.counter("m0_filter_" + k) - f0[k] for k in f0}
    m0f["regime"] = "auto (option m0_filter -1)"
    kernels = kernel_table(ctx, STEP_KERNELS, args.steps)
    ctx.timing(False)
    units = sum(b.nvals for b in timed)
    out = {"workload": f"steady state: {cfg['programs']} programs x {calls} calls x {cfg['pcs_per_call']} PCs drawn "
                       f"from a fixed population of {args.npop} Zipf programs, each PC replaced by a fresh draw with "
                       f"probability {args.noise:g} (flaky coverage), vs maxSignal = the population's signal",
           "value": units / wall, "unit": "PCs/s", "ms_per_step": wall * 1e3 / args.steps,
           "triage_ms_events": float(np.mean(tri)),
           "maxsignal_start": m0_count, "signal_per_step": units / args.steps, "gen_s": round(t_gen, 2),
           "m0_filter": m0f, "kernels": kernels}
    if not args.no_account:
        diff_vals = torch.empty(maxnvals, dtype=torch.int32, device="cuda")
        diff_off = torch.empty(maxnrec + 1, dtype=torch.int64, device="cuda")
        acct = account(ctx, maxsig, m0set, newsig, timed, calls, rec_new, diff_vals, diff_off)
        out["accounting"] = acct
        out["roofline"] = roofline(acct, float(np.mean(tri)), kernels, "steady")
        del diff_vals, diff_off
    if not args.no_cpu:
        call("sg_set_copy", maxsig.h, m0set.h)
        triage(ctx, maxsig, None, timed[0], rec_new)
        torch.cuda.synchronize()
        out["cpu_baseline"] = cpu_baseline(m0set.export(), timed[0], calls, rec_new[: timed[0].nrec].cpu().numpy(),
                                           args.cpu_budget / 2, args.cpu_threads)
    del batches, timed
    torch.cuda.empty_cache()
    if args.from_traces:
        out["from_traces"] = run_steady_traces(ctx, args, cfg, g, maxsig, newsig, m0set, rec_new, min(args.steps, 4))
    return out


def run_steady_traces(ctx, args, cfg, g, maxsig, newsig, m0set, rec_new, steps):
    """The steady state end to end from raw traces, the way the fuzzer
    consumes them: the set-exact triage's flags and set updates, then the
    executor-exact per-call lists of the queued records only (fuzzer.go:678-683
    copies inf.Signal only for them), by sg_exec_signal_queued_dev; against the
    triage alone and against executor-exact lists of every call."""
    traces = []
    for k in range(steps):
        call("sg_gen_population_traces_dev", ctx.h, UNIVERSE_SEED, POP_SEED, args.npop, 5_000 + args.warmup + k,
             args.noise, cfg["zipf_s"], cfg["ranks"], 0, cfg["programs"], cfg["calls"], cfg["pcs_per_call"],
             g.trace.data_ptr())
        traces.append(g.trace.clone())
    so = torch.empty(g.ncalls + 1, dtype=torch.int64, device="cuda")
    states = [SignalSet(ctx) for _ in traces]
    # warm the queued-lists path (a kernel's first launch in the process loads
    # its code): nothing queued, so every program stops before its first call
    rec_new.zero_()
    call("sg_exec_signal_queued_dev", ctx.h, traces[0].data_ptr(), g.call_off.data_ptr(), g.prog_off.data_ptr(),
         cfg["programs"], g.ncalls, g.npcs, rec_new.data_ptr(), g.sig.data_ptr(), so.data_ptr())
    torch.cuda.synchronize()
    res = {}
    queued = []
    for mode in ("flags", "flags+queued", "flags+all"):
        for st in states:
            call("sg_set_copy", st.h, m0set.h)
        torch.cuda.synchronize()
        ev = []
        for tr, st in zip(traces, states):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ev.append(e)
            call("sg_triage_traces_dev", ctx.h, st.h, newsig.h, tr.data_ptr(), g.call_off.data_ptr(), g.npcs,
                 g.ncalls, rec_new.data_ptr())
            if mode == "flags+queued":
                call("sg_exec_signal_queued_dev", ctx.h, tr.data_ptr(), g.call_off.data_ptr(), g.prog_off.data_ptr(),
                     cfg["programs"], g.ncalls, g.npcs, rec_new.data_ptr(), g.sig.data_ptr(), so.data_ptr())
            elif mode == "flags+all":
                call("sg_exec_signal_dev", ctx.h, tr.data_ptr(), g.call_off.data_ptr(), g.prog_off.data_ptr(),
                     cfg["programs"], g.ncalls, g.npcs, g.sig.data_ptr(), so.data_ptr())
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ev.append(e)
            if mode == "flags":
                queued.append(rec_new[: g.ncalls].view(cfg["programs"], cfg["calls"]).clone())
        torch.cuda.synchronize()
        res[mode] = float(np.mean([ev[i].elapsed_time(ev[i + 1]) for i in range(0, len(ev), 2)]))
    for st in states:
        st.close()
    q = torch.stack(queued).to(torch.float32)
    del traces
    torch.cuda.empty_cache()
    return {"workload": f"steady state from {g.npcs} resident raw PCs per step: sg_triage_traces_dev (flags, set "
                        "updates), then sg_exec_signal_queued_dev (executor-exact lists of the queued records)",
            "steps": steps, "ms_flags": res["flags"], "ms_flags_queued_lists": res["flags+queued"],
            "ms_flags_all_lists": res["flags+all"], "queued_lists_over_flags": res["flags+queued"] / res["flags"],
            "queued_record_frac": float(q.mean().item()),
            "programs_with_queued_frac": float((q.amax(2) > 0).float().mean().item()),
            "value": g.npcs / (res["flags+queued"] / 1e3), "unit": "raw PCs/s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mode", choices=["auto", "c2", "c3", "fuzzers"], default="auto",
                    help="auto: c2 at N=1, c3 (hash-sharded one-batch triage) at N>1")
    ap.add_argument("--programs", type=int, default=None, help="programs per GPU (C2: 65536, C3: 131072)")
    ap.add_argument("--calls", type=int, default=16)
    ap.add_argument("--pcs", type=int, default=1024)
    ap.add_argument("--m0", type=int, default=16 << 20, help="entries in the starting maxSignal")
    ap.add_argument("--npop", type=int, default=2048, help="steady state: population size")
    ap.add_argument("--noise", type=float, default=2e-4, help="steady state: per-PC flaky-coverage probability")
    ap.add_argument("--no-steady", dest="steady", action="store_false")
    ap.add_argument("--no-from-traces", dest="from_traces", action="store_false")
    ap.add_argument("--c3-proto", choices=["prefix", "pairs"], default="prefix",
                    help="C3 protocol: bitmap prefixes (default) or candidate pairs hash-sharded by signal")
    ap.add_argument("--c3-form", choices=["auto", "kept", "pairs"], default="auto",
                    help="the prefix protocol's per-batch step-1 form (auto: by the last batch's novelty)")
    ap.add_argument("--c3-exchange", choices=["auto", "dense", "sparse"], default="auto",
                    help="the prefix protocol's exchange: bitmaps, candidate lists, or by the agreed novelty")
    ap.add_argument("--c3-steady", action="store_true",
                    help="measurement: C3 over steady-state batches (a fixed population with flaky coverage)")
    ap.add_argument("--c3-two-phase", action="store_true",
                    help="measurement: the prefix protocol's two-phase path at one rank too")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of single-thread CPU baseline work")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="threads of the CPU-share leg (a second leg always runs nproc threads)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host-api", dest="host_api", action="store_false",
                    help="skip the host entry point leg (C2 batch from pageable host memory)")
    ap.add_argument("--no-account", action="store_true", help="skip the byte-accounting replay")
    ap.add_argument("--no-ordered", dest="ordered", action="store_false",
                    help="skip the timed C2 step with the ordered diff outputs (needs the accounting replay)")
    ap.add_argument("--pipeline", action="store_true",
                    help="C2: also time the two-stage pipelined loop (syzkaller_amd/pipeline.py)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N > 1 paths on a smaller box: SG_BENCH_BACKEND=gloo puts
    # several ranks on one GPU (RCCL refuses that); the driver's runs use RCCL
    backend = os.environ.get("SG_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE={world}"
    mode = args.mode if args.mode != "auto" else ("c2" if world == 1 else "c3")
    if args.programs is None:
        args.programs = 65536 if mode in ("c2", "fuzzers") else 131072
    try:
        args.cpu_threads = min(args.cpu_threads, len(os.sched_getaffinity(0)))
    except AttributeError:
        pass
    cfg = {"programs": args.programs, "calls": args.calls, "pcs_per_call": args.pcs, "zipf_s": 1.1,
           "ranks": 1 << 20}
    ctx = Context(local)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)

    if mode == "c3":
        from bench_c3 import run_c3
        result = run_c3(ctx, args, cfg, rank, world)
    elif mode == "fuzzers":
        from bench_c3 import run_fuzzers
        result = run_fuzzers(ctx, args, cfg, rank, world)
    else:
        if world > 1:
            raise SystemExit("--mode c2 is the single-GPU configuration")
        args.steady = args.steady and True
        r = run_c2(ctx, args, cfg, rank)
        ms_step = r["wall_s"] * 1e3 / args.steps
        acct = r.get("acct")
        result = {
            "metric": METRIC,
            "value": r["units"] / r["wall_s"],
            "unit": "PCs/s",
            "n_gpus": 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (Zipf(1.1) PC traces generated on the GPU, counter-based PRNG)",
            "config": {
                "workload": "C2: 64Ki programs x 16 calls x 1024 Zipf PCs (executor signal, generated before the "
                            "timed region) -> batched new-signal triage vs a 16M-entry maxSignal bitmap (each step against "
                            "its own copy of the 16M-entry state, made before the timed region)",
                "programs_per_gpu": args.programs, "calls": args.calls, "pcs_per_call": args.pcs,
                "signal_per_step_per_gpu": r["units"] / args.steps,
                "maxsignal_start": r["m0"], "maxsignal_at_timing": r["m0"],
                "queued_frac": acct["queued_frac"] if acct else None,
                "parallelism": "single GPU",
            },
            "roofline": roofline(acct, r["triage_ms"], r["kernels"]) if acct else None,
            "cpu_baseline": r.get("cpu"),
            "timing": {"triage_ms_events": r["triage_ms"],
                       "wall_ms_per_step": ms_step},
            "kernels": r["kernels"],
            "accounting": acct,
            "ordered_outputs": r.get("ordered"),
            "steady_state": r.get("steady"),
            "from_traces": r.get("from_traces"),
            "host_api": r.get("host_api"),
            "pipelined": r.get("pipelined"),
            "path": "partitioned (flags + set updates)",
            "gen_s": r["gen_s"],
        }
        if rank != 0:
            result = None
    if rank == 0 and result is not None:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
