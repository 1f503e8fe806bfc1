"""One batch's new-signal triage, hash-sharded by signal across GPUs.

Reference: syz-fuzzer/fuzzer.go:645-693 -- ONE sequential loop over every call
record of the batch (records program-major, call index ascending).  The batch's
records are split contiguously across the ranks of a process group (one GPU
each, RCCL over xGMI); every rank holds the same maxSignal snapshot.  Results
are those of the single sequential loop: record r is queued iff it is the first
record holding some signal s not in maxSignal (the first-owner rule,
DESIGN.md §2), and maxSignal' = maxSignal ∪ every record's signal.

Protocol of one step, per rank:
  1. candidates -- sg_shard_candidates_dev: the rank's distinct s not in the
     snapshot with their first (global) record, grouped by owning shard
     sg_shard_of(s, G).  Only candidates travel.
  2. all-to-all of the pair counts, then of the pairs (RCCL all_to_all_single).
  3. owners -- sg_shard_owners_dev: owner(s) = min record over the pairs this
     shard received; the owners' bits in a batch-wide record bitset; each new s
     once.
  4. all-to-all of each rank's slice of the record bitset back to it, OR of
     the G slices into its records' flags (sg_shard_flags_dev; RCCL has no
     bitwise-OR reduction).
  5. all-gather of every shard's new signal; maxSignal / newSignal ∪= it
     (sg_set_add_dev), so the replicated state stays identical on all ranks.

The stage computations are a backend: HipStages (libsyzsig.so) in the
product; the CPU tests drive the same protocol with a numpy restatement of the
stages over gloo (tests/test_shard.py).  Collectives run on device tensors
under RCCL ("nccl"); under gloo they are staged through host memory.
"""
import ctypes

import torch
import torch.distributed as dist

from ._lib import call, lib


class Comm:
    """The collectives of the protocol over a torch.distributed group (or a
    single rank when torch.distributed is not initialised).

    At one rank every exchange is a local copy, unless `collectives` is set:
    then the group's collectives run anyway (a one-rank RCCL group executes the
    same device-tensor, async and side-stream code as N ranks; tests)."""

    def __init__(self, group=None, collectives=False):
        self.group = group
        self.on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.on else 1
        self.rank = dist.get_rank(group) if self.on else 0
        self.host = self.on and dist.get_backend(group) != "nccl"  # gloo: host-staged
        self.local = self.world == 1 and not (collectives and self.on)  # exchanges are copies

    def _stage(self, t):
        return t.cpu() if self.host and t.is_cuda else t

    def all_gather_i64(self, values):
        """[values of rank 0, values of rank 1, ...] for a short int64 list."""
        dev = "cpu" if (self.host or not torch.cuda.is_available()) else "cuda"
        t = torch.tensor(values, dtype=torch.int64, device=dev)
        if self.local:
            return [values]
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [x.tolist() for x in out]

    def exchange_counts(self, counts):
        """counts[k] goes to rank k; returns what every rank sent here."""
        if self.local:
            return list(counts)
        dev = "cpu" if self.host else "cuda"
        s = torch.tensor(counts, dtype=torch.int64, device=dev)
        r = torch.empty_like(s)
        dist.all_to_all_single(r, s, group=self.group)
        return r.tolist()

    def all_to_all(self, send, send_splits, recv_splits):
        """all_to_all_single with variable splits (element counts)."""
        if self.local:
            return send[: send_splits[0]]
        dev = send.device
        recv = torch.empty(sum(recv_splits), dtype=send.dtype, device="cpu" if self.host else dev)
        dist.all_to_all_single(recv, self._stage(send[: sum(send_splits)]), recv_splits, send_splits, group=self.group)
        return recv.to(dev) if self.host else recv

    def all_to_all_equal(self, out, t):
        """Dense all_to_all_single: part k of t (equal parts) goes to rank k,
        out's part j comes from rank j."""
        if self.local:
            out.copy_(t)
            return out
        if self.host:
            o = torch.empty(out.numel(), dtype=out.dtype)
            dist.all_to_all_single(o, self._stage(t), group=self.group)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, t, group=self.group)
        return out

    def all_gather_equal(self, out, t):
        """out = the t of every rank, concatenated in rank order."""
        if self.local:
            out.copy_(t)
            return out
        if self.host:
            o = torch.empty(out.numel(), dtype=out.dtype)
            dist.all_gather(list(o.view(self.world, -1).unbind(0)), self._stage(t), group=self.group)
            out.copy_(o)
        else:
            dist.all_gather_into_tensor(out, t, group=self.group)
        return out

    def start_all_to_all_equal(self, out, t):
        """all_to_all_equal left running on RCCL's stream (see start_all_gather_equal)."""
        if self.local or self.host:
            self.all_to_all_equal(out, t)
            return _Done()
        return dist.all_to_all_single(out, t, group=self.group, async_op=True)

    def start_all_gather_equal(self, out, t):
        """all_gather_equal left running on RCCL's stream; wait() on the handle
        orders the current stream after it (under gloo: done on return)."""
        if self.local or self.host:
            self.all_gather_equal(out, t)
            return _Done()
        return dist.all_gather_into_tensor(out, t, group=self.group, async_op=True)

    def all_gather_var(self, t, n):
        """The first n elements of t from every rank, concatenated."""
        if self.local:
            return t[:n]
        counts = [c[0] for c in self.all_gather_i64([n])]
        m = max(counts)
        dev = t.device
        buf = torch.zeros(m, dtype=t.dtype, device="cpu" if self.host else dev)
        buf[:n] = self._stage(t[:n])
        out = torch.empty(m * self.world, dtype=t.dtype, device=buf.device)
        if self.host:
            parts = list(out.view(self.world, m).unbind(0))
            dist.all_gather(parts, buf, group=self.group)
        else:
            dist.all_gather_into_tensor(out, buf, group=self.group)
        got = torch.cat([out[k * m: k * m + counts[k]] for k in range(self.world)])
        return got.to(dev) if self.host else got


class _Done:
    def wait(self):
        pass


class HipStages:
    """The stage kernels of libsyzsig.so (include/syzsig.h, sg_shard.hip)."""

    def __init__(self, ctx):
        self.ctx = ctx
        # stage outputs are read with torch (.tolist / .item): queue the
        # library's work on torch's current stream
        ctx.set_stream(torch.cuda.current_stream().cuda_stream)

    def candidates(self, snapshot, vals, off, nvals, nrec, rec_base, nshards, pairs):
        shard_off = torch.empty(nshards + 1, dtype=torch.int64, device="cuda")
        call("sg_shard_candidates_dev", self.ctx.h, snapshot.h, vals.data_ptr() if nvals else None, off.data_ptr(),
             nvals, nrec, rec_base, nshards, pairs.data_ptr() if nvals else None, shard_off.data_ptr())
        return shard_off.tolist()  # the counts are needed on the host for the exchange

    def owners(self, pairs, npairs, nrec_total, rec_bits, new_vals):
        nnew = torch.empty(1, dtype=torch.int64, device="cuda")
        call("sg_shard_owners_dev", self.ctx.h, pairs.data_ptr() if npairs else None, npairs, nrec_total,
             rec_bits.data_ptr(), new_vals.data_ptr() if npairs else None, nnew.data_ptr())
        return int(nnew.item())

    def flags(self, bits, nparts, words_per_part, rec_lo, nrec, rec_new):
        if nrec:
            call("sg_shard_flags_dev", self.ctx.h, bits.data_ptr(), nparts, words_per_part, rec_lo, nrec,
                 rec_new.data_ptr())

    def add(self, sset, vals, n):
        if n:
            call("sg_set_add_dev", sset.h, vals.data_ptr(), n)

    def add_new(self, newset, sset, vals, n):
        """sset |= vals[:n]; newset (nullable) gains those sset lacked."""
        if n:
            call("sg_set_add_new_dev", newset.h if newset is not None else None, sset.h, vals.data_ptr(), n)

    def delete(self, sset, vals, n):
        """Clears the bits of vals[:n]."""
        if n:
            call("sg_set_del_dev", sset.h, vals.data_ptr(), n)

    def prefix_cands(self, out, cap, slot=0):
        """out[:min(count, cap)] = the signals of the slot's pairs-form batch."""
        call("sg_prefix_cands_dev", self.ctx.h, slot, out.data_ptr() if cap else None, cap)

    # the prefix protocol's stages (PrefixTriage)
    words = 1 << 27  # a set's 2^32-bit bitmap

    def new_set(self):
        from .cover import SignalSet

        return SignalSet(self.ctx)

    def wrap(self, t):
        """A set over the first 2^27 words of the int32 device tensor t."""
        return _WrappedSet(self.ctx, t)

    def copy(self, dst, src):
        call("sg_set_copy", dst.h, src.h)

    def clear(self, sset):
        call("sg_set_clear", sset.h)

    def or_words(self, sset, t):
        call("sg_set_or_dev", sset.h, ctypes.c_void_p(t.data_ptr()))

    def or_new_words(self, sset, t, exclude):
        """sset |= t & ~exclude."""
        call("sg_set_or_new_dev", sset.h, ctypes.c_void_p(t.data_ptr()), exclude.h)

    def prefix_or(self, parts, nparts, words, prefix, total):
        call("sg_bitmap_prefix_or_dev", self.ctx.h, parts.data_ptr(), nparts, words, prefix.data_ptr(),
             total.data_ptr())

    def prefix_or_rank(self, parts, nparts, words, rank, prefix, total):
        """prefix (None for rank 0) = OR of parts < rank, total = OR of all."""
        call("sg_bitmap_prefix_or_rank_dev", self.ctx.h, parts.data_ptr(), nparts, words, rank,
             ctypes.c_void_p(prefix.data_ptr()) if prefix is not None else None, total.data_ptr())

    def or_new_or(self, newset, sset, t):
        """newset (nullable) |= t & ~sset, then sset |= t, in one pass."""
        call("sg_set_or_new_or_dev", newset.h if newset is not None else None, sset.h, ctypes.c_void_p(t.data_ptr()))

    def prefix_begin(self, base, marks, vals, off, nvals, nrec, slot=0, form=None, ncand=None):
        """form: None (the library's default), 0 kept partitions, 1 pairs,
        2 partitions only (base, marks None: a plain triage's first half);
        ncand (nullable int64 device tensor): the batch's novelty count."""
        if form is None and ncand is None:
            call("sg_prefix_begin_dev", self.ctx.h, slot, base.h, marks.h, vals.data_ptr() if nvals else None,
                 off.data_ptr(), nvals, nrec)
            return
        call("sg_prefix_begin_form_dev", self.ctx.h, slot, 0 if form is None else form,
             base.h if base is not None else None, marks.h if marks is not None else None,
             vals.data_ptr() if nvals else None, off.data_ptr(), nvals, nrec,
             ctypes.c_void_p(ncand.data_ptr()) if ncand is not None else None)

    def prefix_end(self, maxset, prefix, newset, rec_new, slot=0):
        """prefix: None or an int32 device tensor of >= 2^27 words (bitmap layout)."""
        call("sg_prefix_end_dev", self.ctx.h, slot, maxset.h, ctypes.c_void_p(prefix.data_ptr()) if prefix is not None
             else None, newset.h if newset is not None else None, rec_new.data_ptr())

    def prefix_flags(self, maxset, prefix, rec_new, slot=0):
        """prefix_end's flags; maxset gains at most the batch's marks | prefix."""
        call("sg_prefix_flags_dev", self.ctx.h, slot, maxset.h, ctypes.c_void_p(prefix.data_ptr()) if prefix is not None
             else None, rec_new.data_ptr())

    def triage(self, maxset, newset, vals, off, nvals, nrec, rec_new):
        call("sg_triage_batch_dev", self.ctx.h, maxset.h, newset.h if newset is not None else None,
             vals.data_ptr() if nvals else None, off.data_ptr(), nvals, nrec, rec_new.data_ptr() if nrec else None,
             None, None)


class _WrappedSet:
    """sg_set_wrap_dev over a torch tensor (kept alive with the handle)."""

    def __init__(self, ctx, t):
        h = ctypes.c_void_p()
        call("sg_set_wrap_dev", ctx.h, ctypes.c_void_p(t.data_ptr()), ctypes.byref(h))
        self.h, self.t = h, t

    def close(self):
        if self.h:
            lib.sg_set_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardedTriage:
    """fuzzer.go:645-693 over one batch spread across the ranks of `comm`.

    Buffers are allocated once and grown as needed (the pair buffers hold up to
    one pair per signal entry of the rank's slice)."""

    def __init__(self, stages, comm=None, device="cuda"):
        self.st = stages
        self.comm = comm if comm is not None else Comm()
        self.device = device
        self._bufs = {}
        self.last = {}

    def _buf(self, name, n, dtype=torch.int32):
        b = self._bufs.get(name)
        if b is None or b.numel() < n:
            b = torch.empty(max(n, 1), dtype=dtype, device=self.device)
            self._bufs[name] = b
        return b

    def step(self, maxsig, newsig, vals, off, nvals, nrec, rec_base, rec_new):
        """Triage records rec_base .. rec_base+nrec-1 of the batch held by this
        rank (vals / off its CSR slice, off[0] == 0) against maxsig, the
        replicated snapshot.  rec_new[:nrec] gets their flags; maxsig / newsig
        (nullable) gain every shard's new signal.  Returns the batch's record
        count."""
        c, G = self.comm, self.comm.world
        ranges = c.all_gather_i64([rec_base, nrec])
        nrec_total = max(rb + n for rb, n in ranges)
        # 1. candidates grouped by owning shard
        pairs = self._buf("pairs", 2 * nvals)
        shard_off = self.st.candidates(maxsig, vals, off, nvals, nrec, rec_base, G, pairs)
        send_pairs = [shard_off[k + 1] - shard_off[k] for k in range(G)]
        # 2. route them to their shards
        recv_pairs = c.exchange_counts(send_pairs)
        recv = c.all_to_all(pairs, [2 * x for x in send_pairs], [2 * x for x in recv_pairs])
        npairs = sum(recv_pairs)
        # 3. first owners of this shard's signals
        nwords = (nrec_total + 31) // 32
        rec_bits = self._buf("rec_bits", nwords)
        new_vals = self._buf("new_vals", npairs)
        nnew = self.st.owners(recv, npairs, nrec_total, rec_bits, new_vals)
        # 4. each rank's slice of the record bitset back to it, OR-ed there
        w0 = [rb >> 5 for rb, n in ranges]
        w1 = [((rb + n + 31) >> 5) if n else (rb >> 5) for rb, n in ranges]
        send_w = [w1[k] - w0[k] for k in range(G)]
        if G > 1:
            send = torch.cat([rec_bits[w0[k]:w1[k]] for k in range(G)])
        else:
            send = rec_bits[w0[0]:w1[0]]
        mine = send_w[c.rank]
        got = c.all_to_all(send, send_w, [mine] * G)
        self.st.flags(got, G, mine, rec_base, nrec, rec_new)
        # 5. every shard's new signal into the replicated sets
        allnew = c.all_gather_var(new_vals, nnew)
        n_all = int(allnew.numel())
        self.st.add(maxsig, allnew, n_all)
        if newsig is not None:
            self.st.add(newsig, allnew, n_all)
        self.last = {"pairs_sent": sum(send_pairs), "pairs_received": npairs, "new_signal": n_all,
                     "nrec_total": nrec_total}
        return nrec_total



XGMI_LINK_GBS = 153.0  # one xGMI link, one direction (7 per MI355X, one to each peer of an 8-GPU node)
COLLECTIVE_ALPHA_MS = 0.05  # fixed cost per RCCL collective (launch + handshake), an assumption
PREFIX_OR_GBS = 5500.0  # the prefix-OR / set passes stream at about this rate


def exchange_time_model(world, words=1 << 27, gather=None, cand_max=None, link_gbs=XGMI_LINK_GBS,
                        alpha_ms=COLLECTIVE_ALPHA_MS):
    """Predicted time of one batch's exchange per rank (ms), per form, on a
    fully connected node (one xGMI link to each peer, used in parallel):
    dense all-to-all form (G >= 3): all_to_all of C, all_to_all of P, all_gather
    of T -- each link carries one 1/G slice of the 512 MiB bitmap per
    collective -- plus the prefix-OR over G slices; dense gather form (G <= 2):
    all_gather of the whole C (each link the whole bitmap); sparse: all_gather
    of the (count, entries) words and of the candidate lists padded to the
    longest (cand_max entries).  Bytes over links, not measured (no N > 1
    node was available to the builder): a check for the driver's 8-GPU run."""
    G = world
    if G <= 1:
        return {"dense": 0.0, "sparse": 0.0 if cand_max is not None else None}
    gather = (G <= 2) if gather is None else gather
    bmp = 4 * words
    if gather:
        dense = bmp / (link_gbs * 1e6) + alpha_ms + (G * bmp) / (PREFIX_OR_GBS * 1e6)
    else:
        dense = 3 * ((bmp / G) / (link_gbs * 1e6) + alpha_ms) + (2 * bmp) / (PREFIX_OR_GBS * 1e6)
    sparse = None if cand_max is None else 2 * alpha_ms + (4 * cand_max + 16) / (link_gbs * 1e6)
    return {"dense": dense, "sparse": sparse}


class PrefixTriage:
    """fuzzer.go:645-693 over one batch whose call records are split
    contiguously across the ranks of `comm` (rank order = record order), by
    bitmap prefixes instead of candidate pairs:

      1. C_k = the signal of rank k's records not in M0 (the replicated
         maxSignal): sg_prefix_begin_dev partitions rank k's records once
         (kept for step 3) and marks that signal bucket by bucket.  (Only
         M0 | P_k matters below, so marking every signal would do too; the
         test against M0 keeps the LDS atomics to the candidates: marking
         every signal measured 1.26 vs 1.0 ms per C2-sized slice.)
      2. P_k = OR of C_j over ranks j < k, T = OR of every C_j: all-to-all of
         bitmap slices, an exclusive prefix-OR per slice on the owning rank
         (sg_bitmap_prefix_or_dev; RCCL has no bitwise OR), all-to-all of the
         prefixes back, all-gather of the totals.
      3. The local triage of rank k's records against M0 | P_k
         (sg_prefix_flags_dev, on the partitions of step 1, reading P_k beside
         maxSignal; rank 0 reads none, P_0 being empty).  M0 | P_k is the
         sequential loop's maxSignal before rank k's first record (P_k is the
         new signal of every earlier record), and within the rank the local
         triage is the loop itself, so the flags are the loop's.
      4. maxSignal = M0 | T and newSignal |= T on every rank (step 3 left
         maxSignal between M0 and M0 | T).
    Per rank and step the dense exchange moves about 2.5 bitmaps (512 MiB
    each) whatever the novelty, where ShardedTriage moves 8 B per candidate; at
    one rank it is the plain local triage.

    The sparse exchange (route only the candidates s not in
    M0) moves C_k as a list instead: step 1 in its pairs form keeps each s of
    C_k once, every rank all-gathers the lists (4 B per candidate, after an
    all-gather of the counts), P_k is set in a zeroed bitmap from the lists of
    the ranks before k (and cleared again after step 3, so it stays zero), and
    step 4 adds every list to maxSignal / newSignal.  The fuzzer's steady
    state (139K candidates per C2-sized step) exchanges ~0.5 MB per rank
    instead of ~1 GB.  Every rank gathers its (candidates, entries) after step
    1; the form of batch b is agreed from those counts of batch b - 2 (the
    same numbers on every rank, long arrived): sparse while every rank's
    candidates stay below sparse_below of its entries.

    start() runs steps 1-2 and leaves the exchange running on RCCL's stream
    (the prefix-OR on a side stream between the collectives); finish() runs
    steps 3-4.  Batches alternate between two slots, so the next batch can be
    started -- partitioned and marked while this one's bitmaps travel -- before
    this one is finished:  start(b0), start(b1), finish(b0), start(b2),
    finish(b1), ...  Marking batch i+1 against a maxSignal that still lacks
    batch i's total T_i only adds signal of M0' = M0 | T_i to C, and
    M0' | P' = M0' | P, so the flags are unchanged.

    Step 1's form is chosen per batch (form="auto"): "kept" keeps the rank's
    partitions and step 3 re-runs the bucket stage against M0 | P_k (a mark
    pass more than a plain triage, whatever the novelty); "pairs" keeps each s
    of C_k with its first record and step 3 tests those pairs against the
    current maxSignal | P_k (its cost grows with |C_k|: slower on fresh
    batches, cheaper in the fuzzer's low-novelty steady state; include/syzsig.h,
    sg_bucket.hip).  The rank takes "pairs" while the last batch it has a count
    for had |C_k| below pairs_below of its signal entries; the counts come back
    without a host wait (a pinned copy, read once its event has passed).  The
    forms are interchangeable stage by stage, so ranks may differ.  Stage
    contracts: HipStages."""

    def __init__(self, stages, comm=None, device="cuda", two_phase_at_one=False, side_stages=None, side_stream=None,
                 gather=None, form="auto", pairs_below=0.05, exchange="auto", sparse_below=None):
        self.st = stages
        self.comm = comm if comm is not None else Comm()
        self.device = device
        # (measurement: run the two-phase path with its local exchange at one rank too)
        self.two_phase_at_one = two_phase_at_one
        # the prefix-OR between the two collectives: stages on a second context
        # whose stream is side_stream (None: on the main stream, in start)
        self.side_st, self.side = side_stages, side_stream
        G, W = self.comm.world, stages.words
        self.S = -(-W // G)  # words per slice (the last slice padded)
        # gather mode: one all-gather of the whole C_k, every rank computes its
        # own prefix: (G-1) bitmaps per rank against the all-to-all form's
        # 3 (G-1) / G, so fewer bytes for G = 2 (and at one rank no exchange:
        # T = C)
        self.gather = (G <= 2) if gather is None else gather
        self.W = W
        self.slots = []
        if G > 1 or two_phase_at_one:
            n = self.S * G
            for _ in range(2):
                if self.gather:
                    # (this rank's P_k and T only; at one rank T is C itself)
                    C = torch.zeros(W, dtype=torch.int32, device=device)
                    b = {"C": C, "allc": torch.empty(G * W, dtype=torch.int32, device=device) if G > 1 else C,
                         "P": torch.zeros(W, dtype=torch.int32, device=device) if self.comm.rank > 0 else None,
                         "T": torch.empty(W, dtype=torch.int32, device=device) if G > 1 else C}
                else:
                    b = {k: torch.zeros(n, dtype=torch.int32, device=device) for k in ("C", "P", "T")}
                    b.update(recv=torch.empty(n, dtype=torch.int32, device=device),
                             pref=torch.empty(n, dtype=torch.int32, device=device),
                             tot=torch.empty(self.S, dtype=torch.int32, device=device))
                b["cset"] = stages.wrap(b["C"])
                b["ncand"] = torch.zeros(1, dtype=torch.int64, device=device)
                b["ncand_h"] = torch.zeros(1, dtype=torch.int64, pin_memory=(device != "cpu"))
                # every rank's (candidates, entries) of the slot's batch (the sparse form's
                # counts and the agreed form two batches later); P zero between sparse uses
                b["cnt"] = torch.zeros(2, dtype=torch.int64, device=device)
                b["cnts"] = torch.zeros(2 * G, dtype=torch.int64, device=device)
                b["cnts_h"] = torch.zeros(2 * G, dtype=torch.int64, pin_memory=(device != "cpu"))
                P = b["P"] if self.comm.rank > 0 else None
                b["pset"] = stages.wrap(P) if P is not None else None
                b["pclean"] = True
                self.slots.append(b)
        self.next_slot = 0
        self.last = {}
        self.form, self.pairs_below = form, pairs_below
        self.exchange = exchange
        self.sparse_below = 0.05 if sparse_below is None else sparse_below
        self.counted = []  # (slot, event) of the gathered counts of the last two started batches
        self._bufs = {}
        self.novelty = None  # |C_k| / entries of the last batch whose count has come back
        self._nov = None     # (slot, entries, event) of the count in flight

    def _form(self):
        """This batch's step-1 form (0 kept, 1 pairs; None: the library's default)."""
        if self.form == "kept":
            return 0
        if self.form == "pairs":
            return 1
        if self.form != "auto":
            return None
        if self._nov is not None:
            slot, n, ev = self._nov
            if ev is None or ev.query():
                self.novelty = float(self.slots[slot]["ncand_h"].item()) / max(n, 1)
                self._nov = None
        return 1 if self.novelty is not None and self.novelty < self.pairs_below else 0

    def _exchange_form(self):
        """This batch's exchange ("dense" or "sparse"), the same on every rank:
        from the gathered counts of the batch started two starts ago."""
        if self.exchange in ("dense", "sparse"):
            return self.exchange
        if len(self.counted) < 2:
            return "dense"
        slot, ev = self.counted[-2]
        if ev is not None:
            ev.synchronize()
        c = self.slots[slot]["cnts_h"].view(-1, 2).tolist()
        if any(n < 0 for n, _ in c):  # a rank ran a form that does not count: no data, stay dense
            return "dense"
        frac = max(n / max(e, 1) for n, e in c)
        return "sparse" if frac < self.sparse_below else "dense"

    def exchange_model(self):
        """Bytes per rank that the last finished batch's exchange takes in each
        form, whichever it used: dense (the bitmaps: fixed) and sparse (the
        candidate lists, from every rank's count of distinct signals outside
        maxSignal, gathered with the batch; the caller has synchronised, and
        calls before the batch after next starts: the two slots alternate).
        None when the batch ran without the counts (one rank without
        collectives, or a form that does not count)."""
        last, G = self.last, self.comm.world
        if "slot" not in last or last.get("form") == "default" or self.exchange == "dense":
            return None
        counts = self.slots[last["slot"]]["cnts_h"].view(-1, 2)[:, 0].tolist()
        m = max(counts)
        dense = (4 * self.W * (G - 1) if self.gather else 4 * self.S * (3 * (G - 1))) + 16 * (G - 1)
        return {"dense": dense, "sparse": (4 * m + 16) * (G - 1), "candidates_max": m}

    def _buf(self, name, n, dtype=torch.int32):
        b = self._bufs.get(name)
        if b is None or b.numel() < n:
            b = torch.empty(max(n, 1), dtype=dtype, device=self.device)
            self._bufs[name] = b
        return b

    def step(self, maxsig, newsig, vals, off, nvals, nrec, rec_base, rec_new, nrec_total=None):
        """Same contract as ShardedTriage.step."""
        return self.finish(self.start(maxsig, newsig, vals, off, nvals, nrec, rec_base, rec_new, nrec_total))

    def start(self, maxsig, newsig, vals, off, nvals, nrec, rec_base, rec_new, nrec_total=None):
        """Steps 1-2 for records rec_base .. rec_base+nrec-1 (vals / off this
        rank's CSR slice, off[0] == 0); rec_new gets their flags in finish().
        Returns the pending step.  nrec_total (the batch's record count) may be
        given by the caller; otherwise it is gathered, which waits for the
        collectives already in flight."""
        c, st, G = self.comm, self.st, self.comm.world
        if nrec_total is None:
            nrec_total = max(rb + n for rb, n in c.all_gather_i64([rec_base, nrec]))
        pend = {"maxsig": maxsig, "newsig": newsig, "rec_new": rec_new, "nrec_total": nrec_total}
        if not self.slots:
            st.triage(maxsig, newsig, vals, off, nvals, nrec, rec_new)
            pend["last"] = {"nrec_total": nrec_total, "exchange_bytes": 0}
            return pend
        slot = self.next_slot
        self.next_slot ^= 1
        b = self.slots[slot]
        xform = self._exchange_form()  # (reads this slot's counts of two batches ago)
        # 1. this rank's new signal against M0 (its partitions, or its pairs, kept for 3.)
        form = 1 if xform == "sparse" else self._form()
        if form is None:
            st.prefix_begin(maxsig, b["cset"], vals, off, nvals, nrec, slot)
        else:
            st.prefix_begin(maxsig, b["cset"], vals, off, nvals, nrec, slot, form=form, ncand=b["ncand"])
            if self._nov is None and nvals:  # (one count in flight at a time; an empty batch tells nothing)
                ev = None
                if b["ncand"].is_cuda:
                    b["ncand_h"].copy_(b["ncand"], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record()
                else:
                    b["ncand_h"].copy_(b["ncand"])
                self._nov = (slot, nvals, ev)
        # every rank's (candidates, entries): the sparse form's counts now, the
        # agreed form two batches on (not gathered when the exchange is forced
        # dense: nothing reads them then, and the gather would wait on step 1)
        if self.exchange != "dense":
            if form is None:  # (the library's default form counts nothing: unknown, not 0)
                b["ncand"].fill_(-1)
            b["cnt"][:1].copy_(b["ncand"])
            b["cnt"][1] = nvals
            c.all_gather_equal(b["cnts"], b["cnt"])
            if b["cnts"].is_cuda:
                b["cnts_h"].copy_(b["cnts"], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
            else:
                b["cnts_h"].copy_(b["cnts"])
                ev = None
            self.counted = (self.counted + [(slot, ev)])[-2:]
        pend["slot"] = slot
        if xform == "sparse":
            # 2. the candidate lists of every rank (padded to the longest)
            counts = b["cnts"].view(-1, 2)[:, 0].tolist()  # (waits for step 1 and the counts)
            m = max(counts)
            cand = self._buf(("cand", slot), m)
            st.prefix_cands(cand, m, slot)
            allc = self._buf(("allc", slot), G * m)
            if m:
                c.all_gather_equal(allc[: G * m], cand[:m])
            pend["sparse"] = (allc, counts, m)
            pend["got_p"] = pend["got_t"] = _Done()
            pend["last"] = {"nrec_total": nrec_total, "exchange": "sparse", "form": "pairs",
                            "exchange_bytes": (4 * m + 16) * (G - 1), "candidates": counts, "slot": slot}
            return pend
        if c.rank > 0:
            b["pclean"] = False  # (the dense prefix lands in P)
        # 2. exclusive prefix and total over the ranks (slice by slice, or
        # whole bitmaps in gather mode)
        if self.gather:
            got_c = c.start_all_gather_equal(b["allc"], b["C"]) if G > 1 else _Done()
        else:
            got_c = c.start_all_to_all_equal(b["recv"], b["C"])

        def exchange(stages):
            got_c.wait()
            if self.gather:  # this rank's P_k and T (one part: T = C)
                if G > 1:
                    stages.prefix_or_rank(b["allc"], G, self.W, c.rank, b["P"], b["T"])
                pend["got_p"] = pend["got_t"] = _Done()
            else:
                stages.prefix_or(b["recv"], G, self.S, b["pref"], b["tot"])
                pend["got_p"] = c.start_all_to_all_equal(b["P"], b["pref"])
                pend["got_t"] = c.start_all_gather_equal(b["T"], b["tot"])

        if self.side is not None:
            self.side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.side):
                exchange(self.side_st)
                # (one rank, gloo or gather mode: the side stream's own work)
                pend["side_done"] = torch.cuda.Event()
                pend["side_done"].record(self.side)
        else:
            exchange(st)
        xb = 4 * self.W * (G - 1) if self.gather else 4 * self.S * (3 * (G - 1))
        pend["last"] = {"nrec_total": nrec_total, "exchange": "dense" if G > 1 else "local",
                        "exchange_bytes": xb + 16 * (G - 1),
                        "form": {0: "kept", 1: "pairs", None: "default"}[form], "slot": slot}
        return pend

    def finish(self, pend):
        """Steps 3-4 of a started batch; returns the batch's record count."""
        st = self.st
        if "sparse" in pend:
            b, slot = self.slots[pend["slot"]], pend["slot"]
            maxsig, newsig = pend["maxsig"], pend["newsig"]
            allc, counts, m = pend["sparse"]
            k = self.comm.rank
            # 3. the flags against M0 | P_k, P_k set from the lists of the ranks before this one
            P = None
            if k > 0:
                if not b["pclean"]:
                    st.clear(b["pset"])
                    b["pclean"] = True
                for j in range(k):
                    st.add(b["pset"], allc[j * m:], counts[j])
                P = b["P"]
            st.prefix_flags(maxsig, P, pend["rec_new"], slot)
            # 4. every list into the replicated sets (newSignal: what maxSignal lacked)
            for j in range(len(counts)):
                st.add_new(newsig, maxsig, allc[j * m:], counts[j])
            for j in range(k):  # (P back to zero)
                st.delete(b["pset"], allc[j * m:], counts[j])
            self.last = pend["last"]
            return pend["nrec_total"]
        if "slot" in pend:
            b, slot = self.slots[pend["slot"]], pend["slot"]
            maxsig, newsig = pend["maxsig"], pend["newsig"]
            # 3. the flags against M0 | P_k
            if "side_done" in pend:
                torch.cuda.current_stream().wait_event(pend["side_done"])
            pend["got_p"].wait()
            pend["got_t"].wait()
            # newSignal gains the batch's signal that maxSignal lacks now
            # (fuzzer.go:674): T was computed against the maxSignal of start(),
            # which an overlapped batch finished since may have grown, and
            # newSignal may have been drained (the Poll, fuzzer.go:358-364) in
            # between -- so T & ~maxSignal, before step 3 changes maxSignal
            P = b["P"] if self.comm.rank > 0 else None
            if pend["last"].get("form") == "pairs":
                # the pairs' flags leave maxSignal as it is: 3., then both set
                # updates (4.) in one pass over T
                st.prefix_flags(maxsig, P, pend["rec_new"], slot)
                st.or_new_or(newsig, maxsig, b["T"])
            else:
                if newsig is not None:
                    st.or_new_words(newsig, b["T"], maxsig)
                st.prefix_flags(maxsig, P, pend["rec_new"], slot)
                # 4. the replicated state after the whole batch
                st.or_words(maxsig, b["T"])
        self.last = pend["last"]
        return pend["nrec_total"]
