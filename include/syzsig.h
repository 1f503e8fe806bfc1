/*
 * syzsig.h -- C-ABI of the MI355X coverage-signal triage engine (libsyzsig.so).
 *
 * This is the drop-in boundary for syzkaller's coverage-signal path.  Every
 * entry point names the reference interface it replaces (paths relative to the
 * syzkaller checkout).  The Go side binds it through cgo; INTEGRATION.md shows
 * the binding.  Plain pointers and sizes only.
 *
 * Conventions
 *  - Every function returning int returns SG_OK (0) or a negative SG_E* code;
 *    sg_last_error() gives the message (thread-local).  The Go adapter panics
 *    on failure, as the reference callers do (syz-fuzzer/fuzzer.go:389-391).
 *  - "host" entry points take caller-owned host memory and never retain it
 *    (cgo pointer rules).  "_dev" entry points take device pointers already
 *    resident in HBM and are stream-ordered on the context's stream: they do
 *    not synchronise, and their outputs are valid after sg_ctx_sync().
 *  - Signal / cover values are uint32_t, any value allowed.  Sorted-slice ops
 *    follow pkg/cover/cover.go exactly: multiset semantics; 0xFFFFFFFF
 *    (`sent`, cover.go:17) is dropped by every foreach op (cover.go:97), and
 *    by Canonicalize only when no smaller value precedes it (`last` starts at
 *    sent, cover.go:31).
 *  - A context owns one HIP stream on one device and all device memory it
 *    allocates.  Calls on one context must be serialised by the caller (the
 *    reference already holds signalMu / mgr.mu around them).
 *  - There is no CPU fallback: without a usable gfx950 device every call that
 *    computes returns SG_ENODEV.
 */
#ifndef SYZSIG_H
#define SYZSIG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG_OK 0
#define SG_EINVAL (-1)
#define SG_EHIP (-2)
#define SG_ENOMEM (-3)
#define SG_ENODEV (-4)

typedef struct sg_ctx sg_ctx;
typedef struct sg_set sg_set;

/* Library identification and error reporting. */
const char* sg_version(void);
const char* sg_last_error(void);

/* ---- context ------------------------------------------------------------ */
/* One per fuzzer / manager process (or per GPU rank).  `device` is the HIP
 * device ordinal. */
int sg_ctx_create(int device, sg_ctx** out);
void sg_ctx_destroy(sg_ctx* ctx);
/* Wait for all work queued on the context's stream. */
int sg_ctx_sync(sg_ctx* ctx);
/* Queue all further work on `hip_stream` (e.g. torch's current stream; NULL is
 * the legacy default stream).  The context's own stream is a blocking stream,
 * i.e. ordered with the legacy default stream. */
int sg_ctx_set_stream(sg_ctx* ctx, void* hip_stream);
/* Go back to the context's own stream. */
int sg_ctx_reset_stream(sg_ctx* ctx);
void* sg_ctx_stream(sg_ctx* ctx);
/* Per-kernel device timing with HIP events on the context's stream.
 * enable != 0 starts recording (and resets the tallies). */
int sg_ctx_timing(sg_ctx* ctx, int enable);
/* Total device milliseconds and launch count recorded for kernel `name`
 * (e.g. "bucket_triage"); syncs the stream. */
int sg_ctx_kernel_time(sg_ctx* ctx, const char* name, double* ms, uint64_t* launches);
/* Context counters: "owner_resets" (Minimize's first-owner table generations
 * started after the key space ran out), "owner_floor", "owner_key_space",
 * "max_launch_records"; the host ingest's last call (sg_triage_batch /
 * sg_triage_traces without diff lists): "host_copy_bytes", "host_copy_ns"
 * (pageable -> pinned copies), "host_wait_ns" (waits for a staging slot's DMA),
 * "host_copy_threads"; "cpu_quota_milli" (the CPUs this process may use,
 * x1000); the M0 filter (the flags path's low-novelty regime): "m0_filter_used"
 * and "m0_filter_fallback" (record slices it finished / that went on to pass
 * 2), "m0_filter_survivors" (the last launch's), "m0_filter_queued_milli" (the
 * queued fraction of the last partitioned slice, x1000, that auto reads),
 * "m0_filter_halves_log" (the index parts per slice, log2, auto uses now). */
int sg_ctx_counter(sg_ctx* ctx, const char* name, uint64_t* out);
/* Context options.  Every path is selected by its regime; an option only
 * forces one, for a test or a measurement, and no call reads the environment
 * (sg_ctx_create seeds "debug_part", "bucket_blocks" and "prefix_pairs" from
 * SG_DEBUG_PART / SG_BUCKET_BLOCKS / SG_PREFIX_PAIRS, for the GPU scripts).
 * Keys (-1 = the regime's choice where it applies):
 *   "max_launch_records"   records per partitioned launch (0: 2^24)
 *   "owner_key_space"      Minimize's first-owner key space (0: 2^32 - 1; set
 *                          before the first Minimize)
 *   "debug_part"           phase counters of the partitioned path (stderr)
 *   "bucket_blocks"        cap of the persistent bucket grid (0: none)
 *   "prefix_pairs"         sg_prefix_begin_dev's form (0 kept partitions, 1 pairs)
 *   "fold_map"             sg_union_fold's one-group byte map (-1 by range, 0 never)
 *   "minimize_filter"      Minimize's value filter (1 on, 0 off)
 *   "minimize_filter_ranks" Minimize's phase-A inputs (0: the default 4)
 *   "report_direct"        sg_cover_uncovered's global-search form at any size (1)
 *   "rpc_encode_elems"     delta encode form (-1 by shape, 0 per list, 1 per element)
 *   "rpc_decode_blocks"    delta decode form (-1 by shape, 0 per list, 1 per block)
 *   "host_slice"           host ingest: entries per record slice (0: 64 Mi)
 *   "host_copy_threads"    host ingest: copy threads (0: half the CPU quota, 2..16)
 *   "m0_filter"            the flags path's M0 filter (-1 auto: after a filtered
 *                          slice, or a partitioned one that queued < 1/4 of its
 *                          records, backing off after fallbacks; 1 always; 0 never)
 *   "m0_filter_halves"     its index in 2^k parts per slice (-1 auto: 2 parts once a
 *                          part overflows; 0..2 forced)
 * Unknown keys and out-of-range values return SG_EINVAL. */
int sg_ctx_set_option(sg_ctx* ctx, const char* key, int64_t value);
int sg_ctx_get_option(sg_ctx* ctx, const char* key, int64_t* out);
/* Profiling aid: a one-thread kernel (k_mark_begin, or k_mark_end when end !=
 * 0) on the context's stream, so a kernel trace can cut out a region. */
int sg_ctx_marker(sg_ctx* ctx, int end, uint32_t tag);

/* ---- signal sets: replace map[uint32]struct{} ---------------------------- */
/* maxSignal / corpusSignal / newSignal (syz-fuzzer/fuzzer.go:65-68) and
 * corpusSignal / maxSignal / corpusCover (syz-manager/manager.go:71-73): a
 * direct-indexed 2^32-bit bitmap (512 MiB) resident in HBM. */
int sg_set_create(sg_ctx* ctx, sg_set** out);
void sg_set_destroy(sg_set* set);
int sg_set_clear(sg_set* set);
/* len(map) */
int sg_set_count(sg_set* set, uint64_t* out);
/* All members ascending (the reference iterates map order; payloads of
 * ConnectRes.MaxSignal / PollArgs.MaxSignal, pkg/rpctype/rpctype.go).  Writes
 * min(count, cap) values; *n = count. */
int sg_set_export(sg_set* set, uint32_t* out, size_t cap, size_t* n);
/* pkg/cover/cover.go:178-182  SignalAdd(base, signal) */
int sg_set_add(sg_set* set, const uint32_t* sig, size_t n);
/* pkg/cover/cover.go:160-167  SignalNew(base, signal) -> *out 0/1 */
int sg_set_new(sg_set* set, const uint32_t* sig, size_t n, int* out);
/* pkg/cover/cover.go:169-176  SignalDiff(base, signal): members of sig not in
 * base, in order, duplicates kept.  out capacity n; *nout = count. */
int sg_set_diff(sg_set* set, const uint32_t* sig, size_t n, uint32_t* out, size_t* nout);
/* Device bitmap (2^27 uint32 words) for collectives (OR-reduce across ranks).
 * Layout: signal s = bytes (b3 b2 b1 b0) is bit p = (b2 b1 b3 b0) (bit p & 31
 * of word p >> 5), a fixed permutation of whole words that keeps each (b2, b1)
 * block of 2^16 signals contiguous (the triage's buckets).  Element-wise ops
 * (OR, copy, count) do not depend on it. */
void* sg_set_device_words(sg_set* set);
/* Wrap caller-owned device memory (2^27 uint32 words, e.g. a torch tensor)
 * as a set without copying; sg_set_destroy then frees only the handle. */
int sg_set_wrap_dev(sg_ctx* ctx, void* d_words, sg_set** out);
/* set |= words (device pointer to 2^27 uint32 words). */
int sg_set_or_dev(sg_set* set, const uint32_t* d_words);
/* set |= words & ~exclude (device pointer to 2^27 uint32 words; exclude a set
 * of the same context): the new signal of a batch whose total was computed
 * against an older maxSignal (fuzzer.go:674 adds to newSignal only what
 * maxSignal lacks). */
int sg_set_or_new_dev(sg_set* set, const uint32_t* d_words, sg_set* exclude);
/* Both in one pass over words: newsig |= words & ~maxsig, then maxsig |= words
 * (newsig nullable; the two sets distinct, of one context, neither aliasing
 * words).  Words that are zero are read once and nothing else is touched. */
int sg_set_or_new_or_dev(sg_set* newsig, sg_set* maxsig, const uint32_t* d_words);
/* dst = src (both sets of the same context). */
int sg_set_copy(sg_set* dst, sg_set* src);
/* *out = number of the n device-resident values not in set (duplicates
 * counted), i.e. the candidates a triage of them would test; syncs. */
int sg_set_count_missing_dev(sg_set* set, const uint32_t* d_vals, uint64_t n, uint64_t* out);

/* ---- batched new-signal triage (THE hot path) ----------------------------- */
/* syz-fuzzer/fuzzer.go:645-693 execute(): for call records r = 0..nrec-1 in
 * sequential (program-major, call-index) order, record r's signal is
 * vals[rec_off[r] .. rec_off[r+1]).  Exactly as the sequential loop:
 *   rec_new[r] = SignalNew(maxSignal, S_r) at its turn (fuzzer.go:666);
 *   diff_r     = SignalDiff(maxSignal, S_r) at its turn (fuzzer.go:669);
 *   maxSignal ∪= diff_r; newSignal ∪= diff_r (fuzzer.go:673-674).
 * diff_r is written to diff_vals[diff_off[r] .. diff_off[r+1]) when diff_vals /
 * diff_off are non-NULL (capacity = rec_off[nrec]).  newsig may be NULL.
 * *n_diff (nullable) = total diff elements. */
int sg_triage_batch(sg_ctx* ctx, sg_set* maxsig, sg_set* newsig, const uint32_t* vals, const uint64_t* rec_off,
		    size_t nrec, uint8_t* rec_new, uint32_t* diff_vals, uint64_t* diff_off, uint64_t* n_diff);
/* Same, device-resident: d_vals (nvals = rec_off[nrec] elements), d_rec_off
 * (nrec+1), outputs d_rec_new (nrec bytes), optional d_diff_vals (capacity
 * nvals), d_diff_off (nrec+1).  Stream-ordered, no host synchronisation,
 * except that a flags-only batch of more than 2^24 records runs as record
 * slices with one small device-to-host read per slice.  Limits: nvals <
 * 2^32 - 2^15, nrec < 2^32 - 1. */
int sg_triage_batch_dev(sg_ctx* ctx, sg_set* maxsig, sg_set* newsig, const uint32_t* d_vals,
			const uint64_t* d_rec_off, uint64_t nvals, uint64_t nrec, uint8_t* d_rec_new,
			uint32_t* d_diff_vals, uint64_t* d_diff_off);

/* The same triage fed with raw per-call u32 PC traces (the executor's KCOV
 * buffers, executor/executor_linux.cc:262-313) instead of signal: record r =
 * call r, its trace pcs[call_off[r] .. call_off[r+1]) (call_off[0] == 0),
 * its edges sig = pc ^ hash(previous pc of the call), pc ^ 0 for the call's
 * first pc (executor/executor.h:389-401, hash :497-505), zero edges dropped
 * (dedup(0) reports seen, :507-526).  rec_new and the maxSignal / newSignal
 * updates are exactly those of sg_exec_signal_dev followed by a flags-only
 * sg_triage_batch_dev on its output: the executor writes every non-zero edge
 * at its first occurrence in the program, so the first call holding each
 * edge and the batch's union of edges -- all that decides the flags and the
 * sets (fuzzer.go:665-691) -- do not depend on the edges its lossy dedup
 * table drops or lets through again (set-exact mode).
 * Calls need not be grouped into programs.  Limits as sg_triage_batch_dev. */
int sg_triage_traces(sg_ctx* ctx, sg_set* maxsig, sg_set* newsig, const uint32_t* pcs, const uint64_t* call_off,
		     size_t ncalls, uint8_t* rec_new);
int sg_triage_traces_dev(sg_ctx* ctx, sg_set* maxsig, sg_set* newsig, const uint32_t* d_pcs,
			 const uint64_t* d_call_off, uint64_t npcs, uint64_t ncalls, uint8_t* d_rec_new);

/* ---- one batch hash-sharded by signal across GPUs ------ */
/* The sequential loop of sg_triage_batch (syz-fuzzer/fuzzer.go:645-693) over a
 * batch whose call records are split contiguously across G ranks, one GPU each
 * (the host protocol and its RCCL exchanges: syzkaller_amd/shard.py).  The
 * signal space is sharded by sg_shard_of(s, G), the murmur3 finaliser of s
 * scaled to [0, G); G <= 64.  Every rank holds the same maxSignal snapshot. */
int sg_shard_of(uint32_t s, uint32_t nshards);
/* Local stage, on the rank holding records rec_base .. rec_base+nrec-1 of the
 * batch (d_rec_off[0] == 0, rec_base + nrec < 2^32): every distinct s of those
 * records that is not in `snapshot`, once, as the pair {s, rec_base + its
 * first record}, grouped by owning shard: shard k's pairs are pairs
 * d_shard_off[k] .. d_shard_off[k+1]-1 of d_pairs (u32 pairs, capacity nvals
 * pairs; d_shard_off: G+1 device u64).  The snapshot is only read.  Any
 * number of entries (record slices of < 2^30 entries each). */
int sg_shard_candidates_dev(sg_ctx* ctx, sg_set* snapshot, const uint32_t* d_vals, const uint64_t* d_rec_off,
			    uint64_t nvals, uint64_t nrec, uint64_t rec_base, uint32_t nshards, uint32_t* d_pairs,
			    uint64_t* d_shard_off);
/* Owner stage, on the shard's rank, over the npairs pairs {s, record} it
 * received from all ranks (record < nrec_total, the batch's record count):
 * owner(s) = the smallest record holding s.  Sets bit r of d_rec_bits (nrec_total
 * bits, cleared first) for every owner record r -- record r is queued for
 * triage iff some shard sets its bit (fuzzer.go:678-690) -- and writes every
 * distinct s once to d_new_vals (capacity npairs); *d_nnew (device u64) = count. */
int sg_shard_owners_dev(sg_ctx* ctx, const uint32_t* d_pairs, uint64_t npairs, uint64_t nrec_total,
			uint32_t* d_rec_bits, uint32_t* d_new_vals, uint64_t* d_nnew);
/* d_rec_new[i] = bit rec_lo + i of the OR of nparts record bitsets, part k
 * being words k*words_per_part .. of d_bits, each starting at word rec_lo/32. */
int sg_shard_flags_dev(sg_ctx* ctx, const uint32_t* d_bits, uint32_t nparts, uint64_t words_per_part, uint64_t rec_lo,
		       uint64_t nrec, uint8_t* d_rec_new);
/* SignalAdd of n device-resident values (fuzzer.go:673-674 for the new signal
 * every shard found). */
int sg_set_add_dev(sg_set* set, const uint32_t* d_vals, uint64_t n);
/* maxsig |= the n device values; newsig (nullable) gains those maxsig lacked
 * before this call (fuzzer.go:673-674: newSignal.Merge(diff), diff =
 * maxSignal.Diff(sig)), duplicates in the values included.  The sparse form of
 * the prefix protocol's set updates (syzkaller_amd/shard.py). */
int sg_set_add_new_dev(sg_set* newsig, sg_set* maxsig, const uint32_t* d_vals, uint64_t n);
/* Clears the bits of the n device values (the sparse prefix protocol clears
 * the prefix bits it set, so the bitmap stays zero between batches). */
int sg_set_del_dev(sg_set* set, const uint32_t* d_vals, uint64_t n);
/* Bitmap prefix exchange of the prefix protocol (syzkaller_amd/shard.py
 * PrefixTriage): d_parts holds nparts bitmap slices of `words` u32 words each,
 * part k from rank k.  d_prefix[k] = OR of parts 0..k-1 (part 0: zero),
 * d_total = OR of all parts.  RCCL has no bitwise-OR reduction. */
int sg_bitmap_prefix_or_dev(sg_ctx* ctx, const uint32_t* d_parts, uint32_t nparts, uint64_t words, uint32_t* d_prefix,
			    uint32_t* d_total);
/* One rank's share of it (the gather form, where every rank holds all parts):
 * d_prefix (nullable: rank 0's is zero) = OR of parts 0..rank-1, d_total = OR
 * of all parts; rank < nparts. */
int sg_bitmap_prefix_or_rank_dev(sg_ctx* ctx, const uint32_t* d_parts, uint32_t nparts, uint64_t words, uint32_t rank,
				 uint32_t* d_prefix, uint32_t* d_total);
/* The two halves of sg_triage_batch_dev (flags and set updates, no diff) for
 * the prefix protocol.  Begin: marks (base != marks) = every signal of the
 * batch not in base (the local new signal, fuzzer.go:666), and
 * each such signal's first record in the batch is kept in the context's slot
 * (0 or 1: two batches can be kept, so one batch's exchange runs while the
 * next is begun).  End: the
 * sequential loop's flags (fuzzer.go:645-693) of the batch's nrec records
 * against maxsig | d_prefix (d_prefix: nullable, 2^27 words in the set layout,
 * e.g. another set's or an exchanged bitmap), written to d_rec_new; maxsig must
 * contain begin's base.  End's set updates: newsig (nullable) gains the new
 * signal (marks minus maxsig | d_prefix), and maxsig |= marks -- its new signal
 * and bits of d_prefix (the prefix protocol ORs a superset of d_prefix into
 * maxsig afterwards).  Flags: the flags without newsig; maxsig ends between
 * its value and maxsig | marks | d_prefix (the protocol ORs a superset of
 * marks | d_prefix into it next), so maxsig is written by flags too.  Marks must stay unchanged until end; only begin's launches read the
 * batch's buffers, and other calls may run on the context between begin and
 * end/flags (the slots have workspaces of their own).  End and flags close
 * the slot. */
int sg_prefix_begin_dev(sg_ctx* ctx, uint32_t slot, sg_set* base, sg_set* marks, const uint32_t* d_vals,
			const uint64_t* d_rec_off, uint64_t nvals, uint64_t nrec);
/* sg_prefix_begin_dev with the batch's form chosen by the caller (there:
 * SG_PREFIX_PAIRS): form 0 keeps the batch's partitions (end re-runs the bucket
 * stage against maxsig | d_prefix), form 1 its distinct signals not in base
 * with their first records (end tests those pairs; cheaper when few).  The
 * results are the same.  d_ncand (nullable, device u64) receives the number of
 * distinct signals of the batch not in base -- the novelty a caller picks the
 * next batch's form from (syzkaller_amd/shard.py PrefixTriage).  Form 2 (base,
 * marks and d_ncand NULL) keeps the partitions and marks nothing: begin + end
 * with d_prefix NULL is sg_triage_batch_dev (flags and set updates) cut in
 * two, so a caller can partition batch i+1 (begin, on one stream) while batch
 * i's bucket stage runs (end, on another; the fuzzer loop's order is kept by
 * running the ends in batch order). */
int sg_prefix_begin_form_dev(sg_ctx* ctx, uint32_t slot, uint32_t form, sg_set* base, sg_set* marks,
			     const uint32_t* d_vals, const uint64_t* d_rec_off, uint64_t nvals, uint64_t nrec,
			     uint64_t* d_ncand);
int sg_prefix_end_dev(sg_ctx* ctx, uint32_t slot, sg_set* maxsig, const uint32_t* d_prefix, sg_set* newsig,
		      uint8_t* d_rec_new);
/* The signals of a pairs-form begin's kept pairs (slot's batch: each
 * distinct signal of the batch not in base, once), d_out[i] for i < min(n,
 * cap), n = the count begin wrote to d_ncand.  The candidate lists the sparse
 * prefix exchange all-gathers (shard.py PrefixTriage) instead of bitmaps;
 * fuzzer.go:665-691 over one batch spread across ranks. */
int sg_prefix_cands_dev(sg_ctx* ctx, uint32_t slot, uint32_t* d_out, uint64_t cap);
int sg_prefix_flags_dev(sg_ctx* ctx, uint32_t slot, sg_set* maxsig, const uint32_t* d_prefix,
			uint8_t* d_rec_new);

/* syz-fuzzer/fuzzer.go:467-489 addInput(), over n inputs in order:
 * diff = SignalDiff(maxSignal, S_k); corpusSignal ∪= diff; maxSignal ∪= diff. */
int sg_add_inputs(sg_ctx* ctx, sg_set* corpus, sg_set* maxsig, const uint32_t* vals, const uint64_t* off, size_t n);

/* syz-fuzzer/fuzzer.go:521-611 triageInput()'s signal math, over n inputs at
 * once (the -procs triage goroutines, or a batch of triage candidates).
 * fuzzer.go:526-532: new_k = Canonicalize(SignalDiff(corpusSignal, S_k)),
 * every input against the same corpusSignal (only read).  S_k = vals[off[k] ..
 * off[k+1]); new_vals capacity off[n]; new_off (n+1) gives each new_k. */
int sg_triage_newsig(sg_ctx* ctx, sg_set* corpus, const uint32_t* vals, const uint64_t* off, size_t n,
		     uint32_t* new_vals, uint64_t* new_off);
/* fuzzer.go:567: new_k = Intersection(new_k, Canonicalize(R_k)) for sorted new_k
 * (new_vals[new_off[k] ..]) and raw re-execution signal R_k (r_vals[r_off[k]
 * ..]); the result is written at new_k's own start, out_len[k] = its length. */
int sg_triage_intersect(sg_ctx* ctx, uint32_t* new_vals, const uint64_t* new_off, const uint32_t* r_vals,
			const uint64_t* r_off, size_t n, uint64_t* out_len);
/* fuzzer.go:584-587, the minimisation predicate: ok[k] =
 * len(Intersection(new_k, Canonicalize(R_k))) == len(new_k). */
int sg_triage_subset(sg_ctx* ctx, const uint32_t* new_vals, const uint64_t* new_off, const uint32_t* r_vals,
		     const uint64_t* r_off, size_t n, uint8_t* ok);

/* syz-manager/manager.go:907-912 NewInput() signal part, over n RPCs in
 * arrival order: accepted[k] = SignalNew(corpusSignal, S_k) at its turn; on
 * accept corpusSignal ∪= S_k and corpusCover ∪= Cov_k.  cover may be NULL. */
int sg_accept_batch(sg_ctx* ctx, sg_set* corpus_sig, sg_set* corpus_cov, const uint32_t* sig_vals,
		    const uint64_t* sig_off, const uint32_t* cov_vals, const uint64_t* cov_off, size_t n,
		    uint8_t* accepted);

/* syz-manager/manager.go:949-956 Poll() maxSignal merge over npoll polls in
 * arrival order: poll k's newMaxSignal = members of A_k not yet in maxSignal,
 * first occurrences, in A_k order.  new_vals capacity a_off[npoll]; new_off
 * (npoll+1) gives each poll's slice. */
int sg_merge_poll(sg_ctx* ctx, sg_set* mgr_max, const uint32_t* a_vals, const uint64_t* a_off, size_t npoll,
		  uint32_t* new_vals, uint64_t* new_off);

/* pkg/cover/cover.go:120-146 Minimize() over corpus CSR (vals/off, n inputs)
 * processed in `order` (order[k] = input index processed k-th; the reference
 * takes it from sort.Sort of minInputArray, cover.go:128).  out_idx gets the
 * selected input indices in processing order; *nout their count. */
int sg_minimize(sg_ctx* ctx, const uint32_t* vals, const uint64_t* off, size_t n, const uint32_t* order,
		uint32_t* out_idx, size_t* nout);
/* order of cover.Minimize: Go's sort.Sort over minInputArray (Less = longer
 * first, cover.go:157), restated from the Go 1.8/1.9 sort package. */
int sg_minimize_order(const uint64_t* off, size_t n, uint32_t* order);

/* ---- RPC payloads (pkg/rpctype/rpctype.go:8-63) --------------------------- */
/* Wire form of a sorted []uint32 (RpcInput.Signal / .Cover are canonical;
 * ConnectRes.MaxSignal, PollArgs.MaxSignal and PollRes.MaxSignal are set
 * members): Go's binary.PutUvarint of the first value, then of each successive
 * difference.  A Go peer decodes it with binary.Uvarint and a running sum.
 * Batched over n lists: list k is vals[off[k] .. off[k+1]) (non-decreasing,
 * else SG_EINVAL); its bytes go to out[out_off[k] .. out_off[k+1]).  out_off
 * (n+1) is always filled; the bytes are copied only when out_off[n] <= cap
 * (cap = 5 * off[n] always suffices). */
int sg_delta_encode_batch(sg_ctx* ctx, const uint32_t* vals, const uint64_t* off, size_t n, uint8_t* out, size_t cap,
			  uint64_t* out_off);
/* The inverse: list k from in[in_off[k] .. in_off[k+1]) into vals[off[k] ..)
 * (capacity cap values; in_off[n] always suffices).  SG_EINVAL on a malformed
 * payload (a list ending inside a value, a value or running sum past 32 bits). */
int sg_delta_decode_batch(sg_ctx* ctx, const uint8_t* in, const uint64_t* in_off, size_t n, uint32_t* vals, size_t cap,
			  uint64_t* off);
/* A set's members (ascending) as one payload: fuzzer.go:358-364 (PollArgs.MaxSignal
 * from newSignal), manager.go:801-806 / :962 (ConnectRes / PollRes.MaxSignal).
 * *nbytes = payload size; bytes copied only when it is <= cap. */
int sg_set_encode(sg_set* set, uint8_t* out, size_t cap, size_t* nbytes);
/* SignalAdd of a decoded payload (fuzzer.go:146-151, :392-398); *count
 * (nullable) = values in it. */
int sg_set_decode_add(sg_set* set, const uint8_t* in, size_t nbytes, uint64_t* count);
/* tools/syz-execprog/execprog.go:159-177: the sancov file of each of n calls:
 * u64 0xC0BFFFFFFFFFFF64, then RestorePC(pc, 0xffffffff) (cover.go:23-25) per
 * cover PC, little-endian.  File k is out[8*(k + cov_off[k]) .. 8*(k+1 +
 * cov_off[k+1])) (out: 8*(n + cov_off[n]) bytes). */
int sg_sancov_batch(sg_ctx* ctx, const uint32_t* cov, const uint64_t* cov_off, size_t n, uint8_t* out);
/* (execprog.go:162-164 writes no file for a call without cover: such a call's
 * slice here is the 8-byte header alone.) */

/* ---- sorted-slice algebra (pkg/cover/cover.go:28-117) ---------------------- */
/* Canonicalize (cover.go:28-40): in place, *nout = canonical length. */
int sg_canonicalize(sg_ctx* ctx, uint32_t* v, size_t n, size_t* nout);
/* Batched Canonicalize of CSR segments in place: segment k is
 * vals[off[k] .. off[k+1]); its canonical form is written at its own start,
 * out_len[k] = its length (Go returns cov[:n], aliasing the input). */
int sg_canonicalize_batch(sg_ctx* ctx, uint32_t* vals, const uint64_t* off, size_t nseg, uint64_t* out_len);

#define SG_OP_DIFFERENCE 0 /* cover.go:42-49 */
#define SG_OP_SYMDIFF 1    /* cover.go:51-61 */
#define SG_OP_UNION 2      /* cover.go:63-70 */
#define SG_OP_INTERSECT 3  /* cover.go:72-79 */
/* op(a, b) for sorted a, b; out capacity na+nb; *nout = result length. */
int sg_merge(sg_ctx* ctx, int op, const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out,
	     size_t* nout);
/* Batched op over npair pairs: pair k is a[a_beg[k] .. +a_len[k]) op
 * b[b_beg[k] .. +b_len[k]) (pairs may share b, e.g. one corpus signal);
 * result k is written at out[out_beg[k] ..) (capacity a_len[k]+b_len[k]),
 * out_len[k] = its length.  Arrays are host pointers; a/b/out too. */
int sg_merge_batch(sg_ctx* ctx, int op, const uint32_t* a, size_t a_total, const uint64_t* a_beg,
		   const uint64_t* a_len, const uint32_t* b, size_t b_total, const uint64_t* b_beg,
		   const uint64_t* b_len, size_t npair, uint32_t* out, size_t out_total, const uint64_t* out_beg,
		   uint64_t* out_len);
/* The manager's cover.Union folds (cov = Union(cov, inp.Cover) over inputs:
 * syz-manager/html.go:84 grouped by syscall, :94, :184, :306, and the
 * same-hash merge manager.go:916-917): for each group g < ngroups, the Union
 * (cover.go:63-70) of the sorted lists k with group[k] == g (group NULL: one
 * group of all n lists) -- every value with its largest count over those
 * lists, ascending, 0xFFFFFFFF dropped.  List k is vals[off[k] .. off[k+1]).
 * Group g's fold goes to out_vals[out_off[g] .. out_off[g+1]) (out_off:
 * ngroups+1; capacity cap >= off[n] always suffices). */
int sg_union_fold(sg_ctx* ctx, const uint32_t* vals, const uint64_t* off, size_t n, const uint32_t* group,
		  size_t ngroups, uint32_t* out_vals, size_t cap, uint64_t* out_off);
/* HasDifference (cover.go:106-117): *out = 1 iff a has an element (multiset,
 * no sentinel special case) not matched in b. */
int sg_has_difference(sg_ctx* ctx, const uint32_t* a, size_t na, const uint32_t* b, size_t nb, int* out);
/* Batched HasDifference over npair pairs laid out as in sg_merge_batch (pair
 * k: a[a_beg[k] .. +a_len[k]) against b[b_beg[k] .. +b_len[k]); pairs may
 * share b): out[k] = 1 iff that a has an element not matched in that b, else
 * 0.  Host pointers. */
int sg_has_difference_batch(sg_ctx* ctx, const uint32_t* a, size_t a_total, const uint64_t* a_beg,
			    const uint64_t* a_len, const uint32_t* b, size_t b_total, const uint64_t* b_beg,
			    const uint64_t* b_len, size_t npair, uint8_t* out);

/* ---- executor edge signal (executor/executor.h:389-401, :497-526) --------- */
/* Raw per-call u32 PC traces -> per-call signal, executor-exact: edge
 * sig = pc ^ hash(prev pc) (prev = 0 at each call start), filtered through the
 * executor's lossy 8192-slot / 4-probe dedup table, one fresh table per
 * program shared by its calls in call order.  Programs own calls
 * [prog_off[p], prog_off[p+1]); call c owns pcs[call_off[c] .. call_off[c+1]).
 * Output: sig_vals (capacity call_off[ncalls]) and sig_off (ncalls+1). */
int sg_exec_signal(sg_ctx* ctx, const uint32_t* pcs, const uint64_t* call_off, const uint64_t* prog_off,
		   size_t nprog, uint32_t* sig_vals, uint64_t* sig_off);
int sg_exec_signal_dev(sg_ctx* ctx, const uint32_t* d_pcs, const uint64_t* d_call_off, const uint64_t* d_prog_off,
		       uint64_t nprog, uint64_t ncalls, uint64_t npcs, uint32_t* d_sig_vals, uint64_t* d_sig_off);
/* The executor-exact lists of the queued calls only (syz-fuzzer/fuzzer.go:678-683
 * copies inf.Signal of a record only when it is queued for triage): after a
 * set-exact triage of the same traces (sg_triage_traces_dev, flags d_rec_new),
 * call c's list is exactly sg_exec_signal_dev's when d_rec_new[c] != 0 and
 * empty otherwise.  Each program runs its calls up to its last queued one (the
 * executor's table state at a call depends only on the calls before it);
 * programs without a queued call do not run.  Layout as sg_exec_signal_dev. */
int sg_exec_signal_queued_dev(sg_ctx* ctx, const uint32_t* d_pcs, const uint64_t* d_call_off,
			      const uint64_t* d_prog_off, uint64_t nprog, uint64_t ncalls, uint64_t npcs,
			      const uint8_t* d_rec_new, uint32_t* d_sig_vals, uint64_t* d_sig_off);
/* The fuzzer's step from host traces in one call: sg_triage_traces (flags and
 * set updates, set-exact) and the executor-exact signal lists of the queued
 * calls only (sg_exec_signal_queued_dev), the traces staged once.  Calls are
 * grouped into programs by prog_off (nprog + 1, prog_off[0] == 0; the
 * executor's dedup table is per program); rec_new[c] for every call; the
 * lists in sig_vals / sig_off (ncalls + 1) as sg_exec_signal's, empty for the
 * calls not queued (fuzzer.go:678-683 copies the signal of queued calls
 * only).  sig_vals capacity: call_off[ncalls] values. */
int sg_triage_traces_queued(sg_ctx* ctx, sg_set* maxsig, sg_set* newsig, const uint32_t* pcs,
			    const uint64_t* call_off, const uint64_t* prog_off, size_t nprog, uint8_t* rec_new,
			    uint32_t* sig_vals, uint64_t* sig_off);

/* ---- synthetic Zipf traces (bench / test input generator) ----------------- */
/* Zipf(s) over `nranks` PC ranks mapped through a permutation seeded by
 * universe_seed (the "kernel text": shared by every batch) to
 * pc = 0x81000000 + 16*perm(rank); draws are counter-based
 * (splitmix64 of trace_seed and the global PC index), so any slice is
 * reproducible.  Fills d_pcs with nprog*calls*pcs_per_call PCs of programs
 * prog_base .. prog_base+nprog-1, program-major. */
int sg_gen_zipf_traces_dev(sg_ctx* ctx, uint64_t universe_seed, uint64_t trace_seed, double zipf_s, uint32_t nranks,
			   uint64_t prog_base, uint64_t nprog, uint32_t calls, uint32_t pcs_per_call, uint32_t* d_pcs);
/* A fuzzer's steady state: programs drawn from a fixed population of npop
 * programs (member m's trace is the one sg_gen_zipf_traces_dev gives program m
 * under trace seed pop_seed), re-executed with flaky coverage -- each PC is
 * replaced by a fresh Zipf draw with probability `noise`.  The member of
 * program p and its noise are counter-based in (trace_seed, p). */
int sg_gen_population_traces_dev(sg_ctx* ctx, uint64_t universe_seed, uint64_t pop_seed, uint64_t npop,
				 uint64_t trace_seed, double noise, double zipf_s, uint32_t nranks, uint64_t prog_base,
				 uint64_t nprog, uint32_t calls, uint32_t pcs_per_call, uint32_t* d_pcs);

/* ---- cover report (syz-manager/cover.go:91-103, :257-307) ----------------- */
/* pcs[i] = RestorePC(cov[i], base) - 5; returns the uncovered PC set of
 * uncoveredPcsInFuncs, ascending (the reference returns map order).
 * sym_start/sym_end sorted by start; all_pcs sorted (objdump call sites).
 * out capacity nall; *nout = count. */
int sg_cover_uncovered(sg_ctx* ctx, const uint32_t* cov, size_t ncov, uint32_t base, const uint64_t* sym_start,
		       const uint64_t* sym_end, size_t nsym, const uint64_t* all_pcs, size_t nall, uint64_t* out,
		       size_t* nout);

/* ---- executor output ingest (pkg/ipc/ipc_linux.go:168-307) ---------------- */
/* readOutCoverage over a batch of programs.  Program p's output region (the
 * layout executor/executor.h:369-427 writes) is out[out_off[p] ..
 * out_off[p+1]); its calls are records call_off[p] .. call_off[p+1]
 * (len(p.Calls)); call_nums[r] = c.Meta.ID of record r, or NULL to skip that
 * check (ipc_linux.go:225-230).  Per record: err = Errno (-1 = not executed,
 * else the executor's u32 errno), fault = FaultInjected, its Signal words at
 * sig_vals[sig_off[r] .. sig_off[r+1]) and, when cov_off / cov_vals are
 * given, its Cover words likewise.  Comparisons are walked, not decoded.
 * status[p] = SG_IPC_OK or the Go error path the reader took; the records
 * keep what the reader had set before it (partial info, as in Go).
 * sig_vals / cov_vals capacity: out_off[nprog] words always suffices.
 * Record order is program-major, call index ascending (fuzzer.go:665). */
#define SG_IPC_OK 0
#define SG_IPC_NO_NCMD 1      /* ipc_linux.go:197-200 */
#define SG_IPC_SHORT_HEADER 2 /* :216-219 */
#define SG_IPC_BAD_INDEX 3    /* :220-224 */
#define SG_IPC_BAD_CALLNUM 4  /* :225-230 */
#define SG_IPC_DOUBLE 5       /* :231-235 */
#define SG_IPC_SIGNAL_SIZE 6  /* :238-242 */
#define SG_IPC_COVER_SIZE 7   /* :247-251 */
#define SG_IPC_COMPS_SHORT 8  /* :258-290 */
#define SG_IPC_COMPS_TYPE 9   /* :266-270 */
int sg_ipc_parse(sg_ctx* ctx, const uint32_t* out, const uint64_t* out_off, const uint64_t* call_off,
		 const uint32_t* call_nums, size_t nprog, int64_t* err, uint8_t* fault, int32_t* status,
		 uint64_t* sig_off, uint32_t* sig_vals, uint64_t* cov_off, uint32_t* cov_vals);
/* Device form: every pointer is device memory, stream-ordered, no host sync. */
int sg_ipc_parse_dev(sg_ctx* ctx, const uint32_t* d_out, const uint64_t* d_out_off, const uint64_t* d_call_off,
		     const uint32_t* d_call_nums, uint64_t nprog, uint64_t nrec, int64_t* d_errno, uint8_t* d_fault,
		     int32_t* d_status, uint64_t* d_sig_off, uint32_t* d_sig_vals, uint64_t* d_cov_off,
		     uint32_t* d_cov_vals);

#ifdef __cplusplus
}
#endif

#endif /* SYZSIG_H */
