// sg_internal.h -- shared host/device plumbing of libsyzsig.so (not installed).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/syzsig.h"

namespace sg {

// 2^32-bit direct-indexed signal bitmap: 2^27 words = 512 MiB.
constexpr uint64_t kSetWords = 1ull << 27;
constexpr uint64_t kSetBytes = kSetWords * 4;
// First-owner table: one u32 key per possible signal value = 16 GiB.
constexpr uint64_t kOwnerEntries = 1ull << 32;
constexpr uint32_t kOwnerInf = 0xFFFFFFFFu;
// Records per launch of the partitioned triage (256 groups of 2^16 records);
// larger batches run as consecutive record slices (sg_bucket.hip).
constexpr uint64_t kMaxLaunchRecords = 1ull << 24;

// Element tiles of the streaming kernels: 256 threads, one uint4 (4 values)
// per lane per step, 4 steps per wave -> 4096 values per workgroup tile;
// a "chunk" is one wave-instruction's 256 values and carries a 4 x u64
// ballot mask (bit l of word k <-> value 4l+k of the chunk).
constexpr int kBlock = 256;
constexpr int kChunk = 256;
constexpr int kTile = 4096;
constexpr int kChunksPerTile = kTile / kChunk;  // 16
constexpr int kWin = 1024;                      // record-offset window kept in LDS per tile

void set_error(const char* fmt, ...);

struct KernelTimer {
  bool enabled = false;
  struct Rec {
    int id;
    hipEvent_t a, b;
  };
  std::vector<Rec> pending;
  std::vector<hipEvent_t> pool;
  std::map<std::string, int> ids;
  std::vector<std::string> names;
  std::vector<double> ms;
  std::vector<uint64_t> count;
};

}  // namespace sg

// one record slice of a two-phase (prefix) triage: records [r0, r1),
// entries [e0, e1), its partition at workspace offset ws_base
struct PrefixSlice {
  uint64_t r0, r1, e0, e1;
  size_t ws_base;
};

// One kept batch of the two-phase triage: its record slices and their
// partitions (or, with option prefix_pairs, its first-owner pairs), in a workspace of
// its own (two slots, so one batch's exchange can run while the next one is
// partitioned)
struct PrefixSlot {
  std::vector<PrefixSlice> slices;
  uint64_t nrec = 0;
  uint64_t n = 0;              // signal entries of the batch (bounds the pairs)
  uint32_t* marks = nullptr;   // begin's marks (end's set updates)
  bool keep = false;           // partitions kept instead of pairs
  bool open = false;
  void* ws = nullptr;
  size_t ws_cap = 0;
};
constexpr uint32_t kPrefixSlots = 2;

// Context options (sg_ctx_set_option): each regime selects its own path, and
// an option only forces one, for a test or a measurement.  -1 = the regime's
// choice.  No option is read from the environment on a call; sg_ctx_create
// seeds the diagnostics ones (debug_part, bucket_blocks, prefix_pairs) from
// SG_DEBUG_PART / SG_BUCKET_BLOCKS / SG_PREFIX_PAIRS for the GPU scripts.
enum SgOpt : int {
  kOptBucketBlocks = 0,     // cap of the persistent bucket grid (0: none)
  kOptPrefixPairs,          // prefix_begin's form when the caller passes -1 (0 kept partitions, 1 pairs)
  kOptFoldMap,              // one-group fold: -1 by range, 0 never the byte map
  kOptMinimizeFilter,       // Minimize's value filter: 1 on, 0 off
  kOptMinimizeFilterRanks,  // Minimize phase A length (0: the default)
  kOptReportDirect,         // cover report: 1 the global-search form at any size
  kOptRpcEncodeElems,       // delta encode: -1 by shape, 0 per-list, 1 per-element
  kOptRpcDecodeBlocks,      // delta decode: -1 by shape, 0 per-list, 1 per-block
  kOptHostSlice,            // host ingest: entries per record slice (0: the default)
  kOptHostCopyThreads,      // host ingest: pageable -> pinned copy threads (0: from the CPU quota)
  kOptM0Filter,             // flags path: the M0 filter (sg_bucket.hip): -1 by the last batches, 0 never, 1 always tried
  kOptM0Halves,             // the filter's index per slice in 2^k parts (-1 by its fill, 0..2 forced)
  kOptCount
};

struct sg_ctx {
  int device = 0;
  int64_t opt[kOptCount] = {0, 0, -1, 1, 0, 0, -1, -1, 0, 0, -1, -1};
  // the M0 filter's buffers (lazy, sg_bucket.hip) and its regime state: the
  // last record slice's outcome (1 filtered, 0 partitioned), the queued
  // records of the last partitioned slice (counted on the device, read back
  // through m0f_host once m0f_ev has passed: no host wait) and its record
  // count; slices it filtered and fell back on (counters)
  void* m0f = nullptr;
  uint32_t* m0f_host = nullptr;  // pinned: the queued-record count
  hipEvent_t m0f_ev = nullptr;
  int m0f_last = -1;             // -1 nothing yet
  bool m0f_pending = false;
  uint64_t m0f_nrec = 0;
  double m0f_queued = -1;        // queued fraction of the last partitioned slice (-1 unknown)
  uint64_t m0f_used = 0, m0f_fallback = 0, m0f_survivors = 0;
  uint32_t m0f_backoff = 0, m0f_skip = 0;
  int m0f_logh = 0;  // auto: the index in 2^m0f_logh parts per slice (raised when a slice's index overflows)  // auto: slices not to try after fallbacks (doubling, <= 64)
  // host CPUs this process may use (cgroup cpu.max quota, else the affinity
  // mask), read at creation: sizes the host ingest's copy threads
  double cpu_quota = 0;
  // the host ingest's last call (sg_host.hip): bytes copied pageable -> pinned,
  // the wall time of those copies and of its waits for the staging slots'
  // DMA, and the copy threads used
  uint64_t host_copy_bytes = 0, host_copy_ns = 0, host_wait_ns = 0, host_threads = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  // grow-only device workspace and pinned host staging
  void* ws = nullptr;
  size_t ws_cap = 0;
  void* pin = nullptr;
  size_t pin_cap = 0;
  // grow-only device staging for the host entry points' inputs / outputs
  void* dstage = nullptr;
  size_t dstage_cap = 0;
  // the host ingest pipeline (sg_host.hip): its copy stream and the events
  // between the two staging slots' DMA and triage
  hipStream_t copy_stream = nullptr;
  hipEvent_t pipe_ev[4] = {};
  // first-owner table and its decreasing key floor; the key space is 2^32 - 1
  // (option owner_key_space lowers it, so tests reach the generation reset)
  uint32_t* owner = nullptr;
  uint64_t owner_floor = 0;
  uint64_t owner_key_space = 0xFFFFFFFFull;
  uint64_t owner_resets = 0;
  // partitioned triage: records per launch (option max_launch_records lowers
  // it, for tests of the record slicing) and diagnostics (option debug_part)
  uint64_t max_launch_recs = 0;
  // two-phase triage state (prefix_begin / prefix_end, sg_bucket.hip)
  PrefixSlot prefix[kPrefixSlots];
  bool debug_part = false;
  // rebased record offsets of record slices (grow-only, owned)
  uint64_t* slice_off = nullptr;
  size_t slice_off_cap = 0;
  // a batch's record-slice cuts, found on the device (sg_bucket.hip k_slice_cuts)
  uint64_t* slice_cuts = nullptr;
  // small device scalars (counters / flags)
  uint64_t* dscal = nullptr;
  // cached Zipf generator tables (alias method + rank->pc permutation)
  uint32_t* gen_prob = nullptr;
  uint32_t* gen_alias = nullptr;
  uint32_t* gen_perm = nullptr;
  uint64_t gen_seed = 0;
  double gen_s = 0;
  uint32_t gen_nranks = 0;
  sg::KernelTimer timer;
  std::mutex mu;
};

struct sg_set {
  sg_ctx* ctx = nullptr;
  uint32_t* words = nullptr;
  bool owned = true;
};

namespace sg {

// ---- host helpers (sg_ctx.hip) ----
int hip_fail(hipError_t e, const char* what);
#define SG_HIP(call)                                     \
  do {                                                   \
    hipError_t e_ = (call);                              \
    if (e_ != hipSuccess) return ::sg::hip_fail(e_, #call); \
  } while (0)

int ensure_device(sg_ctx* ctx);
// Carve `n` bump-allocated regions out of the workspace (each 256-B aligned).
struct WsPlan {
  size_t off[32];
  int n = 0;
  size_t total = 0;
  size_t add(size_t bytes) {
    size_t o = total;
    off[n++] = o;
    total += (bytes + 255) & ~size_t(255);
    return o;
  }
};
int ws_reserve(sg_ctx* ctx, size_t bytes);
inline void* ws_at(sg_ctx* ctx, size_t off) { return (char*)ctx->ws + off; }
int pin_reserve(sg_ctx* ctx, size_t bytes);
int dstage_reserve(sg_ctx* ctx, size_t bytes);
// Reserve `nkeys` first-owner keys: returns key_lo such that keys
// key_lo .. key_lo+nkeys-1 are below every key already stored in the table.
int owner_keys(sg_ctx* ctx, uint64_t nkeys, uint32_t* key_lo);

// Kernel timing around launches on ctx->stream.
void timer_begin(sg_ctx* ctx, const char* name, int* slot);
void timer_end(sg_ctx* ctx, int slot);
struct ScopedTimer {
  sg_ctx* c;
  int slot = -1;
  ScopedTimer(sg_ctx* ctx, const char* name) : c(ctx) { timer_begin(ctx, name, &slot); }
  ~ScopedTimer() { timer_end(c, slot); }
};

inline uint32_t div_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// Device exclusive scan of u32 counts into u64 offsets, out[n] = total
// (sg_scan.hip).  Uses the workspace tail beyond `ws_used`.
int scan_counts(sg_ctx* ctx, const uint32_t* d_in, uint64_t* d_out, uint64_t n, size_t ws_used);
size_t scan_ws_bytes(uint64_t n);

// Members of a set, ascending, into device memory (sg_ctx.hip; ctx lock held).
int set_export_dev(sg_set* set, uint32_t* d_out, uint64_t cap, uint64_t* total);
// SignalAdd of device-resident values (sg_ctx.hip; ctx lock held, stream-ordered).
int set_add_dev_locked(sg_set* set, const uint32_t* d_vals, uint64_t n);

// A batch in host memory through pinned double-buffered staging, record
// slice by record slice, each slice's copies overlapping the previous one's
// partitioned triage (sg_host.hip); takes the ctx lock.
double host_cpu_quota();
int host_copy_threads(const sg_ctx* ctx);
int host_pipeline(sg_ctx* ctx, uint32_t* mwords, uint32_t* nwords, const uint32_t* vals, const uint64_t* rec_off,
                  uint64_t nrec, uint8_t* rec_new, bool trace);
// Partitioned flags-only triage (sg_bucket.hip); ctx lock held.  trace:
// d_vals are raw per-call PC traces, triaged by their edge signal.
int bucket_triage(sg_ctx* ctx, uint32_t* mwords, uint32_t* nwords, const uint32_t* d_vals, const uint64_t* d_off,
                  uint64_t n, uint64_t nrec, uint8_t* d_rec_new, bool trace = false);
// Candidate emission of the partitioned path (sharded triage, sg_shard.hip;
// the prefix protocol's pair form): each distinct s not in the snapshot, once
// per launch, as {s, rec_base + first record}, counted per owning shard when
// shard_cnt is given.
struct EmitArgs {
  uint2* pairs;
  unsigned long long* npairs;
  uint32_t rec_base;
  uint32_t nshards;
  unsigned long long* shard_cnt;
  bool update;  // also update the sets (their new bits = the emitted signals); no record flags
  unsigned long long* gcur;  // update form: pairs group-major, group g's at goff[g << 16] + gcur[g]++
  const uint64_t* goff;      //   (goff: the launch's record offsets)
};
// Workgroups of `kernel` resident on the whole device at once (cached per device).
uint32_t persistent_grid(sg_ctx* ctx, const void* kernel, int threads);
// d_out[i] = d_off[i] - base, i < n (a record slice's offsets rebased).
int rebase_offsets(sg_ctx* ctx, const uint64_t* d_off, uint64_t n, uint64_t base, uint64_t* d_out);
// Workspace bytes of one partitioned launch over n entries / nrec records.
size_t bucket_plan_bytes(uint64_t n, uint64_t nrec);
// A batch's record slices (<= max_launch_recs records, <= lim entries unless
// one record alone holds more), as {r0, r1, e0, e1} quadruples: cuts found on
// the device, one wait (sg_bucket.hip k_slice_cuts).
int record_slice_cuts(sg_ctx* ctx, const uint64_t* d_off, uint64_t nrec, uint64_t lim, std::vector<uint64_t>& cuts);
// Two-phase triage (sg_bucket.hip): begin ORs into marks_words the batch's
// signal not in base_words and keeps the batch's partitions (or each such
// signal's first record) in the slot; end flags the records against
// mwords | owords and, with `update`, updates mwords / nwords.
// form: 0 kept partitions, 1 first-owner pairs, -1 from option prefix_pairs; d_ncand
// (nullable, device): the batch's distinct signals not in base_words.
int prefix_begin(sg_ctx* ctx, uint32_t slot, const uint32_t* base_words, uint32_t* marks_words, const uint32_t* d_vals,
                 const uint64_t* d_off, uint64_t n, uint64_t nrec, int form = -1, uint64_t* d_ncand = nullptr);
int prefix_end(sg_ctx* ctx, uint32_t slot, uint32_t* mwords, const uint32_t* owords, uint32_t* nwords, uint8_t* d_rec_new,
               bool update);
// One emitting launch (nrec <= kMaxLaunchRecords, n < 2^32 - 2^15), scratch
// at ws_base (reserved by the caller).
int bucket_emit(sg_ctx* ctx, const uint32_t* mwords, const uint32_t* d_vals, const uint64_t* d_off, uint64_t n,
                uint64_t nrec, const EmitArgs& emit, size_t ws_base);
// The ordered outputs' bucket stage (one launch, limits as bucket_emit):
// mwords / nwords (nullable) gain the batch's new signals, and each new
// signal is written once as {s, its first record} (records launch-relative),
// group-major: the pairs of record group g (records g << 16 ..) at
// pairs[d_off[g << 16] + i], i < gcur[g] (device, zeroed by the caller; a
// group's new signals never outnumber its entries); no record flags.
int bucket_emit_update(sg_ctx* ctx, uint32_t* mwords, uint32_t* nwords, const uint32_t* d_vals, const uint64_t* d_off,
                       uint64_t n, uint64_t nrec, uint2* pairs, unsigned long long* gcur, size_t ws_base);
constexpr uint32_t kRecGroupBits = 16;  // records per group of the partitioned path: 2^16
// Workspace bytes beyond two key buffers of radix_sort_u64 (sg_sort.hip).
size_t radix_sort_ws(uint64_t n);
int radix_sort_u64(sg_ctx* ctx, uint64_t* a, uint64_t* b, uint64_t n, size_t ws_used, uint64_t** sorted,
                   uint64_t vary = 0);
// One stable radix pass over keys in runs of a gapped buffer (run order kept
// within a digit), written contiguously into dst (sg_sort.hip; syncs).
int radix_pass_runs(sg_ctx* ctx, const uint64_t* src, const std::vector<uint64_t>& run_start,
                    const std::vector<uint64_t>& run_cnt, uint32_t shift, uint64_t* dst, size_t ws_used);
size_t radix_pass_runs_ws(uint64_t n, uint64_t nruns);

}  // namespace sg

// ---- device helpers -------------------------------------------------------
namespace sgd {

// Layout of a set's 2^32-bit bitmap: signal s = bytes (b3 b2 b1 b0) is bit
// set_pos(s) = (b2 b1 b3 b0).  The low 5 bits are s's own, so this is a fixed
// permutation of 32-bit words; 8 consecutive words (256 signals, one b0 range)
// stay together.  It makes the 2^16 signals of one (b2, b1) -- the partitioned
// triage's bucket (sg_bucket.hip) -- one contiguous 8 KiB slice: the raw top
// byte of an edge signal is the top byte of hash(prev PC) and would pile the
// edges of the hottest PCs into a few buckets.  Export walks the words in s
// order (sg_ctx.hip), so members still come out ascending.
__host__ __device__ __forceinline__ uint32_t set_pos(uint32_t s) {
  return ((s & 0x00FFFF00u) << 8) | ((s >> 16) & 0xFF00u) | (s & 0xFFu);
}
__host__ __device__ __forceinline__ uint32_t set_sig(uint32_t p) {  // inverse of set_pos
  return ((p & 0xFF00u) << 16) | ((p >> 8) & 0x00FFFF00u) | (p & 0xFFu);
}
// word of the bitmap holding s-order word ws (= s >> 5)
__host__ __device__ __forceinline__ uint32_t set_word(uint32_t ws) {
  return (((ws >> 3) & 0xFFFFu) << 11) | ((ws >> 19) << 3) | (ws & 7u);
}
// The executor's edge hash (executor/executor.h:497-505): an edge's signal
// is pc ^ hash(previous pc of the call), 0 before the call's first pc
// (executor.h:392-396).
__host__ __device__ __forceinline__ uint32_t exec_hash(uint32_t a) {
  a = (a ^ 61) ^ (a >> 16);
  a = a + (a << 3);
  a = a ^ (a >> 4);
  a = a * 0x27d4eb2du;
  a = a ^ (a >> 15);
  return a;
}

__device__ __forceinline__ bool test_bit(const uint32_t* words, uint32_t s) {
  return (words[set_pos(s) >> 5] >> (s & 31)) & 1u;
}
__device__ __forceinline__ void set_bit(uint32_t* words, uint32_t s) {
  atomicOr(&words[set_pos(s) >> 5], 1u << (s & 31));
}

// largest r in [lo, hi] with off[r] <= i (off non-decreasing), searched in
// `off` (global or LDS pointer).
template <typename P>
__device__ __forceinline__ uint64_t seg_search(P off, uint64_t lo, uint64_t hi, uint64_t i) {
  while (lo < hi) {
    uint64_t mid = lo + (hi - lo + 1) / 2;
    if (off[mid] <= i)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

// Inclusive wave64 scans through DPP: row shifts within the 16-lane rows,
// then the row broadcasts of lanes 15 and 31 (no LDS-crossbar shuffles; the
// per-tile scans of the partition and merge kernels run on one wave while
// the others wait at a barrier).
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}

// the same for max over values >= -1 (-1: nothing yet)
__device__ __forceinline__ int wave_incl_max(int x) {
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xF, 0xF, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x112, 0xF, 0xF, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x114, 0xF, 0xF, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x118, 0xF, 0xF, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x142, 0xA, 0xF, false));
  x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x143, 0xC, 0xF, false));
  return x;
}

}  // namespace sgd
