// sg_bucket.hip -- partitioned new-signal triage (the fast path of
// sg_triage_batch when the caller does not ask for the ordered diff lists).
//
// Reference: syz-fuzzer/fuzzer.go:645-693.  Its observable results are which
// call records get queued for triage (fuzzer.go:678-690) and the updated
// maxSignal / newSignal (fuzzer.go:673-674); the diff slice (fuzzer.go:669)
// is a transient that only feeds those SignalAdd calls.
//
// Same first-owner rule as sg_triage.hip: a record is new iff it is the
// first, in sequential order, to contain some signal s not in maxSignal.
// Owners are minima over record indices, so the order of entries inside a
// partition never matters; what has to travel with each entry is its record.
// Every stream here is 4 bytes per signal entry:
//
//   tiles   the batch is cut into pass-1 tiles of <= kPT entries that span
//           <= kRecCap records (cuts at every kPT-th entry and at every
//           kRecCap-th record offset), so an entry's record is
//           trec[tile] + an 8-bit in-tile index;
//   groups  records in runs of 2^16 (group g = records [g << 16, +2^16));
//           every group boundary is a kRecCap-th record offset, hence a
//           tile cut, so a group is a run of whole tiles [gt[g], gt[g+1]);
//   pass 1  partition by the top byte of s (256 slices of 2^24 signals):
//           entry = s << 8 | rec_in_tile, runs laid out [slice][tile];
//   pass 2  per (slice, group), cut into chunks of <= kPT entries;
//           partition by bits 16..23 of s: entry = (s & 0xFFFF) << 16 |
//           record_in_group, runs laid out [byte][chunk];
//   bucket  one workgroup per 2^16-signal bucket (d, f): its 8 KiB maxSignal
//           slice in LDS is the new-signal test; a candidate (s not in
//           maxSignal) at bucket position i has record (group(i) << 16) |
//           (entry & 0xFFFF), group(i) from the bucket's group boundaries,
//           and goes into an LDS hash map s -> min(record).  The
//           bucket's new bits go back to maxSignal / newSignal from their
//           only writer.  Buckets whose distinct candidates overflow the map
//           are redone by a direct-table kernel.
// Each partition pass = a byte histogram per tile (LDS counters) + a device
// exclusive scan + a scatter (tile in registers, LDS counting-rank, staged
// by digit, written in digit runs).  No global atomics on the data path, no
// random HBM access, no 16 GiB owner table.
//   M0 filter (low-novelty batches, "M0 filter" below): between pass 1 and
//           pass 2, each slice's run tested against a packed index of the
//           slice's maxSignal in LDS; only the survivors go on, to a small
//           exact tail, and pass 2 and the bucket stage do not run.
#include "sg_internal.h"

#include <algorithm>

#ifndef SG_EXP
#define SG_EXP 0  // diagnostics builds only
#endif


namespace sg {

#ifndef SG_HT_ABL
#define SG_HT_ABL 0
#endif
#ifndef SG_PT
#define SG_PT 16384
#endif
#ifndef SG_PTHREADS
#define SG_PTHREADS 1024
#endif
constexpr int kPT = SG_PT;                   // entries per partition tile / chunk
constexpr int kPThreads = SG_PTHREADS;       // 16 waves
constexpr int kPWaves = kPThreads / 64;
constexpr int kPerWave = kPT / kPWaves;      // 1024 entries per wave, in order
constexpr int kSteps = kPerWave / 64;        // 16 entries per lane
// Partition key.  The passes and buckets work on t = set_pos(s), the
// position of s in a set's bitmap (sg_internal.h): bytes (b2 b1 b3 b0) of
// s = (b3 b2 b1 b0).  Pass 1 partitions by b2, pass 2 by b1, and a bucket
// holds the 2^16 signals of one (b2, b1): bitmap words [b << 11, +2048), its
// LDS slice bit for t is t & 0xFFFF.
// Entry layouts.  Pass 1: t << 8 | record-in-tile (kRecCap records per tile
// at most).  Pass 2: (t & 0xFFFF) << 16 | record-in-group.
constexpr uint32_t kRecCap = 256;              // records per pass-1 tile
constexpr uint32_t kGroupBits = 16;
constexpr uint32_t kGroupRecs = 1u << kGroupBits;  // records per group
constexpr uint32_t kMaxGroups = 256;           // groups per launch (larger batches run in record slices)
static_assert(kGroupRecs % kRecCap == 0, "group boundaries must be tile cuts");
constexpr uint32_t kNumBuckets = 1u << 16;   // (top byte, second byte) of s
constexpr uint32_t kBucketWords = 2048;      // 2^16 signals
#ifndef SG_BTHREADS
#define SG_BTHREADS 512
#endif
constexpr int kBThreads = SG_BTHREADS;     // bucket-kernel workgroup
constexpr int kBWaves = kBThreads == 512 ? 6 : 8;  // waves per SIMD it is built for
constexpr int kBU = 4;                       // entries per thread per round in the bucket kernel
constexpr uint32_t kHash = 8192;             // candidate map slots per bucket (32 bits each, see map_insert)
constexpr uint32_t kMaxProbe = 31;           // linear-probe cap before a bucket spills
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

__host__ __device__ __forceinline__ uint32_t part_key(uint32_t s) { return sgd::set_pos(s); }
__host__ __device__ __forceinline__ uint32_t part_sig(uint32_t t) { return sgd::set_sig(t); }
__host__ __device__ __forceinline__ uint32_t p1_digit(uint32_t s) { return (s >> 16) & 0xFFu; }  // part_key(s) >> 24
// maxSignal word holding bucket b's LDS slice word j
__host__ __device__ __forceinline__ uint64_t bucket_word(uint32_t b, uint32_t j) {
  return ((uint64_t)b << 11) | j;
}

// Blocks sharing an XCD (bid % 8 under round-robin dispatch) get a contiguous
// run of tiles, so partial lines at the seams of neighbouring tiles' digit
// runs merge in one L2.  A bijection on [0, g) for any g (speed only).
__device__ __forceinline__ uint32_t xcd_tile(uint32_t bid, uint32_t g) {
  const uint32_t x = bid & 7, q = g >> 3, r = g & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// ------------------------------------------------------------- tile cuts ---
// Pass-1 tiles: sorted merge of A = {i * kPT : i < nA} and B = {rec_off[(j +
// 1) * kRecCap] : j < nB} (both non-decreasing; ties put A first).
// start[rank] = cut position (start[nA + nB] = n), aux[rank] = record holding
// the entry at the cut.  Coinciding cuts give empty tiles.
struct Cuts {
  uint64_t nA, step, nB, n;
  const uint64_t* rec_off;
  uint64_t nrec;
  uint32_t* start;
  uint32_t* aux;
  __device__ __forceinline__ uint64_t B(uint64_t j) const { return rec_off[(j + 1) * kRecCap]; }
  // #{j : B[j] < x}
  __device__ __forceinline__ uint64_t countB(uint64_t x) const {
    uint64_t lo = 0, hi = nB;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (B(mid) < x)
        lo = mid + 1;
      else
        hi = mid;
    }
    return lo;
  }
};

__global__ void k_cuts(Cuts c) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t total = c.nA + c.nB;
  if (i > total) return;
  if (i == total) {
    c.start[total] = (uint32_t)c.n;
    return;
  }
  uint64_t x, rank;
  if (i < c.nA) {
    x = i * c.step;
    rank = i + c.countB(x);
  } else {
    const uint64_t j = i - c.nA;
    x = c.B(j);
    const uint64_t a = x / c.step + 1;
    rank = j + (a < c.nA ? a : c.nA);
  }
  c.start[rank] = (uint32_t)x;
  // record holding entry x (largest r with rec_off[r] <= x)
  const uint64_t xe = x < c.n ? x : (c.n ? c.n - 1 : 0);
  c.aux[rank] = (uint32_t)sgd::seg_search(c.rec_off, 0, c.nrec - 1, xe);
}

// Group g's first tile: the rank of the record cut at rec_off[g << 16] (cut
// j = g * kGroupRecs / kRecCap - 1 of B; see k_cuts); gt[NG] = T.
__global__ void k_group_tiles(const uint64_t* __restrict__ rec_off, uint64_t nA, uint32_t NG, uint32_t T,
                              uint32_t* __restrict__ gt) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g > NG) return;
  if (g == 0 || g == NG) {
    gt[g] = g ? T : 0u;
    return;
  }
  const uint64_t a = rec_off[(uint64_t)g * kGroupRecs] / kPT + 1;
  gt[g] = (uint32_t)((uint64_t)g * (kGroupRecs / kRecCap) - 1 + (a < nA ? a : nA));
}

// Pass-2 slice-groups: j = (slice j / NG, group j % NG) covers
// [gstart(j), gstart(j + 1)) of the pass-1 output (gt[NG] = T makes gstart(ng)
// the end); it is cut into ceil(size / kPT) chunks (none when empty).
__device__ __forceinline__ uint32_t group_start(const uint32_t* goff1, uint32_t T, uint32_t NG, const uint32_t* gt,
                                                uint64_t j) {
  return goff1[(j / NG) * T + gt[j % NG]];
}

__global__ void k_group_chunks(const uint32_t* __restrict__ goff1, uint32_t T, uint32_t NG,
                               const uint32_t* __restrict__ gt, uint64_t ng, uint32_t* __restrict__ nch) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ng) return;
  const uint32_t sz = group_start(goff1, T, NG, gt, j + 1) - group_start(goff1, T, NG, gt, j);
  nch[j] = (sz + kPT - 1) / kPT;
}

// cbase = exclusive scan of nch (cbase[ng] = number of chunks G).  Writes the
// chunk list (start, slice-group) for c < G, start = n for G <= c <= gmax (the
// launch grids use gmax, an upper bound known on the host; n = the pass-1
// total, goff1[256 T], which is below the input count when a trace batch
// drops zero edges), and cfirst[d] = first chunk of slice d (cfirst[256] = G).
__global__ void k_chunk_list(const uint32_t* __restrict__ goff1, uint32_t T, uint32_t NG,
                             const uint32_t* __restrict__ gt, uint64_t ng,
                             const uint32_t* __restrict__ cbase, uint64_t gmax, uint32_t* __restrict__ cstart,
                             uint32_t* __restrict__ cgov, uint32_t* __restrict__ cfirst) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t G = cbase[ng], n = goff1[256ull * T];
  if (i < ng) {
    const uint32_t g0 = group_start(goff1, T, NG, gt, i), g1 = group_start(goff1, T, NG, gt, i + 1);
    uint32_t c = cbase[i];
    for (uint32_t e = g0; e < g1; e += kPT, c++) {
      cstart[c] = e;
      cgov[c] = (uint32_t)i;
    }
  }
  if (i >= G && i <= gmax) {
    cstart[i] = n;
    cgov[i] = (uint32_t)(ng - 1);
  }
  if (i <= 256) cfirst[i] = i < 256 ? cbase[i * NG] : G;
}

// last t in [lo, hi) with row[t] <= x (row non-decreasing, row[lo] <= x)
__device__ __forceinline__ uint32_t last_le(const uint32_t* row, uint32_t lo, uint32_t hi, uint32_t x) {
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (row[mid] <= x)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// Per pass-2 block (the grid is the host bound gmax): desc = {start, end,
// slice-group, chunk} of chunk xcd_tile(bid, G) for bid < G, empty past G;
// dtile = the pass-1 tiles [first, last + 1) whose runs the chunk holds.
// Lets the pass-2 kernels start their data loads after one load.
__global__ void k_chunk_desc(const uint32_t* __restrict__ cstart, const uint32_t* __restrict__ cgov,
                             const uint32_t* __restrict__ gcount, uint64_t gmax, const uint32_t* __restrict__ goff1,
                             uint32_t T, uint32_t NG, const uint32_t* __restrict__ gt, uint4* __restrict__ desc,
                             uint2* __restrict__ dtile) {
  const uint64_t bid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (bid >= gmax) return;
  const uint32_t G = *gcount;
  if (bid < G) {
    const uint32_t c = xcd_tile((uint32_t)bid, G), s0 = cstart[c], s1 = cstart[c + 1], j = cgov[c];
    const uint32_t* row = goff1 + (uint64_t)(j / NG) * T;
    const uint32_t lo = gt[j % NG], hi = gt[j % NG + 1];
    desc[bid] = make_uint4(s0, s1, j, c);
    dtile[bid] = make_uint2(last_le(row, lo, hi, s0), last_le(row, lo, hi, s1 - 1) + 1);
  } else {
    desc[bid] = make_uint4(0, 0, 0, 0);
    dtile[bid] = make_uint2(0, 0);
  }
}

// --------------------------------------------------------- byte histogram ---
// hist[(v >> 24) * ncols + col] = count over one job's entries [s0, s1).
// Pass 1: job = tile t = xcd_tile(bid, T), [start[t], start[t+1]), T columns.
// Pass 2: job = the block's chunk descriptor, *ncols_dev columns; blocks
// without a chunk exit.  16-B aligned input (always, for pass 2) goes through
// k_hist_rep; k_p1_hist covers an unaligned caller buffer.
constexpr int kHistQ = kPT / 4 / kPThreads;  // uint4 loads per lane

__global__ __launch_bounds__(kPThreads) void k_p1_hist(const uint32_t* __restrict__ v,
                                                       const uint32_t* __restrict__ start, uint32_t* __restrict__ hist) {
  __shared__ uint32_t cnt[256];
  const uint32_t ncols = gridDim.x, t = xcd_tile(blockIdx.x, ncols), s0 = start[t], s1 = start[t + 1];
  const int tid = threadIdx.x;
  if (tid < 256) cnt[tid] = 0;
  uint32_t x[kPT / kPThreads];
#pragma unroll
  for (int k = 0; k < kPT / kPThreads; k++) {
    const uint32_t e = s0 + k * kPThreads + tid;
    x[k] = e < s1 ? v[e] : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPT / kPThreads; k++)
    if (s0 + k * kPThreads + tid < s1) atomicAdd(&cnt[p1_digit(x[k])], 1u);
  __syncthreads();
  if (tid < 256) hist[(uint64_t)tid * ncols + t] = cnt[tid];
}

// Aligned-input histogram jobs: [s0, s1) of the input, output column col.
struct HistJob {
  uint32_t s0, s1, col;
};

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

struct HistRegs {
  uint4 x[kHistQ + 1];
  uint32_t y;
};

// threads 0-2 take the entries before quad q0, threads 3-5 those after quad q1
__device__ __forceinline__ uint32_t hist_edge(const HistJob& h, int tid) {
  const uint32_t q0 = (h.s0 + 3) >> 2, q1 = h.s1 >> 2;
  if (tid < 3) return h.s0 + tid < q0 * 4 && h.s0 + tid < h.s1 ? h.s0 + tid : 0xFFFFFFFFu;
  if (tid < 6) {
    const uint32_t e = q1 * 4 + (tid - 3);
    return e < h.s1 && e >= h.s0 && q1 >= q0 ? e : 0xFFFFFFFFu;
  }
  return 0xFFFFFFFFu;
}

// Unconditional buffer loads: the descriptor spans exactly the job's whole
// quads (resp. its entries), and the range check returns 0 past the end.
__device__ __forceinline__ void hist_load(const uint32_t* __restrict__ v, const HistJob& h, int tid, HistRegs& r) {
  const uint32_t s0 = rfl(h.s0), s1 = rfl(h.s1);
  const uint32_t q0 = (s0 + 3) >> 2, q1 = s1 >> 2;
  const uint32_t qbytes = q1 > q0 ? (q1 - q0) * 16u : 0u;
  const __amdgpu_buffer_rsrc_t rq =
      __builtin_amdgcn_make_buffer_rsrc((void*)(v + (uint64_t)q0 * 4), 0, (int)qbytes, 0x00020000);
#pragma unroll
  for (int k = 0; k <= kHistQ; k++) {
    const v4u32 t = __builtin_amdgcn_raw_buffer_load_b128(rq, (uint32_t)(k * kPThreads + tid) * 16u, 0, 0);
    r.x[k] = make_uint4(t[0], t[1], t[2], t[3]);
  }
  const __amdgpu_buffer_rsrc_t re =
      __builtin_amdgcn_make_buffer_rsrc((void*)(v + s0), 0, (int)((s1 - s0) * 4u), 0x00020000);
  const uint32_t e = hist_edge(h, tid);
  r.y = __builtin_amdgcn_raw_buffer_load_b32(re, (e - s0) * 4u, 0, 0);
}

// Bank-replicated counting: 32 copies of the 256 counters, copy = lane & 31,
// laid out so that counter (d, copy) sits in LDS bank copy: the 32 lanes of
// a half-wave always hit 32 distinct banks (a shared 256-counter table sees
// ~3.5-way conflicts per half-wave on random digits).  The copies are summed
// per digit at the end, each lane starting at a different copy.
// digit of an input value: pass 1 reads signals (p1_digit), pass 2 pass-1 entries (top byte)
template <bool kP2>
__device__ __forceinline__ uint32_t hist_digit(uint32_t x) { return kP2 ? x >> 24 : p1_digit(x); }

template <bool kP2>
__global__ __launch_bounds__(kPThreads) void k_hist_rep(const uint32_t* __restrict__ v,
                                                        const uint32_t* __restrict__ start,
                                                        const uint4* __restrict__ desc, uint32_t njobs,
                                                        const uint32_t* __restrict__ ncols_dev,
                                                        uint32_t* __restrict__ hist) {
  __shared__ uint32_t rc[256 * 32];
  const int tid = threadIdx.x;
  HistJob h;
  if (kP2) {
    const uint4 d = desc[blockIdx.x];
    h.s0 = d.x;
    h.s1 = d.y;
    h.col = d.w;
    if (h.s0 >= h.s1) return;
  } else {
    h.col = xcd_tile(blockIdx.x, njobs);
    h.s0 = start[h.col];
    h.s1 = start[h.col + 1];
  }
  const uint32_t ncols = kP2 ? *ncols_dev : njobs;
  HistRegs r;
  hist_load(v, h, tid, r);
#pragma unroll
  for (int k = 0; k < 256 * 32 / 4 / kPThreads; k++)
    reinterpret_cast<uint4*>(rc)[k * kPThreads + tid] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  const uint32_t q0 = (h.s0 + 3) >> 2, q1 = h.s1 >> 2, cp = tid & 31;
#pragma unroll
  for (int k = 0; k <= kHistQ; k++)
    if (q0 + k * kPThreads + tid < q1) {
      atomicAdd(&rc[hist_digit<kP2>(r.x[k].x) * 32 + cp], 1u);
      atomicAdd(&rc[hist_digit<kP2>(r.x[k].y) * 32 + cp], 1u);
      atomicAdd(&rc[hist_digit<kP2>(r.x[k].z) * 32 + cp], 1u);
      atomicAdd(&rc[hist_digit<kP2>(r.x[k].w) * 32 + cp], 1u);
    }
  if (hist_edge(h, tid) != 0xFFFFFFFFu) atomicAdd(&rc[hist_digit<kP2>(r.y) * 32 + cp], 1u);
  __syncthreads();
  if (tid < 256) {
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < 32; k++) sum += rc[tid * 32 + ((k + tid) & 31)];
    hist[(uint64_t)tid * ncols + h.col] = sum;
  }
}

// Pass-2 histogram from the byte plane: hist[b * ncols + col] = count of
// byte b over the chunk's positions [s0, s1).  The chunk's <= kPT bytes are
// read as 16-B quads from s0 rounded down (<= kPT / 16 + 1 quads; the plane
// is padded), bytes outside [s0, s1) masked.  512 threads, 16 counter copies
// (the per-block zeroing and final sums are most of the work at 1 B per entry).
constexpr int kHBThreads = 512, kHBCopies = 16;
__global__ __launch_bounds__(kHBThreads) void k_hist_bytes(const uint8_t* __restrict__ v,
                                                            const uint4* __restrict__ desc,
                                                            const uint32_t* __restrict__ ncols_dev,
                                                            uint32_t* __restrict__ hist) {
  __shared__ uint32_t rc[256 * kHBCopies];
  const int tid = threadIdx.x;
  const uint4 d = desc[blockIdx.x];
  const uint32_t s0 = d.x, s1 = d.y, col = d.w;
  if (s0 >= s1) return;
  const uint32_t ncols = *ncols_dev;
  const uint32_t b0 = s0 & ~15u;
  constexpr int kQ = kPT / 16 / kHBThreads + 1;  // quads per thread (the last one only for the rounding)
  uint4 x[kQ];
#pragma unroll
  for (int k = 0; k < kQ; k++) {
    const uint32_t q = b0 + (uint32_t)(k * kHBThreads + tid) * 16u;
    x[k] = q < s1 ? *reinterpret_cast<const uint4*>(v + q) : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int k = 0; k < 256 * kHBCopies / 4 / kHBThreads; k++)
    reinterpret_cast<uint4*>(rc)[k * kHBThreads + tid] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  const uint32_t cp = tid & (kHBCopies - 1);
#pragma unroll
  for (int k = 0; k < kQ; k++) {
    const uint32_t q = b0 + (uint32_t)(k * kHBThreads + tid) * 16u;
    if (q < s1) {
      const uint32_t w[4] = {x[k].x, x[k].y, x[k].z, x[k].w};
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const uint32_t pos = q + j;
        if (pos >= s0 && pos < s1) atomicAdd(&rc[((w[j >> 2] >> (8 * (j & 3))) & 0xFFu) * kHBCopies + cp], 1u);
      }
    }
  }
  __syncthreads();
  if (tid < 256) {
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kHBCopies; k++) sum += rc[tid * kHBCopies + ((k + tid) & (kHBCopies - 1))];
    hist[(uint64_t)tid * ncols + col] = sum;
  }
}

// ------------------------------------------------ trace batches (set-exact) ---
// A batch given as raw per-call PC traces (the executor's KCOV buffers) is
// triaged with its edge signal computed in the pass-1 loads: entry e of a
// call is sig = pc[e] ^ hash(pc[e - 1]), pc[e] ^ 0 for the call's first PC
// (executor/executor.h:392-396), and a zero sig is not an entry (the
// executor's dedup reports 0 as seen, executor.h:507-515).  The executor
// also drops an edge its dedup table still holds; skipping that is exact for
// the triage: every non-zero edge is written at its first occurrence in the
// program (dedup returns false when no slot holds it, executor.h:516-525),
// i.e. in its first call, so the first record holding s and the union of the
// batch's signal -- all that decides the queued records and the set updates
// (fuzzer.go:665-691) -- are the same with or without the repeats.  The
// partition and the buckets are the sort and unique stage.
//
// Repeats inside a pass-1 tile (a hot edge recurs hundreds of times in one
// program's trace; the executor's table drops most of those) are dropped
// before the partition: each edge takes a 64-bit atomicMin of
// (tile position << 32 | sig) on an LDS slot hashed from sig, and an edge
// whose slot ends up holding the same sig at an earlier position is a
// repeat.  Exact: the earlier copy's record is not larger, so the first
// record holding sig and the union are unchanged; a slot taken by another
// edge only leaves a repeat in.  The histogram and the scatter drop the
// same entries (same positions, same hash).
constexpr uint32_t kTraceDedup = 1024;  // slots (8 KiB of LDS)
__device__ __forceinline__ uint32_t dedup_slot(uint32_t sig) { return (sig * 0x9E3779B1u) >> 22; }

// the previous PC of position e for lane-strided loads (x = this lane's PC,
// xp = pcs[e - 1] loaded by lane 0 of the wave)
__device__ __forceinline__ uint32_t trace_prev(uint32_t x, uint32_t xp) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)xp, (int)x, 0x138 /* wave_shr:1 */, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t trace_sig(uint32_t pc, uint32_t prev, bool start) {
  return pc ^ (start ? 0u : sgd::exec_hash(prev));
}

// Pass-1 histogram of a trace batch: b2 counts of the tile's non-zero edges.
// It also records which entries are kept (non-zero, not an in-tile repeat):
// one ballot word per 64 tile positions (keep[t][p / 64], bit p % 64), which
// the scatter reads instead of repeating the dedup.
__global__ __launch_bounds__(kPThreads) void k_hist_trace(const uint32_t* __restrict__ pcs,
                                                          const uint64_t* __restrict__ rec_off, uint64_t nrec,
                                                          const uint32_t* __restrict__ tstart,
                                                          const uint32_t* __restrict__ trec, uint32_t T,
                                                          uint32_t* __restrict__ hist, uint64_t* __restrict__ keep) {
  __shared__ uint32_t rc[256 * 32];
  __shared__ alignas(16) uint32_t cs[kPT / 32];
  __shared__ unsigned long long dd[kTraceDedup];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t t = xcd_tile(blockIdx.x, T), s0 = tstart[t], s1 = tstart[t + 1];
  constexpr int kS = kPT / kPThreads;
  uint32_t x[kS], xp[kS];
#pragma unroll
  for (int k = 0; k < kS; k++) {
    const uint32_t e = s0 + k * kPThreads + tid;
    x[k] = e < s1 ? pcs[e] : 0u;
    xp[k] = lane == 0 && e < s1 && e > 0 ? pcs[e - 1] : 0u;
  }
  // the tile's record offsets, loaded with the PCs (one per thread), so their
  // round trip overlaps the PCs' instead of following the first barrier
  static_assert(kRecCap + 1 <= kPThreads, "one record offset per thread");
  const uint32_t r0 = trec[t];
  const uint32_t wn = (uint32_t)(nrec + 1 - r0 < kRecCap + 1 ? nrec + 1 - r0 : kRecCap + 1);
  const uint64_t ro = (uint32_t)tid < wn ? rec_off[r0 + tid] : ~0ull;
#pragma unroll
  for (int k = 0; k < 256 * 32 / 4 / kPThreads; k++)
    reinterpret_cast<uint4*>(rc)[k * kPThreads + tid] = make_uint4(0, 0, 0, 0);
  for (int i = tid; i < kPT / 32; i += kPThreads) cs[i] = 0;
  for (int i = tid; i < (int)kTraceDedup; i += kPThreads) dd[i] = ~0ull;
  __syncthreads();
#if SG_HT_ABL != 2  // (SG_HT_ABL: timing ablations, wrong results)
  if (ro >= s0 && ro < s1) atomicOr(&cs[(ro - s0) >> 5], 1u << ((ro - s0) & 31));  // call starts in the tile
#endif
  __syncthreads();
  uint32_t live = 0;
#pragma unroll
  for (int k = 0; k < kS; k++) {
    const uint32_t p = k * kPThreads + tid, e = s0 + p;
#if SG_HT_ABL == 3
    x[k] = x[k] ^ ((cs[p >> 5] >> (p & 31)) & 1u) ^ xp[k];
#else
    x[k] = trace_sig(x[k], trace_prev(x[k], xp[k]), (cs[p >> 5] >> (p & 31)) & 1u);
#endif
    if (e < s1 && x[k] != 0) {
      live |= 1u << k;
#if SG_HT_ABL != 1
      atomicMin(&dd[dedup_slot(x[k])], ((unsigned long long)p << 32) | x[k]);
#endif
    }
  }
  __syncthreads();
  const uint32_t cp = tid & 31;
  uint32_t kmask = 0;  // kept steps of this thread (no cross-lane step in this loop)
#pragma unroll
  for (int k = 0; k < kS; k++) {
    const uint32_t p = k * kPThreads + tid;
    if ((live >> k) & 1u) {
#if SG_HT_ABL == 1
      const unsigned long long v = ((unsigned long long)p << 32) | x[k];
#else
      const unsigned long long v = dd[dedup_slot(x[k])];
#endif
      if ((uint32_t)v != x[k] || (uint32_t)(v >> 32) == p) {
        kmask |= 1u << k;
        atomicAdd(&rc[p1_digit(x[k]) * 32 + cp], 1u);
      }
    }
  }
  // the kept words through LDS (cs: the call starts are no longer needed),
  // then one coalesced 2 KiB store per tile
  unsigned long long* kw = reinterpret_cast<unsigned long long*>(cs);
#pragma unroll
  for (int k = 0; k < kS; k++) {
    const uint64_t b = __ballot((kmask >> k) & 1u);  // positions k kPThreads + 64 (tid / 64) ..
    if (lane == 0) kw[(k * kPThreads + tid) >> 6] = b;
  }
  __syncthreads();
  if (tid < 256) {
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < 32; k++) sum += rc[tid * 32 + ((k + tid) & 31)];
    hist[(uint64_t)tid * T + t] = sum;
    keep[(uint64_t)t * (kPT / 64) + tid] = kw[tid];
  }
}

// Counting sort of one tile held in registers (kSteps entries per lane) by an
// 8-bit digit, through LDS: counts, a one-wave exclusive scan, then every
// entry takes a slot with an LDS atomic (order within a digit is arbitrary).
// On return dstart[d] is the digit's first slot and pos[k] entry k's slot.
// cnt[] arrives holding the tile's digit counts (read from the histogram
// pass, not recounted); gbase[d] is lowered by the digit's first slot, so slot
// p of digit d goes to gbase[d] + p.
template <typename DigitF>
__device__ __forceinline__ void tile_rank(const uint32_t (&dv)[kSteps], DigitF digit, uint32_t vmask, uint32_t* cnt,
                                          uint32_t* gbase, uint32_t (&pos)[kSteps]) {
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid < 64) {
    uint32_t carry = 0;
#pragma unroll
    for (int base = 0; base < 256; base += 64) {
      const uint32_t x = cnt[base + lane];
      const uint32_t incl = sgd::wave_incl_add(x);
      const uint32_t ex = carry + incl - x;
      gbase[base + lane] -= ex;
      cnt[base + lane] = ex;
      carry += __builtin_amdgcn_readlane(incl, 63);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kSteps; k++)
    if ((vmask >> k) & 1u) pos[k] = atomicAdd(&cnt[digit(dv[k])], 1u);
}

// Write-out of a ranked tile: after tile_rank and the staging barrier, cnt[d]
// is the end of digit d's slots.  Each half-wave copies whole digit runs
// (16 half-waves, 16 digits each): 32 consecutive slots per store, and no
// per-slot digit array in LDS.
// With `top` (pass 1), the top byte of every entry also goes to the byte
// plane top[] at the same position: the pass-2 digit, which the pass-2
// histogram then reads at 1 B per entry instead of 4.
template <bool kTop>
__device__ __forceinline__ void tile_write(const uint32_t* stage, const uint32_t* cnt, const uint32_t* gbase,
                                           uint32_t* __restrict__ out, uint8_t* __restrict__ top, int tid) {
  const int hw = tid >> 5, hl = tid & 31;
  const bool wtop = kTop && top;  // (none when the M0 filter may end the partition after pass 1)
  for (int d = hw; d < 256; d += kPThreads / 32) {
    const uint32_t e = cnt[d], gb = gbase[d];
    for (uint32_t p = (d ? cnt[d - 1] : 0u) + hl; p < e; p += 32) {
      const uint32_t v = stage[p];
      out[gb + p] = v;
      if (wtop) top[gb + p] = (uint8_t)(v >> 24);
    }
  }
}

// O(1) "value of the segment holding p" inside one tile of <= kPT positions,
// for sorted segment starts st(0..m) given tile-relative and clamped to
// [0, kPT] (st(0) == 0) and segment values val(k) non-decreasing in k
// (< 2^16).  Non-empty segments that start inside the tile are marked: bit
// p of sbits <=> one starts at p > 0, sidx[p] = its value; wmax[w] = value of
// the segment holding position 32w + 31; kinit = that of position 0.
// Replaces a per-entry search (segments can be a few entries long: small
// records, thin slices).
template <typename IdxT>
struct SegLds {
  uint32_t sbits[kPT / 32];
  IdxT wmax[kPT / 32];
  uint32_t kinit;
};

template <typename IdxT>
__device__ __forceinline__ void seg_clear(SegLds<IdxT>& L, int tid) {
  for (int w = tid; w < kPT / 32; w += kPThreads) L.sbits[w] = 0;
  if (tid == 0) L.kinit = 0;
}

// one segment: start p, the next segment's start nx (0xFFFFFFFF: none), value v
template <typename IdxT>
__device__ __forceinline__ void seg_mark(SegLds<IdxT>& L, IdxT* sidx, uint32_t p, uint32_t nx, uint32_t v,
                                         uint32_t n) {
  if (p == 0) {
    if (nx > 0) atomicMax(&L.kinit, v);
  } else if (p < n && nx > p) {
    atomicOr(&L.sbits[p >> 5], 1u << (p & 31));
    sidx[p] = (IdxT)v;
  }
}

template <typename IdxT>
__device__ __forceinline__ void seg_finish(SegLds<IdxT>& L, IdxT* sidx, int tid);

// call after seg_clear + a barrier; ends with a barrier
template <typename IdxT, typename StF, typename ValF>
__device__ __forceinline__ void seg_build(SegLds<IdxT>& L, IdxT* sidx, StF st, ValF val, uint32_t m, uint32_t n,
                                          int tid) {
  for (uint32_t k = tid; k < m; k += kPThreads)
    seg_mark(L, sidx, st(k), k + 1 < m ? st(k + 1) : 0xFFFFFFFFu, val(k), n);
  seg_finish(L, sidx, tid);
}

// the segments' marks -> the per-word maxima (after seg_mark; ends with a barrier)
template <typename IdxT>
__device__ __forceinline__ void seg_finish(SegLds<IdxT>& L, IdxT* sidx, int tid) {
  __syncthreads();
  constexpr int kWL = kPT / 32 / 64;  // bitmap words per lane
  if (tid < 64) {  // prefix max over the kPT / 32 words
    int run = -1;
    int loc[kWL];
#pragma unroll
    for (int j = 0; j < kWL; j++) {
      const int w = tid * kWL + j;
      const uint32_t b = L.sbits[w];
      if (b) run = max(run, (int)sidx[w * 32 + 31 - __clz(b)]);
      loc[j] = run;
    }
    const int incl = sgd::wave_incl_max(run);
    int ex = __builtin_amdgcn_update_dpp(-1, incl, 0x138, 0xF, 0xF, false);  // wave_shr:1 (lane 0: -1)
    ex = max(ex, (int)L.kinit);
#pragma unroll
    for (int j = 0; j < kWL; j++) L.wmax[tid * kWL + j] = (IdxT)max(ex, loc[j]);
  }
  __syncthreads();
}

template <typename IdxT>
__device__ __forceinline__ uint32_t seg_lookup(const SegLds<IdxT>& L, const IdxT* sidx, uint32_t p) {
  const uint32_t w = p >> 5;
  const uint32_t m = L.sbits[w] & (0xFFFFFFFFu >> (31 - (p & 31)));
  return m ? sidx[(w << 5) + 31 - __clz(m)] : (w ? L.wmax[w - 1] : L.kinit);
}

// ---------------------------------------------------------------- pass 1 ---
struct P1Args {
  const uint32_t* vals;
  const uint64_t* rec_off;
  uint64_t nrec;
  const uint32_t* tstart;  // T + 1
  const uint32_t* trec;    // T
  uint32_t T;
  const uint32_t* goff1;   // scanned [slice][tile]
  const uint32_t* hist1;   // [slice][tile] counts
  uint32_t* out;           // s << 8 | rec_in_tile
  uint8_t* top;            // out's top bytes (the pass-2 digits)
  unsigned long long* dbg; // diagnostics (k_p1_scatter<true>): cycles per phase, summed over blocks
  const uint64_t* keep;    // trace batches: k_hist_trace's kept-entry words
};

// One tile.  Only the values and their records (four 8-bit records per
// register) stay live across the rank; digits and keys are recomputed from the
// values (1.85 -> 1.67 ms per C2 launch against keeping digits and keys in
// registers; an unpredicated path for full tiles, as pass 2 has, was slower
// here: 1.93 ms).
// kTrace: a.vals are raw per-call PC traces, each entry's signal computed here
// (see k_hist_trace) and zero edges skipped.
template <bool kDbg, bool kTrace>
__device__ __forceinline__ void p1_tile(const P1Args& a, uint32_t* stage, uint32_t* cnt, uint32_t* gbase,
                                        uint16_t* win, SegLds<uint8_t>& L, uint32_t t,
                                        uint32_t s0, uint32_t s1) {
  uint8_t* sidx = reinterpret_cast<uint8_t*>(stage);  // record-in-tile index; stage is free until the rank
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  uint64_t tk = kDbg ? clock64() : 0;
  auto stamp = [&](int ph) {
    if (kDbg) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const uint64_t now = clock64();
      if (tid == 0) atomicAdd(&a.dbg[ph], (unsigned long long)(now - tk));
      tk = now;
    }
  };
  const uint32_t r0 = a.trec[t];
  const uint32_t wn = (uint32_t)(a.nrec + 1 - r0 < kRecCap + 1 ? a.nrec + 1 - r0 : kRecCap + 1);
  const uint32_t ebase = s0 + w * kPerWave;
  uint32_t sv[kSteps];
  uint32_t vmask = 0;
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    const uint32_t e = ebase + k * 64 + lane;
    const bool ok = e < s1;
    sv[k] = ok ? a.vals[e] : 0u;
    vmask |= (ok ? 1u : 0u) << k;
  }
  // trace batches: the PC before the wave's first position (lane 0; the rest
  // come from the wave itself)
  const uint32_t xp0 = kTrace && lane == 0 && ebase < s1 && ebase > 0 ? a.vals[ebase - 1] : 0u;
  const bool start0 = kTrace && a.rec_off[r0] == s0;  // does a call start at the tile's first position
  // trace batches: the kept-entry words of the wave's steps, loaded with the
  // tile (loaded where they are used, after the segment build, their round
  // trip was exposed: 2.38 -> 2.21 ms per C2 trace launch)
  uint64_t kwv[kTrace ? kSteps : 1];
  if (kTrace) {
    const uint64_t* kw = a.keep + (uint64_t)t * (kPT / 64) + __builtin_amdgcn_readfirstlane(w) * (kPerWave / 64);
#pragma unroll
    for (int k = 0; k < kSteps; k++) kwv[k] = kw[k];
  }
  for (uint32_t i = tid; i < wn; i += kPThreads) {
    const uint64_t o = a.rec_off[r0 + i];
    win[i] = (uint16_t)(o <= s0 ? 0 : (o - s0 >= (uint64_t)kPT ? kPT : o - s0));
  }
  for (int d = tid; d < 256; d += kPThreads) {
    gbase[d] = a.goff1[(uint64_t)d * a.T + t];
    cnt[d] = a.hist1[(uint64_t)d * a.T + t];
  }
  seg_clear(L, tid);
  __syncthreads();
  stamp(0);
  const uint32_t nt = s1 - s0;
  seg_build(
      L, sidx, [&](uint32_t k) { return (uint32_t)win[k]; }, [](uint32_t k) { return k; }, wn, nt, tid);
  uint32_t rp[kSteps / 4] = {};
  const uint32_t el0 = ebase + lane - s0;
  if (kTrace) {
    // entries -> edge signals: the previous PC is the lane before's (lane 0:
    // the previous step's lane 63, or xp0); a call start is a segment start
    // (seg_build marks every non-empty record starting inside the tile)
    uint32_t carry = xp0;
#pragma unroll
    for (int k = 0; k < kSteps; k++) {
      const uint32_t p = el0 + k * 64, pc = sv[k];
      const bool start = p ? ((L.sbits[p >> 5] >> (p & 31)) & 1u) != 0 : start0;
      const uint32_t prev = trace_prev(pc, carry);
      carry = (uint32_t)__builtin_amdgcn_readlane((int)pc, 63);
      sv[k] = trace_sig(pc, prev, start);
      asm volatile("" : "+v"(sv[k]));  // one step at a time (registers)
    }
    // kept entries (non-zero, not an in-tile repeat): the histogram's words,
    // one per 64 positions -- wave w's step k is positions w kPerWave + 64 k ..
#pragma unroll
    for (int k = 0; k < kSteps; k++)
      if (!((kwv[k] >> lane) & 1ull)) vmask &= ~(1u << k);
  }
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    const uint32_t r = ((vmask >> k) & 1u) ? seg_lookup(L, sidx, el0 + k * 64) : 0u;  // record in tile
    rp[k >> 2] |= r << (8 * (k & 3));
  }
  stamp(1);
  uint32_t pos[kSteps];
  tile_rank(sv, [](uint32_t v) { return p1_digit(v); }, vmask, cnt, gbase, pos);
  stamp(2);
#pragma unroll
  for (int k = 0; k < kSteps; k++)
    if ((vmask >> k) & 1u) stage[pos[k]] = (part_key(sv[k]) << 8) | ((rp[k >> 2] >> (8 * (k & 3))) & 0xFFu);
  __syncthreads();
  stamp(3);
  tile_write<true>(stage, cnt, gbase, a.out, a.top, tid);
  stamp(4);
  if (kDbg && tid == 0) atomicAdd(&a.dbg[5], 1ull);
}

template <bool kDbg, bool kTrace>
__global__ __launch_bounds__(kPThreads) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_p1_scatter(P1Args a) {
  __shared__ uint32_t stage[kPT];
  __shared__ uint32_t cnt[256];
  __shared__ uint32_t gbase[256];
  __shared__ uint16_t win[kRecCap + 1];  // tile-relative record starts, clamped to [0, kPT]
  __shared__ SegLds<uint8_t> L;
  const uint32_t t = xcd_tile(blockIdx.x, gridDim.x);
  const uint32_t s0 = a.tstart[t], s1 = a.tstart[t + 1];
  if (s0 >= s1) return;
  p1_tile<kDbg, kTrace>(a, stage, cnt, gbase, win, L, t, s0, s1);
}

// ---------------------------------------------------------------- pass 2 ---
struct P2Args {
  const uint32_t* in;      // pass-1 output
  const uint4* desc;       // per-block chunk descriptors
  const uint2* dtile;      // per-block chunk tile ranges
  const uint32_t* g2;      // device: number of chunks G2 (the grid is an upper bound)
  const uint32_t* goff1;   // pass-1 run starts [slice][tile]
  const uint32_t* trec;    // first record of each pass-1 tile
  uint32_t T, NG;
  const uint32_t* goff2;   // scanned [byte][chunk]
  const uint32_t* hist2;   // [byte][chunk] counts
  uint32_t* out;           // (s & 0xFFFF) << 16 | record_in_group
};

// One chunk; kFull: the chunk holds kPT entries (most do), so no entry is
// predicated (no exec-mask branch per entry and step: the scatters are bound
// by the instructions they issue).  As in pass 1, only the values and the
// records (two 16-bit records per register) stay live across the rank.
template <bool kFull>
__device__ __forceinline__ void p2_chunk(const P2Args& a, uint32_t* stage, uint32_t* cnt, uint32_t* gbase,
                                         SegLds<uint16_t>& L, uint32_t s0, uint32_t s1, uint32_t gov, uint32_t c,
                                         uint2 dt) {
  uint16_t* sidx = reinterpret_cast<uint16_t*>(stage);  // tile's first record in the group; stage is free until the rank
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const uint32_t G2 = *a.g2;
  const uint32_t d = gov / a.NG, rg0 = (gov % a.NG) << kGroupBits, tf = dt.x, m = dt.y - dt.x;
  const uint32_t ebase = s0 + w * kPerWave;
  uint32_t sv[kSteps];
  uint32_t vmask = kFull ? (1u << kSteps) - 1 : 0u;
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    const uint32_t e = ebase + k * 64 + lane;
    if (kFull) {
      sv[k] = a.in[e];
    } else {
      const bool ok = e < s1;
      sv[k] = ok ? a.in[e] : 0u;
      vmask |= (ok ? 1u : 0u) << k;
    }
  }
  for (int f = tid; f < 256; f += kPThreads) {
    gbase[f] = a.goff2[(uint64_t)f * G2 + c];
    cnt[f] = a.hist2[(uint64_t)f * G2 + c];
  }
  // segments = the chunk's tiles (runs of this slice); value = the tile's
  // first record relative to the group.  A chunk of at most kPThreads tiles
  // (nearly all) has thread k's tile loaded with the chunk's entries, so the
  // loads' round trip is not exposed after the barrier.
  const uint32_t* row = a.goff1 + (uint64_t)d * a.T + tf;
  auto clampst = [&](uint32_t o) { return o <= s0 ? 0u : (o - s0 >= (uint32_t)kPT ? (uint32_t)kPT : o - s0); };
  const bool one = m <= (uint32_t)kPThreads;  // (block-uniform)
  const uint32_t ku = (uint32_t)tid;
  uint32_t pst = 0, pnx = 0, pvl = 0;
  if (one && ku < m) {
    pst = row[ku];
    pnx = ku + 1 < m ? row[ku + 1] : 0u;
    pvl = a.trec[tf + ku];
  }
  seg_clear(L, tid);
  __syncthreads();
  const uint32_t nt = s1 - s0;
  if (one) {
    if (ku < m) seg_mark(L, sidx, clampst(pst), ku + 1 < m ? clampst(pnx) : 0xFFFFFFFFu, pvl - rg0, nt);
    seg_finish(L, sidx, tid);
  } else {
    seg_build(
        L, sidx, [&](uint32_t k) { return clampst(row[k]); }, [&](uint32_t k) { return a.trec[tf + k] - rg0; }, m,
        nt, tid);
  }
  const uint32_t el0 = ebase + lane - s0;
  uint32_t rp[kSteps / 2] = {};  // records in group, two 16-bit per register
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    const uint32_t r1 = ((vmask >> k) & 1u) ? seg_lookup(L, sidx, el0 + k * 64) : 0u;  // tile's record in group
    rp[k >> 1] |= (r1 + (sv[k] & (kRecCap - 1))) << (16 * (k & 1));
  }
  uint32_t pos[kSteps];
  tile_rank(sv, [](uint32_t v) { return v >> 24; }, vmask, cnt, gbase, pos);
#pragma unroll
  for (int k = 0; k < kSteps; k++)
    if ((vmask >> k) & 1u) stage[pos[k]] = (((sv[k] >> 8) & 0xFFFFu) << 16) | ((rp[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
  __syncthreads();
  tile_write<false>(stage, cnt, gbase, a.out, nullptr, tid);
}

__global__ __launch_bounds__(kPThreads) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_p2_scatter(P2Args a) {
  __shared__ uint32_t stage[kPT];
  __shared__ uint32_t cnt[256];
  __shared__ uint32_t gbase[256];
  __shared__ SegLds<uint16_t> L;
  const uint4 dsc = a.desc[blockIdx.x];
  const uint2 dt = a.dtile[blockIdx.x];
  const uint32_t s0 = dsc.x, s1 = dsc.y;
  if (s0 >= s1) return;
  if (s1 - s0 == (uint32_t)kPT)
    p2_chunk<true>(a, stage, cnt, gbase, L, s0, s1, dsc.z, dsc.w, dt);
  else
    p2_chunk<false>(a, stage, cnt, gbase, L, s0, s1, dsc.z, dsc.w, dt);
}

// ---------------------------------------------------------------- bucket ---
struct BucketArgs {
  const uint32_t* in;      // pass-2 output
  const uint4* bdesc;      // per-bucket {lo, hi, c0, nch}
  const uint32_t* gbnd;    // [bucket][group]: first bucket position of each group's entries
  uint32_t NG;             // groups
  uint32_t* mwords;        // maxSignal
  const uint32_t* owords;  // nullable: the test is against mwords | owords (words that gain bits get both)
  uint32_t* nwords;        // newSignal (nullable)
  uint8_t* rec_new;        // per record: owns some new signal
  uint32_t* spill;         // buckets left for the direct-table kernel
  uint32_t* nspill;
  uint32_t* ticket;        // persistent bucket kernel: list entries handed out past 2 x grid
  const uint32_t* blist_b; // non-empty buckets, in bucket order ...
  const uint4* blist_q;    // ... and their descriptors
  const uint32_t* nlist;   // device: their number
  uint64_t* dbg;           // diagnostics (k_bucket<true>): per block {start, end, buckets, rounds, 4 phase cycle sums}
  // candidate emission (sharded triage, sg_shard.hip; the prefix protocol's
  // begin): instead of flagging records and updating maxSignal, every
  // distinct candidate s of the batch is written once, with its first
  // record, as {s, rec_base + record}, and set in nwords when that is given
  uint2* pairs;
  unsigned long long* npairs;
  uint32_t rec_base;
  uint32_t nshards;         // pairs are counted per owning shard (shard_of) ...
  unsigned long long* shard_cnt;  // ... when this is given
  uint32_t update;          // emitting form that also updates mwords / nwords (the ordered outputs) ...
  unsigned long long* gcur; // ... with the pairs group-major: pairs of group g's records appended at
  const uint64_t* goff;     //     goff[g << 16] + gcur[g] (goff: the launch's record offsets; a group's
};                          //     pairs never outnumber its entries)

// Owning shard of a signal in the hash-sharded multi-GPU triage: the murmur3
// finaliser of s, scaled to [0, nshards).
__device__ __forceinline__ uint32_t shard_of(uint32_t s, uint32_t nshards) {
  s ^= s >> 16;
  s *= 0x85EBCA6Bu;
  s ^= s >> 13;
  s *= 0xC2B2AE35u;
  s ^= s >> 16;
  return (uint32_t)(((uint64_t)s * nshards) >> 32);
}

constexpr uint32_t kMaxShards = 64;

// Block-aggregated append of up to kPer pairs per lane (valid where rec !=
// kEmpty): one global atomic per call and block (a per-wave atomic on the one
// pair counter was the emitting launch's bottleneck); each pair is also
// counted in the block's LDS shard counters.  Called by every thread.
template <int kPer>
__device__ __forceinline__ void emit_pairs(const BucketArgs& a, const uint32_t (&sig)[kPer], const uint32_t (&rec)[kPer],
                                           uint32_t* shcnt) {
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  __shared__ uint32_t ewc[16];  // per-wave totals, then offsets (<= 1024 threads)
  __shared__ unsigned long long ebase;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < kPer; k++) c += rec[k] != kNone ? 1u : 0u;
  uint32_t incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) ewc[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < nw; i++) {
      const uint32_t v = ewc[i];
      ewc[i] = acc;
      acc += v;
    }
    ebase = acc ? atomicAdd(a.npairs, (unsigned long long)acc) : 0ull;
  }
  __syncthreads();
  uint64_t pos = ebase + ewc[w] + incl - c;
#pragma unroll
  for (int k = 0; k < kPer; k++)
    if (rec[k] != kNone) {
      a.pairs[pos++] = make_uint2(sig[k], a.rec_base + rec[k]);
      if (a.shard_cnt) atomicAdd(&shcnt[shard_of(sig[k], a.nshards)], 1u);
    }
  __syncthreads();  // ewc / ebase are rewritten by the next call
}

// Group-major append (the ordered outputs): up to kPer pairs per thread
// (valid where rec != kEmpty), counted per record group in LDS, one global
// cursor atomic per group and call, then placed.  Order within a group is
// free: the pairs are sorted by record afterwards.  lcnt (LDS, kMaxGroups
// words) is zero on entry and on exit.  Called by every thread.
template <int kPer>
__device__ __forceinline__ void emit_grouped(const BucketArgs& a, const uint32_t (&sig)[kPer], const uint32_t (&rec)[kPer],
                                             uint32_t* lcnt, unsigned long long* lbase) {
  constexpr uint32_t kNone = 0xFFFFFFFFu;
#pragma unroll
  for (int k = 0; k < kPer; k++)
    if (rec[k] != kNone) atomicAdd(&lcnt[rec[k] >> kGroupBits], 1u);
  __syncthreads();
  for (uint32_t g = threadIdx.x; g < a.NG; g += blockDim.x) {
    const uint32_t c = lcnt[g];
    lbase[g] = c ? a.goff[(uint64_t)g << kGroupBits] + atomicAdd(&a.gcur[g], (unsigned long long)c) : 0ull;
    lcnt[g] = 0;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPer; k++)
    if (rec[k] != kNone) {
      const uint32_t g = rec[k] >> kGroupBits;
      a.pairs[lbase[g] + atomicAdd(&lcnt[g], 1u)] = make_uint2(sig[k], rec[k]);
    }
  __syncthreads();
  for (uint32_t g = threadIdx.x; g < a.NG; g += blockDim.x) lcnt[g] = 0;
  __syncthreads();
}

__device__ __forceinline__ void flush_shard_counts(const BucketArgs& a, const uint32_t* shcnt) {
  if (a.shard_cnt)
    for (uint32_t i = threadIdx.x; i < a.nshards; i += blockDim.x)
      if (shcnt[i]) atomicAdd(&a.shard_cnt[i], (unsigned long long)shcnt[i]);
}

__global__ void k_bucket_compact(const uint4* __restrict__ bdesc, const uint32_t* __restrict__ lpos,
                                 uint32_t* __restrict__ blist_b, uint4* __restrict__ blist_q) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= kNumBuckets) return;
  const uint4 q = bdesc[b];
  if (q.x < q.y) {
    blist_b[lpos[b]] = b;
    blist_q[lpos[b]] = q;
  }
}

// {lo, hi, c0, nch} of every bucket, from the pass-2 scan, and its
// non-empty flag (scanned into list positions)
__global__ void k_bucket_desc(const uint32_t* __restrict__ goff2, const uint32_t* __restrict__ gcount,
                              const uint32_t* __restrict__ cfirst, uint4* __restrict__ bdesc, uint32_t* __restrict__ nz) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= kNumBuckets) return;
  const uint32_t d = b >> 8, f = b & 255, c0 = cfirst[d], nch = cfirst[d + 1] - c0;
  const uint32_t* row = goff2 + (uint64_t)f * *gcount + c0;
  const uint32_t lo = row[0], hi = row[nch];
  bdesc[b] = make_uint4(lo, hi, c0, nch);
  nz[b] = lo < hi ? 1u : 0u;
}

// gbnd[b * NG + g]: bucket b = (d, f) holds the runs of slice d's chunks in
// byte row f, chunk-ordered, so group g's entries start at the run of the
// first chunk of slice-group (d, g) (an empty slice-group: the next one's)
__global__ void k_bucket_groups(const uint32_t* __restrict__ goff2, const uint32_t* __restrict__ gcount,
                                const uint32_t* __restrict__ cbase, uint32_t NG, uint32_t* __restrict__ gbnd) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)kNumBuckets * NG) return;
  const uint32_t b = (uint32_t)(i / NG), g = (uint32_t)(i % NG);
  gbnd[i] = goff2[(uint64_t)(b & 255) * *gcount + cbase[(b >> 8) * NG + g]];
}

// group of bucket position p >= gb[0]: last g < NG with gb[g] <= p
__device__ __forceinline__ uint32_t group_of(const uint32_t* gb, uint32_t NG, uint32_t p) {
  uint32_t lo = 0, hi = NG;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (gb[mid] <= p)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// Record of the candidate entry x at a bucket position of group g.  Records
// are what the first-owner rule takes the minimum of (fuzzer.go:665 order).
__device__ __forceinline__ uint32_t entry_record(uint32_t g, uint32_t x) { return (g << kGroupBits) | (x & 0xFFFFu); }

// Persistent: each workgroup takes buckets one after another (the first one
// by its index, then by ticket) and runs through them as one stream of
// rounds of kBU entries per thread.  Per round and thread: the LDS
// new-signal test of its kBU entries, then each candidate's record (group by
// a search over the bucket's group boundaries in LDS) inserted into the map.
// Rounds have no barrier: the waves of a workgroup meet only at bucket ends.
// While a round is processed the thread's next one is in flight -- the same
// bucket's next round, or the next bucket's first round together with its
// maxSignal slice and group boundaries.  The ticket after that is fetched a
// bucket ahead, so no dependent load is exposed.
constexpr uint32_t kGroupWords = (kMaxGroups + kBThreads - 1) / kBThreads;  // group boundaries per thread
constexpr int kWPT = kBucketWords / kBThreads;  // LDS slice words per thread
typedef uint32_t wvec __attribute__((ext_vector_type(kWPT)));
struct BucketPre {  // a bucket's first loads, held in registers
  uint32_t msw[kBucketWords / kBThreads];
  uint32_t nsw[kBucketWords / kBThreads];  // newSignal words (only this block writes them)
  uint32_t gw[kGroupWords];                // group boundaries
};

// Rounds start 4-aligned (the bucket start rounded down): thread t holds
// entries base + kBU t .. + kBU - 1 as 16-B loads (immediate offsets, one
// address); entry i is live iff lo <= i < hi.  The pass-2 buffer is padded,
// so the quad reads past hi stay in bounds.
__device__ __forceinline__ uint32_t round_pos(uint32_t base, int u) { return base + threadIdx.x * kBU + u; }

__device__ __forceinline__ void bucket_round_load(const BucketArgs& a, uint32_t base, uint32_t hi,
                                                  uint32_t (&x)[kBU]) {
  const uint4* p = reinterpret_cast<const uint4*>(a.in + base) + threadIdx.x * (kBU / 4);
#pragma unroll
  for (int j = 0; j < kBU / 4; j++) {
    // non-temporal: the streamed entries would otherwise push the record-flag
    // lines out of L2 (measured: 1.9 -> 1.27 GB of writes per launch)
    uint4 v = make_uint4(0, 0, 0, 0);
    if (round_pos(base, 4 * j) < hi) {
      const v4u32 t = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(p + j));
      v = make_uint4(t[0], t[1], t[2], t[3]);
    }
    x[4 * j] = v.x;
    x[4 * j + 1] = v.y;
    x[4 * j + 2] = v.z;
    x[4 * j + 3] = v.w;
  }
}

__device__ __forceinline__ void bucket_pre_load(const BucketArgs& a, uint32_t b, BucketPre& P) {
  // LDS slice words kWPT tid .. + kWPT - 1
  const uint64_t w0 = bucket_word(b, kWPT * threadIdx.x);
  wvec m = *reinterpret_cast<const wvec*>(a.mwords + w0);
  if (a.owords) m |= *reinterpret_cast<const wvec*>(a.owords + w0);
  wvec nw = {};
  if (a.nwords) nw = *reinterpret_cast<const wvec*>(a.nwords + w0);
#pragma unroll
  for (int j = 0; j < kWPT; j++) {
    P.msw[j] = m[j];
    P.nsw[j] = nw[j];
  }
  const uint32_t* gr = a.gbnd + (uint64_t)b * a.NG;
#pragma unroll
  for (int j = 0; j < (int)kGroupWords; j++) {
    const uint32_t i = j * kBThreads + threadIdx.x;
    P.gw[j] = i < a.NG ? gr[i] : 0u;
  }
}

// thread 0: bucket and descriptor of list entry t (kNumBuckets: past the end)
__device__ __forceinline__ uint32_t list_bucket(const BucketArgs& a, uint32_t t, uint32_t nl, uint4* q) {
  if (t >= nl) return kNumBuckets;
  *q = a.blist_q[t];
  return a.blist_b[t];
}

#ifndef SG_LDS_BARRIER
#define SG_LDS_BARRIER 0
#endif
// Bucket-loop barrier.  SG_LDS_BARRIER=1 waits for LDS operations only and
// leaves global loads and stores in flight across it; measured equal to
// __syncthreads on gfx950 (whose barrier does not wait for them either), so
// the plain barrier is the default.
__device__ __forceinline__ void lds_barrier() {
#if SG_LDS_BARRIER
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
  __syncthreads();
#endif
}

// block-uniform values read from LDS: keep them in scalar registers
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint4 uni(uint4 v) { return make_uint4(uni(v.x), uni(v.y), uni(v.z), uni(v.w)); }

// The candidate map: kHash = 8192 slots of 32 bits, linear probing.  The
// bucket's 16-bit signal sl goes through a bijection y = sl * kMapMul (mod
// 2^16): home slot = y >> 3, tag = y & 7.  A slot holds
//   tag << 29 | displacement << 24 | record        (record < 2^24 = kMaxGroups << 16)
// so the slot index and its top byte give back sl, and one 32-bit atomicMin
// lowers the record of an equal key.  Displacements stay <= kMaxProbe - 1 =
// 30, so no entry equals kEmpty (displacement field 31).
constexpr uint32_t kMapMul = 0x6F4Bu;  // odd: invertible mod 2^16
constexpr uint32_t inv16(uint32_t c) {
  uint32_t x = c;  // Newton: each step doubles the correct low bits (c * c == 1 mod 8 for odd c)
  for (int i = 0; i < 4; i++) x = (x * (2u - c * x)) & 0xFFFFu;
  return x;
}
constexpr uint32_t kMapInv = inv16(kMapMul);
static_assert(((kMapMul * kMapInv) & 0xFFFFu) == 1u, "kMapInv");
static_assert(kHash == 8192 && kMaxProbe <= 31, "13-bit slots, 5-bit displacements");
static_assert((uint64_t)kMaxGroups << kGroupBits <= (1u << 24), "records fit 24 bits");
constexpr uint32_t kRecMask = 0xFFFFFFu;

__device__ __forceinline__ uint32_t map_signal(uint32_t slot, uint32_t v) {  // sl of an occupied slot
  const uint32_t home = (slot - ((v >> 24) & 31u)) & (kHash - 1);
  return (((home << 3) | (v >> 29)) * kMapInv) & 0xFFFFu;
}

// A first insert is one CAS; a repeat of a signal lowers the record with a
// 32-bit min (equal key bits above the record).
__device__ __forceinline__ bool map_insert(uint32_t* ht, uint32_t sl, uint32_t rec, uint32_t disp0 = 0) {
  const uint32_t y = (sl * kMapMul) & 0xFFFFu;
  const uint32_t home = y >> 3, tag = y & 7u;
  for (uint32_t disp = disp0; disp < kMaxProbe; disp++) {
    const uint32_t mine = (tag << 29) | (disp << 24) | rec;
    uint32_t* slot = &ht[(home + disp) & (kHash - 1)];
    const uint32_t old = atomicCAS(slot, kEmpty, mine);
    if (old == kEmpty) return true;
    if ((old >> 24) == (mine >> 24)) {
      if ((old & kRecMask) > rec) atomicMin(slot, mine);
      return true;
    }
  }
  return false;  // map (nearly) full: the bucket spills
}

// A ticket: a plain atomicAdd, its result read at the next install.  (An
// inline-asm atomic waited for only there measured the same, 2.32-2.34 ms,
// and leaves the compiler unaware that its result register is pending: r05
// removed it.)
__device__ __forceinline__ uint32_t take_ticket(uint32_t* p) { return atomicAdd(p, 1u); }
__device__ __forceinline__ void take_wait(uint32_t&) {}

// kEmit: 0 flags and set updates, 1 candidate pairs (counted per owning
// shard), 2 the ordered outputs' new-signal pairs, group-major, with the set
// updates
template <bool kDbg, int kEmit>
__global__ __launch_bounds__(kBThreads) __attribute__((amdgpu_waves_per_eu(kBWaves))) void k_bucket(BucketArgs a) {
  __shared__ uint32_t mslice[kBucketWords];
  __shared__ uint32_t nbits[kBucketWords];
  __shared__ uint32_t ht[kHash];
  __shared__ alignas(16) uint32_t gb[kMaxGroups];  // the bucket's group boundaries (kEmpty past NG)
  __shared__ uint32_t sh_fail;         // some insert found the map full: the bucket spills
  __shared__ uint32_t sh_b[2];
  __shared__ uint4 sh_q[2];
  __shared__ uint32_t shcnt[kEmit == 1 ? kMaxShards : 1];  // emitted pairs per owning shard
  __shared__ uint32_t lcnt[kEmit == 2 ? kMaxGroups : 1];    // group-major emission: pairs per record group ...
  __shared__ unsigned long long lbase[kEmit == 2 ? kMaxGroups : 1];  // ... and where they go
  const int tid = threadIdx.x;
  if (kEmit == 1)
    for (uint32_t i = tid; i < kMaxShards; i += kBThreads) shcnt[i] = 0;
  if (kEmit == 2)
    for (uint32_t i = tid; i < kMaxGroups; i += kBThreads) lcnt[i] = 0;
  const uint32_t NG = a.NG;
  constexpr uint32_t kRound = kBThreads * kBU;
  // diagnostics (kDbg): block span, buckets, rounds, cycles per phase as wave 0 sees them
  const uint64_t t_start = kDbg ? wall_clock64() : 0;
  uint64_t n_buckets = 0, n_rounds = 0;
  uint64_t ph[7] = {0, 0, 0, 0, 0, 0, 0};  // install, rounds, -, flush | rounds: test, inserts, -
  uint64_t tk = kDbg ? clock64() : 0;
  for (uint32_t i = tid; i < kHash; i += kBThreads) ht[i] = kEmpty;
  for (uint32_t i = tid; i < kBucketWords; i += kBThreads) nbits[i] = 0;
  if (tid == 0) sh_fail = 0;
  // list entries: blockIdx and gridDim + blockIdx first, then tickets from
  // 2 x gridDim.  Thread 0 takes each ticket a bucket before it resolves it and
  // resolves it a bucket before it is needed, so neither wait is exposed.
  const uint32_t nl = *a.nlist;
  // (tickets are taken at every install, also past the list's end: waiting
  // for the list entry before taking the next would be another round trip)
  uint32_t pend_t = 0;  // thread 0: ticket taken, not yet resolved
  if (tid == 0) {
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = make_uint4(0, 0, 0, 0);
    sh_b[0] = list_bucket(a, blockIdx.x, nl, &q0);
    sh_q[0] = q0;
    sh_b[1] = list_bucket(a, gridDim.x + blockIdx.x, nl, &q1);
    sh_q[1] = q1;
    pend_t = take_ticket(a.ticket);
  }
  __syncthreads();
  uint32_t b = uni(sh_b[0]), b1 = uni(sh_b[1]);
  uint4 q = uni(sh_q[0]), q1 = uni(sh_q[1]);
  if (b >= kNumBuckets) {
    if (tid == 0) take_wait(pend_t);
    if (kDbg && tid == 0) {
      for (int j = 0; j < 8; j++) a.dbg[8 * blockIdx.x + j] = 0;
      a.dbg[8 * blockIdx.x] = t_start;
      a.dbg[8 * blockIdx.x + 1] = wall_clock64();
    }
    return;
  }
  uint32_t x[kBU], y[kBU];
  BucketPre P;
  bucket_round_load(a, q.x & ~3u, q.y, x);
  bucket_pre_load(a, b, P);
  while (b < kNumBuckets) {
    const uint32_t lo = q.x, hi = q.y;
    lds_barrier();  // the previous bucket is done with the LDS
    {
      wvec mv;
#pragma unroll
      for (int j = 0; j < kWPT; j++) mv[j] = P.msw[j];
      reinterpret_cast<wvec*>(mslice)[tid] = mv;
    }
    uint32_t ns[kWPT];  // newSignal words kWPT tid .. + kWPT - 1
#pragma unroll
    for (int j = 0; j < kWPT; j++) ns[j] = P.nsw[j];
#pragma unroll
    for (int j = 0; j < (int)kGroupWords; j++) {
      const uint32_t i = j * kBThreads + tid;
      if (i < kMaxGroups) gb[i] = i < NG ? P.gw[j] : kEmpty;
    }
    // thread 0: resolve the pending ticket (published after the rounds) and take the next one
    uint32_t pend_b = kNumBuckets;
    uint4 pend_q = make_uint4(0, 0, 0, 0);
    if (tid == 0) {
      take_wait(pend_t);  // (taken a bucket ago; the install waited for older loads already)
      pend_b = list_bucket(a, 2 * gridDim.x + pend_t, nl, &pend_q);
      pend_t = take_ticket(a.ticket);
      if (kEmit) take_wait(pend_t);
      sh_fail = 0;  // (every wave read the previous bucket's before the barrier above)
    }
    lds_barrier();
    const uint32_t gbl = NG <= 64 ? gb[threadIdx.x & 63] : kEmpty;  // boundary of group lane (kEmpty past NG)
    if (kDbg) {
      const uint64_t t = clock64();
      ph[0] += t - tk;
      tk = t;
    }
    n_buckets++;
    // Rounds: no barrier inside -- the waves run through the bucket on their
    // own, meeting only in the map's atomics.
    for (uint32_t base = lo & ~3u;;) {
      n_rounds++;
      // the next round in flight: this bucket's, or the next bucket's first
      // (one load call: separate calls per case load into different
      // registers and their join would wait for them)
      const uint32_t next = base + kRound;
      const bool last = next >= hi;
      if (!last || b1 < kNumBuckets) bucket_round_load(a, last ? q1.x & ~3u : next, last ? q1.y : hi, y);
      if (last && b1 < kNumBuckets) bucket_pre_load(a, b1, P);
      // this thread's kBU consecutive entries: the new-signal test (fuzzer.go:666),
      // all LDS reads issued before the first use
      const uint32_t p0 = round_pos(base, 0);
      // (the spill flag read with the slice words: one LDS wait for both)
      const uint32_t failed = __hip_atomic_load(&sh_fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      uint32_t mw[kBU];
#pragma unroll
      for (int u = 0; u < kBU; u++) mw[u] = mslice[x[u] >> 21];
      uint32_t cm = 0;
#pragma unroll
      for (int u = 0; u < kBU; u++) {
        const uint32_t i = p0 + u;
        const uint32_t miss = ((~mw[u]) >> ((x[u] >> 16) & 31)) & 1u;
        cm |= (miss & (i >= lo ? 1u : 0u) & (i < hi ? 1u : 0u)) << u;
      }
      if (kDbg) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint64_t t = clock64();
        ph[4] += t - tk;
        tk = t;
      }
      // (a relaxed atomic read: a volatile one would wait for every load in flight)
      // each entry's group (its record is group << 16 | the entry's low half;
      // entries are in group order).  Up to 64 groups the bucket's
      // boundaries sit one per lane (gbl): the groups before the wave's
      // first position are counted with a ballot, and the (rare) boundaries
      // inside the wave's kBU * 64 positions are stepped over uniformly.
      uint32_t gu[kBU];
      if (NG <= 64) {
        const uint32_t pw = base + (threadIdx.x & ~63u) * kBU;
        // group of p = (boundaries <= p) - 1; positions before the first
        // boundary are outside the bucket (never candidates): clamped to 0
        const uint32_t nle = (uint32_t)__popcll(__ballot(gbl <= pw));
#pragma unroll
        for (int u = 0; u < kBU; u++) gu[u] = nle;
        for (uint64_t c = __ballot(gbl > pw && gbl < pw + 64 * kBU); c; c &= c - 1) {
          const uint32_t bk = __builtin_amdgcn_readlane(gbl, __ffsll((unsigned long long)c) - 1);
#pragma unroll
          for (int u = 0; u < kBU; u++) gu[u] += p0 + u >= bk ? 1u : 0u;
        }
#pragma unroll
        for (int u = 0; u < kBU; u++) gu[u] = gu[u] ? gu[u] - 1 : 0u;
      }
      if (cm && failed == 0) {
        if (NG > 64) {  // the groups by search, stepped forward
          uint32_t g = group_of(gb, NG, p0 + __builtin_ctz(cm));
          uint32_t nb = g + 1 < NG ? gb[g + 1] : kEmpty;  // next boundary
#pragma unroll
          for (int u = 0; u < kBU; u++) {
            if ((cm >> u) & 1u)
              while (nb <= p0 + u) {
                g++;
                nb = g + 1 < NG ? gb[g + 1] : kEmpty;
              }
            gu[u] = g;
          }
        }
        // first probes of the thread's candidates in flight together, four
        // at a time (straight-line, predicated): most land on an empty slot
        // or on their own key; the rest take the probing loop below
        uint32_t slow = 0;
#pragma unroll
        for (int h = 0; h < kBU; h += 4) {
          uint32_t mine[4], old[4];
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int u = h + j;
            mine[j] = kEmpty;
            old[j] = kEmpty;
            if ((cm >> u) & 1u) {
              const uint32_t y = ((x[u] >> 16) * kMapMul) & 0xFFFFu;
              mine[j] = ((y & 7u) << 29) | entry_record(gu[u], x[u]);
              old[j] = atomicCAS(&ht[y >> 3], kEmpty, mine[j]);
            }
          }
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int u = h + j;
            if ((cm >> u) & 1u) {
              const uint32_t sl = x[u] >> 16;
              if (old[j] == kEmpty) continue;  // inserted (its new bit is set at the flush)
              if ((old[j] >> 24) == (mine[j] >> 24)) {
                if ((old[j] & kRecMask) > (mine[j] & kRecMask))
                  atomicMin(&ht[((sl * kMapMul) & 0xFFFFu) >> 3], mine[j]);
              } else {
                slow |= 1u << u;
              }
            }
          }
        }
        while (slow) {  // collisions: probe on from displacement 1
          const int u = __builtin_ctz(slow);
          slow &= slow - 1;
          uint32_t xu = x[0], gk = gu[0];
#pragma unroll
          for (int k = 1; k < kBU; k++) {
            xu = k == u ? x[k] : xu;
            gk = k == u ? gu[k] : gk;
          }
          if (!map_insert(ht, xu >> 16, entry_record(gk, xu), 1)) {
            // the others stop inserting (the bucket is redone)
            __hip_atomic_store(&sh_fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            break;
          }
        }
      }
      if (kDbg) {
        const uint64_t t = clock64();
        ph[5] += t - tk;
        tk = t;
      }
      if (last) break;
      base = next;
#pragma unroll
      for (int u = 0; u < kBU; u++) x[u] = y[u];
    }
    if (tid == 0) {  // the bucket after next
      sh_b[0] = pend_b;
      sh_q[0] = pend_q;
    }
    if (kDbg) {
      const uint64_t t = clock64();
      ph[1] += t - tk;
      tk = t;
    }
    // (a failing insert stored sh_fail before the barrier: a plain barrier and
    // one LDS read cost less than __syncthreads_or, 2.57 -> 2.43 ms per launch)
    lds_barrier();
    const bool spill = __hip_atomic_load(&sh_fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
    if (kDbg) {  // the wait for the block's slowest wave
      const uint64_t t = clock64();
      ph[2] += t - tk;
      tk = t;
    }
    if (spill) {  // map full: redo with the direct table (no global writes yet)
      if (tid == 0) a.spill[atomicAdd(a.nspill, 1u)] = b;
      for (uint32_t i = tid; i < kHash; i += kBThreads) ht[i] = kEmpty;
      for (uint32_t i = tid; i < kBucketWords; i += kBThreads) nbits[i] = 0;
    } else if (kEmit == 2) {
      // the ordered outputs: every new signal with its first record,
      // group-major (the slots read twice: counted per group, then placed;
      // order inside a group is free, the pairs are sorted by record later)
      constexpr int kOwn = kHash / kBThreads;
#pragma unroll
      for (int k = 0; k < kOwn; k++) {
        const uint32_t v = ht[k * kBThreads + tid];
        if (v != kEmpty) {
          atomicAdd(&lcnt[(v & kRecMask) >> kGroupBits], 1u);
          const uint32_t sl = map_signal(k * kBThreads + tid, v);
          atomicOr(&nbits[sl >> 5], 1u << (sl & 31));
        }
      }
      __syncthreads();
      for (uint32_t g = tid; g < a.NG; g += kBThreads) {
        const uint32_t c = lcnt[g];
        lbase[g] = c ? a.goff[(uint64_t)g << kGroupBits] + atomicAdd(&a.gcur[g], (unsigned long long)c) : 0ull;
        lcnt[g] = 0;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kOwn; k++) {
        const uint32_t i = k * kBThreads + tid;
        const uint32_t v = ht[i];
        if (v != kEmpty) {
          const uint32_t r = v & kRecMask, g = r >> kGroupBits;
          a.pairs[lbase[g] + atomicAdd(&lcnt[g], 1u)] = make_uint2(part_sig((b << 16) | map_signal(i, v)), r);
          ht[i] = kEmpty;
        }
      }
      const wvec nb = reinterpret_cast<const wvec*>(nbits)[tid];
      const wvec mw = reinterpret_cast<const wvec*>(mslice)[tid];
      const uint64_t w0 = bucket_word(b, kWPT * tid);
#pragma unroll
      for (int j = 0; j < kWPT; j++)
        if (nb[j]) {
          a.mwords[w0 + j] = mw[j] | nb[j];
          if (a.nwords) a.nwords[w0 + j] = ns[j] | nb[j];
        }
      reinterpret_cast<wvec*>(nbits)[tid] = wvec{};
      __syncthreads();  // (every placement read its lcnt before the reset)
      for (uint32_t g = tid; g < a.NG; g += kBThreads) lcnt[g] = 0;
    } else if (kEmit == 1) {
      // every distinct candidate of the bucket with its first record: the
      // thread's occupied slots counted, one block scan and one global
      // atomic for the bucket's run of pairs, then the slots re-read and
      // written (two barriers per bucket; with the pairs held in registers
      // between two scans, six)
      constexpr int kOwn = kHash / kBThreads;  // slots per thread
      __shared__ uint32_t ewc[kBThreads / 64];
      __shared__ unsigned long long ebase;
      const int lane = tid & 63, w = tid >> 6;
      uint32_t c = 0;
#pragma unroll
      for (int k = 0; k < kOwn; k++) c += ht[k * kBThreads + tid] != kEmpty ? 1u : 0u;
      const uint32_t incl = sgd::wave_incl_add(c);
      if (lane == 63) ewc[w] = incl;
      __syncthreads();
      if (tid == 0) {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < kBThreads / 64; i++) {
          const uint32_t v = ewc[i];
          ewc[i] = acc;
          acc += v;
        }
        ebase = acc ? atomicAdd(a.npairs, (unsigned long long)acc) : 0ull;
      }
      __syncthreads();
      uint64_t pos = ebase + ewc[w] + incl - c;
      if (c) {
#pragma unroll
        for (int k = 0; k < kOwn; k++) {
          const uint32_t i = k * kBThreads + tid;
          const uint32_t v = ht[i];
          if (v != kEmpty) {
            const uint32_t sl = map_signal(i, v);
            const uint32_t sg = part_sig((b << 16) | sl);
            a.pairs[pos++] = make_uint2(sg, a.rec_base + (v & kRecMask));
            if (a.shard_cnt) atomicAdd(&shcnt[shard_of(sg, a.nshards)], 1u);
            if (a.nwords || a.update) atomicOr(&nbits[sl >> 5], 1u << (sl & 31));
            ht[i] = kEmpty;
          }
        }
      }
      __syncthreads();  // nbits complete; ewc / ebase free for the next bucket
      if (a.update) {  // the candidates are the new signals: words kWPT tid .., this block their only writer
        const wvec nb = reinterpret_cast<const wvec*>(nbits)[tid];
        const wvec mw = reinterpret_cast<const wvec*>(mslice)[tid];
        const uint64_t w0 = bucket_word(b, kWPT * tid);
#pragma unroll
        for (int j = 0; j < kWPT; j++)
          if (nb[j]) {
            a.mwords[w0 + j] = mw[j] | nb[j];
            if (a.nwords) a.nwords[w0 + j] = ns[j] | nb[j];
          }
      } else if (a.nwords) {  // the candidates' bits: words kWPT tid .., written by this block alone
        const wvec nb = reinterpret_cast<const wvec*>(nbits)[tid];
        uint32_t* ng = a.nwords + bucket_word(b, kWPT * tid);
#pragma unroll
        for (int j = 0; j < kWPT; j++)
          if (nb[j]) ng[j] = ns[j] | nb[j];
      }
      reinterpret_cast<wvec*>(nbits)[tid] = wvec{};
    } else {
      // a record is queued iff it owns some signal (fuzzer.go:678-690): its
      // flag is set (a record owns signals in many buckets; all set 1)
      constexpr int kOwn = kHash / kBThreads;  // slots per thread
      // the new-signal bits come from the map here, one pass over the slots
      // with the flag stores (an LDS OR per first insert in the rounds cost
      // more: 2.46 -> 2.34 ms per C2 launch), then the word write-back
      {
#pragma unroll
        for (int k = 0; k < kOwn; k++) {
          const uint32_t i = k * kBThreads + tid;
          const uint32_t v = ht[i];
          ht[i] = kEmpty;
          if (v != kEmpty) {
            const uint32_t sl = map_signal(i, v);
            atomicOr(&nbits[sl >> 5], 1u << (sl & 31));
            a.rec_new[v & kRecMask] = 1;
          }
        }
        lds_barrier();
      }
      {
        // words kWPT tid ..: this block is their only writer
        const uint64_t w0 = bucket_word(b, kWPT * tid);
        uint32_t* mg = a.mwords + w0;
        uint32_t* ng = a.nwords ? a.nwords + w0 : nullptr;
        const wvec nb = reinterpret_cast<const wvec*>(nbits)[tid];
        uint32_t any = 0;
#pragma unroll
        for (int j = 0; j < kWPT; j++) any |= nb[j];
        if (any) {
          const wvec mw = reinterpret_cast<const wvec*>(mslice)[tid];
#pragma unroll
          for (int j = 0; j < kWPT; j++)
            if (nb[j]) {
              mg[j] = mw[j] | nb[j];
              if (ng) ng[j] = ns[j] | nb[j];
            }
          reinterpret_cast<wvec*>(nbits)[tid] = wvec{};
        }
      }
    }
    if (kDbg) {
      const uint64_t t = clock64();
      ph[3] += t - tk;
      tk = t;
    }
    lds_barrier();  // sh_b[0] / sh_q[0] are written
    if (kDbg) {
      const uint64_t t = clock64();
      ph[6] += t - tk;
      tk = t;
    }
    b = b1;
    q = q1;
    b1 = uni(sh_b[0]);
    q1 = uni(sh_q[0]);
#pragma unroll
    for (int u = 0; u < kBU; u++) x[u] = y[u];
  }
  if (kEmit == 1) {
    __syncthreads();
    flush_shard_counts(a, shcnt);
  }
  if (kDbg && tid == 0) {
    a.dbg[8 * blockIdx.x] = t_start;
    a.dbg[8 * blockIdx.x + 1] = wall_clock64();
    a.dbg[8 * blockIdx.x + 2] = n_buckets;
    a.dbg[8 * blockIdx.x + 3] = n_rounds;
    for (int j = 0; j < 4; j++) a.dbg[8 * blockIdx.x + 4 + j] = ph[j];
    a.dbg[8 * gridDim.x + 3 * blockIdx.x] = ph[4];
    a.dbg[8 * gridDim.x + 3 * blockIdx.x + 1] = ph[5];
    a.dbg[8 * gridDim.x + 3 * blockIdx.x + 2] = ph[6];
  }
}

// Buckets with too many distinct candidates: a direct first-owner table over
// one eighth of the bucket (8192 signals, 32 KiB of LDS) per job; the
// (bucket, eighth) jobs are independent (each owns its eighth's 256 bitmap
// words), so a few huge spilled buckets spread over many workgroups.
constexpr int kDThreads = 1024;
template <bool kEmit>
__global__ __launch_bounds__(kDThreads) void k_bucket_direct(BucketArgs a) {
  constexpr uint32_t kQ = 8192, kNQ = 65536 / kQ, kQW = kQ / 32;
  __shared__ uint32_t owner[kQ];
  __shared__ uint32_t mpart[kQW];
  __shared__ uint32_t nbits[kQW];
  __shared__ uint32_t gb[kMaxGroups];
  __shared__ uint32_t shcnt[kEmit ? kMaxShards : 1];
  __shared__ uint32_t lcnt[kEmit ? kMaxGroups : 1];
  __shared__ unsigned long long lbase[kEmit ? kMaxGroups : 1];
  const int tid = threadIdx.x;
  const uint32_t nsp = *a.nspill, NG = a.NG;
  if (kEmit) {
    for (uint32_t i = tid; i < kMaxShards; i += kDThreads) shcnt[i] = 0;
    for (uint32_t i = tid; i < kMaxGroups; i += kDThreads) lcnt[i] = 0;
    __syncthreads();
  }
  for (uint32_t job = blockIdx.x; job < nsp * kNQ; job += gridDim.x) {
    const uint32_t b = a.spill[job / kNQ], qq = job % kNQ;
    const uint4 q = a.bdesc[b];
    for (uint32_t i = tid; i < kQW; i += kDThreads) {
      const uint64_t w = bucket_word(b, qq * kQW + i);
      mpart[i] = a.mwords[w] | (a.owords ? a.owords[w] : 0u);
      nbits[i] = 0;
    }
    for (uint32_t i = tid; i < NG; i += kDThreads) gb[i] = a.gbnd[(uint64_t)b * NG + i];
    for (uint32_t i = tid; i < kQ; i += kDThreads) owner[i] = kEmpty;
    __syncthreads();
    for (uint32_t i = q.x + tid; i < q.y; i += kDThreads) {
      const uint32_t x = a.in[i];
      const uint32_t sl = x >> 16, sq = sl % kQ;
      if (sl / kQ != qq || ((mpart[sq >> 5] >> (sq & 31)) & 1u)) continue;
      atomicMin(&owner[sq], entry_record(group_of(gb, NG, i), x));
      atomicOr(&nbits[sq >> 5], 1u << (sq & 31));
    }
    __syncthreads();
    if (kEmit) {
      constexpr int kPer = kQ / kDThreads;
      uint32_t sig[kPer], rec[kPer];
#pragma unroll
      for (int k = 0; k < kPer; k++) {
        const uint32_t i = k * kDThreads + tid;
        sig[k] = part_sig((b << 16) | (qq * kQ + i));
        rec[k] = owner[i];
      }
      if (a.gcur)
        emit_grouped(a, sig, rec, lcnt, lbase);
      else
        emit_pairs(a, sig, rec, shcnt);
      for (uint32_t i = tid; i < kQW; i += kDThreads) {
        const uint32_t nb = nbits[i];
        if (!nb) continue;
        const uint64_t w = bucket_word(b, qq * kQW + i);
        if (a.update) a.mwords[w] = mpart[i] | nb;
        if (a.nwords) a.nwords[w] |= nb;
      }
    } else {
      for (uint32_t i = tid; i < kQ; i += kDThreads)
        if (owner[i] != kEmpty) a.rec_new[owner[i]] = 1;
      for (uint32_t i = tid; i < kQW; i += kDThreads) {
        const uint32_t nb = nbits[i];
        if (nb) {
          const uint64_t w = bucket_word(b, qq * kQW + i);
          a.mwords[w] = mpart[i] | nb;
          if (a.nwords) a.nwords[w] |= nb;
        }
      }
    }
    __syncthreads();
  }
  if (kEmit) flush_shard_counts(a, shcnt);
}

// ------------------------------------------------------------------ scan ---
// Exclusive scan of u32 counts into u32 offsets (totals < 2^32), out[n] = total.
constexpr int kScanThreads = 1024;
constexpr int kScanPer = 16;
constexpr uint32_t kScanTile = kScanThreads * kScanPer;

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  if (tid < 64) {
    const uint32_t x = tid < (int)(blockDim.x >> 6) ? wsum[tid] : 0u;
    uint32_t wi = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(wi, o);
      if (lane >= o) wi += y;
    }
    if (tid < (int)(blockDim.x >> 6)) wsum[tid] = wi - x;
    if (tid == 63) *total = wi;
  }
  __syncthreads();
  return wsum[w] + incl - v;
}

// n_dev (nullable): the element count is (*n_dev) * mul, <= the host bound n.
__device__ __forceinline__ uint64_t scan_n(uint64_t n, const uint32_t* n_dev, uint32_t mul) {
  return n_dev ? (uint64_t)(*n_dev) * mul : n;
}

__global__ __launch_bounds__(kScanThreads) void k_scan32_reduce(const uint32_t* __restrict__ in, uint64_t n,
                                                                const uint32_t* __restrict__ n_dev, uint32_t mul,
                                                                uint32_t* __restrict__ sums) {
  __shared__ uint32_t wsum[16];
  n = scan_n(n, n_dev, mul);
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  uint32_t s = 0;
  if (base < n) {
#pragma unroll
    for (int k = 0; k < kScanPer; k++) {
      const uint64_t i = base + (uint64_t)k * kScanThreads + threadIdx.x;
      s += i < n ? in[i] : 0u;
    }
  }
  for (int o = 32; o; o >>= 1) s += __shfl_down(s, o);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < kScanThreads / 64; w++) t += wsum[w];
    sums[blockIdx.x] = t;
  }
}

// in place, one block: exclusive scan of nb block sums
__global__ __launch_bounds__(kScanThreads) void k_scan32_top(uint32_t* __restrict__ sums, uint64_t nb) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t tot;
  uint32_t carry = 0;
  for (uint64_t b0 = 0; b0 < nb; b0 += kScanThreads) {
    const uint64_t i = b0 + threadIdx.x;
    const uint32_t v = i < nb ? sums[i] : 0u;
    const uint32_t ex = block_excl_scan(v, wsum, &tot);
    if (i < nb) sums[i] = carry + ex;
    carry += tot;
    __syncthreads();
  }
}

__global__ __launch_bounds__(kScanThreads) void k_scan32_apply(const uint32_t* __restrict__ in, uint64_t n,
                                                               const uint32_t* __restrict__ n_dev, uint32_t mul,
                                                               const uint32_t* __restrict__ sums,
                                                               uint32_t* __restrict__ out) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t tot;
  n = scan_n(n, n_dev, mul);
  const uint64_t b_last = n ? (n - 1) / kScanTile : 0;
  if (blockIdx.x > b_last) return;
  // each thread owns kScanPer consecutive counters
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
  const bool full = base + kScanPer <= n;  // in / out are 256-B aligned: 16-B accesses
  uint32_t v[kScanPer];
  uint32_t s = 0;
  if (full) {
#pragma unroll
    for (int k = 0; k < kScanPer; k += 4) {
      const uint4 q = *reinterpret_cast<const uint4*>(in + base + k);
      v[k] = q.x;
      v[k + 1] = q.y;
      v[k + 2] = q.z;
      v[k + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kScanPer; k++) v[k] = base + k < n ? in[base + k] : 0u;
  }
#pragma unroll
  for (int k = 0; k < kScanPer; k++) s += v[k];
  uint32_t run = (sums ? sums[blockIdx.x] : 0u) + block_excl_scan(s, wsum, &tot);
  uint32_t o[kScanPer];
#pragma unroll
  for (int k = 0; k < kScanPer; k++) {
    o[k] = run;
    run += v[k];
  }
  if (full) {
#pragma unroll
    for (int k = 0; k < kScanPer; k += 4)
      *reinterpret_cast<uint4*>(out + base + k) = make_uint4(o[k], o[k + 1], o[k + 2], o[k + 3]);
  } else {
#pragma unroll
    for (int k = 0; k < kScanPer; k++)
      if (base + k < n) out[base + k] = o[k];
  }
  if (blockIdx.x == b_last && threadIdx.x == kScanThreads - 1) out[n] = run;
}

static size_t scan32_ws(uint64_t n) { return (((n + kScanTile - 1) / kScanTile) * 4 + 255) & ~size_t(255); }

// n = host bound; with n_dev the count is (*n_dev) * mul (<= n)
static int scan32(sg_ctx* ctx, const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* scratch,
                  const uint32_t* n_dev = nullptr, uint32_t mul = 1) {
  ScopedTimer tm(ctx, "scan");
  const uint64_t nb = (n + kScanTile - 1) / kScanTile;
  if (nb == 0) {
    SG_HIP(hipMemsetAsync(out, 0, 4, ctx->stream));
    return SG_OK;
  }
  if (nb == 1) {  // one tile: the apply pass alone
    hipLaunchKernelGGL(k_scan32_apply, dim3(1), dim3(kScanThreads), 0, ctx->stream, in, n, n_dev, mul,
                       (const uint32_t*)nullptr, out);
    SG_HIP(hipGetLastError());
    return SG_OK;
  }
  hipLaunchKernelGGL(k_scan32_reduce, dim3((uint32_t)nb), dim3(kScanThreads), 0, ctx->stream, in, n, n_dev, mul,
                     scratch);
  hipLaunchKernelGGL(k_scan32_top, dim3(1), dim3(kScanThreads), 0, ctx->stream, scratch, nb);
  hipLaunchKernelGGL(k_scan32_apply, dim3((uint32_t)nb), dim3(kScanThreads), 0, ctx->stream, in, n, n_dev, mul,
                     scratch, out);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

// ------------------------------------------------------------- M0 filter ---
// The fuzzer's steady state (r06): nearly every entry of a batch is already
// in maxSignal (fuzzer.go:666 ends most records at the SignalNew test; the
// bench's steady batch: 139K candidates among 880M entries), yet pass 2 and
// the bucket stage move every entry.  A random probe of any exact table of
// maxSignal costs each CU ~10 cycles wherever the table lives (L2, Infinity
// Cache or HBM; scripts/micro/m0_filter.hip: 55-91 G probes/s), so the test
// has to be in LDS -- and pass 1 already groups the entries by slice (b2: 2^24
// signals).  A slice's part of maxSignal is ~50K signals (12.8M / 256): too
// many for its 2 MiB of bitmap, few enough for a packed index in LDS:
//   k_m0_index  per slice, one 16-B header per 2^11-signal filter bucket
//               (8192: 128 KiB): up to 8 of the bucket's set positions as
//               16-bit fields (ascending, 0x8000 in the unused ones), or,
//               past 8, the first 7 and in field 7 0x8000 | the block of the
//               next 8 in a small per-slice pool (kFOvBlocks 8-value blocks);
//               the rest (past 15, or past 7 when the pool is full) in the
//               slice's spill list (kFSpill positions; past it, signals are
//               not proven, only re-checked by the tail); one read of the
//               slice's bitmap;
//   k_m0_filter per slice part, the slice's index in LDS (159 KiB); every
//               pass-1 entry reads its bucket's header and the first block of
//               its overflow list (the pool's dummy block 0 for a bucket
//               without one) -- two ds_read_b128, the second one's address
//               from the first -- and compares its position with the 16
//               fields by packed 16-bit xor / min; an entry not found is
//               looked up in the spill list (held in registers, 8 per lane,
//               a wave-wide compare per such entry) and, not there either,
//               survives, as (position, slice);
//   tail        if the survivors fit (kFSurvCap): each survivor still outside
//               maxSignal (the exact bitmap test) gets its record (its pass-1
//               tile by a search over the slice's run starts) and takes
//               min(record) per signal in a hash table; then every distinct
//               signal sets its first owner's flag and its bits in maxSignal
//               and newSignal -- the bucket stage's results (fuzzer.go:669-690)
//               over the candidates.
// When the survivors overflow, pass 2 and the bucket stage run on the same
// pass-1 output.  Option m0_filter -1 (auto, m0f_try) tries the filter after a
// slice it filtered and after a partitioned slice that queued under a quarter
// of its records.
constexpr uint32_t kFRemBits = 11;                      // positions per filter bucket: 2^11
constexpr uint32_t kFBuckets = 1u << (24 - kFRemBits);  // 8192 per slice
constexpr uint32_t kFOvBlocks = 1984;                   // overflow pool per slice: 8-value u16 blocks (31 KiB);
                                                        // block 0 the dummy
constexpr uint32_t kFPad = 0x8000u;                     // an unused field (no position; >= it: a block link)
constexpr uint32_t kFSpill = 512;                       // spill list per index part (8 registers per lane)
constexpr uint32_t kFHMax = 4;                          // index parts per slice, at most (option m0_filter_halves)
constexpr uint32_t kFIdx = 256 * kFHMax;                // index parts in all
constexpr uint32_t kFSurvCap = 1u << 20;                // survivors per launch
constexpr uint32_t kFTableBits = 21;                    // the tail's table: 2^21 u64 slots
constexpr int kFThreads = 1024;
#ifndef SG_FPARTS
#define SG_FPARTS 8
#endif
#ifndef SG_FU
#define SG_FU 4  // 16-B entry loads per thread per step
#endif
#ifndef SG_FEH
#define SG_FEH 4  // entries whose LDS reads are in flight together
#endif
#ifndef SG_FABL
#define SG_FABL 0  // diagnostics builds (wrong results): 1 the entry stream only, 2 no overflow block reads,
                   // 3 no entry stream past the first three steps, 4 overflow reads at random
                   // blocks, independent of the header, 5 the same, mostly the dummy block
#endif
constexpr uint32_t kFParts = SG_FPARTS;                 // filter workgroups per slice
constexpr uint32_t kFWgCap = 4 * kFSurvCap / (256 * kFParts);  // survivors per filter workgroup (its own region:
                                                              // 4x the mean share at the cap, 32 MiB in all)
constexpr unsigned long long kFEmpty = ~0ull;

struct M0F {
  uint4* tab;                 // [index part][bucket] headers (part = slice << log H | half)
  uint16_t* ovals;            // [index part][8 kFOvBlocks] overflow pool
  uint32_t* cursor;           // [index part] overflow blocks placed (may pass the pool)
  uint32_t* nspill;           // [index part] spilled positions (may pass kFSpill)
  uint32_t* spill;            // [index part][kFSpill] positions in the slice
  uint32_t* nsurv;            // [0] survivors in the regions that held theirs, [1] != 0: some region overflowed,
                              // [2] != 0: some index part overflowed (values past its pool and spill list)
  uint2* surv;                // (position, slice), kFWgCap per filter workgroup
  uint32_t* wgcnt;            // [filter workgroup] survivors in its region
  unsigned long long* table;  // signal << 32 | min record; kFEmpty between launches
};
static size_t m0f_bytes() {
  return (uint64_t)kFIdx * kFBuckets * 16 + (uint64_t)kFIdx * kFOvBlocks * 16 + kFIdx * 4 + 256 + kFIdx * 4 +
         (uint64_t)kFIdx * kFSpill * 4 + 256ull * kFParts * kFWgCap * 8 +
         256ull * kFParts * 4 + (8ull << kFTableBits);
}
static M0F m0f_bind(sg_ctx* ctx) {
  char* b = (char*)ctx->m0f;
  M0F f;
  f.tab = (uint4*)b;
  b += (uint64_t)kFIdx * kFBuckets * 16;
  f.ovals = (uint16_t*)b;
  b += (uint64_t)kFIdx * kFOvBlocks * 16;
  f.cursor = (uint32_t*)b;
  f.nsurv = f.cursor + kFIdx;
  f.nspill = f.cursor + kFIdx + 64;
  b += kFIdx * 4 + 256 + kFIdx * 4;
  f.spill = (uint32_t*)b;
  b += (uint64_t)kFIdx * kFSpill * 4;
  f.surv = (uint2*)b;
  b += 256ull * kFParts * kFWgCap * 8;
  f.wgcnt = (uint32_t*)b;
  b += 256ull * kFParts * 4;
  f.table = (unsigned long long*)b;
  return f;
}

// grid (kFBuckets / 256, 256): thread t of block (e, d) indexes filter
// bucket 256 e + t of slice d, its 64 bitmap words (256 B) read as 16 quads;
// it walks their set bits in order into its header's fields and its overflow
// list, whose blocks one cursor add per wave places.  (A wave per 64 buckets,
// lane l holding word l of each, measured 0.40-0.45 ms per steady step: 128
// wave scans per 64 buckets; this form 0.24 ms.)
// kLogH: the slice's index in 2^kLogH parts (halves h of its positions, each
// with its own 8192 buckets of 2^(11 - kLogH) positions, pool and spill list:
// past ~14M signals of maxSignal one part no longer holds a slice); grid
// (kFBuckets / 256, 256 << kLogH), blockIdx.y = slice << kLogH | h.
template <int kLogH>
__global__ __launch_bounds__(256) void k_m0_index(const uint32_t* __restrict__ mwords, uint4* __restrict__ tab,
                                                   uint16_t* __restrict__ ovals, uint32_t* __restrict__ cursor,
                                                   uint32_t* __restrict__ nspill, uint32_t* __restrict__ spill,
                                                   uint32_t* __restrict__ flags) {
  constexpr int kQ = 16 >> kLogH;                // bitmap quads per bucket
  constexpr uint32_t kRB = kFRemBits - kLogH;    // position bits in a bucket
  const uint32_t dh = blockIdx.y, lane = threadIdx.x & 63;
  const uint32_t d = dh >> kLogH, h = dh & ((1u << kLogH) - 1);
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  const uint4* src = reinterpret_cast<const uint4*>(mwords + ((uint64_t)d << 19) + ((uint64_t)h << (19 - kLogH)) +
                                                    (uint64_t)j * (4 * kQ));
  uint4 q[kQ];
#pragma unroll
  for (int i = 0; i < kQ; i++) q[i] = src[i];
  uint32_t n = 0;
#pragma unroll
  for (int i = 0; i < kQ; i++) n += __popc(q[i].x) + __popc(q[i].y) + __popc(q[i].z) + __popc(q[i].w);
  // the overflow block of a bucket past 8 values
  const uint32_t ob = n > 8 ? 1u : 0u;
  const uint32_t oi = sgd::wave_incl_add(ob);
  const uint32_t otot = (uint32_t)__builtin_amdgcn_readlane((int)oi, 63);
  uint32_t obase = 0;
  if (lane == 0 && otot) obase = atomicAdd(&cursor[dh], otot);
  obase = (uint32_t)__builtin_amdgcn_readfirstlane((int)obase);
  const uint32_t ost = 1 + obase + oi - ob;  // first block (block 0: none, the filter's dummy)
  const bool ok = ob && ost + ob <= kFOvBlocks;  // (else the rest is spilled)
  uint16_t* out = ovals + ((uint64_t)dh * kFOvBlocks + ost) * 8;
  const uint32_t kin = n > 8 ? 7u : 8u;  // values in the header
  // the spill list's slots for the rest (past 15 values, or past 7 with the
  // pool full), one add per wave (past the index's capacity, an add per
  // spilled value -- ~10^4-10^5 per slice on one counter -- took 3.7-14 ms at
  // an 18-41M maxSignal)
  const uint32_t kst = ok ? 15u : 7u, nsw = n > 8 && n > kst ? n - kst : 0u;
  const uint32_t si = sgd::wave_incl_add(nsw);
  const uint32_t stot = (uint32_t)__builtin_amdgcn_readlane((int)si, 63);
  uint32_t sbase = 0;
  if (lane == 0 && stot) sbase = atomicAdd(&nspill[dh], stot);
  sbase = (uint32_t)__builtin_amdgcn_readfirstlane((int)sbase) + si - nsw;
  if (nsw && sbase + nsw > kFSpill) flags[2] = 1u;  // (values past the part's capacity: a larger H would hold them)
  uint64_t lo = 0, hi = 0;               // fields 0..3, 4..7
  uint32_t k = 0;
#pragma unroll
  for (int i = 0; i < kQ; i++) {
    const uint32_t wq[4] = {q[i].x, q[i].y, q[i].z, q[i].w};
#pragma unroll
    for (int c = 0; c < 4; c++) {
      uint32_t m = wq[c];
      while (m) {
        const uint32_t v = (uint32_t)(32 * (4 * i + c)) + (uint32_t)__builtin_ctz(m);  // ascending in k
        m &= m - 1;
        if (k < kin) {
          if (k < 4)
            lo |= (uint64_t)v << (16 * k);
          else
            hi |= (uint64_t)v << (16 * (k - 4));
        } else if (ok && k < 15) {
          out[k - 7] = (uint16_t)v;
        } else {  // (rare: past 15 values, or the pool full)
          const uint32_t at = sbase + k - kst;
          if (at < kFSpill) spill[(uint64_t)dh * kFSpill + at] = (h << (24 - kLogH)) | (j << kRB) | v;
        }
        k++;
      }
    }
  }
  for (uint32_t f = min(n, kin); f < 8; f++) {  // unused fields, and field 7 past 8 values
    const uint64_t v = f == 7 && n > 8 && ok ? kFPad | ost : kFPad;
    if (f < 4)
      lo |= v << (16 * f);
    else
      hi |= v << (16 * (f - 4));
  }
  if (ok)
    for (uint32_t t = n - 7; t < 8; t++) out[t] = (uint16_t)kFPad;  // the block's padding
  tab[(uint64_t)dh * kFBuckets + j] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

typedef unsigned short m0f_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t m0f_min16(uint32_t a, uint32_t b) {  // v_pk_min_u16
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(m0f_u16x2, a),
                                                               __builtin_bit_cast(m0f_u16x2, b)));
}

// grid (kFParts, 256): part x of slice d's pass-1 run.  Per thread and step
// 4 SG_FU entries, the next two steps' loads in flight while one is tested.
// A survivor is written as (position, slice).
template <int kLogH>
__global__ __launch_bounds__(kFThreads) void k_m0_filter(const uint32_t* __restrict__ v1,
                                                          const uint32_t* __restrict__ goff1, uint32_t T,
                                                          const uint4* __restrict__ tab,
                                                          const uint16_t* __restrict__ ovals,
                                                          const uint32_t* __restrict__ cursor,
                                                          const uint32_t* __restrict__ nspill,
                                                          const uint32_t* __restrict__ spill,
                                                          uint2* __restrict__ surv, uint32_t* __restrict__ nsurv,
                                                          uint32_t* __restrict__ wgcnt) {
  constexpr uint32_t logh = kLogH;  // (a constant: as a kernel argument its shifts cost 0.1 ms per launch)
  // the overflow pool, then the headers (one array: both bases fit the
  // ds_read offset field)
  __shared__ v4u32 lds[kFOvBlocks + kFBuckets];
  // the workgroup's survivors so far, in its own region of surv (an LDS
  // cursor: a returning global atomic per survivor wave makes the compiler
  // wait for every load in flight, the next step's entries included; one
  // counter read by every wave each step measured 12 ms per C2 step)
  __shared__ uint32_t wsurv;
  // grid (parts, 256, 2^logh): part x of slice d's run against index part hp
  // (the positions p with p >> (24 - logh) == hp; the other entries pass as
  // found -- each entry is tested by exactly one index part)
  const uint32_t d = blockIdx.y, hp = blockIdx.z, dh = (d << logh) | hp, tid = threadIdx.x, lane = tid & 63;
  const uint32_t R0 = goff1[(uint64_t)d * T], R1 = goff1[(uint64_t)(d + 1) * T];
  const uint64_t len = R1 - R0;
  const uint32_t a = R0 + (uint32_t)(len * blockIdx.x / gridDim.x), b = R0 + (uint32_t)(len * (blockIdx.x + 1) / gridDim.x);
  const uint32_t wg = dh * gridDim.x + blockIdx.x;
  if (a >= b) {
    if (tid == 0) wgcnt[wg] = 0;
    return;
  }
  const uint32_t rb = kFRemBits - logh;  // position bits in a bucket
  constexpr uint32_t topm = logh ? ~0u << (32 - logh) : 0u;  // (the part's bits of an entry)
  const uint32_t toph = logh ? hp << ((32 - logh) & 31) : 0u;
  const uint32_t nob = min(cursor[dh] + 1, kFOvBlocks);
  uint2* wsv = surv + (uint64_t)wg * kFWgCap;
  if (tid == 0) wsurv = 0;
  const v4u32* hsrc = reinterpret_cast<const v4u32*>(tab + (uint64_t)dh * kFBuckets);
  {
    v4u32 t[kFBuckets / kFThreads];  // (all in flight, then stored)
#pragma unroll
    for (uint32_t u = 0; u < kFBuckets / kFThreads; u++) t[u] = hsrc[tid + u * kFThreads];
#pragma unroll
    for (uint32_t u = 0; u < kFBuckets / kFThreads; u++) lds[kFOvBlocks + tid + u * kFThreads] = t[u];
  }
  const v4u32* osrc = reinterpret_cast<const v4u32*>(ovals + (uint64_t)dh * kFOvBlocks * 8);
  for (uint32_t i = 1 + tid; i < nob; i += kFThreads) lds[i] = osrc[i];
  if (tid == 0) lds[0] = v4u32{kFPad * 0x10001u, kFPad * 0x10001u, kFPad * 0x10001u, kFPad * 0x10001u};  // dummy
  // the spill list, entry 64 i + lane in sp[i] (~0u: none)
  const uint32_t nsp = min(nspill[dh], kFSpill);
  uint32_t sp[kFSpill / 64];
#pragma unroll
  for (int i = 0; i < (int)(kFSpill / 64); i++)
    sp[i] = 64 * i + lane < nsp ? spill[(uint64_t)dh * kFSpill + 64 * i + lane] : ~0u;
  __syncthreads();
  // 4 SG_FU entries per thread per step, two more steps in flight (one
  // 16-wave workgroup per CU holds the LDS index, so the stream's depth is
  // per thread)
  constexpr int U = SG_FU;
  constexpr int E = 4 * U;
  constexpr int EH = SG_FEH;
  const uint32_t qa = a & ~3u;
  constexpr uint32_t kStep = 4 * kFThreads * U;
  // (unpredicated loads, clamped to the run's last quad: a load under a
  // branch makes the compiler wait for every load in flight at the join, the
  // next steps' included -- the step then paid a whole memory latency)
  const uint32_t qlast = (b - 1) & ~3u;
  auto load = [&](uint32_t q0, uint32_t(&en)[E]) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (SG_FABL == 3 && q0 >= qa + 4 * tid + 3 * kStep) break;
      const uint32_t q = min(q0 + 4 * kFThreads * u, qlast);
      const v4u32 t = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(v1 + q));
      en[4 * u] = t[0];
      en[4 * u + 1] = t[1];
      en[4 * u + 2] = t[2];
      en[4 * u + 3] = t[3];
    }
  };
  // Three entry buffers in rotation (a register copy from a buffer whose
  // loads are in flight would wait for them): step i tests one while the
  // next two steps' loads land in the others.
  uint32_t bA[E], bB[E], bC[E];
  auto step = [&](uint32_t q0, const uint32_t(&e)[E]) {
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&wsurv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) >
        kFWgCap)
      return;  // (overflowing: the partition goes on)
    // the entries inside [a, b): all of them unless the wave's step crosses
    // an end of the part (a uniform test)
    const uint32_t qw = (uint32_t)__builtin_amdgcn_readfirstlane((int)q0);  // lane 0's
    uint32_t vm = (1u << E) - 1;
    const bool full = qw >= a && qw + 4 * 63 + 3 + 4 * kFThreads * (U - 1) < b;
    if (!full) {
      vm = 0;
#pragma unroll
      for (int k = 0; k < E; k++)
        vm |= (q0 + 4 * kFThreads * (k >> 2) + (k & 3) - a < b - a ? 1u : 0u) << k;
    }
    // Branch-free per entry: the header and its overflow list's first block
    // (else the dummy block 0) are read for every entry; a position past the
    // first block (a bucket past 15 values) is not proven here and survives
    // -- the tail re-checks every survivor against the bitmap.
    uint32_t hm = 0;  // bit k: entry k found
    uint32_t sk = 0;  // the last entry not found (the only survivor of most lanes that have one)
#pragma unroll
    for (int k0 = 0; k0 < E; k0 += EH) {
      if (SG_FABL == 1) {
#pragma unroll
        for (int k = 0; k < EH; k++) hm |= (e[k0 + k] == 0x12345678u ? 0u : 1u) << (k0 + k);
        continue;
      }
      v4u32 h[EH];
#pragma unroll
      for (int k = 0; k < EH; k++) h[k] = lds[kFOvBlocks + ((e[k0 + k] >> (8 + rb)) & (kFBuckets - 1))];
      v4u32 o[EH];
#pragma unroll
      for (int k = 0; k < EH; k++)
        o[k] = SG_FABL == 2   ? h[k]
               : SG_FABL == 4 ? lds[1 + ((e[k0 + k] >> 8) & 1023u)]
               : SG_FABL == 5 ? lds[(e[k0 + k] & 0x80000000u) ? 1u : 0u]
                              : lds[__builtin_elementwise_sub_sat(h[k][3] >> 16, kFPad)];
#pragma unroll
      for (int kk = 0; kk < EH; kk++) {
        const uint32_t rep = ((e[k0 + kk] >> 8) & ((1u << rb) - 1)) * 0x10001u;
        const uint32_t m = m0f_min16(m0f_min16(m0f_min16(h[kk][0] ^ rep, h[kk][1] ^ rep),
                                               m0f_min16(h[kk][2] ^ rep, h[kk][3] ^ rep)),
                                     m0f_min16(m0f_min16(o[kk][0] ^ rep, o[kk][1] ^ rep),
                                               m0f_min16(o[kk][2] ^ rep, o[kk][3] ^ rep)));
        const bool hit = min(m & 0xFFFFu, m >> 16) == 0 || (logh && (e[k0 + kk] & topm) != toph);
        hm |= (hit ? 1u : 0u) << (k0 + kk);
        sk = hit ? sk : e[k0 + kk];
      }
    }
    uint32_t svm = vm & ~hm;  // bit k: entry k survives
    if (SG_FABL) svm = svm == 0x5A5Au ? 1u : 0u;
    const uint64_t anysv = __ballot(svm != 0);
    if (anysv && full && !__ballot(svm & (svm - 1))) {
      // (rare in the steady state) at most one survivor per lane, entry sk:
      // its position against the spill list (all lanes comparing their part
      // of it, one survivor lane after the other), then one slot per survivor
      bool sv = svm != 0;
      if (nsp) {
        const uint32_t key = (sk >> 8) & 0xFFFFFFu;
        for (uint64_t bal = anysv; bal; bal &= bal - 1) {
          const int l = __builtin_ctzll(bal);
          const uint32_t kl = (uint32_t)__builtin_amdgcn_readlane((int)key, l);
          bool f = false;
#pragma unroll
          for (int i = 0; i < (int)(kFSpill / 64); i++) f |= sp[i] == kl;
          if (__ballot(f) && lane == (uint32_t)l) sv = false;
        }
      }
      const uint64_t bal = __ballot(sv);
      if (bal) {
        const int first = __builtin_ctzll(bal);
        uint32_t at = 0;
        if (lane == (uint32_t)first) at = atomicAdd(&wsurv, (uint32_t)__popcll(bal));
        at = (uint32_t)__shfl((int)at, first) + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
        const uint32_t k = (uint32_t)__builtin_ctz(svm | 0x80000000u);
        if (sv && at < kFWgCap) wsv[at] = make_uint2(q0 + 4 * kFThreads * (k >> 2) + (k & 3), d);
      }
    } else if (anysv) {  // several survivors in a lane, or a step across an end of the part
      if (nsp) {
        // each entry not found so far: its position against the spill list,
        // all lanes comparing their part of it
#pragma unroll
        for (int k = 0; k < E; k++) {
          uint64_t bal = __ballot((svm >> k) & 1u);
          while (bal) {
            const int l = __builtin_ctzll(bal);
            bal &= bal - 1;
            const uint32_t key = (uint32_t)__builtin_amdgcn_readlane((int)(e[k] >> 8), l) & 0xFFFFFFu;
            bool f = false;
#pragma unroll
            for (int i = 0; i < (int)(kFSpill / 64); i++) f |= sp[i] == key;
            if (__ballot(f) && lane == (uint32_t)l) svm &= ~(1u << k);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < E; k++) {
        const bool sv = (svm >> k) & 1u;
        const uint64_t bal = __ballot(sv);
        if (!bal) continue;
        const uint32_t p = q0 + 4 * kFThreads * (k >> 2) + (k & 3);
        const int first = __builtin_ctzll(bal);
        uint32_t at = 0;
        if (lane == (uint32_t)first) at = atomicAdd(&wsurv, (uint32_t)__popcll(bal));
        at = (uint32_t)__shfl((int)at, first) + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
        if (sv && at < kFWgCap) wsv[at] = make_uint2(p, d);
      }
    }
  };
  // A wave-uniform loop with one exit, three steps per iteration (lane 0's
  // position qw; every lane runs every step, the positions past b masked by
  // vm, up to two steps past the end).  vmcnt counts in issue order, and the
  // compiler's waits are merged over every path into the loop head: a
  // per-lane exit (a divergent loop), an exit between steps, or the
  // scheduler issuing bA's prologue loads last each made the first step wait
  // for every load in flight.
  uint32_t q0 = qa + 4 * tid;
  uint32_t qw = (uint32_t)__builtin_amdgcn_readfirstlane((int)q0);
  load(q0, bA);
  __builtin_amdgcn_sched_barrier(0);
  load(q0 + kStep, bB);
  __builtin_amdgcn_sched_barrier(0);
  load(q0 + 2 * kStep, bC);
  __builtin_amdgcn_sched_barrier(0);
  while (qw < b) {
    step(q0, bA);
    load(q0 + 3 * kStep, bA);  // (each buffer reloaded right after its step)
    q0 += kStep;
    step(q0, bB);
    load(q0 + 3 * kStep, bB);
    q0 += kStep;
    step(q0, bC);
    load(q0 + 3 * kStep, bC);
    q0 += kStep;
    qw += 3 * kStep;
  }
  __syncthreads();
  if (tid == 0) {
    const uint32_t c = wsurv;
    wgcnt[wg] = c;
    // the total, and a flag past a region (the host then partitions).  (Once
    // the total for an overflowed region was kFSurvCap + 1: 4096 of them
    // wrapped the 32-bit sum to a small count, the tail took the survivors
    // for fitting, and its table filled -- a hang at 16 workgroups per slice.)
    if (c > kFWgCap)
      atomicOr(nsurv + 1, 1u);
    else
      atomicAdd(nsurv, c);
  }
}

__device__ __forceinline__ uint32_t m0f_hash(uint32_t s) {
  s ^= s >> 16;
  s *= 0x7FEB352Du;
  s ^= s >> 15;
  return s;
}

// the survivors still outside maxSignal (a value past an index cap is only
// re-checked here): each one's record (its pass-1 tile by a search over the
// slice's run starts), then min(record) per signal
__global__ void k_m0_tail_insert(const uint2* __restrict__ surv, const uint32_t* __restrict__ wgcnt,
                                 const uint32_t* __restrict__ v1,
                                 const uint32_t* __restrict__ goff1, uint32_t T, const uint32_t* __restrict__ trec,
                                 const uint32_t* __restrict__ mwords, unsigned long long* __restrict__ table) {
  // grid (4, filter workgroups): the survivors of region y, strided
  const uint32_t nw = min(wgcnt[blockIdx.y], kFWgCap);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += gridDim.x * blockDim.x) {
  const uint2 q = surv[(uint64_t)blockIdx.y * kFWgCap + i];  // (position, slice)
  const uint32_t e = v1[q.x], t = (q.y << 24) | (e >> 8);
  if ((mwords[t >> 5] >> (t & 31)) & 1u) continue;
  const uint32_t s = part_sig(t);
  const uint32_t rec = trec[last_le(goff1 + (uint64_t)q.y * T, 0, T, q.x)] + (e & 0xFFu);
  const unsigned long long key = ((unsigned long long)s << 32) | rec;
  constexpr uint32_t mask = (1u << kFTableBits) - 1;
  // (bounded: at most kFSurvCap keys in 2^21 slots, so a free or equal slot
  // always comes first; the bound only keeps a broken invariant from hanging)
  for (uint32_t h = m0f_hash(s) & mask, probe = 0; probe <= mask; h = (h + 1) & mask, probe++) {
    const unsigned long long old = atomicCAS(&table[h], kFEmpty, key);
    if (old == kFEmpty) break;
    if ((uint32_t)(old >> 32) == s) {
      if (old > key) atomicMin(&table[h], key);
      break;
    }
  }
  }
}

// every distinct new signal: its first owner queued, its bits set (and the
// slot emptied for the next launch)
__global__ void k_m0_tail_flush(unsigned long long* __restrict__ table, uint32_t* __restrict__ mwords,
                                uint32_t* __restrict__ nwords, uint8_t* __restrict__ rec_new) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long v = table[i];
  if (v == kFEmpty) return;
  table[i] = kFEmpty;
  rec_new[(uint32_t)v] = 1;
  const uint32_t t = part_key((uint32_t)(v >> 32)), bit = 1u << (t & 31);
  atomicOr(&mwords[t >> 5], bit);
  if (nwords) atomicOr(&nwords[t >> 5], bit);
}

// ------------------------------------------------------------------ host ---
struct BucketPlan {
  uint64_t n, nrec, nA, nB, T, NG, ng, gmax;
  WsPlan p;
  size_t oTS, oTR, oGT, oH1, oO1, oV1, oB1, oNC, oCB, oCS, oCG, oCF, oCD, oDT, oBD, oGB, oH2, oO2, oV2, oSP, oTK, oBN, oBP,
      oLB, oLQ, oSC, oKM;
  BucketPlan(uint64_t n_, uint64_t nrec_) : n(n_), nrec(nrec_) {
    nA = (n + kPT - 1) / kPT;
    nB = nrec ? (nrec - 1) / kRecCap : 0;
    T = nA + nB;
    NG = nrec ? (nrec - 1) / kGroupRecs + 1 : 1;
    ng = 256 * NG;
    gmax = ng + nA;  // sum over slice-groups of ceil(size / kPT) <= ng + n / kPT
    oTS = p.add((T + 1) * 4);
    oTR = p.add((T + 1) * 4);
    oGT = p.add((NG + 1) * 4);
    oH1 = p.add(256 * T * 4);
    oO1 = p.add((256 * T + 1) * 4);
    oV1 = p.add(n * 4);
    oB1 = p.add(n + 64);  // pass-1 top bytes; k_hist_bytes reads 16-B quads past the end
    oNC = p.add(ng * 4);
    oCB = p.add((ng + 1) * 4);
    oCS = p.add((gmax + 1) * 4);
    oCG = p.add((gmax + 1) * 4);
    oCF = p.add(257 * 4);
    oCD = p.add(gmax * 16);
    oDT = p.add(gmax * 8);
    oBD = p.add((uint64_t)kNumBuckets * 16);
    oGB = p.add((uint64_t)kNumBuckets * NG * 4);
    oH2 = p.add(256 * gmax * 4);
    oO2 = p.add((256 * gmax + 1) * 4);
    oV2 = p.add(n * 4 + 64);  // the bucket kernel's 16-B loads may read past the end
    oSP = p.add(((uint64_t)kNumBuckets + 1) * 4);
    oTK = p.add(4);
    oBN = p.add((uint64_t)kNumBuckets * 4);
    oBP = p.add(((uint64_t)kNumBuckets + 1) * 4);
    oLB = p.add((uint64_t)kNumBuckets * 4);
    oLQ = p.add((uint64_t)kNumBuckets * 16);
    oSC = p.add(scan32_ws(256 * (gmax > T ? gmax : T)));
    oKM = p.add(T * (kPT / 8));  // trace batches: kept-entry words
  }
  void rebase(size_t b) {
    for (size_t* o : {&oTS, &oTR, &oGT, &oH1, &oO1, &oV1, &oB1, &oNC, &oCB, &oCS, &oCG, &oCF, &oCD, &oDT, &oBD, &oGB, &oH2,
                      &oO2, &oV2, &oSP, &oTK, &oBN, &oBP, &oLB, &oLQ, &oSC, &oKM})
      *o += b;
  }
};

size_t bucket_plan_bytes(uint64_t n, uint64_t nrec) { return BucketPlan(n, nrec).p.total; }

static_assert(kMaxLaunchRecords == (uint64_t)kMaxGroups * kGroupRecs, "records per partitioned launch");

// Grid of a persistent kernel: every block resident at once (CUs x blocks
// per CU from the occupancy query), cached per kernel.
uint32_t persistent_grid(sg_ctx* ctx, const void* kernel, int threads) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, uint32_t> cache;
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_pair(ctx->device, kernel);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu < 1)
    per_cu = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus < 1)
    cus = 256;
  const uint32_t grid = (uint32_t)(per_cu * cus);
  cache[key] = grid;
  return grid;
}

// Stage A of one partitioned launch: tiles, both partition passes, the
// bucket descriptors and the list of non-empty buckets, in the workspace from
// ws_base (reserved by the caller when `reserved`).  n > 0, nrec > 0.
// stages: 1 the tiles and pass 1 (then bp is rebased), 2 the rest (after a
// stage-1 call with the same bp), 3 both.  plane: pass 1 writes the pass-2
// digit plane (else stage 2 needs k_top_plane first).
static int partition_one(sg_ctx* ctx, const uint32_t* d_vals, const uint64_t* d_off, uint64_t n, uint64_t nrec,
                         size_t ws_base, bool reserved, BucketPlan& bp, bool trace = false, int stages = 3,
                         bool plane = true) {
  int rc = SG_OK;
  if (stages & 1) {
    if (256 * bp.gmax >= 0xFFFFFFFFull || bp.NG > kMaxGroups) {
      set_error("bucket triage: batch too large");
      return SG_EINVAL;
    }
    rc = reserved ? SG_OK : ws_reserve(ctx, ws_base + bp.p.total);
    if (rc) return rc;
    if (ctx->ws_cap < ws_base + bp.p.total) {
      set_error("bucket triage: workspace not reserved");
      return SG_EINVAL;
    }
    bp.rebase(ws_base);
  }
  uint32_t* tstart = (uint32_t*)ws_at(ctx, bp.oTS);
  uint32_t* trec = (uint32_t*)ws_at(ctx, bp.oTR);
  uint32_t* gt = (uint32_t*)ws_at(ctx, bp.oGT);
  uint32_t* hist1 = (uint32_t*)ws_at(ctx, bp.oH1);
  uint32_t* goff1 = (uint32_t*)ws_at(ctx, bp.oO1);
  uint32_t* v1 = (uint32_t*)ws_at(ctx, bp.oV1);
  uint8_t* b1 = (uint8_t*)ws_at(ctx, bp.oB1);
  uint32_t* nch = (uint32_t*)ws_at(ctx, bp.oNC);
  uint32_t* cbase = (uint32_t*)ws_at(ctx, bp.oCB);
  uint32_t* cstart = (uint32_t*)ws_at(ctx, bp.oCS);
  uint32_t* cgov = (uint32_t*)ws_at(ctx, bp.oCG);
  uint32_t* cfirst = (uint32_t*)ws_at(ctx, bp.oCF);
  uint4* cdesc = (uint4*)ws_at(ctx, bp.oCD);
  uint2* dtile = (uint2*)ws_at(ctx, bp.oDT);
  uint4* bdesc = (uint4*)ws_at(ctx, bp.oBD);
  uint32_t* gbnd = (uint32_t*)ws_at(ctx, bp.oGB);
  uint32_t* hist2 = (uint32_t*)ws_at(ctx, bp.oH2);
  uint32_t* goff2 = (uint32_t*)ws_at(ctx, bp.oO2);
  uint32_t* v2 = (uint32_t*)ws_at(ctx, bp.oV2);
    uint32_t* scr = (uint32_t*)ws_at(ctx, bp.oSC);
  const uint32_t T = (uint32_t)bp.T, G = (uint32_t)bp.gmax, NG = (uint32_t)bp.NG;
  const uint32_t* gcount = cbase + bp.ng;  // device: number of pass-2 chunks
  const bool dbg = ctx->debug_part;
  if (stages & 1) {
  // pass-1 tiles
  Cuts c1{};
  c1.nA = bp.nA;
  c1.step = kPT;
  c1.nB = bp.nB;
  c1.n = n;
  c1.rec_off = d_off;
  c1.nrec = nrec;
  c1.start = tstart;
  c1.aux = trec;
  hipLaunchKernelGGL(k_cuts, dim3(div_up(bp.T + 1, 256)), dim3(256), 0, ctx->stream, c1);
  hipLaunchKernelGGL(k_group_tiles, dim3(div_up(bp.NG + 1, 256)), dim3(256), 0, ctx->stream, d_off, bp.nA, NG, T,
                     gt);
  {
    ScopedTimer tm(ctx, "p1_hist");
    if (trace)
      hipLaunchKernelGGL(k_hist_trace, dim3(T), dim3(kPThreads), 0, ctx->stream, d_vals, d_off, nrec,
                         (const uint32_t*)tstart, (const uint32_t*)trec, T, hist1, (uint64_t*)ws_at(ctx, bp.oKM));
    else if (((uintptr_t)d_vals & 15) == 0)
      hipLaunchKernelGGL(k_hist_rep<false>, dim3(T), dim3(kPThreads), 0, ctx->stream, d_vals,
                         (const uint32_t*)tstart, (const uint4*)nullptr, T, (const uint32_t*)nullptr, hist1);
    else
      hipLaunchKernelGGL(k_p1_hist, dim3(T), dim3(kPThreads), 0, ctx->stream, d_vals,
                         (const uint32_t*)tstart, hist1);
  }
  rc = scan32(ctx, hist1, goff1, 256 * bp.T, scr);
  if (rc) return rc;
  P1Args a1{d_vals, d_off, nrec, tstart, trec, T, goff1, hist1, v1, plane ? b1 : nullptr, nullptr,
            (const uint64_t*)ws_at(ctx, bp.oKM)};
  unsigned long long* p1dbg = nullptr;
  if (dbg) {
    SG_HIP(hipMalloc(&p1dbg, 64));
    SG_HIP(hipMemsetAsync(p1dbg, 0, 64, ctx->stream));
    a1.dbg = p1dbg;
  }
  {
    ScopedTimer tm(ctx, "p1_scatter");
    if (dbg && trace)
      hipLaunchKernelGGL((k_p1_scatter<true, true>), dim3(T), dim3(kPThreads), 0, ctx->stream, a1);
    else if (dbg)
      hipLaunchKernelGGL((k_p1_scatter<true, false>), dim3(T), dim3(kPThreads), 0, ctx->stream, a1);
    else if (trace)
      hipLaunchKernelGGL((k_p1_scatter<false, true>), dim3(T), dim3(kPThreads), 0, ctx->stream, a1);
    else
      hipLaunchKernelGGL((k_p1_scatter<false, false>), dim3(T), dim3(kPThreads), 0, ctx->stream, a1);
  }
  if (dbg) {
    unsigned long long h[8];
    SG_HIP(hipMemcpy(h, p1dbg, 64, hipMemcpyDeviceToHost));
    SG_HIP(hipFree(p1dbg));
    fprintf(stderr, "sg p1_scatter per tile (cycles, wave 0): load+meta %.0f build+lookup %.0f rank %.0f stage %.0f "
            "write %.0f (tiles %llu)\n", (double)h[0] / h[5], (double)h[1] / h[5], (double)h[2] / h[5],
            (double)h[3] / h[5], (double)h[4] / h[5], h[5]);
  }
  }
  if (!(stages & 2)) return SG_OK;
  // pass-2 chunks
  hipLaunchKernelGGL(k_group_chunks, dim3(div_up(bp.ng, 256)), dim3(256), 0, ctx->stream, (const uint32_t*)goff1,
                     T, NG, (const uint32_t*)gt, bp.ng, nch);
  rc = scan32(ctx, nch, cbase, bp.ng, scr);
  if (rc) return rc;
  hipLaunchKernelGGL(k_chunk_list, dim3(div_up((bp.ng > bp.gmax ? bp.ng : bp.gmax) + 1, 256)), dim3(256), 0,
                     ctx->stream, (const uint32_t*)goff1, T, NG, (const uint32_t*)gt, bp.ng,
                     (const uint32_t*)cbase, bp.gmax, cstart, cgov, cfirst);
  hipLaunchKernelGGL(k_chunk_desc, dim3(div_up(bp.gmax, 256)), dim3(256), 0, ctx->stream, (const uint32_t*)cstart,
                     (const uint32_t*)cgov, gcount, bp.gmax, (const uint32_t*)goff1, T, NG, (const uint32_t*)gt,
                     cdesc, dtile);
  {
    ScopedTimer tm(ctx, "p2_hist");
    hipLaunchKernelGGL(k_hist_bytes, dim3(G), dim3(kHBThreads), 0, ctx->stream, (const uint8_t*)b1,
                       (const uint4*)cdesc, gcount, hist2);
  }
  rc = scan32(ctx, hist2, goff2, 256 * bp.gmax, scr, gcount, 256);
  if (rc) return rc;
  P2Args a2{v1, cdesc, dtile, gcount, goff1, trec, T, NG, goff2, hist2, v2};
  {
    ScopedTimer tm(ctx, "p2_scatter");
    hipLaunchKernelGGL(k_p2_scatter, dim3(G), dim3(kPThreads), 0, ctx->stream, a2);
  }
  uint32_t* bnz = (uint32_t*)ws_at(ctx, bp.oBN);
  uint32_t* blpos = (uint32_t*)ws_at(ctx, bp.oBP);
  hipLaunchKernelGGL(k_bucket_desc, dim3(kNumBuckets / 256), dim3(256), 0, ctx->stream, (const uint32_t*)goff2,
                     gcount, (const uint32_t*)cfirst, bdesc, bnz);
  hipLaunchKernelGGL(k_bucket_groups, dim3(div_up((uint64_t)kNumBuckets * NG, 256)), dim3(256), 0, ctx->stream,
                     (const uint32_t*)goff2, gcount, (const uint32_t*)cbase, NG, gbnd);
  rc = scan32(ctx, bnz, blpos, kNumBuckets, scr);
  if (rc) return rc;
  hipLaunchKernelGGL(k_bucket_compact, dim3(kNumBuckets / 256), dim3(256), 0, ctx->stream, (const uint4*)bdesc,
                     (const uint32_t*)blpos, (uint32_t*)ws_at(ctx, bp.oLB), (uint4*)ws_at(ctx, bp.oLQ));
  SG_HIP(hipGetLastError());
  return SG_OK;
}

// Stage B: the bucket kernels over stage A's buckets (bp rebased by stage A):
// flags and set updates, or (emit) the candidate pairs.
static int buckets_one(sg_ctx* ctx, const BucketPlan& bp, uint32_t* mwords, uint32_t* nwords, uint8_t* d_rec_new,
                       const EmitArgs* emit, uint64_t n, uint64_t nrec, const uint32_t* owords = nullptr) {
  const uint32_t NG = (uint32_t)bp.NG;
  const uint32_t* cbase = (const uint32_t*)ws_at(ctx, bp.oCB);
  const uint32_t* gcount = cbase + bp.ng;  // device: number of pass-2 chunks
  uint4* bdesc = (uint4*)ws_at(ctx, bp.oBD);
  uint32_t* gbnd = (uint32_t*)ws_at(ctx, bp.oGB);
  uint32_t* v2 = (uint32_t*)ws_at(ctx, bp.oV2);
  uint32_t* nspill = (uint32_t*)ws_at(ctx, bp.oSP);
  uint32_t* blpos = (uint32_t*)ws_at(ctx, bp.oBP);
  const bool dbg = ctx->debug_part;
  BucketArgs ba{};
  ba.in = v2;
  ba.bdesc = bdesc;
  ba.gbnd = gbnd;
  ba.NG = NG;
  ba.mwords = mwords;
  ba.owords = owords;
  ba.nwords = nwords;
  ba.rec_new = d_rec_new;
  ba.nspill = nspill;
  ba.spill = nspill + 1;
  ba.ticket = (uint32_t*)ws_at(ctx, bp.oTK);
  if (emit) {
    ba.pairs = emit->pairs;
    ba.npairs = emit->npairs;
    ba.rec_base = emit->rec_base;
    ba.nshards = emit->nshards;
    ba.shard_cnt = emit->shard_cnt;
    ba.update = emit->update ? 1u : 0u;
    ba.gcur = emit->gcur;
    ba.goff = emit->goff;
  }
  uint32_t bgrid = persistent_grid(ctx, (const void*)k_bucket<false, 0>, kBThreads);
  // diagnostics: option bucket_blocks caps the persistent grid (leaves CUs
  // to kernels on other streams)
  const int64_t cap_blocks = ctx->opt[kOptBucketBlocks];
  if (cap_blocks > 0 && (uint64_t)cap_blocks < bgrid) bgrid = (uint32_t)cap_blocks;
  uint64_t* ddbg = nullptr;
  if (dbg) {
    SG_HIP(hipMalloc(&ddbg, (size_t)bgrid * 88));
    ba.dbg = ddbg;
  }
  SG_HIP(hipMemsetAsync(ba.ticket, 0, 4, ctx->stream));
  SG_HIP(hipMemsetAsync(nspill, 0, 4, ctx->stream));
  ba.blist_b = (const uint32_t*)ws_at(ctx, bp.oLB);
  ba.blist_q = (const uint4*)ws_at(ctx, bp.oLQ);
  ba.nlist = blpos + kNumBuckets;
  {
    ScopedTimer tm(ctx, "bucket_triage");
    if (emit && emit->gcur)
      hipLaunchKernelGGL((k_bucket<false, 2>), dim3(bgrid), dim3(kBThreads), 0, ctx->stream, ba);
    else if (emit)
      hipLaunchKernelGGL((k_bucket<false, 1>), dim3(bgrid), dim3(kBThreads), 0, ctx->stream, ba);
    else if (dbg)
      hipLaunchKernelGGL((k_bucket<true, 0>), dim3(bgrid), dim3(kBThreads), 0, ctx->stream, ba);
    else
      hipLaunchKernelGGL((k_bucket<false, 0>), dim3(bgrid), dim3(kBThreads), 0, ctx->stream, ba);
  }
  {
    ScopedTimer tm(ctx, "bucket_spill");
    if (emit)
      hipLaunchKernelGGL(k_bucket_direct<true>, dim3(512), dim3(kDThreads), 0, ctx->stream, ba);
    else
      hipLaunchKernelGGL(k_bucket_direct<false>, dim3(512), dim3(kDThreads), 0, ctx->stream, ba);
  }
  SG_HIP(hipGetLastError());
  if (dbg) {  // diagnostics: chunk and spill counts (syncs)
    uint32_t g = 0, sp = 0;
    SG_HIP(hipMemcpyAsync(&g, gcount, 4, hipMemcpyDeviceToHost, ctx->stream));
    SG_HIP(hipMemcpyAsync(&sp, nspill, 4, hipMemcpyDeviceToHost, ctx->stream));
    SG_HIP(hipStreamSynchronize(ctx->stream));
    fprintf(stderr, "sg part: n=%llu nrec=%llu tiles=%llu chunks=%u (bound %llu) spilled_buckets=%u\n",
            (unsigned long long)n, (unsigned long long)nrec, (unsigned long long)bp.T, g,
            (unsigned long long)bp.gmax, sp);
    std::vector<uint4> bd(kNumBuckets);
    std::vector<uint64_t> hd((size_t)bgrid * 11);
    SG_HIP(hipMemcpy(bd.data(), bdesc, bd.size() * 16, hipMemcpyDeviceToHost));
    SG_HIP(hipMemcpy(hd.data(), ddbg, hd.size() * 8, hipMemcpyDeviceToHost));
    double qa = 0, qb = 0, qc = 0;
    for (uint32_t i = 0; i < bgrid; i++) {
      qa += hd[8 * bgrid + 3 * i];
      qb += hd[8 * bgrid + 3 * i + 1];
      qc += hd[8 * bgrid + 3 * i + 2];
    }
    SG_HIP(hipFree(ddbg));
    std::vector<uint32_t> sz(kNumBuckets);
    uint64_t rounds = 0;
    for (uint32_t b = 0; b < kNumBuckets; b++) {
      sz[b] = bd[b].y - bd[b].x;
      rounds += (sz[b] + 8191) / 8192;
    }
    std::sort(sz.begin(), sz.end());
    uint64_t t0 = ~0ull, t1 = 0;
    std::vector<double> dur;
    uint64_t maxr = 0;
    double phs[4] = {0, 0, 0, 0}, nbk = 0, nrd = 0;
    for (uint32_t i = 0; i < bgrid; i++) {
      t0 = std::min(t0, hd[8 * i]);
      t1 = std::max(t1, hd[8 * i + 1]);
      dur.push_back((hd[8 * i + 1] - hd[8 * i]) / 100.0);  // 100 MHz clock -> us
      maxr = std::max(maxr, hd[8 * i + 3]);
      nbk += hd[8 * i + 2];
      nrd += hd[8 * i + 3];
      for (int j = 0; j < 4; j++) phs[j] += hd[8 * i + 4 + j];
    }
    fprintf(stderr, "sg bucket per bucket (cycles, wave 0): install %.0f | rounds: test %.0f insert %.0f tail %.0f | "
            "end barrier %.0f flush %.0f final barrier %.0f | rounds/bucket %.2f\n", phs[0] / nbk, qa / nbk, qb / nbk,
            phs[1] / nbk, phs[2] / nbk, phs[3] / nbk, qc / nbk, nrd / nbk);
    std::sort(dur.begin(), dur.end());
    fprintf(stderr,
            "sg bucket: sizes max=%u p99=%u median=%u rounds=%llu | blocks=%u span=%.1fus dur min=%.1f med=%.1f "
            "max=%.1f us, max rounds/block=%llu\n",
            sz.back(), sz[kNumBuckets * 99 / 100], sz[kNumBuckets / 2], (unsigned long long)rounds, bgrid,
            (t1 - t0) / 100.0, dur.front(), dur[dur.size() / 2], dur.back(), (unsigned long long)maxr);
  }
  return SG_OK;
}

// One launch sequence over a batch of <= kMaxGroups groups (rec_new zeroed).
// With `emit`, the bucket stage writes the distinct candidates instead of
// flagging records and updating the sets (mwords is then only read).  The
// launch's scratch starts at workspace offset ws_base (reserved by the caller
// when ws_base != 0).
// The M0 filter on stage 1's output (bp rebased): *done when its tail has
// produced the flags and set updates; otherwise the survivors overflowed and
// the caller goes on with stage 2 and the bucket stage (nothing written yet).
static int m0_filter(sg_ctx* ctx, const BucketPlan& bp, uint32_t* mwords, uint32_t* nwords, uint8_t* d_rec_new,
                     bool* done) {
  *done = false;
  if (!ctx->m0f) {
    SG_HIP(hipMalloc(&ctx->m0f, m0f_bytes()));
    const M0F f0 = m0f_bind(ctx);
    SG_HIP(hipMemsetAsync(f0.table, 0xFF, 8ull << kFTableBits, ctx->stream));
  }
  const M0F f = m0f_bind(ctx);
  const uint32_t T = (uint32_t)bp.T;
  SG_HIP(hipMemsetAsync(f.cursor, 0, kFIdx * 4 + 256 + kFIdx * 4, ctx->stream));  // cursors, survivor and spill counts
  // the index in 2^logh parts per slice (auto: 1, or 2 after a part
  // overflowed and the survivors with it; 4 only forced; the filter's
  // workgroups stay 2048: kFParts >> logh per slice and part, each part's pass
  // reading the whole slice run)
  const int logh = ctx->opt[kOptM0Halves] >= 0 ? (int)ctx->opt[kOptM0Halves] : ctx->m0f_logh;
  {
    ScopedTimer tm(ctx, "m0_index");
    const dim3 ig(kFBuckets / 256, 256u << logh);
    if (logh == 0)
      hipLaunchKernelGGL(k_m0_index<0>, ig, dim3(256), 0, ctx->stream, (const uint32_t*)mwords, f.tab, f.ovals,
                         f.cursor, f.nspill, f.spill, f.nsurv);
    else if (logh == 1)
      hipLaunchKernelGGL(k_m0_index<1>, ig, dim3(256), 0, ctx->stream, (const uint32_t*)mwords, f.tab, f.ovals,
                         f.cursor, f.nspill, f.spill, f.nsurv);
    else
      hipLaunchKernelGGL(k_m0_index<2>, ig, dim3(256), 0, ctx->stream, (const uint32_t*)mwords, f.tab, f.ovals,
                         f.cursor, f.nspill, f.spill, f.nsurv);
  }
  {
    ScopedTimer tm(ctx, "m0_filter");
    auto kf = logh == 0 ? k_m0_filter<0> : logh == 1 ? k_m0_filter<1> : k_m0_filter<2>;
    hipLaunchKernelGGL(kf, dim3(kFParts >> logh, 256, 1u << logh), dim3(kFThreads), 0, ctx->stream,
                       (const uint32_t*)ws_at(ctx, bp.oV1), (const uint32_t*)ws_at(ctx, bp.oO1), T,
                       (const uint4*)f.tab, (const uint16_t*)f.ovals, (const uint32_t*)f.cursor,
                       (const uint32_t*)f.nspill, (const uint32_t*)f.spill, f.surv, f.nsurv, f.wgcnt);
  }
  SG_HIP(hipGetLastError());
  // (the host ingest's pinned staging may be in a DMA now: a pageable read)
  uint32_t nsv[3] = {0, 0, 0};
  SG_HIP(hipMemcpyAsync(nsv, f.nsurv, 12, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  const uint32_t ns = nsv[0];
  ctx->m0f_survivors = nsv[1] ? kFSurvCap + 1 : ns;
  if (nsv[1] || ns > kFSurvCap) {
    ctx->m0f_fallback++;
    ctx->m0f_last = 0;
    // auto: a fallback on a slice that was expected to filter (a maxSignal
    // past the index's capacity, or a novelty burst) -- the next 1, 2, 4 ..
    // 64 slices are not tried
    if (ctx->opt[kOptM0Halves] < 0 && nsv[2] && ctx->m0f_logh < 1) {
      // an index part overflowed: two parts, tried again at once (each part's
      // pass streams the whole run: at 18M signals two parts filter in 1.6 ms
      // against 2.8 ms of pass 2 and buckets; four, at 41M, took 3.9 ms --
      // past two parts auto backs off to the partition instead)
      ctx->m0f_logh++;
    } else if (ctx->opt[kOptM0Filter] < 0) {
      ctx->m0f_backoff = ctx->m0f_backoff ? std::min<uint32_t>(2 * ctx->m0f_backoff, 64) : 1;
      ctx->m0f_skip = ctx->m0f_backoff;
    }
    return SG_OK;
  }
  if (ns) {
    ScopedTimer tm(ctx, "m0_tail");
    hipLaunchKernelGGL(k_m0_tail_insert, dim3(4, 256 * kFParts), dim3(256), 0, ctx->stream,
                       (const uint2*)f.surv, (const uint32_t*)f.wgcnt,
                       (const uint32_t*)ws_at(ctx, bp.oV1), (const uint32_t*)ws_at(ctx, bp.oO1), T,
                       (const uint32_t*)ws_at(ctx, bp.oTR), (const uint32_t*)mwords, f.table);
    hipLaunchKernelGGL(k_m0_tail_flush, dim3((1u << kFTableBits) / 256), dim3(256), 0, ctx->stream, f.table, mwords,
                       nwords, d_rec_new);
  }
  SG_HIP(hipGetLastError());
  ctx->m0f_used++;
  ctx->m0f_last = 1;
  ctx->m0f_backoff = ctx->m0f_skip = 0;
  *done = true;
  return SG_OK;
}

// the pass-2 digit plane of pass-1 entries (top byte of each), after a pass 1
// that did not write it: 4 entries per thread and step
__global__ void k_top_plane(const uint32_t* __restrict__ v1, uint64_t n, uint8_t* __restrict__ b1) {
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n;
       i += (uint64_t)gridDim.x * blockDim.x * 4) {
    if (i + 4 <= n && ((uintptr_t)(v1 + i) & 15) == 0) {
      const uint4 q = *reinterpret_cast<const uint4*>(v1 + i);
      *reinterpret_cast<uint32_t*>(b1 + i) = (q.x >> 24) | ((q.y >> 24) << 8) | ((q.z >> 24) << 16) | (q.w & 0xFF000000u);
    } else {
      for (uint64_t k = i; k < i + 4 && k < n; k++) b1[k] = (uint8_t)(v1[k] >> 24);
    }
  }
}

// queued records of a partitioned slice: one add per block
__global__ void k_count_flags(const uint8_t* __restrict__ f, uint64_t n, uint32_t* __restrict__ out) {
  uint32_t c = 0;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += (uint64_t)gridDim.x * blockDim.x * 4)
    for (int k = 0; k < 4; k++) c += i + k < n && f[i + k] ? 1u : 0u;
  c = sgd::wave_incl_add(c);
  if ((threadIdx.x & 63) == 63 && c) atomicAdd(out, c);
}

// After a partitioned slice (auto regime): its queued records counted on the
// device and copied to pinned memory behind an event, read by a later m0f_try.
static int m0f_note_partitioned(sg_ctx* ctx, const uint8_t* d_rec_new, uint64_t nrec) {
  ctx->m0f_last = 0;
  if (ctx->opt[kOptM0Filter] >= 0 || ctx->m0f_pending) return SG_OK;
  if (!ctx->m0f_host) {
    SG_HIP(hipHostMalloc((void**)&ctx->m0f_host, 64, hipHostMallocDefault));
    SG_HIP(hipEventCreateWithFlags(&ctx->m0f_ev, hipEventDisableTiming));
  }
  uint32_t* dcnt = (uint32_t*)ctx->dscal + 32;  // (a device scalar of the context)
  SG_HIP(hipMemsetAsync(dcnt, 0, 4, ctx->stream));
  hipLaunchKernelGGL(k_count_flags, dim3(std::min<uint64_t>(256, div_up(nrec, 1024))), dim3(256), 0, ctx->stream,
                     d_rec_new, nrec, dcnt);
  SG_HIP(hipMemcpyAsync(ctx->m0f_host, dcnt, 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipEventRecord(ctx->m0f_ev, ctx->stream));
  ctx->m0f_pending = true;
  ctx->m0f_nrec = nrec;
  return SG_OK;
}

// The M0 filter's regime: option m0_filter 1 always tries it, 0 never.  auto
// (the fuzzer's loop, batch after batch) tries it after a slice it filtered,
// and after a partitioned slice whose queued fraction was below kFTryQueued
// (in the steady state 9 % of the records are queued, in a fresh batch all:
// fresh batches then never pay for it); on the context's first slice it is
// tried.  A queued count still in flight keeps the previous choice.  After a
// fallback it backs off (m0f_skip): a low-novelty batch whose maxSignal is
// past the index's capacity would otherwise fall back on every slice.
constexpr double kFTryQueued = 0.25;
static bool m0f_try(sg_ctx* ctx) {
  const int64_t o = ctx->opt[kOptM0Filter];
  if (o >= 0) return o != 0;
  if (ctx->m0f_pending && hipEventQuery(ctx->m0f_ev) == hipSuccess) {
    ctx->m0f_pending = false;
    ctx->m0f_queued = (double)*ctx->m0f_host / (double)(ctx->m0f_nrec ? ctx->m0f_nrec : 1);
  }
  if (ctx->m0f_skip) {  // (backing off after fallbacks)
    ctx->m0f_skip--;
    return false;
  }
  if (ctx->m0f_last < 0) return true;
  if (ctx->m0f_last == 1) return true;
  return ctx->m0f_queued >= 0 && ctx->m0f_queued < kFTryQueued;
}

static int bucket_triage_one(sg_ctx* ctx, uint32_t* mwords, uint32_t* nwords, const uint32_t* d_vals,
                             const uint64_t* d_off, uint64_t n, uint64_t nrec, uint8_t* d_rec_new,
                             const EmitArgs* emit = nullptr, size_t ws_base = 0, bool trace = false) {
  if (n == 0) return SG_OK;
  if (nrec == 0) {
    set_error("bucket triage: signal entries without records");
    return SG_EINVAL;
  }
  BucketPlan bp(n, nrec);
  if (emit || ws_base) {
    int rc = partition_one(ctx, d_vals, d_off, n, nrec, ws_base, ws_base != 0, bp, trace);
    if (rc) return rc;
    return buckets_one(ctx, bp, mwords, nwords, d_rec_new, emit, n, nrec);
  }
  if (!m0f_try(ctx)) {
    int rc = partition_one(ctx, d_vals, d_off, n, nrec, 0, false, bp, trace);
    if (!rc) rc = buckets_one(ctx, bp, mwords, nwords, d_rec_new, nullptr, n, nrec);
    if (!rc) rc = m0f_note_partitioned(ctx, d_rec_new, nrec);
    return rc;
  }
  // the flags path with the M0 filter between the two partition passes
  // (pass 1 without the pass-2 digit plane: -0.88 GB of writes per C2 step;
  // when the survivors overflow, the plane is made from the pass-1 entries)
  int rc = partition_one(ctx, d_vals, d_off, n, nrec, 0, false, bp, trace, 1, false);
  if (rc) return rc;
  bool done = false;
  rc = m0_filter(ctx, bp, mwords, nwords, d_rec_new, &done);
  if (rc || done) return rc;
  hipLaunchKernelGGL(k_top_plane, dim3((uint32_t)std::min<uint64_t>(4096, div_up(n, 1024))), dim3(256), 0,
                     ctx->stream, (const uint32_t*)ws_at(ctx, bp.oV1), n, (uint8_t*)ws_at(ctx, bp.oB1));
  SG_HIP(hipGetLastError());
  rc = partition_one(ctx, d_vals, d_off, n, nrec, 0, false, bp, trace, 2);
  if (!rc) rc = buckets_one(ctx, bp, mwords, nwords, d_rec_new, nullptr, n, nrec);
  if (!rc) rc = m0f_note_partitioned(ctx, d_rec_new, nrec);
  return rc;
}

// Marks: nwords |= every signal of stage A's buckets that is not in mwords
// (a workgroup per bucket: its maxSignal slice in LDS, its newSignal words
// written by it alone).  Entries are read as 16-B quads from the bucket start
// rounded down (the pass-2 buffer is padded), kMarkU quads per thread in
// flight; the first ones are issued before the slice is installed.  kFirst:
// nwords = those signals (every word written, empty buckets' too: no clear
// beforehand and no read of the old words).
constexpr int kMarkT = 256, kMarkU = 2;
// bcnt (nullable): per bucket, the signals this launch newly marks (summed by
// k_sum_counts into the batch's count of distinct signals not in mwords; one
// atomic per wave on a single counter serialised: 2 x 3.3 ms per C3 slice)
template <bool kFirst>
__global__ __launch_bounds__(kMarkT) void k_bucket_mark(const uint32_t* __restrict__ in, const uint4* __restrict__ bdesc,
                                                        const uint32_t* __restrict__ mwords,
                                                        uint32_t* __restrict__ nwords,
                                                        uint32_t* __restrict__ bcnt) {
  __shared__ uint32_t mslice[kBucketWords];
  __shared__ uint32_t nbits[kBucketWords];
  __shared__ uint32_t wcnt[kMarkT / 64];
  constexpr int kW = kBucketWords / kMarkT;  // slice words per thread
  typedef uint32_t mvec __attribute__((ext_vector_type(kW)));
  const uint32_t b = blockIdx.x, tid = threadIdx.x;
  const uint4 q = bdesc[b];
  if (q.x >= q.y) {
    if (kFirst) *reinterpret_cast<mvec*>(nwords + bucket_word(b, kW * tid)) = mvec{};
    if (bcnt && tid == 0) bcnt[b] = 0;
    return;
  }
  constexpr uint32_t kStep = kMarkT * 4 * kMarkU;
  auto load = [&](uint32_t base, v4u32 (&v)[kMarkU]) {
#pragma unroll
    for (int u = 0; u < kMarkU; u++) {
      const uint32_t p = base + (u * kMarkT + tid) * 4;
      v[u] = v4u32{0, 0, 0, 0};
      if (p < q.y) v[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(in + p));
    }
  };
  uint32_t base = q.x & ~3u;
  v4u32 v[kMarkU];
  load(base, v);
  {
    const uint64_t w0 = bucket_word(b, kW * tid);
    reinterpret_cast<mvec*>(mslice)[tid] = *reinterpret_cast<const mvec*>(mwords + w0);
    reinterpret_cast<mvec*>(nbits)[tid] = mvec{};
  }
  __syncthreads();
  for (;;) {
    const uint32_t next = base + kStep;
    v4u32 y[kMarkU];
    if (next < q.y) load(next, y);
#pragma unroll
    for (int u = 0; u < kMarkU; u++) {
      const uint32_t p = base + (u * kMarkT + tid) * 4;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t sl = v[u][j] >> 16;
        const bool live = p + j >= q.x && p + j < q.y;
        if (live && !((mslice[sl >> 5] >> (sl & 31)) & 1u)) atomicOr(&nbits[sl >> 5], 1u << (sl & 31));
      }
    }
    if (next >= q.y) break;
    base = next;
    for (int u = 0; u < kMarkU; u++) v[u] = y[u];
  }
  __syncthreads();
  uint32_t fresh = 0;  // this thread's newly marked signals
  if (kFirst) {
    const mvec nb = reinterpret_cast<const mvec*>(nbits)[tid];
    *reinterpret_cast<mvec*>(nwords + bucket_word(b, kW * tid)) = nb;
#pragma unroll
    for (int j = 0; j < kW; j++) fresh += __popc(nb[j]);
  } else {
    for (uint32_t i = tid; i < kBucketWords; i += kMarkT)
      if (nbits[i]) {
        uint32_t* w = nwords + bucket_word(b, i);
        const uint32_t old = *w;
        fresh += __popc(nbits[i] & ~old);
        *w = old | nbits[i];
      }
  }
  if (bcnt) {
    const uint32_t wsum = __builtin_amdgcn_readlane(sgd::wave_incl_add(fresh), 63);
    if ((tid & 63) == 0) wcnt[tid >> 6] = wsum;
    __syncthreads();
    if (tid == 0) {
      uint32_t t = 0;
#pragma unroll
      for (int i = 0; i < kMarkT / 64; i++) t += wcnt[i];
      bcnt[b] = t;
    }
  }
}

// *acc += the n counts (one workgroup)
__global__ __launch_bounds__(1024) void k_sum_counts(const uint32_t* __restrict__ c, uint32_t n,
                                                     unsigned long long* __restrict__ acc) {
  __shared__ unsigned long long ws[16];
  unsigned long long t = 0;
  for (uint32_t i = threadIdx.x; i < n; i += 1024) t += c[i];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = 0;
    for (int i = 0; i < 16; i++) s += ws[i];
    *acc += s;
  }
}

__global__ void k_rebase(const uint64_t* __restrict__ off, uint64_t n, uint64_t base, uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = off[i] - base;
}

int rebase_offsets(sg_ctx* ctx, const uint64_t* d_off, uint64_t n, uint64_t base, uint64_t* d_out) {
  hipLaunchKernelGGL(k_rebase, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, d_off, n, base, d_out);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

// Flags-only triage of a device-resident batch (ctx lock held).  Batches of
// more than ctx->max_launch_recs records run as consecutive record slices:
// the sequential loop (fuzzer.go:665) cut between two records sees the same
// maxSignal at every record.  The rebased offsets of a slice live in a
// grow-only context buffer.
static int read_off(sg_ctx* ctx, const uint64_t* d_off, uint64_t r, uint64_t* v) {
  SG_HIP(hipMemcpyAsync(v, d_off + r, 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

// Entries per launch above which a batch is cut into record slices: about one
// C2 batch.  Twice that makes the (b2, b1) buckets twice as large, and a
// tenth of them overflow the LDS candidate map into the slow spill kernel.
constexpr uint64_t kSliceEntries = 1ull << 30;

// The record slices of a batch: <= max_launch_recs records and <=
// kSliceEntries entries each (unless one record alone holds more).
struct RecSlice {
  uint64_t r0, r1, e0, e1;
};

// The cuts by one device thread (a binary search per entry-limited slice):
// out[0] = the number of slices, then {r0, r1, e0, e1} per slice, at most
// kCutCap of them (a count past kCutCap: the host walks them itself).  One
// launch, one small read and one wait per batch, where the host's own search
// waited on the stream ~20 times (each wait an idle GPU between two batches).
constexpr uint32_t kCutCap = 4096;
constexpr uint32_t kCutHead = 64;  // slices read back with the count
__global__ void k_slice_cuts(const uint64_t* __restrict__ off, uint64_t nrec, uint64_t m, uint64_t lim,
                             uint64_t* __restrict__ out) {
  if (threadIdx.x || blockIdx.x) return;
  uint64_t r0 = 0, e0 = off[0], k = 0;
  while (r0 < nrec && k <= kCutCap) {
    uint64_t r1 = nrec - r0 < m ? nrec : r0 + m, e1 = off[r1];
    if (e1 - e0 > lim) {  // largest r1 > r0 with off[r1] - e0 <= lim (at least one record)
      uint64_t lo = r0 + 1, hi = r1;
      while (lo < hi) {
        const uint64_t mid = (lo + hi + 1) / 2;
        if (off[mid] - e0 <= lim)
          lo = mid;
        else
          hi = mid - 1;
      }
      r1 = lo;
      e1 = off[r1];
    }
    if (k < kCutCap) {
      out[1 + 4 * k] = r0;
      out[2 + 4 * k] = r1;
      out[3 + 4 * k] = e0;
      out[4 + 4 * k] = e1;
    }
    k++;
    r0 = r1;
    e0 = e1;
  }
  out[0] = k;
}

static int record_slices_host(sg_ctx* ctx, const uint64_t* d_off, uint64_t nrec, std::vector<RecSlice>& out,
                              uint64_t lim) {
  out.clear();
  const uint64_t m = ctx->max_launch_recs;
  uint64_t e0 = 0;
  int rc = read_off(ctx, d_off, 0, &e0);
  if (rc) return rc;
  for (uint64_t r0 = 0; r0 < nrec;) {
    uint64_t r1 = nrec - r0 < m ? nrec : r0 + m, e1 = 0;
    rc = read_off(ctx, d_off, r1, &e1);
    if (rc) return rc;
    if (e1 - e0 > lim) {
      uint64_t lo = r0 + 1, hi = r1;
      while (lo < hi) {
        const uint64_t mid = (lo + hi + 1) / 2;
        uint64_t em = 0;
        rc = read_off(ctx, d_off, mid, &em);
        if (rc) return rc;
        if (em - e0 <= lim)
          lo = mid;
        else
          hi = mid - 1;
      }
      r1 = lo;
      rc = read_off(ctx, d_off, r1, &e1);
      if (rc) return rc;
    }
    out.push_back({r0, r1, e0, e1});
    r0 = r1;
    e0 = e1;
  }
  return SG_OK;
}

static int record_slices(sg_ctx* ctx, const uint64_t* d_off, uint64_t nrec, std::vector<RecSlice>& out,
                         uint64_t lim = kSliceEntries) {
  out.clear();
  if (nrec == 0) return SG_OK;
  if (!ctx->slice_cuts) SG_HIP(hipMalloc(&ctx->slice_cuts, (1 + 4 * (size_t)kCutCap) * 8));
  hipLaunchKernelGGL(k_slice_cuts, dim3(1), dim3(64), 0, ctx->stream, d_off, nrec, (uint64_t)ctx->max_launch_recs,
                     lim, ctx->slice_cuts);
  SG_HIP(hipGetLastError());
  std::vector<uint64_t> h(1 + 4 * (size_t)kCutHead);
  SG_HIP(hipMemcpyAsync(h.data(), ctx->slice_cuts, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  const uint64_t k = h[0];
  if (k > kCutCap) return record_slices_host(ctx, d_off, nrec, out, lim);
  if (k > kCutHead) {
    h.resize(1 + 4 * k);
    SG_HIP(hipMemcpy(h.data(), ctx->slice_cuts, h.size() * 8, hipMemcpyDeviceToHost));
  }
  for (uint64_t j = 0; j < k; j++) out.push_back({h[1 + 4 * j], h[2 + 4 * j], h[3 + 4 * j], h[4 + 4 * j]});
  return SG_OK;
}

int record_slice_cuts(sg_ctx* ctx, const uint64_t* d_off, uint64_t nrec, uint64_t lim, std::vector<uint64_t>& cuts) {
  std::vector<RecSlice> sl;
  const int rc = record_slices(ctx, d_off, nrec, sl, lim);
  cuts.clear();
  for (const RecSlice& x : sl) cuts.insert(cuts.end(), {x.r0, x.r1, x.e0, x.e1});
  return rc;
}

int bucket_triage(sg_ctx* ctx, uint32_t* mwords, uint32_t* nwords, const uint32_t* d_vals, const uint64_t* d_off,
                  uint64_t n, uint64_t nrec, uint8_t* d_rec_new, bool trace) {
  if (nrec >= 0xFFFFFFFFull || n >= 0xFFFFFFFFull - 2 * kPT) {
    set_error("bucket triage: a batch holds < 2^32 signal entries and < 2^32 - 1 records");
    return SG_EINVAL;
  }
  if (nrec) SG_HIP(hipMemsetAsync(d_rec_new, 0, nrec, ctx->stream));
  const uint64_t m = ctx->max_launch_recs;
  if (nrec <= m && n <= kSliceEntries)
    return bucket_triage_one(ctx, mwords, nwords, d_vals, d_off, n, nrec, d_rec_new, nullptr, 0, trace);
  std::vector<RecSlice> sl;
  int rc = record_slices(ctx, d_off, nrec, sl);
  if (rc) return rc;
  // every slice's rebased offsets at once (no wait between two slices)
  const size_t need = nrec + sl.size();
  if (ctx->slice_off_cap < need) {
    SG_HIP(hipStreamSynchronize(ctx->stream));
    if (ctx->slice_off) SG_HIP(hipFree(ctx->slice_off));
    ctx->slice_off = nullptr;
    ctx->slice_off_cap = 0;
    SG_HIP(hipMalloc(&ctx->slice_off, need * 8));
    ctx->slice_off_cap = need;
  }
  size_t at = 0;
  for (const RecSlice& x : sl) {
    // the sequential loop (fuzzer.go:665) cut between two records sees the
    // same maxSignal at every record; a slice starts at a record boundary (a
    // trace slice's first entry is a call start)
    const uint64_t nr = x.r1 - x.r0;
    uint64_t* roff = ctx->slice_off + at;
    at += nr + 1;
    if (x.e1 == x.e0) continue;  // records without entries (flags cleared above)
    rc = rebase_offsets(ctx, d_off + x.r0, nr + 1, x.e0, roff);
    if (rc) return rc;
    rc = bucket_triage_one(ctx, mwords, nwords, d_vals + x.e0, roff, x.e1 - x.e0, nr, d_rec_new + x.r0, nullptr, 0,
                           trace);
    if (rc) return rc;
  }
  return SG_OK;
}

// Two-phase triage (the prefix protocol, syzkaller_amd/shard.py).  Begin runs
// the bucket stage of each record slice against base in emitting form: the
// batch's signal not in base is set in marks, and each such s is kept once,
// with its first record, as a pair in the slot's workspace.  Slice j is
// tested against base | marks, so a signal of an earlier slice is not
// re-emitted by a later one: the pairs are the first owners over the whole
// batch.  End: record r is queued iff it owns a pair whose s is in neither
// maxSignal nor the prefix (k_prefix_flags).  That is the sequential loop
// against M = maxsig | prefix for any M containing base: every s of the batch
// outside M is outside base, so its pair is kept, and its first owner is the
// loop's (a record is queued iff it is the first to hold some s outside M).
// That is the form option prefix_pairs 1 selects.  The default keeps the
// partitions instead: begin marks the buckets (k_bucket_mark, the base slice
// in LDS), end runs the bucket stage against maxsig | prefix.  On a fresh C3
// slice (1.76G entries, 361M pairs) the pairs' flag pass (3.9 ms: two random
// cache lines per pair) costs more than the mark pass (2 x 1.0 ms); the pair
// form's end shrinks with the batch's novelty, the kept partitions' does not.
static size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// The slot's workspace stands in for the context's during one call (the
// partition code addresses the workspace through ctx->ws); grown to the exact
// size, since it is kept.
struct SlotWs {
  sg_ctx* c;
  PrefixSlot& s;
  void* ws;
  size_t cap;
  SlotWs(sg_ctx* c_, PrefixSlot& s_) : c(c_), s(s_), ws(c_->ws), cap(c_->ws_cap) {
    c->ws = s.ws;
    c->ws_cap = s.ws_cap;
  }
  ~SlotWs() {
    s.ws = c->ws;
    s.ws_cap = c->ws_cap;
    c->ws = ws;
    c->ws_cap = cap;
  }
};

static int slot_reserve(sg_ctx* ctx, PrefixSlot& s, size_t bytes) {
  if (bytes <= s.ws_cap) return SG_OK;
  const size_t cap = (bytes + (64u << 20) - 1) & ~size_t((64u << 20) - 1);
  if (s.ws) {
    SG_HIP(hipStreamSynchronize(ctx->stream));
    SG_HIP(hipFree(s.ws));
    s.ws = nullptr;
    s.ws_cap = 0;
  }
  SG_HIP(hipMalloc(&s.ws, cap));
  s.ws_cap = cap;
  return SG_OK;
}

// flags of the kept pairs {s, record}: kFixU pairs per thread in flight (one
// pair per thread and step: 7.2 ms per C3 slice, eight: 3.9 ms).  Bound by
// the random cache-line accesses, two per pair (the bitmap word, the flag
// byte): 361M pairs of a fresh C3 slice at ~0.2 G lines/s/CU
constexpr int kFixT = 256, kFixU = 8;
__global__ __launch_bounds__(kFixT) void k_prefix_flags(const uint2* __restrict__ pairs,
                                                        const unsigned long long* __restrict__ npairs,
                                                        const uint32_t* __restrict__ mwords,
                                                        const uint32_t* __restrict__ owords, uint8_t* __restrict__ rec_new) {
  constexpr uint32_t kNone = 0xFFFFFFFFu;  // (records < 2^32 - 1)
  const uint64_t n = *npairs, stride = (uint64_t)gridDim.x * kFixT * kFixU;
  for (uint64_t base = (uint64_t)blockIdx.x * kFixT * kFixU + threadIdx.x; base < n; base += stride) {
    uint2 p[kFixU];
#pragma unroll
    for (int u = 0; u < kFixU; u++) {
      const uint64_t i = base + (uint64_t)u * kFixT;
      if (i < n) {
        const unsigned long long v = __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(pairs) + i);
        p[u] = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
      } else {
        p[u] = make_uint2(0u, kNone);
      }
    }
    uint32_t t[kFixU], w[kFixU];
#pragma unroll
    for (int u = 0; u < kFixU; u++) {
      t[u] = sgd::set_pos(p[u].x);
      w[u] = p[u].y != kNone ? mwords[t[u] >> 5] : ~0u;
    }
    if (owords) {
#pragma unroll
      for (int u = 0; u < kFixU; u++)
        if (p[u].y != kNone) w[u] |= owords[t[u] >> 5];
    }
#pragma unroll
    for (int u = 0; u < kFixU; u++)
      if (!((w[u] >> (t[u] & 31)) & 1u)) rec_new[p[u].y] = 1;
  }
}

// end's set updates: newsig |= marks & ~(maxsig | prefix), maxsig |= marks
__global__ void k_prefix_merge(const uint32_t* __restrict__ marks, uint32_t* __restrict__ mwords,
                               const uint32_t* __restrict__ owords, uint32_t* __restrict__ nwords) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < kSetWords / 4; w += stride) {
    const uint4 c = reinterpret_cast<const uint4*>(marks)[w];
    if (!(c.x | c.y | c.z | c.w)) continue;
    uint4 m = reinterpret_cast<uint4*>(mwords)[w];
    if (nwords) {
      uint4 o = owords ? reinterpret_cast<const uint4*>(owords)[w] : make_uint4(0, 0, 0, 0);
      uint4 nw = reinterpret_cast<uint4*>(nwords)[w];
      nw.x |= c.x & ~(m.x | o.x);
      nw.y |= c.y & ~(m.y | o.y);
      nw.z |= c.z & ~(m.z | o.z);
      nw.w |= c.w & ~(m.w | o.w);
      reinterpret_cast<uint4*>(nwords)[w] = nw;
    }
    m.x |= c.x;
    m.y |= c.y;
    m.z |= c.z;
    m.w |= c.w;
    reinterpret_cast<uint4*>(mwords)[w] = m;
  }
}

int prefix_begin(sg_ctx* ctx, uint32_t slot, const uint32_t* base_words, uint32_t* marks_words, const uint32_t* d_vals,
                 const uint64_t* d_off, uint64_t n, uint64_t nrec, int form, uint64_t* d_ncand) {
  if (slot >= kPrefixSlots) {
    set_error("prefix triage: slot %u out of range", slot);
    return SG_EINVAL;
  }
  if (nrec >= 0xFFFFFFFFull || n >= 0xFFFFFFFFull - 2 * kPT) {
    set_error("prefix triage: a batch holds < 2^32 signal entries and < 2^32 - 1 records");
    return SG_EINVAL;
  }
  PrefixSlot& S = ctx->prefix[slot];
  S.slices.clear();
  S.open = false;
  S.keep = form < 0 ? ctx->opt[kOptPrefixPairs] == 0 : form != 1;
  const bool mark = form != 2;  // form 2: the partitions alone (a plain triage split in two)
  if (d_ncand) SG_HIP(hipMemsetAsync(d_ncand, 0, 8, ctx->stream));
  S.marks = marks_words;
  S.n = n;
  std::vector<RecSlice> sl;
  int rc = nrec ? record_slices(ctx, d_off, nrec, sl) : SG_OK;
  if (rc) return rc;
  if (!S.keep) {
    // the pairs: a counter, then <= n pairs
    rc = slot_reserve(ctx, S, 256 + n * 8);
    if (rc) return rc;
    unsigned long long* np = (unsigned long long*)S.ws;
    uint2* pairs = (uint2*)((char*)S.ws + 256);
    SG_HIP(hipMemsetAsync(np, 0, 8, ctx->stream));
    SG_HIP(hipMemsetAsync(marks_words, 0, kSetBytes, ctx->stream));  // (the later slices' filter)
    size_t need = 0;
    for (const RecSlice& x : sl)
      if (x.e1 > x.e0)
        need = std::max(need, align256(bucket_plan_bytes(x.e1 - x.e0, x.r1 - x.r0)) + align256((x.r1 - x.r0 + 1) * 8));
    if (need) {
      rc = ws_reserve(ctx, need);
      if (rc) return rc;
    }
    for (const RecSlice& x : sl) {
      if (x.e1 == x.e0) continue;
      const uint64_t ns = x.e1 - x.e0, nr = x.r1 - x.r0;
      BucketPlan bp(ns, nr);
      uint64_t* roff = (uint64_t*)ws_at(ctx, align256(bucket_plan_bytes(ns, nr)));
      hipLaunchKernelGGL(k_rebase, dim3(div_up(nr + 1, 256)), dim3(256), 0, ctx->stream, d_off + x.r0, nr + 1, x.e0,
                         roff);
      rc = partition_one(ctx, d_vals + x.e0, roff, ns, nr, 0, true, bp);
      if (rc) return rc;
      const EmitArgs e{pairs, np, (uint32_t)x.r0, 1, nullptr};
      rc = buckets_one(ctx, bp, const_cast<uint32_t*>(base_words), marks_words, nullptr, &e, ns, nr, marks_words);
      if (rc) return rc;
    }
    // (each distinct signal not in base is one pair)
    if (d_ncand) SG_HIP(hipMemcpyAsync(d_ncand, np, 8, hipMemcpyDeviceToDevice, ctx->stream));
    S.nrec = nrec;
    S.open = true;
    return SG_OK;
  }
  size_t total = 0;
  for (const RecSlice& x : sl)
    if (x.e1 > x.e0) total += align256(bucket_plan_bytes(x.e1 - x.e0, x.r1 - x.r0)) + align256((x.r1 - x.r0 + 1) * 8);
  rc = slot_reserve(ctx, S, total ? total : 256);
  if (rc) return rc;
  SlotWs guard(ctx, S);
  size_t base = 0;
  bool first = true;
  for (const RecSlice& x : sl) {
    PrefixSlice ps{x.r0, x.r1, x.e0, x.e1, base};
    if (x.e1 > x.e0) {
      const uint64_t ns = x.e1 - x.e0, nr = x.r1 - x.r0;
      BucketPlan bp(ns, nr);
      const size_t roff_at = base + align256(bucket_plan_bytes(ns, nr));
      uint64_t* roff = (uint64_t*)ws_at(ctx, roff_at);
      hipLaunchKernelGGL(k_rebase, dim3(div_up(nr + 1, 256)), dim3(256), 0, ctx->stream, d_off + x.r0, nr + 1, x.e0,
                         roff);
      rc = partition_one(ctx, d_vals + x.e0, roff, ns, nr, base, true, bp);
      if (rc) return rc;
      if (mark) {
        ScopedTimer tm(ctx, "bucket_mark");
        const uint32_t* v2 = (const uint32_t*)ws_at(ctx, bp.oV2);
        const uint4* bd = (const uint4*)ws_at(ctx, bp.oBD);
        // (per-bucket counts in the partition's non-empty flags, which the
        // bucket stage does not read)
        uint32_t* bc = d_ncand ? (uint32_t*)ws_at(ctx, bp.oBN) : nullptr;
        if (first)  // the batch's first slice writes every marks word
          hipLaunchKernelGGL(k_bucket_mark<true>, dim3(kNumBuckets), dim3(kMarkT), 0, ctx->stream, v2, bd, base_words,
                             marks_words, bc);
        else
          hipLaunchKernelGGL(k_bucket_mark<false>, dim3(kNumBuckets), dim3(kMarkT), 0, ctx->stream, v2, bd,
                             base_words, marks_words, bc);
        if (bc)
          hipLaunchKernelGGL(k_sum_counts, dim3(1), dim3(1024), 0, ctx->stream, (const uint32_t*)bc, kNumBuckets,
                             (unsigned long long*)d_ncand);
        first = false;
      }
      SG_HIP(hipGetLastError());
      base = roff_at + align256((nr + 1) * 8);
    }
    S.slices.push_back(ps);
  }
  if (first && mark) SG_HIP(hipMemsetAsync(marks_words, 0, kSetBytes, ctx->stream));  // no entries
  S.nrec = nrec;
  S.open = true;
  return SG_OK;
}

int prefix_end(sg_ctx* ctx, uint32_t slot, uint32_t* mwords, const uint32_t* owords, uint32_t* nwords,
               uint8_t* d_rec_new, bool update) {
  if (slot >= kPrefixSlots || !ctx->prefix[slot].open) {
    set_error("prefix triage: no batch begun in slot %u", slot);
    return SG_EINVAL;
  }
  PrefixSlot& S = ctx->prefix[slot];
  S.open = false;
  if (S.nrec) SG_HIP(hipMemsetAsync(d_rec_new, 0, S.nrec, ctx->stream));
  if (!S.keep) {
    if (S.n) {
      ScopedTimer tm(ctx, "prefix_flags");
      hipLaunchKernelGGL(k_prefix_flags, dim3((uint32_t)std::min<uint64_t>(div_up(S.n, kFixT * kFixU), 2048)),
                         dim3(kFixT), 0,
                         ctx->stream, (const uint2*)((char*)S.ws + 256), (const unsigned long long*)S.ws, mwords,
                         owords, d_rec_new);
    }
    if (ctx->debug_part && S.n) {  // diagnostics (syncs): the kept pairs
      unsigned long long np = 0;
      SG_HIP(hipMemcpyAsync(&np, S.ws, 8, hipMemcpyDeviceToHost, ctx->stream));
      SG_HIP(hipStreamSynchronize(ctx->stream));
      fprintf(stderr, "sg prefix: %llu entries, %llu pairs\n", (unsigned long long)S.n, np);
    }
    if (update && S.n) {
      ScopedTimer tm(ctx, "prefix_merge");
      hipLaunchKernelGGL(k_prefix_merge, dim3(8192), dim3(256), 0, ctx->stream, S.marks, mwords, owords, nwords);
    }
    SG_HIP(hipGetLastError());
    return SG_OK;
  }
  SlotWs guard(ctx, S);
  for (const PrefixSlice& x : S.slices) {
    if (x.e1 == x.e0) continue;
    const uint64_t ns = x.e1 - x.e0, nr = x.r1 - x.r0;
    BucketPlan bp(ns, nr);
    bp.rebase(x.ws_base);
    const int rc = buckets_one(ctx, bp, mwords, nwords, d_rec_new + x.r0, nullptr, ns, nr, owords);
    if (rc) return rc;
  }
  return SG_OK;
}

int bucket_emit(sg_ctx* ctx, const uint32_t* mwords, const uint32_t* d_vals, const uint64_t* d_off, uint64_t n,
                uint64_t nrec, const EmitArgs& emit, size_t ws_base) {
  if (nrec > kMaxLaunchRecords || n >= 0xFFFFFFFFull - 2 * kPT) {
    set_error("bucket emit: a launch holds <= 2^24 records and < 2^32 - 2^15 entries");
    return SG_EINVAL;
  }
  return bucket_triage_one(ctx, const_cast<uint32_t*>(mwords), nullptr, d_vals, d_off, n, nrec, nullptr, &emit,
                           ws_base);
}

int bucket_emit_update(sg_ctx* ctx, uint32_t* mwords, uint32_t* nwords, const uint32_t* d_vals, const uint64_t* d_off,
                       uint64_t n, uint64_t nrec, uint2* pairs, unsigned long long* gcur, size_t ws_base) {
  if (nrec > kMaxLaunchRecords || n >= 0xFFFFFFFFull - 2 * kPT) {
    set_error("bucket emit: a launch holds <= 2^24 records and < 2^32 - 2^15 entries");
    return SG_EINVAL;
  }
  EmitArgs e{};
  e.pairs = pairs;
  e.update = true;
  e.gcur = gcur;
  e.goff = d_off;
  return bucket_triage_one(ctx, mwords, nwords, d_vals, d_off, n, nrec, nullptr, &e, ws_base);
}

}  // namespace sg
