// sg_bucket.hip -- partitioned new-signal triage (the fast path of
// sg_triage_batch when the caller does not ask for the ordered diff lists).
//
// Reference: syz-fuzzer/fuzzer.go:645-693.  Its observable results are which
// call records get queued for triage (fuzzer.go:678-690) and the updated
// maxSignal / newSignal (fuzzer.go:673-674); the diff slice (fuzzer.go:669)
// is a transient that only feeds those SignalAdd calls.
//
// Same first-owner rule as sg_triage.hip (a record is new iff it is the
// first, in sequential order, to contain some signal s not in maxSignal),
// organised so that no access is random across HBM:
//   1. stable LSD partition of (s, record) pairs by bits 15..22 of s,
//   2. stable LSD partition by bits 23..31 -> pairs grouped by the 17-bit
//      bucket s >> 15 (32768 signals, a 4 KiB slice of the bitmap),
//   3. one workgroup per bucket: the bucket's maxSignal slice, its new bits,
//      and a small LDS hash map signal -> min(record) over the candidates
//      (signals not in maxSignal) decide which records are new; the slice's
//      new bits go back to maxSignal / newSignal from the bucket's only
//      writer.  Buckets with more candidates than the LDS lists hold are
//      redone by a second kernel with a direct 32768-entry LDS table.
// No global atomics, no 16 GiB owner table, every HBM stream coalesced.
//
// Partition pass = histogram kernel (per 8192-value tile, LDS counters) +
// device exclusive scan over [digit][tile] + scatter kernel: each wave holds
// its 1024 values in registers, ranks them in order with a ballot multisplit
// (stable), the tile is reordered by digit in LDS and written out in digit
// runs.
#include "sg_internal.h"

#include <cstdlib>

namespace sg {

constexpr int kPT = 8192;                   // partition tile (values): LDS fits two tiles per CU
constexpr int kPThreads = 512;              // 8 waves
constexpr int kPWaves = kPThreads / 64;
constexpr int kPerWave = kPT / kPWaves;     // 1024 values per wave, in order
constexpr int kSteps = kPerWave / 64;       // 16 values per lane
constexpr int kBucketBits = 15;             // 32768 signals per bucket
constexpr uint32_t kBucketSig = 1u << kBucketBits;
constexpr uint32_t kBucketWords = kBucketSig / 32;  // 1024
constexpr uint32_t kNumBuckets = 1u << (32 - kBucketBits);  // 131072
constexpr int kD0Shift = 15, kD0Bits = 8;   // pass 1 digit: bits 15..22
constexpr int kD1Shift = 23, kD1Bits = 9;   // pass 2 digit: bits 23..31
constexpr int kRecWin = 512;                // record offsets kept in LDS per tile
constexpr int kBTThreads = 512;             // bucket kernel
constexpr int kHashBits = 11;
constexpr int kHash = 1 << kHashBits;       // candidate hash slots per bucket
constexpr int kCandCap = 2048;              // candidates kept per bucket

struct PartArgs {
  const uint32_t* vals;    // pass 1 input
  const uint64_t* pairs;   // pass 2 input: (s << 32) | record
  uint64_t n;
  uint64_t ntiles;
  const uint64_t* rec_off; // pass 1: record offsets (nrec+1)
  uint64_t nrec;
  const uint32_t* tile_rec;// pass 1: record of each tile's first value (ntiles+1)
  uint32_t* hist;          // [digit][tile]
  const uint64_t* goff;    // scanned hist: output start of (digit, tile)
  uint64_t* out;           // pairs out
};

template <int kShift, int kBits>
__device__ __forceinline__ uint32_t digit_of(uint32_t s) {
  return (s >> kShift) & ((1u << kBits) - 1);
}

// lanes of this wave holding the same digit as this lane (valid lanes only)
template <int kBits>
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < kBits; b++) {
    const bool bit = (d >> b) & 1u;
    const uint64_t bb = __ballot(valid && bit);
    m &= bit ? bb : ~bb;
  }
  return valid ? m : 0ull;
}

template <bool kPairs, int kShift, int kBits>
__global__ __launch_bounds__(kPThreads) void k_part_hist(PartArgs a) {
  constexpr int R = 1 << kBits;
  __shared__ uint32_t cnt[R];
  for (int i = threadIdx.x; i < R; i += kPThreads) cnt[i] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * kPT;
  if (kPairs) {  // 16-B loads: 2 pairs per lane per load, 8 loads per lane
    const bool full = t0 + kPT <= a.n && (((uintptr_t)a.pairs & 15) == 0);
    if (full) {
      const uint4* p4 = reinterpret_cast<const uint4*>(a.pairs + t0);
      uint4 q[kPT / 2 / kPThreads];
#pragma unroll
      for (int j = 0; j < kPT / 2 / kPThreads; j++) q[j] = p4[j * kPThreads + threadIdx.x];
#pragma unroll
      for (int j = 0; j < kPT / 2 / kPThreads; j++) {
        atomicAdd(&cnt[digit_of<kShift, kBits>(q[j].y)], 1u);
        atomicAdd(&cnt[digit_of<kShift, kBits>(q[j].w)], 1u);
      }
    } else {
      for (int i = threadIdx.x; i < kPT; i += kPThreads) {
        const uint64_t e = t0 + i;
        if (e < a.n) atomicAdd(&cnt[digit_of<kShift, kBits>((uint32_t)(a.pairs[e] >> 32))], 1u);
      }
    }
  } else {  // 16-B loads: 4 values per lane per load, 4 loads per lane
    const bool full = t0 + kPT <= a.n && (((uintptr_t)a.vals & 15) == 0);
    if (full) {
      const uint4* v4 = reinterpret_cast<const uint4*>(a.vals + t0);
      uint4 q[kPT / 4 / kPThreads];
#pragma unroll
      for (int j = 0; j < kPT / 4 / kPThreads; j++) q[j] = v4[j * kPThreads + threadIdx.x];
#pragma unroll
      for (int j = 0; j < kPT / 4 / kPThreads; j++) {
        atomicAdd(&cnt[digit_of<kShift, kBits>(q[j].x)], 1u);
        atomicAdd(&cnt[digit_of<kShift, kBits>(q[j].y)], 1u);
        atomicAdd(&cnt[digit_of<kShift, kBits>(q[j].z)], 1u);
        atomicAdd(&cnt[digit_of<kShift, kBits>(q[j].w)], 1u);
      }
    } else {
      for (int i = threadIdx.x; i < kPT; i += kPThreads) {
        const uint64_t e = t0 + i;
        if (e < a.n) atomicAdd(&cnt[digit_of<kShift, kBits>(a.vals[e])], 1u);
      }
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < R; d += kPThreads) a.hist[(uint64_t)d * a.ntiles + blockIdx.x] = cnt[d];
}

template <bool kPairs, int kShift, int kBits, bool kDirect>
__global__ __launch_bounds__(kPThreads) void k_part_scatter(PartArgs a) {
  constexpr int R = 1 << kBits;
  constexpr int W = kPairs ? 1 : kRecWin;
  __shared__ uint64_t stage[kDirect ? 1 : kPT];  // the tile, reordered by digit (64 KiB)
  __shared__ uint16_t cur[kPWaves][R];        // per-wave digit cursors
  __shared__ uint32_t cur32[kDirect ? kPWaves : 1][kDirect ? R : 1];
  __shared__ uint16_t dstart[R];              // tile-local start of each digit
  __shared__ uint32_t tot[R];
  __shared__ uint64_t gbase[R];               // global start of (digit, this tile)
  __shared__ uint64_t win[W];                 // pass 1: record offsets of the tile
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint64_t tile = blockIdx.x, t0 = tile * kPT;
  const uint64_t ebase = t0 + (uint64_t)w * kPerWave;
  // this wave's 1024 values in registers, every load in flight at once
  uint64_t pv[kSteps];
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    const uint64_t e = ebase + (uint64_t)k * 64 + lane;
    if (kPairs)
      pv[k] = e < a.n ? a.pairs[e] : 0ull;
    else
      pv[k] = e < a.n ? ((uint64_t)a.vals[e] << 32) : 0ull;
  }
  uint64_t ra = 0, rb = 0, wn = 0;
  if (!kPairs) {
    ra = a.tile_rec[tile];
    rb = a.tile_rec[tile + 1];
    wn = rb - ra + 1;
    if (wn <= (uint64_t)W)
      for (uint64_t i = tid; i < wn; i += kPThreads) win[i] = a.rec_off[ra + i];
  }
  for (int d = lane; d < R; d += 64) cur[w][d] = 0;
  for (int d = tid; d < R; d += kPThreads) gbase[d] = a.goff[(uint64_t)d * a.ntiles + tile];
  // walk 1: per-wave digit counts (not unrolled: unrolling piles up 16 steps of ballots and spills)
#pragma unroll 1
  for (int k = 0; k < kSteps; k++) {
    const bool v = ebase + (uint64_t)k * 64 + lane < a.n;
    const uint32_t d = digit_of<kShift, kBits>((uint32_t)(pv[k] >> 32));
    const uint64_t m = match_digit<kBits>(d, v);
    if (v && !(m & lt)) cur[w][d] += (uint16_t)__popcll(m);
    __builtin_amdgcn_sched_barrier(0);  // keep the steps' ballots from piling up in SGPRs
  }
  __syncthreads();
  // exclusive prefix over waves per digit, then over digits
  for (int d = tid; d < R; d += kPThreads) {
    uint32_t acc = 0;
    for (int q = 0; q < kPWaves; q++) {
      const uint32_t c = cur[q][d];
      cur[q][d] = (uint16_t)acc;
      acc += c;
    }
    tot[d] = acc;
  }
  __syncthreads();
  if (tid < 64) {  // one wave scans the R digit totals
    uint32_t carry = 0;
    for (int base = 0; base < R; base += 64) {
      uint32_t x = tot[base + lane];
      uint32_t incl = x;
      for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      dstart[base + lane] = (uint16_t)(carry + incl - x);
      carry += __shfl(incl, 63);
    }
  }
  __syncthreads();
  if (kDirect) {  // cursors become global positions of this wave's values
    for (int d = lane; d < R; d += 64) cur32[w][d] = (uint32_t)cur[w][d];
  } else {
    for (int d = lane; d < R; d += 64) cur[w][d] += dstart[d];
  }
  // record of this lane's first value; later values of the lane only move forward
  uint64_t r = 0;
  if (!kPairs) {
    const uint64_t e0 = ebase + lane;
    if (e0 < a.n)
      r = wn <= (uint64_t)W ? ra + sgd::seg_search(win, 0, wn - 1, e0) : sgd::seg_search(a.rec_off, ra, rb, e0);
  }
  // walk 2: stable rank -> LDS position
#pragma unroll 1
  for (int k = 0; k < kSteps; k++) {
    const uint64_t e = ebase + (uint64_t)k * 64 + lane;
    const bool v = e < a.n;
    uint64_t pair = pv[k];
    if (!kPairs && v) {
      if (wn <= (uint64_t)W) {
        while (r < rb && win[r + 1 - ra] <= e) r++;
      } else {
        r = sgd::seg_search(a.rec_off, r, rb, e);
      }
      pair |= (uint32_t)r;
    }
    const uint32_t d = digit_of<kShift, kBits>((uint32_t)(pair >> 32));
    const uint64_t m = match_digit<kBits>(d, v);
    if (v) {
      if (kDirect) {
        const uint32_t base = cur32[w][d];
        a.out[gbase[d] + base + __popcll(m & lt)] = pair;
        if (!(m & lt)) cur32[w][d] = base + __popcll(m);
      } else {
        const uint32_t base = cur[w][d];
        stage[base + __popcll(m & lt)] = pair;
        if (!(m & lt)) cur[w][d] = (uint16_t)(base + __popcll(m));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (kDirect) return;
  __syncthreads();
  // write out in digit runs (consecutive threads -> consecutive addresses)
  const uint32_t ntile = (uint32_t)(a.n - t0 < (uint64_t)kPT ? a.n - t0 : (uint64_t)kPT);
  for (uint32_t p = tid; p < ntile; p += kPThreads) {
    const uint64_t pair = stage[p];
    const uint32_t d = digit_of<kShift, kBits>((uint32_t)(pair >> 32));
    a.out[gbase[d] + (p - dstart[d])] = pair;
  }
}

__global__ void k_tile_rec_pt(const uint64_t* __restrict__ off, uint64_t nseg, uint64_t n, uint64_t ntiles,
                              uint32_t* __restrict__ tile_rec) {
  uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > ntiles) return;
  uint64_t e = t * kPT;
  if (e >= n) e = n - 1;
  tile_rec[t] = (uint32_t)sgd::seg_search(off, 0, nseg - 1, e);
}

// first pair index of every bucket (pairs grouped by s >> 15, ascending)
__global__ void k_bucket_bounds(const uint64_t* __restrict__ pairs, uint64_t n, uint64_t* __restrict__ bounds) {
  uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b > kNumBuckets) return;
  const uint64_t key = b << kBucketBits;  // first signal of bucket b (2^32 for b == kNumBuckets)
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if ((pairs[mid] >> 32) < key)
      lo = mid + 1;
    else
      hi = mid;
  }
  bounds[b] = lo;
}

struct BucketArgs {
  const uint64_t* pairs;
  const uint64_t* bounds;
  uint32_t* mwords;     // maxSignal
  uint32_t* nwords;     // newSignal (nullable)
  uint8_t* rec_new;
  uint32_t* spill;      // buckets left for the direct-table kernel
  uint32_t* nspill;
};

__device__ __forceinline__ uint32_t slot_of(uint32_t sl) { return (sl * 2654435761u) >> (32 - kHashBits); }

// Write the bucket's new bits: maxSignal = slice | new, newSignal |= new.
__device__ __forceinline__ void flush_new_bits(const BucketArgs& a, uint32_t b, const uint32_t* mslice,
                                               const uint32_t* nbits, int tid, int nthreads) {
  uint32_t* mg = a.mwords + (uint64_t)b * kBucketWords;
  uint32_t* ng = a.nwords ? a.nwords + (uint64_t)b * kBucketWords : nullptr;
  for (uint32_t i = tid; i < kBucketWords; i += nthreads) {
    const uint32_t nb = nbits[i];
    if (nb) {
      mg[i] = mslice[i] | nb;
      if (ng) ng[i] |= nb;
    }
  }
}

__global__ __launch_bounds__(kBTThreads) void k_bucket_triage(BucketArgs a) {
  __shared__ uint32_t mslice[kBucketWords];
  __shared__ uint32_t nbits[kBucketWords];
  __shared__ uint32_t hkey[kHash];
  __shared__ uint32_t hval[kHash];
  __shared__ uint64_t cand[kCandCap];   // (signal & 32767) << 32 | record
  __shared__ uint32_t ncand, overflow;
  const uint32_t b = blockIdx.x;
  const uint64_t lo = a.bounds[b], hi = a.bounds[b + 1];
  if (lo == hi) return;  // no signal of this batch falls in the bucket
  const int tid = threadIdx.x;
  const uint32_t* mg = a.mwords + (uint64_t)b * kBucketWords;
  for (uint32_t i = tid; i < kBucketWords; i += kBTThreads) {
    mslice[i] = mg[i];
    nbits[i] = 0;
  }
  for (uint32_t i = tid; i < kHash; i += kBTThreads) {
    hkey[i] = ~0u;
    hval[i] = ~0u;
  }
  if (tid == 0) {
    ncand = 0;
    overflow = 0;
  }
  __syncthreads();
  // candidates: signals not in maxSignal; owner = min record per signal
  constexpr int kU = 8;
  for (uint64_t base = lo; base < hi; base += (uint64_t)kBTThreads * kU) {
    uint64_t p[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const uint64_t i = base + (uint64_t)u * kBTThreads + tid;
      p[u] = i < hi ? a.pairs[i] : ~0ull;
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      if (p[u] == ~0ull) continue;
      const uint32_t sl = (uint32_t)(p[u] >> 32) & (kBucketSig - 1);
      const uint32_t rec = (uint32_t)p[u];
      if ((mslice[sl >> 5] >> (sl & 31)) & 1u) continue;
      atomicOr(&nbits[sl >> 5], 1u << (sl & 31));
      const uint32_t c = atomicAdd(&ncand, 1u);
      if (c < (uint32_t)kCandCap) cand[c] = ((uint64_t)sl << 32) | rec;
      uint32_t h = slot_of(sl);
      int probes = 0;
      for (;;) {
        const uint32_t k = atomicCAS(&hkey[h], ~0u, sl);
        if (k == ~0u || k == sl) {
          atomicMin(&hval[h], rec);
          break;
        }
        h = (h + 1) & (kHash - 1);
        if (++probes == kHash) {
          overflow = 1;
          break;
        }
      }
    }
  }
  __syncthreads();
  if (overflow || ncand > (uint32_t)kCandCap) {  // redo with the direct table (no global writes yet)
    if (tid == 0) a.spill[atomicAdd(a.nspill, 1u)] = b;
    return;
  }
  // a record is queued iff it owns some signal (fuzzer.go:666, :678-690)
  for (uint32_t i = tid; i < ncand; i += kBTThreads) {
    const uint64_t c = cand[i];
    const uint32_t sl = (uint32_t)(c >> 32), rec = (uint32_t)c;
    uint32_t h = slot_of(sl);
    while (hkey[h] != sl) h = (h + 1) & (kHash - 1);
    if (hval[h] == rec) a.rec_new[rec] = 1;
  }
  flush_new_bits(a, b, mslice, nbits, tid, kBTThreads);
}

// Buckets with too many candidates: direct first-owner table in LDS.
__global__ __launch_bounds__(kPThreads) void k_bucket_triage_direct(BucketArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t owner[kBucketSig];  // 128 KiB
  __shared__ uint32_t mslice[kBucketWords];
  __shared__ uint32_t nbits[kBucketWords];
  const int tid = threadIdx.x;
  const uint32_t nsp = *a.nspill;
  for (uint32_t j = blockIdx.x; j < nsp; j += gridDim.x) {
    const uint32_t b = a.spill[j];
    const uint64_t lo = a.bounds[b], hi = a.bounds[b + 1];
    const uint32_t* mg = a.mwords + (uint64_t)b * kBucketWords;
    for (uint32_t i = tid; i < kBucketWords; i += kPThreads) {
      mslice[i] = mg[i];
      nbits[i] = 0;
    }
    uint4* o4 = reinterpret_cast<uint4*>(owner);
    for (uint32_t i = tid; i < kBucketSig / 4; i += kPThreads) o4[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
    __syncthreads();
    for (uint64_t i = lo + tid; i < hi; i += kPThreads) {
      const uint64_t p = a.pairs[i];
      const uint32_t sl = (uint32_t)(p >> 32) & (kBucketSig - 1);
      if ((mslice[sl >> 5] >> (sl & 31)) & 1u) continue;
      atomicMin(&owner[sl], (uint32_t)p);
      atomicOr(&nbits[sl >> 5], 1u << (sl & 31));
    }
    __syncthreads();
    for (uint64_t i = lo + tid; i < hi; i += kPThreads) {
      const uint64_t p = a.pairs[i];
      const uint32_t sl = (uint32_t)(p >> 32) & (kBucketSig - 1);
      if (owner[sl] == (uint32_t)p) a.rec_new[(uint32_t)p] = 1;  // owner set => candidate
    }
    flush_new_bits(a, b, mslice, nbits, tid, kPThreads);
    __syncthreads();
  }
}

// Experiment switch: SG_PART_DIRECT=1 scatters straight from registers to HBM
// (no LDS reorder; more blocks per CU, partial-line writes).
static bool part_direct() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SG_PART_DIRECT");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  return v == 1;
}

size_t bucket_ws_bytes(uint64_t n) {
  const uint64_t nt = (n + kPT - 1) / kPT;
  WsPlan p;
  p.add(n * 8);
  p.add(n * 8);
  p.add((uint64_t)(1 << kD0Bits) * nt * 4);
  p.add(((uint64_t)(1 << kD0Bits) * nt + 1) * 8);
  p.add((uint64_t)(1 << kD1Bits) * nt * 4);
  p.add(((uint64_t)(1 << kD1Bits) * nt + 1) * 8);
  p.add((nt + 1) * 4);
  p.add(((uint64_t)kNumBuckets + 1) * 8);
  p.add(((uint64_t)kNumBuckets + 1) * 4);
  return p.total + scan_ws_bytes((uint64_t)(1 << kD1Bits) * nt);
}

// Flags-only triage of a device-resident batch (ctx lock held).
int bucket_triage(sg_ctx* ctx, uint32_t* mwords, uint32_t* nwords, const uint32_t* d_vals, const uint64_t* d_off,
                  uint64_t n, uint64_t nrec, uint8_t* d_rec_new) {
  if (nrec >= 0xFFFFFFFFull) {
    set_error("bucket triage: record index must fit 32 bits");
    return SG_EINVAL;
  }
  if (nrec) SG_HIP(hipMemsetAsync(d_rec_new, 0, nrec, ctx->stream));
  if (n == 0) return SG_OK;
  const uint64_t nt = (n + kPT - 1) / kPT;
  WsPlan p;
  const size_t oA = p.add(n * 8), oB = p.add(n * 8);
  const size_t oH1 = p.add((uint64_t)(1 << kD0Bits) * nt * 4), oO1 = p.add(((uint64_t)(1 << kD0Bits) * nt + 1) * 8);
  const size_t oH2 = p.add((uint64_t)(1 << kD1Bits) * nt * 4), oO2 = p.add(((uint64_t)(1 << kD1Bits) * nt + 1) * 8);
  const size_t oTR = p.add((nt + 1) * 4), oBB = p.add(((uint64_t)kNumBuckets + 1) * 8);
  const size_t oSP = p.add(((uint64_t)kNumBuckets + 1) * 4);
  const size_t scan_off = p.total;
  int rc = ws_reserve(ctx, bucket_ws_bytes(n));
  if (rc) return rc;
  uint64_t* A = (uint64_t*)ws_at(ctx, oA);
  uint64_t* B = (uint64_t*)ws_at(ctx, oB);
  PartArgs pa{};
  pa.n = n;
  pa.ntiles = nt;
  pa.rec_off = d_off;
  pa.nrec = nrec;
  pa.tile_rec = (uint32_t*)ws_at(ctx, oTR);
  hipLaunchKernelGGL(k_tile_rec_pt, dim3(div_up(nt + 1, 256)), dim3(256), 0, ctx->stream, d_off, nrec, n, nt,
                     (uint32_t*)pa.tile_rec);
  {
    ScopedTimer tm(ctx, "part1_hist");
    pa.vals = d_vals;
    pa.hist = (uint32_t*)ws_at(ctx, oH1);
    hipLaunchKernelGGL((k_part_hist<false, kD0Shift, kD0Bits>), dim3((uint32_t)nt), dim3(kPThreads), 0, ctx->stream,
                       pa);
  }
  rc = scan_counts(ctx, pa.hist, (uint64_t*)ws_at(ctx, oO1), (uint64_t)(1 << kD0Bits) * nt, scan_off);
  if (rc) return rc;
  {
    ScopedTimer tm(ctx, "part1_scatter");
    pa.goff = (uint64_t*)ws_at(ctx, oO1);
    pa.out = A;
    if (part_direct())
      hipLaunchKernelGGL((k_part_scatter<false, kD0Shift, kD0Bits, true>), dim3((uint32_t)nt), dim3(kPThreads), 0,
                         ctx->stream, pa);
    else
      hipLaunchKernelGGL((k_part_scatter<false, kD0Shift, kD0Bits, false>), dim3((uint32_t)nt), dim3(kPThreads), 0,
                         ctx->stream, pa);
  }
  {
    ScopedTimer tm(ctx, "part2_hist");
    pa.vals = nullptr;
    pa.pairs = A;
    pa.hist = (uint32_t*)ws_at(ctx, oH2);
    hipLaunchKernelGGL((k_part_hist<true, kD1Shift, kD1Bits>), dim3((uint32_t)nt), dim3(kPThreads), 0, ctx->stream,
                       pa);
  }
  rc = scan_counts(ctx, pa.hist, (uint64_t*)ws_at(ctx, oO2), (uint64_t)(1 << kD1Bits) * nt, scan_off);
  if (rc) return rc;
  {
    ScopedTimer tm(ctx, "part2_scatter");
    pa.goff = (uint64_t*)ws_at(ctx, oO2);
    pa.out = B;
    if (part_direct())
      hipLaunchKernelGGL((k_part_scatter<true, kD1Shift, kD1Bits, true>), dim3((uint32_t)nt), dim3(kPThreads), 0,
                         ctx->stream, pa);
    else
      hipLaunchKernelGGL((k_part_scatter<true, kD1Shift, kD1Bits, false>), dim3((uint32_t)nt), dim3(kPThreads), 0,
                         ctx->stream, pa);
  }
  BucketArgs ba{};
  ba.pairs = B;
  ba.bounds = (uint64_t*)ws_at(ctx, oBB);
  ba.mwords = mwords;
  ba.nwords = nwords;
  ba.rec_new = d_rec_new;
  ba.nspill = (uint32_t*)ws_at(ctx, oSP);
  ba.spill = ba.nspill + 1;
  SG_HIP(hipMemsetAsync(ba.nspill, 0, 4, ctx->stream));
  {
    ScopedTimer tm(ctx, "bucket_bounds");
    hipLaunchKernelGGL(k_bucket_bounds, dim3(div_up((uint64_t)kNumBuckets + 1, 256)), dim3(256), 0, ctx->stream, B,
                       n, (uint64_t*)ba.bounds);
  }
  {
    ScopedTimer tm(ctx, "bucket_triage");
    hipLaunchKernelGGL(k_bucket_triage, dim3(kNumBuckets), dim3(kBTThreads), 0, ctx->stream, ba);
  }
  {
    ScopedTimer tm(ctx, "bucket_spill");
    hipLaunchKernelGGL(k_bucket_triage_direct, dim3(512), dim3(kPThreads), 0, ctx->stream, ba);
  }
  SG_HIP(hipGetLastError());
  return SG_OK;
}

}  // namespace sg
