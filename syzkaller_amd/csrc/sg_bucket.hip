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
//   1. stable MSD partition of the batch by the coarse digit s >> 23: 512
//      slices of 2^23 signals, each backed by 1 MiB of the maxSignal bitmap;
//      out: (s, record) in two u32 arrays,
//   2. per coarse slice, a stable partition by the fine digit (s >> 15) & 255
//      that DROPS every s already in maxSignal.  The workgroups of one XCD
//      walk consecutive tiles, so the slice they probe is the same 1 MiB and
//      stays in that XCD's L2; only the candidates (signals not in
//      maxSignal, ~12 % of a C2 batch, far fewer in a warm fuzzer) go on,
//      as (s << 32 | record) pairs grouped by the 17-bit bucket s >> 15,
//   3. one workgroup per bucket (32768 signals): an LDS hash map
//      signal -> min(record) over its candidates decides the new records
//      and the bucket's new bits go back to maxSignal / newSignal from its
//      only writer.  Buckets with more distinct candidates than the map
//      holds are redone by a second kernel with a direct 32768-entry table.
// No global atomics, no 16 GiB owner table, every HBM stream coalesced.
//
// A partition pass = histogram kernel (per 8192-value tile, LDS counters) +
// device exclusive scan over [digit][tile] + scatter kernel: each wave holds
// its 1024 values in registers, ranks them in order with a ballot multisplit
// (stable), the tile is reordered by digit in LDS and written out in digit
// runs.  Both scatters map blocks to tiles XCD-contiguously (T1 swizzle), so
// the partial lines at digit-run seams of neighbouring tiles merge in one L2.
#include "sg_internal.h"

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
constexpr int kCShift = 23, kCBits = 9;     // pass 1 (coarse) digit: bits 23..31
constexpr int kFShift = 15, kFBits = 8;     // pass 2 (fine) digit: bits 15..22
constexpr uint32_t kNumCoarse = 1u << kCBits;
constexpr int kRecWin = 1024;               // record offsets kept in LDS per tile (tile-relative u16)
constexpr int kBTThreads = 512;             // bucket kernel
constexpr int kBU = 16;                     // pairs per thread in flight (8192 per block)
constexpr int kHash = 4096;                 // max candidate hash slots per bucket

// blocks sharing an XCD (bid % 8 under round-robin dispatch) get a contiguous
// run of tiles; a bijection on [0, g) for any g (speed only, never correctness)
__device__ __forceinline__ uint32_t xcd_tile(uint32_t bid, uint32_t g) {
  const uint32_t x = bid & 7, q = g >> 3, r = g & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

template <int kShift, int kBits>
__device__ __forceinline__ uint32_t digit_of(uint32_t s) {
  return (s >> kShift) & ((1u << kBits) - 1);
}

// Counting sort of one tile held in registers (kSteps values per lane) by
// digit, through LDS: counts, one-wave exclusive scan, then every value takes
// a slot with an LDS atomic.  The order within a digit is NOT the input order
// -- nothing downstream needs it: first owners are minima over records.
// On return cnt[] is free, dstart[d] is the digit's first slot in the tile
// and pos[k] the slot of value k (valid lanes only).
template <int kBits>
__device__ __forceinline__ void tile_rank(const uint32_t (&dv)[kSteps], uint32_t vmask, uint32_t* cnt,
                                          uint16_t* dstart, uint32_t (&pos)[kSteps]) {
  constexpr int R = 1 << kBits;
  const int tid = threadIdx.x, lane = tid & 63;
#pragma unroll
  for (int k = 0; k < kSteps; k++)
    if ((vmask >> k) & 1u) atomicAdd(&cnt[dv[k]], 1u);
  __syncthreads();
  if (tid < 64) {  // one wave scans the R digit counts; cnt becomes the cursor
    uint32_t carry = 0;
    for (int base = 0; base < R; base += 64) {
      const uint32_t x = cnt[base + lane];
      uint32_t incl = x;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      const uint32_t ex = carry + incl - x;
      dstart[base + lane] = (uint16_t)ex;
      cnt[base + lane] = ex;
      carry += __shfl(incl, 63);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kSteps; k++)
    if ((vmask >> k) & 1u) pos[k] = atomicAdd(&cnt[dv[k]], 1u);
}

// ---------------------------------------------------------------- pass 1 ---

struct P1Args {
  const uint32_t* vals;
  uint64_t n;
  uint64_t ntiles;
  const uint64_t* rec_off;  // nrec + 1
  const uint32_t* tile_rec; // record of each tile's first value (ntiles + 1)
  uint32_t* hist;           // [coarse digit][tile]
  const uint64_t* goff;     // scanned hist
  uint32_t* s_out;          // partitioned signals
  uint32_t* r_out;          // their records
};

__global__ __launch_bounds__(kPThreads) void k_p1_hist(P1Args a) {
  constexpr int R = 1 << kCBits;
  __shared__ uint32_t cnt[R];
  for (int i = threadIdx.x; i < R; i += kPThreads) cnt[i] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * kPT;
  if (t0 + kPT <= a.n && (((uintptr_t)a.vals & 15) == 0)) {  // 16-B loads, 4 per lane
    const uint4* v4 = reinterpret_cast<const uint4*>(a.vals + t0);
    uint4 q[kPT / 4 / kPThreads];
#pragma unroll
    for (int j = 0; j < kPT / 4 / kPThreads; j++) q[j] = v4[j * kPThreads + threadIdx.x];
#pragma unroll
    for (int j = 0; j < kPT / 4 / kPThreads; j++) {
      atomicAdd(&cnt[digit_of<kCShift, kCBits>(q[j].x)], 1u);
      atomicAdd(&cnt[digit_of<kCShift, kCBits>(q[j].y)], 1u);
      atomicAdd(&cnt[digit_of<kCShift, kCBits>(q[j].z)], 1u);
      atomicAdd(&cnt[digit_of<kCShift, kCBits>(q[j].w)], 1u);
    }
  } else {
    for (int i = threadIdx.x; i < kPT; i += kPThreads) {
      const uint64_t e = t0 + i;
      if (e < a.n) atomicAdd(&cnt[digit_of<kCShift, kCBits>(a.vals[e])], 1u);
    }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < R; d += kPThreads) a.hist[(uint64_t)d * a.ntiles + blockIdx.x] = cnt[d];
}

__global__ __launch_bounds__(kPThreads) void k_p1_scatter(P1Args a) {
  constexpr int R = 1 << kCBits;
  __shared__ uint64_t stage[kPT];        // the tile grouped by digit: (s << 32) | record (64 KiB)
  __shared__ uint32_t cnt[R];
  __shared__ uint16_t dstart[R];         // tile-local start of each digit
  __shared__ uint64_t gbase[R];          // global start of (digit, this tile)
  __shared__ uint16_t win[kRecWin];      // record offsets of the tile, clamped to [t0, t0 + kPT] - t0
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x), t0 = tile * kPT;
  const uint64_t ebase = t0 + (uint64_t)w * kPerWave;
  // this wave's 1024 values in registers, every load in flight at once
  uint32_t sv[kSteps];
  uint32_t vmask = 0;
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    const uint64_t e = ebase + (uint64_t)k * 64 + lane;
    sv[k] = e < a.n ? a.vals[e] : 0u;
    vmask |= (e < a.n ? 1u : 0u) << k;
  }
  const uint64_t ra = a.tile_rec[tile], rb = a.tile_rec[tile + 1], wn = rb - ra + 1;
  const bool inwin = wn <= (uint64_t)kRecWin;
  if (inwin)
    for (uint64_t i = tid; i < wn; i += kPThreads) {
      const uint64_t o = a.rec_off[ra + i];
      win[i] = (uint16_t)(o <= t0 ? 0 : (o - t0 >= (uint64_t)kPT ? kPT : o - t0));
    }
  for (int d = tid; d < R; d += kPThreads) {
    gbase[d] = a.goff[(uint64_t)d * a.ntiles + tile];
    cnt[d] = 0;
  }
  __syncthreads();
  // records: a lane's values are in order, so its record only moves forward
  uint32_t rv[kSteps];
  {
    uint64_t r = 0;
    const uint64_t e0 = ebase + lane;
    if (e0 < a.n) r = inwin ? ra + sgd::seg_search(win, 0, wn - 1, e0 - t0) : sgd::seg_search(a.rec_off, ra, rb, e0);
#pragma unroll
    for (int k = 0; k < kSteps; k++) {
      const uint64_t e = ebase + (uint64_t)k * 64 + lane;
      if ((vmask >> k) & 1u) {
        if (inwin) {
          const uint32_t el = (uint32_t)(e - t0);
          while (r < rb && win[r + 1 - ra] <= el) r++;
        } else {
          r = sgd::seg_search(a.rec_off, r, rb, e);
        }
      }
      rv[k] = (uint32_t)r;
    }
  }
  uint32_t dv[kSteps], pos[kSteps];
#pragma unroll
  for (int k = 0; k < kSteps; k++) dv[k] = digit_of<kCShift, kCBits>(sv[k]);
  tile_rank<kCBits>(dv, vmask, cnt, dstart, pos);
#pragma unroll
  for (int k = 0; k < kSteps; k++)
    if ((vmask >> k) & 1u) stage[pos[k]] = ((uint64_t)sv[k] << 32) | rv[k];
  __syncthreads();
  // write out in digit runs (consecutive threads -> consecutive addresses)
  const uint32_t ntile = (uint32_t)(a.n - t0 < (uint64_t)kPT ? a.n - t0 : (uint64_t)kPT);
  for (uint32_t p = tid; p < ntile; p += kPThreads) {
    const uint64_t pair = stage[p];
    const uint32_t d = digit_of<kCShift, kCBits>((uint32_t)(pair >> 32));
    const uint64_t o = gbase[d] + (p - dstart[d]);
    a.s_out[o] = (uint32_t)(pair >> 32);
    a.r_out[o] = (uint32_t)pair;
  }
}

// Tiles of pass 2: coarse slice c covers [cs[c], cs[c+1]) of the pass-1
// output and owns tiles [tb[c], tb[c+1]); tb[512] = number of tiles.
__global__ __launch_bounds__(kNumCoarse) void k_p2_tiles(const uint64_t* __restrict__ goff1, uint64_t nt, uint64_t n,
                                                         uint64_t* __restrict__ cs, uint32_t* __restrict__ tb) {
  __shared__ uint32_t k[kNumCoarse];
  const uint32_t c = threadIdx.x;
  const uint64_t lo = goff1[(uint64_t)c * nt];
  const uint64_t hi = c + 1 < kNumCoarse ? goff1[(uint64_t)(c + 1) * nt] : n;
  cs[c] = lo;
  if (c == 0) cs[kNumCoarse] = n;
  k[c] = (uint32_t)((hi - lo + kPT - 1) / kPT);
  __syncthreads();
  if (c < 64) {
    uint32_t carry = 0;
    for (uint32_t base = 0; base < kNumCoarse; base += 64) {
      const uint32_t x = k[base + c];
      uint32_t incl = x;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if ((int)c >= o) incl += y;
      }
      tb[base + c] = carry + incl - x;
      carry += __shfl(incl, 63);
    }
    if (c == 0) tb[kNumCoarse] = carry;
  }
}

struct P2Args {
  const uint32_t* s_in;
  const uint32_t* r_in;
  const uint64_t* cs;       // coarse slice starts (513)
  const uint32_t* tb;       // coarse slice first tiles (513)
  uint32_t* hist;           // [c][fine digit][tile of c], base 256 * tb[c]
  const uint64_t* goff;     // scanned hist
  uint64_t* out;            // pairs (s << 32) | record grouped by s >> 15
};

struct P2Tile {
  uint32_t c, j, kc;
  uint64_t e0, e1;
  bool live;
};

__device__ __forceinline__ P2Tile p2_tile(const P2Args& a) {
  P2Tile t;
  const uint32_t t2 = xcd_tile(blockIdx.x, gridDim.x);
  const uint32_t nt2 = a.tb[kNumCoarse];
  t.live = t2 < nt2;
  if (!t.live) {
    t.c = t.kc = 0;
    t.j = t2;
    t.e0 = t.e1 = 0;
    return t;
  }
  t.c = (uint32_t)sgd::seg_search(a.tb, 0, kNumCoarse - 1, t2);  // largest c with tb[c] <= t2
  t.j = t2 - a.tb[t.c];
  t.kc = a.tb[t.c + 1] - a.tb[t.c];
  t.e0 = a.cs[t.c] + (uint64_t)t.j * kPT;
  const uint64_t end = a.cs[t.c + 1];
  t.e1 = t.e0 + kPT < end ? t.e0 + kPT : end;
  return t;
}

__device__ __forceinline__ uint64_t p2_hist_index(const P2Args& a, const P2Tile& t, uint32_t d) {
  return ((uint64_t)a.tb[t.c] << kFBits) + (uint64_t)d * t.kc + t.j;
}

__global__ __launch_bounds__(kPThreads) void k_p2_hist(P2Args a) {
  constexpr int R = 1 << kFBits;
  __shared__ uint32_t cnt[R];
  const P2Tile t = p2_tile(a);
  if (!t.live) {  // tail of the upper-bound grid: zero its own slots
    for (int d = threadIdx.x; d < R; d += kPThreads) a.hist[((uint64_t)t.j << kFBits) + d] = 0;
    return;
  }
  for (int i = threadIdx.x; i < R; i += kPThreads) cnt[i] = 0;
  uint32_t sv[kPT / kPThreads];
#pragma unroll
  for (int k = 0; k < kPT / kPThreads; k++) {
    const uint64_t e = t.e0 + (uint64_t)k * kPThreads + threadIdx.x;
    sv[k] = e < t.e1 ? a.s_in[e] : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPT / kPThreads; k++)
    if (t.e0 + (uint64_t)k * kPThreads + threadIdx.x < t.e1) atomicAdd(&cnt[digit_of<kFShift, kFBits>(sv[k])], 1u);
  __syncthreads();
  for (int d = threadIdx.x; d < R; d += kPThreads) a.hist[p2_hist_index(a, t, d)] = cnt[d];
}

__global__ __launch_bounds__(kPThreads) void k_p2_scatter(P2Args a) {
  constexpr int R = 1 << kFBits;
  __shared__ uint64_t stage[kPT];
  __shared__ uint32_t cnt[R];
  __shared__ uint16_t dstart[R];
  __shared__ uint64_t gbase[R];
  const P2Tile t = p2_tile(a);
  if (!t.live) return;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const uint64_t ebase = t.e0 + (uint64_t)w * kPerWave;
  uint32_t sv[kSteps], rv[kSteps];
  uint32_t vmask = 0;
#pragma unroll
  for (int k = 0; k < kSteps; k++) {
    const uint64_t e = ebase + (uint64_t)k * 64 + lane;
    const bool v = e < t.e1;
    sv[k] = v ? a.s_in[e] : 0u;
    rv[k] = v ? a.r_in[e] : 0u;
    vmask |= (v ? 1u : 0u) << k;
  }
  for (int d = tid; d < R; d += kPThreads) {
    gbase[d] = a.goff[p2_hist_index(a, t, d)];
    cnt[d] = 0;
  }
  __syncthreads();
  uint32_t dv[kSteps], pos[kSteps];
#pragma unroll
  for (int k = 0; k < kSteps; k++) dv[k] = digit_of<kFShift, kFBits>(sv[k]);
  tile_rank<kFBits>(dv, vmask, cnt, dstart, pos);
#pragma unroll
  for (int k = 0; k < kSteps; k++)
    if ((vmask >> k) & 1u) stage[pos[k]] = ((uint64_t)sv[k] << 32) | rv[k];
  __syncthreads();
  const uint32_t ntile = (uint32_t)(t.e1 - t.e0);
  for (uint32_t p = tid; p < ntile; p += kPThreads) {
    const uint64_t pair = stage[p];
    const uint32_t d = digit_of<kFShift, kFBits>((uint32_t)(pair >> 32));
    a.out[gbase[d] + (p - dstart[d])] = pair;
  }
}

// First pair of every bucket b = (c << 8) | d, read off the pass-2 scan:
// (c, d)'s first tile slot; empty slices point at the next slice's start.
__global__ void k_bucket_bounds(const uint64_t* __restrict__ goff2, const uint32_t* __restrict__ tb,
                                uint64_t nslots, uint64_t* __restrict__ bounds) {
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b > kNumBuckets) return;
  if (b == kNumBuckets) {
    bounds[b] = goff2[nslots];
    return;
  }
  const uint32_t c = (uint32_t)(b >> kFBits), d = (uint32_t)(b & ((1u << kFBits) - 1));
  bounds[b] = goff2[((uint64_t)tb[c] << kFBits) + (uint64_t)d * (tb[c + 1] - tb[c])];
}

struct BucketArgs {
  const uint64_t* pairs;  // (s << 32) | record, grouped by bucket s >> 15
  const uint64_t* bounds;
  uint32_t* mwords;       // maxSignal
  uint32_t* nwords;       // newSignal (nullable)
  uint8_t* rec_new;
  uint32_t* spill;        // buckets left for the direct-table kernel
  uint32_t* nspill;
};

__device__ __forceinline__ uint32_t slot_of(uint32_t sl, int hbits) { return (sl * 2654435761u) >> (32 - hbits); }

// The bucket's new bits: maxSignal = slice | new, newSignal |= new (this
// block is the only writer of the bucket's 1024 words).
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

__device__ __forceinline__ bool hash_insert(uint32_t* hkey, uint32_t* hval, uint32_t hsize, int hbits,
                                            uint32_t* nbits, uint32_t sl, uint32_t rec) {
  uint32_t h = slot_of(sl, hbits);
  for (uint32_t probes = 0; probes < hsize; probes++) {
    const uint32_t k = atomicCAS(&hkey[h], ~0u, sl);
    if (k == ~0u) atomicOr(&nbits[sl >> 5], 1u << (sl & 31));
    if (k == ~0u || k == sl) {
      atomicMin(&hval[h], rec);
      return true;
    }
    h = (h + 1) & (hsize - 1);
  }
  return false;  // map full
}

__global__ __launch_bounds__(kBTThreads) void k_bucket_triage(BucketArgs a) {
  __shared__ uint32_t mslice[kBucketWords];
  __shared__ uint32_t nbits[kBucketWords];
  __shared__ __attribute__((aligned(16))) uint32_t hkey[kHash];
  __shared__ __attribute__((aligned(16))) uint32_t hval[kHash];
  __shared__ uint32_t ncand;
  const uint32_t b = blockIdx.x;
  const uint64_t lo = a.bounds[b], hi = a.bounds[b + 1];
  if (lo == hi) return;  // no signal of this batch falls in the bucket
  const int tid = threadIdx.x;
  constexpr uint64_t kChunkPairs = (uint64_t)kBTThreads * kBU;
  // the first chunk of pairs (all of a typical bucket) in flight at once
  uint64_t p[kBU];
#pragma unroll
  for (int u = 0; u < kBU; u++) {
    const uint64_t i = lo + (uint64_t)u * kBTThreads + tid;
    p[u] = i < hi ? a.pairs[i] : ~0ull;
  }
  const uint32_t* mg = a.mwords + (uint64_t)b * kBucketWords;
  for (uint32_t i = tid; i < kBucketWords; i += kBTThreads) {
    mslice[i] = mg[i];
    nbits[i] = 0;
  }
  if (tid == 0) ncand = 0;
  __syncthreads();
  // candidates = signals not in maxSignal (fuzzer.go:666)
  uint32_t cm = 0;
#pragma unroll
  for (int u = 0; u < kBU; u++) {
    const uint32_t sl = (uint32_t)(p[u] >> 32) & (kBucketSig - 1);
    if (p[u] != ~0ull && !((mslice[sl >> 5] >> (sl & 31)) & 1u)) cm |= 1u << u;
  }
  if (cm) atomicAdd(&ncand, (uint32_t)__popc(cm));
  __syncthreads();
  // map size: >= 2x the candidates (all could be distinct), capped
  const uint64_t nc = hi - lo > kChunkPairs ? ~0ull : ncand;
  int hbits = 6;
  while ((1 << hbits) < kHash && (1ull << hbits) < 2 * nc) hbits++;
  const uint32_t hsize = 1u << hbits;
  for (uint32_t i = tid; i < hsize; i += kBTThreads) {
    hkey[i] = ~0u;
    hval[i] = ~0u;
  }
  __syncthreads();
  // owner = min record per candidate signal
  bool ok = true;
#pragma unroll
  for (int u = 0; u < kBU; u++)
    if ((cm >> u) & 1u) ok &= hash_insert(hkey, hval, hsize, hbits, nbits, (uint32_t)(p[u] >> 32) & (kBucketSig - 1),
                                          (uint32_t)p[u]);
  for (uint64_t base = lo + kChunkPairs; base < hi; base += kChunkPairs) {  // big buckets
#pragma unroll
    for (int u = 0; u < kBU; u++) {
      const uint64_t i = base + (uint64_t)u * kBTThreads + tid;
      p[u] = i < hi ? a.pairs[i] : ~0ull;
    }
#pragma unroll
    for (int u = 0; u < kBU; u++) {
      const uint32_t sl = (uint32_t)(p[u] >> 32) & (kBucketSig - 1);
      if (p[u] != ~0ull && !((mslice[sl >> 5] >> (sl & 31)) & 1u))
        ok &= hash_insert(hkey, hval, hsize, hbits, nbits, sl, (uint32_t)p[u]);
    }
  }
  if (__syncthreads_or(!ok)) {  // redo with the direct table (no global writes yet)
    if (tid == 0) a.spill[atomicAdd(a.nspill, 1u)] = b;
    return;
  }
  // a record is queued iff it owns some signal (fuzzer.go:678-690)
  for (uint32_t i = tid; i < hsize; i += kBTThreads)
    if (hkey[i] != ~0u) a.rec_new[hval[i]] = 1;
  flush_new_bits(a, b, mslice, nbits, tid, kBTThreads);
}

// Buckets with too many distinct candidates: direct first-owner table in LDS.
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
    for (uint32_t i = tid; i < kBucketSig; i += kPThreads)
      if (owner[i] != ~0u) a.rec_new[owner[i]] = 1;
    flush_new_bits(a, b, mslice, nbits, tid, kPThreads);
    __syncthreads();
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

struct BucketPlan {
  uint64_t nt, g2, nslots;
  WsPlan p;
  size_t oS, oR, oB, oH1, oO1, oTR, oCS, oTB, oH2, oO2, oBB, oSP, scan_off;
  explicit BucketPlan(uint64_t n) {
    nt = (n + kPT - 1) / kPT;
    g2 = nt + kNumCoarse;  // upper bound on pass-2 tiles
    nslots = g2 << kFBits;
    oS = p.add(n * 4);
    oR = p.add(n * 4);
    oB = p.add(n * 8);
    oH1 = p.add((uint64_t)kNumCoarse * nt * 4);
    oO1 = p.add(((uint64_t)kNumCoarse * nt + 1) * 8);
    oTR = p.add((nt + 1) * 4);
    oCS = p.add((kNumCoarse + 1) * 8);
    oTB = p.add((kNumCoarse + 1) * 4);
    oH2 = p.add(nslots * 4);
    oO2 = p.add((nslots + 1) * 8);
    oBB = p.add(((uint64_t)kNumBuckets + 1) * 8);
    oSP = p.add(((uint64_t)kNumBuckets + 1) * 4);
    scan_off = p.total;
  }
  size_t bytes() const {
    const uint64_t m = (uint64_t)kNumCoarse * nt > nslots ? (uint64_t)kNumCoarse * nt : nslots;
    return p.total + scan_ws_bytes(m);
  }
};

size_t bucket_ws_bytes(uint64_t n) { return BucketPlan(n).bytes(); }

// Flags-only triage of a device-resident batch (ctx lock held).
int bucket_triage(sg_ctx* ctx, uint32_t* mwords, uint32_t* nwords, const uint32_t* d_vals, const uint64_t* d_off,
                  uint64_t n, uint64_t nrec, uint8_t* d_rec_new) {
  if (nrec >= 0xFFFFFFFFull) {
    set_error("bucket triage: record index must fit 32 bits");
    return SG_EINVAL;
  }
  if (nrec) SG_HIP(hipMemsetAsync(d_rec_new, 0, nrec, ctx->stream));
  if (n == 0) return SG_OK;
  if ((n + kPT - 1) / kPT + kNumCoarse >= 0xFFFFFFFFull) {
    set_error("bucket triage: batch too large");
    return SG_EINVAL;
  }
  const BucketPlan bp(n);
  int rc = ws_reserve(ctx, bp.bytes());
  if (rc) return rc;
  const uint64_t nt = bp.nt;
  P1Args a1{};
  a1.vals = d_vals;
  a1.n = n;
  a1.ntiles = nt;
  a1.rec_off = d_off;
  a1.tile_rec = (uint32_t*)ws_at(ctx, bp.oTR);
  a1.hist = (uint32_t*)ws_at(ctx, bp.oH1);
  a1.goff = (uint64_t*)ws_at(ctx, bp.oO1);
  a1.s_out = (uint32_t*)ws_at(ctx, bp.oS);
  a1.r_out = (uint32_t*)ws_at(ctx, bp.oR);
  hipLaunchKernelGGL(k_tile_rec_pt, dim3(div_up(nt + 1, 256)), dim3(256), 0, ctx->stream, d_off, nrec, n, nt,
                     (uint32_t*)a1.tile_rec);
  {
    ScopedTimer tm(ctx, "part1_hist");
    hipLaunchKernelGGL(k_p1_hist, dim3((uint32_t)nt), dim3(kPThreads), 0, ctx->stream, a1);
  }
  rc = scan_counts(ctx, a1.hist, (uint64_t*)a1.goff, (uint64_t)kNumCoarse * nt, bp.scan_off);
  if (rc) return rc;
  {
    ScopedTimer tm(ctx, "part1_scatter");
    hipLaunchKernelGGL(k_p1_scatter, dim3((uint32_t)nt), dim3(kPThreads), 0, ctx->stream, a1);
  }
  P2Args a2{};
  a2.s_in = a1.s_out;
  a2.r_in = a1.r_out;
  a2.cs = (uint64_t*)ws_at(ctx, bp.oCS);
  a2.tb = (uint32_t*)ws_at(ctx, bp.oTB);
  a2.hist = (uint32_t*)ws_at(ctx, bp.oH2);
  a2.goff = (uint64_t*)ws_at(ctx, bp.oO2);
  a2.out = (uint64_t*)ws_at(ctx, bp.oB);
  hipLaunchKernelGGL(k_p2_tiles, dim3(1), dim3(kNumCoarse), 0, ctx->stream, a1.goff, nt, n, (uint64_t*)a2.cs,
                     (uint32_t*)a2.tb);
  {
    ScopedTimer tm(ctx, "part2_hist");
    hipLaunchKernelGGL(k_p2_hist, dim3((uint32_t)bp.g2), dim3(kPThreads), 0, ctx->stream, a2);
  }
  rc = scan_counts(ctx, a2.hist, (uint64_t*)a2.goff, bp.nslots, bp.scan_off);
  if (rc) return rc;
  {
    ScopedTimer tm(ctx, "part2_scatter");
    hipLaunchKernelGGL(k_p2_scatter, dim3((uint32_t)bp.g2), dim3(kPThreads), 0, ctx->stream, a2);
  }
  BucketArgs ba{};
  ba.pairs = a2.out;
  ba.bounds = (uint64_t*)ws_at(ctx, bp.oBB);
  ba.mwords = mwords;
  ba.nwords = nwords;
  ba.rec_new = d_rec_new;
  ba.nspill = (uint32_t*)ws_at(ctx, bp.oSP);
  ba.spill = ba.nspill + 1;
  SG_HIP(hipMemsetAsync(ba.nspill, 0, 4, ctx->stream));
  {
    ScopedTimer tm(ctx, "bucket_bounds");
    hipLaunchKernelGGL(k_bucket_bounds, dim3(div_up((uint64_t)kNumBuckets + 1, 256)), dim3(256), 0, ctx->stream,
                       a2.goff, a2.tb, bp.nslots, (uint64_t*)ba.bounds);
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
