// sg_triage.hip -- the first-owner family: batched new-signal triage and its
// relatives, all reproducing a sequential loop over items exactly.
//
// Reference loops (every one only ever skips an item whose elements are all
// already in the running set, so the running set before item k is
// S0 ∪ ⋃_{j<k} items_j; SURVEY.md §0 finding 1):
//   syz-fuzzer/fuzzer.go:645-693   execute() new-signal check      -> sg_triage_batch
//   syz-fuzzer/fuzzer.go:467-489   addInput()                      -> sg_add_inputs
//   syz-manager/manager.go:907-912 NewInput() acceptance           -> sg_accept_batch
//   syz-manager/manager.go:949-956 Poll() maxSignal merge          -> sg_merge_poll
//   pkg/cover/cover.go:120-146     Minimize()                      -> sg_minimize
//   pkg/cover/cover.go:169-176     SignalDiff()                    -> sg_set_diff
//
// Parallel form: owner(s) = min{key(item) : s ∈ item, s ∉ S0}.  Item k is
// "new" iff some element s ∉ S0 has owner(s) == key(k); its diff is exactly
// those elements, in item order with duplicates.  The triage-shaped loops
// (A8 with its diff lists, A11, A12) take the owners from the partitioned
// path's bucket stage (sg_bucket.hip) and emit the ordered lists from them
// here (owned_outputs); Minimize keeps a direct-indexed owner table (2^32 x
// u32, 16 GiB) whose keys decrease from call to call (sg::owner_keys), so it
// never needs resetting.
#include "sg_internal.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace sg {

__device__ __forceinline__ void load4(const uint32_t* __restrict__ v, uint64_t n, uint64_t e0, int aligned,
                                      uint32_t (&x)[4], uint32_t& okbits) {
  if (aligned && e0 + 4 <= n) {
    uint4 q = *reinterpret_cast<const uint4*>(v + e0);
    x[0] = q.x;
    x[1] = q.y;
    x[2] = q.z;
    x[3] = q.w;
    okbits = 0xF;
  } else {
    okbits = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      bool ok = e0 + k < n;
      x[k] = ok ? v[e0 + k] : 0u;
      okbits |= (ok ? 1u : 0u) << k;
    }
  }
}

__device__ __forceinline__ void store_ballots(uint64_t* mask, uint64_t c, int lane, uint32_t bits4) {
  uint64_t b0 = __ballot(bits4 & 1u);
  uint64_t b1 = __ballot(bits4 & 2u);
  uint64_t b2 = __ballot(bits4 & 4u);
  uint64_t b3 = __ballot(bits4 & 8u);
  uint64_t mine = lane == 0 ? b0 : lane == 1 ? b1 : lane == 2 ? b2 : b3;
  if (lane < 4) mask[c * 4 + lane] = mine;
}

// ---- ordered outputs from the partitioned path ------------------------------
// The bucket stage in its update-emitting form (sg_bucket.hip) writes every
// new signal s of a record slice once, with its first record r, as the key
// r << 32 | s; sorted by record (a stable LSD radix over the record bits),
// record r's keys are O_r, the signals it owns.  Its diff is S_r's elements
// that lie in O_r, in S_r order with duplicates (cover.go:169-176), or with
// `dedup` only the first occurrence of each (the Poll merge's element loop,
// manager.go:949-956).  One wave per record holds O_r as an LDS hash set and
// sweeps S_r by 256-element chunks, lane l testing elements 4l .. 4l + 3, so
// its four ballots are the chunk's words of the batch's diff mask; the ordered
// compaction below (k_scatter, k_seg_offsets) turns the mask into the CSR.  A
// record owning more than kOwnWave signals is listed for k_own_big (a
// workgroup per record, O_r in pieces of kOwnBigCap).
constexpr int kOwnWaves = 4;
constexpr uint32_t kOwnSlots = 2048;          // hash slots per wave: 512 buckets of 4
constexpr uint32_t kOwnWave = kOwnSlots / 4;  // the largest O_r of the wave path (load <= 1/4)
constexpr int kOwnBigT = 1024;
constexpr uint32_t kOwnBigSlots = 16384;
constexpr uint32_t kOwnBigCap = kOwnBigSlots / 4;
constexpr uint32_t kOwnEmpty = 0xFFFFFFFFu;  // an empty slot (the signal 0xFFFFFFFF is held by a flag)

struct OwnArgs {
  const uint32_t* vals;  // the batch (element e at vals[e])
  const uint64_t* roff;  // the slice's record offsets, rebased: record r = elements e0 + roff[r] ..
  uint64_t e0;
  uint32_t nrec;         // records in the slice
  const uint64_t* keys;  // r << 32 | s, sorted by record within each record group
  const uint2* po;       // record r's keys are [po[r].x, po[r].y)
  uint8_t* rec_new;      // the slice's record flags (nullable)
  uint64_t* mask;        // the batch's diff ballots, zeroed: 4 words per chunk
  uint32_t* big;         // [0]: count, then the records left for k_own_big
  uint64_t n;            // elements in the batch (vals[0 .. n) readable)
  uint32_t* ticket;      // k_own_pipe's next block of 64 records (zeroed)
};

// The set: 1 << bb buckets of four slots, a key in the first bucket from its
// home with a free slot (a bucket's slots fill in order, so a lookup reads one
// 16-B bucket and stops at the first one not full; at load <= 1/4 nearly
// every lookup is that one read).
__device__ __forceinline__ uint32_t own_home(uint32_t s, uint32_t bb) { return (s * 0x9E3779B1u) >> (32 - bb); }

__device__ __forceinline__ void own_insert(uint32_t* ht, uint32_t bb, uint32_t s) {
  const uint32_t m = (1u << bb) - 1;
  for (uint32_t b = own_home(s, bb);; b = (b + 1) & m)
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (atomicCAS(&ht[4 * b + j], kOwnEmpty, s) == kOwnEmpty) return;
}

// Membership of the lane's four values: the four home buckets read together,
// straight-line (a bucket holds s iff the min of its slots XOR s is 0); the
// rare value whose home bucket is full and does not hold it probes on in a
// loop the wave enters only then.  kSlot: also each hit's slot (4 << bb for
// the 0xFFFFFFFF signal, held by has_ff).
__device__ __forceinline__ bool own_has(const uint4& v, uint32_t s) {
  return min(min(v.x ^ s, v.y ^ s), min(v.z ^ s, v.w ^ s)) == 0u;
}
__device__ __forceinline__ uint32_t own_slot(const uint4& v, uint32_t s, uint32_t b) {
  return 4 * b + (v.x == s ? 0u : v.y == s ? 1u : v.z == s ? 2u : 3u);
}

template <bool kSlot>
__device__ __forceinline__ uint32_t own_probe(const uint32_t* ht, uint32_t bb, bool has_ff, const uint32_t (&x)[4],
                                              uint32_t (&slot)[4]) {
  const uint32_t m = (1u << bb) - 1;
  uint32_t h[4];
  uint4 v[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    h[k] = own_home(x[k], bb);
    v[k] = reinterpret_cast<const uint4*>(ht)[h[k]];
  }
  uint32_t hit = 0, more = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const bool ff = x[k] == kOwnEmpty;  // (equal to every empty slot: never stored)
    const bool any = own_has(v[k], x[k]);
    if (kSlot) slot[k] = ff ? (4u << bb) : own_slot(v[k], x[k], h[k]);
    hit |= ((ff ? has_ff : any) ? 1u : 0u) << k;
    more |= (!ff && !any && v[k].w != kOwnEmpty ? 1u : 0u) << k;
  }
  if (__builtin_expect(__ballot(more != 0) != 0, 0)) {
#pragma unroll
    for (int k = 0; k < 4; k++)
      if ((more >> k) & 1u)
        for (uint32_t b = (h[k] + 1) & m;; b = (b + 1) & m) {
          const uint4 w = reinterpret_cast<const uint4*>(ht)[b];
          if (own_has(w, x[k])) {
            hit |= 1u << k;
            if (kSlot) slot[k] = own_slot(w, x[k], b);
            break;
          }
          if (w.w == kOwnEmpty) break;
        }
  }
  return hit;
}

// The lane's four values of chunk c (a chunk inside the batch is loaded whole
// whatever the record bounds: one 16-B load, or four 4-B loads when vals is
// not 16-B aligned; only the batch's last, partial chunk takes guarded loads).
template <bool kAligned>
__device__ __forceinline__ void own_load(const OwnArgs& a, uint64_t c, int lane, uint32_t (&x)[4]) {
  const uint64_t p = c * kChunk + 4 * (uint64_t)lane;
  if ((c + 1) * kChunk <= a.n) {
    if (kAligned) {
      const uint4 q = *reinterpret_cast<const uint4*>(a.vals + p);
      x[0] = q.x;
      x[1] = q.y;
      x[2] = q.z;
      x[3] = q.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++) x[k] = a.vals[p + k];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++) x[k] = p + k < a.n ? a.vals[p + k] : 0u;
  }
}

// the chunk's four ballots into the mask (lane 0 writes all four; none when
// all are 0): stored where the chunk lies inside one record (this wave its
// only writer), OR-ed where it is shared
__device__ __forceinline__ void own_store(uint64_t* mask, uint64_t c, int lane, uint32_t bits4, bool shared) {
  const uint64_t b0 = __ballot(bits4 & 1u), b1 = __ballot(bits4 & 2u), b2 = __ballot(bits4 & 4u),
                 b3 = __ballot(bits4 & 8u);
  if ((b0 | b1 | b2 | b3) == 0) return;
  if (lane == 0) {
    unsigned long long* p = reinterpret_cast<unsigned long long*>(mask + c * 4);
    if (shared) {
      if (b0) atomicOr(p, (unsigned long long)b0);
      if (b1) atomicOr(p + 1, (unsigned long long)b1);
      if (b2) atomicOr(p + 2, (unsigned long long)b2);
      if (b3) atomicOr(p + 3, (unsigned long long)b3);
    } else {
      reinterpret_cast<ulonglong2*>(p)[0] = make_ulonglong2(b0, b1);
      reinterpret_cast<ulonglong2*>(p)[1] = make_ulonglong2(b2, b3);
    }
  }
}

// One chunk of record [lo, hi) (wave-uniform).  pass 0 (dedup): each
// member's first position per slot; pass 1: the ballots (always OR-ed with
// kOr: a record swept once per piece of O_r).
template <bool kDedup, int kPass>
__device__ __forceinline__ uint32_t own_hits(const uint32_t* ht, uint32_t* pm, uint32_t bb, bool has_ff, int lane,
                                             uint64_t lo, uint64_t hi, uint64_t c, const uint32_t (&x)[4]) {
  const uint64_t cs = c * kChunk;
  const bool inner = cs >= lo && cs + kChunk <= hi;
  uint32_t ok = 0xFu;
  if (!inner) {
    const int32_t l = lo > cs ? (int32_t)(lo - cs) : 0, h = hi - cs < (uint64_t)kChunk ? (int32_t)(hi - cs) : kChunk;
    ok = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int32_t qv = 4 * lane + k;
      ok |= (qv >= l && qv < h ? 1u : 0u) << k;
    }
  }
  uint32_t slot[4];
  uint32_t hit = own_probe<kDedup>(ht, bb, has_ff, x, slot) & ok;
  if (kDedup) {
    const uint32_t cr = (uint32_t)(cs - lo);  // (record positions fit 32 bits; wraps before the record)
#pragma unroll
    for (int k = 0; k < 4; k++)
      if ((hit >> k) & 1u) {
        const uint32_t pos = cr + 4 * lane + k;
        if (kPass == 0)
          atomicMin(&pm[slot[k]], pos);
        else if (pm[slot[k]] != pos)
          hit &= ~(1u << k);
      }
  }
  return hit;
}

__device__ __forceinline__ bool own_inner(uint64_t lo, uint64_t hi, uint64_t c) {
  return c * kChunk >= lo && (c + 1) * kChunk <= hi;
}

// One chunk of record [lo, hi) (wave-uniform).  pass 0 (dedup): each
// member's first position per slot; pass 1: the ballots (always OR-ed with
// kOr: a record swept once per piece of O_r).
template <bool kDedup, int kPass, bool kOr>
__device__ __forceinline__ void own_chunk(const OwnArgs& a, const uint32_t* ht, uint32_t* pm, uint32_t bb, bool has_ff,
                                          int lane, uint64_t lo, uint64_t hi, uint64_t c, const uint32_t (&x)[4]) {
  const uint32_t hit = own_hits<kDedup, kPass>(ht, pm, bb, has_ff, lane, lo, hi, c, x);
  if (kPass == 1) own_store(a.mask, c, lane, hit, kOr || !own_inner(lo, hi, c));
}

// A wave's LDS operations take effect in order; this only keeps the compiler
// from moving them across (a fence would also wait for the wave's global
// loads and stores in flight).
__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

constexpr int kOwnKB = 8;  // keys per lane loaded together
constexpr int kOwnCB = 5;  // chunks loaded together (a 1024-entry record spans <= 5)

template <bool kAligned, bool kDedup, int kPass, bool kOr = false>
__device__ __forceinline__ void own_sweep(const OwnArgs& a, const uint32_t* ht, uint32_t* pm, uint32_t bb, bool has_ff,
                                          int lane, uint64_t lo, uint64_t hi, uint64_t c0, uint64_t c1) {
  for (uint64_t cb = c0; cb <= c1; cb += kOwnCB) {
    uint32_t x[kOwnCB][4];
#pragma unroll
    for (int j = 0; j < kOwnCB; j++)
      if (cb + j <= c1) own_load<kAligned>(a, cb + j, lane, x[j]);
#pragma unroll
    for (int j = 0; j < kOwnCB; j++)
      if (cb + j <= c1) own_chunk<kDedup, kPass, kOr>(a, ht, pm, bb, has_ff, lane, lo, hi, cb + j, x[j]);
  }
}

__device__ __forceinline__ uint32_t uni32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) | __builtin_amdgcn_readfirstlane((uint32_t)v);
}

template <bool kAligned, bool kDedup>
__global__ __launch_bounds__(kOwnWaves * 64) void k_own_wave(OwnArgs a) {
  __shared__ alignas(16) uint32_t hts[kOwnWaves][kOwnSlots];
  __shared__ uint32_t pms[kDedup ? kOwnWaves : 1][kDedup ? kOwnSlots + 1 : 1];  // first position per slot
  static_assert(kOwnWave <= 64 * kOwnKB, "a wave-path record's keys: one batch");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t* ht = hts[w];
  uint32_t* pm = pms[kDedup ? w : 0];
  const uint32_t stride = gridDim.x * kOwnWaves;
  uint32_t r = blockIdx.x * kOwnWaves + w;
  // the next record's keys range and element range, loaded a record ahead
  uint2 q = make_uint2(0, 0);
  uint64_t lo = 0, hi = 0;
  if (r < a.nrec) {
    q = a.po[r];
    lo = a.roff[r];
    hi = a.roff[r + 1];
  }
  for (; r < a.nrec; r += stride) {
    // (wave-uniform: in scalar registers, so every branch on them is a scalar one)
    const uint32_t p0 = uni32(q.x), np = uni32(q.y) - p0;
    const uint64_t elo = a.e0 + uni64(lo), ehi = a.e0 + uni64(hi);
    if (r + stride < a.nrec) {
      q = a.po[r + stride];
      lo = a.roff[r + stride];
      hi = a.roff[r + stride + 1];
    }
    if (a.rec_new && lane == 0) a.rec_new[r] = np ? 1 : 0;  // queued iff it owns a signal (fuzzer.go:678-690)
    if (!np) continue;
    if (np > kOwnWave) {
      if (lane == 0) a.big[1 + atomicAdd(a.big, 1u)] = r;
      continue;
    }
    // the keys and the first chunks in flight together, the set cleared meanwhile
    uint32_t kv[kOwnKB];
#pragma unroll
    for (int j = 0; j < kOwnKB; j++) {
      const uint32_t i = j * 64 + lane;
      if (j * 64 < np) kv[j] = i < np ? (uint32_t)a.keys[p0 + i] : 0u;
    }
    const uint64_t c0 = elo / kChunk, c1 = (ehi - 1) / kChunk;  // (a record owning a signal has elements)
    uint32_t x[kOwnCB][4];
    if (!kDedup) {
#pragma unroll
      for (int j = 0; j < kOwnCB; j++)
        if (c0 + j <= c1) own_load<kAligned>(a, c0 + j, lane, x[j]);
    }
    uint32_t bb = 4;  // buckets: >= np (load <= 1/4)
    while ((1u << bb) < np) bb++;
    const uint32_t size = 4u << bb;
    for (uint32_t i = 4 * lane; i < size; i += 256)
      *reinterpret_cast<uint4*>(ht + i) = make_uint4(kOwnEmpty, kOwnEmpty, kOwnEmpty, kOwnEmpty);
    if (kDedup)
      for (uint32_t i = lane; i <= size; i += 64) pm[i] = kOwnEmpty;
    wave_sync();
    bool ff = false;
#pragma unroll
    for (int j = 0; j < kOwnKB; j++) {
      if (j * 64 >= np) break;
      if (j * 64 + lane >= np) continue;
      if (kv[j] == kOwnEmpty)
        ff = true;
      else
        own_insert(ht, bb, kv[j]);
    }
    const bool has_ff = __ballot(ff) != 0;
    wave_sync();
    if (kDedup) {
      own_sweep<kAligned, true, 0>(a, ht, pm, bb, has_ff, lane, elo, ehi, c0, c1);
      wave_sync();
      own_sweep<kAligned, true, 1>(a, ht, pm, bb, has_ff, lane, elo, ehi, c0, c1);
    } else {  // the first batch was loaded with the keys
#pragma unroll
      for (int j = 0; j < kOwnCB; j++)
        if (c0 + j <= c1) own_chunk<false, 1, false>(a, ht, pm, bb, has_ff, lane, elo, ehi, c0 + j, x[j]);
      if (c0 + kOwnCB <= c1) own_sweep<kAligned, false, 1>(a, ht, pm, bb, has_ff, lane, elo, ehi, c0 + kOwnCB, c1);
    }
    wave_sync();  // (the set is cleared for the next record)
  }
}

// The flags-and-diff sweep (no dedup).  A wave takes 64 consecutive records
// at a time: their keys ranges and element ranges come in one coalesced load
// (a lane per record) and their flags go out as one 64-byte store.  The
// records of the block it decides here (owning 1 .. kOwnWave signals, spanning
// <= kOwnCB chunks, not the batch's partial last chunk; the rest are listed for
// k_own_big) are software-pipelined: the next record's keys and chunks are
// loaded before this record is decided, and every record issues the same
// memory instructions (kOwnKB + kOwnCB loads, clamped to readable addresses
// when unused; one 64-lane atomic OR of its mask words), so the compiler's
// wait for a record's loads leaves the next record's loads and the previous
// record's OR in flight.
__device__ __forceinline__ uint32_t lane_get(uint32_t v, int i) { return __builtin_amdgcn_readlane(v, i); }
__device__ __forceinline__ uint64_t lane_get(uint64_t v, int i) {
  return ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), i) << 32) | __builtin_amdgcn_readlane((uint32_t)v, i);
}

struct OwnSet {
  uint32_t kv[kOwnKB];
  uint32_t x[kOwnCB][4];
};

template <bool kAligned>
__device__ __forceinline__ void own_fetch(const OwnArgs& a, int lane, uint32_t p0, uint32_t np, uint64_t c0,
                                          uint64_t c1, OwnSet& d) {
#pragma unroll
  for (int j = 0; j < kOwnKB; j++) d.kv[j] = (uint32_t)a.keys[p0 + min((uint32_t)(j * 64 + lane), np - 1)];
#pragma unroll
  for (int j = 0; j < kOwnCB; j++) {
    const uint64_t p = min(c0 + j, c1) * kChunk + 4 * (uint64_t)lane;
    if (kAligned) {
      const uint4 q = *reinterpret_cast<const uint4*>(a.vals + p);
      d.x[j][0] = q.x;
      d.x[j][1] = q.y;
      d.x[j][2] = q.z;
      d.x[j][3] = q.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++) d.x[j][k] = a.vals[p + k];
    }
  }
}

template <bool kAligned>
__global__ __launch_bounds__(kOwnWaves * 64) __attribute__((amdgpu_waves_per_eu(4))) void k_own_pipe(OwnArgs a) {
  __shared__ alignas(16) uint32_t hts[kOwnWaves][kOwnSlots];
  __shared__ alignas(16) uint32_t hcs[kOwnWaves][kOwnSlots / 4];  // keys per bucket
  static_assert(kOwnWave <= 64 * kOwnKB, "a wave-path record's keys: one batch");
  static_assert(4 * kOwnCB <= 64, "a record's mask words: one per lane");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t* ht = hts[w];
  uint32_t* hc = hcs[w];
  const uint32_t nblk = (a.nrec + 63) / 64;
  const uint64_t nfull = a.n / kChunk;  // chunks wholly inside the batch
  // blocks by ticket (records own very different amounts of work)
  for (uint32_t blk = uni32(lane == 0 ? atomicAdd(a.ticket, 1u) : 0u); blk < nblk;
       blk = uni32(lane == 0 ? atomicAdd(a.ticket, 1u) : 0u)) {
    const uint32_t R0 = blk * 64, nb = min(64u, a.nrec - R0);
    uint2 gq = make_uint2(0, 0);
    uint64_t glo = 0, ghi = 0;
    if ((uint32_t)lane < nb) {
      gq = a.po[R0 + lane];
      glo = a.e0 + a.roff[R0 + lane];
      ghi = a.e0 + a.roff[R0 + lane + 1];
    }
    const uint32_t gnp = gq.y - gq.x;
    if (a.rec_new && (uint32_t)lane < nb) a.rec_new[R0 + lane] = gnp ? 1 : 0;  // queued iff it owns a signal (fuzzer.go:678-690)
    const uint64_t gc0 = glo / kChunk, gc1 = gnp ? (ghi - 1) / kChunk : gc0;
    const bool mine = gnp && gnp <= kOwnWave && gc1 - gc0 < (uint64_t)kOwnCB && gc1 < nfull;
    if (gnp && !mine) a.big[1 + atomicAdd(a.big, 1u)] = R0 + lane;
    uint64_t vm = __ballot(mine);
    if (!vm) continue;
    int i = __builtin_ctzll(vm);
    vm &= vm - 1;
    OwnSet A, B;
    own_fetch<kAligned>(a, lane, lane_get(gq.x, i), lane_get(gnp, i), lane_get(gc0, i), lane_get(gc1, i), A);
    for (;;) {
      const bool more = vm != 0;
      const int in = more ? __builtin_ctzll(vm) : i;  // (no next record: this one's loads again)
      vm &= vm - 1;
      own_fetch<kAligned>(a, lane, lane_get(gq.x, in), lane_get(gnp, in), lane_get(gc0, in), lane_get(gc1, in), B);
      // decide record i from A
      const uint32_t np = lane_get(gnp, i);
      const uint64_t elo = lane_get(glo, i), ehi = lane_get(ghi, i), c0 = lane_get(gc0, i), c1 = lane_get(gc1, i);
      uint32_t bb = 4;  // buckets: >= np (load <= 1/4)
      while ((1u << bb) < np) bb++;
      const uint32_t size = 4u << bb;
      for (uint32_t t = 4 * lane; t < size; t += 256)
        *reinterpret_cast<uint4*>(ht + t) = make_uint4(kOwnEmpty, kOwnEmpty, kOwnEmpty, kOwnEmpty);
      for (uint32_t t = 4 * lane; t < (1u << bb); t += 256) *reinterpret_cast<uint4*>(hc + t) = make_uint4(0, 0, 0, 0);
      wave_sync();
      // inserts by counting: a key takes the next slot of its home bucket
      // (one LDS round trip, no compare-and-swap retries), the next bucket's
      // when it is full -- the buckets still fill in slot order
      bool ff = false;
#pragma unroll
      for (int j = 0; j < kOwnKB; j++) {
        if (j * 64 >= np) break;
        if (j * 64 + lane >= np) continue;
        if (A.kv[j] == kOwnEmpty) {
          ff = true;
        } else {
          const uint32_t m = (1u << bb) - 1;
          for (uint32_t b = own_home(A.kv[j], bb);; b = (b + 1) & m) {
            const uint32_t at = atomicAdd(&hc[b], 1u);
            if (at < 4) {
              ht[4 * b + at] = A.kv[j];
              break;
            }
          }
        }
      }
      const bool has_ff = __ballot(ff) != 0;
      wave_sync();
      // lane 4 j + k ORs word k of chunk c0 + j (past c1: 0 into chunk c1)
      uint64_t word = 0;
#pragma unroll
      for (int j = 0; j < kOwnCB; j++)
        if (c0 + j <= c1) {
          const uint32_t hit = own_hits<false, 1>(ht, nullptr, bb, has_ff, lane, elo, ehi, c0 + j, A.x[j]);
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const uint64_t bk = __ballot((hit >> k) & 1u);
            word = lane == 4 * j + k ? bk : word;
          }
        }
      const uint64_t cj = min(c0 + (uint64_t)(lane >> 2), c1);
      atomicOr(reinterpret_cast<unsigned long long*>(a.mask + cj * 4 + (lane & 3)),
               (unsigned long long)(lane < 4 * kOwnCB ? word : 0ull));
      wave_sync();  // (the set is cleared for the next record)
      if (!more) break;
      A = B;
      i = in;
    }
  }
}

// Records owning more than kOwnWave signals: a workgroup each, O_r in pieces
// of kOwnBigCap signals, each piece a sweep of S_r (two with dedup) whose
// ballots are OR-ed into the mask.
template <bool kAligned, bool kDedup>
__global__ __launch_bounds__(kOwnBigT) void k_own_big(OwnArgs a) {
  __shared__ alignas(16) uint32_t ht[kOwnBigSlots];
  __shared__ uint32_t pm[kDedup ? kOwnBigSlots + 1 : 1];
  __shared__ uint32_t sh_ff;
  constexpr int kW = kOwnBigT / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t nbig = a.big[0];
  for (uint32_t j = blockIdx.x; j < nbig; j += gridDim.x) {
    const uint32_t r = uni32(a.big[1 + j]);
    const uint2 q = make_uint2(uni32(a.po[r].x), uni32(a.po[r].y));
    const uint64_t lo = a.e0 + uni64(a.roff[r]), hi = a.e0 + uni64(a.roff[r + 1]);
    const uint64_t c0 = lo / kChunk, c1 = (hi - 1) / kChunk;
    for (uint32_t q0 = q.x; q0 < q.y; q0 += kOwnBigCap) {
      const uint32_t q1 = min(q.y, q0 + kOwnBigCap);
      uint32_t bb = 4;  // buckets: >= the piece's keys
      while ((1u << bb) < q1 - q0) bb++;
      const uint32_t size = 4u << bb;
      for (uint32_t i = tid; i < size; i += kOwnBigT) ht[i] = kOwnEmpty;
      if (kDedup)
        for (uint32_t i = tid; i <= size; i += kOwnBigT) pm[i] = kOwnEmpty;
      if (tid == 0) sh_ff = 0;
      __syncthreads();
      for (uint32_t i = q0 + tid; i < q1; i += kOwnBigT) {
        const uint32_t sv = (uint32_t)a.keys[i];
        if (sv == kOwnEmpty)
          sh_ff = 1;
        else
          own_insert(ht, bb, sv);
      }
      __syncthreads();
      const bool has_ff = sh_ff != 0;
      // the waves take chunk batches kW apart: wave w's chunks c0 + kOwnCB (w + kW i) ..
      for (uint64_t cb = c0 + (uint64_t)w * kOwnCB; kDedup && cb <= c1; cb += (uint64_t)kW * kOwnCB)
        own_sweep<kAligned, true, 0>(a, ht, pm, bb, has_ff, lane, lo, hi, cb, min(c1, cb + kOwnCB - 1));
      if (kDedup) __syncthreads();
      for (uint64_t cb = c0 + (uint64_t)w * kOwnCB; cb <= c1; cb += (uint64_t)kW * kOwnCB)
        own_sweep<kAligned, kDedup, 1, true>(a, ht, pm, bb, has_ff, lane, lo, hi, cb, min(c1, cb + kOwnCB - 1));
      __syncthreads();
    }
  }
}

// [po[r].x, po[r].y): record r's keys.  The sorted keys are ordered by
// (record & 0xFFFF, record >> 16) -- two 8-bit passes over the low 16 bits
// of group-major pairs -- so a thread per record finds the first and
// one-past-last positions of its composite rank with two interleaved binary
// searches (every record written, no memset).  (r05: 0.31 ms per C2 batch
// against 0.40 for a coalesced pass over all 208M keys comparing neighbours.)
__device__ __forceinline__ uint32_t own_rank(uint32_t rec) { return (rec << 16) | (rec >> 16); }

__global__ __launch_bounds__(256) void k_own_bounds_search(const uint64_t* __restrict__ k, uint64_t n, uint32_t nr,
                                                           uint2* __restrict__ po) {
  const uint32_t r = blockIdx.x * 256 + threadIdx.x;
  if (r >= nr) return;
  const uint32_t t = own_rank(r);
  uint64_t lo0 = 0, hi0 = n, lo1 = 0, hi1 = n;  // first rank >= t, first rank > t
  while (lo0 < hi0 || lo1 < hi1) {
    const uint64_t m0 = (lo0 + hi0) >> 1, m1 = (lo1 + hi1) >> 1;
    const uint32_t c0 = lo0 < hi0 ? own_rank((uint32_t)(k[m0] >> 32)) : 0u;
    const uint32_t c1 = lo1 < hi1 ? own_rank((uint32_t)(k[m1] >> 32)) : 0u;
    if (lo0 < hi0) {
      if (c0 < t)
        lo0 = m0 + 1;
      else
        hi0 = m0;
    }
    if (lo1 < hi1) {
      if (c1 <= t)
        lo1 = m1 + 1;
      else
        hi1 = m1;
    }
  }
  po[r] = make_uint2((uint32_t)lo0, (uint32_t)lo1);
}

// gs[g] = roff[g << 16] (g < ng): where group g's pairs start
__global__ void k_group_starts(const uint64_t* __restrict__ roff, uint32_t ng, uint64_t* __restrict__ gs) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < ng) gs[g] = roff[(uint64_t)g << kRecGroupBits];
}

// diff elements per chunk, from its ballots
__global__ void k_mask_count(const uint64_t* __restrict__ mask, uint64_t nchunks, uint32_t* __restrict__ cnt) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks) return;
  const ulonglong2 u = reinterpret_cast<const ulonglong2*>(mask)[2 * c];
  const ulonglong2 v = reinterpret_cast<const ulonglong2*>(mask)[2 * c + 1];
  cnt[c] = __popcll(u.x) + __popcll(u.y) + __popcll(v.x) + __popcll(v.y);
}

// ---- ordered compaction by ballot masks --------------------------------------
// Position of value 4l+k of a chunk among the chunk's masked values.
__device__ __forceinline__ uint32_t rank_in_chunk(const uint64_t m[4], int lane, int k) {
  uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t r = __popcll(m[0] & lt) + __popcll(m[1] & lt) + __popcll(m[2] & lt) + __popcll(m[3] & lt);
  for (int q = 0; q < k; q++) r += (uint32_t)((m[q] >> lane) & 1ull);
  return r;
}

// Masked values written in order: out[chunk_base[c] + rank].
__global__ __launch_bounds__(kBlock) void k_scatter(const uint32_t* __restrict__ vals, uint64_t n, int aligned,
                                                    const uint64_t* __restrict__ mask, const uint64_t* __restrict__ base,
                                                    uint64_t nchunks, uint32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  uint64_t c = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  uint64_t m[4] = {mask[c * 4], mask[c * 4 + 1], mask[c * 4 + 2], mask[c * 4 + 3]};
  if (!(m[0] | m[1] | m[2] | m[3])) return;
  uint32_t mine = 0;
  for (int k = 0; k < 4; k++) mine |= (uint32_t)((m[k] >> lane) & 1ull) << k;
  if (!mine) return;
  uint64_t e0 = c * kChunk + lane * 4;
  uint32_t x[4], ok;
  load4(vals, n, e0, aligned, x, ok);
  uint64_t b = base[c];
  for (int k = 0; k < 4; k++)
    if ((mine >> k) & 1u) out[b + rank_in_chunk(m, lane, k)] = x[k];
}

// Output offset of each segment: number of masked values before off[r].
__global__ void k_seg_offsets(const uint64_t* __restrict__ off, uint64_t nseg, uint64_t n,
                              const uint64_t* __restrict__ mask, const uint64_t* __restrict__ base, uint64_t nchunks,
                              uint64_t* __restrict__ out_off) {
  uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > nseg) return;
  uint64_t p = off ? off[r] : r;
  uint64_t c = p / kChunk;
  if (c >= nchunks) {
    out_off[r] = base[nchunks];
    return;
  }
  uint32_t q = (uint32_t)(p % kChunk);
  uint64_t acc = base[c];
  for (int k = 0; k < 4; k++) {
    int lim = q > (uint32_t)k ? (int)((q - k + 3) / 4) : 0;  // lanes l with 4l+k < q
    uint64_t lm = lim >= 64 ? ~0ull : ((1ull << lim) - 1);
    acc += __popcll(mask[c * 4 + k] & lm);
  }
  out_off[r] = acc;
}

// Predicate masks (no owner table): value not in `set` [SignalDiff].
template <class Pred>
__global__ __launch_bounds__(kBlock) void k_mask(const uint32_t* __restrict__ vals, uint64_t n, int aligned, Pred pred,
                                                 uint64_t nchunks, uint64_t* __restrict__ mask,
                                                 uint32_t* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  uint64_t c = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  uint64_t e0 = c * kChunk + lane * 4;
  uint32_t x[4], ok;
  load4(vals, n, e0, aligned, x, ok);
  uint32_t bits = 0;
  for (int k = 0; k < 4; k++)
    if (((ok >> k) & 1u) && pred(e0 + k, x[k])) bits |= 1u << k;
  store_ballots(mask, c, lane, bits);
  uint32_t cc = __popcll(__ballot(bits & 1u)) + __popcll(__ballot(bits & 2u)) + __popcll(__ballot(bits & 4u)) +
                __popcll(__ballot(bits & 8u));
  if (lane == 0) cnt[c] = cc;
}

struct NotIn {
  const uint32_t* words;
  __device__ bool operator()(uint64_t, uint32_t v) const { return !sgd::test_bit(words, v); }
};
struct FlagAt {  // keep element i iff flag[i]
  const uint8_t* flag;
  __device__ bool operator()(uint64_t i, uint32_t) const { return flag[i] != 0; }
};

// set bits of masked values into up to two sets (addInput)
__global__ __launch_bounds__(kBlock) void k_apply_mask(const uint32_t* __restrict__ vals, uint64_t n, int aligned,
                                                       const uint64_t* __restrict__ mask, uint64_t nchunks,
                                                       uint32_t* set_a, uint32_t* set_b) {
  const int lane = threadIdx.x & 63;
  uint64_t c = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  uint32_t mine = 0;
  for (int k = 0; k < 4; k++) mine |= (uint32_t)((mask[c * 4 + k] >> lane) & 1ull) << k;
  if (!mine) return;
  uint32_t x[4], ok;
  load4(vals, n, c * kChunk + lane * 4, aligned, x, ok);
  for (int k = 0; k < 4; k++)
    if ((mine >> k) & 1u) {
      if (set_a) sgd::set_bit(set_a, x[k]);
      if (set_b) sgd::set_bit(set_b, x[k]);
    }
}

// corpusCover ∪= Cov_k for accepted k (NewInput, manager.go:912)
__global__ __launch_bounds__(kBlock) void k_add_flagged_segs(const uint32_t* __restrict__ vals, uint64_t n,
                                                             const uint64_t* __restrict__ off, uint64_t nseg,
                                                             const uint8_t* __restrict__ flag, uint32_t* set) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t r = sgd::seg_search(off, 0, nseg - 1, i);
    if (flag[r]) sgd::set_bit(set, vals[i]);
  }
}

// ---- Minimize (cover.go:120-146) -----------------------------------------------
// One workgroup per input: its elements all carry its rank key, so there is
// no per-element item search.  Each element lowers owner[v] to the key
// (read-checked atomicMin: the smallest key -- the earliest input -- owns v).  An element
// that reads a key of an older generation (>= key_end: no element of this
// call has written v yet) also sets v's bit in the touched bitmap (2^32 bits,
// the set layout), so about one global atomicOr per distinct value: the
// first current-generation writer of v always sets it.  The owners are then
// flagged from the touched bitmap alone (k_min_owners, one read of 512 MiB)
// instead of re-reading the corpus.
// Workgroups run in processing order (block b = the input of rank b, key
// key_lo + b): the early ranks claim the corpus's common values first, so a
// later element's read-check mostly finds a smaller key and issues no atomic,
// and the longest inputs (sort.Sort puts them first, cover.go:157) start first.
__global__ __launch_bounds__(kBlock) void k_min_claim(const uint32_t* __restrict__ vals, const uint64_t* __restrict__ off,
                                                      const uint32_t* __restrict__ order, uint32_t key_lo,
                                                      uint32_t key_end, uint32_t* __restrict__ owner,
                                                      uint32_t* __restrict__ touched) {
  const uint64_t k = order[blockIdx.x];
  const uint64_t b = off[k], e = off[k + 1];
  const uint32_t key = key_lo + blockIdx.x;
  for (uint64_t i = b + threadIdx.x; i < e; i += kBlock) {
    const uint32_t v = vals[i];
    uint32_t* p = owner + v;
    const uint32_t o = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (o > key) {
      atomicMin(p, key);
      if (o >= key_end) sgd::set_bit(touched, v);
    }
  }
}

// flag[order[owner rank]] for every touched value (bit q of word w is signal
// set_sig(32 w + q))
__global__ void k_min_owners(const uint32_t* __restrict__ touched, const uint32_t* __restrict__ owner, uint32_t key_lo,
                             const uint32_t* __restrict__ order, uint8_t* __restrict__ flag) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w4 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w4 < kSetWords / 4; w4 += stride) {
    const uint4 q = reinterpret_cast<const uint4*>(touched)[w4];
    const uint32_t ws[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 4; j++)
      for (uint32_t m = ws[j]; m; m &= m - 1) {
        const uint32_t v = sgd::set_sig((uint32_t)((w4 * 4 + j) << 5) | (uint32_t)__builtin_ctz(m));
        flag[order[owner[v] - key_lo]] = 1;
      }
  }
}

// Filtered claim for the later ranks.  The values of the first R inputs in
// processing order (the longest ones, cover.go:157: they hold the corpus's
// common values) are owned by ranks < R, so a later element of one of them can
// never lower its owner: it is skipped without touching the owner table.  A
// subset of those values -- an open-addressing set of kFilt slots, each value
// at most kFiltProbe slots from its home (values that find no slot there are
// simply left out) -- is loaded into each persistent workgroup's LDS once; the
// elements of ranks >= R stream through in rank order (windows of the virtual
// concatenation, taken by ticket) and only the ones the set does not hold
// make the read-checked claim.  Exact for any subset the set holds.
constexpr uint32_t kFilt = 16384, kFiltProbe = 8, kFiltEmpty = 0xFFFFFFFFu;
// Phase A: the first R = kFiltRanks inputs in processing order, claimed one
// workgroup per input.  The filter's values: those of input 0 that inputs 1 ..
// R - 1 also hold -- the values common to the longest covers, i.e.
// the corpus's most common ones (a value one long cover holds is as likely
// rare).
constexpr uint32_t kFiltRanks = 4;
constexpr uint32_t kFirstSlots = 1u << 16;  // set of input 0's values (bounded probes: extras left out)
constexpr int kFT = 1024;              // persistent claim workgroup
constexpr uint32_t kFWin = 4 * kFT;    // elements per window
__device__ __forceinline__ uint32_t filt_home(uint32_t v) { return (v * 0x9E3779B1u) >> 18; }  // 14 bits
__device__ __forceinline__ uint32_t first_home(uint32_t v) { return (v * 0x85EBCA6Bu) >> 16; }  // 16 bits

__device__ __forceinline__ void set_insert(uint32_t* tab, uint32_t mask, uint32_t h, uint32_t v, uint32_t probes) {
  for (uint32_t d = 0; d < probes; d++) {
    uint32_t* slot = &tab[(h + d) & mask];
    const uint32_t cur = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == v) return;
    if (cur == kFiltEmpty) {
      const uint32_t old = atomicCAS(slot, kFiltEmpty, v);
      if (old == kFiltEmpty || old == v) return;
    }
  }
}

// input 0's values into the first-values set
__global__ __launch_bounds__(kBlock) void k_min_first(const uint32_t* __restrict__ vals,
                                                      const uint64_t* __restrict__ off,
                                                      const uint32_t* __restrict__ order, uint32_t* __restrict__ first) {
  const uint64_t k = order[0];
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = off[k] + (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < off[k + 1]; i += stride) {
    const uint32_t v = vals[i];
    if (v != kFiltEmpty) set_insert(first, kFirstSlots - 1, first_home(v), v, 16);  // (the empty marker: never filtered)
  }
}

// values of inputs 1 .. R - 1 (phase A) that the first-values set holds into the filter
__global__ __launch_bounds__(kBlock) void k_min_filter(const uint32_t* __restrict__ vals,
                                                       const uint64_t* __restrict__ off,
                                                       const uint32_t* __restrict__ order,
                                                       const uint32_t* __restrict__ first, uint32_t* __restrict__ filt) {
  const uint64_t k = order[1 + blockIdx.y];
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = off[k] + (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < off[k + 1]; i += stride) {
    const uint32_t v = vals[i];
    if (v == kFiltEmpty) continue;
    const uint32_t h = first_home(v);
    bool in = false;
    for (uint32_t d = 0; d < 16; d++) {
      const uint32_t c = first[(h + d) & (kFirstSlots - 1)];
      if (c == v) in = true;
      if (c == v || c == kFiltEmpty) break;
    }
    if (in) set_insert(filt, kFilt - 1, filt_home(v), v, kFiltProbe);
  }
}

// phase B's geometry: lengths and starts of ranks R.. (in processing order)
__global__ void k_min_ranks(const uint64_t* __restrict__ off, const uint32_t* __restrict__ order, uint64_t R,
                            uint64_t nr, uint32_t* __restrict__ lens, uint64_t* __restrict__ soff) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nr) return;
  const uint32_t k = order[R + j];
  soff[j] = off[k];
  lens[j] = (uint32_t)(off[k + 1] - off[k]);
}

// each window's first rank: last r with roff[r] <= w kFWin
__global__ void k_min_wrank(const uint64_t* __restrict__ roff, uint64_t nr, uint64_t nwin,
                            uint32_t* __restrict__ wrank) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nwin) return;
  const uint64_t p = w * kFWin;
  uint64_t lo = 0, hi = nr - 1;
  while (lo < hi) {
    const uint64_t mid = (lo + hi + 1) >> 1;
    if (roff[mid] <= p)
      lo = mid;
    else
      hi = mid - 1;
  }
  wrank[w] = (uint32_t)lo;
}

struct MinClaimF {
  const uint32_t* vals;
  const uint64_t* roff;   // [n - R + 1] element offsets of ranks R.. in the virtual concatenation
  const uint64_t* soff;   // [n - R] where rank R + j's elements start in vals
  uint64_t nr;            // ranks in this phase
  uint64_t nel;           // their elements
  uint32_t key0;          // key of rank R
  uint32_t key_end;
  uint32_t* owner;
  uint32_t* touched;
  const uint32_t* filt;
  const uint32_t* wrank;  // [windows] rank (relative to R) holding each window's first element
};

__global__ __launch_bounds__(kFT) void k_min_claim_f(MinClaimF a) {
  __shared__ uint32_t fs[kFilt];
  for (uint32_t i = threadIdx.x; i < kFilt; i += kFT) fs[i] = a.filt[i];
  __syncthreads();
  const uint64_t nwin = (a.nel + kFWin - 1) / kFWin;
  // windows blockIdx.x, + gridDim.x, ...: the grid sweeps them in rank order
  constexpr int kE = kFWin / kFT;  // elements per thread per window, loads in flight together
  for (uint64_t w = blockIdx.x; w < nwin; w += gridDim.x) {
    uint64_t r = a.wrank[w], rend = a.roff[r + 1];
    int64_t base = (int64_t)a.soff[r] - (int64_t)a.roff[r];  // vals index = base + position
    const uint64_t p0 = w * kFWin + threadIdx.x, p1 = min<uint64_t>((w + 1) * kFWin, a.nel);
    uint32_t v[kE], rk[kE];
#pragma unroll
    for (int e = 0; e < kE; e++) {
      const uint64_t p = p0 + (uint64_t)e * kFT;
      rk[e] = 0xFFFFFFFFu;
      if (p < p1) {
        while (rend <= p) {
          rend = a.roff[++r + 1];
          base = (int64_t)a.soff[r] - (int64_t)a.roff[r];
        }
        v[e] = a.vals[base + (int64_t)p];
        rk[e] = (uint32_t)r;
      }
    }
#pragma unroll
    for (int e = 0; e < kE; e++) {
      if (rk[e] == 0xFFFFFFFFu) continue;
      const uint32_t x = v[e];
      bool held = false;
      if (x != kFiltEmpty) {
        const uint32_t h = filt_home(x);
#pragma unroll
        for (uint32_t d = 0; d < kFiltProbe; d++) {
          const uint32_t c = fs[(h + d) & (kFilt - 1)];
          if (c == x) held = true;
          if (c == x || c == kFiltEmpty) break;
        }
      }
      if (held) continue;
      const uint32_t key = a.key0 + rk[e];
      uint32_t* q = a.owner + x;
      const uint32_t o = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (o > key) {
        atomicMin(q, key);
        if (o >= a.key_end) sgd::set_bit(a.touched, x);
      }
    }
  }
}

__global__ void k_invert_perm(const uint32_t* __restrict__ order, uint64_t n, uint32_t* __restrict__ rank) {
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) rank[order[k]] = (uint32_t)k;
}
__global__ void k_gather_flag(const uint32_t* __restrict__ order, uint64_t n, const uint8_t* __restrict__ flag,
                              uint8_t* __restrict__ out) {
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[k] = flag[order[k]];
}

// ---- host-side pipeline ------------------------------------------------------
struct Scratch {
  uint64_t ntiles = 0, nchunks = 0;
  uint64_t *cmask = nullptr, *dmask = nullptr, *base = nullptr;
  uint32_t *dcnt = nullptr, *tile_rec = nullptr;
};

static size_t scratch_plan(WsPlan& p, uint64_t n, size_t o[5]) {
  uint64_t ntiles = n ? (n + kTile - 1) / kTile : 0;
  uint64_t nchunks = ntiles * kChunksPerTile;
  o[0] = p.add(nchunks * 32);
  o[1] = p.add(nchunks * 32);
  o[2] = p.add(nchunks * 4);
  o[3] = p.add((nchunks + 1) * 8);
  o[4] = p.add((ntiles + 1) * 4);
  return scan_ws_bytes(nchunks);
}

static Scratch scratch_bind(sg_ctx* ctx, uint64_t n, const size_t o[5]) {
  Scratch s;
  s.ntiles = n ? (n + kTile - 1) / kTile : 0;
  s.nchunks = s.ntiles * kChunksPerTile;
  s.cmask = (uint64_t*)ws_at(ctx, o[0]);
  s.dmask = (uint64_t*)ws_at(ctx, o[1]);
  s.dcnt = (uint32_t*)ws_at(ctx, o[2]);
  s.base = (uint64_t*)ws_at(ctx, o[3]);
  s.tile_rec = (uint32_t*)ws_at(ctx, o[4]);
  return s;
}

// ordered emission of the masked values (+ per-segment offsets)
static int run_emit(sg_ctx* ctx, const uint32_t* vals, uint64_t n, const uint64_t* mask, const uint32_t* cnt,
                    const Scratch& s, size_t scan_ws_off, const uint64_t* off, uint64_t nseg, uint32_t* out_vals,
                    uint64_t* out_off) {
  int rc = scan_counts(ctx, cnt, s.base, s.nchunks, scan_ws_off);
  if (rc) return rc;
  ScopedTimer tm(ctx, "emit");
  int aligned = ((uintptr_t)vals & 15) == 0;
  if (out_vals && s.nchunks)
    hipLaunchKernelGGL(k_scatter, dim3(div_up(s.nchunks, kBlock / 64)), dim3(kBlock), 0, ctx->stream, vals, n,
                       aligned, mask, s.base, s.nchunks, out_vals);
  if (out_off)
    hipLaunchKernelGGL(k_seg_offsets, dim3(div_up(nseg + 1, 256)), dim3(256), 0, ctx->stream, off, nseg, n, mask,
                       s.base, s.nchunks, out_off);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

static size_t al256(size_t x) { return (x + 255) & ~size_t(255); }

// the per-record sweeps of one slice: the wave kernel over the resident grid
// (records every grid-th, or blocks of 64 by ticket), then the listed large
// records
template <bool kAligned>
static int launch_own(sg_ctx* ctx, const OwnArgs& oa, uint64_t nr, bool dedup) {
  const void* kw = dedup ? (const void*)k_own_wave<kAligned, true> : (const void*)k_own_pipe<kAligned>;
  const uint32_t wg = std::min<uint32_t>(div_up(nr, dedup ? kOwnWaves : 64 * kOwnWaves),
                                         persistent_grid(ctx, kw, kOwnWaves * 64));
  if (dedup) {
    hipLaunchKernelGGL((k_own_wave<kAligned, true>), dim3(wg), dim3(kOwnWaves * 64), 0, ctx->stream, oa);
    hipLaunchKernelGGL((k_own_big<kAligned, true>), dim3(512), dim3(kOwnBigT), 0, ctx->stream, oa);
  } else {
    hipLaunchKernelGGL((k_own_pipe<kAligned>), dim3(wg), dim3(kOwnWaves * 64), 0, ctx->stream, oa);
    hipLaunchKernelGGL((k_own_big<kAligned, false>), dim3(512), dim3(kOwnBigT), 0, ctx->stream, oa);
  }
  SG_HIP(hipGetLastError());
  return SG_OK;
}

// Ordered outputs of a first-owner loop over records (ctx lock held): flags
// (nullable), mwords / nwords (nullable) updated, the diff CSR (out_vals,
// out_off; either nullable).  Record slices as the flags path cuts them; per
// slice: partition + the update-emitting bucket stage, the pairs sorted by
// record, the per-record sweeps into the batch's diff mask; then one ordered
// compaction.  Workspace: the batch's masks, then one slice's region -- the
// partition's scratch, which the radix sort reuses as its second key buffer
// once the bucket stage is done, the pairs, the sort's counts and the
// per-record tables.
static int owned_outputs(sg_ctx* ctx, uint32_t* mwords, uint32_t* nwords, const uint32_t* d_vals,
                         const uint64_t* d_off, uint64_t nvals, uint64_t nrec, uint8_t* d_rec_new, uint32_t* d_out_vals,
                         uint64_t* d_out_off, bool dedup) {
  if (nrec >= 0xFFFFFFFFull || nvals >= 0xFFFFFFFFull - (1ull << 16)) {
    set_error("ordered triage: a batch holds < 2^32 signal entries and < 2^32 - 1 records");
    return SG_EINVAL;
  }
  if (nrec && d_rec_new) SG_HIP(hipMemsetAsync(d_rec_new, 0, nrec, ctx->stream));
  if (nvals == 0) {
    if (d_out_off) SG_HIP(hipMemsetAsync(d_out_off, 0, (nrec + 1) * 8, ctx->stream));
    return SG_OK;
  }
  if (nrec == 0) {
    set_error("ordered triage: signal entries without records");
    return SG_EINVAL;
  }
  std::vector<uint64_t> cuts;
  int rc = record_slice_cuts(ctx, d_off, nrec, 1ull << 30, cuts);
  if (rc) return rc;
  WsPlan p;
  size_t o[5];
  const size_t scan_b = scratch_plan(p, nvals, o);
  const size_t scan_off = p.total;
  const size_t S0 = al256(p.total + scan_b);
  size_t part = 0, tail = 0;
  for (size_t j = 0; j + 3 < cuts.size(); j += 4) {
    const uint64_t nr = cuts[j + 1] - cuts[j], ns = cuts[j + 3] - cuts[j + 2];
    if (!ns) continue;
    part = std::max(part, al256(std::max<size_t>(bucket_plan_bytes(ns, nr), ns * 8)));
    tail = std::max(tail, al256(ns * 8) + al256(std::max(radix_sort_ws(ns), radix_pass_runs_ws(ns, (nr >> 16) + 1))) + al256(nr * 8) + al256((nr + 2) * 4) +
                               al256((nr + 1) * 8) + al256(((nr >> kRecGroupBits) + 1) * 16));
  }
  rc = ws_reserve(ctx, S0 + part + tail);
  if (rc) return rc;
  Scratch s = scratch_bind(ctx, nvals, o);
  SG_HIP(hipMemsetAsync(s.dmask, 0, s.nchunks * 32, ctx->stream));
  const int aligned = ((uintptr_t)d_vals & 15) == 0;
  for (size_t j = 0; j + 3 < cuts.size(); j += 4) {
    const uint64_t r0 = cuts[j], nr = cuts[j + 1] - r0, e0 = cuts[j + 2], ns = cuts[j + 3] - e0;
    if (!ns) continue;  // (flags cleared above)
    uint64_t* keys_b = (uint64_t*)ws_at(ctx, S0);
    size_t at = S0 + part;
    uint64_t* keys_a = (uint64_t*)ws_at(ctx, at);
    at += al256(ns * 8);
    const size_t sort_at = at;
    at += al256(std::max(radix_sort_ws(ns), radix_pass_runs_ws(ns, (nr >> 16) + 1)));
    uint2* po = (uint2*)ws_at(ctx, at);
    at += al256(nr * 8);
    uint32_t* big = (uint32_t*)ws_at(ctx, at);  // count, records, ticket
    at += al256((nr + 2) * 4);
    uint64_t* roff = (uint64_t*)ws_at(ctx, at);
    at += al256((nr + 1) * 8);
    const uint32_t ng = (uint32_t)((nr + (1u << kRecGroupBits) - 1) >> kRecGroupBits);
    unsigned long long* gcur = (unsigned long long*)ws_at(ctx, at);  // ng cursors, then ng starts
    uint64_t* gs = (uint64_t*)(gcur + ng);
    rc = rebase_offsets(ctx, d_off + r0, nr + 1, e0, roff);
    if (rc) return rc;
    SG_HIP(hipMemsetAsync(gcur, 0, ng * 8, ctx->stream));
    SG_HIP(hipMemsetAsync(big, 0, 4, ctx->stream));
    hipLaunchKernelGGL(k_group_starts, dim3(div_up(ng, 256)), dim3(256), 0, ctx->stream, (const uint64_t*)roff, ng, gs);
    rc = bucket_emit_update(ctx, mwords, nwords, d_vals + e0, roff, ns, nr, (uint2*)keys_a, gcur, S0);
    if (rc) return rc;
    std::vector<uint64_t> gh(2 * (size_t)ng);  // counts, starts
    SG_HIP(hipMemcpyAsync(gh.data(), gcur, gh.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    SG_HIP(hipStreamSynchronize(ctx->stream));
    // the pairs by record: two stable passes over the record's low 16 bits,
    // the first reading the groups' runs in group order, so equal low bits
    // keep group order and every record's pairs end up together (records in
    // (low 16 bits, group) order)
    std::vector<uint64_t> rs, rc_;
    uint64_t np = 0;
    for (uint32_t g = 0; g < ng; g++)
      if (gh[g]) {
        rs.push_back(gh[ng + g]);
        rc_.push_back(gh[g]);
        np += gh[g];
      }
    uint64_t* sorted = keys_b;
    {
      ScopedTimer tm(ctx, "owned_sort");
      if (np >= 2) {
        rc = radix_pass_runs(ctx, keys_a, rs, rc_, 32, keys_b, sort_at);
        if (rc) return rc;
        rc = radix_sort_u64(ctx, keys_b, keys_a, np, sort_at, &sorted, 0xFF00ull << 32);
        if (rc) return rc;
      } else if (np == 1) {
        SG_HIP(hipMemcpyAsync(keys_b, keys_a + rs[0], 8, hipMemcpyDeviceToDevice, ctx->stream));
      }
    }
    ScopedTimer tm(ctx, "owned_sweep");
    hipLaunchKernelGGL(k_own_bounds_search, dim3(div_up(nr, 256)), dim3(256), 0, ctx->stream, (const uint64_t*)sorted,
                       np, (uint32_t)nr, po);
    OwnArgs oa{d_vals, roff, e0, (uint32_t)nr, sorted, po, d_rec_new ? d_rec_new + r0 : nullptr, s.dmask, big, nvals,
               big + nr + 1};
    SG_HIP(hipMemsetAsync(big + nr + 1, 0, 4, ctx->stream));
    if (aligned)
      rc = launch_own<true>(ctx, oa, nr, dedup);
    else
      rc = launch_own<false>(ctx, oa, nr, dedup);
    if (rc) return rc;
    SG_HIP(hipGetLastError());
  }
  if (!d_out_vals && !d_out_off) return SG_OK;
  hipLaunchKernelGGL(k_mask_count, dim3(div_up(s.nchunks, 256)), dim3(256), 0, ctx->stream, (const uint64_t*)s.dmask,
                     s.nchunks, s.dcnt);
  return run_emit(ctx, d_vals, nvals, s.dmask, s.dcnt, s, scan_off, d_off, nrec, d_out_vals, d_out_off);
}

static int check_alloc(sg_ctx* ctx) { return ensure_device(ctx); }

}  // namespace sg

using namespace sg;

extern "C" {

int sg_triage_batch_dev(sg_ctx* ctx, sg_set* maxsig, sg_set* newsig, const uint32_t* d_vals,
                        const uint64_t* d_rec_off, uint64_t nvals, uint64_t nrec, uint8_t* d_rec_new,
                        uint32_t* d_diff_vals, uint64_t* d_diff_off) {
  if (!ctx || !maxsig || !d_rec_off || (nrec && !d_rec_new) || (nvals && !d_vals)) {
    set_error("sg_triage_batch_dev: invalid argument");
    return SG_EINVAL;
  }
  if (maxsig->ctx != ctx || (newsig && newsig->ctx != ctx)) {
    set_error("sg_triage_batch_dev: set belongs to another context");
    return SG_EINVAL;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = check_alloc(ctx);
  if (rc) return rc;
  if (!d_diff_vals && !d_diff_off)  // flags + set updates only: partitioned path
    return bucket_triage(ctx, maxsig->words, newsig ? newsig->words : nullptr, d_vals, d_rec_off, nvals, nrec,
                         d_rec_new);
  // the ordered diff lists (fuzzer.go:669 SignalDiff per record) from the
  // update-emitting bucket stage's first owners
  return owned_outputs(ctx, maxsig->words, newsig ? newsig->words : nullptr, d_vals, d_rec_off, nvals, nrec, d_rec_new,
                       d_diff_vals, d_diff_off, false);
}

int sg_triage_batch(sg_ctx* ctx, sg_set* maxsig, sg_set* newsig, const uint32_t* vals, const uint64_t* rec_off,
                    size_t nrec, uint8_t* rec_new, uint32_t* diff_vals, uint64_t* diff_off, uint64_t* n_diff) {
  if (!ctx || !maxsig || !rec_off || (nrec && !rec_new)) {
    set_error("sg_triage_batch: invalid argument");
    return SG_EINVAL;
  }
  uint64_t nvals = rec_off[nrec] - rec_off[0];
  if (rec_off[0] != 0) {
    set_error("sg_triage_batch: rec_off[0] must be 0");
    return SG_EINVAL;
  }
  for (size_t r = 0; r < nrec; r++)
    if (rec_off[r + 1] < rec_off[r]) {
      set_error("sg_triage_batch: rec_off not non-decreasing at %zu", r);
      return SG_EINVAL;
    }
  if (nvals && !vals) return SG_EINVAL;
  bool want_diff = diff_vals || diff_off || n_diff;
  if (!want_diff) {  // flags and set updates: the pipelined ingest (sg_host.hip)
    if (maxsig->ctx != ctx || (newsig && newsig->ctx != ctx)) {
      set_error("sg_triage_batch: set belongs to another context");
      return SG_EINVAL;
    }
    return host_pipeline(ctx, maxsig->words, newsig ? newsig->words : nullptr, vals, rec_off, nrec, rec_new, false);
  }
  // device staging: vals, off, rec_new, diff_vals, diff_off  (pipeline scratch
  // is carved behind these by the _dev entry point, which reserves again).
  uint32_t* dv;
  uint64_t* doff;
  uint8_t* dflag;
  uint32_t* ddv;
  uint64_t* ddo;
  // staged batch lives in the context's device staging buffer (the workspace
  // stays free for the pipeline)
  size_t b_vals = (nvals * 4 + 255) & ~size_t(255), b_off = ((nrec + 1) * 8 + 255) & ~size_t(255),
         b_flag = (nrec + 256) & ~size_t(255);
  size_t b_dv = want_diff ? b_vals : 0, b_do = want_diff ? b_off : 0;
  char* stage = nullptr;
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    int rc = check_alloc(ctx);
    if (rc) return rc;
    rc = dstage_reserve(ctx, b_vals + b_off + b_flag + b_dv + b_do + 256);
    if (rc) return rc;
    stage = (char*)ctx->dstage;
  }
  dv = (uint32_t*)stage;
  doff = (uint64_t*)(stage + b_vals);
  dflag = (uint8_t*)(stage + b_vals + b_off);
  ddv = want_diff ? (uint32_t*)(stage + b_vals + b_off + b_flag) : nullptr;
  ddo = want_diff ? (uint64_t*)(stage + b_vals + b_off + b_flag + b_dv) : nullptr;
  if (nvals) SG_HIP(hipMemcpyAsync(dv, vals, nvals * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(doff, rec_off, (nrec + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  int rc = sg_triage_batch_dev(ctx, maxsig, newsig, dv, doff, nvals, nrec, dflag, ddv, ddo);
  if (rc) return rc;
  if (nrec) SG_HIP(hipMemcpyAsync(rec_new, dflag, nrec, hipMemcpyDeviceToHost, ctx->stream));
  uint64_t total = 0;
  if (want_diff) SG_HIP(hipMemcpyAsync(&total, ddo + nrec, 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (diff_off) SG_HIP(hipMemcpyAsync(diff_off, ddo, (nrec + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  if (diff_vals && total) SG_HIP(hipMemcpyAsync(diff_vals, ddv, total * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (n_diff) *n_diff = total;
  return SG_OK;
}

int sg_triage_traces_dev(sg_ctx* ctx, sg_set* maxsig, sg_set* newsig, const uint32_t* d_pcs,
                         const uint64_t* d_call_off, uint64_t npcs, uint64_t ncalls, uint8_t* d_rec_new) {
  if (!ctx || !maxsig || !d_call_off || (ncalls && !d_rec_new) || (npcs && !d_pcs)) {
    set_error("sg_triage_traces_dev: invalid argument");
    return SG_EINVAL;
  }
  if (maxsig->ctx != ctx || (newsig && newsig->ctx != ctx)) {
    set_error("sg_triage_traces_dev: set belongs to another context");
    return SG_EINVAL;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = check_alloc(ctx);
  if (rc) return rc;
  return bucket_triage(ctx, maxsig->words, newsig ? newsig->words : nullptr, d_pcs, d_call_off, npcs, ncalls,
                       d_rec_new, true);
}

int sg_triage_traces(sg_ctx* ctx, sg_set* maxsig, sg_set* newsig, const uint32_t* pcs, const uint64_t* call_off,
                     size_t ncalls, uint8_t* rec_new) {
  if (!ctx || !maxsig || !call_off || (ncalls && !rec_new)) {
    set_error("sg_triage_traces: invalid argument");
    return SG_EINVAL;
  }
  if (call_off[0] != 0) {
    set_error("sg_triage_traces: call_off[0] must be 0");
    return SG_EINVAL;
  }
  for (size_t r = 0; r < ncalls; r++)
    if (call_off[r + 1] < call_off[r]) {
      set_error("sg_triage_traces: call_off not non-decreasing at %zu", r);
      return SG_EINVAL;
    }
  const uint64_t npcs = call_off[ncalls];
  if (npcs && !pcs) return SG_EINVAL;
  if (maxsig->ctx != ctx || (newsig && newsig->ctx != ctx)) {
    set_error("sg_triage_traces: set belongs to another context");
    return SG_EINVAL;
  }
  // the pipelined ingest (sg_host.hip): record (call) slices, each a trace slice
  // starting at a call start
  return host_pipeline(ctx, maxsig->words, newsig ? newsig->words : nullptr, pcs, call_off, ncalls, rec_new, true);
}

int sg_set_diff(sg_set* set, const uint32_t* sig, size_t n, uint32_t* out, size_t* nout) {
  if (!set || !nout || (n && (!sig || !out))) return SG_EINVAL;
  *nout = 0;
  if (n == 0) return SG_OK;
  sg_ctx* ctx = set->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = check_alloc(ctx);
  if (rc) return rc;
  WsPlan p;
  size_t o[5];
  size_t o_in = p.add(n * 4);
  size_t o_out = p.add(n * 4);
  size_t scan_b = scratch_plan(p, n, o);
  size_t scan_off = p.total;
  rc = ws_reserve(ctx, p.total + scan_b);
  if (rc) return rc;
  Scratch s = scratch_bind(ctx, n, o);
  uint32_t* din = (uint32_t*)ws_at(ctx, o_in);
  uint32_t* dout = (uint32_t*)ws_at(ctx, o_out);
  SG_HIP(hipMemcpyAsync(din, sig, n * 4, hipMemcpyHostToDevice, ctx->stream));
  {
    ScopedTimer tm(ctx, "set_diff");
    hipLaunchKernelGGL(k_mask<NotIn>, dim3(div_up(s.nchunks, kBlock / 64)), dim3(kBlock), 0, ctx->stream, din,
                       (uint64_t)n, 1, NotIn{set->words}, s.nchunks, s.cmask, s.dcnt);
  }
  rc = run_emit(ctx, din, n, s.cmask, s.dcnt, s, scan_off, nullptr, 0, dout, nullptr);
  if (rc) return rc;
  uint64_t total = 0;
  SG_HIP(hipMemcpyAsync(&total, s.base + s.nchunks, 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (total) SG_HIP(hipMemcpyAsync(out, dout, total * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  *nout = (size_t)total;
  return SG_OK;
}

int sg_add_inputs(sg_ctx* ctx, sg_set* corpus, sg_set* maxsig, const uint32_t* vals, const uint64_t* off, size_t n) {
  if (!ctx || !corpus || !maxsig || !off) return SG_EINVAL;
  uint64_t nv = off[n] - off[0];
  if (off[0] != 0 || (nv && !vals)) return SG_EINVAL;
  if (nv == 0) return SG_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = check_alloc(ctx);
  if (rc) return rc;
  WsPlan p;
  size_t o[5];
  size_t o_in = p.add(nv * 4);
  scratch_plan(p, nv, o);
  rc = ws_reserve(ctx, p.total);
  if (rc) return rc;
  Scratch s = scratch_bind(ctx, nv, o);
  uint32_t* din = (uint32_t*)ws_at(ctx, o_in);
  SG_HIP(hipMemcpyAsync(din, vals, nv * 4, hipMemcpyHostToDevice, ctx->stream));
  // corpus ∪= ⋃S \ M0 ; maxSignal ∪= ⋃S \ M0   (fuzzer.go:485-487)
  hipLaunchKernelGGL(k_mask<NotIn>, dim3(div_up(s.nchunks, kBlock / 64)), dim3(kBlock), 0, ctx->stream, din, nv, 1,
                     NotIn{maxsig->words}, s.nchunks, s.cmask, s.dcnt);
  hipLaunchKernelGGL(k_apply_mask, dim3(div_up(s.nchunks, kBlock / 64)), dim3(kBlock), 0, ctx->stream, din, nv, 1,
                     s.cmask, s.nchunks, corpus->words, maxsig->words);
  SG_HIP(hipGetLastError());
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

int sg_accept_batch(sg_ctx* ctx, sg_set* corpus_sig, sg_set* corpus_cov, const uint32_t* sig_vals,
                    const uint64_t* sig_off, const uint32_t* cov_vals, const uint64_t* cov_off, size_t n,
                    uint8_t* accepted) {
  if (!ctx || !corpus_sig || !sig_off || (n && !accepted)) return SG_EINVAL;
  uint64_t nv = sig_off[n] - sig_off[0];
  uint64_t nc = (corpus_cov && cov_off) ? cov_off[n] - cov_off[0] : 0;
  if (sig_off[0] != 0 || (nv && !sig_vals) || (nc && !cov_vals)) return SG_EINVAL;
  if (n == 0) return SG_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = check_alloc(ctx);
  if (rc) return rc;
  // The NewInput loop (manager.go:907-911) is the fuzzer's new-signal loop
  // with corpusSignal as the running set and no newSignal: the partitioned
  // triage path.  The batch is staged in dstage (the workspace is the
  // partition's).
  const size_t b_in = (nv * 4 + 255) & ~size_t(255), b_off = ((n + 1) * 8 + 255) & ~size_t(255),
               b_flag = (n + 255) & ~size_t(255), b_cv = (nc * 4 + 255) & ~size_t(255);
  rc = dstage_reserve(ctx, b_in + 2 * b_off + b_flag + b_cv + 256);
  if (rc) return rc;
  char* st = (char*)ctx->dstage;
  uint32_t* din = (uint32_t*)st;
  uint64_t* doff = (uint64_t*)(st + b_in);
  uint8_t* dflag = (uint8_t*)(st + b_in + b_off);
  if (nv) SG_HIP(hipMemcpyAsync(din, sig_vals, nv * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(doff, sig_off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  rc = bucket_triage(ctx, corpus_sig->words, nullptr, din, doff, nv, n, dflag);
  if (rc) return rc;
  if (nc) {
    uint32_t* dcv = (uint32_t*)(st + b_in + b_off + b_flag);
    uint64_t* dco = (uint64_t*)(st + b_in + b_off + b_flag + b_cv);
    SG_HIP(hipMemcpyAsync(dcv, cov_vals, nc * 4, hipMemcpyHostToDevice, ctx->stream));
    SG_HIP(hipMemcpyAsync(dco, cov_off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_add_flagged_segs, dim3(std::min<uint64_t>(div_up(nc, 256), 8192)), dim3(256), 0,
                       ctx->stream, dcv, nc, dco, (uint64_t)n, dflag, corpus_cov->words);
    SG_HIP(hipGetLastError());
  }
  SG_HIP(hipMemcpyAsync(accepted, dflag, n, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

int sg_merge_poll(sg_ctx* ctx, sg_set* mgr_max, const uint32_t* a_vals, const uint64_t* a_off, size_t npoll,
                  uint32_t* new_vals, uint64_t* new_off) {
  if (!ctx || !mgr_max || !a_off || !new_off) return SG_EINVAL;
  uint64_t nv = a_off[npoll] - a_off[0];
  if (a_off[0] != 0 || (nv && (!a_vals || !new_vals))) return SG_EINVAL;
  if (nv == 0) {
    for (size_t k = 0; k <= npoll; k++) new_off[k] = 0;
    return SG_OK;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = check_alloc(ctx);
  if (rc) return rc;
  // the Poll loop (manager.go:949-956) is a first-owner loop over the polls
  // with mgr.maxSignal as the running set, each poll's new signals in its
  // order, once each (its first occurrence): the ordered-output path with
  // dedup.  The batch is staged in dstage (the workspace is the partition's).
  const size_t b_in = al256(nv * 4), b_off = al256((npoll + 1) * 8);
  rc = dstage_reserve(ctx, 2 * b_in + 2 * b_off + 256);
  if (rc) return rc;
  char* st = (char*)ctx->dstage;
  uint32_t* din = (uint32_t*)st;
  uint64_t* doff = (uint64_t*)(st + b_in);
  uint32_t* dout = (uint32_t*)(st + b_in + b_off);
  uint64_t* doo = (uint64_t*)(st + 2 * b_in + b_off);
  SG_HIP(hipMemcpyAsync(din, a_vals, nv * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(doff, a_off, (npoll + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  rc = owned_outputs(ctx, mgr_max->words, nullptr, din, doff, nv, npoll, nullptr, dout, doo, true);
  if (rc) return rc;
  SG_HIP(hipMemcpyAsync(new_off, doo, (npoll + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (new_off[npoll])
    SG_HIP(hipMemcpyAsync(new_vals, dout, new_off[npoll] * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

int sg_minimize(sg_ctx* ctx, const uint32_t* vals, const uint64_t* off, size_t n, const uint32_t* order,
                uint32_t* out_idx, size_t* nout) {
  if (!ctx || !off || !nout || (n && (!order || !out_idx))) return SG_EINVAL;
  *nout = 0;
  uint64_t nv = off[n] - off[0];
  if (off[0] != 0 || (nv && !vals)) return SG_EINVAL;
  if (n == 0 || nv == 0) return SG_OK;
  {
    // order must be a permutation of 0..n-1
    std::vector<uint8_t> seen(n, 0);
    for (size_t k = 0; k < n; k++) {
      if (order[k] >= n || seen[order[k]]) {
        set_error("sg_minimize: order is not a permutation");
        return SG_EINVAL;
      }
      seen[order[k]] = 1;
    }
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = check_alloc(ctx);
  if (rc) return rc;
  WsPlan p;
  size_t o_in = p.add(nv * 4), o_off = p.add((n + 1) * 8), o_ord = p.add(n * 4),
         o_flag = p.add(n), o_fr = p.add(n), o_out = p.add(n * 4), o_m = p.add(((n + kTile - 1) / kTile) * kTile / 8),
         o_c = p.add(((n + kTile - 1) / kTile) * kChunksPerTile * 4), o_b = p.add(((n + kTile - 1) / kTile) * kChunksPerTile * 8 + 8),
         o_t = p.add(kSetBytes), o_fs = p.add(kFilt * 4), o_ro = p.add((n + 1) * 8), o_so = p.add(n * 8),
         o_tk = p.add((nv / kFWin + 2) * 4), o_ct = p.add(((size_t)kFirstSlots + n) * 4);
  size_t scan_off = p.total;
  size_t scan_b2 = std::max(scan_ws_bytes(((n + kTile - 1) / kTile) * kChunksPerTile), scan_ws_bytes(n));
  rc = ws_reserve(ctx, p.total + scan_b2);
  if (rc) return rc;
  uint32_t* dtouch = (uint32_t*)ws_at(ctx, o_t);  // touched values (set layout)
  uint32_t* din = (uint32_t*)ws_at(ctx, o_in);
  uint64_t* doff = (uint64_t*)ws_at(ctx, o_off);
  uint32_t* dord = (uint32_t*)ws_at(ctx, o_ord);
  uint8_t* dflag = (uint8_t*)ws_at(ctx, o_flag);
  uint8_t* dfr = (uint8_t*)ws_at(ctx, o_fr);
  uint32_t* dout = (uint32_t*)ws_at(ctx, o_out);
  SG_HIP(hipMemcpyAsync(din, vals, nv * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(doff, off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dord, order, n * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemsetAsync(dflag, 0, n, ctx->stream));
  uint32_t key_lo;
  rc = owner_keys(ctx, n, &key_lo);
  if (rc) return rc;
  // the owner table: every element lowers its value's owner to its input's
  // rank key (covered starts empty, cover.go:130); the inputs owning some
  // value are the selected ones (cover.go:133-141)
  // phase A: ranks < R (the first ~kFiltElems elements in processing order)
  // claim one workgroup per input and fill the filter set; phase B: the rest
  // through the persistent filtered claim (k_min_claim_f)
  const bool use_filt = ctx->opt[kOptMinimizeFilter] != 0;
  // phase A: the first kFiltRanks inputs (option minimize_filter_ranks: tests
  // raise it past the filter's values' inputs)
  const uint64_t fr = ctx->opt[kOptMinimizeFilterRanks] > 0 ? (uint64_t)ctx->opt[kOptMinimizeFilterRanks] : 0;
  const uint64_t R = use_filt && n > kFiltRanks ? std::min<uint64_t>(n - 1, std::max<uint64_t>(kFiltRanks, fr)) : n;
  {
    ScopedTimer tm(ctx, "min_claim");
    SG_HIP(hipMemsetAsync(dtouch, 0, kSetBytes, ctx->stream));
    hipLaunchKernelGGL(k_min_claim, dim3((uint32_t)R), dim3(kBlock), 0, ctx->stream, (const uint32_t*)din,
                       (const uint64_t*)doff, (const uint32_t*)dord, key_lo, (uint32_t)(key_lo + n), ctx->owner,
                       dtouch);
    if (R < n) {
      uint32_t* dfilt = (uint32_t*)ws_at(ctx, o_fs);
      uint64_t* droff = (uint64_t*)ws_at(ctx, o_ro);
      uint64_t* dsoff = (uint64_t*)ws_at(ctx, o_so);
      uint32_t* dwr = (uint32_t*)ws_at(ctx, o_tk);
      uint32_t* dfirst = (uint32_t*)ws_at(ctx, o_ct);
      uint32_t* dlens = dfirst + kFirstSlots;
      const uint64_t nr = n - R;
      uint64_t nel = nv;
      for (uint64_t r = 0; r < R; r++) nel -= off[order[r] + 1] - off[order[r]];
      const uint64_t nwin = (nel + kFWin - 1) / kFWin;
      hipLaunchKernelGGL(k_min_ranks, dim3(div_up(nr, 256)), dim3(256), 0, ctx->stream, (const uint64_t*)doff,
                         (const uint32_t*)dord, R, nr, dlens, dsoff);
      rc = scan_counts(ctx, dlens, droff, nr, scan_off);
      if (rc) return rc;
      if (nwin)
        hipLaunchKernelGGL(k_min_wrank, dim3(div_up(nwin, 256)), dim3(256), 0, ctx->stream, (const uint64_t*)droff,
                           nr, nwin, dwr);
      SG_HIP(hipMemsetAsync(dfilt, 0xFF, kFilt * 4, ctx->stream));
      SG_HIP(hipMemsetAsync(dfirst, 0xFF, kFirstSlots * 4, ctx->stream));
      hipLaunchKernelGGL(k_min_first, dim3(16), dim3(kBlock), 0, ctx->stream, (const uint32_t*)din,
                         (const uint64_t*)doff, (const uint32_t*)dord, dfirst);
      hipLaunchKernelGGL(k_min_filter, dim3(16, (uint32_t)R - 1), dim3(kBlock), 0, ctx->stream, (const uint32_t*)din,
                         (const uint64_t*)doff, (const uint32_t*)dord, (const uint32_t*)dfirst, dfilt);
      MinClaimF f{(const uint32_t*)din, droff, dsoff, nr, nel, (uint32_t)(key_lo + R), (uint32_t)(key_lo + n),
                  ctx->owner, dtouch, dfilt, dwr};
      if (nel) {
      int per_cu = 0, cus = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_min_claim_f, kFT, 0) != hipSuccess ||
          per_cu < 1)
        per_cu = 1;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || cus < 1)
        cus = 256;
      hipLaunchKernelGGL(k_min_claim_f, dim3((uint32_t)(per_cu * cus)), dim3(kFT), 0, ctx->stream, f);
      }
    }
  }
  {
    ScopedTimer tm(ctx, "min_owners");
    hipLaunchKernelGGL(k_min_owners, dim3(4096), dim3(256), 0, ctx->stream, (const uint32_t*)dtouch,
                       (const uint32_t*)ctx->owner, key_lo, (const uint32_t*)dord, dflag);
  }
  SG_HIP(hipGetLastError());
  // selected indices in processing order: compact order[k] where flag[order[k]]
  hipLaunchKernelGGL(k_gather_flag, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, dord, (uint64_t)n, dflag, dfr);
  Scratch s2;
  s2.ntiles = (n + kTile - 1) / kTile;
  s2.nchunks = s2.ntiles * kChunksPerTile;
  s2.cmask = (uint64_t*)ws_at(ctx, o_m);
  s2.dcnt = (uint32_t*)ws_at(ctx, o_c);
  s2.base = (uint64_t*)ws_at(ctx, o_b);
  hipLaunchKernelGGL(k_mask<FlagAt>, dim3(div_up(s2.nchunks, kBlock / 64)), dim3(kBlock), 0, ctx->stream, dord,
                     (uint64_t)n, ((uintptr_t)dord & 15) == 0, FlagAt{dfr}, s2.nchunks, s2.cmask, s2.dcnt);
  rc = run_emit(ctx, dord, n, s2.cmask, s2.dcnt, s2, scan_off, nullptr, 0, dout, nullptr);
  if (rc) return rc;
  uint64_t total = 0;
  SG_HIP(hipMemcpyAsync(&total, s2.base + s2.nchunks, 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (total) SG_HIP(hipMemcpyAsync(out_idx, dout, total * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  *nout = (size_t)total;
  return SG_OK;
}

}  // extern "C"
