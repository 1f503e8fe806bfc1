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
// those elements, in item order with duplicates.  Two streaming kernels:
//   claim   : probe the S0 bitmap per element; for s ∉ S0 atomicMin its key
//             into the direct-indexed owner table (2^32 x u32, 16 GiB);
//             record the candidates as per-chunk ballot masks.
//   resolve : for candidates only, owner[s] == own key -> diff element; set
//             the bits of the running sets, flag the item, ballot-mask it.
// The ordered diff output is a stream compaction of the resolve masks.
// Owner keys decrease from batch to batch (sg::owner_keys), so the table
// never needs resetting between batches.
#include "sg_internal.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace sg {

struct PipeArgs {
  const uint32_t* vals;
  uint64_t n;
  const uint64_t* off;      // nseg+1 (null: element-level items)
  uint64_t nseg;
  const uint32_t* filter;   // S0 words (null: S0 = ∅)
  const uint32_t* rank;     // rank of item (null: identity)
  const uint32_t* tile_rec; // ntiles+1: item of the first element of each tile
  uint32_t* owner;
  uint32_t key_lo;
  uint64_t* cmask;          // nchunks*4 candidate ballots
  uint64_t* dmask;          // nchunks*4 diff ballots
  uint32_t* dcnt;           // nchunks diff counts
  uint8_t* seg_flag;        // nseg (nullable)
  uint32_t* set_a;          // running sets updated with diff elements (nullable)
  uint32_t* set_b;
  int aligned;              // vals is 16-B aligned
};

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

// chunk c of tile t handled by wave w at step j (interleaved so the block's
// loads at one step cover 4 KiB contiguously).
__device__ __forceinline__ uint64_t chunk_of(uint64_t tile, int j, int wave) {
  return tile * kChunksPerTile + (uint64_t)(j * 4 + wave);
}

// Item window of one tile kept in LDS.
struct Win {
  uint64_t r_a, r_b, wn;
};

__device__ __forceinline__ void win_setup(const PipeArgs& a, uint64_t tile, uint64_t* win, Win& w) {
  w.r_a = a.tile_rec[tile];
  w.r_b = a.tile_rec[tile + 1];
  w.wn = w.r_b - w.r_a + 1;
  if (w.wn <= (uint64_t)kWin)
    for (uint64_t k = threadIdx.x; k < w.wn; k += blockDim.x) win[k] = a.off[w.r_a + k];
}

__device__ __forceinline__ uint64_t win_lookup(const PipeArgs& a, const uint64_t* win, const Win& w, uint64_t e) {
  if (w.wn <= (uint64_t)kWin) return w.r_a + sgd::seg_search(win, 0, w.wn - 1, e);
  return sgd::seg_search(a.off, w.r_a, w.r_b, e);
}

__device__ __forceinline__ void store_ballots(uint64_t* mask, uint64_t c, int lane, uint32_t bits4) {
  uint64_t b0 = __ballot(bits4 & 1u);
  uint64_t b1 = __ballot(bits4 & 2u);
  uint64_t b2 = __ballot(bits4 & 4u);
  uint64_t b3 = __ballot(bits4 & 8u);
  uint64_t mine = lane == 0 ? b0 : lane == 1 ? b1 : lane == 2 ? b2 : b3;
  if (lane < 4) mask[c * 4 + lane] = mine;
}

__global__ void k_tile_rec(const uint64_t* __restrict__ off, uint64_t nseg, uint64_t n, uint64_t ntiles,
                           uint32_t* __restrict__ tile_rec) {
  uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > ntiles) return;
  uint64_t e = t * kTile;
  if (e >= n) e = n - 1;
  tile_rec[t] = (uint32_t)sgd::seg_search(off, 0, nseg - 1, e);
}

template <bool kSeg>
__global__ __launch_bounds__(kBlock) void k_claim(PipeArgs a) {
  __shared__ uint64_t win[kWin];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t tile = blockIdx.x;
  uint32_t x[4][4];
  uint32_t cand = 0;  // bit 4j+k
#pragma unroll
  for (int j = 0; j < 4; j++) {
    uint64_t c = chunk_of(tile, j, wave);
    uint32_t ok;
    load4(a.vals, a.n, c * kChunk + lane * 4, a.aligned, x[j], ok);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      bool cnd = (ok >> k) & 1u;
      if (a.filter) cnd = cnd && !sgd::test_bit(a.filter, x[j][k]);
      cand |= (cnd ? 1u : 0u) << (4 * j + k);
    }
  }
  int any = __syncthreads_or(cand != 0);
  if (any) {
    Win w;
    if (kSeg) {
      win_setup(a, tile, win, w);
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
#pragma unroll
      for (int k = 0; k < 4; k++) {  // static indices keep x[][] in registers
        if (!((cand >> (4 * j + k)) & 1u)) continue;
        uint64_t e = chunk_of(tile, j, wave) * kChunk + lane * 4 + k;
        uint64_t r = kSeg ? win_lookup(a, win, w, e) : e;
        uint32_t rk = a.rank ? a.rank[r] : (uint32_t)r;
        uint32_t key = a.key_lo + rk;
        uint32_t* p = a.owner + x[j][k];
        if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > key) atomicMin(p, key);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; j++) store_ballots(a.cmask, chunk_of(tile, j, wave), lane, (cand >> (4 * j)) & 0xFu);
}

template <bool kSeg>
__global__ __launch_bounds__(kBlock) void k_resolve(PipeArgs a) {
  __shared__ uint64_t win[kWin];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t tile = blockIdx.x;
  uint32_t cand = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    uint64_t c = chunk_of(tile, j, wave);
    const uint64_t* m = a.cmask + c * 4;
#pragma unroll
    for (int k = 0; k < 4; k++) cand |= (uint32_t)((m[k] >> lane) & 1ull) << (4 * j + k);
  }
  uint32_t diff = 0;
  int any = __syncthreads_or(cand != 0);
  if (any) {
    Win w;
    if (kSeg) {
      win_setup(a, tile, win, w);
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint32_t cj = (cand >> (4 * j)) & 0xFu;
      if (!cj) continue;
      uint64_t e0 = chunk_of(tile, j, wave) * kChunk + lane * 4;
      uint32_t x[4], ok;
      load4(a.vals, a.n, e0, a.aligned, x, ok);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (!((cj >> k) & 1u)) continue;
        uint64_t e = e0 + k;
        uint64_t r = kSeg ? win_lookup(a, win, w, e) : e;
        uint32_t rk = a.rank ? a.rank[r] : (uint32_t)r;
        if (a.owner[x[k]] != a.key_lo + rk) continue;
        diff |= 1u << (4 * j + k);
        if (a.set_a) sgd::set_bit(a.set_a, x[k]);
        if (a.set_b) sgd::set_bit(a.set_b, x[k]);
        if (a.seg_flag) a.seg_flag[r] = 1;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; j++) {
    uint64_t c = chunk_of(tile, j, wave);
    uint32_t dj = (diff >> (4 * j)) & 0xFu;
    store_ballots(a.dmask, c, lane, dj);
    uint32_t cntj = __popcll(__ballot(dj & 1u)) + __popcll(__ballot(dj & 2u)) + __popcll(__ballot(dj & 4u)) +
                    __popcll(__ballot(dj & 8u));
    if (lane == 0) a.dcnt[c] = cntj;
  }
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
// (read-checked atomicMin, the same first-owner rule as k_claim).  An element
// that reads a key of an older generation (>= key_end: no element of this
// call has written v yet) also sets v's bit in the touched bitmap (2^32 bits,
// the set layout), so about one global atomicOr per distinct value: the
// first current-generation writer of v always sets it.  The owners are then
// flagged from the touched bitmap alone (k_min_owners, one read of 512 MiB)
// instead of re-reading the corpus (k_resolve).
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

// claim + resolve over a batch already on the device.
static int run_pipe(sg_ctx* ctx, PipeArgs a, const Scratch& s) {
  if (a.n == 0) return SG_OK;
  a.cmask = s.cmask;
  a.dmask = s.dmask;
  a.dcnt = s.dcnt;
  a.tile_rec = s.tile_rec;
  a.owner = ctx->owner;
  a.aligned = ((uintptr_t)a.vals & 15) == 0;
  if (a.off) {
    ScopedTimer tm(ctx, "tile_rec");
    hipLaunchKernelGGL(k_tile_rec, dim3(div_up(s.ntiles + 1, 256)), dim3(256), 0, ctx->stream, a.off, a.nseg, a.n,
                       s.ntiles, s.tile_rec);
  }
  {
    ScopedTimer tm(ctx, "triage_claim");
    if (a.off)
      hipLaunchKernelGGL(k_claim<true>, dim3((uint32_t)s.ntiles), dim3(kBlock), 0, ctx->stream, a);
    else
      hipLaunchKernelGGL(k_claim<false>, dim3((uint32_t)s.ntiles), dim3(kBlock), 0, ctx->stream, a);
  }
  {
    ScopedTimer tm(ctx, "triage_resolve");
    if (a.off)
      hipLaunchKernelGGL(k_resolve<true>, dim3((uint32_t)s.ntiles), dim3(kBlock), 0, ctx->stream, a);
    else
      hipLaunchKernelGGL(k_resolve<false>, dim3((uint32_t)s.ntiles), dim3(kBlock), 0, ctx->stream, a);
  }
  SG_HIP(hipGetLastError());
  return SG_OK;
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
  WsPlan p;
  size_t o[5];
  size_t scan_b = scratch_plan(p, nvals, o);
  size_t scan_off = p.total;
  rc = ws_reserve(ctx, p.total + scan_b);
  if (rc) return rc;
  Scratch s = scratch_bind(ctx, nvals, o);
  uint32_t key_lo = 0;
  if (nrec) {
    rc = owner_keys(ctx, nrec, &key_lo);
    if (rc) return rc;
    SG_HIP(hipMemsetAsync(d_rec_new, 0, nrec, ctx->stream));
  }
  if (nvals == 0) {
    if (d_diff_off) SG_HIP(hipMemsetAsync(d_diff_off, 0, (nrec + 1) * 8, ctx->stream));
    return SG_OK;
  }
  PipeArgs a{};
  a.vals = d_vals;
  a.n = nvals;
  a.off = d_rec_off;
  a.nseg = nrec;
  a.filter = maxsig->words;
  a.key_lo = key_lo;
  a.seg_flag = d_rec_new;
  a.set_a = maxsig->words;
  a.set_b = newsig ? newsig->words : nullptr;
  rc = run_pipe(ctx, a, s);
  if (rc) return rc;
  if (d_diff_vals || d_diff_off)
    rc = run_emit(ctx, d_vals, nvals, s.dmask, s.dcnt, s, scan_off, d_rec_off, nrec, d_diff_vals, d_diff_off);
  return rc;
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
  WsPlan p;
  size_t o[5];
  size_t o_in = p.add(nv * 4), o_off = p.add((npoll + 1) * 8), o_out = p.add(nv * 4), o_oo = p.add((npoll + 1) * 8);
  size_t scan_b = scratch_plan(p, nv, o);
  size_t scan_off = p.total;
  rc = ws_reserve(ctx, p.total + scan_b);
  if (rc) return rc;
  Scratch s = scratch_bind(ctx, nv, o);
  uint32_t* din = (uint32_t*)ws_at(ctx, o_in);
  uint64_t* doff = (uint64_t*)ws_at(ctx, o_off);
  uint32_t* dout = (uint32_t*)ws_at(ctx, o_out);
  uint64_t* doo = (uint64_t*)ws_at(ctx, o_oo);
  SG_HIP(hipMemcpyAsync(din, a_vals, nv * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(doff, a_off, (npoll + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  uint32_t key_lo;
  rc = owner_keys(ctx, nv, &key_lo);  // one key per element: first occurrence wins
  if (rc) return rc;
  PipeArgs a{};
  a.vals = din;
  a.n = nv;
  a.off = nullptr;
  a.nseg = nv;
  a.filter = mgr_max->words;
  a.key_lo = key_lo;
  a.set_a = mgr_max->words;  // manager.go:953
  rc = run_pipe(ctx, a, s);
  if (rc) return rc;
  rc = run_emit(ctx, din, nv, s.dmask, s.dcnt, s, scan_off, doff, npoll, dout, doo);
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
  const char* filt_env = getenv("SG_MINIMIZE_FILTER");
  const bool use_filt = !filt_env || atoi(filt_env);
  // phase A: the first kFiltRanks inputs (SG_MINIMIZE_FILTER_RANKS: tests
  // raise it past the filter's values' inputs)
  const char* fr_env = getenv("SG_MINIMIZE_FILTER_RANKS");
  const uint64_t R = use_filt && n > kFiltRanks ? std::min<uint64_t>(n - 1, std::max<uint64_t>(
                                                       kFiltRanks, fr_env ? (uint64_t)atoll(fr_env) : 0))
                                                 : n;
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
