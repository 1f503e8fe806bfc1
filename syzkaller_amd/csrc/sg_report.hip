// sg_report.hip -- cover report: PCs -> uncovered call sites of the touched
// functions.
//
// Reference: syz-manager/cover.go:91-103 (pcs[i] = RestorePC(cov[i], base) -
// callLen, RestorePC at pkg/cover/cover.go:23-25, callLen = 5 at
// syz-manager/cover.go:61) and uncoveredPcsInFuncs, syz-manager/cover.go:257-307:
//
//   for pc in pcs (in order):
//     idx = sort.Search(symbols, pc < end); skip unless start <= pc <= end
//     first time this start is seen: uncovered ∪= allCoverPCs[start..end]
//     delete(uncovered, pc)
//
// Parallel form: a call-site PC c ends up uncovered iff the latest event that
// touches it is an add, i.e. max(add times) > max(delete times), where the
// add time of a function is the index of the first query that lands in it and
// a delete at query i comes after that query's own add.  Kernels: per query
// (two radix-indexed searches, first-query atomicMin per symbol, last-delete
// atomicMax per call site), per symbol group (the first query per start
// decides which symbol's range is added), per call site (final verdict), then
// an ordered compaction.  The per-query work runs grouped by chunks of call
// sites (k_q_count / k_q_scatter / k_q_chunk: every lookup and both
// reductions in LDS); past 16M call sites it is two passes of radix-indexed
// global searches (k_rep_first, k_rep_del), each in the query order its
// read-check needs.  Symbols must be sorted by start with non-decreasing
// ends (the condition under which the reference's binary search over ends is
// meaningful).
#include "sg_internal.h"

#include <algorithm>
#include <cstdlib>


namespace sg {

__device__ __forceinline__ uint64_t lb64(const uint64_t* a, uint64_t n, uint64_t v) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (a[mid] < v)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}
__device__ __forceinline__ uint64_t ub64(const uint64_t* a, uint64_t n, uint64_t v) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (a[mid] <= v)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// Radix index over a sorted u64 array A[0..n): r[k] = lower_bound(A, lo + (k
// << sh)) for k <= nb (lo = A[0]), so a lower_bound of x only searches
// [r[k], r[k+1]] for x's bucket k (about one entry per bucket): two adjacent
// loads and a short search instead of log2(n) dependent loads (the C5
// queries are 100M random lookups into 5M call sites and 50K symbols).
struct RadixIdx {
  const uint32_t* r;
  uint64_t lo;
  uint32_t sh, nb;
};

__device__ __forceinline__ uint64_t radix_bucket(uint64_t x, uint64_t lo, uint32_t sh, uint32_t nb) {
  if (x < lo) return 0;
  const uint64_t k = (x - lo) >> sh;
  return k < nb ? k : nb;
}

__global__ void k_radix_index(const uint64_t* __restrict__ a, uint64_t n, uint64_t lo, uint32_t sh, uint32_t nb,
                              uint32_t* __restrict__ r) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > nb) return;
  const uint64_t d = k << sh;
  const uint64_t x = ((d >> sh) != k || lo + d < lo) ? ~0ull : lo + d;  // saturate past the top of u64
  r[k] = (uint32_t)lb64(a, n, x);
}

// lower_bound(a, x) through the index
__device__ __forceinline__ uint64_t lb_idx(const uint64_t* a, uint64_t n, const RadixIdx& I, uint64_t x) {
  const uint64_t k = radix_bucket(x, I.lo, I.sh, I.nb);
  uint64_t lo = x < I.lo ? 0 : I.r[k], hi = x < I.lo ? I.r[0] : (k < I.nb ? I.r[k + 1] : n);
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (a[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// upper_bound(a, x) = lower_bound(a, x + 1)
__device__ __forceinline__ uint64_t ub_idx(const uint64_t* a, uint64_t n, const RadixIdx& I, uint64_t x) {
  return x == ~0ull ? n : lb_idx(a, n, I, x + 1);
}

struct RepArgs {
  const uint32_t* cov;
  uint64_t ncov;
  uint32_t base;
  const uint64_t* sstart;
  const uint64_t* send;
  uint64_t nsym;
  const uint64_t* pcs;
  uint64_t npcs;
  uint32_t* first_q;      // per symbol: first query index landing in it (0xFFFFFFFF none)
  uint64_t* group_first;  // per group leader: (first query << 32) | symbol
  uint32_t* last_del;     // per call site: 1 + last deleting query (0 none)
  uint8_t* flag;          // per call site: uncovered
  uint64_t* qbits;        // per query: inside a symbol (pass 1 -> pass 2)
  uint32_t* leader;       // per symbol: the first symbol with its start (handledFuncs' key, cover.go:288)
  RadixIdx iend, ipcs;    // indexes over send and pcs
  RadixIdx istart;        // index over sstart
};

// Two passes over the queries, each ordered so that its read-check skips
// almost every atomic: the first-query minimum per symbol wants ascending
// query order, the last-delete maximum per call site descending order (a
// call site is queried ~400 times in the C5 workload; one atomicMax per
// query serialised ~100M memory-side atomics on a few 100K addresses).
//
// Pass 1, ascending: symbol (cover.go:278-285) through the radix index over
// ends, the symbol's first query (atomicMin, issued only while below the
// stored value), and one bit per query: "inside a symbol" (ballot words).
// The grid stride is a multiple of 64, so a wave's lanes hold 64 consecutive
// queries starting at a multiple of 64.
__global__ __launch_bounds__(256) void k_rep_first(RepArgs a) {
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t n64 = (a.ncov + 63) & ~63ull;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n64; i += S) {
    bool hit = false;
    if (i < a.ncov) {
      const uint64_t pc = ((uint64_t)a.base << 32) + (uint64_t)a.cov[i] - 5;  // cover.go:101
      const uint64_t idx = ub_idx(a.send, a.nsym, a.iend, pc);                // cover.go:278
      hit = idx < a.nsym && pc >= a.sstart[idx] && pc <= a.send[idx];         // cover.go:285
      if (hit) {
        const uint32_t qi = (uint32_t)i;
        if (a.first_q[idx] > qi) atomicMin(&a.first_q[idx], qi);
      }
    }
    const uint64_t w = __ballot(hit);
    if ((threadIdx.x & 63) == 0) a.qbits[i >> 6] = w;
  }
}

// Pass 2, descending: for the queries inside a symbol, the call site it
// deletes (delete(uncovered, pc), cover.go:299) and its last deleting query
// (atomicMax, issued only while above the stored value; a read may see an
// older, smaller value than memory holds: then the atomic is merely
// redundant).  Measured (C5): lookups, not atomics, bound this pass; a
// call-site hash table and XCD-partitioned site ranges were both slower.
__global__ __launch_bounds__(256) void k_rep_del(RepArgs a) {
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.ncov) return;
  for (uint64_t k = (a.ncov - 1 - t) / S + 1; k-- > 0;) {
    const uint64_t i = t + k * S;
    if (!((a.qbits[i >> 6] >> (i & 63)) & 1ull)) continue;
    const uint64_t pc = ((uint64_t)a.base << 32) + (uint64_t)a.cov[i] - 5;
    const uint64_t j = lb_idx(a.pcs, a.npcs, a.ipcs, pc);
    const uint32_t q1 = (uint32_t)i + 1;
    if (j < a.npcs && a.pcs[j] == pc && a.last_del[j] < q1) atomicMax(&a.last_del[j], q1);
  }
}

// ---- chunked query path --------------------------------------------------
// The two per-query reductions (first query per symbol: a minimum; last
// deleting query per call site: a maximum) do not depend on the order in
// which queries are visited, so the queries can be regrouped freely.  The
// call sites are cut into chunks of kSites consecutive sites (32 KiB of u64
// PCs); a query belongs to the chunk that holds lower_bound(sites, pc), i.e.
// the chunk c with bnd[c-1] < pc <= bnd[c] (bnd[c] = the chunk's last site;
// chunk nch = above every site).  The queries are counted and scattered by
// chunk (k_q_count, k_q_scatter: chunk found by a search over bnd in LDS),
// then each chunk's queries run against its sites, and the symbols its PC
// range can land in, held in LDS (k_q_chunk): every lookup is an LDS search,
// the two reductions are LDS atomics, flushed once per (tile, chunk).
constexpr uint32_t kSites = 4096;        // call sites per chunk
constexpr uint32_t kMaxChunks = 4096;    // chunk bounds held in LDS (16M sites)
constexpr uint32_t kChunkIdx = 8192;     // radix buckets over the chunk bounds
constexpr uint32_t kSiteIdx = 1024;      // radix buckets over one chunk's sites
constexpr uint32_t kSymCap = 1024;       // symbols of a chunk held in LDS
constexpr int kQT = 1024;                // threads of the count / scatter kernels
constexpr int kSQPer = 8;                // queries per thread there, per sub-tile
constexpr int kSQSub = 8;                // sub-tiles per query tile (64K queries: one count-table column)
constexpr int kCT = 512;                 // threads of the chunk kernel
constexpr uint32_t kCTile = 32768;       // grouped queries per chunk-kernel tile

struct ChunkArgs {
  const uint32_t* cov;
  uint64_t ncov;
  uint64_t hi32;           // base << 32
  const uint64_t* pcs;     // call sites, sorted
  uint64_t npcs;
  const uint64_t* sstart;
  const uint64_t* send;
  uint64_t nsym;
  RadixIdx iend;           // over send (chunks whose symbols exceed kSymCap)
  uint32_t nch;            // chunks with sites; chunk nch: above every site
  uint32_t csh;            // radix shift of the chunk index (over pc - bnd[0])
  uint64_t* bnd;           // [nch] last site of each chunk
  uint16_t* cidx;          // [kChunkIdx + 1] bounds below bnd[0] + (k << csh)
  uint2* symr;             // [nch + 1] symbol range a chunk's queries can land in (lo, hi inclusive)
  uint32_t* ssh;           // [nch] radix shift of each chunk's site index
  uint16_t* sidx;          // [nch][kSiteIdx + 1] the chunk's sites below first + (k << ssh)
  uint32_t* ssym;          // [npcs] upper_bound(send, site): the symbol a query at the site lands in
  uint32_t ntiles;         // query tiles of the count / scatter kernels
  uint32_t tw;             // width of a chunk's row of tiles: 8 ceil(ntiles / 8)
  uint32_t* tcount;        // [nch + 1][tw] queries per (chunk, tile), tiles at tile_col
  uint64_t* toff;          // [(nch + 1) tw + 1] exclusive scan of tcount: each (chunk, tile)'s first slot
  uint32_t* jparts;        // [nch + 1] chunk-kernel jobs per chunk
  uint64_t* jstart;        // [nch + 2] scan of jparts
  uint64_t* qoff;          // [nch + 2] each chunk's first slot
  uint2* grouped;          // [ncov] (cov, query index) grouped by chunk
  uint16_t* qchunk;        // [ncov] each query's chunk (written by the count kernel)
  uint32_t* first_q;
  uint32_t* last_del;
};

__device__ __forceinline__ uint64_t query_pc(uint64_t hi32, uint32_t cov) { return hi32 + (uint64_t)cov - 5; }

// Column of tile t in a chunk's row of the count table: the tiles that run on
// one XCD (blockIdx % 8, round-robin dispatch: speed only) side by side, so
// the runs that neighbouring tiles of one XCD write for a chunk share cache
// lines in that XCD's L2 instead of leaving partial lines in several.
__device__ __forceinline__ uint32_t tile_col(uint32_t t, uint32_t tw) { return (t & 7u) * (tw >> 3) + (t >> 3); }

// chunk bounds and, per chunk, the range of upper_bound(send, pc) over its PCs
__global__ void k_chunk_prep(ChunkArgs a) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c > a.nch) return;
  uint64_t lo = 0, hi = a.nsym;
  // the previous chunk's last site (chunk nch, above every site, follows a
  // possibly partial last chunk: its bound is the last site, not pcs[nch kSites - 1])
  if (c > 0) lo = ub64(a.send, a.nsym, a.pcs[min<uint64_t>(c * kSites, a.npcs) - 1]);
  if (c < a.nch) {
    const uint64_t last = a.pcs[min<uint64_t>((c + 1) * kSites, a.npcs) - 1];
    a.bnd[c] = last;
    hi = ub64(a.send, a.nsym, last);
    const uint64_t span = last - a.pcs[c * kSites];
    uint32_t sh = 0;
    while (sh < 63 && (span >> sh) >= kSiteIdx) sh++;
    a.ssh[c] = sh;
  }
  a.symr[c] = make_uint2((uint32_t)lo, (uint32_t)hi);
}

// per site, the symbol a query at it lands in (cover.go:278)
__global__ void k_site_sym(ChunkArgs a) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < a.npcs) a.ssym[j] = (uint32_t)ub_idx(a.send, a.nsym, a.iend, a.pcs[j]);
}

// per chunk, a radix index over its sites: sidx[c][k] = sites of chunk c
// below first + (k << ssh[c]) (saturated at the top of u64)
__global__ void k_site_index(ChunkArgs a) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c = (uint32_t)(t / (kSiteIdx + 1)), k = (uint32_t)(t % (kSiteIdx + 1));
  if (c >= a.nch) return;
  const uint64_t* ps = a.pcs + (uint64_t)c * kSites;
  const uint32_t m = (uint32_t)min<uint64_t>(kSites, a.npcs - (uint64_t)c * kSites);
  const uint32_t sh = a.ssh[c];
  const uint64_t s0 = ps[0], d = (uint64_t)k << sh, x0 = s0 + d;
  const uint64_t x = (sh < 64 && (d >> sh) == k && x0 >= s0) ? x0 : ~0ull;  // saturate a wrapped bound
  uint32_t lo = 0, hi = m;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ps[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  a.sidx[t] = (uint16_t)lo;
}

// chunk index: cidx[k] = number of chunk bounds below bnd[0] + (k << csh)
__global__ void k_chunk_index(ChunkArgs a) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > kChunkIdx) return;
  const uint64_t b0 = a.pcs[kSites - 1 < a.npcs ? kSites - 1 : a.npcs - 1];  // bnd[0]
  const uint64_t d = (uint64_t)k << a.csh;
  const uint64_t x = (a.csh < 64 && (d >> a.csh) == k && b0 + d >= b0) ? b0 + d : ~0ull;
  // bnd[c] = pcs[min((c+1) kSites, n) - 1]: search over c
  uint32_t lo = 0, hi = a.nch;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a.pcs[min<uint64_t>((uint64_t)(mid + 1) * kSites, a.npcs) - 1] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  a.cidx[k] = (uint16_t)lo;
}

// number of b[lo..hi) below x plus lo (b sorted), b in LDS
__device__ __forceinline__ uint32_t lds_lb(const uint64_t* b, uint32_t lo, uint32_t hi, uint64_t x) {
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (b[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

struct ChunkLds {
  uint64_t bnd[kMaxChunks];
  uint16_t idx[kChunkIdx + 1];
};

__device__ __forceinline__ void load_chunks(const ChunkArgs& a, ChunkLds& L) {
  for (uint32_t i = threadIdx.x; i < a.nch; i += blockDim.x) L.bnd[i] = a.bnd[i];
  for (uint32_t i = threadIdx.x; i <= kChunkIdx; i += blockDim.x) L.idx[i] = a.cidx[i];
}

// chunk of pc: the number of chunk bounds below it
__device__ __forceinline__ uint32_t chunk_of(const ChunkArgs& a, const ChunkLds& L, uint64_t pc) {
  const uint64_t b0 = L.bnd[0];
  if (pc <= b0) return 0;
  const uint64_t k = (pc - b0) >> a.csh;
  if (k >= kChunkIdx) return lds_lb(L.bnd, L.idx[kChunkIdx], a.nch, pc);
  return lds_lb(L.bnd, L.idx[k], L.idx[k + 1], pc);
}

// Query tiles of kQT kPer kSub queries: one column of the count table each
// (a table of 8K-query columns was 15M counts per 100M queries, and its scan
// and the scatter's column reads -- a cache line per (chunk, tile) -- cost
// more than the scatter's stores).
template <int kPer, int kSub>
__global__ __launch_bounds__(kQT) void k_q_count(ChunkArgs a) {
  __shared__ ChunkLds L;
  __shared__ uint32_t hist[kMaxChunks + 1];
  load_chunks(a, L);
  for (uint32_t i = threadIdx.x; i <= a.nch; i += kQT) hist[i] = 0;
  __syncthreads();
  const uint64_t q0 = (uint64_t)blockIdx.x * kQT * kPer * kSub + threadIdx.x;
  // each sub-tile's loads issued before the one before is looked up
  uint32_t cn[kPer];
  auto load = [&](int sub) {
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const uint64_t i = q0 + (uint64_t)(sub * kPer + k) * kQT;
      cn[k] = a.cov[i < a.ncov ? i : 0];
    }
  };
  load(0);
  for (int sub = 0; sub < kSub; sub++) {
    uint32_t cv[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) cv[k] = cn[k];
    if (sub + 1 < kSub) load(sub + 1);
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const uint64_t i = q0 + (uint64_t)(sub * kPer + k) * kQT;
      if (i < a.ncov) {
        const uint32_t c = chunk_of(a, L, query_pc(a.hi32, cv[k]));
        atomicAdd(&hist[c], 1u);
        a.qchunk[i] = (uint16_t)c;  // (kMaxChunks + 1 <= 2^16)
      }
    }
  }
  __syncthreads();
  const uint32_t col = tile_col(blockIdx.x, a.tw);
  for (uint32_t i = threadIdx.x; i <= a.nch; i += kQT) a.tcount[(uint64_t)i * a.tw + col] = hist[i];
}

// each chunk's first slot (the scan at its first tile) and the total
__global__ void k_q_chunk_off(ChunkArgs a) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c <= (uint64_t)a.nch + 1) a.qoff[c] = a.toff[c * a.tw];
  if (c <= a.nch) a.jparts[c] = (uint32_t)((a.toff[(c + 1) * a.tw] - a.toff[c * a.tw] + kCTile - 1) / kCTile);
}

// (cov, query index) into the chunk's range: per workgroup a rank per chunk
// (LDS atomics) on top of the (chunk, tile) offset from the scan; each
// query's chunk comes from the count kernel.  The tile is staged in LDS in
// chunk order, then written out slot by slot, so a wave's stores are runs of
// consecutive addresses.  A workgroup takes kSub sub-tiles of one count-table
// column, each chunk's slots carried from one sub-tile to the next.  (Measured
// and removed: one 8-B store per query, 1.08 ms against 0.84 per 100M
// queries; the chunk searched again instead of read back, +0.27 ms; r05:
// sub-tiles of 4K queries at two workgroups per CU, 0.74 against 0.61 ms --
// the shorter runs cost more than the occupancy gains; the next sub-tile's
// loads issued before the write-out, no change; 8K-query sub-tiles at two
// workgroups per CU -- each staged entry carrying its chunk, the slots in
// registers, 80 KiB of LDS -- 0.64 ms: the write pattern, not occupancy,
// bounds this kernel.)
template <int kPer, int kSub>
__global__ __launch_bounds__(kQT) void k_q_scatter(ChunkArgs a) {
  constexpr uint32_t kT = kQT * kPer;
  __shared__ uint32_t hist[kMaxChunks + 1];  // counts, then the sub-tile's chunk offsets
  __shared__ uint32_t base[kMaxChunks + 1];  // each chunk's next slot (the tile's first, then carried)
  __shared__ uint2 stage[kT];
  __shared__ uint16_t cid[kT];
  __shared__ uint32_t wsum[kQT / 64 + 1];
  {
    const uint32_t col = tile_col(blockIdx.x, a.tw);
    for (uint32_t c = threadIdx.x; c <= a.nch; c += kQT) base[c] = (uint32_t)a.toff[(uint64_t)c * a.tw + col];
  }
  for (int sub = 0; sub < kSub; sub++) {
    const uint64_t t0 = ((uint64_t)blockIdx.x * kSub + sub) * kT;
    if (t0 >= a.ncov) break;  // (block-uniform)
    for (uint32_t i = threadIdx.x; i <= a.nch; i += kQT) hist[i] = 0;
    __syncthreads();
    const uint64_t q0 = t0 + threadIdx.x;
    uint32_t cv[kPer], ch[kPer], rk[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const uint64_t i = q0 + (uint64_t)k * kQT;
      ch[k] = 0xFFFFFFFFu;
      if (i < a.ncov) {
        cv[k] = a.cov[i];
        ch[k] = a.qchunk[i];
      }
    }
#pragma unroll
    for (int k = 0; k < kPer; k++)
      if (ch[k] != 0xFFFFFFFFu) rk[k] = atomicAdd(&hist[ch[k]], 1u);
    __syncthreads();
    // per thread kPerT consecutive chunks: the (chunk, tile) base and the
    // exclusive scan of the counts (the chunk's first staging slot)
    constexpr uint32_t kPerT = (kMaxChunks + 1 + kQT - 1) / kQT;
    const uint32_t c0 = threadIdx.x * kPerT;
    uint32_t h[kPerT], run = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPerT; j++) {
      const uint32_t c = c0 + j;
      h[j] = c <= a.nch ? hist[c] : 0u;
      run += h[j];
    }
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t incl = sgd::wave_incl_add(run);
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    if (threadIdx.x < 64) {
      const uint32_t x = threadIdx.x < kQT / 64 ? wsum[threadIdx.x] : 0u;
      const uint32_t xi = sgd::wave_incl_add(x);
      if (threadIdx.x < kQT / 64) wsum[threadIdx.x] = xi - x;
    }
    __syncthreads();
    uint32_t off = wsum[wv] + incl - run;
#pragma unroll
    for (uint32_t j = 0; j < kPerT; j++) {
      const uint32_t c = c0 + j;
      if (c <= a.nch) hist[c] = off;
      off += h[j];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; k++)
      if (ch[k] != 0xFFFFFFFFu) {
        const uint32_t slot = hist[ch[k]] + rk[k];
        stage[slot] = make_uint2(cv[k], (uint32_t)(q0 + (uint64_t)k * kQT));
        cid[slot] = (uint16_t)ch[k];
      }
    __syncthreads();
    const uint32_t nv = (uint32_t)min<uint64_t>(kT, a.ncov - t0);
    for (uint32_t i = threadIdx.x; i < nv; i += kQT) {
      const uint32_t c = cid[i];
      a.grouped[base[c] + (i - hist[c])] = stage[i];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kPerT; j++)  // (the next sub-tile's slots follow this one's)
      if (c0 + j <= a.nch) base[c0 + j] += h[j];
  }
}

// Queries in PC order (a canonical cover.Cover, as html.go:177-189 passes:
// one input's cover or a cover.Union): every chunk's queries are already a
// contiguous range, found by a search, and nothing is regrouped.
// k_q_sorted: flag = 1 if some query's PC is below its predecessor's (16
// consecutive queries per thread: four 16-B loads and the predecessor's).
__global__ void k_q_sorted(ChunkArgs a, uint32_t* flag) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 16;
  const bool al = ((uintptr_t)a.cov & 15) == 0;
  bool bad = false;
  for (uint64_t i0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; i0 < a.ncov; i0 += stride) {
    uint32_t v[16];
    if (al && i0 + 16 <= a.ncov) {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint4 x = reinterpret_cast<const uint4*>(a.cov + i0)[q];
        v[4 * q] = x.x;
        v[4 * q + 1] = x.y;
        v[4 * q + 2] = x.z;
        v[4 * q + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; q++) v[q] = i0 + q < a.ncov ? a.cov[i0 + q] : a.cov[a.ncov - 1];
    }
    uint64_t prev = i0 ? query_pc(a.hi32, a.cov[i0 - 1]) : 0;
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const uint64_t pc = query_pc(a.hi32, v[q]);
      bad |= pc < prev;
      prev = pc;
    }
  }
  if (__syncthreads_or(bad) && threadIdx.x == 0) atomicOr(flag, 1u);  // (one atomic per workgroup)
}

// sorted queries: qoff[c] = queries with pc <= bnd[c - 1], and the jobs per chunk
__global__ void k_q_direct_off(ChunkArgs a) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c > (uint64_t)a.nch + 1) return;
  uint64_t q = a.ncov;
  if (c == 0) {
    q = 0;
  } else if (c <= a.nch) {
    const uint64_t x = a.bnd[c - 1];
    uint64_t lo = 0, hi = a.ncov;  // first query with pc > x
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (query_pc(a.hi32, a.cov[mid]) <= x)
        lo = mid + 1;
      else
        hi = mid;
    }
    q = lo;
  }
  a.qoff[c] = q;
}

__global__ void k_q_parts(ChunkArgs a) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c <= a.nch) a.jparts[c] = (uint32_t)((a.qoff[c + 1] - a.qoff[c] + kCTile - 1) / kCTile);
}

// last chunk c with qoff[c] <= p (qoff non-decreasing, qoff[0] = 0; also the
// chunk of job p over jstart)
__device__ __forceinline__ uint32_t chunk_of_pos(const uint64_t* qoff, uint32_t nch, uint64_t p) {
  uint32_t lo = 0, hi = nch;  // chunks 0 .. nch
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (qoff[mid] <= p)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

// One job per kCTile grouped queries of one chunk: the chunk's sites,
// their symbols and the chunk's radix index over them, and the symbols its PC
// range can land in, into LDS.  Each query finds its call site through the
// index (the delete, cover.go:299); a query at a call site takes the site's
// symbol (cover.go:278-285), any other searches the held symbols.  First
// query per symbol and last deleting query per site are LDS atomics, flushed
// with one global atomic per touched symbol / site.
template <bool kDirect>
__global__ __launch_bounds__(kCT) void k_q_chunk(ChunkArgs a) {
  __shared__ uint64_t site[kSites];
  __shared__ uint32_t ldel[kSites];
  __shared__ uint16_t srel[kSites];  // site's symbol - the chunk's first held symbol (0xFFFF: none)
  __shared__ uint16_t sidx[kSiteIdx + 1];
  __shared__ uint64_t s_end[kSymCap], s_start[kSymCap];
  __shared__ uint32_t fq[kSymCap];
  // job: part `part` (kCTile queries) of chunk c
  const uint32_t j = blockIdx.x;
  if (j >= a.jstart[a.nch + 1]) return;
  const uint32_t c = chunk_of_pos(a.jstart, a.nch, j);
  {
    const uint64_t p = a.qoff[c] + (uint64_t)(j - a.jstart[c]) * kCTile;
    const uint64_t e = min<uint64_t>(a.qoff[c + 1], p + kCTile);
    const uint64_t sbase = (uint64_t)c * kSites;
    const uint32_t m = c < a.nch ? (uint32_t)min<uint64_t>(kSites, a.npcs - sbase) : 0u;
    const uint2 sr = a.symr[c];
    const uint32_t shi = sr.y < a.nsym ? sr.y : (uint32_t)a.nsym - 1;  // last symbol held
    const uint32_t nsl = sr.x <= shi && sr.x < a.nsym ? shi - sr.x + 1 : 0u;
    const bool sym_lds = nsl <= kSymCap;
    const uint64_t s0 = m ? a.pcs[sbase] : 0;
    const uint32_t ssh = m ? a.ssh[c] : 0;
    for (uint32_t i = threadIdx.x; i < m; i += kCT) {
      site[i] = a.pcs[sbase + i];
      ldel[i] = 0;
      const uint32_t y = a.ssym[sbase + i];
      srel[i] = sym_lds && y < a.nsym ? (uint16_t)(y - sr.x) : (uint16_t)0xFFFF;
    }
    if (m)
      for (uint32_t k = threadIdx.x; k <= kSiteIdx; k += kCT) sidx[k] = a.sidx[(uint64_t)c * (kSiteIdx + 1) + k];
    if (sym_lds)
      for (uint32_t i = threadIdx.x; i < nsl; i += kCT) {
        s_end[i] = a.send[sr.x + i];
        s_start[i] = a.sstart[sr.x + i];
        fq[i] = 0xFFFFFFFFu;
      }
    __syncthreads();
    // a query's call site (exact: pc is site j) and symbol (hit: pc inside
    // symbol sym -- an index into the held symbols, or a global index when
    // they are not held)
    auto lookup = [&](uint64_t pc, uint32_t& j, bool& exact, bool& hit, uint64_t& sym) {
      j = 0;
      exact = false;
      if (m && pc >= s0) {
        const uint64_t k = (pc - s0) >> ssh;
        if (k < kSiteIdx) {  // (past the index: above the chunk's last site)
          j = lds_lb(site, sidx[k], sidx[k + 1], pc);
          exact = j < m && site[j] == pc;
        }
      }
      if (sym_lds) {
        uint32_t k;
        if (exact) {
          k = srel[j];
        } else {
          // upper_bound(send, pc) lies in [sr.x, sr.y]; within the held symbols
          // it is sr.x + (held ends <= pc), and sr.y (maybe nsym) past them
          k = 0;
          for (uint32_t step = 1u << (31 - __builtin_clz(nsl | 1)); step; step >>= 1)
            if (k + step <= nsl && s_end[k + step - 1] <= pc) k += step;
        }
        hit = k < nsl && pc >= s_start[k];  // (pc < end: pc <= end holds)
        sym = k;
      } else {
        const uint64_t idx = exact ? a.ssym[sbase + j] : ub_idx(a.send, a.nsym, a.iend, pc);
        hit = idx < a.nsym && pc >= a.sstart[idx] && pc <= a.send[idx];
        sym = idx;
      }
    };
    auto first_query = [&](uint64_t sym, uint32_t qi) {
      if (sym_lds) {
        if (fq[sym] > qi) atomicMin(&fq[sym], qi);
      } else if (a.first_q[sym] > qi) {
        atomicMin(&a.first_q[sym], qi);
      }
    };
    if (!kDirect) {
      // four queries per thread per step, the next step's loads in flight
      // while this one's are looked up
      constexpr int kU = 4;
      uint2 gn[kU];
      auto load = [&](uint64_t i0) {
#pragma unroll
        for (int u = 0; u < kU; u++) {
          const uint64_t i = i0 + (uint64_t)u * kCT;
          gn[u] = a.grouped[i < e ? i : p];
        }
      };
      load(p + threadIdx.x);
      for (uint64_t i0 = p + threadIdx.x; i0 < e; i0 += (uint64_t)kU * kCT) {
        uint2 gq[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) gq[u] = gn[u];
        load(i0 + (uint64_t)kU * kCT);
#pragma unroll
        for (int u = 0; u < kU; u++) {
          if (i0 + (uint64_t)u * kCT >= e) break;
          const uint2 g = gq[u];
          uint32_t j;
          bool exact, hit;
          uint64_t sym;
          lookup(query_pc(a.hi32, g.x), j, exact, hit, sym);
          if (hit) first_query(sym, g.y);
          if (hit && exact && ldel[j] < g.y + 1) atomicMax(&ldel[j], g.y + 1);
        }
      }
    } else {
      // Queries in PC order: each thread takes a contiguous run, so a PC
      // repeated by the next query reuses its lookup, a symbol's first query
      // in the run is its only minimum candidate (symbols are non-decreasing
      // in PC), and a site's last deleting query in the run is flushed once,
      // when the PC moves on.
      const uint64_t per = (e - p + kCT - 1) / kCT;
      const uint64_t b0 = min<uint64_t>(p + threadIdx.x * per, e), b1 = min<uint64_t>(b0 + per, e);
      uint64_t prev = 0, psym = ~0ull;
      bool have = false, pdel = false;
      uint32_t pj = 0, pmax = 0;
      for (uint64_t i0 = b0; i0 < b1; i0 += 4) {
        uint32_t cv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) cv[u] = i0 + u < b1 ? a.cov[i0 + u] : 0u;
#pragma unroll
        for (int u = 0; u < 4; u++) {
          if (i0 + u >= b1) break;
          const uint32_t qi = (uint32_t)(i0 + u);
          const uint64_t pc = query_pc(a.hi32, cv[u]);
          if (have && pc == prev) {
            pmax = qi + 1;
            continue;
          }
          if (pdel && ldel[pj] < pmax) atomicMax(&ldel[pj], pmax);
          uint32_t j;
          bool exact, hit;
          uint64_t sym;
          lookup(pc, j, exact, hit, sym);
          if (hit && sym != psym) {
            first_query(sym, qi);
            psym = sym;
          }
          have = true;
          prev = pc;
          pdel = hit && exact;
          pj = j;
          pmax = qi + 1;
        }
      }
      if (pdel && ldel[pj] < pmax) atomicMax(&ldel[pj], pmax);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < m; i += kCT)
      if (ldel[i]) atomicMax(&a.last_del[sbase + i], ldel[i]);
    if (sym_lds)
      for (uint32_t i = threadIdx.x; i < nsl; i += kCT)
        if (fq[i] != 0xFFFFFFFFu) atomicMin(&a.first_q[sr.x + i], fq[i]);
  }
}

// per symbol, the first symbol with the same start (handledFuncs is keyed by
// start, cover.go:288)
__global__ void k_sym_leader(RepArgs a) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < a.nsym) a.leader[s] = (uint32_t)lb_idx(a.sstart, a.nsym, a.istart, a.sstart[s]);
}

__global__ void k_rep_group(RepArgs a) {
  uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.nsym) return;
  uint32_t f = a.first_q[s];
  if (f == 0xFFFFFFFFu) return;
  atomicMin((unsigned long long*)&a.group_first[a.leader[s]], ((unsigned long long)f << 32) | (unsigned long long)s);
}

__global__ void k_rep_final(RepArgs a) {
  uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.npcs) return;
  uint64_t c = a.pcs[j];
  int64_t best = -1;  // latest add time
  uint64_t g = ub_idx(a.sstart, a.nsym, a.istart, c);  // symbols [0, g) have start <= c
  while (g > 0) {
    uint64_t last = g - 1;                 // last symbol of the group
    if (a.send[last] < c) break;           // ends non-decreasing: nothing earlier reaches c
    uint64_t leader = a.leader[last];
    uint64_t gf = a.group_first[leader];
    if (gf != ~0ull) {
      uint32_t sym = (uint32_t)gf;
      if (c >= a.sstart[sym] && c <= a.send[sym]) best = max(best, (int64_t)(gf >> 32));
    }
    g = leader;
  }
  a.flag[j] = best >= 0 && (int64_t)a.last_del[j] <= best ? 1 : 0;
}

__global__ __launch_bounds__(kBlock) void k_flag_mask(const uint8_t* __restrict__ flag, uint64_t n, uint64_t nchunks,
                                                      uint64_t* __restrict__ mask, uint32_t* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  uint64_t c = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  uint32_t bits = 0;
  for (int q = 0; q < 4; q++) {
    uint64_t u = c * kChunk + lane * 4 + q;
    if (u < n && flag[u]) bits |= 1u << q;
  }
  uint64_t b0 = __ballot(bits & 1u), b1 = __ballot(bits & 2u), b2 = __ballot(bits & 4u), b3 = __ballot(bits & 8u);
  uint64_t mine = lane == 0 ? b0 : lane == 1 ? b1 : lane == 2 ? b2 : b3;
  if (lane < 4) mask[c * 4 + lane] = mine;
  if (lane == 0) cnt[c] = __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
}

__global__ __launch_bounds__(kBlock) void k_scatter_u64(const uint64_t* __restrict__ vals, uint64_t n,
                                                        const uint64_t* __restrict__ mask,
                                                        const uint64_t* __restrict__ base, uint64_t nchunks,
                                                        uint64_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  uint64_t c = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  uint64_t m[4] = {mask[c * 4], mask[c * 4 + 1], mask[c * 4 + 2], mask[c * 4 + 3]};
  uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t below = __popcll(m[0] & lt) + __popcll(m[1] & lt) + __popcll(m[2] & lt) + __popcll(m[3] & lt);
  for (int k = 0; k < 4; k++) {
    if (!((m[k] >> lane) & 1ull)) continue;
    uint32_t r = below;
    for (int q = 0; q < k; q++) r += (uint32_t)((m[q] >> lane) & 1ull);
    out[base[c] + r] = vals[c * kChunk + lane * 4 + k];
  }
}

}  // namespace sg

using namespace sg;

extern "C" {

int sg_cover_uncovered(sg_ctx* ctx, const uint32_t* cov, size_t ncov, uint32_t base, const uint64_t* sym_start,
                       const uint64_t* sym_end, size_t nsym, const uint64_t* all_pcs, size_t nall, uint64_t* out,
                       size_t* nout) {
  if (!ctx || !nout || (ncov && !cov) || (nsym && (!sym_start || !sym_end)) || (nall && (!all_pcs || !out)))
    return SG_EINVAL;
  *nout = 0;
  if (ncov >= 0xFFFFFFFFull || nsym >= 0xFFFFFFFFull || nall >= 0xFFFFFFFFull) {
    set_error("sg_cover_uncovered: too many PCs, symbols or call sites for one call");
    return SG_EINVAL;
  }
  for (size_t s = 1; s < nsym; s++)
    if (sym_start[s] < sym_start[s - 1] || sym_end[s] < sym_end[s - 1]) {
      set_error("sg_cover_uncovered: symbols must be sorted by start with non-decreasing ends");
      return SG_EINVAL;
    }
  for (size_t j = 1; j < nall; j++)
    if (all_pcs[j] <= all_pcs[j - 1]) {
      set_error("sg_cover_uncovered: call-site PCs must be sorted and unique");
      return SG_EINVAL;
    }
  if (ncov == 0 || nsym == 0 || nall == 0) return SG_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  uint64_t ntiles = (nall + kTile - 1) / kTile, nchunks = ntiles * kChunksPerTile;
  WsPlan p;
  size_t o_cov = p.add(ncov * 4), o_ss = p.add(nsym * 8), o_se = p.add(nsym * 8), o_pcs = p.add(nall * 8),
         o_fq = p.add(nsym * 4), o_gf = p.add(nsym * 8), o_ld = p.add(nall * 4), o_fl = p.add(nall),
         o_m = p.add(nchunks * 32), o_c = p.add(nchunks * 4), o_b = p.add((nchunks + 1) * 8),
         o_out = p.add(nall * 8), o_qb = p.add(((ncov + 63) / 64) * 8);

  // radix indexes: about one entry per bucket, at most 2^20 buckets (4 MiB: one XCD L2)
  auto plan_idx = [](uint64_t n, uint64_t lo, uint64_t hi, RadixIdx& I) {
    uint32_t nb = 1024;
    while (nb < (1u << 20) && nb < n) nb <<= 1;
    uint32_t sh = 0;
    while (sh < 63 && ((hi - lo) >> sh) >= nb) sh++;
    I.lo = lo;
    I.sh = sh;
    I.nb = nb;
  };
  RadixIdx iend{}, ipcs{}, istart{};
  plan_idx(nsym, sym_end[0], sym_end[nsym - 1], iend);
  plan_idx(nall, all_pcs[0], all_pcs[nall - 1], ipcs);
  plan_idx(nsym, sym_start[0], sym_start[nsym - 1], istart);
  const size_t o_ie = p.add(((uint64_t)iend.nb + 1) * 4), o_ip = p.add(((uint64_t)ipcs.nb + 1) * 4),
               o_is = p.add(((uint64_t)istart.nb + 1) * 4), o_ld2 = p.add(nsym * 4);
  // chunked query path (k_q_*) up to kMaxChunks chunks of call sites, the
  // per-query search passes (k_rep_first / k_rep_del) past them;
  // option report_direct 1 takes the latter at any size (a test hook for the
  // > 16M-site regime)
  const bool chunked = nall <= (uint64_t)kSites * kMaxChunks && ctx->opt[kOptReportDirect] <= 0;
  const uint32_t nch = div_up(nall, kSites);
  // query tiles: 64K queries per count / scatter workgroup
  const uint32_t ntq = div_up(ncov, (uint64_t)kQT * kSQPer * kSQSub);
  const uint32_t tw = 8 * div_up(ntq, 8);
  const uint64_t ntc = chunked ? ((uint64_t)nch + 1) * tw : 1;
  const size_t o_bnd = p.add((uint64_t)nch * 8), o_sr = p.add(((uint64_t)nch + 1) * 8),
               o_qo = p.add(((uint64_t)nch + 2) * 8), o_gq = p.add(chunked ? ncov * 8 : 8),
               o_ci = p.add(((uint64_t)kChunkIdx + 1) * 2), o_sh = p.add((uint64_t)nch * 4),
               o_si = p.add((uint64_t)nch * (kSiteIdx + 1) * 2), o_sy = p.add(chunked ? nall * 4 : 4),
               o_tc = p.add(ntc * 4), o_to = p.add((ntc + 1) * 8), o_jp = p.add(((uint64_t)nch + 1) * 4),
               o_js = p.add(((uint64_t)nch + 2) * 8), o_srt = p.add(4);
  // the count kernel's per-query chunks, read back by the scatter
  const size_t o_qc = p.add(chunked ? ncov * 2 : 2);
  size_t scan_off = p.total;
  rc = ws_reserve(ctx, p.total + std::max(scan_ws_bytes(nchunks), scan_ws_bytes(ntc)));
  if (rc) return rc;
  RepArgs a{};
  a.cov = (uint32_t*)ws_at(ctx, o_cov);
  a.ncov = ncov;
  a.base = base;
  a.sstart = (uint64_t*)ws_at(ctx, o_ss);
  a.send = (uint64_t*)ws_at(ctx, o_se);
  a.nsym = nsym;
  a.pcs = (uint64_t*)ws_at(ctx, o_pcs);
  a.npcs = nall;
  a.first_q = (uint32_t*)ws_at(ctx, o_fq);
  a.group_first = (uint64_t*)ws_at(ctx, o_gf);
  a.last_del = (uint32_t*)ws_at(ctx, o_ld);
  a.flag = (uint8_t*)ws_at(ctx, o_fl);
  a.qbits = (uint64_t*)ws_at(ctx, o_qb);
  uint64_t* mask = (uint64_t*)ws_at(ctx, o_m);
  uint32_t* cnt = (uint32_t*)ws_at(ctx, o_c);
  uint64_t* bs = (uint64_t*)ws_at(ctx, o_b);
  uint64_t* dout = (uint64_t*)ws_at(ctx, o_out);
  iend.r = (const uint32_t*)ws_at(ctx, o_ie);
  ipcs.r = (const uint32_t*)ws_at(ctx, o_ip);
  istart.r = (const uint32_t*)ws_at(ctx, o_is);
  a.iend = iend;
  a.ipcs = ipcs;
  a.istart = istart;
  a.leader = (uint32_t*)ws_at(ctx, o_ld2);
  SG_HIP(hipMemcpyAsync((void*)a.cov, cov, ncov * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync((void*)a.sstart, sym_start, nsym * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync((void*)a.send, sym_end, nsym * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync((void*)a.pcs, all_pcs, nall * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemsetAsync(a.first_q, 0xFF, nsym * 4, ctx->stream));
  SG_HIP(hipMemsetAsync(a.group_first, 0xFF, nsym * 8, ctx->stream));
  SG_HIP(hipMemsetAsync(a.last_del, 0, nall * 4, ctx->stream));

  {
    ScopedTimer tm(ctx, "report_index");
    hipLaunchKernelGGL(k_radix_index, dim3(div_up((uint64_t)iend.nb + 1, 256)), dim3(256), 0, ctx->stream, a.send,
                       (uint64_t)nsym, iend.lo, iend.sh, iend.nb, (uint32_t*)iend.r);
    hipLaunchKernelGGL(k_radix_index, dim3(div_up((uint64_t)ipcs.nb + 1, 256)), dim3(256), 0, ctx->stream, a.pcs,
                       (uint64_t)nall, ipcs.lo, ipcs.sh, ipcs.nb, (uint32_t*)ipcs.r);
    hipLaunchKernelGGL(k_radix_index, dim3(div_up((uint64_t)istart.nb + 1, 256)), dim3(256), 0, ctx->stream,
                       a.sstart, (uint64_t)nsym, istart.lo, istart.sh, istart.nb, (uint32_t*)istart.r);
    hipLaunchKernelGGL(k_sym_leader, dim3(div_up(nsym, 256)), dim3(256), 0, ctx->stream, a);
  }
  if (chunked) {
    ChunkArgs k{};
    k.cov = a.cov;
    k.ncov = ncov;
    k.hi32 = (uint64_t)base << 32;
    k.pcs = a.pcs;
    k.npcs = nall;
    k.sstart = a.sstart;
    k.send = a.send;
    k.nsym = nsym;
    k.iend = iend;
    k.nch = nch;
    k.bnd = (uint64_t*)ws_at(ctx, o_bnd);
    k.cidx = (uint16_t*)ws_at(ctx, o_ci);
    k.ssh = (uint32_t*)ws_at(ctx, o_sh);
    k.sidx = (uint16_t*)ws_at(ctx, o_si);
    k.ssym = (uint32_t*)ws_at(ctx, o_sy);
    {  // radix shift over [bnd[0], bnd[nch - 1]]
      const uint64_t b0 = all_pcs[std::min<uint64_t>(kSites, nall) - 1], span = all_pcs[nall - 1] - b0;
      uint32_t sh = 0;
      while (sh < 63 && (span >> sh) >= kChunkIdx) sh++;
      k.csh = sh;
    }
    k.symr = (uint2*)ws_at(ctx, o_sr);
    k.ntiles = ntq;
    k.tw = tw;
    k.jparts = (uint32_t*)ws_at(ctx, o_jp);
    k.jstart = (uint64_t*)ws_at(ctx, o_js);
    k.tcount = (uint32_t*)ws_at(ctx, o_tc);
    k.toff = (uint64_t*)ws_at(ctx, o_to);
    k.qoff = (uint64_t*)ws_at(ctx, o_qo);
    k.grouped = (uint2*)ws_at(ctx, o_gq);
    k.qchunk = (uint16_t*)ws_at(ctx, o_qc);
    k.first_q = a.first_q;
    k.last_del = a.last_del;
    // queries in PC order (the reference's canonical covers) need no regrouping
    uint32_t* dsorted = (uint32_t*)ws_at(ctx, o_srt);
    uint32_t unsorted = 1;
    {
      // a prefix first: queries in random order show it within the first few
      // (one 4 MiB read instead of the whole 400 MB), sorted ones go on to the
      // full check
      ScopedTimer tm(ctx, "report_sorted_q");
      const uint64_t pre = std::min<uint64_t>(ncov, 1u << 20);
      for (uint64_t lim : {pre, (uint64_t)ncov}) {
        ChunkArgs kp = k;
        kp.ncov = lim;
        SG_HIP(hipMemsetAsync(dsorted, 0, 4, ctx->stream));
        hipLaunchKernelGGL(k_q_sorted, dim3(std::min<uint32_t>(div_up(lim, 256 * 16), 8192)), dim3(256), 0,
                           ctx->stream, kp, dsorted);
        SG_HIP(hipMemcpyAsync(&unsorted, dsorted, 4, hipMemcpyDeviceToHost, ctx->stream));
        SG_HIP(hipStreamSynchronize(ctx->stream));
        if (unsorted || lim == (uint64_t)ncov) break;
      }
    }
    if (!unsorted) {
      ScopedTimer tm(ctx, "report_count_q");
      hipLaunchKernelGGL(k_chunk_prep, dim3(div_up((uint64_t)nch + 1, 256)), dim3(256), 0, ctx->stream, k);
      hipLaunchKernelGGL(k_site_sym, dim3(div_up(nall, 256)), dim3(256), 0, ctx->stream, k);
      hipLaunchKernelGGL(k_site_index, dim3(div_up((uint64_t)nch * (kSiteIdx + 1), 256)), dim3(256), 0, ctx->stream,
                         k);
      hipLaunchKernelGGL(k_q_direct_off, dim3(div_up((uint64_t)nch + 2, 256)), dim3(256), 0, ctx->stream, k);
      hipLaunchKernelGGL(k_q_parts, dim3(div_up((uint64_t)nch + 1, 256)), dim3(256), 0, ctx->stream, k);
      rc = scan_counts(ctx, k.jparts, k.jstart, (uint64_t)nch + 1, scan_off);
      if (rc) return rc;
    }
    if (unsorted) {
      ScopedTimer tm(ctx, "report_count_q");
      hipLaunchKernelGGL(k_chunk_prep, dim3(div_up((uint64_t)nch + 1, 256)), dim3(256), 0, ctx->stream, k);
      hipLaunchKernelGGL(k_chunk_index, dim3(div_up((uint64_t)kChunkIdx + 1, 256)), dim3(256), 0, ctx->stream, k);
      hipLaunchKernelGGL(k_site_sym, dim3(div_up(nall, 256)), dim3(256), 0, ctx->stream, k);
      hipLaunchKernelGGL(k_site_index, dim3(div_up((uint64_t)nch * (kSiteIdx + 1), 256)), dim3(256), 0, ctx->stream,
                         k);
      if (tw != ntq) SG_HIP(hipMemsetAsync(k.tcount, 0, ntc * 4, ctx->stream));  // (the padding columns)
      hipLaunchKernelGGL((k_q_count<kSQPer, kSQSub>), dim3(ntq), dim3(kQT), 0, ctx->stream, k);
      rc = scan_counts(ctx, k.tcount, k.toff, ntc, scan_off);
      if (rc) return rc;
      hipLaunchKernelGGL(k_q_chunk_off, dim3(div_up((uint64_t)nch + 2, 256)), dim3(256), 0, ctx->stream, k);
      rc = scan_counts(ctx, k.jparts, k.jstart, (uint64_t)nch + 1, scan_off);
      if (rc) return rc;
    }
    if (unsorted) {
      ScopedTimer tm(ctx, "report_scatter_q");
      hipLaunchKernelGGL((k_q_scatter<kSQPer, kSQSub>), dim3(ntq), dim3(kQT), 0, ctx->stream, k);
    }
    {
      ScopedTimer tm(ctx, "report_chunks");
      // jobs: sum over chunks of ceil(count / kCTile) <= ncov / kCTile + nch + 1
      const dim3 jgrid(div_up(ncov, kCTile) + nch + 1);
      if (unsorted)
        hipLaunchKernelGGL(k_q_chunk<false>, jgrid, dim3(kCT), 0, ctx->stream, k);
      else
        hipLaunchKernelGGL(k_q_chunk<true>, jgrid, dim3(kCT), 0, ctx->stream, k);
    }
  } else {
    const dim3 qgrid((uint32_t)std::min<uint64_t>(div_up(ncov, 256), 16384));
    {
      ScopedTimer tm(ctx, "report_first");
      hipLaunchKernelGGL(k_rep_first, qgrid, dim3(256), 0, ctx->stream, a);
    }
    {
      ScopedTimer tm(ctx, "report_del");
      hipLaunchKernelGGL(k_rep_del, qgrid, dim3(256), 0, ctx->stream, a);
    }
  }
  {
    ScopedTimer tm(ctx, "report_sites");
    hipLaunchKernelGGL(k_rep_group, dim3(div_up(nsym, 256)), dim3(256), 0, ctx->stream, a);
    hipLaunchKernelGGL(k_rep_final, dim3(div_up(nall, 256)), dim3(256), 0, ctx->stream, a);
    hipLaunchKernelGGL(k_flag_mask, dim3(div_up(nchunks, kBlock / 64)), dim3(kBlock), 0, ctx->stream, a.flag,
                       (uint64_t)nall, nchunks, mask, cnt);
    rc = scan_counts(ctx, cnt, bs, nchunks, scan_off);
    if (rc) return rc;
    hipLaunchKernelGGL(k_scatter_u64, dim3(div_up(nchunks, kBlock / 64)), dim3(kBlock), 0, ctx->stream, a.pcs,
                       (uint64_t)nall, mask, bs, nchunks, dout);
  }
  SG_HIP(hipGetLastError());
  uint64_t total = 0;
  SG_HIP(hipMemcpyAsync(&total, bs + nchunks, 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (total) SG_HIP(hipMemcpyAsync(out, dout, total * 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  *nout = (size_t)total;
  return SG_OK;
}

}  // extern "C"
