// sg_merge.hip -- sorted-slice algebra of pkg/cover on the GPU.
//
// Reference: pkg/cover/cover.go:28-40 Canonicalize, :42-102 Difference /
// SymmetricDifference / Union / Intersection via foreach, :106-117
// HasDifference.
//
// foreach (cover.go:81-102) is a two-pointer walk that, for a value v seen a
// times in cov0 and b times in cov1, emits max(a,b) (Union), min(a,b)
// (Intersection), max(a-b,0) (Difference) or |a-b| (SymmetricDifference)
// copies, and drops every 0xFFFFFFFF.  Here every element decides on its own:
// element i of one list, the t-th copy of its value there (t = i - first
// index of the value), is kept iff t < or >= the value's count in the other
// list (binary searches), and lands at
//   (kept elements of its own list before it) + (kept elements of the other
//   list with a smaller value; ties: cov0's copies first)
// so any pair size runs fully parallel with one ballot-mask compaction.
//
// Canonicalize = segmented sort (4096-value LDS bitonic tiles, then rank-merge
// passes for longer segments) + unique in place.  `last` starts at sent
// (cover.go:31), so a value is kept iff it differs from its predecessor, the
// first one iff it is not 0xFFFFFFFF.  The tail beyond the canonical length
// keeps the sorted values, exactly like Go's in-place loop.
#include "sg_internal.h"

#include <algorithm>
#include <numeric>

namespace sg {

constexpr uint32_t kSent = 0xFFFFFFFFu;  // cover.go:17

__device__ __forceinline__ uint64_t lower_bound(const uint32_t* a, uint64_t n, uint32_t v) {
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
__device__ __forceinline__ uint64_t upper_bound(const uint32_t* a, uint64_t n, uint32_t v) {
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

// number of mask bits at positions < p (masks in chunk-ballot layout)
__device__ __forceinline__ uint64_t mask_prefix(const uint64_t* mask, const uint64_t* base, uint64_t nchunks,
                                                uint64_t p) {
  uint64_t c = p / kChunk;
  if (c >= nchunks) return base[nchunks];
  uint32_t q = (uint32_t)(p % kChunk);
  uint64_t acc = base[c];
  for (int k = 0; k < 4; k++) {
    int lim = q > (uint32_t)k ? (int)((q - k + 3) / 4) : 0;
    uint64_t lm = lim >= 64 ? ~0ull : ((1ull << lim) - 1);
    acc += __popcll(mask[c * 4 + k] & lm);
  }
  return acc;
}

__device__ __forceinline__ bool mask_bit(const uint64_t* mask, uint64_t u) {
  uint64_t c = u / kChunk;
  uint32_t q = (uint32_t)(u % kChunk);
  return (mask[c * 4 + (q & 3)] >> (q >> 2)) & 1ull;
}

// element u of a chunk-ballot space: chunk c = u/256, lane = (u%256)/4, k = u%4
struct Side {
  const uint32_t* v;     // values
  const uint64_t* beg;   // per pair
  const uint64_t* len;
  const uint64_t* off;   // exclusive scan of len (npair+1): virtual element space
};

struct MergeArgs {
  int op;
  Side a, b;
  uint64_t npair;
  uint64_t* mask[2];
  uint32_t* cnt[2];
  uint64_t* base[2];
  uint64_t nchunks[2];
  uint32_t* out;
  const uint64_t* out_beg;
  uint64_t* out_len;
};

template <int kSide>  // 0: cov0 (a), 1: cov1 (b)
__device__ __forceinline__ bool merge_keep(const MergeArgs& m, uint64_t u, uint64_t& k, uint32_t& x) {
  const Side& me = kSide == 0 ? m.a : m.b;
  const Side& ot = kSide == 0 ? m.b : m.a;
  k = sgd::seg_search(me.off, 0, m.npair - 1, u);
  uint64_t i = u - me.off[k];
  const uint32_t* mine = me.v + me.beg[k];
  x = mine[i];
  if (x == kSent) return false;  // cover.go:97
  const uint32_t* other = ot.v + ot.beg[k];
  uint64_t on = ot.len[k];
  uint64_t t = i - lower_bound(mine, i, x);
  uint64_t c = upper_bound(other, on, x) - lower_bound(other, on, x);
  switch (m.op) {
    case SG_OP_DIFFERENCE: return kSide == 0 && t >= c;
    case SG_OP_INTERSECT: return kSide == 0 && t < c;
    case SG_OP_UNION: return kSide == 0 ? true : t >= c;
    default: return t >= c;  // SG_OP_SYMDIFF
  }
}

template <int kSide>
__global__ __launch_bounds__(kBlock) void k_merge_keep(MergeArgs m) {
  const int lane = threadIdx.x & 63;
  uint64_t c = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (c >= m.nchunks[kSide]) return;
  const Side& me = kSide == 0 ? m.a : m.b;
  uint64_t n = me.off[m.npair];
  uint32_t bits = 0;
  for (int q = 0; q < 4; q++) {
    uint64_t u = c * kChunk + lane * 4 + q;
    if (u >= n) continue;
    uint64_t k;
    uint32_t x;
    if (merge_keep<kSide>(m, u, k, x)) bits |= 1u << q;
  }
  uint64_t b0 = __ballot(bits & 1u), b1 = __ballot(bits & 2u), b2 = __ballot(bits & 4u), b3 = __ballot(bits & 8u);
  uint64_t mine = lane == 0 ? b0 : lane == 1 ? b1 : lane == 2 ? b2 : b3;
  if (lane < 4) m.mask[kSide][c * 4 + lane] = mine;
  if (lane == 0) m.cnt[kSide][c] = __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
}

template <int kSide>
__global__ void k_merge_scatter(MergeArgs m) {
  const Side& me = kSide == 0 ? m.a : m.b;
  const Side& ot = kSide == 0 ? m.b : m.a;
  uint64_t n = me.off[m.npair];
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += stride) {
    if (!mask_bit(m.mask[kSide], u)) continue;
    uint64_t k = sgd::seg_search(me.off, 0, m.npair - 1, u);
    uint64_t i = u - me.off[k];
    uint32_t x = me.v[me.beg[k] + i];
    uint64_t pos = mask_prefix(m.mask[kSide], m.base[kSide], m.nchunks[kSide], u) -
                   mask_prefix(m.mask[kSide], m.base[kSide], m.nchunks[kSide], me.off[k]);
    const uint32_t* other = ot.v + ot.beg[k];
    uint64_t j = kSide == 0 ? lower_bound(other, ot.len[k], x) : upper_bound(other, ot.len[k], x);
    if (m.nchunks[1 - kSide])
      pos += mask_prefix(m.mask[1 - kSide], m.base[1 - kSide], m.nchunks[1 - kSide], ot.off[k] + j) -
             mask_prefix(m.mask[1 - kSide], m.base[1 - kSide], m.nchunks[1 - kSide], ot.off[k]);
    m.out[m.out_beg[k] + pos] = x;
  }
}

// ---- one small side per pair (C1: traces against one large corpus signal) --
// Union / SymmetricDifference keep elements of both lists.  When one list of
// a pair fits in LDS (<= kMS values) a workgroup per pair does the whole
// merge: the small list S, its keep flags and kept-prefix live in LDS; the
// large list L streams through once in index order; each L element's count
// in S and its insertion point come from LDS searches, its rank from wave
// ballots; S's kept elements land when the L tile holding their insertion
// point is processed.  Same keep rule and positions as k_merge_keep /
// k_merge_scatter (copy t of a value against its count c in the other list;
// ties: cov0's copies first).
constexpr int kMS = 4096;               // max small side
// A pair takes the gap-copy path (k_merge_small) when the large side is at
// least this many times the small one (long gaps); dense interleavings (the
// corpus folds of similar-sized lists) merge tile by tile.
constexpr uint64_t kGapRatio = 32;
constexpr int kMT = 1024;               // threads
constexpr int kMU = kMS / kMT;          // small elements per thread (consecutive)
#ifndef SG_KML
#define SG_KML 8
#endif
constexpr int kML = SG_KML;             // large elements per thread per tile
constexpr int kMTile = kMT * kML;       // 8192
constexpr int kMWaves = kMT / 64;       // 16

struct SmallArgs {
  int op;
  const uint32_t* a;
  const uint32_t* b;
  const uint64_t* abeg;
  const uint64_t* alen;
  const uint64_t* bbeg;
  const uint64_t* blen;
  const uint64_t* obeg;
  uint64_t* olen;
  uint32_t* out;
};

__device__ __forceinline__ bool keep_rule(int op, int side, uint64_t t, uint64_t c) {
  switch (op) {
    case SG_OP_DIFFERENCE: return side == 0 && t >= c;
    case SG_OP_INTERSECT: return side == 0 && t < c;
    case SG_OP_UNION: return side == 0 ? true : t >= c;
    default: return t >= c;  // SG_OP_SYMDIFF
  }
}

// first index in p[0..n) with p[idx] >= v (kUpper: > v); all kN searches of a
// thread advance level by level so their loads are in flight together
template <int kN, bool kUpper, typename P>
__device__ __forceinline__ void multi_bound(P p, uint64_t n, const uint32_t (&v)[kN], uint64_t (&lo)[kN]) {
  // branch-free halving: the answer stays in [base, base + len]; len depends
  // only on n, so every search takes the same steps
  uint64_t base[kN];
#pragma unroll
  for (int u = 0; u < kN; u++) base[u] = 0;
  uint64_t len = n;
  while (len > 1) {
    const uint64_t half = len >> 1;
#pragma unroll
    for (int u = 0; u < kN; u++) {
      const uint32_t pv = p[base[u] + half];
      if (kUpper ? pv <= v[u] : pv < v[u]) base[u] += half;
    }
    len -= half;
  }
#pragma unroll
  for (int u = 0; u < kN; u++) {
    if (n == 0) {
      lo[u] = 0;
    } else {
      const uint32_t pv = p[base[u]];
      lo[u] = base[u] + ((kUpper ? pv <= v[u] : pv < v[u]) ? 1 : 0);
    }
  }
}

// #{j in [j0, ns): S[j] < x} + j0 (kLe: <= x) for sorted S in LDS, j0 below
// the answer: a wave's ballot per 64 candidates (the lanes where it holds
// are a prefix)
template <bool kLe>
__device__ __forceinline__ uint32_t ballot_count(const uint32_t* sv, uint32_t ns, uint32_t j0, uint32_t x, int lane) {
  for (;;) {
    const uint32_t j = j0 + (uint32_t)lane;
    const bool c = j < ns && (kLe ? sv[j] <= x : sv[j] < x);
    const uint64_t b = __ballot(c);
    if (b != ~0ull) return j0 + (uint32_t)__popcll(b);
    j0 += 64;
  }
}

// Difference / Intersection with every pair's first list of <= kMS values (C1:
// traces against one large corpus signal): a workgroup per pair keeps a's
// copy t of value x iff t >= (Difference) / < (Intersection) the count of x
// in b, i.e. iff b[lower_bound(b, x) + t] != x (resp. ==); t from a search of
// the staged a in LDS, the kept values written in order by a block scan (the
// sentinel never kept, cover.go:97).  One
// launch, no masks or global scan; each thread's four searches of b
// interleaved.
constexpr int kDU = 4;  // consecutive a elements per thread (kMT kDU = kMS)
static_assert(kMT * kDU == kMS, "k_diff_small covers a small side");
__global__ __launch_bounds__(kMT) void k_diff_small(SmallArgs m) {
  __shared__ uint32_t sv[kMS];
  __shared__ uint32_t wsum[kMWaves + 1];
  const uint32_t k = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t na = (uint32_t)m.alen[k];
  const uint64_t nb = m.blen[k];
  const uint32_t* A = m.a + m.abeg[k];
  const uint32_t* B = m.b + m.bbeg[k];
  uint32_t x[kDU];
#pragma unroll
  for (int u = 0; u < kDU; u++) {
    const uint32_t j = (uint32_t)tid * kDU + u;
    x[u] = j < na ? A[j] : 0u;
  }
#pragma unroll
  for (int u = 0; u < kDU; u++) {
    const uint32_t j = (uint32_t)tid * kDU + u;
    if (j < na) sv[j] = x[u];
  }
  __syncthreads();
  // t: the copy index of x among a's equal values (a sorted)
  uint32_t t[kDU];
#pragma unroll
  for (int u = 0; u < kDU; u++) {
    const uint32_t j = (uint32_t)tid * kDU + u;
    uint32_t lo = 0, hi = j < na ? j : 0;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (sv[mid] < x[u])
        lo = mid + 1;
      else
        hi = mid;
    }
    t[u] = j - lo;
  }
  // lower_bound(b, x), four searches in flight
  uint64_t lo[kDU], hi[kDU];
#pragma unroll
  for (int u = 0; u < kDU; u++) {
    lo[u] = 0;
    hi[u] = (uint32_t)tid * kDU + u < na ? nb : 0;
  }
  for (;;) {
    bool any = false;
    uint32_t v[kDU];
#pragma unroll
    for (int u = 0; u < kDU; u++) v[u] = lo[u] < hi[u] ? B[(lo[u] + hi[u]) >> 1] : 0u;
#pragma unroll
    for (int u = 0; u < kDU; u++)
      if (lo[u] < hi[u]) {
        const uint64_t mid = (lo[u] + hi[u]) >> 1;
        if (v[u] < x[u])
          lo[u] = mid + 1;
        else
          hi[u] = mid;
        any |= lo[u] < hi[u];
      }
    if (!any) break;
  }
  // the count of x in b exceeds t iff b[lo + t] == x
  uint32_t keep = 0, nk = 0;
#pragma unroll
  for (int u = 0; u < kDU; u++) {
    const uint32_t j = (uint32_t)tid * kDU + u;
    const uint64_t q = lo[u] + t[u];
    const bool more = j < na && q < nb && B[q] == x[u];
    const bool kp = j < na && x[u] != kSent && (m.op == SG_OP_DIFFERENCE ? !more : more);  // (cover.go:97)
    keep |= (kp ? 1u : 0u) << u;
    nk += kp ? 1u : 0u;
  }
  const uint32_t incl = sgd::wave_incl_add(nk);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (int i = 0; i < kMWaves; i++) {
      const uint32_t c = wsum[i];
      wsum[i] = acc;
      acc += c;
    }
    wsum[kMWaves] = acc;
  }
  __syncthreads();
  uint32_t at = wsum[w] + incl - nk;
  uint32_t* out = m.out + m.obeg[k];
#pragma unroll
  for (int u = 0; u < kDU; u++)
    if ((keep >> u) & 1u) out[at++] = x[u];
  if (tid == 0) m.olen[k] = wsum[kMWaves];
}

template <bool kGap>
__global__ __launch_bounds__(kMT) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_merge_small(SmallArgs m) {
  __shared__ uint32_t sv[kMS];
  __shared__ uint32_t sdx[kGap ? kMS : 1];  // gap path: dropped L elements of the values before element j's
  __shared__ uint16_t rll[kGap ? kMS : 1];  // gap path: last S index of each run (distinct value)
  __shared__ uint32_t red2[kMWaves + 1];
  __shared__ uint64_t nl_eff_s;
  __shared__ uint32_t skp[kMS + 1];    // kept small elements before j
  __shared__ uint32_t sidx[kMS];       // insertion point of small element j in L
  __shared__ unsigned long long tw[kGap ? 1 : kML * kMWaves];
  __shared__ uint32_t twp[kGap ? 1 : kML * kMWaves + 1];
  __shared__ uint32_t red[kMWaves + 1];
  const uint32_t k = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t na = m.alen[k], nb = m.blen[k];
  const int sS = na <= nb ? 0 : 1, sL = 1 - sS;  // side of S / L (0: cov0)
  const uint32_t* S = sS == 0 ? m.a + m.abeg[k] : m.b + m.bbeg[k];
  const uint32_t* L = sS == 0 ? m.b + m.bbeg[k] : m.a + m.abeg[k];
  const uint32_t ns = (uint32_t)(sS == 0 ? na : nb);
  const uint64_t nl = sS == 0 ? nb : na;
  uint32_t* out = m.out + m.obeg[k];
  for (uint32_t j = tid; j < ns; j += kMT) sv[j] = S[j];
  __syncthreads();
  // S: keep flags (copy t against the count in L) and insertion points in L
  uint32_t flags = 0;
  if ((nl >= kGapRatio * ns) != kGap) return;  // the other instantiation's pair
  constexpr bool gap = kGap;
  // gap path: L copies of a value S also holds are dropped up to S's count (the keep
  // rule for L's side: Union when L is cov1, SymmetricDifference)
  const bool ldrop = m.op == SG_OP_SYMDIFF || sL == 1;
  uint32_t rlast = 0;  // bit u: element u is the last copy of its value in S
  uint64_t dpk = 0;    // its value's dropped L copies, 16 bits per u
  {
    uint32_t x[kMU];
    uint64_t lb[kMU], ub[kMU];
#pragma unroll
    for (int u = 0; u < kMU; u++) {
      const uint32_t j = tid * kMU + u;
      x[u] = j < ns ? sv[j] : 0u;
    }
    multi_bound<kMU, false>(L, nl, x, lb);
    multi_bound<kMU, true>(L, nl, x, ub);
#pragma unroll
    for (int u = 0; u < kMU; u++) {
      const uint32_t j = tid * kMU + u;
      if (j >= ns) continue;
      uint64_t t = 0;
      if (j > 0 && sv[j - 1] == x[u]) {  // later copy: t = j - first index of the value
        uint32_t lo = 0, hi = j;
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (sv[mid] < x[u]) lo = mid + 1; else hi = mid;
        }
        t = j - lo;
      }
      const bool kp = x[u] != kSent && keep_rule(m.op, sS, t, ub[u] - lb[u]);  // cover.go:97
      flags |= (kp ? 1u : 0u) << u;
      if (gap) {
      sidx[j] = (uint32_t)lb[u];
      // the last copy of its value in S: the value's dropped L copies (the
      // first min(cS, cL), cS = t + 1) are counted here, so the exclusive
      // sum at any copy of a value excludes the value's own drops
      const bool last = j + 1 == ns || sv[j + 1] != x[u];
      if (last) {
        const uint64_t cl = ub[u] - lb[u];
        const uint32_t d = ldrop && x[u] != kSent ? (uint32_t)(cl < t + 1 ? cl : t + 1) : 0u;
        rlast |= 1u << u;
        dpk |= (uint64_t)d << (16 * u);
      }
      } else {
        sidx[j] = (uint32_t)(sS == 0 ? lb[u] : ub[u]);
      }
    }
  }
  {  // exclusive scan of the kept counts, thread order = element order
    const uint32_t c = __popc(flags);
    const uint32_t incl = sgd::wave_incl_add(c);
    if (lane == 63) red[w] = incl;
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      for (int i = 0; i < kMWaves; i++) {
        const uint32_t v = red[i];
        red[i] = acc;
        acc += v;
      }
      red[kMWaves] = acc;
    }
    __syncthreads();
    uint32_t base = red[w] + incl - c;
#pragma unroll
    for (int u = 0; u < kMU; u++) {
      const uint32_t j = tid * kMU + u;
      if (j < ns) skp[j] = base;
      base += (flags >> u) & 1u;
    }
    if (tid == 0) skp[ns] = red[kMWaves];
  }
  __syncthreads();
  const uint32_t KS = skp[ns];
  if (gap) {
    // L is S's values' runs and the gaps between them: every kept L element
    // of a gap moves by the same amount (kept S elements before it minus
    // dropped L elements before it), so the gaps are copied whole, as
    // coalesced streams, and the kept S elements are written on their own.
    // Equal values: S's kept copies go first (they are identical values).
    // L's sentinels (its sorted tail) are dropped (cover.go:97).
    if (tid == 0) {
      uint64_t lo = 0, hi = nl;  // first sentinel in L
      while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (L[mid] < kSent) lo = mid + 1; else hi = mid;
      }
      nl_eff_s = lo;
    }
    // exclusive scan of (run-last flag, drops): run ranks and drops before
    uint32_t c = 0;
#pragma unroll
    for (int u = 0; u < kMU; u++) c += ((rlast >> u) & 1u) + ((uint32_t)(dpk >> (16 * u)) & 0xFFFFu) * 65536u;
    const uint32_t incl = sgd::wave_incl_add(c);
    if (lane == 63) red2[w] = incl;
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      for (int i = 0; i < kMWaves; i++) {
        const uint32_t v = red2[i];
        red2[i] = acc;
        acc += v;
      }
      red2[kMWaves] = acc;
    }
    __syncthreads();
    uint32_t run = red2[w] + incl - c;
#pragma unroll
    for (int u = 0; u < kMU; u++) {
      const uint32_t j = tid * kMU + u;
      if (j < ns) {
        sdx[j] = run >> 16;  // drops of the values before j's
        if ((rlast >> u) & 1u) rll[run & 0xFFFFu] = (uint16_t)j;
      }
      run += ((rlast >> u) & 1u) + ((uint32_t)(dpk >> (16 * u)) & 0xFFFFu) * 65536u;
    }
    __syncthreads();
    const uint32_t nruns = red2[kMWaves] & 0xFFFFu, dtot = red2[kMWaves] >> 16;
    const uint64_t nle = nl_eff_s;
    // kept S elements
#pragma unroll
    for (int u = 0; u < kMU; u++) {
      const uint32_t j = tid * kMU + u;
      if (j < ns && ((flags >> u) & 1u)) out[(uint64_t)sidx[j] - sdx[j] + skp[j]] = sv[j];
    }
    // gaps: g = 0 before S's first value, g = r + 1 after run r; wave by wave
    for (uint32_t g = w; g <= nruns; g += kMWaves) {
      uint64_t a, b;
      int64_t sh;
      if (g == 0) {
        a = 0;
        b = ns ? sidx[0] : nle;
        sh = 0;
      } else {
        const uint32_t jl = rll[g - 1];
        const uint32_t dr = sdx[jl] + (jl + 1 < ns ? sdx[jl + 1] - sdx[jl] : dtot - sdx[jl]);  // drops through this run
        const uint32_t dj = dr - sdx[jl];
        a = (uint64_t)sidx[jl] + dj;
        b = jl + 1 < ns ? sidx[jl + 1] : nle;
        sh = (int64_t)skp[jl + 1] - (int64_t)dr;
      }
      if (b > nle) b = nle;
      for (uint64_t p0 = a; p0 < b; p0 += 256) {
        uint32_t v[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint64_t pp = p0 + q * 64 + lane;
          v[q] = pp < b ? L[pp] : 0u;
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint64_t pp = p0 + q * 64 + lane;
          if (pp < b) out[(uint64_t)((int64_t)pp + sh)] = v[q];
        }
      }
    }
    if (tid == 0) m.olen[k] = (uint64_t)KS + nle - dtot;
    return;
  }
  // L: stream tiles in index order
  uint32_t KL = 0, jlo = 0, jp = 0;
  uint32_t xn[kML];  // the next tile's L values, in flight while a tile is processed
#pragma unroll
  for (int s = 0; s < kML; s++) {
    const uint64_t i = (uint64_t)s * kMT + tid;
    xn[s] = i < nl ? L[i] : kSent;
  }
  for (uint64_t tb = 0; tb < nl; tb += kMTile) {
    uint32_t x[kML];
    uint32_t lbs[kML], ubs[kML];  // bounds in S (<= kMS)
    bool valid[kML];
#pragma unroll
    for (int s = 0; s < kML; s++) {
      const uint64_t i = tb + (uint64_t)s * kMT + tid;
      valid[s] = i < nl;
      x[s] = xn[s];
      const uint64_t in = i + kMTile;
      xn[s] = in < nl ? L[in] : kSent;
    }
    // each step s of a wave covers 64 consecutive L values: the S elements in
    // their value range are found with ballots from the wave's running
    // position jp (usually none or one), so the per-element bounds need no
    // search; a dense range falls back to a search inside it
#pragma unroll
    for (int s = 0; s < kML; s++) {
      const uint64_t vb = __ballot(valid[s]);
      if (!vb) {
        lbs[s] = ubs[s] = 0;
        continue;
      }
      const uint32_t xf = __builtin_amdgcn_readfirstlane(x[s]);
      const uint32_t xl = __builtin_amdgcn_readlane(x[s], 63 - __clzll((unsigned long long)vb));
      const uint32_t jA = ballot_count<false>(sv, ns, jp, xf, lane);
      const uint32_t jB = ballot_count<true>(sv, ns, jA, xl, lane);
      jp = jA;
      uint32_t lt = jA, le = jA;
      if (jB - jA <= 16) {
        for (uint32_t j = jA; j < jB; j++) {
          const uint32_t v = sv[j];
          lt += v < x[s] ? 1u : 0u;
          le += v <= x[s] ? 1u : 0u;
        }
      } else {
        uint32_t lo = jA, hi = jB;
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (sv[mid] < x[s]) lo = mid + 1; else hi = mid;
        }
        lt = lo;
        hi = jB;
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (sv[mid] <= x[s]) lo = mid + 1; else hi = mid;
        }
        le = lo;
      }
      lbs[s] = lt;
      ubs[s] = le;
    }
    bool kp[kML];
#pragma unroll
    for (int s = 0; s < kML; s++) {
      const uint64_t i = tb + (uint64_t)s * kMT + tid;
      uint64_t t = 0;
      // the copy index t only matters against a non-zero count in S (every
      // keep rule keeps all copies of a value S lacks): rare, so only then
      // look at L[i - 1] and search for the value's first index
      if (valid[s] && ubs[s] > lbs[s] && i > 0 && L[i - 1] == x[s]) {
        uint64_t lo = 0, hi = i;
        while (lo < hi) {
          const uint64_t mid = (lo + hi) >> 1;
          if (L[mid] < x[s]) lo = mid + 1; else hi = mid;
        }
        t = i - lo;
      }
      kp[s] = valid[s] && x[s] != kSent && keep_rule(m.op, sL, t, ubs[s] - lbs[s]);
      const unsigned long long bw = __ballot(kp[s]);
      if (lane == 0) tw[s * kMWaves + w] = bw;
    }
    __syncthreads();
    if (tid < 64) {  // word prefix over the tile (index order = (s, wave)); kWL words per lane
      constexpr int kNWd = kML * kMWaves, kWL = (kNWd + 63) / 64;
      uint32_t cw[kWL], c = 0;
#pragma unroll
      for (int q = 0; q < kWL; q++) {
        const int wi = tid * kWL + q;
        cw[q] = wi < kNWd ? (uint32_t)__popcll(tw[wi]) : 0u;
        c += cw[q];
      }
      const uint32_t incl = sgd::wave_incl_add(c);
      uint32_t run = KL + incl - c;
#pragma unroll
      for (int q = 0; q < kWL; q++) {
        const int wi = tid * kWL + q;
        if (wi < kNWd) twp[wi] = run;
        run += cw[q];
      }
      if (tid == 63) twp[kNWd] = KL + incl;
    }
    __syncthreads();
    const unsigned long long below = (1ull << lane) - 1;
#pragma unroll
    for (int s = 0; s < kML; s++)
      if (kp[s]) {
        const uint32_t q = s * kMWaves + w;
        const uint32_t rank = twp[q] + (uint32_t)__popcll(tw[q] & below);
        out[rank + skp[sL == 0 ? lbs[s] : ubs[s]]] = x[s];
      }
    // S elements whose insertion point lies in this tile
    uint32_t jhi;
    {  // #{j : sidx[j] < tile end} by ballots from jlo (sidx is non-decreasing)
      const uint64_t end = tb + kMTile;
      uint32_t j0 = jlo;
      for (;;) {
        const uint32_t j = j0 + (uint32_t)lane;
        const uint64_t b = __ballot(j < ns && sidx[j] < end);
        if (b != ~0ull) {
          jhi = j0 + (uint32_t)__popcll(b);
          break;
        }
        j0 += 64;
      }
    }
    for (uint32_t j = jlo + tid; j < jhi; j += kMT)
      if (skp[j + 1] > skp[j]) {
        const uint32_t p = (uint32_t)(sidx[j] - tb), q = (p / kMT) * kMWaves + (p % kMT) / 64, bit = p % 64;
        const uint32_t kb = twp[q] + (uint32_t)__popcll(tw[q] & ((1ull << bit) - 1));
        out[skp[j] + kb] = sv[j];
      }
    KL = twp[kML * kMWaves];
    jlo = jhi;
    __syncthreads();
  }
  for (uint32_t j = jlo + tid; j < ns; j += kMT)  // insertion point past the end of L
    if (skp[j + 1] > skp[j]) out[skp[j] + KL] = sv[j];
  if (tid == 0) m.olen[k] = (uint64_t)KS + KL;
}

__global__ void k_merge_len(MergeArgs m) {
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m.npair) return;
  uint64_t L = 0;
  for (int s = 0; s < 2; s++) {
    if (!m.nchunks[s]) continue;
    const Side& me = s == 0 ? m.a : m.b;
    L += mask_prefix(m.mask[s], m.base[s], m.nchunks[s], me.off[k + 1]) -
         mask_prefix(m.mask[s], m.base[s], m.nchunks[s], me.off[k]);
  }
  m.out_len[k] = L;
}

// HasDifference: some element of a (t-th copy) with t >= count in b.
__global__ void k_has_difference(const uint32_t* __restrict__ a, uint64_t na, const uint32_t* __restrict__ b,
                                 uint64_t nb, uint64_t* flag) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  bool hit = false;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na; i += stride) {
    uint32_t x = a[i];
    uint64_t t = i - lower_bound(a, i, x);
    uint64_t c = upper_bound(b, nb, x) - lower_bound(b, nb, x);
    hit |= t >= c;
  }
  if (__any(hit) && (threadIdx.x & 63) == 0) *flag = 1;
}

// Batched HasDifference: a workgroup per pair, its a-range strided over the
// threads (element t-th copy of x vs x's count in b, both by binary search in
// the pair's own ranges); one flag byte per pair.
constexpr int kHdT = 256;
__global__ __launch_bounds__(kHdT) void k_has_difference_batch(const uint32_t* __restrict__ a,
                                                               const uint64_t* __restrict__ a_beg,
                                                               const uint64_t* __restrict__ a_len,
                                                               const uint32_t* __restrict__ b,
                                                               const uint64_t* __restrict__ b_beg,
                                                               const uint64_t* __restrict__ b_len, uint8_t* out) {
  const uint64_t k = blockIdx.x;
  const uint32_t* pa = a + a_beg[k];
  const uint32_t* pb = b + b_beg[k];
  const uint64_t na = a_len[k], nb = b_len[k];
  bool hit = false;
  for (uint64_t i = threadIdx.x; i < na && !hit; i += kHdT) {
    const uint32_t x = pa[i];
    const uint64_t t = i - lower_bound(pa, i, x);
    hit = t >= upper_bound(pb, nb, x) - lower_bound(pb, nb, x);
  }
  if (__syncthreads_or(hit) && threadIdx.x == 0) out[k] = 1;
}

// ---- segmented sort ----------------------------------------------------------
struct SortChunk {
  uint64_t start;  // global element index
  uint32_t len;    // <= 4096
};

__global__ __launch_bounds__(kBlock) void k_sort_chunks(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                        const SortChunk* __restrict__ chunks) {
  __shared__ uint32_t s[kTile];
  SortChunk ch = chunks[blockIdx.x];
  // bitonic sort over the next power of two >= len (per-call signal lists are
  // mostly far shorter than a tile: 4096 slots for each cost 3.6 ms per 64Ki
  // lists), up to 8 compare-exchanges per thread per stage
  uint32_t P = 2;
  while (P < ch.len) P <<= 1;
  for (uint32_t i = threadIdx.x; i < P; i += kBlock) s[i] = i < ch.len ? in[ch.start + i] : kSent;
  __syncthreads();
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t t = threadIdx.x; t < P / 2; t += kBlock) {
        uint32_t i = 2 * t - (t & (j - 1));  // index with bit j clear
        uint32_t l = i + j;
        bool up = (i & k) == 0;
        uint32_t x = s[i], y = s[l];
        if ((x > y) == up) {
          s[i] = y;
          s[l] = x;
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t i = threadIdx.x; i < ch.len; i += kBlock) out[ch.start + i] = s[i];
}

// Bitonic sort of P (a power of two, <= kBlock * E) values held E per thread
// (element i = thread * E + r) in registers: partners within a thread swap in
// registers, partners within a wave (distance < 64 E) come by __shfl_xor, and
// only the longer distances go through LDS (s, >= kBlock * E slots) with
// barriers -- 3 of the 55 stages for P = 1024.  Threads past P / E hold
// padding and only ever meet each other.
template <int E>
__device__ __forceinline__ void bitonic_regs(uint32_t (&v)[E], uint32_t P, uint32_t* s) {
  const uint32_t t = threadIdx.x;
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      if (j < (uint32_t)E) {
#pragma unroll
        for (int r = 0; r < E; r++) {
          if ((r & j) == 0) {
            const uint32_t i = t * E + r;
            const bool up = (i & k) == 0;
            const uint32_t x = v[r], y = v[r | j];
            if ((x > y) == up) {
              v[r] = y;
              v[r | j] = x;
            }
          }
        }
      } else if (j / E < 64) {
        const int m = (int)(j / E);
#pragma unroll
        for (int r = 0; r < E; r++) {
          const uint32_t i = t * E + r, y = __shfl_xor(v[r], m);
          const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
          v[r] = keep_min ? min(v[r], y) : max(v[r], y);
        }
      } else {
#pragma unroll
        for (int r = 0; r < E; r++) s[t * E + r] = v[r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < E; r++) {
          const uint32_t i = t * E + r, y = s[i ^ j];
          const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
          v[r] = keep_min ? min(v[r], y) : max(v[r], y);
        }
        __syncthreads();
      }
    }
  }
}

// chunk [start, start + len) sorted into s[0 .. P) (padding kSent)
template <int E>
__device__ __forceinline__ void sort_chunk_regs(const uint32_t* vals, const SortChunk& ch, uint32_t P, uint32_t* s) {
  uint32_t v[E];
#pragma unroll
  for (int r = 0; r < E; r++) {
    const uint32_t i = threadIdx.x * E + r;
    v[r] = i < ch.len ? vals[ch.start + i] : kSent;
  }
  bitonic_regs<E>(v, P, s);
  __syncthreads();  // (the last LDS stage's reads are done)
#pragma unroll
  for (int r = 0; r < E; r++) s[threadIdx.x * E + r] = v[r];
  __syncthreads();
}

// Canonicalize of a batch whose segments all fit one tile (<= kTile): each
// chunk is one whole segment, so the unique pass runs in LDS right after the
// chunk's sort (no mask, scan or search passes): the kept values (cover.go:31-37:
// x != the previous sorted value, the first against kSent) go to the
// segment's start in order, the positions past them keep the sorted values,
// out_len[seg] = their number.  In place (the chunk is read whole first).
__global__ __launch_bounds__(kBlock) void k_sort_unique_chunks(uint32_t* vals, const SortChunk* __restrict__ chunks,
                                                               const uint32_t* __restrict__ seg,
                                                               uint64_t* __restrict__ out_len) {
  __shared__ uint32_t s[kTile];
  __shared__ uint32_t wsum[kBlock / 64];
  const SortChunk ch = chunks[blockIdx.x];
  uint32_t P = 2;
  while (P < ch.len) P <<= 1;
  // values per thread: the fewest that hold P (register bitonic stages)
  if (P <= kBlock)
    sort_chunk_regs<1>(vals, ch, P, s);
  else if (P <= 2 * kBlock)
    sort_chunk_regs<2>(vals, ch, P, s);
  else if (P <= 4 * kBlock)
    sort_chunk_regs<4>(vals, ch, P, s);
  else if (P <= 8 * kBlock)
    sort_chunk_regs<8>(vals, ch, P, s);
  else
    sort_chunk_regs<16>(vals, ch, P, s);
  // each thread: kTile / kBlock consecutive positions
  constexpr int kPer = kTile / kBlock;
  const uint32_t i0 = threadIdx.x * kPer;
  uint32_t keep = 0;
#pragma unroll
  for (int q = 0; q < kPer; q++) {
    const uint32_t i = i0 + q;
    if (i < ch.len && s[i] != (i ? s[i - 1] : kSent)) keep |= 1u << q;
  }
  const uint32_t c = __popc(keep), lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t pos = incl - c, total = 0;
#pragma unroll
  for (int v = 0; v < kBlock / 64; v++) {
    pos += v < (int)w ? wsum[v] : 0u;
    total += wsum[v];
  }
  uint32_t* out = vals + ch.start;
  for (uint32_t m = keep; m; m &= m - 1) out[pos++] = s[i0 + __builtin_ctz(m)];
  for (uint32_t i = total + threadIdx.x; i < ch.len; i += kBlock) out[i] = s[i];  // the stale tail
  if (threadIdx.x == 0) out_len[seg[blockIdx.x]] = total;
}

// Lists of <= kWaveList values: one wave per list, sorted by a bitonic
// network over the wave's registers (E = P / 64 values per lane, element i =
// lane E + r; partners inside a lane swap in registers, the rest come by
// __shfl_xor -- no LDS and no barrier), then deduplicated and written back in
// place with a wave prefix sum.  Four lists per workgroup.  (A workgroup per
// list, with LDS stages and barriers, spent most of its time on the padding
// of short lists and on its barriers.)
constexpr uint32_t kWaveList = 1024;

template <int E>
__device__ __forceinline__ void canon_wave(uint32_t* __restrict__ vals, const SortChunk& ch, uint64_t* out_len_slot) {
  const uint32_t lane = threadIdx.x & 63;
  constexpr uint32_t P = 64 * E;
  uint32_t v[E];
#pragma unroll
  for (int r = 0; r < E; r++) {
    const uint32_t i = lane * E + r;
    v[r] = i < ch.len ? vals[ch.start + i] : kSent;
  }
#pragma unroll
  for (uint32_t k = 2; k <= P; k <<= 1) {
#pragma unroll
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      if (j < (uint32_t)E) {
#pragma unroll
        for (int r = 0; r < E; r++) {
          if ((r & j) == 0) {
            const uint32_t i = lane * E + r;
            const bool up = (i & k) == 0;
            const uint32_t x = v[r], y = v[r | j];
            const bool sw = (x > y) == up;
            v[r] = sw ? y : x;
            v[r | j] = sw ? x : y;
          }
        }
      } else {
        const int m = (int)(j / E);
#pragma unroll
        for (int r = 0; r < E; r++) {
          const uint32_t i = lane * E + r, y = (uint32_t)__shfl_xor((int)v[r], m);
          const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
          v[r] = keep_min ? min(v[r], y) : max(v[r], y);
        }
      }
    }
  }
  // cover.go:31-37: x != the previous sorted value, the first against kSent
  const uint32_t before = (uint32_t)__shfl_up((int)v[E - 1], 1);
  uint32_t keep = 0;
#pragma unroll
  for (int r = 0; r < E; r++) {
    const uint32_t i = lane * E + r;
    const uint32_t prev = r ? v[r - 1] : (lane ? before : kSent);
    if (i < ch.len && v[r] != prev) keep |= 1u << r;
  }
  const uint32_t c = __popc(keep), incl = sgd::wave_incl_add(c);
  const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
  uint32_t pos = incl - c;
  uint32_t* out = vals + ch.start;
#pragma unroll
  for (int r = 0; r < E; r++) {
    const uint32_t i = lane * E + r;
    if ((keep >> r) & 1u) out[pos++] = v[r];
    if (i >= total && i < ch.len) out[i] = v[r];  // the stale tail: the sorted values (disjoint positions)
  }
  if (lane == 0) *out_len_slot = total;
}

__global__ __launch_bounds__(256) void k_canon_waves(uint32_t* __restrict__ vals, const SortChunk* __restrict__ chunks,
                                                     const uint32_t* __restrict__ seg, uint32_t n,
                                                     uint64_t* __restrict__ out_len) {
  const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= n) return;  // (a wave leaves whole: no block barrier follows)
  const SortChunk ch = chunks[w];
  uint64_t* slot = out_len + seg[w];
  if (ch.len <= 64)
    canon_wave<1>(vals, ch, slot);
  else if (ch.len <= 128)
    canon_wave<2>(vals, ch, slot);
  else if (ch.len <= 256)
    canon_wave<4>(vals, ch, slot);
  else if (ch.len <= 512)
    canon_wave<8>(vals, ch, slot);
  else
    canon_wave<16>(vals, ch, slot);
}

struct BigSeg {
  uint64_t start;  // global element index of the segment
  uint64_t len;
};

// one rank-merge pass of width w over the big segments [0, nbig) (sorted by
// length descending, so the active ones form a prefix); `vs` = exclusive scan
// of their lengths (virtual element space).
__global__ void k_merge_pass(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                             const BigSeg* __restrict__ segs, const uint64_t* __restrict__ vs, uint64_t nbig,
                             uint64_t w) {
  uint64_t n = vs[nbig];
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += stride) {
    uint64_t si = sgd::seg_search(vs, 0, nbig - 1, u);
    BigSeg sg = segs[si];
    uint64_t i = u - vs[si];
    const uint32_t* src = in + sg.start;
    uint64_t r = i / w, pair0 = (r & ~1ull) * w;
    uint32_t x = src[i];
    uint64_t pos;
    if ((r & 1) == 0) {
      uint64_t rs = pair0 + w;
      uint64_t rl = rs < sg.len ? std::min<uint64_t>(w, sg.len - rs) : 0;
      pos = pair0 + (i - pair0) + lower_bound(src + rs, rl, x);
    } else {
      uint64_t ls = pair0;
      pos = pair0 + (i - (pair0 + w)) + upper_bound(src + ls, w, x);
    }
    out[sg.start + pos] = x;
  }
}

struct CanonArgs {
  const uint32_t* buf[2];
  const uint64_t* off;
  uint64_t nseg;
  uint64_t n;
  const uint8_t* parity;  // per segment: which buffer holds its sorted values
  uint64_t* mask;
  uint32_t* cnt;
  uint64_t* base;
  uint64_t nchunks;
  uint32_t* out;
  uint64_t* out_len;
  uint64_t* ks;  // ks[w] = segment of element min(64 w + 63, n - 1)
};

// Element u's segment lies between ks[w - 1] and ks[w] (w = u / 64; almost
// always one segment), so the per-element search is one or two cached loads
// instead of a chain of ~17 dependent ones over the whole offset table.
__global__ void k_canon_segs(CanonArgs a) {
  const uint64_t nw = (a.n + 63) / 64, stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride)
    a.ks[w] = sgd::seg_search(a.off, 0, a.nseg - 1, std::min<uint64_t>(64 * w + 63, a.n - 1));
}

__device__ __forceinline__ uint64_t canon_seg(const CanonArgs& a, uint64_t u) {
  const uint64_t w = u >> 6;
  return sgd::seg_search(a.off, w ? a.ks[w - 1] : 0, a.ks[w], u);
}

__global__ __launch_bounds__(kBlock) void k_unique_keep(CanonArgs a) {
  const int lane = threadIdx.x & 63;
  uint64_t c = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (c >= a.nchunks) return;
  uint32_t bits = 0;
  for (int q = 0; q < 4; q++) {
    uint64_t u = c * kChunk + lane * 4 + q;
    if (u >= a.n) continue;
    uint64_t k = canon_seg(a, u);
    const uint32_t* b = a.buf[a.parity[k]];
    uint32_t x = b[u];
    uint32_t last = u == a.off[k] ? kSent : b[u - 1];  // cover.go:31-37
    if (x != last) bits |= 1u << q;
  }
  uint64_t b0 = __ballot(bits & 1u), b1 = __ballot(bits & 2u), b2 = __ballot(bits & 4u), b3 = __ballot(bits & 8u);
  uint64_t mine = lane == 0 ? b0 : lane == 1 ? b1 : lane == 2 ? b2 : b3;
  if (lane < 4) a.mask[c * 4 + lane] = mine;
  if (lane == 0) a.cnt[c] = __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
}

__global__ void k_unique_len(CanonArgs a) {
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.nseg) return;
  a.out_len[k] = mask_prefix(a.mask, a.base, a.nchunks, a.off[k + 1]) -
                 mask_prefix(a.mask, a.base, a.nchunks, a.off[k]);
}

// out = sorted values with the first out_len[k] positions of each segment
// replaced by the kept (unique) ones.
__global__ void k_unique_write(CanonArgs a) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < a.n; u += stride) {
    uint64_t k = canon_seg(a, u);
    const uint32_t* b = a.buf[a.parity[k]];
    uint32_t x = b[u];
    uint64_t s = a.off[k];
    if (u - s >= a.out_len[k]) a.out[u] = x;  // stale tail: the sorted value
    if (mask_bit(a.mask, u)) {
      uint64_t pos = mask_prefix(a.mask, a.base, a.nchunks, u) - mask_prefix(a.mask, a.base, a.nchunks, s);
      a.out[s + pos] = x;
    }
  }
}

// ---- host orchestration ----------------------------------------------------------
// chunks: one per non-empty segment, in segment order
static int canonicalize_small(sg_ctx* ctx, uint32_t* d_vals, const uint64_t* off, uint64_t nseg,
                              const std::vector<SortChunk>& chunks, uint64_t* out_len) {
  // lists of <= kWaveList values a wave each (k_canon_waves), longer ones a
  // workgroup each (k_sort_unique_chunks); chunks are the non-empty segments
  std::vector<SortChunk> wch, bch;
  std::vector<uint32_t> wseg, bseg;
  size_t ci = 0;
  for (uint64_t k = 0; k < nseg; k++)
    if (off[k + 1] > off[k]) {
      const SortChunk& c = chunks[ci++];
      if (c.len <= kWaveList) {
        wch.push_back(c);
        wseg.push_back((uint32_t)k);
      } else {
        bch.push_back(c);
        bseg.push_back((uint32_t)k);
      }
    }
  WsPlan p;
  const size_t o_wch = p.add(wch.size() * sizeof(SortChunk)), o_wseg = p.add(wseg.size() * 4),
               o_bch = p.add(bch.size() * sizeof(SortChunk)), o_bseg = p.add(bseg.size() * 4), o_len = p.add(nseg * 8);
  int rc = ws_reserve(ctx, p.total);
  if (rc) return rc;
  uint64_t* dlen = (uint64_t*)ws_at(ctx, o_len);
  SG_HIP(hipMemsetAsync(dlen, 0, nseg * 8, ctx->stream));  // (empty segments)
  if (!wch.empty() || !bch.empty()) {
    ScopedTimer tm(ctx, "canon_sort");
    if (!wch.empty()) {
      SortChunk* dch = (SortChunk*)ws_at(ctx, o_wch);
      uint32_t* dseg = (uint32_t*)ws_at(ctx, o_wseg);
      SG_HIP(hipMemcpyAsync(dch, wch.data(), wch.size() * sizeof(SortChunk), hipMemcpyHostToDevice, ctx->stream));
      SG_HIP(hipMemcpyAsync(dseg, wseg.data(), wseg.size() * 4, hipMemcpyHostToDevice, ctx->stream));
      hipLaunchKernelGGL(k_canon_waves, dim3((uint32_t)div_up(wch.size(), 4)), dim3(256), 0, ctx->stream, d_vals,
                         (const SortChunk*)dch, (const uint32_t*)dseg, (uint32_t)wch.size(), dlen);
    }
    if (!bch.empty()) {
      SortChunk* dch = (SortChunk*)ws_at(ctx, o_bch);
      uint32_t* dseg = (uint32_t*)ws_at(ctx, o_bseg);
      SG_HIP(hipMemcpyAsync(dch, bch.data(), bch.size() * sizeof(SortChunk), hipMemcpyHostToDevice, ctx->stream));
      SG_HIP(hipMemcpyAsync(dseg, bseg.data(), bseg.size() * 4, hipMemcpyHostToDevice, ctx->stream));
      hipLaunchKernelGGL(k_sort_unique_chunks, dim3((uint32_t)bch.size()), dim3(kBlock), 0, ctx->stream, d_vals, dch,
                         dseg, dlen);
    }
  }
  SG_HIP(hipGetLastError());
  SG_HIP(hipMemcpyAsync(out_len, dlen, nseg * 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));  // (the host vectors above are read by the queued copies)
  return SG_OK;
}

int canonicalize_dev(sg_ctx* ctx, uint32_t* d_vals, const uint64_t* off, uint64_t nseg, uint64_t* out_len) {
  // off: host offsets (nseg+1); d_vals: device values (sorted+uniqued in place)
  uint64_t n = off[nseg];
  std::vector<SortChunk> chunks;
  std::vector<BigSeg> big;
  std::vector<uint8_t> parity(nseg, 0);
  for (uint64_t k = 0; k < nseg; k++) {
    uint64_t L = off[k + 1] - off[k];
    for (uint64_t q = 0; q < L; q += kTile) chunks.push_back({off[k] + q, (uint32_t)std::min<uint64_t>(kTile, L - q)});
    if (L > (uint64_t)kTile) {
      big.push_back({off[k], L});
      int passes = 0;
      for (uint64_t w = kTile; w < L; w <<= 1) passes++;
      parity[k] = passes & 1;
    }
  }
  if (big.empty() && nseg <= 0xFFFFFFFFull)  // every segment fits one tile: sort and unique in one pass
    return canonicalize_small(ctx, d_vals, off, nseg, chunks, out_len);
  std::sort(big.begin(), big.end(), [](const BigSeg& x, const BigSeg& y) { return x.len > y.len; });
  std::vector<uint64_t> vs(big.size() + 1, 0);
  for (size_t i = 0; i < big.size(); i++) vs[i + 1] = vs[i] + big[i].len;
  uint64_t ntiles = (n + kTile - 1) / kTile, nchunks = ntiles * kChunksPerTile;
  WsPlan p;
  size_t o_b0 = p.add(n * 4), o_b1 = p.add(n * 4), o_ch = p.add(chunks.size() * sizeof(SortChunk)),
         o_big = p.add(big.size() * sizeof(BigSeg)), o_vs = p.add(vs.size() * 8), o_off = p.add((nseg + 1) * 8),
         o_par = p.add(nseg), o_mask = p.add(nchunks * 32), o_cnt = p.add(nchunks * 4),
         o_base = p.add((nchunks + 1) * 8), o_len = p.add(nseg * 8), o_ks = p.add((n + 63) / 64 * 8);
  size_t scan_off = p.total;
  int rc = ws_reserve(ctx, p.total + scan_ws_bytes(nchunks));
  if (rc) return rc;
  uint32_t* b0 = (uint32_t*)ws_at(ctx, o_b0);
  uint32_t* b1 = (uint32_t*)ws_at(ctx, o_b1);
  SortChunk* dch = (SortChunk*)ws_at(ctx, o_ch);
  BigSeg* dbig = (BigSeg*)ws_at(ctx, o_big);
  uint64_t* dvs = (uint64_t*)ws_at(ctx, o_vs);
  uint64_t* doff = (uint64_t*)ws_at(ctx, o_off);
  uint8_t* dpar = (uint8_t*)ws_at(ctx, o_par);
  uint64_t* dlen = (uint64_t*)ws_at(ctx, o_len);
  if (!chunks.empty())
    SG_HIP(hipMemcpyAsync(dch, chunks.data(), chunks.size() * sizeof(SortChunk), hipMemcpyHostToDevice, ctx->stream));
  if (!big.empty()) {
    SG_HIP(hipMemcpyAsync(dbig, big.data(), big.size() * sizeof(BigSeg), hipMemcpyHostToDevice, ctx->stream));
    SG_HIP(hipMemcpyAsync(dvs, vs.data(), vs.size() * 8, hipMemcpyHostToDevice, ctx->stream));
  }
  SG_HIP(hipMemcpyAsync(doff, off, (nseg + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dpar, parity.data(), nseg, hipMemcpyHostToDevice, ctx->stream));
  {
    ScopedTimer tm(ctx, "canon_sort");
    if (!chunks.empty())
      hipLaunchKernelGGL(k_sort_chunks, dim3((uint32_t)chunks.size()), dim3(kBlock), 0, ctx->stream, d_vals, b0,
                         dch);
    // rank-merge passes: active segments (len > w) are a prefix of `big`
    uint32_t* bufs[2] = {b0, b1};
    int pass = 0;
    for (uint64_t w = kTile;; w <<= 1, pass++) {
      uint64_t nact = 0;
      while (nact < big.size() && big[nact].len > w) nact++;
      if (nact == 0) break;
      uint64_t nel = vs[nact];
      hipLaunchKernelGGL(k_merge_pass, dim3((uint32_t)std::min<uint64_t>(div_up(nel, 256), 16384)), dim3(256), 0,
                         ctx->stream, bufs[pass & 1], bufs[(pass + 1) & 1], dbig, dvs, nact, w);
    }
  }
  CanonArgs a{};
  a.buf[0] = b0;
  a.buf[1] = b1;
  a.off = doff;
  a.nseg = nseg;
  a.n = n;
  a.parity = dpar;
  a.mask = (uint64_t*)ws_at(ctx, o_mask);
  a.cnt = (uint32_t*)ws_at(ctx, o_cnt);
  a.base = (uint64_t*)ws_at(ctx, o_base);
  a.nchunks = nchunks;
  a.out = d_vals;
  a.out_len = dlen;
  a.ks = (uint64_t*)ws_at(ctx, o_ks);
  {
    ScopedTimer tm(ctx, "canon_unique");
    if (n)
      hipLaunchKernelGGL(k_canon_segs, dim3((uint32_t)std::min<uint64_t>(div_up((n + 63) / 64, 256), 16384)), dim3(256),
                         0, ctx->stream, a);
    hipLaunchKernelGGL(k_unique_keep, dim3(div_up(nchunks, kBlock / 64)), dim3(kBlock), 0, ctx->stream, a);
    rc = scan_counts(ctx, a.cnt, a.base, nchunks, scan_off);
    if (rc) return rc;
    hipLaunchKernelGGL(k_unique_len, dim3(div_up(nseg, 256)), dim3(256), 0, ctx->stream, a);
    hipLaunchKernelGGL(k_unique_write, dim3((uint32_t)std::min<uint64_t>(div_up(n, 256), 16384)), dim3(256), 0,
                       ctx->stream, a);
  }
  SG_HIP(hipGetLastError());
  SG_HIP(hipMemcpyAsync(out_len, dlen, nseg * 8, hipMemcpyDeviceToHost, ctx->stream));
  // the chunk / segment descriptors above are host locals: the queued copies
  // may still read them, so drain before they go out of scope
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

// Batched merge of device-resident lists: pair k is da[a_beg[k] .. +a_len[k])
// op db[b_beg[k] .. +b_len[k]) into dout[out_beg[k] ..) (capacity a_len[k] +
// b_len[k]).  The pair descriptors are host arrays (their lengths size the
// launches); out_len (host) gets the result lengths.  da / db / dout must not
// live in the workspace.  Syncs.
int merge_dev(sg_ctx* ctx, int op, const uint32_t* da, const uint32_t* db, uint32_t* dout, const uint64_t* a_beg,
              const uint64_t* a_len, const uint64_t* b_beg, const uint64_t* b_len, const uint64_t* out_beg,
              size_t npair, uint64_t* out_len) {
  std::vector<uint64_t> aoff(npair + 1, 0), boff(npair + 1, 0);
  for (size_t k = 0; k < npair; k++) {
    aoff[k + 1] = aoff[k] + a_len[k];
    boff[k + 1] = boff[k] + b_len[k];
  }
  bool bside = op == SG_OP_UNION || op == SG_OP_SYMDIFF;
  bool small = bside;  // every pair has a side that fits in LDS: one workgroup per pair
  for (size_t k = 0; k < npair && small; k++) small = std::min(a_len[k], b_len[k]) <= (uint64_t)kMS;
  bool asmall = !bside;  // Difference / Intersection, every first list fits in LDS
  for (size_t k = 0; k < npair && asmall; k++) asmall = a_len[k] <= (uint64_t)kMS;
  uint64_t na = aoff[npair], nb = bside ? boff[npair] : 0;
  uint64_t nca = ((na + kTile - 1) / kTile) * kChunksPerTile, ncb = ((nb + kTile - 1) / kTile) * kChunksPerTile;
  WsPlan p;
  size_t o_meta = p.add((npair * 2 + (npair + 1)) * 8 * 2 + npair * 8 * 2);
  size_t o_m0 = p.add(nca * 32), o_m1 = p.add(ncb * 32), o_c0 = p.add(nca * 4), o_c1 = p.add(ncb * 4),
         o_s0 = p.add((nca + 1) * 8), o_s1 = p.add((ncb + 1) * 8);
  size_t scan_off = p.total;
  int rc = ws_reserve(ctx, p.total + scan_ws_bytes(std::max(nca, ncb)));
  if (rc) return rc;
  uint64_t* meta = (uint64_t*)ws_at(ctx, o_meta);
  // meta layout: a_beg a_len aoff b_beg b_len boff out_beg out_len
  uint64_t *m_abeg = meta, *m_alen = m_abeg + npair, *m_aoff = m_alen + npair, *m_bbeg = m_aoff + npair + 1,
           *m_blen = m_bbeg + npair, *m_boff = m_blen + npair, *m_obeg = m_boff + npair + 1,
           *m_olen = m_obeg + npair;
  SG_HIP(hipMemcpyAsync(m_abeg, a_beg, npair * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(m_alen, a_len, npair * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(m_aoff, aoff.data(), (npair + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(m_bbeg, b_beg, npair * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(m_blen, b_len, npair * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(m_boff, boff.data(), (npair + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(m_obeg, out_beg, npair * 8, hipMemcpyHostToDevice, ctx->stream));
  if (asmall) {
    SmallArgs sm{op, da, db, m_abeg, m_alen, m_bbeg, m_blen, m_obeg, m_olen, dout};
    ScopedTimer tm(ctx, "merge_small");
    hipLaunchKernelGGL(k_diff_small, dim3((uint32_t)npair), dim3(kMT), 0, ctx->stream, sm);
  } else if (small) {
    SmallArgs sm{op, da, db, m_abeg, m_alen, m_bbeg, m_blen, m_obeg, m_olen, dout};
    {
      ScopedTimer tm(ctx, "merge_small");
      hipLaunchKernelGGL(k_merge_small<true>, dim3((uint32_t)npair), dim3(kMT), 0, ctx->stream, sm);
      hipLaunchKernelGGL(k_merge_small<false>, dim3((uint32_t)npair), dim3(kMT), 0, ctx->stream, sm);
    }
  } else {
    MergeArgs m{};
    m.op = op;
    m.a = {da, m_abeg, m_alen, m_aoff};
    m.b = {db, m_bbeg, m_blen, m_boff};
    m.npair = npair;
    m.mask[0] = (uint64_t*)ws_at(ctx, o_m0);
    m.mask[1] = (uint64_t*)ws_at(ctx, o_m1);
    m.cnt[0] = (uint32_t*)ws_at(ctx, o_c0);
    m.cnt[1] = (uint32_t*)ws_at(ctx, o_c1);
    m.base[0] = (uint64_t*)ws_at(ctx, o_s0);
    m.base[1] = (uint64_t*)ws_at(ctx, o_s1);
    m.nchunks[0] = nca;
    m.nchunks[1] = ncb;
    m.out = dout;
    m.out_beg = m_obeg;
    m.out_len = m_olen;
    {
      ScopedTimer tm(ctx, "merge_keep");
      if (nca) hipLaunchKernelGGL(k_merge_keep<0>, dim3(div_up(nca, kBlock / 64)), dim3(kBlock), 0, ctx->stream, m);
      if (ncb) hipLaunchKernelGGL(k_merge_keep<1>, dim3(div_up(ncb, kBlock / 64)), dim3(kBlock), 0, ctx->stream, m);
    }
    if (nca) {
      rc = scan_counts(ctx, m.cnt[0], m.base[0], nca, scan_off);
      if (rc) return rc;
    }
    if (ncb) {
      rc = scan_counts(ctx, m.cnt[1], m.base[1], ncb, scan_off);
      if (rc) return rc;
    }
    {
      ScopedTimer tm(ctx, "merge_scatter");
      if (na)
        hipLaunchKernelGGL(k_merge_scatter<0>, dim3((uint32_t)std::min<uint64_t>(div_up(na, 256), 16384)), dim3(256),
                           0, ctx->stream, m);
      if (nb)
        hipLaunchKernelGGL(k_merge_scatter<1>, dim3((uint32_t)std::min<uint64_t>(div_up(nb, 256), 16384)), dim3(256),
                           0, ctx->stream, m);
    }
    hipLaunchKernelGGL(k_merge_len, dim3(div_up(npair, 256)), dim3(256), 0, ctx->stream, m);
  }
  SG_HIP(hipGetLastError());
  SG_HIP(hipMemcpyAsync(out_len, m_olen, npair * 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

static int merge_run(sg_ctx* ctx, int op, const uint32_t* a, size_t a_total, const uint64_t* a_beg,
                     const uint64_t* a_len, const uint32_t* b, size_t b_total, const uint64_t* b_beg,
                     const uint64_t* b_len, size_t npair, uint32_t* out, size_t out_total, const uint64_t* out_beg,
                     uint64_t* out_len) {
  for (size_t k = 0; k < npair; k++) {
    if (a_beg[k] + a_len[k] > a_total || b_beg[k] + b_len[k] > b_total ||
        out_beg[k] + a_len[k] + b_len[k] > out_total) {
      set_error("sg_merge_batch: pair %zu out of bounds", k);
      return SG_EINVAL;
    }
  }
  const size_t b_a = (a_total * 4 + 255) & ~size_t(255), b_b = (b_total * 4 + 255) & ~size_t(255);
  int rc = dstage_reserve(ctx, b_a + b_b + out_total * 4 + 256);
  if (rc) return rc;
  uint32_t* da = (uint32_t*)ctx->dstage;
  uint32_t* db = (uint32_t*)((char*)ctx->dstage + b_a);
  uint32_t* dout = (uint32_t*)((char*)ctx->dstage + b_a + b_b);
  if (a_total) SG_HIP(hipMemcpyAsync(da, a, a_total * 4, hipMemcpyHostToDevice, ctx->stream));
  if (b_total) SG_HIP(hipMemcpyAsync(db, b, b_total * 4, hipMemcpyHostToDevice, ctx->stream));
  rc = merge_dev(ctx, op, da, db, dout, a_beg, a_len, b_beg, b_len, out_beg, npair, out_len);
  if (rc) return rc;
  // copy back only each pair's result range
  for (size_t k = 0; k < npair; k++)
    if (out_len[k])
      SG_HIP(hipMemcpyAsync(out + out_beg[k], dout + out_beg[k], out_len[k] * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

}  // namespace sg

using namespace sg;

extern "C" {

int sg_canonicalize_batch(sg_ctx* ctx, uint32_t* vals, const uint64_t* off, size_t nseg, uint64_t* out_len) {
  if (!ctx || !off || (nseg && !out_len)) return SG_EINVAL;
  if (nseg == 0) return SG_OK;
  if (off[0] != 0) return SG_EINVAL;
  for (size_t k = 0; k < nseg; k++)
    if (off[k + 1] < off[k]) return SG_EINVAL;
  uint64_t n = off[nseg];
  if (n && !vals) return SG_EINVAL;
  if (n == 0) {
    for (size_t k = 0; k < nseg; k++) out_len[k] = 0;
    return SG_OK;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  rc = dstage_reserve(ctx, n * 4);
  if (rc) return rc;
  uint32_t* dv = (uint32_t*)ctx->dstage;
  SG_HIP(hipMemcpyAsync(dv, vals, n * 4, hipMemcpyHostToDevice, ctx->stream));
  rc = canonicalize_dev(ctx, dv, off, nseg, out_len);
  if (rc) return rc;
  SG_HIP(hipMemcpyAsync(vals, dv, n * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

int sg_canonicalize(sg_ctx* ctx, uint32_t* v, size_t n, size_t* nout) {
  if (!ctx || !nout || (n && !v)) return SG_EINVAL;
  uint64_t off[2] = {0, n}, len = 0;
  int rc = sg_canonicalize_batch(ctx, v, off, 1, &len);
  *nout = (size_t)len;
  return rc;
}

int sg_merge_batch(sg_ctx* ctx, int op, const uint32_t* a, size_t a_total, const uint64_t* a_beg,
                   const uint64_t* a_len, const uint32_t* b, size_t b_total, const uint64_t* b_beg,
                   const uint64_t* b_len, size_t npair, uint32_t* out, size_t out_total, const uint64_t* out_beg,
                   uint64_t* out_len) {
  if (!ctx || op < 0 || op > 3 || (npair && (!a_beg || !a_len || !b_beg || !b_len || !out_beg || !out_len)) ||
      (a_total && !a) || (b_total && !b) || (out_total && !out)) {
    set_error("sg_merge_batch: invalid argument");
    return SG_EINVAL;
  }
  if (npair == 0) return SG_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  return merge_run(ctx, op, a, a_total, a_beg, a_len, b, b_total, b_beg, b_len, npair, out, out_total, out_beg,
                   out_len);
}

int sg_merge(sg_ctx* ctx, int op, const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out,
             size_t* nout) {
  if (!nout) return SG_EINVAL;
  uint64_t ab = 0, al = na, bb = 0, bl = nb, ob = 0, ol = 0;
  *nout = 0;
  if (na + nb == 0) return ctx ? SG_OK : SG_EINVAL;
  int rc = sg_merge_batch(ctx, op, a, na, &ab, &al, b, nb, &bb, &bl, 1, out, na + nb, &ob, &ol);
  *nout = (size_t)ol;
  return rc;
}

int sg_has_difference(sg_ctx* ctx, const uint32_t* a, size_t na, const uint32_t* b, size_t nb, int* out) {
  if (!ctx || !out || (na && !a) || (nb && !b)) return SG_EINVAL;
  *out = 0;
  if (na == 0) return SG_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  WsPlan p;
  size_t o_a = p.add(na * 4), o_b = p.add(nb * 4);
  rc = ws_reserve(ctx, p.total);
  if (rc) return rc;
  uint32_t* da = (uint32_t*)ws_at(ctx, o_a);
  uint32_t* db = (uint32_t*)ws_at(ctx, o_b);
  SG_HIP(hipMemcpyAsync(da, a, na * 4, hipMemcpyHostToDevice, ctx->stream));
  if (nb) SG_HIP(hipMemcpyAsync(db, b, nb * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemsetAsync(ctx->dscal, 0, 8, ctx->stream));
  hipLaunchKernelGGL(k_has_difference, dim3((uint32_t)std::min<uint64_t>(div_up(na, 256), 4096)), dim3(256), 0,
                     ctx->stream, da, (uint64_t)na, db, (uint64_t)nb, ctx->dscal);
  SG_HIP(hipGetLastError());
  uint64_t f = 0;
  SG_HIP(hipMemcpyAsync(&f, ctx->dscal, 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  *out = f ? 1 : 0;
  return SG_OK;
}

int sg_has_difference_batch(sg_ctx* ctx, const uint32_t* a, size_t a_total, const uint64_t* a_beg,
                            const uint64_t* a_len, const uint32_t* b, size_t b_total, const uint64_t* b_beg,
                            const uint64_t* b_len, size_t npair, uint8_t* out) {
  if (!ctx || (npair && (!a_beg || !a_len || !b_beg || !b_len || !out)) || (a_total && !a) || (b_total && !b) ||
      npair > 0x7FFFFFFFu)
    return SG_EINVAL;
  for (size_t k = 0; k < npair; k++)
    if (a_beg[k] + a_len[k] > a_total || b_beg[k] + b_len[k] > b_total) {
      set_error("sg_has_difference_batch: pair %zu out of range", k);
      return SG_EINVAL;
    }
  if (npair == 0) return SG_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  WsPlan p;
  const size_t o_a = p.add(a_total * 4), o_b = p.add(b_total * 4), o_m = p.add(npair * 32), o_o = p.add(npair);
  rc = ws_reserve(ctx, p.total);
  if (rc) return rc;
  uint32_t* da = (uint32_t*)ws_at(ctx, o_a);
  uint32_t* db = (uint32_t*)ws_at(ctx, o_b);
  uint64_t* dm = (uint64_t*)ws_at(ctx, o_m);
  uint8_t* dout = (uint8_t*)ws_at(ctx, o_o);
  if (a_total) SG_HIP(hipMemcpyAsync(da, a, a_total * 4, hipMemcpyHostToDevice, ctx->stream));
  if (b_total) SG_HIP(hipMemcpyAsync(db, b, b_total * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dm, a_beg, npair * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dm + npair, a_len, npair * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dm + 2 * npair, b_beg, npair * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dm + 3 * npair, b_len, npair * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemsetAsync(dout, 0, npair, ctx->stream));
  {
    ScopedTimer tm(ctx, "has_difference");
    hipLaunchKernelGGL(k_has_difference_batch, dim3((uint32_t)npair), dim3(kHdT), 0, ctx->stream, da, dm, dm + npair,
                       db, dm + 2 * npair, dm + 3 * npair, dout);
  }
  SG_HIP(hipGetLastError());
  SG_HIP(hipMemcpyAsync(out, dout, npair, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

}  // extern "C"
