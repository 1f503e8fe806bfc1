// sg_fold.hip -- the manager's corpus / cover aggregation.
//
// Reference: the cover.Union folds of syz-manager, all of the shape
//   var cov cover.Cover
//   for _, inp := range <inputs> { cov = cover.Union(cov, inp.Cover) }
// at syz-manager/html.go:84 (per syscall: the corpus grouped by inp.Call),
// :94 (over those per-call covers), :184 (/cover: the corpus, or one call's
// inputs) and :306 (/rawcover: the whole corpus), and the same-hash merge
// manager.go:916-917.  Union (cover.go:63-70) keeps max(a, b) copies of a value
// seen a and b times and drops 0xFFFFFFFF (cover.go:97), so a fold is: every
// value with its largest count over the folded lists, ascending, sentinel
// dropped -- associative and commutative.  The reference walks the inputs one
// after another, O(inputs x |cov|) element copies.
//
// Here: one k-way segmented sort + unique.  Element i of list k (group g)
// gets its copy index j = i - (start of its run of equal values in the list;
// lists are sorted); the fold of g is then the distinct (g, v, j), sorted:
// a value with largest count c over the lists comes with j = 0 .. c - 1.  So
// each element becomes one 64-bit key g << (32 + jb) | v << jb | j (jb = the
// bits of the largest j, 0 for canonical covers), the keys are radix-sorted
// (sg_sort.hip), and the first key of each run is kept unless v is the
// sentinel.  A group's output starts at the number of kept keys before its
// first key.  Where g, v and j do not fit 64 bits the lists are merged
// pairwise in a balanced tree instead (merge_dev, sg_merge.hip).
#include "sg_internal.h"

#include <algorithm>

namespace sg {

int merge_dev(sg_ctx* ctx, int op, const uint32_t* da, const uint32_t* db, uint32_t* dout, const uint64_t* a_beg,
              const uint64_t* a_len, const uint64_t* b_beg, const uint64_t* b_len, const uint64_t* out_beg,
              size_t npair, uint64_t* out_len);

namespace {

// dst[dst_off[k] ..] = src[src_beg[k] .. + len[k]), one wave per segment
__global__ void k_fold_pack(const uint32_t* __restrict__ src, const uint64_t* __restrict__ src_beg,
                            const uint64_t* __restrict__ len, const uint64_t* __restrict__ dst_off, uint64_t n,
                            uint32_t* __restrict__ dst) {
  const uint64_t k = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (k >= n) return;
  const uint64_t s = src_beg[k], d = dst_off[k], L = len[k];
  for (uint64_t i = threadIdx.x & 63; i < L; i += 64) dst[d + i] = src[s + i];
}

// the same, and *rep = 1 when some list holds a value twice in a row (then
// the lists are not canonical covers and the per-group LDS fold is not theirs)
__global__ void k_fold_pack_chk(const uint32_t* __restrict__ src, const uint64_t* __restrict__ src_beg,
                                const uint64_t* __restrict__ len, const uint64_t* __restrict__ dst_off, uint64_t n,
                                uint32_t* __restrict__ dst, uint32_t* __restrict__ rep) {
  const uint64_t k = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (k >= n) return;
  const uint64_t s = src_beg[k], d = dst_off[k], L = len[k];
  bool r = false;
  for (uint64_t i = threadIdx.x & 63; i < L; i += 64) {
    const uint32_t v = src[s + i];
    dst[d + i] = v;
    r |= i > 0 && src[s + i - 1] == v;
  }
  if (__ballot(r) && (threadIdx.x & 63) == 0) *rep = 1;
}

struct Item {
  uint64_t beg, len;
};

// One wave per list: the copy index of each element (its position in its run
// of equal values), by a wave max-scan of run starts carried across chunks.
// kKeys: write the element's key; else the largest index into stats[0] and
// the AND / OR of the values into stats[1] / stats[2] (the key bits that vary).
template <bool kKeys>
__global__ void k_fold_runs(const uint32_t* __restrict__ vals, const uint64_t* __restrict__ off, uint64_t n,
                            const uint32_t* __restrict__ group, uint32_t jb, unsigned long long* __restrict__ stats,
                            uint64_t* __restrict__ keys) {
  const uint64_t k = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (k >= n) return;
  const int lane = threadIdx.x & 63;
  const uint64_t b = off[k], e = off[k + 1];
  const uint64_t gtop = kKeys ? (uint64_t)(group ? group[k] : 0u) << (32 + jb) : 0;
  int carry = -1;  // the last run start (list-relative) before this chunk
  uint32_t mj = 0, va = 0xFFFFFFFFu, vo = 0;
  for (uint64_t c = b; c < e; c += 64) {
    const uint64_t i = c + lane;
    const bool live = i < e;
    const uint32_t v = live ? vals[i] : 0u;
    const bool start = live && (i == b || vals[i - 1] != v);
    const int rs = max(sgd::wave_incl_max(start ? (int)(i - b) : -1), carry);
    const uint32_t j = (uint32_t)((int)(i - b) - rs);
    if (live) {
      if (kKeys)
        keys[i] = gtop | ((uint64_t)v << jb) | j;
      else {
        mj = max(mj, j);
        va &= v;
        vo |= v;
      }
    }
    carry = __builtin_amdgcn_readlane(rs, 63);
  }
  if (!kKeys) {
    for (int d = 32; d; d >>= 1) {
      mj = max(mj, (uint32_t)__shfl_xor((int)mj, d));
      va &= (uint32_t)__shfl_xor((int)va, d);
      vo |= (uint32_t)__shfl_xor((int)vo, d);
    }
    // (read-checked: an atomic only when it changes the word -- every wave's
    // atomic on the same three words cost ~1 ms per 50K lists)
    if (lane == 0) {
      if (mj > __hip_atomic_load(&stats[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMax(&stats[0], (unsigned long long)mj);
      const unsigned long long a = __hip_atomic_load(&stats[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((a & va) != a) atomicAnd(&stats[1], (unsigned long long)va);
      const unsigned long long o = __hip_atomic_load(&stats[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((o | vo) != o) atomicOr(&stats[2], (unsigned long long)vo);
    }
  }
}

// The unique pass over the sorted keys, as a tile compaction (tiles of 8192
// keys, 512 threads, wave w owning positions [1024 w, +1024) as 16 steps of
// 64): a key is kept when it starts its run and its value is not the sentinel
// (cover.go:97).  k_fold_count counts a tile's kept keys; k_fold_write, after
// a scan of those counts, writes the kept values in order and, at each
// group's first key, the group's output start (the kept keys before it).
constexpr int kFuThreads = 512, kFuSteps = 16;
constexpr uint32_t kFuTile = kFuThreads * kFuSteps;

__device__ __forceinline__ bool fold_kept(const uint64_t* keys, uint64_t i, uint32_t jb) {
  const uint64_t k = keys[i];
  return (i == 0 || keys[i - 1] != k) && (uint32_t)(k >> jb) != 0xFFFFFFFFu;
}

__global__ __launch_bounds__(kFuThreads) void k_fold_count(const uint64_t* __restrict__ keys, uint64_t n, uint32_t jb,
                                                           uint32_t* __restrict__ tcnt) {
  __shared__ uint32_t ws[kFuThreads / 64];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const uint64_t base = (uint64_t)blockIdx.x * kFuTile + (uint64_t)w * (64 * kFuSteps);
  uint32_t c = 0;
  for (int s = 0; s < kFuSteps; s++) {
    const uint64_t i = base + s * 64 + lane;
    c += (uint32_t)__popcll(__ballot(i < n && fold_kept(keys, i, jb)));
  }
  if (lane == 0) ws[w] = c;
  __syncthreads();
  if (tid == 0) {
    uint32_t t = 0;
    for (int j = 0; j < kFuThreads / 64; j++) t += ws[j];
    tcnt[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kFuThreads) void k_fold_write(const uint64_t* __restrict__ keys, uint64_t n, uint32_t jb,
                                                           const uint64_t* __restrict__ tpos, uint32_t* __restrict__ out,
                                                           uint64_t* __restrict__ first) {
  __shared__ uint32_t ws[kFuThreads / 64];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const uint64_t base = (uint64_t)blockIdx.x * kFuTile + (uint64_t)w * (64 * kFuSteps);
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t c = 0;
  for (int s = 0; s < kFuSteps; s++) {
    const uint64_t i = base + s * 64 + lane;
    c += (uint32_t)__popcll(__ballot(i < n && fold_kept(keys, i, jb)));
  }
  if (lane == 0) ws[w] = c;
  __syncthreads();
  uint64_t pos = tpos[blockIdx.x];
  for (int j = 0; j < w; j++) pos += ws[j];
  for (int s = 0; s < kFuSteps; s++) {
    const uint64_t i = base + s * 64 + lane;
    const bool live = i < n;
    const uint64_t k = live ? keys[i] : 0ull;
    const uint64_t prev = live && i ? keys[i - 1] : ~k;
    const bool kept = live && prev != k && (uint32_t)(k >> jb) != 0xFFFFFFFFu;
    const uint64_t m = __ballot(kept);
    const uint64_t at = pos + (uint64_t)__popcll(m & lt);
    if (kept) out[at] = (uint32_t)(k >> jb);
    const uint64_t g = k >> (32 + jb);
    if (live && (i == 0 || (prev >> (32 + jb)) != g)) first[g] = at;  // this group's first key
    pos += (uint64_t)__popcll(m);
  }
}

// One group of canonical lists (no value repeats inside a list, jb = 0; the
// corpus fold of html.go:306 is one) whose values span at most 2^28: the fold
// is the set of values seen, ascending, the sentinel dropped (cover.go:63-70,
// :97 with every count 1), i.e. a byte map over [AND, OR] of the values --
// byte stores of 1 (no atomics; repeats across lists store the same byte),
// then one ordered compaction of the map -- instead of sorting 64-bit keys.
constexpr uint64_t kFoldMapMax = 1ull << 28;
constexpr int kFmThreads = 256;
constexpr uint32_t kFmTile = kFmThreads * 16;  // map bytes per compaction tile

__global__ void k_fold_mark(const uint32_t* __restrict__ v, uint64_t n, uint32_t lo, uint8_t* __restrict__ map) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t x = v[i];
    if (x != 0xFFFFFFFFu) map[x - lo] = 1;
  }
}

__device__ __forceinline__ uint32_t nz_bytes(uint32_t w) {  // nonzero bytes of w (bytes are 0 or 1)
  return (uint32_t)__popc(w & 0x01010101u);
}

__global__ __launch_bounds__(kFmThreads) void k_fold_map_count(const uint8_t* __restrict__ map, uint64_t range,
                                                               uint32_t* __restrict__ tcnt) {
  __shared__ uint32_t ws[kFmThreads / 64];
  const uint64_t b = (uint64_t)blockIdx.x * kFmTile + threadIdx.x * 16u;
  uint32_t c = 0;
  if (b < range) {  // (the map is padded to whole tiles, zeroed)
    const uint4 q = *reinterpret_cast<const uint4*>(map + b);
    c = nz_bytes(q.x) + nz_bytes(q.y) + nz_bytes(q.z) + nz_bytes(q.w);
  }
  c = sgd::wave_incl_add(c);
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int i = 0; i < kFmThreads / 64; i++) t += ws[i];
    tcnt[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kFmThreads) void k_fold_map_write(const uint8_t* __restrict__ map, uint64_t range,
                                                               uint32_t lo, const uint64_t* __restrict__ tpos,
                                                               uint32_t* __restrict__ out) {
  __shared__ uint32_t ws[kFmThreads / 64];
  const uint64_t b = (uint64_t)blockIdx.x * kFmTile + threadIdx.x * 16u;
  uint4 q = make_uint4(0, 0, 0, 0);
  if (b < range) q = *reinterpret_cast<const uint4*>(map + b);
  const uint32_t c = nz_bytes(q.x) + nz_bytes(q.y) + nz_bytes(q.z) + nz_bytes(q.w);
  const uint32_t incl = sgd::wave_incl_add(c);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) ws[w] = incl;
  __syncthreads();
  uint32_t before = 0;
  for (int i = 0; i < w; i++) before += ws[i];
  uint64_t at = tpos[blockIdx.x] + before + incl - c;
  const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int j = 0; j < 16; j++)
    if ((qw[j >> 2] >> (8 * (j & 3))) & 0xFFu) out[at++] = lo + (uint32_t)(b + j);
}

// Many groups of canonical lists (the per-syscall folds of html.go:84, each
// group a few thousand PCs): a workgroup per group sorts the group's values in
// LDS (stable 8-bit LSD passes over the bits that vary within the group, each
// pass a wave multisplit rank, a scan of the 256 digit counts and a scatter
// through LDS) and keeps the first of each run, the sentinel dropped -- one
// read of the values and one write of the folds, where the 64-bit key sort
// made five passes over (group, value) keys.  Groups are packed group-major
// first; the groups of more than kFgCap values take the key sort, beside.
constexpr int kFgSteps = 16;
constexpr uint32_t kFgCap = 1024 * 2 * kFgSteps;  // 32768 values per group (the 1024 x 32 form)

__device__ __forceinline__ uint64_t fg_peers(uint32_t d, bool live) {  // lanes holding digit d
  uint64_t eq = __ballot(live);
#pragma unroll
  for (int b = 0; b < 8; b++) {
    const uint64_t bal = __ballot((d >> b) & 1u);
    eq &= ((d >> b) & 1u) ? bal : ~bal;
  }
  return eq;
}

// kT threads, kS steps of 64 values per wave: groups of <= kT kS values (the
// host gives each form its groups: 512 x 16 for <= 8192 values, four
// workgroups per CU; 1024 x 16 for <= 16384; 1024 x 32, 144 KiB of LDS, for
// <= 32768).  A wave's steps past the group's end are skipped (wave-uniform).
template <int kT, int kS>
__global__ __launch_bounds__(kT) void k_fold_lds(const uint32_t* __restrict__ packed, const uint64_t* __restrict__ gstart,
                                                 const uint32_t* __restrict__ glist, uint32_t* __restrict__ out,
                                                 uint32_t* __restrict__ gcnt, const uint32_t* __restrict__ rep) {
  constexpr int kW = kT / 64;
  constexpr uint32_t kCap = kT * kS;
  __shared__ uint32_t stage[kCap];
  __shared__ uint32_t cnt[kW][256];  // per-wave digit counts, then the waves' offsets in the digit
  __shared__ uint32_t dstart[256];
  __shared__ uint32_t red[2][kW];
  // a list repeats a value (k_fold_pack_chk, stream-ordered before): the host
  // redoes the fold through the multiset key path, so this one does nothing
  if (__builtin_amdgcn_readfirstlane(*rep)) return;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const uint32_t g = glist[blockIdx.x];
  const uint64_t b0 = gstart[g];
  const uint32_t n = (uint32_t)(gstart[g + 1] - b0);
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  // positions of wave w: [64 kS w, + 64 kS), step s at + 64 s + lane
  const uint32_t base = (uint32_t)w * 64 * kS;
  const int nst = base >= n ? 0 : (int)min<uint32_t>(kS, (n - base + 63) / 64);  // this wave's live steps
  uint32_t k[kS];
  uint32_t va = 0xFFFFFFFFu, vo = 0;
#pragma unroll
  for (int st = 0; st < kS; st++) {
    const uint32_t p = base + st * 64 + lane;
    k[st] = 0xFFFFFFFFu;
    if (st < nst && p < n) {
      k[st] = packed[b0 + p];
      va &= k[st];
      vo |= k[st];
    }
  }
  // the bits that vary within the group
#pragma unroll
  for (int d = 32; d; d >>= 1) {
    va &= (uint32_t)__shfl_xor((int)va, d);
    vo |= (uint32_t)__shfl_xor((int)vo, d);
  }
  if (lane == 0) {
    red[0][w] = va;
    red[1][w] = vo;
  }
  __syncthreads();
  uint32_t A = 0xFFFFFFFFu, O = 0;
#pragma unroll
  for (int i = 0; i < kW; i++) {
    A &= red[0][i];
    O |= red[1][i];
  }
  const uint32_t vary = A ^ O;
  // 8-bit digits from the lowest varying bit (PCs 16 B apart: bits 4.. -- one
  // pass fewer than digits at bit 0)
  for (uint32_t shift = vary ? (uint32_t)__builtin_ctz(vary) : 32u; shift < 32; shift += 8) {
    if (((vary >> shift) & 255u) == 0) continue;  // (block-uniform)
    for (int i = tid; i < kW * 256; i += kT) (&cnt[0][0])[i] = 0;
    __syncthreads();
    uint32_t rank[kS];
#pragma unroll
    for (int st = 0; st < kS; st++) {
      rank[st] = 0;
      if (st < nst) {  // (wave-uniform)
        const bool live = base + st * 64 + lane < n;
        const uint32_t d = (k[st] >> shift) & 255u;
        const uint64_t eq = fg_peers(d, live);
        const uint32_t before = live ? cnt[w][d] : 0u;
        rank[st] = before + (uint32_t)__popcll(eq & lt);
        if (live && (eq & lt) == 0) cnt[w][d] = before + (uint32_t)__popcll(eq);
      }
    }
    __syncthreads();
    if (tid < 256) {  // per digit: the waves' offsets, the digit's count
      uint32_t acc = 0;
#pragma unroll
      for (int i = 0; i < kW; i++) {
        const uint32_t c = cnt[i][tid];
        cnt[i][tid] = acc;
        acc += c;
      }
      dstart[tid] = acc;
    }
    __syncthreads();
    if (tid < 64) {  // exclusive scan of the 256 digit counts
      uint32_t c[4], sum = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        c[j] = dstart[tid * 4 + j];
        sum += c[j];
      }
      uint32_t run = sgd::wave_incl_add(sum) - sum;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        dstart[tid * 4 + j] = run;
        run += c[j];
      }
    }
    __syncthreads();
#pragma unroll
    for (int st = 0; st < kS; st++) {
      if (st >= nst) break;
      if (base + st * 64 + lane < n) {
        const uint32_t d = (k[st] >> shift) & 255u;
        stage[dstart[d] + cnt[w][d] + rank[st]] = k[st];
      }
    }
    __syncthreads();
#pragma unroll
    for (int st = 0; st < kS; st++) {
      if (st >= nst) break;
      const uint32_t p = base + st * 64 + lane;
      k[st] = p < n ? stage[p] : 0xFFFFFFFFu;
    }
    __syncthreads();
  }
  // sorted: keep the first of each run, the sentinel dropped (cover.go:63-70, :97)
#pragma unroll
  for (int st = 0; st < kS; st++) {
    if (st >= nst) break;
    stage[base + st * 64 + lane] = k[st];
  }
  __syncthreads();
  uint32_t keep = 0, c = 0;
#pragma unroll
  for (int st = 0; st < kS; st++) {
    if (st < nst) {
      const uint32_t p = base + st * 64 + lane;
      const bool kp = p < n && k[st] != 0xFFFFFFFFu && (p == 0 || stage[p - 1] != k[st]);
      keep |= (kp ? 1u : 0u) << st;
      c += (uint32_t)__popcll(__ballot(kp));
    }
  }
  if (lane == 0) red[0][w] = c;
  __syncthreads();
  uint32_t at = 0;
  for (int i = 0; i < w; i++) at += red[0][i];
  if (tid == kT - 1) {
    uint32_t t = 0;
    for (int i = 0; i < kW; i++) t += red[0][i];
    gcnt[g] = t;
  }
#pragma unroll
  for (int st = 0; st < kS; st++) {
    if (st < nst) {
      const bool kp = (keep >> st) & 1u;
      const uint64_t m = __ballot(kp);
      if (kp) out[b0 + at + (uint32_t)__popcll(m & lt)] = k[st];
      at += (uint32_t)__popcll(m);
    }
  }
}

// dst[doff[g] ..] = src[sbeg[g] .. + len[g]) for u32 lengths, one wave per group
__global__ void k_fold_move(const uint32_t* __restrict__ src, const uint64_t* __restrict__ sbeg,
                            const uint32_t* __restrict__ len, const uint64_t* __restrict__ doff, uint64_t n,
                            uint32_t* __restrict__ dst, const uint32_t* __restrict__ rep) {
  if (__builtin_amdgcn_readfirstlane(*rep)) return;  // (the LDS folds were skipped: the lengths are stale)
  const uint64_t g = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (g >= n) return;
  const uint64_t s = sbeg[g], d = doff[g], L = len[g];
  for (uint64_t i = threadIdx.x & 63; i < L; i += 64) dst[d + i] = src[s + i];
}

// Groups of more than kFgCap values (beside the LDS-folded ones): each big
// group's packed values as keys b << 32 | v (b = the group's index among the
// big ones) at bk[b] .., for the key sort; grid (x, nbig).
__global__ void k_fold_bigkeys(const uint32_t* __restrict__ packed, const uint64_t* __restrict__ gs,
                               const uint32_t* __restrict__ blist, const uint64_t* __restrict__ bk,
                               uint64_t* __restrict__ keys) {
  const uint32_t b = blockIdx.y, g = blist[b];
  const uint64_t src = gs[g], len = gs[g + 1] - src, dst = bk[b];
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (uint64_t)gridDim.x * blockDim.x)
    keys[dst + i] = ((uint64_t)b << 32) | packed[src + i];
}

// Each big group's fold (the unique pass's output from first[b] to first[b +
// 1], or the total for the last) into folded at the group's start, its count
// into gcnt -- where the LDS fold leaves the small groups'.  A block per group.
__global__ void k_fold_bigmove(const uint32_t* __restrict__ uout, const uint64_t* __restrict__ first,
                               const uint64_t* __restrict__ total, uint32_t nbig, const uint32_t* __restrict__ blist,
                               const uint64_t* __restrict__ gs, uint32_t* __restrict__ folded,
                               uint32_t* __restrict__ gcnt) {
  const uint32_t b = blockIdx.x, g = blist[b];
  const uint64_t s = first[b], e = b + 1 < nbig ? first[b + 1] : *total, d = gs[g];
  for (uint64_t i = threadIdx.x; i < e - s; i += blockDim.x) folded[d + i] = uout[s + i];
  if (threadIdx.x == 0) gcnt[g] = (uint32_t)(e - s);
}

constexpr int SG_EOVERFLOW_FOLD = 1;  // internal: the keys do not fit 64 bits
constexpr int SG_EREPEATS_FOLD = 2;   // internal: not the per-group LDS fold's (a list repeats a value, or
                                      // more big groups than one launch's grid holds): the key sort

static uint32_t bits_for(uint64_t x) { return x ? 64u - (uint32_t)__builtin_clzll(x) : 0u; }

// The per-group LDS fold (k_fold_lds): the lists packed group-major, a
// workgroup per group, the folds moved together (ctx lock held).  Groups of
// more than kFgCap values (a few, when some inputs are long) are folded beside
// them by the 64-bit key sort over their values alone.
static int fold_groups_lds(sg_ctx* ctx, const uint32_t* dv, const uint64_t* off, size_t n, const uint32_t* group,
                           size_t ngroups, const std::vector<uint64_t>& gs, uint32_t* out_vals, size_t cap,
                           uint64_t* out_off) {
  const uint64_t N = gs[ngroups];
  // every list's place in the group-major packing: its group's start + the
  // lengths of the group's earlier lists (host, from the offsets it was given)
  std::vector<uint64_t> lst(n), len(n), at(gs.begin(), gs.end() - 1);
  // the big groups, their keys' places
  std::vector<uint32_t> bl;
  std::vector<uint64_t> bk(1, 0);
  for (uint32_t gi = 0; gi < ngroups; gi++)
    if (gs[gi + 1] - gs[gi] > kFgCap) {
      bl.push_back(gi);
      bk.push_back(bk.back() + (gs[gi + 1] - gs[gi]));
    }
  if (bl.size() > 65535) return SG_EREPEATS_FOLD;  // (k_fold_bigkeys: a grid row per big group)
  const uint32_t nbig = (uint32_t)bl.size();
  const uint64_t NB = bk.back(), ntb = div_up(NB, (uint64_t)kFuTile);
  WsPlan p;
  const size_t oP = p.add(N * 4), oO = p.add(N * 4), oG = p.add((ngroups + 1) * 8), oL = p.add(n * 8),
               oB = p.add(n * 8), oN = p.add(n * 8), oC = p.add(ngroups * 4), oF = p.add((ngroups + 1) * 8),
               oQ = p.add(ngroups * 4), oR = p.add(4), oKA = p.add(NB * 8), oKB = p.add(NB * 8),
               oBL = p.add(nbig * 4 + 4), oBK = p.add((nbig + 1) * 8), oBF = p.add(nbig * 8 + 8),
               oTC = p.add(ntb * 4 + 4), oTP = p.add((ntb + 1) * 8);
  int rc = ws_reserve(ctx, p.total + std::max({scan_ws_bytes(ngroups), nbig ? radix_sort_ws(NB) : 0,
                                               nbig ? scan_ws_bytes(ntb) : 0}));
  if (rc) return rc;
  uint32_t* packed = (uint32_t*)ws_at(ctx, oP);
  uint32_t* folded = (uint32_t*)ws_at(ctx, oO);
  uint64_t* dgs = (uint64_t*)ws_at(ctx, oG);
  uint64_t* dlst = (uint64_t*)ws_at(ctx, oL);
  uint64_t* dbeg = (uint64_t*)ws_at(ctx, oB);
  uint64_t* dlen = (uint64_t*)ws_at(ctx, oN);
  uint32_t* gcnt = (uint32_t*)ws_at(ctx, oC);
  uint64_t* fo = (uint64_t*)ws_at(ctx, oF);
  uint32_t* dq = (uint32_t*)ws_at(ctx, oQ);
  uint32_t* rep = (uint32_t*)ws_at(ctx, oR);
  // the groups by form: <= 8192 values (512 x 16), <= 16384 (1024 x 16),
  // <= kFgCap (1024 x 32), the big ones (the key sort)
  std::vector<uint32_t> ql;
  uint32_t nform[3] = {0, 0, 0};
  const uint64_t lim[4] = {0, 512u * kFgSteps, 1024u * kFgSteps, kFgCap};
  for (int f = 0; f < 3; f++) {
    for (uint32_t gi = 0; gi < ngroups; gi++)
      if ((f == 0 || gs[gi + 1] - gs[gi] > lim[f]) && gs[gi + 1] - gs[gi] <= lim[f + 1]) ql.push_back(gi);
    nform[f] = (uint32_t)ql.size();
  }
  ql.resize(ngroups);  // (the tail unused)
  for (size_t k = 0; k < n; k++) {
    const uint32_t gi = group ? group[k] : 0u;
    len[k] = off[k + 1] - off[k];
    lst[k] = at[gi];
    at[gi] += len[k];
  }
  SG_HIP(hipMemcpyAsync(dgs, gs.data(), (ngroups + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dq, ql.data(), ngroups * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemsetAsync(rep, 0, 4, ctx->stream));
  SG_HIP(hipMemcpyAsync(dlst, lst.data(), n * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dbeg, off, n * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dlen, len.data(), n * 8, hipMemcpyHostToDevice, ctx->stream));
  {
    ScopedTimer tm(ctx, "union_fold");
    {
      ScopedTimer tk(ctx, "fold_pack");
      hipLaunchKernelGGL(k_fold_pack_chk, dim3(div_up(n, 4)), dim3(256), 0, ctx->stream, dv, (const uint64_t*)dbeg,
                         (const uint64_t*)dlen, (const uint64_t*)dlst, (uint64_t)n, packed, rep);
    }
    {
      ScopedTimer tk(ctx, "fold_lds");
      if (nform[0])
        hipLaunchKernelGGL((k_fold_lds<512, kFgSteps>), dim3(nform[0]), dim3(512), 0, ctx->stream,
                           (const uint32_t*)packed, (const uint64_t*)dgs, (const uint32_t*)dq, folded, gcnt, (const uint32_t*)rep);
      if (nform[1] > nform[0])
        hipLaunchKernelGGL((k_fold_lds<1024, kFgSteps>), dim3(nform[1] - nform[0]), dim3(1024), 0, ctx->stream,
                           (const uint32_t*)packed, (const uint64_t*)dgs, (const uint32_t*)dq + nform[0], folded,
                           gcnt, (const uint32_t*)rep);
      if (nform[2] > nform[1])
        hipLaunchKernelGGL((k_fold_lds<1024, 2 * kFgSteps>), dim3(nform[2] - nform[1]), dim3(1024), 0, ctx->stream,
                           (const uint32_t*)packed, (const uint64_t*)dgs, (const uint32_t*)dq + nform[1], folded,
                           gcnt, (const uint32_t*)rep);
    }
    if (nbig) {
      ScopedTimer tk(ctx, "fold_big");
      uint64_t* ka = (uint64_t*)ws_at(ctx, oKA);
      uint64_t* kb = (uint64_t*)ws_at(ctx, oKB);
      uint32_t* dbl = (uint32_t*)ws_at(ctx, oBL);
      uint64_t* dbk = (uint64_t*)ws_at(ctx, oBK);
      uint64_t* bfirst = (uint64_t*)ws_at(ctx, oBF);
      uint32_t* tcnt = (uint32_t*)ws_at(ctx, oTC);
      uint64_t* tpos = (uint64_t*)ws_at(ctx, oTP);
      SG_HIP(hipMemcpyAsync(dbl, bl.data(), nbig * 4, hipMemcpyHostToDevice, ctx->stream));
      SG_HIP(hipMemcpyAsync(dbk, bk.data(), (nbig + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
      hipLaunchKernelGGL(k_fold_bigkeys, dim3(64, nbig), dim3(256), 0, ctx->stream, (const uint32_t*)packed,
                         (const uint64_t*)dgs, (const uint32_t*)dbl, (const uint64_t*)dbk, ka);
      const uint32_t bb = bits_for(nbig - 1);
      uint64_t* sorted = nullptr;
      rc = radix_sort_u64(ctx, ka, kb, NB, p.total, &sorted, (((1ull << bb) - 1) << 32) | 0xFFFFFFFFull);
      if (rc) return rc;
      uint32_t* uout = (uint32_t*)(sorted == ka ? kb : ka);  // (the other key buffer, free now)
      hipLaunchKernelGGL(k_fold_count, dim3((uint32_t)ntb), dim3(kFuThreads), 0, ctx->stream, (const uint64_t*)sorted,
                         NB, 0u, tcnt);
      rc = scan_counts(ctx, tcnt, tpos, ntb, p.total);
      if (rc) return rc;
      hipLaunchKernelGGL(k_fold_write, dim3((uint32_t)ntb), dim3(kFuThreads), 0, ctx->stream, (const uint64_t*)sorted,
                         NB, 0u, (const uint64_t*)tpos, uout, bfirst);
      hipLaunchKernelGGL(k_fold_bigmove, dim3(nbig), dim3(256), 0, ctx->stream, (const uint32_t*)uout,
                         (const uint64_t*)bfirst, (const uint64_t*)(tpos + ntb), nbig, (const uint32_t*)dbl,
                         (const uint64_t*)dgs, folded, gcnt);
    }
    rc = scan_counts(ctx, gcnt, fo, ngroups, p.total);
    if (rc) return rc;
    {
      ScopedTimer tk(ctx, "fold_move");
      hipLaunchKernelGGL(k_fold_move, dim3(div_up(ngroups, 4)), dim3(256), 0, ctx->stream, (const uint32_t*)folded,
                         (const uint64_t*)dgs, (const uint32_t*)gcnt, (const uint64_t*)fo, (uint64_t)ngroups, packed,
                         (const uint32_t*)rep);
    }
    SG_HIP(hipGetLastError());
  }
  uint32_t hrep = 0;
  SG_HIP(hipMemcpyAsync(out_off, fo, (ngroups + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipMemcpyAsync(&hrep, rep, 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (hrep) return SG_EREPEATS_FOLD;  // (not canonical: the multiset fold)
  const uint64_t total = out_off[ngroups];
  if (total > cap) {
    set_error("sg_union_fold: %llu values, capacity %zu", (unsigned long long)total, cap);
    return SG_EINVAL;
  }
  if (total == 0) return SG_OK;
  if (!out_vals) return SG_EINVAL;
  SG_HIP(hipMemcpyAsync(out_vals, packed, total * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

// The sort + unique fold (ctx lock held; arguments checked, N > 0).
static int fold_sorted(sg_ctx* ctx, const uint32_t* vals, const uint64_t* off, size_t n, const uint32_t* group,
                       size_t ngroups, uint32_t* out_vals, size_t cap, uint64_t* out_off) {
  const uint64_t N = off[n];
  const uint32_t gb = bits_for(ngroups - 1);
  if (gb + 32 > 64) return SG_EOVERFLOW_FOLD;
  // inputs: values, offsets, groups (device staging)
  const size_t b_v = (N * 4 + 255) & ~size_t(255), b_o = ((n + 1) * 8 + 255) & ~size_t(255),
               b_g = (n * 4 + 255) & ~size_t(255);
  int rc = dstage_reserve(ctx, b_v + b_o + b_g + 256);
  if (rc) return rc;
  uint32_t* dv = (uint32_t*)ctx->dstage;
  uint64_t* doff = (uint64_t*)((char*)ctx->dstage + b_v);
  uint32_t* dgrp = group ? (uint32_t*)((char*)ctx->dstage + b_v + b_o) : nullptr;
  // workspace: keys (2 buffers), keep flags, their scan, group first indices / positions, max j
  WsPlan p;
  const uint64_t ntile = (N + kFuTile - 1) / kFuTile;
  const size_t oA = p.add(N * 8), oB = p.add(N * 8), oK = p.add(ntile * 4), oP = p.add((ntile + 1) * 8),
               oF = p.add(ngroups * 8), oJ = p.add(24);
  const size_t sort_at = p.total, need = p.total + std::max(radix_sort_ws(N), scan_ws_bytes(ntile));
  rc = ws_reserve(ctx, need);
  if (rc) return rc;
  uint64_t *ka = (uint64_t*)ws_at(ctx, oA), *kb = (uint64_t*)ws_at(ctx, oB), *tpos = (uint64_t*)ws_at(ctx, oP);
  uint32_t* tcnt = (uint32_t*)ws_at(ctx, oK);
  uint64_t* first = (uint64_t*)ws_at(ctx, oF);
  unsigned long long* stats = (unsigned long long*)ws_at(ctx, oJ);  // max j, AND and OR of the values
  SG_HIP(hipMemcpyAsync(dv, vals, N * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(doff, off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  if (group) SG_HIP(hipMemcpyAsync(dgrp, group, n * 4, hipMemcpyHostToDevice, ctx->stream));
  if (ngroups > 1) {
    // many groups of canonical covers: the per-group fold (it checks for
    // repeats itself; a list with one takes the key sort below)
    std::vector<uint64_t> gs(ngroups + 1, 0);
    for (size_t k = 0; k < n; k++) gs[(group ? group[k] : 0) + 1] += off[k + 1] - off[k];
    uint64_t gmax = 0;
    for (size_t gi = 0; gi < ngroups; gi++) {
      gmax = std::max(gmax, gs[gi + 1]);
      gs[gi + 1] += gs[gi];
    }
    if (gmax < (1ull << 32)) {  // (group folds counted in 32 bits)
      rc = fold_groups_lds(ctx, dv, off, n, group, ngroups, gs, out_vals, cap, out_off);
      if (rc != SG_EREPEATS_FOLD) return rc;
      rc = ws_reserve(ctx, need);  // (the workspace may have moved)
      if (rc) return rc;
      ka = (uint64_t*)ws_at(ctx, oA), kb = (uint64_t*)ws_at(ctx, oB), tpos = (uint64_t*)ws_at(ctx, oP);
      tcnt = (uint32_t*)ws_at(ctx, oK);
      first = (uint64_t*)ws_at(ctx, oF);
      stats = (unsigned long long*)ws_at(ctx, oJ);
    }
  }
  unsigned long long st[3] = {0, 0xFFFFFFFFull, 0};
  SG_HIP(hipMemcpyAsync(stats, st, 24, hipMemcpyHostToDevice, ctx->stream));
  const dim3 lgrid(div_up(n, 4));
  {
    ScopedTimer tm(ctx, "union_fold");
    hipLaunchKernelGGL(k_fold_runs<false>, lgrid, dim3(256), 0, ctx->stream, dv, doff, (uint64_t)n, dgrp, 0u, stats,
                       nullptr);
  }
  SG_HIP(hipMemcpyAsync(st, stats, 24, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  const uint32_t jb = bits_for(st[0]);
  if (gb + 32 + jb > 64) return SG_EOVERFLOW_FOLD;
  const uint64_t range = st[2] - st[1] + 1;     // values lie in [AND, OR]
  // the map's passes cost ~3 bytes of traffic per value of the range, the
  // sort ~48 per key: the map only for a range dense enough (a few thousand
  // PCs spread over 2^28 would memset and scan 256 MiB -- and keep it in the
  // grow-only workspace -- to fold what the sort folds in microseconds)
  const bool dense = range <= kFoldMapMax && range <= std::max<uint64_t>(1ull << 20, 16 * N);
  if (ngroups == 1 && jb == 0 && dense && ctx->opt[kOptFoldMap] != 0) {  // (option fold_map 0: always the sort, a test hook)
    const uint64_t nt = div_up(range, (uint64_t)kFmTile);
    WsPlan q;
    const size_t qM = q.add(nt * kFmTile), qC = q.add(nt * 4), qP = q.add((nt + 1) * 8), qO = q.add(N * 4);
    rc = ws_reserve(ctx, q.total + scan_ws_bytes(nt));
    if (rc) return rc;
    uint8_t* map = (uint8_t*)ws_at(ctx, qM);
    uint32_t* mc = (uint32_t*)ws_at(ctx, qC);
    uint64_t* mp = (uint64_t*)ws_at(ctx, qP);
    uint32_t* mo = (uint32_t*)ws_at(ctx, qO);
    const uint32_t lo = (uint32_t)st[1];
    {
      ScopedTimer tm(ctx, "union_fold");
      ScopedTimer tk(ctx, "fold_map");
      SG_HIP(hipMemsetAsync(map, 0, nt * kFmTile, ctx->stream));
      hipLaunchKernelGGL(k_fold_mark, dim3((uint32_t)std::min<uint64_t>(div_up(N, 256), 8192)), dim3(256), 0,
                         ctx->stream, dv, N, lo, map);
      hipLaunchKernelGGL(k_fold_map_count, dim3((uint32_t)nt), dim3(kFmThreads), 0, ctx->stream, map, range, mc);
      rc = scan_counts(ctx, mc, mp, nt, q.total);
      if (rc) return rc;
      hipLaunchKernelGGL(k_fold_map_write, dim3((uint32_t)nt), dim3(kFmThreads), 0, ctx->stream, map, range, lo,
                         (const uint64_t*)mp, mo);
      SG_HIP(hipGetLastError());
    }
    uint64_t total = 0;
    SG_HIP(hipMemcpyAsync(&total, mp + nt, 8, hipMemcpyDeviceToHost, ctx->stream));
    SG_HIP(hipStreamSynchronize(ctx->stream));
    out_off[0] = 0;
    out_off[1] = total;
    if (total > cap) {
      set_error("sg_union_fold: %llu values, capacity %zu", (unsigned long long)total, cap);
      return SG_EINVAL;
    }
    if (total == 0) return SG_OK;
    if (!out_vals) return SG_EINVAL;
    SG_HIP(hipMemcpyAsync(out_vals, mo, total * 4, hipMemcpyDeviceToHost, ctx->stream));
    SG_HIP(hipStreamSynchronize(ctx->stream));
    return SG_OK;
  }
  // the key bits that vary: the group's, the values' (AND vs OR), the copy index's
  const uint64_t vary = ((gb ? ((1ull << gb) - 1) : 0ull) << (32 + jb)) | ((st[1] ^ st[2]) << jb) |
                        (jb ? (1ull << jb) - 1 : 0ull);
  uint64_t* sorted = nullptr;
  uint32_t* dout = nullptr;
  {
    ScopedTimer tm(ctx, "union_fold");
    {
      ScopedTimer tk(ctx, "fold_keys");
      hipLaunchKernelGGL(k_fold_runs<true>, lgrid, dim3(256), 0, ctx->stream, dv, doff, (uint64_t)n, dgrp, jb, stats,
                         ka);
    }
    {
      ScopedTimer ts(ctx, "fold_sort");
      rc = radix_sort_u64(ctx, ka, kb, N, sort_at, &sorted, vary);
      if (rc) return rc;
    }
    ScopedTimer tu(ctx, "fold_unique");
    SG_HIP(hipMemsetAsync(first, 0xFF, ngroups * 8, ctx->stream));
    hipLaunchKernelGGL(k_fold_count, dim3((uint32_t)ntile), dim3(kFuThreads), 0, ctx->stream, (const uint64_t*)sorted, N,
                       jb, tcnt);
    rc = scan_counts(ctx, tcnt, tpos, ntile, sort_at);
    if (rc) return rc;
    dout = (uint32_t*)(sorted == ka ? kb : ka);  // the other key buffer, free now
    hipLaunchKernelGGL(k_fold_write, dim3((uint32_t)ntile), dim3(kFuThreads), 0, ctx->stream, (const uint64_t*)sorted, N,
                       jb, (const uint64_t*)tpos, dout, first);
    SG_HIP(hipGetLastError());
  }
  std::vector<uint64_t> f(ngroups);
  uint64_t total = 0;
  SG_HIP(hipMemcpyAsync(f.data(), first, ngroups * 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipMemcpyAsync(&total, tpos + ntile, 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  out_off[ngroups] = total;
  for (size_t gi = ngroups; gi-- > 0;) out_off[gi] = f[gi] == ~0ull ? out_off[gi + 1] : f[gi];
  if (total > cap) {
    set_error("sg_union_fold: %llu values, capacity %zu", (unsigned long long)total, cap);
    return SG_EINVAL;
  }
  if (total == 0) return SG_OK;
  if (!out_vals) return SG_EINVAL;
  SG_HIP(hipMemcpyAsync(out_vals, dout, total * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

}  // namespace
}  // namespace sg

using namespace sg;

extern "C" {

int sg_union_fold(sg_ctx* ctx, const uint32_t* vals, const uint64_t* off, size_t n, const uint32_t* group,
                  size_t ngroups, uint32_t* out_vals, size_t cap, uint64_t* out_off) {
  if (!ctx || !off || !out_off || ngroups == 0 || (off[n] && !vals)) {
    set_error("sg_union_fold: invalid argument");
    return SG_EINVAL;
  }
  if (off[0] != 0) {
    set_error("sg_union_fold: off[0] != 0");
    return SG_EINVAL;
  }
  for (size_t k = 0; k < n; k++) {
    if (off[k + 1] < off[k] || (group && group[k] >= ngroups)) {
      set_error("sg_union_fold: list %zu: bad offsets or group", k);
      return SG_EINVAL;
    }
  }
  const uint64_t N = off[n];
  std::fill(out_off, out_off + ngroups + 1, 0);
  if (N == 0) return SG_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  rc = fold_sorted(ctx, vals, off, n, group, ngroups, out_vals, cap, out_off);
  if (rc != SG_EOVERFLOW_FOLD) return rc;
  // (g, v, j) does not fit 64 bits: a balanced tree of batched Unions, one
  // launch per level over all groups
  std::fill(out_off, out_off + ngroups + 1, 0);
  // the lists of each group, in input order (the order does not change the result)
  std::vector<std::vector<Item>> items(ngroups);
  for (size_t k = 0; k < n; k++) items[group ? group[k] : 0].push_back({off[k], off[k + 1] - off[k]});
  // two ping-pong buffers of N values: a level's results never exceed its inputs
  const size_t b_v = (N * 4 + 255) & ~size_t(255);
  rc = dstage_reserve(ctx, 2 * b_v + 4 * ((ngroups + 1) * 8 + 256));
  if (rc) return rc;
  uint32_t* buf[2] = {(uint32_t*)ctx->dstage, (uint32_t*)((char*)ctx->dstage + b_v)};
  SG_HIP(hipMemcpyAsync(buf[0], vals, N * 4, hipMemcpyHostToDevice, ctx->stream));
  int cur = 0;
  std::vector<uint64_t> ab, al, bb, bl, ob, ol;
  std::vector<std::pair<size_t, size_t>> who;  // (group, new item index) of each pair
  // level 0 puts every list through one Union (Union(nil, c) drops 0xFFFFFFFF,
  // as the reference's first step does); later levels pair the survivors
  for (bool first = true;; first = false) {
    ab.clear(), al.clear(), bb.clear(), bl.clear(), ob.clear(), who.clear();
    uint64_t pos = 0;
    std::vector<std::vector<Item>> next(ngroups);
    for (size_t gi = 0; gi < ngroups; gi++) {
      const auto& it = items[gi];
      if (it.empty() || (!first && it.size() == 1)) {
        if (!it.empty()) {  // carried over: copied to the other buffer below
          ab.push_back(it[0].beg), al.push_back(it[0].len), bb.push_back(0), bl.push_back(0), ob.push_back(pos);
          who.push_back({gi, next[gi].size()});
          next[gi].push_back({pos, 0});
          pos += it[0].len;
        }
        continue;
      }
      for (size_t i = 0; i < it.size(); i += 2) {
        const Item a = it[i], b = i + 1 < it.size() ? it[i + 1] : Item{0, 0};
        ab.push_back(a.beg), al.push_back(a.len), bb.push_back(b.beg), bl.push_back(b.len), ob.push_back(pos);
        who.push_back({gi, next[gi].size()});
        next[gi].push_back({pos, 0});
        pos += a.len + b.len;
      }
    }
    bool more = false;
    for (size_t gi = 0; gi < ngroups; gi++) more |= items[gi].size() > 1;
    if (!first && !more) break;  // every group is down to its fold
    ol.assign(ab.size(), 0);
    if (!ab.empty()) {
      ScopedTimer tm(ctx, "union_fold");
      rc = merge_dev(ctx, SG_OP_UNION, buf[cur], buf[cur], buf[1 - cur], ab.data(), al.data(), bb.data(), bl.data(),
                     ob.data(), ab.size(), ol.data());
      if (rc) return rc;
    }
    for (size_t p = 0; p < who.size(); p++) next[who[p].first][who[p].second].len = ol[p];
    items.swap(next);
    cur = 1 - cur;
  }
  // pack the folds: group g at out_off[g]
  std::vector<uint64_t> beg(ngroups, 0), len(ngroups, 0);
  for (size_t gi = 0; gi < ngroups; gi++) {
    if (!items[gi].empty()) beg[gi] = items[gi][0].beg, len[gi] = items[gi][0].len;
    out_off[gi + 1] = out_off[gi] + len[gi];
  }
  if (out_off[ngroups] > cap) {
    set_error("sg_union_fold: %llu values, capacity %zu", (unsigned long long)out_off[ngroups], cap);
    return SG_EINVAL;
  }
  if (out_off[ngroups] == 0) return SG_OK;
  if (!out_vals) return SG_EINVAL;
  const size_t b_o = ((ngroups + 1) * 8 + 255) & ~size_t(255);
  uint64_t* dmeta = (uint64_t*)((char*)ctx->dstage + 2 * b_v);
  uint64_t *dbeg = dmeta, *dlen = (uint64_t*)((char*)dmeta + b_o), *doff = (uint64_t*)((char*)dmeta + 2 * b_o);
  SG_HIP(hipMemcpyAsync(dbeg, beg.data(), ngroups * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dlen, len.data(), ngroups * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(doff, out_off, ngroups * 8, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_fold_pack, dim3(div_up(ngroups, 4)), dim3(256), 0, ctx->stream, buf[cur], dbeg, dlen, doff,
                     (uint64_t)ngroups, buf[1 - cur]);
  SG_HIP(hipGetLastError());
  SG_HIP(hipMemcpyAsync(out_vals, buf[1 - cur], out_off[ngroups] * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

}  // extern "C"
