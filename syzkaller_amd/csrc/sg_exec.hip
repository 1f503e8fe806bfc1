// sg_exec.hip -- executor edge signal (trace -> per-call signal) and the
// synthetic Zipf trace generator.
//
// Reference: executor/executor.h:389-401 (the signal loop of
// handle_completion), :497-505 hash(), :507-526 dedup(); the dedup table is
// fresh per program because the executor forks a child per program
// (executor/executor_linux.cc:174-194) and shared by that program's calls.
//
// The dedup decisions are inherently sequential within a program (each
// insert can change later lookups), so one workgroup owns one program and its
// 8192-slot table lives in LDS.  k_exec_region2 decides a window of edges at
// once by slot regions (below): a deciding wave whose lanes own disjoint
// table regions, and a producer wave that hashes, sorts and compacts the
// windows around it.
#include "sg_internal.h"

#include <cmath>
#include <cstring>

namespace sg {

constexpr uint32_t kDedupSize = 8192;  // executor.h:506

using sgd::exec_hash;  // executor.h:497-505


// Slot regions (r04): lane r of the deciding wave owns the 128 table slots
// [128 r, 128 r + 127] and decides, in program order, the window's edges whose
// home slot sig % 8192 lies there.  An edge reads and writes only its probe
// slots home .. home + 3, so two edges can interact only when those ranges
// meet: edges of one region (one lane, taken in order), or an edge whose
// range runs into the next region (home % 128 >= 125, "spanning") and an edge
// of that next region with home % 128 <= 2 ("low": the only ones that reach
// slots 0..2 of their region).  A low edge waits until the lane to its left
// has decided every edge before it, a spanning edge until the lane to its
// right has; the earliest undecided edge of the window is always free, so
// every step decides at least one edge, and any two edges sharing a slot are
// decided in program order: the table ends each window exactly as the
// sequential loop leaves it, and each edge sees exactly what it would.
//
// Per window of W = 64 K edges: each edge ORs its bit into its (row, region)
// mask; the masks give every edge its place in a region-major list of
// (position, signal) (regions' bases by a wave scan of their counts, the
// rank inside a region by popcounts of the masks), so a lane then walks its
// region's entries in program order with one LDS round trip per step (the
// four probe slots and the next entry together); the decisions are bytes per
// position, read back per row for the compaction stores.  Steps per window =
// the most edges any region holds plus the waits (C2 traces, W = 256: ~10).
//
// The producer wave (r04) does everything but the steps: while wave 0 walks
// the region lists of window i, wave 1 compacts window i - 1's kept signals
// into the output and builds window i + 1 (PC loads a window ahead, hashes,
// the region masks and the region-major list) into the other of two buffers.
// One barrier per window (LDS only: the producer's PC loads stay in flight
// across it).  39 KiB of LDS: four programs per CU.  (Measured and removed in
// r05: a speculative one-wave kernel -- every edge of a window probes at
// once, the decided prefix commits -- 1.96 ms per 134M PCs against 1.51, a
// one-wave slot-region kernel 2.01 ms, 2 or 4 deciding waves 1.59 / 3.09 ms.
// Also measured in r05: the table as 22-bit slot codes -- a signal's low 13
// bits are implied by its slot and probe offset -- in a 16-bit and an 8-bit
// array, 24 KiB, five programs per CU: steady flags + queued lists 14.3 ->
// 18.3 ms, executor-exact C2 from traces 19.9 -> 27.3 ms; each deciding step
// then reads eight LDS values instead of four, on the critical chain.)
constexpr uint32_t kNoPos = 0xFFFFFFFFu;


__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// kDbg (option debug_part): per program, as its waves see them, dbg[8 p + j]:
// 0 deciding-wave cycles in its steps, 1 its cycles at the window barrier,
// 2 steps, 3 windows, 4 producer cycles compacting, 5 building, 6 at the
// barrier, 7 the block's cycles in the window loop
template <int K, bool kDbg>
__global__ __launch_bounds__(128) void k_exec_region2(const uint32_t* __restrict__ pcs,
                                                      const uint64_t* __restrict__ call_off,
                                                      const uint64_t* __restrict__ prog_off, uint32_t* __restrict__ tmp,
                                                      uint32_t* __restrict__ cnt, const uint64_t* __restrict__ pstop,
                                                      const uint8_t* __restrict__ emit,
                                                      unsigned long long* __restrict__ dbg) {
  constexpr int W = 64 * K;
  __shared__ uint32_t table[kDedupSize + 8];        // + mirror of slots 0..2, dummy slot 8196
  __shared__ unsigned long long wlist[2][W];        // position << 32 | signal, region-major
  __shared__ uint32_t wbc[2][64];                   // region lane: base << 16 | count
  __shared__ uint32_t wlive[2];                     // buffer holds a window to decide
  __shared__ unsigned long long wmask[K][64];       // producer scratch
  __shared__ uint8_t wres[2][W + 4];                // decision of position 64 k + l at l K + k; W: dummy
  const int tid = threadIdx.x, lane = tid & 63;
  const bool prod = tid >= 64;
  const uint64_t p = blockIdx.x;
  const uint64_t c0 = prog_off[p], c1 = pstop ? pstop[p] : prog_off[p + 1];
  if (c1 <= c0) return;
  for (uint32_t i = tid; i < kDedupSize + 8; i += 128) table[i] = 0;
  if (prod) {
#pragma unroll
    for (int k = 0; k < K; k++) wmask[k][lane] = 0;
  }
  __syncthreads();
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  // producer state: the window to build (call bc, start bj), the carried hash;
  // the call's bounds and emit flag, and the next call's, loaded a call ahead
  // (a global load waited for inside the loop would also wait for the PC
  // loads in flight)
  uint64_t bc = c0, bj = call_off[c0];
  // (loads a call ahead are unconditional and clamped, and tested only when
  // used: a select on a value just loaded would wait for it there)
  uint64_t cb_b = bj, cb_e = call_off[c0 + 1], nx_e = call_off[c0 + 2 < c1 ? c0 + 2 : c1];
  bool cb_em = !emit || emit[c0] != 0;
  uint32_t nx_em = 1;
  if (emit) nx_em = emit[c0 + 1 < c1 ? c0 + 1 : c1 - 1];
  uint32_t carry = 0;
  const uint64_t pend = call_off[c1];
  uint32_t npc[K];  // the PCs of the window to build
  // pending windows: d = being decided, q = decided, to compact; per window its
  // call, the call's first position, emit flag, first / last window of the call
  uint32_t sd[K], sq[K];
  int nd = 0, nq = 0;                 // valid positions (0: no window)
  uint64_t cd = 0, cq = 0, bd = 0, bq = 0;
  bool ld = false, lq = false, fd = false, fq = false, ed = false, eq = false;
  uint64_t outpos = 0;
  if (prod) {
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint64_t q = bj + 64 * k + lane;
      npc[k] = q < pend ? pcs[q] : 0u;
    }
  }
  // the producer: build the next window into buffer nb (kNoPos-free: wlive[nb] = 0 when none)
  auto build = [&](uint32_t nb, uint32_t (&sb)[K], int& nv, uint64_t& cb, uint64_t& bb, bool& lb, bool& fb,
                   bool& eb) {
    // past the call's end: the next call (an empty one's count stays 0, from the memset)
    while (bc < c1 && bj >= cb_e) {
      bc++;
      if (bc >= c1) break;
      cb_b = cb_e;
      cb_e = nx_e;
      cb_em = nx_em != 0;
      nx_e = call_off[bc + 2 < c1 ? bc + 2 : c1];
      if (emit) nx_em = emit[bc + 1 < c1 ? bc + 1 : c1 - 1];
    }
    if (bc >= c1) {
      nv = 0;
      if (lane == 0) wlive[nb] = 0;
      return;
    }
    const uint64_t e = cb_e;
    fb = bj == cb_b;
    if (fb) carry = 0;  // prev = 0 at call start (executor.h:389)
    nv = (int)((e - bj) < (uint64_t)W ? (e - bj) : (uint64_t)W);
    cb = bc;
    bb = cb_b;
    eb = cb_em;
    lb = bj + (uint64_t)nv >= e;
    uint32_t pc[K];
#pragma unroll
    for (int k = 0; k < K; k++) pc[k] = 64 * k + lane < nv ? npc[k] : 0u;
    const uint64_t nj = bj + (uint64_t)nv;  // the next window's first position (this call's next, or the next call's)
#pragma unroll
    for (int k = 0; k < K; k++) {  // (past the program: a clamped load; the next build zeroes past its window)
      const uint64_t q = nj + 64 * k + lane;
      npc[k] = pcs[q < pend ? q : pend - 1];
    }
    uint32_t h[K];
#pragma unroll
    for (int k = 0; k < K; k++) h[k] = exec_hash(pc[k]);
    uint32_t in = carry;
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t hp = (uint32_t)__builtin_amdgcn_update_dpp((int)in, (int)h[k], 0x138 /* wave_shr:1 */, 0xF, 0xF,
                                                                false);
      sb[k] = pc[k] ^ hp;  // executor.h:393-395
      in = __builtin_amdgcn_readlane(h[k], 63);
    }
    {
      const int lastk = (nv - 1) >> 6, lastl = (nv - 1) & 63;
      uint32_t cv = 0;
#pragma unroll
      for (int k = 0; k < K; k++)
        if (k == lastk) cv = __builtin_amdgcn_readlane(h[k], lastl);
      carry = cv;
    }
    bj = nj;
    uint32_t rg[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      rg[k] = (sb[k] >> 7) & 63u;
      if (64 * k + lane < nv)
        __hip_atomic_fetch_or(&wmask[k][rg[k]], 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __builtin_amdgcn_wave_barrier();
    uint64_t em_[K], om[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      em_[k] = __hip_atomic_load(&wmask[k][rg[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      om[k] = __hip_atomic_load(&wmask[k][lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < K; k++)
      __hip_atomic_store(&wmask[k][lane], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    uint32_t n_r = 0, rowb[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      rowb[k] = n_r;
      n_r += (uint32_t)__popcll(om[k]);
    }
    const uint32_t base = sgd::wave_incl_add(n_r) - n_r;
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t at = (uint32_t)__shfl((int)(base + rowb[k]), (int)rg[k]);
      if (64 * k + lane < nv)
        wlist[nb][at + (uint32_t)__popcll(em_[k] & lt)] = ((unsigned long long)(64u * k + lane) << 32) | sb[k];
    }
    wbc[nb][lane] = (base << 16) | n_r;
    if (lane == 0) wlive[nb] = 1;
  };
  // the producer: the decided window's kept signals into the output
  auto compact = [&](uint32_t qb) {
    if (fq) outpos = bq;
    uint64_t keep[K];
    {
      uint8_t rb[K];
#pragma unroll
      for (int k = 0; k < K; k++) rb[k] = wres[qb][lane * K + k];
#pragma unroll
      for (int k = 0; k < K; k++) keep[k] = __ballot(64 * k + lane < nq && rb[k] != 0);
    }
    if (eq) {
#pragma unroll
      for (int k = 0; k < K; k++) {
        if ((keep[k] >> lane) & 1ull) tmp[outpos + __popcll(keep[k] & lt)] = sq[k];
        outpos += __popcll(keep[k]);
      }
    }
    if (lq && lane == 0) cnt[cq] = (uint32_t)(outpos - bq);
  };
  unsigned long long dc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_loop = kDbg ? clock64() : 0, tk = t_loop;
  if (prod) build(0, sd, nd, cd, bd, ld, fd, ed);
  lds_sync();
  for (uint32_t it = 0;; it++) {
    const uint32_t buf = it & 1;
    const bool live = __hip_atomic_load(&wlive[buf], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
    if (kDbg) tk = clock64();
    if (!prod) {
      if (kDbg && live) dc[3]++;
      if (live) {
        const uint32_t bcw = wbc[buf][lane];
        const uint32_t base = bcw >> 16, iend = base + (bcw & 0xFFFFu);
        uint32_t i = base;
        // the lane's next two edges: a second one is decided in the same step
        // when it is interior (home % 128 in 3..124: its probe slots belong to
        // this lane alone, and no neighbour waits on it) and its probe range
        // is disjoint from the first's, so neither reads what the other writes.
        // (r05: 62 % of the steps on Zipf traces, but 140 instructions per step
        // against 76: a0 1.53 -> 1.49 ms, steady queued lists 1.99 -> 1.97x.)
        unsigned long long cur = wlist[buf][i < iend ? i : 0], cu2 = wlist[buf][i + 1 < iend ? i + 1 : 0];
        uint32_t pos = i < iend ? (uint32_t)(cur >> 32) : kNoPos, pos2 = i + 1 < iend ? (uint32_t)(cu2 >> 32) : kNoPos;
        uint32_t s = (uint32_t)cur, s2 = (uint32_t)cu2;
        while (__ballot(pos != kNoPos)) {
          if (kDbg) dc[2]++;
          const uint32_t left = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pos, 0x13C /* wave_ror:1 */, 0xF, 0xF, false);
          const uint32_t right = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pos, 0x134 /* wave_rol:1 */, 0xF, 0xF, false);
          const uint32_t hr = s & 127u, hr2 = s2 & 127u;
          const bool go = (pos != kNoPos) & ((hr > 2u) | (left > pos)) & ((hr < 125u) | (right > pos));
          const uint32_t home = s & (kDedupSize - 1), home2 = s2 & (kDedupSize - 1);
          const uint32_t dh = (home2 - home) & (kDedupSize - 1);  // (ring distance: ranges of 4 slots)
          const bool two = go & (pos2 != kNoPos) & (hr2 > 2u) & (hr2 < 125u) & (dh >= 4u) & (dh <= kDedupSize - 4u);
          const uint32_t i2 = i + (go ? 1u : 0u) + (two ? 1u : 0u);
          const uint32_t t0 = table[home], t1 = table[home + 1], t2 = table[home + 2], t3 = table[home + 3];
          const uint32_t u0 = table[home2], u1 = table[home2 + 1], u2 = table[home2 + 2], u3 = table[home2 + 3];
          const unsigned long long nx = wlist[buf][i2 < iend ? i2 : 0], nx2 = wlist[buf][i2 + 1 < iend ? i2 + 1 : 0];
          const bool h0 = (t0 == s) | (t0 == 0u), h1 = (t1 == s) | (t1 == 0u), h2 = (t2 == s) | (t2 == 0u);
          const bool h3 = (t3 == s) | (t3 == 0u);
          const uint32_t q = h0 ? 0u : h1 ? 1u : h2 ? 2u : h3 ? 3u : 0u;
          const uint32_t tq = h0 ? t0 : h1 ? t1 : h2 ? t2 : t3;
          const bool dup = (tq == s) & (h0 | h1 | h2 | h3);
          const bool wr = go & !dup;
          const uint32_t dd = (home + q) & (kDedupSize - 1);
          const bool g0 = (u0 == s2) | (u0 == 0u), g1 = (u1 == s2) | (u1 == 0u), g2 = (u2 == s2) | (u2 == 0u);
          const bool g3 = (u3 == s2) | (u3 == 0u);
          const uint32_t q2 = g0 ? 0u : g1 ? 1u : g2 ? 2u : g3 ? 3u : 0u;
          const uint32_t uq = g0 ? u0 : g1 ? u1 : g2 ? u2 : u3;
          const bool dup2 = (uq == s2) & (g0 | g1 | g2 | g3);
          table[wr ? dd : kDedupSize + 4] = s;
          table[wr && dd < 3u ? dd + kDedupSize : kDedupSize + 4] = s;
          table[two && !dup2 ? home2 + q2 : kDedupSize + 4] = s2;  // (interior: no wrap, no mirror)
          wres[buf][go ? (pos & 63u) * K + (pos >> 6) : (uint32_t)W] = dup ? 0 : 1;
          wres[buf][two ? (pos2 & 63u) * K + (pos2 >> 6) : (uint32_t)W + 1] = dup2 ? 0 : 1;
          i = i2;
          pos = i < iend ? (uint32_t)(nx >> 32) : kNoPos;
          pos2 = i + 1 < iend ? (uint32_t)(nx2 >> 32) : kNoPos;
          s = (uint32_t)nx;
          s2 = (uint32_t)nx2;
        }
      }
      if (kDbg) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const unsigned long long t = clock64();
        dc[0] += t - tk;
        tk = t;
      }
    } else {
      if (nq) compact(buf ^ 1);  // the window decided in the last iteration
      if (kDbg) {
        const unsigned long long t = clock64();
        dc[4] += t - tk;
        tk = t;
      }
      uint32_t sb[K];
      int nb_ = 0;
      uint64_t cb = 0, bb = 0;
      bool lb = false, fb = false, eb = false;
      if (live) build(buf ^ 1, sb, nb_, cb, bb, lb, fb, eb);
      if (kDbg) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const unsigned long long t = clock64();
        dc[5] += t - tk;
        tk = t;
      }
      // shift: decided -> to compact, being decided -> decided next, built -> being decided
#pragma unroll
      for (int k = 0; k < K; k++) {
        sq[k] = sd[k];
        sd[k] = sb[k];
      }
      nq = live ? nd : 0;
      cq = cd;
      bq = bd;
      lq = ld;
      fq = fd;
      eq = ed;
      nd = nb_;
      cd = cb;
      bd = bb;
      ld = lb;
      fd = fb;
      ed = eb;
    }
    lds_sync();
    if (kDbg) {
      const unsigned long long t = clock64();
      dc[prod ? 6 : 1] += t - tk;
    }
    if (!live) break;
  }
  // (the last decided window: compacted in the iteration that found no window to decide)
  if (kDbg) {
    dc[7] = clock64() - t_loop;
    if (!prod && lane == 0)
      for (int j : {0, 1, 2, 3, 7}) dbg[8 * p + j] = dc[j];
    if (prod && lane == 0)
      for (int j : {4, 5, 6}) dbg[8 * p + j] = dc[j];
  }
}

// the calls each program has to run for its queued calls' lists: up to and
// including its last queued call (fuzzer.go:678-683 copies the signal of
// queued records only); pstop[p] = prog_off[p] when it has none
__global__ void k_prog_stop(const uint64_t* __restrict__ prog_off, const uint8_t* __restrict__ rec_new, uint64_t nprog,
                            uint64_t* __restrict__ pstop) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nprog) return;
  const uint64_t c0 = prog_off[p];
  uint64_t stop = c0;
  for (uint64_t c = prog_off[p + 1]; c > c0; c--)
    if (rec_new[c - 1]) {
      stop = c;
      break;
    }
  pstop[p] = stop;
}

// dense CSR from the per-call capacity layout: one wave per call
__global__ __launch_bounds__(256) void k_exec_compact(const uint32_t* __restrict__ tmp,
                                                      const uint64_t* __restrict__ call_off,
                                                      const uint64_t* __restrict__ sig_off, uint64_t ncalls,
                                                      uint32_t* __restrict__ out) {
  uint64_t c = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= ncalls) return;
  const int lane = threadIdx.x & 63;
  uint64_t src = call_off[c], dst = sig_off[c], n = sig_off[c + 1] - sig_off[c];
  // four loads per lane in flight before their stores
  for (uint64_t i0 = 0; i0 < n; i0 += 256) {
    uint32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint64_t i = i0 + u * 64 + lane;
      v[u] = i < n ? __builtin_nontemporal_load(tmp + src + i) : 0u;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint64_t i = i0 + u * 64 + lane;
      if (i < n) out[dst + i] = v[u];
    }
  }
}

// ---- Zipf generator ----------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_gen_traces(uint64_t seed, uint32_t nranks, uint64_t g0, uint64_t n, const uint32_t* __restrict__ prob,
                             const uint32_t* __restrict__ alias, const uint32_t* __restrict__ perm,
                             uint32_t* __restrict__ out) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t h = mix64(seed + 0x9E3779B97F4A7C15ull * (g0 + i + 1));
    uint32_t bucket = (uint32_t)(((h >> 32) * (uint64_t)nranks) >> 32);
    uint32_t frac = (uint32_t)h;
    uint32_t rank = frac < prob[bucket] ? bucket : alias[bucket];
    out[i] = 0x81000000u + 16u * perm[rank];
  }
}

// Programs drawn from a fixed population, re-executed with flaky coverage:
// program p of the batch is population member m = pick(trace_seed, p) <
// npop, whose trace is exactly the one k_gen_traces gives program m under
// pop_seed; each PC is independently replaced by a fresh Zipf draw with
// probability noise / 2^32 (interrupts, timing-dependent paths).
__global__ void k_gen_pop_traces(uint64_t pop_seed, uint64_t trace_seed, uint32_t nranks, uint64_t npop, uint32_t noise,
                                 uint64_t prog_base, uint64_t nprog, uint64_t per_prog,
                                 const uint32_t* __restrict__ prob, const uint32_t* __restrict__ alias,
                                 const uint32_t* __restrict__ perm, uint32_t* __restrict__ out) {
  const uint64_t n = nprog * per_prog;
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t p = prog_base + i / per_prog, j = i % per_prog;
    const uint64_t m = ((mix64(trace_seed ^ 0xA0761D6478BD642Full) + p) * 0x9E3779B97F4A7C15ull) >> 32;
    const uint64_t member = (mix64(m) >> 32) * npop >> 32;
    uint64_t h = mix64(pop_seed + 0x9E3779B97F4A7C15ull * (member * per_prog + j + 1));
    const uint64_t hn = mix64(trace_seed + 0x9E3779B97F4A7C15ull * (p * per_prog + j + 1));
    if ((uint32_t)hn < noise) h = mix64(hn ^ 0xD1B54A32D192ED03ull);
    uint32_t bucket = (uint32_t)(((h >> 32) * (uint64_t)nranks) >> 32);
    uint32_t frac = (uint32_t)h;
    uint32_t rank = frac < prob[bucket] ? bucket : alias[bucket];
    out[i] = 0x81000000u + 16u * perm[rank];
  }
}

// Vose alias tables for Zipf(s) over ranks 1..N (rank r has weight r^-s) and a
// seeded Fisher-Yates permutation rank -> pc slot.  Host-side, deterministic.
static void build_zipf_tables(uint64_t seed, double s, uint32_t N, std::vector<uint32_t>& prob,
                              std::vector<uint32_t>& alias, std::vector<uint32_t>& perm) {
  std::vector<double> q(N);
  double sum = 0;
  for (uint32_t k = 0; k < N; k++) {
    q[k] = std::pow((double)(k + 1), -s);
    sum += q[k];
  }
  for (uint32_t k = 0; k < N; k++) q[k] = q[k] * N / sum;
  prob.assign(N, 0);
  alias.assign(N, 0);
  std::vector<uint32_t> small, large;
  for (uint32_t k = 0; k < N; k++) (q[k] < 1.0 ? small : large).push_back(k);
  while (!small.empty() && !large.empty()) {
    uint32_t l = small.back();
    small.pop_back();
    uint32_t g = large.back();
    large.pop_back();
    double t = q[l] * 4294967296.0;
    prob[l] = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
    alias[l] = g;
    q[g] = (q[g] + q[l]) - 1.0;
    (q[g] < 1.0 ? small : large).push_back(g);
  }
  for (uint32_t k : large) {
    prob[k] = 0xFFFFFFFFu;
    alias[k] = k;
  }
  for (uint32_t k : small) {
    prob[k] = 0xFFFFFFFFu;
    alias[k] = k;
  }
  perm.resize(N);
  for (uint32_t k = 0; k < N; k++) perm[k] = k;
  uint64_t st = seed ^ 0x5EEDC0DEull;
  for (uint32_t k = N - 1; k > 0; k--) {
    st += 0x9E3779B97F4A7C15ull;
    uint64_t r = mix64(st);
    uint32_t j = (uint32_t)(((r >> 32) * (uint64_t)(k + 1)) >> 32);
    uint32_t t = perm[k];
    perm[k] = perm[j];
    perm[j] = t;
  }
}

}  // namespace sg

using namespace sg;

extern "C" {

static int exec_signal(sg_ctx* ctx, const uint32_t* d_pcs, const uint64_t* d_call_off, const uint64_t* d_prog_off,
                       uint64_t nprog, uint64_t ncalls, uint64_t npcs, const uint8_t* d_rec_new, uint32_t* d_sig_vals,
                       uint64_t* d_sig_off) {
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  if (ncalls == 0) {
    SG_HIP(hipMemsetAsync(d_sig_off, 0, 8, ctx->stream));
    return SG_OK;
  }
  WsPlan p;
  size_t o_tmp = p.add(npcs * 4), o_cnt = p.add(ncalls * 4), o_stop = p.add(d_rec_new ? nprog * 8 : 0);
  size_t scan_off = p.total;
  rc = ws_reserve(ctx, p.total + scan_ws_bytes(ncalls));
  if (rc) return rc;
  uint32_t* tmp = (uint32_t*)ws_at(ctx, o_tmp);
  uint32_t* cnt = (uint32_t*)ws_at(ctx, o_cnt);
  uint64_t* pstop = d_rec_new ? (uint64_t*)ws_at(ctx, o_stop) : nullptr;
  SG_HIP(hipMemsetAsync(cnt, 0, ncalls * 4, ctx->stream));
  if (pstop && nprog)
    hipLaunchKernelGGL(k_prog_stop, dim3(div_up(nprog, 256)), dim3(256), 0, ctx->stream, d_prog_off, d_rec_new, nprog,
                       pstop);
  unsigned long long* ddbg = nullptr;
  if (ctx->debug_part && nprog) {  // diagnostics: the per-program cycle breakdown (stderr)
    SG_HIP(hipMalloc(&ddbg, nprog * 64));
    SG_HIP(hipMemsetAsync(ddbg, 0, nprog * 64, ctx->stream));
  }
  if (nprog) {
    ScopedTimer tm(ctx, "exec_signal");
    if (ddbg)
      hipLaunchKernelGGL((k_exec_region2<4, true>), dim3((uint32_t)nprog), dim3(128), 0, ctx->stream, d_pcs,
                         d_call_off, d_prog_off, tmp, cnt, (const uint64_t*)pstop, d_rec_new, ddbg);
    else
      hipLaunchKernelGGL((k_exec_region2<4, false>), dim3((uint32_t)nprog), dim3(128), 0, ctx->stream, d_pcs,
                         d_call_off, d_prog_off, tmp, cnt, (const uint64_t*)pstop, d_rec_new, nullptr);
  }
  if (ddbg) {
    std::vector<unsigned long long> h(nprog * 8);
    SG_HIP(hipMemcpyAsync(h.data(), ddbg, nprog * 64, hipMemcpyDeviceToHost, ctx->stream));
    SG_HIP(hipStreamSynchronize(ctx->stream));
    hipFree(ddbg);
    double t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t nrun = 0;
    for (uint64_t q = 0; q < nprog; q++) {
      if (!h[8 * q + 3]) continue;
      nrun++;
      for (int j = 0; j < 8; j++) t[j] += (double)h[8 * q + j];
    }
    const double W = t[3] ? t[3] : 1;
    fprintf(stderr,
            "[exec dbg] programs run %llu of %llu, windows %.0f (%.1f per program), steps %.2f per window; cycles "
            "per window: decide %.0f (%.1f per step), decider at barrier %.0f, producer compact %.0f, build %.0f, "
            "producer at barrier %.0f; block loop %.0f per window\n",
            (unsigned long long)nrun, (unsigned long long)nprog, t[3], t[3] / (nrun ? nrun : 1), t[2] / W, t[0] / W,
            t[2] ? t[0] / t[2] : 0.0, t[1] / W, t[4] / W, t[5] / W, t[6] / W, t[7] / W);
  }
  SG_HIP(hipGetLastError());
  rc = scan_counts(ctx, cnt, d_sig_off, ncalls, scan_off);
  if (rc) return rc;
  {
    ScopedTimer tm(ctx, "exec_compact");
    hipLaunchKernelGGL(k_exec_compact, dim3(div_up(ncalls, 4)), dim3(256), 0, ctx->stream, tmp, d_call_off, d_sig_off,
                       ncalls, d_sig_vals);
  }
  SG_HIP(hipGetLastError());
  return SG_OK;
}

int sg_exec_signal_dev(sg_ctx* ctx, const uint32_t* d_pcs, const uint64_t* d_call_off, const uint64_t* d_prog_off,
                       uint64_t nprog, uint64_t ncalls, uint64_t npcs, uint32_t* d_sig_vals, uint64_t* d_sig_off) {
  if (!ctx || !d_call_off || !d_prog_off || !d_sig_off || (npcs && (!d_pcs || !d_sig_vals))) return SG_EINVAL;
  return exec_signal(ctx, d_pcs, d_call_off, d_prog_off, nprog, ncalls, npcs, nullptr, d_sig_vals, d_sig_off);
}

int sg_exec_signal_queued_dev(sg_ctx* ctx, const uint32_t* d_pcs, const uint64_t* d_call_off,
                              const uint64_t* d_prog_off, uint64_t nprog, uint64_t ncalls, uint64_t npcs,
                              const uint8_t* d_rec_new, uint32_t* d_sig_vals, uint64_t* d_sig_off) {
  if (!ctx || !d_call_off || !d_prog_off || !d_sig_off || (npcs && (!d_pcs || !d_sig_vals)) ||
      (ncalls && !d_rec_new)) {
    set_error("sg_exec_signal_queued_dev: invalid argument");
    return SG_EINVAL;
  }
  return exec_signal(ctx, d_pcs, d_call_off, d_prog_off, nprog, ncalls, npcs, d_rec_new, d_sig_vals, d_sig_off);
}

int sg_exec_signal(sg_ctx* ctx, const uint32_t* pcs, const uint64_t* call_off, const uint64_t* prog_off,
                   size_t nprog, uint32_t* sig_vals, uint64_t* sig_off) {
  if (!ctx || !call_off || !prog_off || !sig_off) return SG_EINVAL;
  uint64_t ncalls = prog_off[nprog];
  uint64_t npcs = call_off[ncalls];
  if (prog_off[0] != 0 || call_off[0] != 0 || (npcs && (!pcs || !sig_vals))) return SG_EINVAL;
  char* st = nullptr;
  size_t b0 = (npcs * 4 + 255) & ~size_t(255), b1 = ((ncalls + 1) * 8 + 255) & ~size_t(255),
         b2 = ((nprog + 1) * 8 + 255) & ~size_t(255);
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    int rc = ensure_device(ctx);
    if (rc) return rc;
    rc = dstage_reserve(ctx, 2 * b0 + 2 * b1 + b2 + 256);
    if (rc) return rc;
    st = (char*)ctx->dstage;
  }
  uint32_t* dp = (uint32_t*)st;
  uint32_t* dsv = (uint32_t*)(st + b0);
  uint64_t* dco = (uint64_t*)(st + 2 * b0);
  uint64_t* dso = (uint64_t*)(st + 2 * b0 + b1);
  uint64_t* dpo = (uint64_t*)(st + 2 * b0 + 2 * b1);
  if (npcs) SG_HIP(hipMemcpyAsync(dp, pcs, npcs * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dco, call_off, (ncalls + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dpo, prog_off, (nprog + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  int rc = sg_exec_signal_dev(ctx, dp, dco, dpo, nprog, ncalls, npcs, dsv, dso);
  if (rc) return rc;
  SG_HIP(hipMemcpyAsync(sig_off, dso, (ncalls + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (sig_off[ncalls]) SG_HIP(hipMemcpyAsync(sig_vals, dsv, sig_off[ncalls] * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

// The fuzzer's whole step from host traces: the set-exact triage (flags,
// maxSignal / newSignal) and the executor-exact signal lists of the queued
// calls only (the Input.Signal copies, fuzzer.go:678-683), one staging of the
// traces for both.
int sg_triage_traces_queued(sg_ctx* ctx, sg_set* maxsig, sg_set* newsig, const uint32_t* pcs,
                            const uint64_t* call_off, const uint64_t* prog_off, size_t nprog, uint8_t* rec_new,
                            uint32_t* sig_vals, uint64_t* sig_off) {
  if (!ctx || !maxsig || !call_off || !prog_off || !sig_off) {
    set_error("sg_triage_traces_queued: invalid argument");
    return SG_EINVAL;
  }
  const uint64_t ncalls = prog_off[nprog];
  const uint64_t npcs = call_off[ncalls];
  if (prog_off[0] != 0 || call_off[0] != 0 || (npcs && (!pcs || !sig_vals)) || (ncalls && !rec_new)) {
    set_error("sg_triage_traces_queued: invalid argument (offsets must start at 0; null buffers)");
    return SG_EINVAL;
  }
  char* st = nullptr;
  const size_t b0 = (npcs * 4 + 255) & ~size_t(255), b1 = ((ncalls + 1) * 8 + 255) & ~size_t(255),
               b2 = ((nprog + 1) * 8 + 255) & ~size_t(255), b3 = (ncalls + 255) & ~size_t(255);
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    int rc = ensure_device(ctx);
    if (rc) return rc;
    rc = dstage_reserve(ctx, 2 * b0 + 2 * b1 + b2 + b3 + 256);
    if (rc) return rc;
    st = (char*)ctx->dstage;
  }
  uint32_t* dp = (uint32_t*)st;
  uint32_t* dsv = (uint32_t*)(st + b0);
  uint64_t* dco = (uint64_t*)(st + 2 * b0);
  uint64_t* dso = (uint64_t*)(st + 2 * b0 + b1);
  uint64_t* dpo = (uint64_t*)(st + 2 * b0 + 2 * b1);
  uint8_t* drn = (uint8_t*)(st + 2 * b0 + 2 * b1 + b2);
  if (npcs) SG_HIP(hipMemcpyAsync(dp, pcs, npcs * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dco, call_off, (ncalls + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dpo, prog_off, (nprog + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  int rc = sg_triage_traces_dev(ctx, maxsig, newsig, dp, dco, npcs, ncalls, drn);
  if (rc) return rc;
  rc = sg_exec_signal_queued_dev(ctx, dp, dco, dpo, nprog, ncalls, npcs, drn, dsv, dso);
  if (rc) return rc;
  if (ncalls) SG_HIP(hipMemcpyAsync(rec_new, drn, ncalls, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipMemcpyAsync(sig_off, dso, (ncalls + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (sig_off[ncalls]) SG_HIP(hipMemcpyAsync(sig_vals, dsv, sig_off[ncalls] * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

}  // extern "C"

namespace sg {
// Alias tables and permutation of the Zipf generator, cached per context.
static int gen_tables(sg_ctx* ctx, uint64_t seed, double zipf_s, uint32_t nranks) {
  if (ctx->gen_prob && ctx->gen_seed == seed && ctx->gen_s == zipf_s && ctx->gen_nranks == nranks) return SG_OK;
  std::vector<uint32_t> prob, alias, perm;
  build_zipf_tables(seed, zipf_s, nranks, prob, alias, perm);
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (ctx->gen_prob) {
    hipFree(ctx->gen_prob);
    hipFree(ctx->gen_alias);
    hipFree(ctx->gen_perm);
    ctx->gen_prob = ctx->gen_alias = ctx->gen_perm = nullptr;
  }
  SG_HIP(hipMalloc(&ctx->gen_prob, nranks * 4));
  SG_HIP(hipMalloc(&ctx->gen_alias, nranks * 4));
  SG_HIP(hipMalloc(&ctx->gen_perm, nranks * 4));
  SG_HIP(hipMemcpy(ctx->gen_prob, prob.data(), nranks * 4, hipMemcpyHostToDevice));
  SG_HIP(hipMemcpy(ctx->gen_alias, alias.data(), nranks * 4, hipMemcpyHostToDevice));
  SG_HIP(hipMemcpy(ctx->gen_perm, perm.data(), nranks * 4, hipMemcpyHostToDevice));
  ctx->gen_seed = seed;
  ctx->gen_s = zipf_s;
  ctx->gen_nranks = nranks;
  return SG_OK;
}
}  // namespace sg

extern "C" {

int sg_gen_zipf_traces_dev(sg_ctx* ctx, uint64_t seed, uint64_t trace_seed, double zipf_s, uint32_t nranks,
                           uint64_t prog_base, uint64_t nprog, uint32_t calls, uint32_t pcs_per_call, uint32_t* d_pcs) {
  if (!ctx || !d_pcs || nranks == 0 || nranks > (1u << 24) || !(zipf_s > 0)) return SG_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  rc = gen_tables(ctx, seed, zipf_s, nranks);
  if (rc) return rc;
  uint64_t per_prog = (uint64_t)calls * pcs_per_call;
  uint64_t n = nprog * per_prog;
  if (n == 0) return SG_OK;
  hipLaunchKernelGGL(k_gen_traces, dim3(std::min<uint64_t>(div_up(n, 256), 65536)), dim3(256), 0, ctx->stream, trace_seed,
                     nranks, prog_base * per_prog, n, ctx->gen_prob, ctx->gen_alias, ctx->gen_perm, d_pcs);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

int sg_gen_population_traces_dev(sg_ctx* ctx, uint64_t universe_seed, uint64_t pop_seed, uint64_t npop,
                                 uint64_t trace_seed, double noise, double zipf_s, uint32_t nranks, uint64_t prog_base,
                                 uint64_t nprog, uint32_t calls, uint32_t pcs_per_call, uint32_t* d_pcs) {
  if (!ctx || !d_pcs || nranks == 0 || nranks > (1u << 24) || !(zipf_s > 0) || npop == 0 || npop > (1ull << 32) ||
      !(noise >= 0 && noise <= 1))
    return SG_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  rc = gen_tables(ctx, universe_seed, zipf_s, nranks);
  if (rc) return rc;
  const uint64_t per_prog = (uint64_t)calls * pcs_per_call;
  const uint64_t n = nprog * per_prog;
  if (n == 0) return SG_OK;
  const double q = noise * 4294967296.0;
  const uint32_t thr = q >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)q;
  hipLaunchKernelGGL(k_gen_pop_traces, dim3(std::min<uint64_t>(div_up(n, 256), 65536)), dim3(256), 0, ctx->stream,
                     pop_seed, trace_seed, nranks, npop, thr, prog_base, nprog, per_prog, ctx->gen_prob,
                     ctx->gen_alias, ctx->gen_perm, d_pcs);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

}  // extern "C"
