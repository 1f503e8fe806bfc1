// sg_exec.hip -- executor edge signal (trace -> per-call signal) and the
// synthetic Zipf trace generator.
//
// Reference: executor/executor.h:389-401 (the signal loop of
// handle_completion), :497-505 hash(), :507-526 dedup(); the dedup table is
// fresh per program because the executor forks a child per program
// (executor/executor_linux.cc:174-194) and shared by that program's calls.
//
// The dedup decisions are inherently sequential within a program (each
// insert can change later lookups), so one wave owns one program and its
// 8192-slot table lives in that wave's LDS (32 KiB).  The wave computes 64
// edges at a time in parallel (pc ^ hash(prev pc) needs only a neighbour
// shift) and decides their dedup speculatively: all of them probe the table at
// once, and the decisions are kept up to the first edge whose decision slot an
// earlier writer of the window takes (then the rest probe again); kept edges
// are written with coalesced compaction stores.
#include "sg_internal.h"

#include <cmath>
#include <cstring>

#ifndef SG_COMPACT_UNROLL
#define SG_COMPACT_UNROLL 1
#endif
#ifndef SG_EXEC_FENCE
#define SG_EXEC_FENCE 0
#endif

namespace sg {

constexpr uint32_t kDedupSize = 8192;  // executor.h:506

using sgd::exec_hash;  // executor.h:497-505

__device__ __forceinline__ unsigned long long mark_load(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The speculative pass, per edge j of the window (positions start..nvalid-1
// of up to 128 edges: lane l holds positions l and 64 + l), all deciding
// against the table as it stands:
//   decision slot d_j: the slot holding sig (dup), the first empty slot
//   (insert), or sig % 8192 (overwrite, all four taken); writers = inserts
//   and overwrites, each writing d_j.
// A write by an earlier edge i changes edge j's outcome only if it lands on
// d_j: the window slots before d_j are taken and stay taken (an insert only
// fills an empty slot, an overwrite keeps a slot taken), and the slots after
// d_j are not looked at (or, for an overwrite, stay taken).  An earlier writer
// with the same sig always writes d_j too (same window, same table).  So with
// m = the first earlier writer on d_j:
//   sig_m == sig_j  -> edge j is a duplicate (sequentially it finds sig at d_j)
//   sig_m != sig_j  -> edge j is undecided (it decides again next pass).
// Any later writer on d_j with another sig is itself undecided, so it cannot
// commit before j.  The first writer per slot comes from two small mark
// tables (bucket d & 511 and bucket d >> 4): each writer posts
// position << 45 | d << 32 | sig there with a 64-bit LDS atomicMin, so a
// bucket's mark is its first writer together with that writer's slot and
// signal.  If either of j's buckets has no writer before j, no earlier writer
// is on d_j; otherwise a bucket mark on exactly d_j is the first writer on d_j
// (every writer on d_j is in both buckets); if both marks are on other slots
// (aliasing in both tables) edge j is conservatively undecided.  The decided
// prefix commits (its writers hit distinct slots); each pass commits at least
// one edge.
constexpr uint32_t kMarkN = 512;       // per mark table: 2 x 512 x 8 B = 8 KiB; table + marks = 40 KiB, 4 programs per CU
constexpr unsigned long long kNoMark = ~0ull;

// (every lane probes: an inactive lane's result is not used, and unpredicated
// LDS reads keep the probe free of exec-mask branches)
__device__ __forceinline__ void probe(const uint32_t* table, uint32_t sig, uint32_t& d, bool& dup) {
  uint32_t t[4];
#pragma unroll
  for (int q = 0; q < 4; q++) t[q] = table[(sig + (uint32_t)q) & (kDedupSize - 1)];
  // executor.h:509-525: probe (s+q) % 8192 for q = 0..3 in order; a slot
  // equal to s means duplicate, an empty slot takes s, and when all four are
  // taken slot s % 8192 is overwritten.
  uint32_t q = 0;
  dup = false;
#pragma unroll
  for (int k = 3; k >= 0; k--)
    if (t[k] == sig || t[k] == 0u) {
      q = (uint32_t)k;
      dup = t[k] == sig;
    }
  d = (sig + q) & (kDedupSize - 1);
}

// position pos (act) against its two bucket marks: bdup / undecided
__device__ __forceinline__ void resolve(unsigned long long ma, unsigned long long mb, uint32_t pos, uint32_t d,
                                        uint32_t sig, bool act, bool& bdup, bool& dirty) {
  bdup = dirty = false;
  if (!act || (uint32_t)(ma >> 45) >= pos || (uint32_t)(mb >> 45) >= pos) return;  // no earlier writer on d
  if ((uint32_t)(ma >> 32 & 0x1FFFu) == d)
    bdup = (uint32_t)ma == sig;
  else if ((uint32_t)(mb >> 32 & 0x1FFFu) == d)
    bdup = (uint32_t)mb == sig;
  dirty = !bdup;
}

__device__ __forceinline__ unsigned long long mark_val(uint32_t pos, uint32_t d, uint32_t sig) {
  return ((unsigned long long)pos << 45) | ((unsigned long long)d << 32) | sig;
}

// kCount (diagnostics, SG_DEBUG_PART): stats[0..2] += windows, speculative
// passes, edges of the wave's program.
// pstop (nullable): the wave runs its program's calls [prog_off[p], pstop[p])
// only -- the executor's table state at a call depends on the calls before it,
// never on later ones; emit (nullable): only calls with emit[c] != 0 write
// their signal (the others still update the table; cnt[c] stays 0).
template <bool kCount>
__global__ __launch_bounds__(64) void k_exec_signal(const uint32_t* __restrict__ pcs,
                                                    const uint64_t* __restrict__ call_off,
                                                    const uint64_t* __restrict__ prog_off, uint32_t* __restrict__ tmp,
                                                    uint32_t* __restrict__ cnt, unsigned long long* stats,
                                                    const uint64_t* __restrict__ pstop = nullptr,
                                                    const uint8_t* __restrict__ emit = nullptr) {
  uint64_t n_win = 0, n_pass = 0, n_edge = 0;
  __shared__ uint32_t table[kDedupSize];
  __shared__ unsigned long long markA[kMarkN], markB[kMarkN];
  const int lane = threadIdx.x;
  const uint32_t pos0 = (uint32_t)lane, pos1 = 64u + (uint32_t)lane;
  const uint64_t p = blockIdx.x;
  const uint64_t c0 = prog_off[p], c1 = pstop ? pstop[p] : prog_off[p + 1];
  if (c1 <= c0) return;  // (one wave: the whole workgroup leaves)
  for (uint32_t i = lane; i < kDedupSize; i += 64) table[i] = 0;
  for (uint32_t i = lane; i < kMarkN; i += 64) markA[i] = markB[i] = kNoMark;
  __syncthreads();
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  // the program's calls are contiguous in the trace: the next 128 PCs are
  // always in flight (the next window of this call, or the next call's first)
  const uint64_t pend = call_off[c1];
  uint64_t w0 = call_off[c0];
  uint32_t npc0 = w0 + pos0 < pend ? pcs[w0 + pos0] : 0u, npc1 = w0 + pos1 < pend ? pcs[w0 + pos1] : 0u;
  for (uint64_t c = c0; c < c1; c++) {
    const uint64_t b = call_off[c], e = call_off[c + 1];
    const bool em = !emit || emit[c] != 0;
    uint32_t carry = 0;  // hash of the previous PC; prev = 0 at call start (executor.h:389)
    uint64_t outpos = b;
    for (uint64_t j = b; j < e; j += 128) {
      const int nvalid = (int)((e - j) < 128 ? (e - j) : 128);
      const uint32_t pc0 = pos0 < (uint32_t)nvalid ? npc0 : 0u, pc1 = pos1 < (uint32_t)nvalid ? npc1 : 0u;
      // (unpredicated loads at clamped addresses: with no branch around them the
      // wait for them lands where they are used, a window later, not here)
      const uint64_t nj = j + 128 < e ? j + 128 : e;
      const uint32_t l0 = pcs[nj + pos0 < pend ? nj + pos0 : pend - 1];
      const uint32_t l1 = pcs[nj + pos1 < pend ? nj + pos1 : pend - 1];
      npc0 = nj + pos0 < pend ? l0 : 0u;
      npc1 = nj + pos1 < pend ? l1 : 0u;
      const uint32_t h0 = exec_hash(pc0), h1 = exec_hash(pc1);
      // the previous PC's hash: the position before's (a DPP wave shift; lane 0
      // of the first half takes the carry, of the second half lane 63's)
      const uint32_t hp0 =
          (uint32_t)__builtin_amdgcn_update_dpp((int)carry, (int)h0, 0x138 /* wave_shr:1 */, 0xF, 0xF, false);
      const uint32_t hp1 = (uint32_t)__builtin_amdgcn_update_dpp((int)__builtin_amdgcn_readlane(h0, 63), (int)h1, 0x138,
                                                                 0xF, 0xF, false);
      const uint32_t sig0 = pc0 ^ hp0, sig1 = pc1 ^ hp1;  // executor.h:393-395
      carry = nvalid > 64 ? __builtin_amdgcn_readlane(h1, nvalid - 65) : __builtin_amdgcn_readlane(h0, nvalid - 1);
      uint64_t keep0 = 0, keep1 = 0;
      if (kCount) {
        n_win++;
        n_edge += (uint64_t)nvalid;
      }
      for (int start = 0; start < nvalid;) {
        if (kCount) n_pass++;
        const bool act0 = (int)pos0 >= start && (int)pos0 < nvalid, act1 = (int)pos1 >= start && (int)pos1 < nvalid;
        uint32_t d0, d1;
        bool dup0, dup1;
        probe(table, sig0, d0, dup0);
        probe(table, sig1, d1, dup1);
        const bool wr0 = act0 && !dup0, wr1 = act1 && !dup1;
        const uint64_t wm0 = __ballot(wr0), wm1 = __ballot(wr1);
        int f = nvalid;
        bool bd0 = false, bd1 = false;
        if (wm0 | wm1) {
          bool dt0, dt1;
          if (__popcll(wm0) + __popcll(wm1) == 1) {  // one writer: compare against it directly
            const uint32_t i = wm0 ? (uint32_t)(__ffsll((unsigned long long)wm0) - 1)
                                   : 64u + (uint32_t)(__ffsll((unsigned long long)wm1) - 1);
            const uint32_t di = i < 64 ? __builtin_amdgcn_readlane(d0, i) : __builtin_amdgcn_readlane(d1, i - 64);
            const uint32_t si = i < 64 ? __builtin_amdgcn_readlane(sig0, i) : __builtin_amdgcn_readlane(sig1, i - 64);
            const bool e0 = act0 && pos0 > i && d0 == di, e1 = act1 && pos1 > i && d1 == di;
            bd0 = e0 && sig0 == si;
            bd1 = e1 && sig1 == si;
            dt0 = e0 && !bd0;
            dt1 = e1 && !bd1;
          } else {
            if (wr0) {
              const unsigned long long v = mark_val(pos0, d0, sig0);
              __hip_atomic_fetch_min(&markA[d0 & (kMarkN - 1)], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              __hip_atomic_fetch_min(&markB[d0 >> 4], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (wr1) {
              const unsigned long long v = mark_val(pos1, d1, sig1);
              __hip_atomic_fetch_min(&markA[d1 & (kMarkN - 1)], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              __hip_atomic_fetch_min(&markB[d1 >> 4], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
#if SG_EXEC_FENCE
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
#endif
            // (one wave: its LDS operations complete in issue order, so the
            // reads below see every lane's atomicMin without a fence; they are
            // relaxed atomic loads, not plain reads of locations other lanes
            // update atomically, so the memory model allows no reordering)
            __builtin_amdgcn_wave_barrier();
            const unsigned long long a0 = mark_load(&markA[d0 & (kMarkN - 1)]), b0 = mark_load(&markB[d0 >> 4]);
            const unsigned long long a1 = mark_load(&markA[d1 & (kMarkN - 1)]), b1 = mark_load(&markB[d1 >> 4]);
#if SG_EXEC_FENCE
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
#endif
            __builtin_amdgcn_wave_barrier();
            if (wr0) markA[d0 & (kMarkN - 1)] = markB[d0 >> 4] = kNoMark;
            if (wr1) markA[d1 & (kMarkN - 1)] = markB[d1 >> 4] = kNoMark;
            resolve(a0, b0, pos0, d0, sig0, act0, bd0, dt0);
            resolve(a1, b1, pos1, d1, sig1, act1, bd1, dt1);
          }
          const uint64_t um0 = __ballot(dt0), um1 = __ballot(dt1);
          f = um0 ? __ffsll((unsigned long long)um0) - 1 : (um1 ? 64 + __ffsll((unsigned long long)um1) - 1 : nvalid);
          // a zero signal's overwrite empties its slot (see k_exec_signal_k)
          const uint64_t zm0 = __ballot(wr0 && sig0 == 0u), zm1 = __ballot(wr1 && sig1 == 0u);
          const int fz = zm0 ? __ffsll((unsigned long long)zm0) : (zm1 ? 64 + __ffsll((unsigned long long)zm1) : nvalid);
          f = fz < f ? fz : f;
        }
        const bool cm0 = wr0 && !bd0 && (int)pos0 < f, cm1 = wr1 && !bd1 && (int)pos1 < f;
        if (cm0) table[d0] = sig0;
        if (cm1) table[d1] = sig1;
        keep0 |= __ballot(cm0);
        keep1 |= __ballot(cm1);
        start = f;
      }
      // the next window's PCs are needed from here on: waiting for them before
      // the (exec-masked, so branched-around) stores keeps the wait off the
      // next window's critical path
      asm volatile("" ::"v"(npc0), "v"(npc1));
      if (em) {
        if ((keep0 >> lane) & 1ull) tmp[outpos + __popcll(keep0 & lt)] = sig0;
        outpos += __popcll(keep0);
        if ((keep1 >> lane) & 1ull) tmp[outpos + __popcll(keep1 & lt)] = sig1;
        outpos += __popcll(keep1);
      }
    }
    if (lane == 0) cnt[c] = (uint32_t)(outpos - b);
  }
  if (kCount && lane == 0) {
    atomicAdd(&stats[0], (unsigned long long)n_win);
    atomicAdd(&stats[1], (unsigned long long)n_pass);
    atomicAdd(&stats[2], (unsigned long long)n_edge);
  }
}

// The product kernel: k_exec_signal's speculative window with W edges held
// in K slots per lane (position 64 k + lane in slot k); the mark tables and
// the decision rules are k_exec_signal's (whose 128-edge window, K = 2, is
// kept for the pass counters of SG_DEBUG_PART).  One 64-edge window per
// wave step is fastest: a wider window decides more edges per pass but needs
// more passes (the first undecided edge ends a pass), a narrower one idles
// lanes.
template <int K, int W = 64 * K>
__global__ __launch_bounds__(64) void k_exec_signal_k(const uint32_t* __restrict__ pcs,
                                                      const uint64_t* __restrict__ call_off,
                                                      const uint64_t* __restrict__ prog_off, uint32_t* __restrict__ tmp,
                                                      uint32_t* __restrict__ cnt, const uint64_t* __restrict__ pstop,
                                                      const uint8_t* __restrict__ emit) {
  static_assert(W <= 64 * K && W > 64 * (K - 1), "W edges per window in K slots");
  __shared__ uint32_t table[kDedupSize];
  __shared__ unsigned long long markA[kMarkN], markB[kMarkN];
  const int lane = threadIdx.x;
  const uint64_t p = blockIdx.x;
  const uint64_t c0 = prog_off[p], c1 = pstop ? pstop[p] : prog_off[p + 1];
  if (c1 <= c0) return;
  for (uint32_t i = lane; i < kDedupSize; i += 64) table[i] = 0;
  for (uint32_t i = lane; i < kMarkN; i += 64) markA[i] = markB[i] = kNoMark;
  __syncthreads();
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint64_t pend = call_off[c1];
  const uint64_t w0 = call_off[c0];
  uint32_t npc[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const uint64_t q = w0 + 64 * k + lane;
    npc[k] = q < pend ? pcs[q] : 0u;
  }
  for (uint64_t c = c0; c < c1; c++) {
    const uint64_t b = call_off[c], e = call_off[c + 1];
    const bool em = !emit || emit[c] != 0;
    uint32_t carry = 0;  // hash of the previous PC; prev = 0 at call start (executor.h:389)
    uint64_t outpos = b;
    for (uint64_t j = b; j < e; j += W) {
      const int nvalid = (int)((e - j) < (uint64_t)W ? (e - j) : (uint64_t)W);
      uint32_t pc[K], sig[K];
#pragma unroll
      for (int k = 0; k < K; k++) pc[k] = 64 * k + lane < nvalid ? npc[k] : 0u;
      const uint64_t nj = j + W < e ? j + W : e;
#pragma unroll
      for (int k = 0; k < K; k++) {
        const uint64_t q = nj + 64 * k + lane;
        const uint32_t l = pcs[q < pend ? q : pend - 1];
        npc[k] = q < pend ? l : 0u;
      }
      uint32_t h[K];
#pragma unroll
      for (int k = 0; k < K; k++) h[k] = exec_hash(pc[k]);
      uint32_t in = carry;
#pragma unroll
      for (int k = 0; k < K; k++) {
        const uint32_t hp = (uint32_t)__builtin_amdgcn_update_dpp((int)in, (int)h[k], 0x138 /* wave_shr:1 */, 0xF, 0xF,
                                                                  false);
        sig[k] = pc[k] ^ hp;  // executor.h:393-395
        in = __builtin_amdgcn_readlane(h[k], 63);
      }
      {
        const int lastk = (nvalid - 1) >> 6, lastl = (nvalid - 1) & 63;
        uint32_t cv = 0;
#pragma unroll
        for (int k = 0; k < K; k++)
          if (k == lastk) cv = __builtin_amdgcn_readlane(h[k], lastl);
        carry = cv;
      }
      uint64_t keep[K];
#pragma unroll
      for (int k = 0; k < K; k++) keep[k] = 0;
      for (int start = 0; start < nvalid;) {
        bool act[K], wr[K], bd[K], dt[K];
        uint32_t d[K];
        uint64_t wm[K];
        int nw = 0;
#pragma unroll
        for (int k = 0; k < K; k++) {
          const int pos = 64 * k + lane;
          act[k] = pos >= start && pos < nvalid;
          bool dup;
          probe(table, sig[k], d[k], dup);
          wr[k] = act[k] && !dup;
          wm[k] = __ballot(wr[k]);
          nw += __popcll(wm[k]);
          bd[k] = dt[k] = false;
        }
        int f = nvalid;
        if (nw) {
          if (nw == 1) {  // one writer: compare against it directly
            uint32_t di = 0, si = 0, iw = 0;
#pragma unroll
            for (int k = 0; k < K; k++)
              if (wm[k]) {
                const uint32_t l = (uint32_t)(__ffsll((unsigned long long)wm[k]) - 1);
                di = __builtin_amdgcn_readlane(d[k], l);
                si = __builtin_amdgcn_readlane(sig[k], l);
                iw = 64u * k + l;
              }
#pragma unroll
            for (int k = 0; k < K; k++) {
              const bool ek = act[k] && (uint32_t)(64 * k + lane) > iw && d[k] == di;
              bd[k] = ek && sig[k] == si;
              dt[k] = ek && !bd[k];
            }
          } else {
#pragma unroll
            for (int k = 0; k < K; k++)
              if (wr[k]) {
                const unsigned long long v = mark_val(64u * k + lane, d[k], sig[k]);
                __hip_atomic_fetch_min(&markA[d[k] & (kMarkN - 1)], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_min(&markB[d[k] >> 4], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              }
            __builtin_amdgcn_wave_barrier();
            unsigned long long ma[K], mb[K];
#pragma unroll
            for (int k = 0; k < K; k++) {
              ma[k] = mark_load(&markA[d[k] & (kMarkN - 1)]);
              mb[k] = mark_load(&markB[d[k] >> 4]);
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = 0; k < K; k++)
              if (wr[k]) markA[d[k] & (kMarkN - 1)] = markB[d[k] >> 4] = kNoMark;
#pragma unroll
            for (int k = 0; k < K; k++) resolve(ma[k], mb[k], 64u * k + lane, d[k], sig[k], act[k], bd[k], dt[k]);
          }
#pragma unroll
          for (int k = K - 1; k >= 0; k--) {  // the first undecided position
            const uint64_t um = __ballot(dt[k]);
            if (um) f = 64 * k + __ffsll((unsigned long long)um) - 1;
          }
          // A zero signal writes only when its four slots are taken, and then
          // overwrites slot 0 with 0: it EMPTIES a slot, which can change any
          // later edge's outcome (the rules above assume slots stay taken).
          // The pass ends after the first zero writer.
          int fz = nvalid;
#pragma unroll
          for (int k = K - 1; k >= 0; k--) {
            const uint64_t zm = __ballot(wr[k] && sig[k] == 0u);
            if (zm) fz = 64 * k + __ffsll((unsigned long long)zm);
          }
          f = fz < f ? fz : f;
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
          const bool cm = wr[k] && !bd[k] && 64 * k + lane < f;
          if (cm) table[d[k]] = sig[k];
          keep[k] |= __ballot(cm);
        }
        start = f;
      }
      asm volatile("" ::"v"(npc[0]));
      if (em) {
#pragma unroll
        for (int k = 0; k < K; k++) {
          if ((keep[k] >> lane) & 1ull) tmp[outpos + __popcll(keep[k] & lt)] = sig[k];
          outpos += __popcll(keep[k]);
        }
      }
    }
    if (lane == 0) cnt[c] = (uint32_t)(outpos - b);
  }
}

// Slot regions (r04): lane r of the wave owns the 128 table slots
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
// the most edges any region holds plus the waits (C2 traces, W = 256: ~25
// edges per step, against ~28 per speculative pass of several LDS round trips
// in k_exec_signal_k).
constexpr uint32_t kNoPos = 0xFFFFFFFFu;

// stats (nullable, SG_DEBUG_PART): [0] windows, [1] steps, [2] cycles in
// the steps, [3] cycles in the whole program loop, [4] edges
template <int K>
__global__ __launch_bounds__(64) void k_exec_region(const uint32_t* __restrict__ pcs,
                                                    const uint64_t* __restrict__ call_off,
                                                    const uint64_t* __restrict__ prog_off, uint32_t* __restrict__ tmp,
                                                    uint32_t* __restrict__ cnt, const uint64_t* __restrict__ pstop,
                                                    const uint8_t* __restrict__ emit,
                                                    unsigned long long* __restrict__ stats = nullptr) {
  unsigned long long n_win = 0, n_step = 0, cy_step = 0, n_edge = 0;
  const unsigned long long cy0 = stats ? clock64() : 0;
  constexpr int W = 64 * K;
  // slots 8192..8194 mirror slots 0..2 (a probe reads 4 consecutive words);
  // 8196 is a dummy slot that predicated-off writes go to
  __shared__ uint32_t table[kDedupSize + 8];
  __shared__ unsigned long long wlist[W];  // position << 32 | signal, region-major
  __shared__ unsigned long long wmask[K][64];
  __shared__ uint8_t wres[W + 4];  // the decision of position 64 k + l at l K + k; W: dummy
  const int lane = threadIdx.x;
  const uint64_t p = blockIdx.x;
  const uint64_t c0 = prog_off[p], c1 = pstop ? pstop[p] : prog_off[p + 1];
  if (c1 <= c0) return;
  for (uint32_t i = lane; i < kDedupSize + 8; i += 64) table[i] = 0;
#pragma unroll
  for (int k = 0; k < K; k++) wmask[k][lane] = 0;
  __syncthreads();
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint64_t pend = call_off[c1];
  const uint64_t w0 = call_off[c0];
  uint32_t npc[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const uint64_t q = w0 + 64 * k + lane;
    npc[k] = q < pend ? pcs[q] : 0u;
  }
  for (uint64_t c = c0; c < c1; c++) {
    const uint64_t b = call_off[c], e = call_off[c + 1];
    const bool em = !emit || emit[c] != 0;
    uint32_t carry = 0;  // hash of the previous PC; prev = 0 at call start (executor.h:389)
    uint64_t outpos = b;
    for (uint64_t j = b; j < e; j += W) {
      const int nvalid = (int)((e - j) < (uint64_t)W ? (e - j) : (uint64_t)W);
      uint32_t pc[K], sig[K];
#pragma unroll
      for (int k = 0; k < K; k++) pc[k] = 64 * k + lane < nvalid ? npc[k] : 0u;
      const uint64_t nj = j + W < e ? j + W : e;
#pragma unroll
      for (int k = 0; k < K; k++) {
        const uint64_t q = nj + 64 * k + lane;
        const uint32_t l = pcs[q < pend ? q : pend - 1];
        npc[k] = q < pend ? l : 0u;
      }
      uint32_t h[K];
#pragma unroll
      for (int k = 0; k < K; k++) h[k] = exec_hash(pc[k]);
      uint32_t in = carry;
#pragma unroll
      for (int k = 0; k < K; k++) {
        const uint32_t hp = (uint32_t)__builtin_amdgcn_update_dpp((int)in, (int)h[k], 0x138 /* wave_shr:1 */, 0xF, 0xF,
                                                                  false);
        sig[k] = pc[k] ^ hp;  // executor.h:393-395
        in = __builtin_amdgcn_readlane(h[k], 63);
      }
      {
        const int lastk = (nvalid - 1) >> 6, lastl = (nvalid - 1) & 63;
        uint32_t cv = 0;
#pragma unroll
        for (int k = 0; k < K; k++)
          if (k == lastk) cv = __builtin_amdgcn_readlane(h[k], lastl);
        carry = cv;
      }
      uint32_t rg[K];
#pragma unroll
      for (int k = 0; k < K; k++) {
        rg[k] = (sig[k] >> 7) & 63u;
        if (64 * k + lane < nvalid)
          __hip_atomic_fetch_or(&wmask[k][rg[k]], 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      // (one wave: its LDS operations complete in issue order, so relaxed
      // atomic loads after the wave barrier see every lane's OR; no
      // __syncthreads, whose fence would also wait for the next window's PC loads)
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
      // region lane: its count, its base in the list, each row's start in it
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
        if (64 * k + lane < nvalid)
          wlist[at + (uint32_t)__popcll(em_[k] & lt)] = ((unsigned long long)(64u * k + lane) << 32) | sig[k];
      }
      __builtin_amdgcn_wave_barrier();
      const uint32_t iend = base + n_r;
      uint32_t i = base;
      unsigned long long cur = wlist[i < iend ? i : 0];
      uint32_t pos = i < iend ? (uint32_t)(cur >> 32) : kNoPos;
      uint32_t s = (uint32_t)cur;
      // branch-free steps: every lane probes and writes, a lane with nothing
      // to decide into the dummy slot / byte
      const unsigned long long cs0 = stats ? clock64() : 0;
      if (stats) {
        n_win++;
        n_edge += nvalid;
      }
      while (__ballot(pos != kNoPos)) {
        if (stats) n_step++;
        // the neighbours' next undecided positions (kNoPos: none left)
        const uint32_t left = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pos, 0x13C /* wave_ror:1 */, 0xF, 0xF, false);
        const uint32_t right = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pos, 0x134 /* wave_rol:1 */, 0xF, 0xF, false);
        const uint32_t hr = s & 127u;
        const bool go = (pos != kNoPos) & ((hr > 2u) | (left > pos)) & ((hr < 125u) | (right > pos));
        const uint32_t i2 = i + (go ? 1u : 0u);
        const uint32_t home = s & (kDedupSize - 1);
        const uint32_t t0 = table[home], t1 = table[home + 1], t2 = table[home + 2], t3 = table[home + 3];
        const unsigned long long nx = wlist[i2 < iend ? i2 : 0];
        // executor.h:509-525: the first of the four slots holding s (dup) or
        // empty (insert there); all four taken: overwrite the home slot
        const bool h0 = (t0 == s) | (t0 == 0u), h1 = (t1 == s) | (t1 == 0u), h2 = (t2 == s) | (t2 == 0u);
        const uint32_t q = h0 ? 0u : h1 ? 1u : h2 ? 2u : ((t3 == s) | (t3 == 0u)) ? 3u : 0u;
        const uint32_t tq = h0 ? t0 : h1 ? t1 : h2 ? t2 : t3;
        const bool dup = (tq == s) & (h0 | h1 | h2 | (t3 == s) | (t3 == 0u));
        const bool wr = go & !dup;
        const uint32_t d = home + q;  // < 8195; slots 8192.. are the mirror of 0..2
        const uint32_t dd = d & (kDedupSize - 1);
        table[wr ? dd : kDedupSize + 4] = s;
        table[wr && dd < 3u ? dd + kDedupSize : kDedupSize + 4] = s;
        wres[go ? (pos & 63u) * K + (pos >> 6) : (uint32_t)W] = dup ? 0 : 1;
        i = i2;
        pos = i < iend ? (uint32_t)(nx >> 32) : kNoPos;
        s = (uint32_t)nx;
      }
      if (stats) cy_step += clock64() - cs0;
      __builtin_amdgcn_wave_barrier();
      uint64_t keep[K];
      {
        uint8_t rb[K];
#pragma unroll
        for (int k = 0; k < K; k++) rb[k] = wres[lane * K + k];
#pragma unroll
        for (int k = 0; k < K; k++) keep[k] = __ballot(64 * k + lane < nvalid && rb[k] != 0);
      }
      asm volatile("" ::"v"(npc[0]));
      if (em) {
#pragma unroll
        for (int k = 0; k < K; k++) {
          if ((keep[k] >> lane) & 1ull) tmp[outpos + __popcll(keep[k] & lt)] = sig[k];
          outpos += __popcll(keep[k]);
        }
      }
    }
    if (lane == 0) cnt[c] = (uint32_t)(outpos - b);
  }
  if (stats && lane == 0) {
    atomicAdd(&stats[0], n_win);
    atomicAdd(&stats[1], n_step);
    atomicAdd(&stats[2], cy_step);
    atomicAdd(&stats[3], clock64() - cy0);
    atomicAdd(&stats[4], n_edge);
  }
}

// Slot regions with a producer wave (r04): k_exec_region's decisions, with
// everything but the steps moved to a second wave of the workgroup.  Wave 0
// only walks the region lists of window i; wave 1 meanwhile compacts window
// i - 1's kept signals into the output and builds window i + 1 (PC loads a
// window ahead, hashes, the region masks and the region-major list) into the
// other of two buffers.  One barrier per window (LDS only: the producer's PC
// loads stay in flight across it).  39 KiB of LDS: four programs per CU, as
// the one-wave kernels.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int K>
__global__ __launch_bounds__(128) void k_exec_region2(const uint32_t* __restrict__ pcs,
                                                      const uint64_t* __restrict__ call_off,
                                                      const uint64_t* __restrict__ prog_off, uint32_t* __restrict__ tmp,
                                                      uint32_t* __restrict__ cnt, const uint64_t* __restrict__ pstop,
                                                      const uint8_t* __restrict__ emit) {
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
  if (prod) build(0, sd, nd, cd, bd, ld, fd, ed);
  lds_sync();
  for (uint32_t it = 0;; it++) {
    const uint32_t buf = it & 1;
    const bool live = __hip_atomic_load(&wlive[buf], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
    if (!prod) {
      if (live) {
        const uint32_t bcw = wbc[buf][lane];
        const uint32_t base = bcw >> 16, iend = base + (bcw & 0xFFFFu);
        uint32_t i = base;
        unsigned long long cur = wlist[buf][i < iend ? i : 0];
        uint32_t pos = i < iend ? (uint32_t)(cur >> 32) : kNoPos;
        uint32_t s = (uint32_t)cur;
        while (__ballot(pos != kNoPos)) {
          const uint32_t left = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pos, 0x13C /* wave_ror:1 */, 0xF, 0xF, false);
          const uint32_t right = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pos, 0x134 /* wave_rol:1 */, 0xF, 0xF, false);
          const uint32_t hr = s & 127u;
          const bool go = (pos != kNoPos) & ((hr > 2u) | (left > pos)) & ((hr < 125u) | (right > pos));
          const uint32_t i2 = i + (go ? 1u : 0u);
          const uint32_t home = s & (kDedupSize - 1);
          const uint32_t t0 = table[home], t1 = table[home + 1], t2 = table[home + 2], t3 = table[home + 3];
          const unsigned long long nx = wlist[buf][i2 < iend ? i2 : 0];
          const bool h0 = (t0 == s) | (t0 == 0u), h1 = (t1 == s) | (t1 == 0u), h2 = (t2 == s) | (t2 == 0u);
          const bool h3 = (t3 == s) | (t3 == 0u);
          const uint32_t q = h0 ? 0u : h1 ? 1u : h2 ? 2u : h3 ? 3u : 0u;
          const uint32_t tq = h0 ? t0 : h1 ? t1 : h2 ? t2 : t3;
          const bool dup = (tq == s) & (h0 | h1 | h2 | h3);
          const bool wr = go & !dup;
          const uint32_t dd = (home + q) & (kDedupSize - 1);
          table[wr ? dd : kDedupSize + 4] = s;
          table[wr && dd < 3u ? dd + kDedupSize : kDedupSize + 4] = s;
          wres[buf][go ? (pos & 63u) * K + (pos >> 6) : (uint32_t)W] = dup ? 0 : 1;
          i = i2;
          pos = i < iend ? (uint32_t)(nx >> 32) : kNoPos;
          s = (uint32_t)nx;
        }
      }
    } else {
      if (nq) compact(buf ^ 1);  // the window decided in the last iteration
      uint32_t sb[K];
      int nb_ = 0;
      uint64_t cb = 0, bb = 0;
      bool lb = false, fb = false, eb = false;
      if (live) build(buf ^ 1, sb, nb_, cb, bb, lb, fb, eb);
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
    if (!live) break;
  }
  // (the last decided window: compacted in the iteration that found no window to decide)
}

// Slot regions over D deciding waves (r04): k_exec_region2 with 64 D regions
// of 128 / D slots, wave w's lane l deciding region 64 w + l.  More regions
// split a window's edges finer (C2 traces, 256-edge windows: 10.0 steps per
// window at 64 regions, 7.4 at 128, 5.9 at 256) and the waves step in
// parallel.  A region edge between two waves (lane 63 of wave w and lane 0
// of wave w + 1, cyclically) is checked through LDS: lanes 0 and 63 publish
// their next undecided position every step and read the neighbouring wave's.
// A value read late is smaller than the current one, so the check only
// waits longer; the producer zeroes the window's published positions before
// the window starts (nothing decided yet), and a wave publishes "none left"
// when it is done.  LDS order makes the neighbour's table writes visible
// before the position it publishes after them.  The producer places the
// edges into the region-major list in two passes (counts, then row by row in
// program order), with one row's masks at a time.
template <int K, int D>
__global__ __launch_bounds__(64 * (D + 1)) void k_exec_region3(const uint32_t* __restrict__ pcs,
                                                               const uint64_t* __restrict__ call_off,
                                                               const uint64_t* __restrict__ prog_off,
                                                               uint32_t* __restrict__ tmp, uint32_t* __restrict__ cnt,
                                                               const uint64_t* __restrict__ pstop,
                                                               const uint8_t* __restrict__ emit) {
  constexpr int W = 64 * K;
  constexpr uint32_t R = 64 * D, S = kDedupSize / R;  // regions, slots per region
  static_assert(W <= 256, "positions fit a byte");
  __shared__ uint32_t table[kDedupSize + 4];  // + mirror of slots 0..2, dummy slot 8195
  __shared__ uint32_t wsig[2][W];             // region-major
  __shared__ uint8_t wpos[2][W];
  __shared__ uint32_t wbc[2][R];              // region: base << 16 | count
  __shared__ uint32_t pubp[2][2][D];          // [buf][lane 0 / lane 63][wave]: next undecided position
  __shared__ uint32_t wlive[2];
  __shared__ unsigned long long wmask[R];     // producer scratch: one row's masks
  __shared__ uint32_t run[R];                 // producer scratch: counts, then running slots
  __shared__ uint8_t wres[2][W + 1];          // decision of position 64 k + l at l K + k; W: dummy
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const bool prod = wv == D;
  const uint64_t p = blockIdx.x;
  const uint64_t c0 = prog_off[p], c1 = pstop ? pstop[p] : prog_off[p + 1];
  if (c1 <= c0) return;
  for (uint32_t i = tid; i < kDedupSize + 4; i += 64 * (D + 1)) table[i] = 0;
  if (prod) {
    for (uint32_t r = lane; r < R; r += 64) {
      wmask[r] = 0;
      run[r] = 0;
    }
  }
  __syncthreads();
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint64_t bc = c0, bj = call_off[c0];
  uint64_t cb_b = bj, cb_e = call_off[c0 + 1], nx_e = call_off[c0 + 2 < c1 ? c0 + 2 : c1];
  bool cb_em = !emit || emit[c0] != 0;
  uint32_t nx_em = 1;
  if (emit) nx_em = emit[c0 + 1 < c1 ? c0 + 1 : c1 - 1];
  uint32_t carry = 0;
  const uint64_t pend = call_off[c1];
  uint32_t npc[K];
  uint32_t sd[K], sq[K];
  int nd = 0, nq = 0;
  uint64_t cd = 0, cq = 0, bd = 0, bq = 0;
  bool ld = false, lq = false, fd = false, fq = false, ed = false, eq = false;
  uint64_t outpos = 0;
  if (prod) {
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint64_t q = bj + 64 * k + lane;
      npc[k] = pcs[q < pend ? q : pend - 1];
    }
  }
  auto build = [&](uint32_t nb, uint32_t (&sb)[K], int& nv, uint64_t& cb, uint64_t& bb, bool& lb, bool& fb,
                   bool& eb) {
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
    const uint64_t nj = bj + (uint64_t)nv;
#pragma unroll
    for (int k = 0; k < K; k++) {
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
      rg[k] = ((sb[k] & (kDedupSize - 1)) * R) >> 13;
      if (64 * k + lane < nv) __hip_atomic_fetch_add(&run[rg[k]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __builtin_amdgcn_wave_barrier();
    // each region's base (regions d 64 + lane of this lane: a wave scan of their sum)
    uint32_t cr[D], tot = 0;
#pragma unroll
    for (int d = 0; d < D; d++) {
      cr[d] = __hip_atomic_load(&run[d * 64 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      tot += cr[d];
    }
    uint32_t at = sgd::wave_incl_add(tot) - tot;
#pragma unroll
    for (int d = 0; d < D; d++) {
      wbc[nb][d * 64 + lane] = (at << 16) | cr[d];
      __hip_atomic_store(&run[d * 64 + lane], at, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      at += cr[d];
    }
    __builtin_amdgcn_wave_barrier();
    // row by row in program order: the row's masks give each edge its rank in its region
#pragma unroll
    for (int k = 0; k < K; k++) {
      const bool ok = 64 * k + lane < nv;
      if (ok) __hip_atomic_fetch_or(&wmask[rg[k]], 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __builtin_amdgcn_wave_barrier();
      const uint64_t m = __hip_atomic_load(&wmask[rg[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const uint32_t r0 = __hip_atomic_load(&run[rg[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      uint64_t om[D];
      uint32_t orun[D];
#pragma unroll
      for (int d = 0; d < D; d++) {
        om[d] = __hip_atomic_load(&wmask[d * 64 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        orun[d] = __hip_atomic_load(&run[d * 64 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      __builtin_amdgcn_wave_barrier();
      if (ok) {
        const uint32_t slot = r0 + (uint32_t)__popcll(m & lt);
        wsig[nb][slot] = sb[k];
        wpos[nb][slot] = (uint8_t)(64 * k + lane);
      }
#pragma unroll
      for (int d = 0; d < D; d++) {
        __hip_atomic_store(&run[d * 64 + lane], orun[d] + (uint32_t)__popcll(om[d]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&wmask[d * 64 + lane], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int d = 0; d < D; d++)
      __hip_atomic_store(&run[d * 64 + lane], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (lane < 2 * D) pubp[nb][lane / D][lane % D] = 0;  // nothing decided yet
    if (lane == 0) wlive[nb] = 1;
  };
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
  if (prod) build(0, sd, nd, cd, bd, ld, fd, ed);
  lds_sync();
  for (uint32_t it = 0;; it++) {
    const uint32_t buf = it & 1;
    const bool live = __hip_atomic_load(&wlive[buf], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
    if (!prod) {
      if (live) {
        const uint32_t r = (uint32_t)wv * 64 + lane;
        const uint32_t bcw = wbc[buf][r];
        const uint32_t base = bcw >> 16, iend = base + (bcw & 0xFFFFu);
        uint32_t i = base;
        uint32_t pos = i < iend ? (uint32_t)wpos[buf][i] : kNoPos;
        uint32_t s = wsig[buf][i < iend ? i : 0];
        // lanes 0 / 63: their slot in pubp, and the neighbouring wave's to read
        const uint32_t wl = (uint32_t)(wv + D - 1) % D, wr = (uint32_t)(wv + 1) % D;
        uint32_t* pub_mine = lane == 0 ? &pubp[buf][0][wv] : lane == 63 ? &pubp[buf][1][wv] : nullptr;
        const uint32_t* pub_nb = lane == 0 ? &pubp[buf][1][wl] : lane == 63 ? &pubp[buf][0][wr] : nullptr;
        while (__ballot(pos != kNoPos)) {
          uint32_t left = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pos, 0x13C /* wave_ror:1 */, 0xF, 0xF, false);
          uint32_t right = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pos, 0x134 /* wave_rol:1 */, 0xF, 0xF, false);
          if (D > 1) {
            // (compiler barriers: the last step's table writes stay before the
            // published position, the neighbour's position is read before this
            // step's table reads; the LDS keeps one wave's operations in order)
            asm volatile("" ::: "memory");
            if (pub_mine) __hip_atomic_store(pub_mine, pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (pub_nb) {
              const uint32_t x = __hip_atomic_load(pub_nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              if (lane == 0) left = x;
              else right = x;
            }
            asm volatile("" ::: "memory");
          }
          const uint32_t hr = s & (S - 1);
          const bool go = (pos != kNoPos) & ((hr > 2u) | (left > pos)) & ((hr < S - 3) | (right > pos));
          const uint32_t i2 = i + (go ? 1u : 0u);
          const uint32_t home = s & (kDedupSize - 1);
          const uint32_t t0 = table[home], t1 = table[home + 1], t2 = table[home + 2], t3 = table[home + 3];
          const uint32_t ni = i2 < iend ? i2 : 0;
          const uint32_t nsg = wsig[buf][ni];
          const uint32_t npo = wpos[buf][ni];
          const bool h0 = (t0 == s) | (t0 == 0u), h1 = (t1 == s) | (t1 == 0u), h2 = (t2 == s) | (t2 == 0u);
          const bool h3 = (t3 == s) | (t3 == 0u);
          const uint32_t q = h0 ? 0u : h1 ? 1u : h2 ? 2u : h3 ? 3u : 0u;
          const uint32_t tq = h0 ? t0 : h1 ? t1 : h2 ? t2 : t3;
          const bool dup = (tq == s) & (h0 | h1 | h2 | h3);
          const bool wr_ = go & !dup;
          const uint32_t dd = (home + q) & (kDedupSize - 1);
          table[wr_ ? dd : kDedupSize + 3] = s;
          table[wr_ && dd < 3u ? dd + kDedupSize : kDedupSize + 3] = s;
          wres[buf][go ? (pos & 63u) * K + (pos >> 6) : (uint32_t)W] = dup ? 0 : 1;
          i = i2;
          pos = i < iend ? npo : kNoPos;
          s = nsg;
        }
        if (D > 1 && pub_mine) __hip_atomic_store(pub_mine, kNoPos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else {
      if (nq) compact(buf ^ 1);
      uint32_t sb[K];
      int nb_ = 0;
      uint64_t cb = 0, bb = 0;
      bool lb = false, fb = false, eb = false;
      if (live) build(buf ^ 1, sb, nb_, cb, bb, lb, fb, eb);
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
    if (!live) break;
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
#if SG_COMPACT_UNROLL
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
#else
  for (uint64_t i = lane; i < n; i += 64) out[dst + i] = tmp[src + i];
#endif
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
  // SG_EXEC_REGION (read at each call: tests switch it): 104 (default) the
  // slot-region kernel with a producer wave, 256-edge windows; 102 the same at
  // 128; 1 / 2 / 4 / 8 / 16 the one-wave slot-region kernel at 64 K-edge
  // windows; 0 the speculative kernel (SG_EXEC_K picks its window)
  const int kr = [] {
    const char* e = getenv("SG_EXEC_REGION");
    return e ? atoi(e) : 104;
  }();
  if (nprog && ctx->debug_part && kr == 4) {  // diagnostics: steps and cycles of the slot-region kernel (syncs)
    unsigned long long* st = nullptr;
    SG_HIP(hipMalloc(&st, 40));
    SG_HIP(hipMemsetAsync(st, 0, 40, ctx->stream));
    hipLaunchKernelGGL((k_exec_region<4>), dim3((uint32_t)nprog), dim3(64), 0, ctx->stream, d_pcs, d_call_off, d_prog_off,
                       tmp, cnt, (const uint64_t*)pstop, d_rec_new, st);
    unsigned long long h[5] = {0, 0, 0, 0, 0};
    SG_HIP(hipMemcpy(h, st, 40, hipMemcpyDeviceToHost));
    SG_HIP(hipFree(st));
    fprintf(stderr,
            "sg exec region: programs %llu windows %llu steps %llu (%.2f per window, %.1f edges per step) "
            "cycles per step %.0f, per window %.0f (steps %.0f)\n",
            (unsigned long long)nprog, h[0], h[1], h[0] ? (double)h[1] / h[0] : 0.0, h[1] ? (double)h[4] / h[1] : 0.0,
            h[1] ? (double)h[2] / h[1] : 0.0, h[0] ? (double)h[3] / h[0] : 0.0, h[0] ? (double)h[2] / h[0] : 0.0);
  } else if (nprog && ctx->debug_part) {  // diagnostics: speculative passes per 128-edge window (syncs)
    unsigned long long* st = nullptr;
    SG_HIP(hipMalloc(&st, 32));
    SG_HIP(hipMemsetAsync(st, 0, 32, ctx->stream));
    hipLaunchKernelGGL(k_exec_signal<true>, dim3((uint32_t)nprog), dim3(64), 0, ctx->stream, d_pcs, d_call_off,
                       d_prog_off, tmp, cnt, st, (const uint64_t*)pstop, d_rec_new);
    unsigned long long h[3] = {0, 0, 0};
    SG_HIP(hipMemcpy(h, st, 24, hipMemcpyDeviceToHost));
    SG_HIP(hipFree(st));
    fprintf(stderr, "sg exec: programs %llu windows %llu passes %llu (%.2f per window) edges %llu\n",
            (unsigned long long)nprog, h[0], h[1], h[0] ? (double)h[1] / h[0] : 0.0, h[2]);
  } else if (nprog) {
    ScopedTimer tm(ctx, "exec_signal");
    // window of 64 edges by default (SG_EXEC_K = 2, 3, 4: 64 K edges; 32 / 48:
    // part-filled windows -- measurements; 1.89 ms per 134M PCs at 64 against
    // 2.24 at 128, 2.69 at 192, 3.41 at 256, 2.32 at 48 and 3.06 at 32)
    static const int kx = [] {
      const char* e = getenv("SG_EXEC_K");
      return e ? atoi(e) : 1;
    }();
    // slot-region kernel: SG_EXEC_REGION = rows per window (0: the speculative kernel)
    const dim3 g((uint32_t)nprog), t(64);
    const uint64_t* ps = (const uint64_t*)pstop;
    if (kr == 1)
      hipLaunchKernelGGL((k_exec_region<1>), g, t, 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps, d_rec_new);
    else if (kr == 2)
      hipLaunchKernelGGL((k_exec_region<2>), g, t, 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps, d_rec_new);
    else if (kr == 4)
      hipLaunchKernelGGL((k_exec_region<4>), g, t, 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps, d_rec_new);
    else if (kr == 8)
      hipLaunchKernelGGL((k_exec_region<8>), g, t, 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps, d_rec_new);
    else if (kr == 16)
      hipLaunchKernelGGL((k_exec_region<16>), g, t, 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps,
                         d_rec_new);
    else if (kr == 102)  // (102 / 104: the producer-wave kernel, 2 / 4 rows per window)
      hipLaunchKernelGGL((k_exec_region2<2>), g, dim3(128), 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps,
                         d_rec_new);
    else if (kr == 142)  // (1KD: the D-wave kernel, K rows per window)
      hipLaunchKernelGGL((k_exec_region3<4, 2>), g, dim3(192), 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps,
                         d_rec_new);
    else if (kr == 141)
      hipLaunchKernelGGL((k_exec_region3<4, 1>), g, dim3(128), 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps,
                         d_rec_new);
    else if (kr == 144)
      hipLaunchKernelGGL((k_exec_region3<4, 4>), g, dim3(320), 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps,
                         d_rec_new);
    else if (kr == 104)
      hipLaunchKernelGGL((k_exec_region2<4>), g, dim3(128), 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps,
                         d_rec_new);
    else if (kx == 2)
      hipLaunchKernelGGL((k_exec_signal_k<2>), g, t, 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps, d_rec_new);
    else if (kx == 3)
      hipLaunchKernelGGL((k_exec_signal_k<3>), g, t, 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps, d_rec_new);
    else if (kx == 4)
      hipLaunchKernelGGL((k_exec_signal_k<4>), g, t, 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps, d_rec_new);
    else if (kx == 32)
      hipLaunchKernelGGL((k_exec_signal_k<1, 32>), g, t, 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps,
                         d_rec_new);
    else if (kx == 48)
      hipLaunchKernelGGL((k_exec_signal_k<1, 48>), g, t, 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps,
                         d_rec_new);
    else
      hipLaunchKernelGGL((k_exec_signal_k<1>), g, t, 0, ctx->stream, d_pcs, d_call_off, d_prog_off, tmp, cnt, ps, d_rec_new);
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
