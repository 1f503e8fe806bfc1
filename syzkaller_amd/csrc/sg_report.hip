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
// an ordered compaction.  The per-query pass is split in two (k_rep_first,
// k_rep_del) so that each runs in the query order its read-check needs.  Symbols must be sorted by start with non-decreasing
// ends (the condition under which the reference's binary search over ends is
// meaningful).
#include "sg_internal.h"

#include <algorithm>

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
  RadixIdx iend, ipcs;    // indexes over send and pcs
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

__global__ void k_rep_group(RepArgs a) {
  uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.nsym) return;
  uint32_t f = a.first_q[s];
  if (f == 0xFFFFFFFFu) return;
  uint64_t leader = lb64(a.sstart, a.nsym, a.sstart[s]);  // handledFuncs keyed by start, cover.go:288
  atomicMin((unsigned long long*)&a.group_first[leader], ((unsigned long long)f << 32) | (unsigned long long)s);
}

__global__ void k_rep_final(RepArgs a) {
  uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.npcs) return;
  uint64_t c = a.pcs[j];
  int64_t best = -1;  // latest add time
  uint64_t g = ub64(a.sstart, a.nsym, c);  // symbols [0, g) have start <= c
  while (g > 0) {
    uint64_t last = g - 1;                 // last symbol of the group
    if (a.send[last] < c) break;           // ends non-decreasing: nothing earlier reaches c
    uint64_t leader = lb64(a.sstart, a.nsym, a.sstart[last]);
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
  RadixIdx iend{}, ipcs{};
  plan_idx(nsym, sym_end[0], sym_end[nsym - 1], iend);
  plan_idx(nall, all_pcs[0], all_pcs[nall - 1], ipcs);
  const size_t o_ie = p.add(((uint64_t)iend.nb + 1) * 4), o_ip = p.add(((uint64_t)ipcs.nb + 1) * 4);
  size_t scan_off = p.total;
  rc = ws_reserve(ctx, p.total + scan_ws_bytes(nchunks));
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
  a.iend = iend;
  a.ipcs = ipcs;
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
  }
  const dim3 qgrid((uint32_t)std::min<uint64_t>(div_up(ncov, 256), 16384));
  {
    ScopedTimer tm(ctx, "report_first");
    hipLaunchKernelGGL(k_rep_first, qgrid, dim3(256), 0, ctx->stream, a);
  }
  {
    ScopedTimer tm(ctx, "report_del");
    hipLaunchKernelGGL(k_rep_del, qgrid, dim3(256), 0, ctx->stream, a);
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
