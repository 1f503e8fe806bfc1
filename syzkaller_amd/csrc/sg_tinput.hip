// sg_tinput.hip -- triageInput's signal math over a batch of inputs.
//
// Reference: syz-fuzzer/fuzzer.go:521-611 triageInput():
//   :526-532  newSignal = Canonicalize(SignalDiff(corpusSignal, inp.signal))
//   :567      newSignal = Intersection(newSignal, Canonicalize(inf.Signal))
//             after each of the 3 re-executions
//   :584-587  the minimisation predicate
//             len(Intersection(newSignal, Canonicalize(inf.Signal))) == len(newSignal)
// A fuzzer runs -procs triage goroutines; these entry points take the inputs
// of all of them (or of a whole batch of triage candidates) at once.  The
// executions in between stay with the caller.
//
// Intersection(a, Canonicalize(r)) for a sorted a (cover.go:72-102): r's
// canonical form holds each value at most once, so the foreach keeps the
// first copy of every value of a that occurs in r, except 0xFFFFFFFF (which
// foreach always drops), in a's order.  No sort of r is needed: one
// workgroup per input holds a (in LDS chunks of kCap values) and every element
// of r marks the first copy of its value in a by a binary search.
#include "sg_internal.h"

#include <algorithm>

namespace sg {

int canonicalize_dev(sg_ctx* ctx, uint32_t* d_vals, const uint64_t* off, uint64_t nseg, uint64_t* out_len);

namespace {

constexpr uint32_t kSentT = 0xFFFFFFFFu;  // cover.go:17
constexpr int kTB = 256;                  // threads per input
constexpr uint32_t kCap = 8192;           // a values per LDS chunk (32 KiB)

// Order-preserving compaction of one round of kTB flags inside a workgroup:
// returns this thread's rank among the kept ones; *total = kept in the round.
__device__ __forceinline__ uint32_t block_rank(bool keep, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t m = __ballot(keep);
  const uint32_t below = __popcll(m & (lane ? (~0ull >> (64 - lane)) : 0ull));
  if (lane == 0) wsum[w] = __popcll(m);
  __syncthreads();
  uint32_t base = 0, t = 0;
#pragma unroll
  for (int k = 0; k < kTB / 64; k++) {
    const uint32_t c = wsum[k];
    base += k < w ? c : 0u;
    t += c;
  }
  __syncthreads();
  *total = t;
  return base + below;
}

// SignalDiff (cover.go:169-176) per segment: count, then write in order.
template <bool kWrite>
__global__ __launch_bounds__(kTB) void k_tin_diff(const uint32_t* __restrict__ words, const uint32_t* __restrict__ v,
                                                  const uint64_t* __restrict__ off, uint32_t* __restrict__ cnt,
                                                  const uint64_t* __restrict__ dst_off, uint32_t* __restrict__ dst) {
  __shared__ uint32_t wsum[kTB / 64];
  const uint64_t k = blockIdx.x, b = off[k], e = off[k + 1];
  uint64_t pos = kWrite ? dst_off[k] : 0;
  uint32_t n = 0;
  for (uint64_t base = b; base < e; base += kTB) {
    const uint64_t i = base + threadIdx.x;
    uint32_t s = 0;
    bool miss = false;
    if (i < e) {
      s = v[i];
      miss = !sgd::test_bit(words, s);
    }
    uint32_t tot;
    const uint32_t r = block_rank(miss, wsum, &tot);
    if (kWrite && miss) dst[pos + r] = s;
    pos += tot;
    n += tot;
  }
  if (!kWrite && threadIdx.x == 0) cnt[k] = n;
}

// Intersection(a_k, Canonicalize(r_k)) for every input k (see the header):
// kIntersect writes the kept values at a_k's own start and out_len[k];
// otherwise ok[k] = (kept == len(a_k)).
template <bool kIntersect>
__global__ __launch_bounds__(kTB) void k_tin_intersect(uint32_t* __restrict__ a, const uint64_t* __restrict__ a_off,
                                                       const uint32_t* __restrict__ r,
                                                       const uint64_t* __restrict__ r_off,
                                                       uint64_t* __restrict__ out_len, uint8_t* __restrict__ ok) {
  __shared__ uint32_t av[kCap];
  __shared__ uint32_t found[kCap / 32];
  __shared__ uint32_t wsum[kTB / 64];
  const uint64_t k = blockIdx.x, a0 = a_off[k], a1 = a_off[k + 1], r0 = r_off[k], r1 = r_off[k + 1];
  uint64_t kept = 0;
  for (uint64_t c0 = a0; c0 < a1; c0 += kCap) {
    const uint32_t m = (uint32_t)std::min<uint64_t>(kCap, a1 - c0);
    __syncthreads();  // the previous chunk is written out
    for (uint32_t j = threadIdx.x; j < m; j += kTB) av[j] = a[c0 + j];
    for (uint32_t j = threadIdx.x; j < kCap / 32; j += kTB) found[j] = 0;
    __syncthreads();
    for (uint64_t i = r0 + threadIdx.x; i < r1; i += kTB) {
      const uint32_t x = r[i];
      uint32_t lo = 0, hi = m;  // first j with av[j] >= x
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (av[mid] < x)
          lo = mid + 1;
        else
          hi = mid;
      }
      if (lo < m && av[lo] == x) atomicOr(&found[lo >> 5], 1u << (lo & 31));
    }
    __syncthreads();
    // c0 > a0: the value before the chunk decides whether its first element is a first copy
    const uint32_t before = c0 > a0 ? a[c0 - 1] : 0u;
    for (uint32_t j0 = 0; j0 < m; j0 += kTB) {
      const uint32_t j = j0 + threadIdx.x;
      bool keep = false;
      uint32_t x = 0;
      if (j < m) {
        x = av[j];
        const bool first = j ? av[j - 1] != x : (c0 == a0 || before != x);
        keep = ((found[j >> 5] >> (j & 31)) & 1u) && first && x != kSentT;
      }
      uint32_t tot;
      const uint32_t rk = block_rank(keep, wsum, &tot);
      if (kIntersect && keep) a[a0 + kept + rk] = x;  // never past the chunk: kept + rk <= c0 - a0 + j
      kept += tot;
    }
  }
  if (threadIdx.x == 0) {
    if (kIntersect)
      out_len[k] = kept;
    else
      ok[k] = kept == a1 - a0 ? 1 : 0;
  }
}

// dst[dst_off[k] ..] = src[src_off[k] .. + len[k]), one wave per segment
__global__ void k_seg_pack(const uint32_t* __restrict__ src, const uint64_t* __restrict__ src_off,
                           const uint64_t* __restrict__ len, const uint64_t* __restrict__ dst_off, uint64_t n,
                           uint32_t* __restrict__ dst) {
  const uint64_t k = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (k >= n) return;
  const uint64_t s = src_off[k], d = dst_off[k], L = len[k];
  for (uint64_t i = threadIdx.x & 63; i < L; i += 64) dst[d + i] = src[s + i];
}

bool offsets_ok(const uint64_t* off, size_t n) {
  if (off[0] != 0) return false;
  for (size_t k = 0; k < n; k++)
    if (off[k + 1] < off[k]) return false;
  return true;
}

// Stage a CSR (host) into dstage at byte offset `at`: values then offsets.
struct Staged {
  uint32_t* v;
  uint64_t* off;
};

}  // namespace
}  // namespace sg

using namespace sg;

extern "C" {

int sg_triage_newsig(sg_ctx* ctx, sg_set* corpus, const uint32_t* vals, const uint64_t* off, size_t n,
                     uint32_t* new_vals, uint64_t* new_off) {
  if (!ctx || !corpus || corpus->ctx != ctx || !off || !new_off || !offsets_ok(off, n) ||
      (off[n] && (!vals || !new_vals))) {
    set_error("sg_triage_newsig: invalid argument");
    return SG_EINVAL;
  }
  const uint64_t N = off[n];
  if (n == 0 || N == 0) {
    for (size_t k = 0; k <= n; k++) new_off[k] = 0;
    return SG_OK;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  // dstage: S vals | S off | diff vals | diff off | canonical lengths | packed off | packed vals
  const size_t b_v = (N * 4 + 255) & ~size_t(255), b_o = ((n + 1) * 8 + 255) & ~size_t(255);
  rc = dstage_reserve(ctx, 3 * b_v + 3 * b_o + b_o);
  if (rc) return rc;
  char* st = (char*)ctx->dstage;
  uint32_t* dv = (uint32_t*)st;
  uint64_t* doff = (uint64_t*)(st + b_v);
  uint32_t* ddiff = (uint32_t*)(st + b_v + b_o);
  uint64_t* ddoff = (uint64_t*)(st + 2 * b_v + b_o);
  uint64_t* dlen = (uint64_t*)(st + 2 * b_v + 2 * b_o);
  uint64_t* dpoff = (uint64_t*)(st + 2 * b_v + 3 * b_o);
  uint32_t* dpack = (uint32_t*)(st + 2 * b_v + 4 * b_o);
  WsPlan p;
  const size_t o_cnt = p.add(n * 4);
  rc = ws_reserve(ctx, p.total + scan_ws_bytes(n));
  if (rc) return rc;
  uint32_t* dcnt = (uint32_t*)ws_at(ctx, o_cnt);
  SG_HIP(hipMemcpyAsync(dv, vals, N * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(doff, off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  {
    ScopedTimer tm(ctx, "tinput_diff");
    hipLaunchKernelGGL(k_tin_diff<false>, dim3((uint32_t)n), dim3(kTB), 0, ctx->stream, corpus->words, dv, doff, dcnt,
                       nullptr, nullptr);
    rc = scan_counts(ctx, dcnt, ddoff, n, p.total);
    if (rc) return rc;
    hipLaunchKernelGGL(k_tin_diff<true>, dim3((uint32_t)n), dim3(kTB), 0, ctx->stream, corpus->words, dv, doff, nullptr,
                       ddoff, ddiff);
  }
  SG_HIP(hipGetLastError());
  std::vector<uint64_t> hdoff(n + 1), len(n);
  SG_HIP(hipMemcpyAsync(hdoff.data(), ddoff, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (hdoff[n] == 0) {
    for (size_t k = 0; k <= n; k++) new_off[k] = 0;
    return SG_OK;
  }
  // Canonicalize (cover.go:28-40) of every diff segment, in place
  rc = canonicalize_dev(ctx, ddiff, hdoff.data(), n, len.data());
  if (rc) return rc;
  new_off[0] = 0;
  for (size_t k = 0; k < n; k++) new_off[k + 1] = new_off[k] + len[k];
  SG_HIP(hipMemcpyAsync(dlen, len.data(), n * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dpoff, new_off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_seg_pack, dim3(div_up(n, 4)), dim3(256), 0, ctx->stream, ddiff, ddoff, dlen, dpoff,
                     (uint64_t)n, dpack);
  SG_HIP(hipGetLastError());
  if (new_off[n]) SG_HIP(hipMemcpyAsync(new_vals, dpack, new_off[n] * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

static int tinput_intersect(sg_ctx* ctx, uint32_t* a, const uint64_t* a_off, const uint32_t* r, const uint64_t* r_off,
                            size_t n, uint64_t* out_len, uint8_t* ok) {
  const uint64_t NA = a_off[n], NR = r_off[n];
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  const size_t b_a = (NA * 4 + 255) & ~size_t(255), b_r = (NR * 4 + 255) & ~size_t(255),
               b_o = ((n + 1) * 8 + 255) & ~size_t(255), b_f = (n + 255) & ~size_t(255);
  rc = dstage_reserve(ctx, b_a + b_r + 3 * b_o + b_f);
  if (rc) return rc;
  char* st = (char*)ctx->dstage;
  uint32_t* da = (uint32_t*)st;
  uint32_t* dr = (uint32_t*)(st + b_a);
  uint64_t* dao = (uint64_t*)(st + b_a + b_r);
  uint64_t* dro = (uint64_t*)(st + b_a + b_r + b_o);
  uint64_t* dlen = (uint64_t*)(st + b_a + b_r + 2 * b_o);
  uint8_t* dok = (uint8_t*)(st + b_a + b_r + 3 * b_o);
  if (NA) SG_HIP(hipMemcpyAsync(da, a, NA * 4, hipMemcpyHostToDevice, ctx->stream));
  if (NR) SG_HIP(hipMemcpyAsync(dr, r, NR * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dao, a_off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dro, r_off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  {
    ScopedTimer tm(ctx, "tinput_intersect");
    if (out_len)
      hipLaunchKernelGGL(k_tin_intersect<true>, dim3((uint32_t)n), dim3(kTB), 0, ctx->stream, da, dao, dr, dro, dlen,
                         nullptr);
    else
      hipLaunchKernelGGL(k_tin_intersect<false>, dim3((uint32_t)n), dim3(kTB), 0, ctx->stream, da, dao, dr, dro,
                         nullptr, dok);
  }
  SG_HIP(hipGetLastError());
  if (out_len) {
    SG_HIP(hipMemcpyAsync(out_len, dlen, n * 8, hipMemcpyDeviceToHost, ctx->stream));
    if (NA) SG_HIP(hipMemcpyAsync(a, da, NA * 4, hipMemcpyDeviceToHost, ctx->stream));
  } else {
    SG_HIP(hipMemcpyAsync(ok, dok, n, hipMemcpyDeviceToHost, ctx->stream));
  }
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

int sg_triage_intersect(sg_ctx* ctx, uint32_t* new_vals, const uint64_t* new_off, const uint32_t* r_vals,
                        const uint64_t* r_off, size_t n, uint64_t* out_len) {
  if (!ctx || !new_off || !r_off || (n && !out_len) || !offsets_ok(new_off, n) || !offsets_ok(r_off, n) ||
      (new_off[n] && !new_vals) || (r_off[n] && !r_vals)) {
    set_error("sg_triage_intersect: invalid argument");
    return SG_EINVAL;
  }
  if (n == 0) return SG_OK;
  if (new_off[n] == 0) {
    for (size_t k = 0; k < n; k++) out_len[k] = 0;
    return SG_OK;
  }
  return tinput_intersect(ctx, new_vals, new_off, r_vals, r_off, n, out_len, nullptr);
}

int sg_triage_subset(sg_ctx* ctx, const uint32_t* new_vals, const uint64_t* new_off, const uint32_t* r_vals,
                     const uint64_t* r_off, size_t n, uint8_t* ok) {
  if (!ctx || !new_off || !r_off || (n && !ok) || !offsets_ok(new_off, n) || !offsets_ok(r_off, n) ||
      (new_off[n] && !new_vals) || (r_off[n] && !r_vals)) {
    set_error("sg_triage_subset: invalid argument");
    return SG_EINVAL;
  }
  if (n == 0) return SG_OK;
  if (new_off[n] == 0) {
    for (size_t k = 0; k < n; k++) ok[k] = 1;  // len(Intersection(nil, x)) == 0 == len(nil)
    return SG_OK;
  }
  return tinput_intersect(ctx, const_cast<uint32_t*>(new_vals), new_off, r_vals, r_off, n, nullptr, ok);
}

}  // extern "C"
