// sg_sort.hip -- a stable LSD radix sort of 64-bit keys (device-resident).
//
// Used where the path needs sorted, deduplicated (key, value) streams rather
// than the partitioned triage's buckets: the manager's Union folds
// (sg_fold.hip, syz-manager/html.go:84,94,184,306).  8-bit digits from the
// lowest bit that varies between keys, a pass skipped when its digit is the
// same in every key (the varying bits come from the caller or one AND / OR
// reduction), so a fold of 2M 16-B-aligned kernel-text PCs sorts in 3
// passes, over a few thousand groups in 5, not 8.
//
// One pass = a per-tile digit histogram, an exclusive scan of the counts laid
// out [digit][tile] (scan_counts, sg_ctx.hip), and a scatter.  Tiles are 8192
// keys (512 threads x 16).  Stability, which LSD needs: wave w of a tile owns
// positions [1024 w, 1024 (w + 1)), 16 steps of 64; within a step the lanes
// holding a digit are found with 8 ballots (a wave-level multisplit) and
// ranked by lane, each wave keeps running per-digit counts in LDS, and one
// scan over the waves per digit orders the waves.  Keys are staged in LDS in
// tile-sorted order and written as per-digit runs, 32 keys per half-wave
// store.
#include "sg_internal.h"

#include <algorithm>
#include <vector>

namespace sg {

constexpr int kRsThreads = 512;
constexpr int kRsWaves = kRsThreads / 64;
constexpr int kRsSteps = 16;                      // keys per lane
constexpr uint32_t kRsTile = kRsThreads * kRsSteps;  // 8192

__global__ void k_rs_andor(const uint64_t* __restrict__ k, uint64_t n, unsigned long long* __restrict__ out) {
  uint64_t a = ~0ull, o = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    a &= k[i];
    o |= k[i];
  }
  for (int d = 32; d; d >>= 1) {
    a &= __shfl_xor(a, d);
    o |= __shfl_xor(o, d);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAnd(&out[0], a);
    atomicOr(&out[1], o);
  }
}

__device__ __forceinline__ uint32_t rs_digit(uint64_t k, uint32_t shift) { return (uint32_t)(k >> shift) & 255u; }

// hist[d * ntiles + t] = number of keys of tile t with digit d
// Tile t's keys: keys[tile_base(t) ..], n_t of them.  Contiguous tiles of
// kRsTile, or (tsrc != null) tile t = tsrc[t], tcnt[t] keys: a first pass
// reading runs scattered over a gapped buffer.
__device__ __forceinline__ void rs_tile(uint64_t n, const uint64_t* tsrc, const uint32_t* tcnt, uint32_t t,
                                        uint64_t& base, uint64_t& nt) {
  if (tsrc) {
    base = tsrc[t];
    nt = tcnt[t];
  } else {
    base = (uint64_t)t * kRsTile;
    nt = min<uint64_t>(kRsTile, n - base);
  }
}

__global__ __launch_bounds__(kRsThreads) void k_rs_hist(const uint64_t* __restrict__ keys, uint64_t n, uint32_t shift,
                                                        uint32_t ntiles, uint32_t* __restrict__ hist,
                                                        const uint64_t* __restrict__ tsrc,
                                                        const uint32_t* __restrict__ tcnt) {
  __shared__ uint32_t cnt[kRsWaves][256];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  for (int i = tid; i < kRsWaves * 256; i += kRsThreads) (&cnt[0][0])[i] = 0;
  __syncthreads();
  uint64_t tb, tn;
  rs_tile(n, tsrc, tcnt, blockIdx.x, tb, tn);
  keys += tb;
  n = tn;
  const uint64_t base = (uint64_t)w * (64 * kRsSteps);
#pragma unroll 4
  for (int s = 0; s < kRsSteps; s++) {
    const uint64_t e = base + s * 64 + lane;
    if (e < n) atomicAdd(&cnt[w][rs_digit(keys[e], shift)], 1u);
  }
  __syncthreads();
  if (tid < 256) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < kRsWaves; i++) c += cnt[i][tid];
    hist[(uint64_t)tid * ntiles + blockIdx.x] = c;
  }
}

// lanes of the wave whose digit equals this lane's (8 ballots)
__device__ __forceinline__ uint64_t rs_peers(uint32_t d, bool live) {
  uint64_t eq = __ballot(live);
#pragma unroll
  for (int b = 0; b < 8; b++) {
    const uint64_t bal = __ballot((d >> b) & 1u);
    eq &= ((d >> b) & 1u) ? bal : ~bal;
  }
  return eq;
}

__global__ __launch_bounds__(kRsThreads) void k_rs_scatter(const uint64_t* __restrict__ in, uint64_t n, uint32_t shift,
                                                           uint32_t ntiles, const uint64_t* __restrict__ goff,
                                                           uint64_t* __restrict__ out, const uint64_t* __restrict__ tsrc,
                                                           const uint32_t* __restrict__ tcnt) {
  __shared__ uint64_t stage[kRsTile];
  __shared__ uint32_t cnt[kRsWaves][256];  // per-wave running counts, then per-wave offsets in the tile
  __shared__ uint32_t dstart[256];         // digit start in the tile (stage)
  __shared__ uint32_t dend[256];
  __shared__ uint64_t gb[256];             // global start of the tile's digit run
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const uint32_t t = blockIdx.x;
  for (int i = tid; i < kRsWaves * 256; i += kRsThreads) (&cnt[0][0])[i] = 0;
  if (tid < 256) gb[tid] = goff[(uint64_t)tid * ntiles + t];
  uint64_t tb, tn;
  rs_tile(n, tsrc, tcnt, t, tb, tn);
  in += tb;
  n = tn;
  const uint64_t base = (uint64_t)w * (64 * kRsSteps);
  uint64_t k[kRsSteps];
#pragma unroll
  for (int s = 0; s < kRsSteps; s++) {
    const uint64_t e = base + s * 64 + lane;
    k[s] = e < n ? in[e] : 0ull;
  }
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t rank[kRsSteps];
#pragma unroll
  for (int s = 0; s < kRsSteps; s++) {
    const bool live = base + s * 64 + lane < n;
    const uint32_t d = rs_digit(k[s], shift);
    const uint64_t eq = rs_peers(d, live);
    const uint32_t before = live ? cnt[w][d] : 0u;  // this wave's keys of digit d in earlier steps
    rank[s] = before + (uint32_t)__popcll(eq & lt);
    // the lowest lane of each digit group advances the count (after every
    // lane of the wave has read it: one wave's LDS operations are in order)
    if (live && (eq & lt) == 0) cnt[w][d] = before + (uint32_t)__popcll(eq);
  }
  __syncthreads();
  // per digit: the waves' offsets and the digit's start in the tile
  if (tid < 256) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < kRsWaves; i++) {
      const uint32_t c = cnt[i][tid];
      cnt[i][tid] = acc;
      acc += c;
    }
    dend[tid] = acc;  // the digit's count (scanned below)
  }
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the 256 digit counts (one wave, 4 per lane)
    uint32_t c[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      c[j] = dend[tid * 4 + j];
      s += c[j];
    }
    const uint32_t incl = sgd::wave_incl_add(s);
    uint32_t run = incl - s;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      dstart[tid * 4 + j] = run;
      run += c[j];
      dend[tid * 4 + j] = run;
    }
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < kRsSteps; s++) {
    if (base + s * 64 + lane < n) {
      const uint32_t d = rs_digit(k[s], shift);
      stage[dstart[d] + cnt[w][d] + rank[s]] = k[s];
    }
  }
  __syncthreads();
  // runs out: half-wave h copies digits h, h + 16, ...
  const int hw = tid >> 5, hl = tid & 31;
  for (int d = hw; d < 256; d += kRsThreads / 32) {
    const uint32_t s0 = dstart[d], s1 = dend[d];
    const uint64_t g = gb[d] - s0;
    for (uint32_t p = s0 + hl; p < s1; p += 32) out[g + p] = stage[p];
  }
}

// Workspace bytes radix_sort_u64 needs beyond the two key buffers.
size_t radix_sort_ws(uint64_t n) {
  const uint64_t nt = (n + kRsTile - 1) / kRsTile;
  return ((256 * nt * 4 + 255) & ~255ull) + (((256 * nt + 1) * 8 + 255) & ~255ull) + 256 + scan_ws_bytes(256 * nt);
}

// Sorts n keys of a (device) stably; b is scratch of n keys.  *sorted is a
// or b, whichever holds the result.  Uses the workspace from ws_used on
// (radix_sort_ws(n) bytes, reserved by the caller).  vary: the key bits that
// may differ between keys (a superset is fine), or 0 to find them with one
// reduction and a host sync.
int radix_sort_u64(sg_ctx* ctx, uint64_t* a, uint64_t* b, uint64_t n, size_t ws_used, uint64_t** sorted,
                   uint64_t vary) {
  *sorted = a;
  if (n < 2) return SG_OK;
  const uint64_t nt = (n + kRsTile - 1) / kRsTile;
  char* ws = (char*)ws_at(ctx, ws_used);
  uint32_t* hist = (uint32_t*)ws;
  uint64_t* goff = (uint64_t*)(ws + ((256 * nt * 4 + 255) & ~255ull));
  unsigned long long* ao = (unsigned long long*)((char*)goff + (((256 * nt + 1) * 8 + 255) & ~255ull));
  const size_t scan_at = ws_used + ((256 * nt * 4 + 255) & ~255ull) + (((256 * nt + 1) * 8 + 255) & ~255ull) + 256;
  if (!vary) {
    unsigned long long init[2] = {~0ull, 0ull}, got[2];
    SG_HIP(hipMemcpyAsync(ao, init, 16, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_rs_andor, dim3(1024), dim3(256), 0, ctx->stream, (const uint64_t*)a, n, ao);
    SG_HIP(hipMemcpyAsync(got, ao, 16, hipMemcpyDeviceToHost, ctx->stream));
    SG_HIP(hipStreamSynchronize(ctx->stream));
    vary = got[0] ^ got[1];
  }
  uint64_t* src = a;
  uint64_t* dst = b;
  if (!vary) return SG_OK;  // every key equal
  // digits start at the lowest bit that varies (kernel-text PCs are 16-B
  // aligned: their low 4 bits never do), and skip digits that do not vary
  const uint32_t lo = (uint32_t)__builtin_ctzll(vary), hi = 64 - (uint32_t)__builtin_clzll(vary);
  for (uint32_t shift = lo; shift < hi; shift += 8) {
    if (((vary >> shift) & 255u) == 0) continue;  // the same digit in every key
    hipLaunchKernelGGL(k_rs_hist, dim3((uint32_t)nt), dim3(kRsThreads), 0, ctx->stream, (const uint64_t*)src, n, shift,
                       (uint32_t)nt, hist, nullptr, nullptr);
    int rc = scan_counts(ctx, hist, goff, 256 * nt, scan_at);
    if (rc) return rc;
    hipLaunchKernelGGL(k_rs_scatter, dim3((uint32_t)nt), dim3(kRsThreads), 0, ctx->stream, (const uint64_t*)src, n,
                       shift, (uint32_t)nt, (const uint64_t*)goff, dst, nullptr, nullptr);
    SG_HIP(hipGetLastError());
    std::swap(src, dst);
  }
  *sorted = src;
  return SG_OK;
}

// One stable pass (digit at `shift`) over keys held in runs of a gapped
// buffer: the host's runs (start, count) are cut into tiles of <= kRsTile,
// and the pass writes the n keys contiguously into dst, ordered by digit,
// then by run order.  Workspace from ws_used on: radix_sort_ws(n) plus the
// tile table (runs + n / kRsTile tiles).
int radix_pass_runs(sg_ctx* ctx, const uint64_t* src, const std::vector<uint64_t>& run_start,
                    const std::vector<uint64_t>& run_cnt, uint32_t shift, uint64_t* dst, size_t ws_used) {
  std::vector<uint64_t> ts;
  std::vector<uint32_t> tc;
  uint64_t n = 0;
  for (size_t i = 0; i < run_start.size(); i++)
    for (uint64_t o = 0; o < run_cnt[i]; o += kRsTile) {
      ts.push_back(run_start[i] + o);
      tc.push_back((uint32_t)std::min<uint64_t>(kRsTile, run_cnt[i] - o));
      n += tc.back();
    }
  const uint64_t nt = ts.size();
  if (!nt) return SG_OK;
  char* ws = (char*)ws_at(ctx, ws_used);
  uint32_t* hist = (uint32_t*)ws;
  const size_t o_goff = (256 * nt * 4 + 255) & ~255ull;
  uint64_t* goff = (uint64_t*)(ws + o_goff);
  const size_t o_ts = o_goff + ((((256 * nt + 1) * 8) + 255) & ~255ull);
  uint64_t* dts = (uint64_t*)(ws + o_ts);
  const size_t o_tc = o_ts + ((nt * 8 + 255) & ~255ull);
  uint32_t* dtc = (uint32_t*)(ws + o_tc);
  const size_t scan_at = ws_used + o_tc + ((nt * 4 + 255) & ~255ull);
  SG_HIP(hipMemcpyAsync(dts, ts.data(), nt * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dtc, tc.data(), nt * 4, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_rs_hist, dim3((uint32_t)nt), dim3(kRsThreads), 0, ctx->stream, src, n, shift, (uint32_t)nt, hist,
                     (const uint64_t*)dts, (const uint32_t*)dtc);
  int rc = scan_counts(ctx, hist, goff, 256 * nt, scan_at);
  if (rc) return rc;
  hipLaunchKernelGGL(k_rs_scatter, dim3((uint32_t)nt), dim3(kRsThreads), 0, ctx->stream, src, n, shift, (uint32_t)nt,
                     (const uint64_t*)goff, dst, (const uint64_t*)dts, (const uint32_t*)dtc);
  SG_HIP(hipGetLastError());
  // (the host tables must outlive the copies)
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

// Workspace bytes of radix_pass_runs over n keys in nruns runs.
size_t radix_pass_runs_ws(uint64_t n, uint64_t nruns) {
  const uint64_t nt = n / kRsTile + nruns + 1;
  return ((256 * nt * 4 + 255) & ~255ull) + (((256 * nt + 1) * 8 + 255) & ~255ull) + ((nt * 8 + 255) & ~255ull) +
         ((nt * 4 + 255) & ~255ull) + scan_ws_bytes(256 * nt);
}

}  // namespace sg
