// sg_shard.hip -- one batch's new-signal triage hash-sharded by signal across
// GPUs (the host protocol is syzkaller_amd/shard.py).
//
// Reference: syz-fuzzer/fuzzer.go:645-693, one sequential loop over every
// call record of the batch.  By the first-owner rule (sg_triage.hip), record
// r is queued iff some s not in maxSignal has owner(s) = min{r : s in S_r} =
// r, and maxSignal' = maxSignal ∪ ⋃ S_r.  owner(s) depends only on the
// records holding s, so the signal space shards cleanly:
//
//   candidates  (every rank, its contiguous slice of the batch's records)
//               the partitioned path (sg_bucket.hip) in emission mode: each
//               distinct s not in the replicated maxSignal snapshot, once,
//               with its first record of the slice (global index), grouped
//               by owning shard shard_of(s) -- only candidates travel;
//   [RCCL all-to-all of the pairs to their owning shard]
//   owners      (every rank, the pairs of its shard from all ranks) owner(s)
//               = min record over them (atomicMin into the first-owner
//               table), then the owners' bits in a batch-wide record bitset
//               and each new signal once;
//   [RCCL all-to-all of the bitset slices back to the records' ranks,
//    all-gather of the new signals]
//   flags       (every rank) its records' flags = OR of the received slices;
//               maxSignal / newSignal ∪= the new signals of every shard.
#include "sg_internal.h"

namespace sg {

constexpr uint32_t kShardMax = 64;  // == kMaxShards of sg_bucket.hip
// entries per emitting launch: about one C2 batch, so the buckets stay the
// size the LDS candidate map is built for (a launch twice that spilled a
// tenth of its buckets to the slow direct-table kernel); well under the
// partition's 2^32 cap
constexpr uint64_t kLaunchEntries = 1ull << 30;

__device__ __forceinline__ uint32_t shard_hash(uint32_t s, uint32_t nshards) {  // == shard_of (sg_bucket.hip)
  s ^= s >> 16;
  s *= 0x85EBCA6Bu;
  s ^= s >> 13;
  s *= 0xC2B2AE35u;
  s ^= s >> 16;
  return (uint32_t)(((uint64_t)s * nshards) >> 32);
}

__global__ void k_shard_offsets(const unsigned long long* __restrict__ cnt, uint32_t nshards,
                                uint64_t* __restrict__ off, unsigned long long* __restrict__ cursor) {
  if (threadIdx.x != 0) return;
  uint64_t run = 0;
  for (uint32_t k = 0; k < nshards; k++) {
    off[k] = run;
    cursor[k] = run;
    run += cnt[k];
  }
  off[nshards] = run;
}

// Pairs grouped by owning shard: per round of 1024 pairs a block ranks them
// per shard in LDS and reserves each shard's run with one global atomic.
constexpr int kRouteThreads = 256;
constexpr int kRoutePer = 4;
__global__ __launch_bounds__(kRouteThreads) void k_shard_route(const uint2* __restrict__ in,
                                                               const unsigned long long* __restrict__ npairs,
                                                               uint32_t nshards,
                                                               unsigned long long* __restrict__ cursor,
                                                               uint2* __restrict__ out) {
  __shared__ uint32_t cnt[kShardMax];
  __shared__ unsigned long long gb[kShardMax];
  const uint64_t n = *npairs;
  const int tid = threadIdx.x;
  constexpr uint64_t kRound = (uint64_t)kRouteThreads * kRoutePer;
  for (uint64_t base = (uint64_t)blockIdx.x * kRound; base < n; base += (uint64_t)gridDim.x * kRound) {
    if (tid < (int)kShardMax) cnt[tid] = 0;
    __syncthreads();
    uint2 v[kRoutePer];
    uint32_t sh[kRoutePer], loc[kRoutePer];
#pragma unroll
    for (int k = 0; k < kRoutePer; k++) {
      const uint64_t i = base + (uint64_t)k * kRouteThreads + tid;
      sh[k] = kShardMax;
      if (i < n) {
        v[k] = in[i];
        sh[k] = shard_hash(v[k].x, nshards);
        loc[k] = atomicAdd(&cnt[sh[k]], 1u);
      }
    }
    __syncthreads();
    if (tid < (int)nshards && cnt[tid]) gb[tid] = atomicAdd(&cursor[tid], (unsigned long long)cnt[tid]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRoutePer; k++)
      if (sh[k] < kShardMax) out[gb[sh[k]] + loc[k]] = v[k];
    __syncthreads();
  }
}

// owner(s) = min record over the received pairs (keys key_lo + record, below
// every key already in the table: sg::owner_keys)
__global__ void k_shard_claim(const uint2* __restrict__ pairs, uint64_t n, uint32_t* __restrict__ owner,
                              uint32_t key_lo) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint2 p = pairs[i];
    const uint32_t key = key_lo + p.y;
    uint32_t* o = owner + p.x;
    if (__hip_atomic_load(o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > key) atomicMin(o, key);
  }
}

// the owning pair of each s: its record's flag (a byte store: a record owns
// many signals, and atomics on its bit word were the stage's bottleneck), and
// s once in the new list, each block reserving its round's run with one
// atomic
constexpr int kResT = 1024, kResPer = 4;
__global__ __launch_bounds__(kResT) void k_shard_resolve(const uint2* __restrict__ pairs, uint64_t n,
                                                         const uint32_t* __restrict__ owner, uint32_t key_lo,
                                                         uint8_t* __restrict__ rec_flag, uint32_t* __restrict__ new_vals,
                                                         unsigned long long* __restrict__ nnew) {
  __shared__ uint32_t wcnt[kResT / 64 + 1];
  __shared__ unsigned long long sbase;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  constexpr uint64_t kRound = (uint64_t)kResT * kResPer;
  for (uint64_t base = (uint64_t)blockIdx.x * kRound; base < n; base += (uint64_t)gridDim.x * kRound) {
    uint2 p[kResPer];
    bool own[kResPer];
#pragma unroll
    for (int k = 0; k < kResPer; k++) {
      const uint64_t i = base + (uint64_t)k * kResT + tid;
      own[k] = false;
      p[k] = make_uint2(0, 0);
      if (i < n) p[k] = pairs[i];
    }
#pragma unroll
    for (int k = 0; k < kResPer; k++)
      if (base + (uint64_t)k * kResT + tid < n) own[k] = owner[p[k].x] == key_lo + p[k].y;
    uint64_t m[kResPer];
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < kResPer; k++) {
      if (own[k]) rec_flag[p[k].y] = 1;
      m[k] = __ballot(own[k]);
      c += (uint32_t)__popcll(m[k]);
    }
    if (lane == 0) wcnt[w] = c;
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      for (int i = 0; i < kResT / 64; i++) {
        const uint32_t v = wcnt[i];
        wcnt[i] = acc;
        acc += v;
      }
      sbase = acc ? atomicAdd(nnew, (unsigned long long)acc) : 0ull;
    }
    __syncthreads();
    uint64_t pos = sbase + wcnt[w];
#pragma unroll
    for (int k = 0; k < kResPer; k++) {
      if (own[k]) new_vals[pos + __popcll(m[k] & lt)] = p[k].x;
      pos += __popcll(m[k]);
    }
    __syncthreads();
  }
}

// bit r of bits = flag[r]
__global__ void k_pack_flags(const uint8_t* __restrict__ flag, uint64_t n, uint32_t* __restrict__ bits) {
  const uint64_t wi = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (wi * 32 >= n) return;
  uint32_t v = 0;
  for (int b = 0; b < 32; b++) {
    const uint64_t r = wi * 32 + b;
    if (r < n && flag[r]) v |= 1u << b;
  }
  bits[wi] = v;
}

// rec_new[i] = bit (rec_lo + i) of the OR of nparts bitsets, each holding
// the words from rec_lo / 32 on
__global__ void k_shard_flags(const uint32_t* __restrict__ bits, uint32_t nparts, uint64_t wpp, uint64_t rec_lo,
                              uint64_t nrec, uint8_t* __restrict__ rec_new) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrec) return;
  const uint64_t r = rec_lo + i, w = (r >> 5) - (rec_lo >> 5);
  uint32_t v = 0;
  for (uint32_t k = 0; k < nparts; k++) v |= bits[(uint64_t)k * wpp + w];
  rec_new[i] = (v >> (r & 31)) & 1u;
}

__global__ void k_set_add_vals(uint32_t* __restrict__ words, const uint32_t* __restrict__ v, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) sgd::set_bit(words, v[i]);
}

// maxsig |= v; newsig (nullable) gains the values maxsig lacked (fuzzer.go:673-674).
// The atomic's old word decides: of several copies of one value only the
// first setter sees its bit clear.
__global__ void k_set_add_new_vals(uint32_t* __restrict__ nwords, uint32_t* __restrict__ mwords,
                                   const uint32_t* __restrict__ v, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t s = v[i], w = sgd::set_pos(s) >> 5, b = 1u << (s & 31);
    const uint32_t old = atomicOr(&mwords[w], b);
    if (nwords && !(old & b)) atomicOr(&nwords[w], b);
  }
}

__global__ void k_set_del_vals(uint32_t* __restrict__ words, const uint32_t* __restrict__ v, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t s = v[i];
    atomicAnd(&words[sgd::set_pos(s) >> 5], ~(1u << (s & 31)));
  }
}

// the signals of a pairs-form begin's kept pairs {s, first record}, <= cap
__global__ void k_pair_sigs(const uint2* __restrict__ pairs, const unsigned long long* __restrict__ np, uint64_t cap,
                            uint32_t* __restrict__ out) {
  const uint64_t n = *np < cap ? *np : cap, stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = pairs[i].x;
}

// exclusive prefix-OR over the parts, word by word, and the total
__global__ void k_prefix_or(const uint32_t* __restrict__ parts, uint32_t nparts, uint64_t words,
                            uint32_t* __restrict__ prefix, uint32_t* __restrict__ total) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += stride) {
    uint32_t acc = 0;
    for (uint32_t k = 0; k < nparts; k++) {
      prefix[(uint64_t)k * words + w] = acc;
      acc |= parts[(uint64_t)k * words + w];
    }
    total[w] = acc;
  }
}

// The same over 16-B quads (words % 4 == 0, 16-B aligned buffers), kPoU
// quads per thread in flight: one word per thread and step left the pass
// latency-bound (0.58 ms for one 512 MiB part at one rank)
constexpr int kPoU = 4;
__global__ __launch_bounds__(256) void k_prefix_or4(const uint4* __restrict__ parts, uint32_t nparts, uint64_t quads,
                                                    uint4* __restrict__ prefix, uint4* __restrict__ total) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * kPoU;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x * kPoU + threadIdx.x; i0 < quads; i0 += stride) {
    uint4 acc[kPoU];
#pragma unroll
    for (int u = 0; u < kPoU; u++) acc[u] = make_uint4(0, 0, 0, 0);
    for (uint32_t k = 0; k < nparts; k++) {
      uint4 v[kPoU];
#pragma unroll
      for (int u = 0; u < kPoU; u++) {
        const uint64_t i = i0 + u * blockDim.x;
        v[u] = i < quads ? parts[(uint64_t)k * quads + i] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kPoU; u++) {
        const uint64_t i = i0 + u * blockDim.x;
        if (i < quads) prefix[(uint64_t)k * quads + i] = acc[u];
        acc[u].x |= v[u].x;
        acc[u].y |= v[u].y;
        acc[u].z |= v[u].z;
        acc[u].w |= v[u].w;
      }
    }
#pragma unroll
    for (int u = 0; u < kPoU; u++) {
      const uint64_t i = i0 + u * blockDim.x;
      if (i < quads) total[i] = acc[u];
    }
  }
}

// P_rank (nullable) and the total only
__global__ void k_prefix_or_rank(const uint32_t* __restrict__ parts, uint32_t nparts, uint64_t words, uint32_t rank,
                                 uint32_t* __restrict__ prefix, uint32_t* __restrict__ total) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += stride) {
    uint32_t acc = 0;
    for (uint32_t k = 0; k < nparts; k++) {
      if (k == rank && prefix) prefix[w] = acc;
      acc |= parts[(uint64_t)k * words + w];
    }
    total[w] = acc;
  }
}

__global__ __launch_bounds__(256) void k_prefix_or_rank4(const uint4* __restrict__ parts, uint32_t nparts,
                                                         uint64_t quads, uint32_t rank, uint4* __restrict__ prefix,
                                                         uint4* __restrict__ total) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * kPoU;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x * kPoU + threadIdx.x; i0 < quads; i0 += stride) {
    uint4 acc[kPoU];
#pragma unroll
    for (int u = 0; u < kPoU; u++) acc[u] = make_uint4(0, 0, 0, 0);
    for (uint32_t k = 0; k < nparts; k++) {
      uint4 v[kPoU];
#pragma unroll
      for (int u = 0; u < kPoU; u++) {
        const uint64_t i = i0 + u * blockDim.x;
        v[u] = i < quads ? parts[(uint64_t)k * quads + i] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kPoU; u++) {
        const uint64_t i = i0 + u * blockDim.x;
        if (k == rank && prefix && i < quads) prefix[i] = acc[u];
        acc[u].x |= v[u].x;
        acc[u].y |= v[u].y;
        acc[u].z |= v[u].z;
        acc[u].w |= v[u].w;
      }
    }
#pragma unroll
    for (int u = 0; u < kPoU; u++) {
      const uint64_t i = i0 + u * blockDim.x;
      if (i < quads) total[i] = acc[u];
    }
  }
}

}  // namespace sg

using namespace sg;

extern "C" {

int sg_shard_of(uint32_t s, uint32_t nshards) {
  if (nshards == 0) return -1;
  s ^= s >> 16;
  s *= 0x85EBCA6Bu;
  s ^= s >> 13;
  s *= 0xC2B2AE35u;
  s ^= s >> 16;
  return (int)(((uint64_t)s * nshards) >> 32);
}

int sg_shard_candidates_dev(sg_ctx* ctx, sg_set* snapshot, const uint32_t* d_vals, const uint64_t* d_rec_off,
                            uint64_t nvals, uint64_t nrec, uint64_t rec_base, uint32_t nshards, uint32_t* d_pairs,
                            uint64_t* d_shard_off) {
  if (!ctx || !snapshot || snapshot->ctx != ctx || !d_rec_off || !d_shard_off || (nvals && (!d_vals || !d_pairs)) ||
      nshards == 0 || nshards > kShardMax || rec_base + nrec > 0xFFFFFFFFull) {
    set_error("sg_shard_candidates_dev: invalid argument");
    return SG_EINVAL;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  ScopedTimer tm(ctx, "shard_local");
  const uint64_t m = ctx->max_launch_recs;
  const uint64_t max_n = nvals < kLaunchEntries ? nvals : kLaunchEntries;
  WsPlan p;
  const size_t o_tmp = p.add(nvals * 8 + 64), o_cnt = p.add(kShardMax * 8 + 8), o_cur = p.add(kShardMax * 8);
  const size_t o_plan = p.total;
  rc = ws_reserve(ctx, o_plan + bucket_plan_bytes(max_n ? max_n : 1, nrec < m ? (nrec ? nrec : 1) : m));
  if (rc) return rc;
  uint2* tmp = (uint2*)ws_at(ctx, o_tmp);
  unsigned long long* cnt = (unsigned long long*)ws_at(ctx, o_cnt);
  unsigned long long* npairs = cnt + kShardMax;
  unsigned long long* cursor = (unsigned long long*)ws_at(ctx, o_cur);
  SG_HIP(hipMemsetAsync(cnt, 0, kShardMax * 8 + 8, ctx->stream));
  const bool single = nrec <= m && nvals < kLaunchEntries;
  if (nvals && single) {
    EmitArgs e{tmp, npairs, (uint32_t)rec_base, nshards, cnt};
    rc = bucket_emit(ctx, snapshot->words, d_vals, d_rec_off, nvals, nrec, e, o_plan);
    if (rc) return rc;
  } else if (nvals) {
    // record slices of <= m records and < 2^30 entries, cut on the device;
    // every slice's rebased offsets side by side (no wait between slices)
    std::vector<uint64_t> cuts;
    rc = record_slice_cuts(ctx, d_rec_off, nrec, kLaunchEntries - 1, cuts);
    if (rc) return rc;
    const size_t ns = cuts.size() / 4, need = nrec + ns;
    for (size_t j = 0; j < ns; j++)
      if (cuts[4 * j + 3] - cuts[4 * j + 2] >= kLaunchEntries) {
        set_error("sg_shard_candidates_dev: a record holds >= 2^30 signal entries");
        return SG_EINVAL;
      }
    if (ctx->slice_off_cap < need) {
      SG_HIP(hipStreamSynchronize(ctx->stream));
      if (ctx->slice_off) SG_HIP(hipFree(ctx->slice_off));
      ctx->slice_off = nullptr;
      ctx->slice_off_cap = 0;
      SG_HIP(hipMalloc(&ctx->slice_off, need * 8));
      ctx->slice_off_cap = need;
    }
    size_t at = 0;
    for (size_t j = 0; j < ns; j++) {
      const uint64_t r0 = cuts[4 * j], r1 = cuts[4 * j + 1], e0 = cuts[4 * j + 2], e1 = cuts[4 * j + 3];
      uint64_t* roff = ctx->slice_off + at;
      at += r1 - r0 + 1;
      if (e1 == e0) continue;
      rc = rebase_offsets(ctx, d_rec_off + r0, r1 - r0 + 1, e0, roff);
      if (rc) return rc;
      EmitArgs e{tmp, npairs, (uint32_t)(rec_base + r0), nshards, cnt};
      rc = bucket_emit(ctx, snapshot->words, d_vals + e0, roff, e1 - e0, r1 - r0, e, o_plan);
      if (rc) return rc;
    }
  }
  hipLaunchKernelGGL(k_shard_offsets, dim3(1), dim3(64), 0, ctx->stream, (const unsigned long long*)cnt, nshards,
                     d_shard_off, cursor);
  if (nvals) {
    ScopedTimer tr(ctx, "shard_route");
    hipLaunchKernelGGL(k_shard_route, dim3(std::min<uint64_t>(div_up(nvals, kRouteThreads * kRoutePer), 8192)),
                       dim3(kRouteThreads), 0, ctx->stream, (const uint2*)tmp, (const unsigned long long*)npairs,
                       nshards, cursor, (uint2*)d_pairs);
  }
  SG_HIP(hipGetLastError());
  return SG_OK;
}

int sg_shard_owners_dev(sg_ctx* ctx, const uint32_t* d_pairs, uint64_t npairs, uint64_t nrec_total,
                        uint32_t* d_rec_bits, uint32_t* d_new_vals, uint64_t* d_nnew) {
  if (!ctx || !d_rec_bits || !d_nnew || (npairs && (!d_pairs || !d_new_vals)) || nrec_total > 0xFFFFFFFFull) {
    set_error("sg_shard_owners_dev: invalid argument");
    return SG_EINVAL;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  SG_HIP(hipMemsetAsync(d_rec_bits, 0, ((nrec_total + 31) / 32) * 4, ctx->stream));
  SG_HIP(hipMemsetAsync(d_nnew, 0, 8, ctx->stream));
  if (npairs == 0) return SG_OK;
  rc = dstage_reserve(ctx, nrec_total + 64);
  if (rc) return rc;
  uint8_t* rec_flag = (uint8_t*)ctx->dstage;
  SG_HIP(hipMemsetAsync(rec_flag, 0, nrec_total, ctx->stream));
  uint32_t key_lo = 0;
  rc = owner_keys(ctx, nrec_total ? nrec_total : 1, &key_lo);
  if (rc) return rc;
  const uint32_t grid = std::min<uint64_t>(div_up(npairs, 256), 16384);
  {
    ScopedTimer tm(ctx, "shard_owner");
    hipLaunchKernelGGL(k_shard_claim, dim3(grid), dim3(256), 0, ctx->stream, (const uint2*)d_pairs, npairs,
                       ctx->owner, key_lo);
  }
  {
    ScopedTimer tm(ctx, "shard_resolve");
    hipLaunchKernelGGL(k_shard_resolve, dim3(std::min<uint64_t>(div_up(npairs, (uint64_t)kResT * kResPer), 4096)),
                       dim3(kResT), 0, ctx->stream, (const uint2*)d_pairs, npairs, (const uint32_t*)ctx->owner, key_lo,
                       rec_flag, d_new_vals, (unsigned long long*)d_nnew);
    hipLaunchKernelGGL(k_pack_flags, dim3(div_up(div_up(nrec_total, 32), 256)), dim3(256), 0, ctx->stream,
                       (const uint8_t*)rec_flag, nrec_total, d_rec_bits);
  }
  SG_HIP(hipGetLastError());
  return SG_OK;
}

int sg_shard_flags_dev(sg_ctx* ctx, const uint32_t* d_bits, uint32_t nparts, uint64_t words_per_part, uint64_t rec_lo,
                       uint64_t nrec, uint8_t* d_rec_new) {
  if (!ctx || (nrec && (!d_bits || !d_rec_new || nparts == 0)) ||
      (nrec && ((rec_lo + nrec + 31) >> 5) - (rec_lo >> 5) > words_per_part)) {
    set_error("sg_shard_flags_dev: invalid argument");
    return SG_EINVAL;
  }
  if (nrec == 0) return SG_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  ScopedTimer tm(ctx, "shard_flags");
  hipLaunchKernelGGL(k_shard_flags, dim3(div_up(nrec, 256)), dim3(256), 0, ctx->stream, d_bits, nparts,
                     words_per_part, rec_lo, nrec, d_rec_new);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

int sg_bitmap_prefix_or_dev(sg_ctx* ctx, const uint32_t* d_parts, uint32_t nparts, uint64_t words, uint32_t* d_prefix,
                            uint32_t* d_total) {
  if (!ctx || nparts == 0 || (words && (!d_parts || !d_prefix || !d_total))) {
    set_error("sg_bitmap_prefix_or_dev: invalid argument");
    return SG_EINVAL;
  }
  if (words == 0) return SG_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  ScopedTimer tm(ctx, "prefix_or");
  if (words % 4 == 0 && (((uintptr_t)d_parts | (uintptr_t)d_prefix | (uintptr_t)d_total) & 15) == 0)
    hipLaunchKernelGGL(k_prefix_or4, dim3((uint32_t)std::min<uint64_t>(div_up(words / 4, 256 * kPoU), 4096)),
                       dim3(256), 0, ctx->stream, (const uint4*)d_parts, nparts, words / 4, (uint4*)d_prefix,
                       (uint4*)d_total);
  else
    hipLaunchKernelGGL(k_prefix_or, dim3(std::min<uint64_t>(div_up(words, 256), 16384)), dim3(256), 0, ctx->stream,
                       d_parts, nparts, words, d_prefix, d_total);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

int sg_bitmap_prefix_or_rank_dev(sg_ctx* ctx, const uint32_t* d_parts, uint32_t nparts, uint64_t words, uint32_t rank,
                                 uint32_t* d_prefix, uint32_t* d_total) {
  if (!ctx || nparts == 0 || rank >= nparts || (words && (!d_parts || !d_total))) {
    set_error("sg_bitmap_prefix_or_rank_dev: invalid argument");
    return SG_EINVAL;
  }
  if (words == 0) return SG_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  ScopedTimer tm(ctx, "prefix_or");
  if (words % 4 == 0 && (((uintptr_t)d_parts | (uintptr_t)d_prefix | (uintptr_t)d_total) & 15) == 0)
    hipLaunchKernelGGL(k_prefix_or_rank4, dim3((uint32_t)std::min<uint64_t>(div_up(words / 4, 256 * kPoU), 4096)),
                       dim3(256), 0, ctx->stream, (const uint4*)d_parts, nparts, words / 4, rank,
                       rank ? (uint4*)d_prefix : nullptr, (uint4*)d_total);
  else
    hipLaunchKernelGGL(k_prefix_or_rank, dim3(std::min<uint64_t>(div_up(words, 256), 16384)), dim3(256), 0,
                       ctx->stream, d_parts, nparts, words, rank, rank ? d_prefix : nullptr, d_total);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

int sg_prefix_begin_dev(sg_ctx* ctx, uint32_t slot, sg_set* base, sg_set* marks, const uint32_t* d_vals,
                        const uint64_t* d_rec_off, uint64_t nvals, uint64_t nrec) {
  if (!ctx || !base || !marks || base == marks || base->ctx != ctx || marks->ctx != ctx || !d_rec_off ||
      (nvals && !d_vals)) {
    set_error("sg_prefix_begin_dev: invalid argument");
    return SG_EINVAL;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  return prefix_begin(ctx, slot, base->words, marks->words, d_vals, d_rec_off, nvals, nrec);
}

int sg_prefix_begin_form_dev(sg_ctx* ctx, uint32_t slot, uint32_t form, sg_set* base, sg_set* marks,
                             const uint32_t* d_vals, const uint64_t* d_rec_off, uint64_t nvals, uint64_t nrec,
                             uint64_t* d_ncand) {
  const bool sets = form != 2;  // form 2 (partitions only) reads neither set
  if (!ctx || form > 2 || !d_rec_off || (nvals && !d_vals) ||
      (sets && (!base || !marks || base == marks || base->ctx != ctx || marks->ctx != ctx)) ||
      (!sets && (base || marks || d_ncand))) {
    set_error("sg_prefix_begin_form_dev: invalid argument");
    return SG_EINVAL;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  return prefix_begin(ctx, slot, sets ? base->words : nullptr, sets ? marks->words : nullptr, d_vals, d_rec_off, nvals,
                      nrec, (int)form, d_ncand);
}

int sg_prefix_end_dev(sg_ctx* ctx, uint32_t slot, sg_set* maxsig, const uint32_t* d_prefix, sg_set* newsig,
                      uint8_t* d_rec_new) {
  if (!ctx || !maxsig || maxsig->ctx != ctx || (newsig && newsig->ctx != ctx)) {
    set_error("sg_prefix_end_dev: invalid argument");
    return SG_EINVAL;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  if (slot < kPrefixSlots && ctx->prefix[slot].nrec && !d_rec_new) {
    set_error("sg_prefix_end_dev: no flag buffer");
    return SG_EINVAL;
  }
  return prefix_end(ctx, slot, maxsig->words, d_prefix, newsig ? newsig->words : nullptr, d_rec_new, true);
}

int sg_prefix_flags_dev(sg_ctx* ctx, uint32_t slot, sg_set* maxsig, const uint32_t* d_prefix,
                        uint8_t* d_rec_new) {
  if (!ctx || !maxsig || maxsig->ctx != ctx) {
    set_error("sg_prefix_flags_dev: invalid argument");
    return SG_EINVAL;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  if (slot < kPrefixSlots && ctx->prefix[slot].nrec && !d_rec_new) {
    set_error("sg_prefix_flags_dev: no flag buffer");
    return SG_EINVAL;
  }
  return prefix_end(ctx, slot, maxsig->words, d_prefix, nullptr, d_rec_new, false);
}

int sg_set_add_dev(sg_set* set, const uint32_t* d_vals, uint64_t n) {
  if (!set || (n && !d_vals)) return SG_EINVAL;
  if (n == 0) return SG_OK;
  sg_ctx* ctx = set->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  ScopedTimer tm(ctx, "set_add");
  hipLaunchKernelGGL(k_set_add_vals, dim3(std::min<uint64_t>(div_up(n, 256), 16384)), dim3(256), 0, ctx->stream,
                     set->words, d_vals, n);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

int sg_set_add_new_dev(sg_set* newsig, sg_set* maxsig, const uint32_t* d_vals, uint64_t n) {
  if (!maxsig || (n && !d_vals) || (newsig && (newsig->ctx != maxsig->ctx || newsig == maxsig))) {
    set_error("sg_set_add_new_dev: invalid argument");
    return SG_EINVAL;
  }
  if (n == 0) return SG_OK;
  sg_ctx* ctx = maxsig->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  ScopedTimer tm(ctx, "set_add");
  hipLaunchKernelGGL(k_set_add_new_vals, dim3(std::min<uint64_t>(div_up(n, 256), 16384)), dim3(256), 0, ctx->stream,
                     newsig ? newsig->words : nullptr, maxsig->words, d_vals, n);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

int sg_set_del_dev(sg_set* set, const uint32_t* d_vals, uint64_t n) {
  if (!set || (n && !d_vals)) return SG_EINVAL;
  if (n == 0) return SG_OK;
  sg_ctx* ctx = set->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  ScopedTimer tm(ctx, "set_add");
  hipLaunchKernelGGL(k_set_del_vals, dim3(std::min<uint64_t>(div_up(n, 256), 16384)), dim3(256), 0, ctx->stream,
                     set->words, d_vals, n);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

int sg_prefix_cands_dev(sg_ctx* ctx, uint32_t slot, uint32_t* d_out, uint64_t cap) {
  if (!ctx || slot >= kPrefixSlots || (cap && !d_out)) {
    set_error("sg_prefix_cands_dev: invalid argument");
    return SG_EINVAL;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  const PrefixSlot& S = ctx->prefix[slot];
  if (!S.open || S.keep) {
    set_error("sg_prefix_cands_dev: slot %u holds no pairs-form batch", slot);
    return SG_EINVAL;
  }
  if (!cap || !S.n) return SG_OK;
  hipLaunchKernelGGL(k_pair_sigs, dim3(std::min<uint64_t>(div_up(cap, 256), 8192)), dim3(256), 0, ctx->stream,
                     (const uint2*)((char*)S.ws + 256), (const unsigned long long*)S.ws, cap, d_out);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

}  // extern "C"
