// Microbenchmark for an exact M0 pre-filter (round-5 review, item 1): random
// 16-B bucket probes of a compact hash table of maxSignal's signals (full
// 32-bit values, 4 slots per bucket, empty = 0), driven by a batch's entry
// stream read with non-temporal loads.  Built as a shared object and driven by
// m0_filter.py (device pointers from torch, torch's stream).
//
// Variants (mf_probe `mode`):
//   0  stream only: read every entry, count the non-zero ones (the read floor)
//   1  one table: every entry probes its bucket
//   2  hot table first (a small table of the batch's most frequent signals,
//      meant to stay in each XCD's L2), the big table only on a hot miss
//   3  as 1, but the bucket of a value is chosen by its low bits (no hash)
#include <hip/hip_runtime.h>
#include <cstdint>

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__global__ void k_build(uint32_t* __restrict__ tab, uint32_t bmask, const uint32_t* __restrict__ v, uint64_t n,
                        unsigned long long* __restrict__ dropped) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = v[i];
  if (s == 0) return;
  uint32_t* b = tab + 4ull * (mix32(s) & bmask);
  for (int j = 0; j < 4; j++) {
    const uint32_t old = atomicCAS(b + j, 0u, s);
    if (old == 0u || old == s) return;
  }
  atomicAdd(dropped, 1ull);
}

__device__ __forceinline__ bool in_bucket(uint4 t, uint32_t s) {
  return s != 0u && (t.x == s || t.y == s || t.z == s || t.w == s);
}

template <int kMode>
__global__ __launch_bounds__(256) void k_probe(const uint4* __restrict__ v, uint64_t nq,
                                               const uint4* __restrict__ tab, uint32_t bmask,
                                               const uint4* __restrict__ hot, uint32_t hmask,
                                               unsigned long long* __restrict__ hits) {
  constexpr int U = 2;  // quads per thread per iteration: 8 probes in flight
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * U;
  uint32_t cnt = 0;
  for (uint64_t q0 = ((uint64_t)blockIdx.x * blockDim.x) * U + threadIdx.x; q0 < nq; q0 += stride) {
    uint32_t s[4 * U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t q = q0 + (uint64_t)u * blockDim.x;
      uint4 x = make_uint4(0, 0, 0, 0);
      if (q < nq) {
        const v4u32 y = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(v + q));
        x = make_uint4(y.x, y.y, y.z, y.w);
      }
      s[4 * u + 0] = x.x;
      s[4 * u + 1] = x.y;
      s[4 * u + 2] = x.z;
      s[4 * u + 3] = x.w;
    }
    if (kMode == 0) {
#pragma unroll
      for (int k = 0; k < 4 * U; k++) cnt += s[k] != 0u;
    } else if (kMode == 1 || kMode == 3) {
      uint4 t[4 * U];
#pragma unroll
      for (int k = 0; k < 4 * U; k++) t[k] = tab[(kMode == 1 ? mix32(s[k]) : s[k]) & bmask];
#pragma unroll
      for (int k = 0; k < 4 * U; k++) cnt += in_bucket(t[k], s[k]);
    } else {
      uint4 t[4 * U];
#pragma unroll
      for (int k = 0; k < 4 * U; k++) t[k] = hot[mix32(s[k]) & hmask];
      bool h[4 * U];
#pragma unroll
      for (int k = 0; k < 4 * U; k++) h[k] = in_bucket(t[k], s[k]);
#pragma unroll
      for (int k = 0; k < 4 * U; k++)
        if (!h[k]) t[k] = tab[mix32(s[k]) & bmask];
#pragma unroll
      for (int k = 0; k < 4 * U; k++) cnt += h[k] || in_bucket(t[k], s[k]);
    }
  }
  // wave reduce, one atomic per wave
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(hits, (unsigned long long)cnt);
}

extern "C" int mf_build(void* tab, uint32_t log2_buckets, const void* vals, uint64_t n, void* dropped,
                        void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_build, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (uint32_t*)tab,
                     (1u << log2_buckets) - 1u, (const uint32_t*)vals, n, (unsigned long long*)dropped);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int mf_probe(int mode, const void* vals, uint64_t n, const void* tab, uint32_t log2_buckets,
                        const void* hot, uint32_t log2_hot, void* hits, int blocks, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const uint64_t nq = n / 4;
  const uint32_t bm = (1u << log2_buckets) - 1u, hm = (1u << log2_hot) - 1u;
  const dim3 g(blocks), b(256);
  const uint4* v = (const uint4*)vals;
  switch (mode) {
    case 0:
      hipLaunchKernelGGL(k_probe<0>, g, b, 0, st, v, nq, (const uint4*)tab, bm, (const uint4*)hot, hm,
                         (unsigned long long*)hits);
      break;
    case 1:
      hipLaunchKernelGGL(k_probe<1>, g, b, 0, st, v, nq, (const uint4*)tab, bm, (const uint4*)hot, hm,
                         (unsigned long long*)hits);
      break;
    case 2:
      hipLaunchKernelGGL(k_probe<2>, g, b, 0, st, v, nq, (const uint4*)tab, bm, (const uint4*)hot, hm,
                         (unsigned long long*)hits);
      break;
    case 3:
      hipLaunchKernelGGL(k_probe<3>, g, b, 0, st, v, nq, (const uint4*)tab, bm, (const uint4*)hot, hm,
                         (unsigned long long*)hits);
      break;
    default:
      return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
