// Microbenchmark: do exec-masked-off lanes of a scattered byte store cost
// anything?  The bucket kernel's flush stores one record flag per occupied map
// slot (about 40 % of a thread's slots), as predicated stores.  Same number of
// active stores (208M into a 1 MiB flag array) issued (A) with every lane
// active, (B) with each lane active with probability 40 % (2.5x the
// instructions), (C) as (B) but compacted in registers across slots with
// ds_permute before the store, every store instruction full but the last.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint32_t hsh(uint64_t i) {
  uint32_t x = (uint32_t)i * 0x9E3779B1u ^ (uint32_t)(i >> 32);
  x ^= x >> 15;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  return x ^ (x >> 16);
}

// slots per thread, as the flush's 16
constexpr int kSlots = 16;

template <int kMode>
__global__ __launch_bounds__(256) void k_store(uint64_t nslots, uint32_t pct, uint32_t nrec, uint8_t* __restrict__ f) {
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x * kSlots;
  const int lane = threadIdx.x & 63;
  for (uint64_t base = ((uint64_t)blockIdx.x * blockDim.x) * kSlots + threadIdx.x; base < nslots; base += S) {
    uint32_t pend = 0, npend = 0;  // (C): compacted records in lanes 0..npend-1
#pragma unroll
    for (int k = 0; k < kSlots; k++) {
      const uint64_t i = base + (uint64_t)k * blockDim.x;
      const uint32_t h = hsh(i);
      const bool act = i < nslots && (h % 100u) < pct;
      const uint32_t rec = (h >> 7) % nrec;
      if (kMode != 2) {
        if (act) f[rec] = 1;
      } else {
        const uint64_t m = __ballot(act);
        const uint32_t n = (uint32_t)__popcll(m);
        const uint32_t r = (uint32_t)__popcll(m & ((1ull << lane) - 1));  // rank among the active lanes
        // active lane with rank r goes to lane (npend + r) mod 64, the inactive
        // ones to the lanes after (a permutation: no two lanes collide)
        const uint32_t dst = (act ? npend + r : npend + n + ((uint32_t)lane - r)) & 63;
        const uint32_t moved = (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)rec);  // push to lane dst
        const bool land_lo = (uint32_t)lane >= npend && (uint32_t)lane < npend + n;       // no wrap
        const bool land_hi = npend + n > 64 && (uint32_t)lane < npend + n - 64;           // wrapped
        if (npend + n >= 64) {
          // lanes >= npend of this step complete a full wave with pend
          const uint32_t full = (uint32_t)lane < npend ? pend : moved;
          f[full] = 1;
          pend = land_hi ? moved : 0u;
          npend = npend + n - 64;
        } else {
          if (land_lo) pend = moved;
          npend += n;
        }
      }
    }
    if (kMode == 2 && (uint32_t)lane < npend) f[pend] = 1;
  }
}

int main() {
  const uint32_t nrec = 1 << 20;
  const uint64_t nstores = 208ull << 20;
  uint8_t* f;
  (void)hipMalloc(&f, nrec);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int rep = 0; rep < 3; rep++) {
    for (int mode = 0; mode < 3; mode++) {
      const uint32_t pct = mode == 0 ? 100u : 40u;
      const uint64_t nslots = nstores * 100 / pct;
      (void)hipMemset(f, 0, nrec);
      (void)hipEventRecord(a);
      if (mode == 0) k_store<0><<<4096, 256>>>(nslots, pct, nrec, f);
      if (mode == 1) k_store<1><<<4096, 256>>>(nslots, pct, nrec, f);
      if (mode == 2) k_store<2><<<4096, 256>>>(nslots, pct, nrec, f);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      printf("%s: %.3f ms for ~%llu active stores (%llu slots)\n",
             mode == 0 ? "(A) all lanes active" : mode == 1 ? "(B) 40%% active, predicated" : "(C) 40%% active, compacted",
             ms, (unsigned long long)nstores, (unsigned long long)nslots);
    }
  }
  return 0;
}
