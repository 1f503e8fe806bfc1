// Microbenchmark: global u32 atomicMin throughput at random addresses -- the
// access of a first-owner table (Minimize's k_min_claim, and round 4's
// claim path for the triage: a relaxed load, then atomicMin if it lowers the
// owner; 4 B per signal, 2^32 entries = 16 GiB).  Forms: no-return atomicMin, returning atomicMin, and the
// read-checked form (load, then atomicMin when larger) on a table whose
// entries are all larger (every check passes: the claim path's worst case).
// Tables of 256 MiB, 4 GiB and 16 GiB; 256M atomics per launch.  Rates in
// G atomics/s, the empirical peak the claim kernels are set against.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// mode 0: no return; 1: returning (result summed into a sink); 2: read-checked
template <int kMode>
__global__ __launch_bounds__(256) void k_atomics(uint32_t* __restrict__ t, uint64_t mask, uint64_t n, uint32_t seed,
                                                 uint32_t* __restrict__ sink) {
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += S) {
    const uint64_t h = mix64(i * 0x9E3779B97F4A7C15ull + seed);
    uint32_t* p = t + (h & mask);
    const uint32_t key = (uint32_t)(h >> 40);
    if (kMode == 0) {
      atomicMin(p, key);
    } else if (kMode == 1) {
      acc += atomicMin(p, key);
    } else {
      if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > key) atomicMin(p, key);
    }
  }
  if (kMode == 1 && acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const uint64_t kMaxBytes = 16ull << 30;
  uint32_t* t = nullptr;
  uint32_t* sink = nullptr;
  CK(hipMalloc(&t, kMaxBytes));
  CK(hipMalloc(&sink, 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const uint64_t n = 256ull << 20;
  const int grid = 256 * 32;
  printf("%10s %14s %14s %14s  (G atomics/s, %llu per launch, random addresses)\n", "table", "no-return",
         "returning", "read-checked", (unsigned long long)n);
  for (uint64_t bytes : {256ull << 20, 4ull << 30, 16ull << 30}) {
    const uint64_t mask = bytes / 4 - 1;
    double r[3] = {0, 0, 0};
    for (int mode = 0; mode < 3; mode++) {
      for (int rep = 0; rep < 3; rep++) {
        CK(hipMemset(t, 0xFF, bytes));  // every entry larger than every key
        CK(hipEventRecord(a));
        if (mode == 0) k_atomics<0><<<grid, 256>>>(t, mask, n, 17u + rep, sink);
        if (mode == 1) k_atomics<1><<<grid, 256>>>(t, mask, n, 17u + rep, sink);
        if (mode == 2) k_atomics<2><<<grid, 256>>>(t, mask, n, 17u + rep, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        const double rate = n / (ms * 1e-3) / 1e9;
        if (rate > r[mode]) r[mode] = rate;
      }
    }
    printf("%7llu MiB %14.1f %14.1f %14.1f\n", (unsigned long long)(bytes >> 20), r[0], r[1], r[2]);
  }
  return 0;
}
