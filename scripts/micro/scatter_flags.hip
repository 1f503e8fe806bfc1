// Microbenchmark: scattered byte stores of record flags (208M stores into a
// 1 MiB flag array, the C2 owner count), from a coalesced owner log.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_fill(uint32_t* log, uint64_t n, uint32_t nrec) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    uint32_t x = (uint32_t)i * 0x9E3779B1u;
    x ^= x >> 15;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    log[i] = x % nrec;
  }
}

template <int kU>
__global__ __launch_bounds__(256) void k_flags(const uint32_t* __restrict__ log, uint64_t n, uint8_t* __restrict__ f) {
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x * kU;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * kU; i < n; i += S) {
    if (kU == 4) {
      const uint4 q = *reinterpret_cast<const uint4*>(log + i);
      f[q.x] = 1;
      f[q.y] = 1;
      f[q.z] = 1;
      f[q.w] = 1;
    } else {
      f[log[i]] = 1;
    }
  }
}

int main() {
  const uint64_t n = 208u << 20;
  const uint32_t nrec = 1 << 20;
  uint32_t* log;
  uint8_t* f;
  (void)hipMalloc(&log, n * 4);
  (void)hipMalloc(&f, nrec);
  k_fill<<<(n + 255) / 256, 256>>>(log, n, nrec);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int rep = 0; rep < 3; rep++) {
    (void)hipMemset(f, 0, nrec);
    (void)hipEventRecord(a);
    k_flags<4><<<4096, 256>>>(log, n, f);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("uint4 log reads, 4 byte stores per lane: %.3f ms for %llu stores\n", ms, (unsigned long long)n);
    (void)hipMemset(f, 0, nrec);
    (void)hipEventRecord(a);
    k_flags<1><<<8192, 256>>>(log, n, f);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    printf("dword log reads, 1 byte store per lane: %.3f ms\n", ms);
  }
  return 0;
}
