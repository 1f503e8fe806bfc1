// Microbenchmark: scattered byte stores of record flags (208M stores into a
// 1 MiB flag array, the C2 owner count), from a coalesced owner log; and
// (r06, the round-5 review's item 2) the same flags set only where a read of
// the flag -- or of a 128 KiB bitmap of the records -- finds it clear: every
// store after a record's first is redundant.
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

// kMode 0: read the flag byte, store where it is 0; 1: read the flag byte only
// (sum, no store); 2: read a word of a 128 KiB record bitmap, where the bit is
// clear store the flag byte and OR the bit (atomicOr, rare)
template <int kMode>
__global__ __launch_bounds__(256) void k_check(const uint32_t* __restrict__ log, uint64_t n, uint8_t* __restrict__ f,
                                               uint32_t* __restrict__ bits, uint32_t* __restrict__ sink) {
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x * 4;
  uint32_t acc = 0;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += S) {
    const uint4 q = *reinterpret_cast<const uint4*>(log + i);
    const uint32_t r[4] = {q.x, q.y, q.z, q.w};
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = kMode == 2 ? bits[r[k] >> 5] : f[r[k]];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (kMode == 0 && v[k] == 0) f[r[k]] = 1;
      if (kMode == 1) acc += v[k];
      if (kMode == 2 && !((v[k] >> (r[k] & 31)) & 1u)) {
        f[r[k]] = 1;
        atomicOr(bits + (r[k] >> 5), 1u << (r[k] & 31));
      }
    }
  }
  if (kMode == 1 && acc == 0xFFFFFFFFu) *sink = acc;
}

int main() {
  const uint64_t n = 208u << 20;
  const uint32_t nrec = 1 << 20;
  uint32_t* log;
  uint8_t* f;
  uint32_t *bits, *sink;
  (void)hipMalloc(&log, n * 4);
  (void)hipMalloc(&f, nrec);
  (void)hipMalloc(&bits, nrec / 8);
  (void)hipMalloc(&sink, 4);
  k_fill<<<(n + 255) / 256, 256>>>(log, n, nrec);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float ms = 0;
  auto timed = [&](const char* what, auto launch) {
    (void)hipMemset(f, 0, nrec);
    (void)hipMemset(bits, 0, nrec / 8);
    (void)hipEventRecord(a);
    launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    printf("%-72s %.3f ms\n", what, ms);
  };
  for (int rep = 0; rep < 3; rep++) {
    timed("uint4 log reads, 4 byte stores per lane", [&] { k_flags<4><<<4096, 256>>>(log, n, f); });
    timed("dword log reads, 1 byte store per lane", [&] { k_flags<1><<<8192, 256>>>(log, n, f); });
    timed("flag byte read, store where 0", [&] { k_check<0><<<4096, 256>>>(log, n, f, bits, sink); });
    timed("flag byte read only", [&] { k_check<1><<<4096, 256>>>(log, n, f, bits, sink); });
    timed("128 KiB bitmap word read, byte store + atomicOr where clear",
          [&] { k_check<2><<<4096, 256>>>(log, n, f, bits, sink); });
  }
  return 0;
}
