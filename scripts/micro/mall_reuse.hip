// Microbenchmark: does a second read of a region that was just streamed come
// from the MALL (infinity cache)?  For region sizes R: a streaming read of R
// (a histogram pass stands for it), then either the same read again or a copy
// of R into a second buffer (a scatter pass stands for it), each timed with
// events.  Tells whether running the pass-1 histogram and scatter unit by unit
// (each unit re-read while cached) could take the scatter's read off HBM.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ p, uint64_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += S) {
    const uint4 v = p[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ p, uint64_t n, uint4* __restrict__ q) {
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += S) q[i] = p[i];
}

__global__ void k_fill(uint4* p, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = make_uint4((uint32_t)i, (uint32_t)(i * 3), (uint32_t)(i * 7), 1u);
}

int main() {
  const uint64_t kMax = 4ull << 30;  // bytes per buffer
  uint4 *a, *b;
  uint32_t* sink;
  CK(hipMalloc(&a, kMax));
  CK(hipMalloc(&b, kMax));
  CK(hipMalloc(&sink, 4));
  k_fill<<<(kMax / 16 + 255) / 256, 256>>>(a, kMax / 16);
  k_fill<<<(kMax / 16 + 255) / 256, 256>>>(b, kMax / 16);
  CK(hipDeviceSynchronize());
  hipEvent_t e[4];
  for (auto& x : e) CK(hipEventCreate(&x));
  const int grid = 256 * 8;
  const uint64_t sizes[] = {32ull << 20, 64ull << 20, 128ull << 20, 192ull << 20, 256ull << 20, 512ull << 20,
                            2ull << 30};
  printf("%10s %12s %12s %12s %12s\n", "MiB", "read1 GB/s", "read2 GB/s", "copy cold", "copy warm");
  for (uint64_t R : sizes) {
    const uint64_t n = R / 16;
    double r1 = 0, r2 = 0, r3 = 0, cp = 0;
    const int reps = 8;
    for (int rep = 0; rep < reps; rep++) {
      // flush: stream an unrelated 4 GiB region first
      k_read<<<grid, 256>>>(b, kMax / 16, sink);
      uint4* base = a + (rep % 4) * (R < (1ull << 30) ? R / 16 : 0);
      CK(hipEventRecord(e[0]));
      k_read<<<grid, 256>>>(base, n, sink);
      CK(hipEventRecord(e[1]));
      k_read<<<grid, 256>>>(base, n, sink);
      CK(hipEventRecord(e[2]));
      CK(hipEventSynchronize(e[2]));
      float t1, t2;
      CK(hipEventElapsedTime(&t1, e[0], e[1]));
      CK(hipEventElapsedTime(&t2, e[1], e[2]));
      // a copy of the region cold, then one right after a read of it
      k_read<<<grid, 256>>>(b, kMax / 16, sink);
      CK(hipEventRecord(e[0]));
      k_copy<<<grid, 256>>>(base, n, b + (kMax / 16) / 2);
      CK(hipEventRecord(e[1]));
      k_read<<<grid, 256>>>(b, kMax / 16, sink);
      k_read<<<grid, 256>>>(base, n, sink);
      CK(hipEventRecord(e[2]));
      k_copy<<<grid, 256>>>(base, n, b + (kMax / 16) / 2);
      CK(hipEventRecord(e[3]));
      CK(hipEventSynchronize(e[3]));
      float t3, t4;
      CK(hipEventElapsedTime(&t3, e[0], e[1]));
      CK(hipEventElapsedTime(&t4, e[2], e[3]));
      if (rep) {  // first rep warms up
        r1 += R / (t1 * 1e-3) / 1e9;
        r2 += R / (t2 * 1e-3) / 1e9;
        r3 += 2.0 * R / (t3 * 1e-3) / 1e9;
        cp += 2.0 * R / (t4 * 1e-3) / 1e9;
      }
    }
    printf("%10llu %12.0f %12.0f %12.0f %12.0f\n", (unsigned long long)(R >> 20), r1 / (reps - 1), r2 / (reps - 1),
           r3 / (reps - 1), cp / (reps - 1));
  }
  return 0;
}
