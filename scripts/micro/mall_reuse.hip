// Microbenchmark: which second touches of a region come from a cache?
//  (1) read→read: a streaming read of R, then the same read again (MALL reuse
//      of a read; r02).
//  (2) read→copy: a copy of R right after a read of its source (r02).
//  (3) write→read: a kernel writes R, a second kernel on the same stream reads
//      it back, against a cold read of R (r04: would a pass-2 → bucket ring in
//      the MALL keep pass 2's output off HBM?).
//  (4) one XCD: the same write→read with every working workgroup on XCD 0
//      (workgroup i runs on XCD i % 8; the others exit at once), against a
//      cold read on XCD 0 -- the L2 (4 MB per XCD) as the ring.
// Each timed with events; rates in GB/s of the bytes the timed kernel moves.
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

// xcd_only: 0 = every workgroup works; 1 = only workgroups of XCD 0
__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ p, uint64_t n, uint32_t* __restrict__ sink,
                                              int xcd_only) {
  uint32_t acc = 0;
  uint64_t b = blockIdx.x, nb = gridDim.x;
  if (xcd_only) {
    if (b & 7) return;
    b >>= 3;
    nb >>= 3;
  }
  const uint64_t S = nb * blockDim.x * 4;
  for (uint64_t i = b * blockDim.x * 4 + threadIdx.x; i < n; i += S) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = i + u * blockDim.x < n ? p[i + u * blockDim.x] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 4; u++) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_write(uint4* __restrict__ p, uint64_t n, uint32_t seed, int xcd_only) {
  uint64_t b = blockIdx.x, nb = gridDim.x;
  if (xcd_only) {
    if (b & 7) return;
    b >>= 3;
    nb >>= 3;
  }
  const uint64_t S = nb * blockDim.x;
  for (uint64_t i = b * blockDim.x + threadIdx.x; i < n; i += S)
    p[i] = make_uint4((uint32_t)i ^ seed, (uint32_t)(i * 3), (uint32_t)(i * 7), seed);
}

__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ p, uint64_t n, uint4* __restrict__ q) {
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += S) q[i] = p[i];
}

static hipEvent_t e[4];

static float span(int a, int b) {
  float t = 0;
  hipEventElapsedTime(&t, e[a], e[b]);
  return t;
}

int main() {
  const uint64_t kMax = 4ull << 30;  // bytes per buffer
  uint4 *a, *b;
  uint32_t* sink;
  CK(hipMalloc(&a, kMax));
  CK(hipMalloc(&b, kMax));
  CK(hipMalloc(&sink, 4));
  k_write<<<4096, 256>>>(a, kMax / 16, 1, 0);
  k_write<<<4096, 256>>>(b, kMax / 16, 2, 0);
  CK(hipDeviceSynchronize());
  for (auto& x : e) CK(hipEventCreate(&x));
  const int grid = 256 * 8;
  const int reps = 8;
  auto flush = [&]() { k_read<<<grid, 256>>>(b, kMax / 16, sink, 0); };

  printf("# (1)-(3) whole chip; GB/s of the timed kernel's bytes (a copy counts read + write)\n");
  printf("%8s %10s %10s %10s %10s %10s %10s\n", "MiB", "read cold", "read→read", "copy cold", "read→copy", "write",
         "write→read");
  const uint64_t sizes[] = {8ull << 20,   16ull << 20,  32ull << 20,  64ull << 20, 128ull << 20,
                            192ull << 20, 256ull << 20, 512ull << 20, 2ull << 30};
  for (uint64_t R : sizes) {
    const uint64_t n = R / 16;
    double r1 = 0, r2 = 0, c1 = 0, c2 = 0, w = 0, wr = 0;
    for (int rep = 0; rep < reps; rep++) {
      uint4* base = a + (rep % 4) * (R < (1ull << 30) ? R / 16 : 0);
      flush();
      CK(hipEventRecord(e[0]));
      k_read<<<grid, 256>>>(base, n, sink, 0);
      CK(hipEventRecord(e[1]));
      k_read<<<grid, 256>>>(base, n, sink, 0);
      CK(hipEventRecord(e[2]));
      CK(hipEventSynchronize(e[2]));
      const float t1 = span(0, 1), t2 = span(1, 2);
      flush();
      CK(hipEventRecord(e[0]));
      k_copy<<<grid, 256>>>(base, n, b + (kMax / 16) / 2);
      CK(hipEventRecord(e[1]));
      flush();
      k_read<<<grid, 256>>>(base, n, sink, 0);
      CK(hipEventRecord(e[2]));
      k_copy<<<grid, 256>>>(base, n, b + (kMax / 16) / 2);
      CK(hipEventRecord(e[3]));
      CK(hipEventSynchronize(e[3]));
      const float t3 = span(0, 1), t4 = span(2, 3);
      flush();
      CK(hipEventRecord(e[0]));
      k_write<<<grid, 256>>>(base, n, 7u + rep, 0);
      CK(hipEventRecord(e[1]));
      k_read<<<grid, 256>>>(base, n, sink, 0);
      CK(hipEventRecord(e[2]));
      CK(hipEventSynchronize(e[2]));
      const float t5 = span(0, 1), t6 = span(1, 2);
      if (rep) {  // the first rep warms up
        r1 += R / (t1 * 1e-3) / 1e9;
        r2 += R / (t2 * 1e-3) / 1e9;
        c1 += 2.0 * R / (t3 * 1e-3) / 1e9;
        c2 += 2.0 * R / (t4 * 1e-3) / 1e9;
        w += R / (t5 * 1e-3) / 1e9;
        wr += R / (t6 * 1e-3) / 1e9;
      }
    }
    const double k = 1.0 / (reps - 1);
    printf("%8llu %10.0f %10.0f %10.0f %10.0f %10.0f %10.0f\n", (unsigned long long)(R >> 20), r1 * k, r2 * k, c1 * k,
           c2 * k, w * k, wr * k);
  }

  // launch + event overhead of one kernel, subtracted in (4) where regions are small
  double ovh = 0;
  for (int rep = 0; rep < reps; rep++) {
    CK(hipEventRecord(e[0]));
    k_read<<<grid, 256>>>(a, 0, sink, 1);
    CK(hipEventRecord(e[1]));
    CK(hipEventSynchronize(e[1]));
    if (rep) ovh += span(0, 1) / (reps - 1);
  }
  printf("# (4) XCD 0 only (grid %d, %d working workgroups); GB/s after %.1f us of launch overhead\n", grid,
         grid / 8, ovh * 1e3);
  printf("%8s %10s %10s %10s\n", "MiB", "read cold", "write", "write→read");
  const uint64_t xs[] = {1ull << 20, 2ull << 20, 3ull << 20, 4ull << 20, 8ull << 20, 16ull << 20, 64ull << 20};
  for (uint64_t R : xs) {
    const uint64_t n = R / 16;
    double r1 = 0, w = 0, wr = 0;
    for (int rep = 0; rep < reps; rep++) {
      uint4* base = a + (rep % 4) * (R / 16);
      flush();
      CK(hipEventRecord(e[0]));
      k_read<<<grid, 256>>>(base, n, sink, 1);
      CK(hipEventRecord(e[1]));
      flush();
      CK(hipEventRecord(e[2]));
      k_write<<<grid, 256>>>(base, n, 11u + rep, 1);
      CK(hipEventRecord(e[3]));
      CK(hipEventSynchronize(e[3]));
      const float t1 = span(0, 1) - ovh, t2 = span(2, 3) - ovh;
      CK(hipEventRecord(e[0]));
      k_read<<<grid, 256>>>(base, n, sink, 1);
      CK(hipEventRecord(e[1]));
      CK(hipEventSynchronize(e[1]));
      const float t3 = span(0, 1) - ovh;
      if (rep) {
        r1 += R / (t1 * 1e-3) / 1e9;
        w += R / (t2 * 1e-3) / 1e9;
        wr += R / (t3 * 1e-3) / 1e9;
      }
    }
    const double k = 1.0 / (reps - 1);
    printf("%8llu %10.0f %10.0f %10.0f\n", (unsigned long long)(R >> 20), r1 * k, w * k, wr * k);
  }
  return 0;
}
