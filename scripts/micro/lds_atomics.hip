// Microbenchmark: LDS atomic / read throughput per CU on gfx950 (random
// addresses in a 32 KiB table, 512-thread blocks, 3 blocks per CU).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int kOp>
__global__ __launch_bounds__(512) void k_lds(uint32_t* out, int iters, uint32_t seed) {
  __shared__ uint32_t t[8192];
  for (int i = threadIdx.x; i < 8192; i += 512) t[i] = 0xFFFFFFFFu;
  __syncthreads();
  uint32_t x = seed ^ (blockIdx.x * 512 + threadIdx.x) * 0x9E3779B9u;
  uint32_t acc = 0;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      x = x * 1664525u + 1013904223u;
      const uint32_t a = (x >> 13) & 8191u;
      if (kOp == 0) acc += t[a];                                   // ds_read_b32
      if (kOp == 1) acc += atomicCAS(&t[a], 0xFFFFFFFFu, x);       // ds_cmpst_rtn_b32
      if (kOp == 2) atomicMin(&t[a], x);                           // ds_min_u32 (no rtn)
      if (kOp == 3) atomicOr(&t[a], x);                            // ds_or_b32
      if (kOp == 4) acc += atomicAdd(&t[a], 1u);                   // ds_add_rtn_u32
      if (kOp == 5) acc += atomicMin(&t[a], x);                    // ds_min_rtn_u32
      if (kOp == 6) t[a] = x;                                      // ds_write_b32
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = acc + t[x & 8191];
}

template <int kOp>
static void run(const char* name, uint32_t* d, int grid) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 2000;
  k_lds<kOp><<<grid, 512>>>(d, 10, 1);
  hipEventRecord(a);
  k_lds<kOp><<<grid, 512>>>(d, iters, 2);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double ops = (double)grid * 512 * iters * 4;
  const double clk = ms * 1e-3 * 2.4e9 * 256;  // CU-cycles
  printf("%-16s %8.3f ms  %.3f CU-cycles per lane-op  (%.2f lane-ops/clk/CU)\n", name, ms, clk / ops, ops / clk);
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 1 << 20);
  const int grid = 256 * 3;
  run<0>("ds_read_b32", d, grid);
  run<1>("ds_cmpst_rtn", d, grid);
  run<2>("ds_min_u32", d, grid);
  run<3>("ds_or_b32", d, grid);
  run<4>("ds_add_rtn_u32", d, grid);
  run<5>("ds_min_rtn_u32", d, grid);
  run<6>("ds_write_b32", d, grid);
  return 0;
}
