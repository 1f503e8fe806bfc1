// Microbenchmark: host -> device rates for a C2-sized batch (GB/s), to choose
// the host entry points' staging (sg_triage.hip):
//  (a) hipMemcpyAsync from pageable memory (the runtime stages it);
//  (b) from pinned memory (hipHostMalloc);
//  (c) hipHostRegister of the pageable buffer, DMA, hipHostUnregister (per call);
//  (d) memcpy into pinned memory by T host threads (the CPU side of a staging copy).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 0) : 1ull << 30);
  const int reps = 3;
  char* pageable = (char*)aligned_alloc(4096, bytes);
  memset(pageable, 1, bytes);
  char *pinned = nullptr, *dev = nullptr;
  CK(hipHostMalloc((void**)&pinned, bytes, hipHostMallocDefault));
  memset(pinned, 2, bytes);
  CK(hipMalloc((void**)&dev, bytes));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  auto rate = [&](double s) { return bytes / s / 1e9; };
  double best[4] = {0, 0, 0, 0};
  for (int r = 0; r < reps; r++) {
    double t = now();
    CK(hipMemcpyAsync(dev, pageable, bytes, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    best[0] = std::max(best[0], rate(now() - t));
    t = now();
    CK(hipMemcpyAsync(dev, pinned, bytes, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    best[1] = std::max(best[1], rate(now() - t));
    t = now();
    CK(hipHostRegister(pageable, bytes, hipHostRegisterDefault));
    const double treg = now() - t;
    void* dp = nullptr;
    CK(hipHostGetDevicePointer(&dp, pageable, 0));
    CK(hipMemcpyAsync(dev, pageable, bytes, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    const double tcopy = now() - t - treg;
    CK(hipHostUnregister(pageable));
    best[2] = std::max(best[2], rate(now() - t));
    printf("rep %d: register %.1f ms, registered copy %.1f GB/s, unregister included total %.1f GB/s\n", r,
           treg * 1e3, rate(tcopy), rate(now() - t));
  }
  printf("%.2f GiB: pageable %.1f GB/s, pinned %.1f GB/s, register+copy+unregister %.1f GB/s\n",
         bytes / 1073741824.0, best[0], best[1], best[2]);
  for (int T : {1, 2, 4, 8, 16}) {
    double b = 0;
    for (int r = 0; r < reps; r++) {
      const double t = now();
      std::vector<std::thread> th;
      for (int i = 0; i < T; i++)
        th.emplace_back([&, i] {
          const size_t lo = bytes / T * i, hi = i == T - 1 ? bytes : bytes / T * (i + 1);
          memcpy(pinned + lo, pageable + lo, hi - lo);
        });
      for (auto& x : th) x.join();
      b = std::max(b, rate(now() - t));
    }
    printf("memcpy pageable -> pinned, %2d threads: %.1f GB/s\n", T, b);
  }
  return 0;
}
