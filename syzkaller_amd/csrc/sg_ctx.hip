// sg_ctx.hip -- context, workspace, timing, device scan and the signal-set
// (map[uint32]struct{} replacement) entry points of libsyzsig.so.
//
// Reference: the Go maps maxSignal / corpusSignal / newSignal
// (syz-fuzzer/fuzzer.go:65-68, syz-manager/manager.go:71-73) and the map
// helpers SignalNew / SignalDiff / SignalAdd (pkg/cover/cover.go:160-182).
// A set is a 2^32-bit bitmap in HBM: membership of s is bit s of word s>>5.
#include "sg_internal.h"

#include <cstring>

namespace sg {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

int hip_fail(hipError_t e, const char* what) {
  set_error("HIP error %d (%s) in %s", (int)e, hipGetErrorString(e), what);
  if (e == hipErrorOutOfMemory) return SG_ENOMEM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice || e == hipErrorNoBinaryForGpu) return SG_ENODEV;
  return SG_EHIP;
}

int ensure_device(sg_ctx* ctx) {
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  // hipGetLastError after our launches must see only our errors.  The one
  // known stale code left on this thread by another library (torch's
  // "invalid device ordinal" after spawning multiprocess workers) is dropped
  // silently; any other pending error belongs to the caller's own HIP work,
  // so it is reported on stderr before it is cleared, not hidden.
  const hipError_t stale = hipPeekAtLastError();
  if (stale != hipSuccess) {
    if (stale != hipErrorInvalidDevice)
      fprintf(stderr, "libsyzsig: clearing a pending HIP error of the calling thread: %d (%s)\n", (int)stale,
              hipGetErrorString(stale));
    (void)hipGetLastError();
  }
  return SG_OK;
}

int ws_reserve(sg_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->ws_cap) return SG_OK;
  size_t cap = ctx->ws_cap ? ctx->ws_cap : (64u << 20);
  while (cap < bytes) cap *= 2;
  if (ctx->ws) {
    SG_HIP(hipStreamSynchronize(ctx->stream));
    SG_HIP(hipFree(ctx->ws));
    ctx->ws = nullptr;
    ctx->ws_cap = 0;
  }
  SG_HIP(hipMalloc(&ctx->ws, cap));
  ctx->ws_cap = cap;
  return SG_OK;
}

int pin_reserve(sg_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->pin_cap) return SG_OK;
  size_t cap = ctx->pin_cap ? ctx->pin_cap : (16u << 20);
  while (cap < bytes) cap *= 2;
  if (ctx->pin) {
    SG_HIP(hipStreamSynchronize(ctx->stream));
    if (ctx->copy_stream) SG_HIP(hipStreamSynchronize(ctx->copy_stream));  // (the host pipeline's DMAs)
    SG_HIP(hipHostFree(ctx->pin));
    ctx->pin = nullptr;
    ctx->pin_cap = 0;
  }
  SG_HIP(hipHostMalloc(&ctx->pin, cap, hipHostMallocDefault));
  ctx->pin_cap = cap;
  return SG_OK;
}

int dstage_reserve(sg_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->dstage_cap) return SG_OK;
  size_t cap = ctx->dstage_cap ? ctx->dstage_cap : (16u << 20);
  while (cap < bytes) cap *= 2;
  if (ctx->dstage) {
    SG_HIP(hipStreamSynchronize(ctx->stream));
    if (ctx->copy_stream) SG_HIP(hipStreamSynchronize(ctx->copy_stream));  // (the host pipeline's DMAs)
    SG_HIP(hipFree(ctx->dstage));
    ctx->dstage = nullptr;
    ctx->dstage_cap = 0;
  }
  SG_HIP(hipMalloc(&ctx->dstage, cap));
  ctx->dstage_cap = cap;
  return SG_OK;
}

int owner_keys(sg_ctx* ctx, uint64_t nkeys, uint32_t* key_lo) {
  if (nkeys > ctx->owner_key_space) {
    set_error("batch of %llu keys exceeds the first-owner key space (%llu)", (unsigned long long)nkeys,
              (unsigned long long)ctx->owner_key_space);
    return SG_EINVAL;
  }
  if (!ctx->owner) {
    SG_HIP(hipMalloc(&ctx->owner, kOwnerEntries * sizeof(uint32_t)));
    SG_HIP(hipMemsetAsync(ctx->owner, 0xFF, kOwnerEntries * sizeof(uint32_t), ctx->stream));
    ctx->owner_floor = ctx->owner_key_space;
  }
  if (ctx->owner_floor < nkeys) {
    // Key space exhausted (after ~4G keys): start a fresh generation.
    SG_HIP(hipMemsetAsync(ctx->owner, 0xFF, kOwnerEntries * sizeof(uint32_t), ctx->stream));
    ctx->owner_floor = ctx->owner_key_space;
    ctx->owner_resets++;
  }
  ctx->owner_floor -= nkeys;
  *key_lo = (uint32_t)ctx->owner_floor;
  return SG_OK;
}

// ---- kernel timing ---------------------------------------------------------
void timer_begin(sg_ctx* ctx, const char* name, int* slot) {
  KernelTimer& t = ctx->timer;
  *slot = -1;
  if (!t.enabled) return;
  auto it = t.ids.find(name);
  int id;
  if (it == t.ids.end()) {
    id = (int)t.names.size();
    t.ids[name] = id;
    t.names.push_back(name);
    t.ms.push_back(0);
    t.count.push_back(0);
  } else {
    id = it->second;
  }
  hipEvent_t a, b;
  if (t.pool.size() >= 2) {
    a = t.pool.back();
    t.pool.pop_back();
    b = t.pool.back();
    t.pool.pop_back();
  } else {
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
  }
  hipEventRecord(a, ctx->stream);
  t.pending.push_back({id, a, b});
  *slot = (int)t.pending.size() - 1;
}

void timer_end(sg_ctx* ctx, int slot) {
  if (slot < 0) return;
  hipEventRecord(ctx->timer.pending[slot].b, ctx->stream);
}

static void timer_collect(sg_ctx* ctx) {
  KernelTimer& t = ctx->timer;
  for (auto& r : t.pending) {
    hipEventSynchronize(r.b);
    float ms = 0;
    hipEventElapsedTime(&ms, r.a, r.b);
    t.ms[r.id] += ms;
    t.count[r.id] += 1;
    t.pool.push_back(r.a);
    t.pool.push_back(r.b);
  }
  t.pending.clear();
}

// ---- device scan: exclusive prefix of u32 counts into u64 offsets ----------
constexpr int kScanItems = 16;
constexpr int kScanTile = kBlock * kScanItems;  // 4096

__global__ __launch_bounds__(kBlock) void k_scan_tile(const uint32_t* __restrict__ in, uint64_t n,
                                                      uint64_t* __restrict__ out, uint64_t* __restrict__ tile_sum) {
  __shared__ uint64_t part[kBlock];
  uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  uint32_t v[kScanItems];
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; i++) {
    uint64_t idx = base + i;
    v[i] = idx < n ? in[idx] : 0u;
    s += v[i];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  // Hillis-Steele over 256 partials (inclusive)
  for (int d = 1; d < kBlock; d <<= 1) {
    uint64_t x = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += x;
    __syncthreads();
  }
  uint64_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
#pragma unroll
  for (int i = 0; i < kScanItems; i++) {
    uint64_t idx = base + i;
    if (idx < n) out[idx] = run;
    run += v[i];
  }
  if (threadIdx.x == kBlock - 1) tile_sum[blockIdx.x] = part[kBlock - 1];
}

__global__ __launch_bounds__(kBlock) void k_scan_u64_tile(uint64_t* __restrict__ data, uint64_t n,
                                                          uint64_t* __restrict__ tile_sum) {
  // in-place exclusive scan of u64 values, per 4096-tile
  __shared__ uint64_t part[kBlock];
  uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  uint64_t v[kScanItems];
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; i++) {
    uint64_t idx = base + i;
    v[i] = idx < n ? data[idx] : 0u;
    s += v[i];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int d = 1; d < kBlock; d <<= 1) {
    uint64_t x = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += x;
    __syncthreads();
  }
  uint64_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
#pragma unroll
  for (int i = 0; i < kScanItems; i++) {
    uint64_t idx = base + i;
    if (idx < n) data[idx] = run;
    run += v[i];
  }
  if (threadIdx.x == kBlock - 1) tile_sum[blockIdx.x] = part[kBlock - 1];
}

__global__ void k_scan_add(uint64_t* __restrict__ out, uint64_t n, const uint64_t* __restrict__ tile_base) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] += tile_base[i / kScanTile];
}

__global__ void k_scan_total(uint64_t* out, uint64_t n, const uint64_t* tile_base, const uint64_t* tile_sum,
                             uint64_t ntiles) {
  out[n] = ntiles ? tile_base[ntiles - 1] + tile_sum[ntiles - 1] : 0;
}

size_t scan_ws_bytes(uint64_t n) {
  size_t b = 0;
  while (n > 1) {
    uint64_t t = (n + kScanTile - 1) / kScanTile;
    b += 2 * ((t * 8 + 255) & ~255ull);
    n = t;
  }
  return b + 512;
}

__global__ void k_copy_u64(const uint64_t* __restrict__ in, uint64_t n, uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[i];
}

static int scan_u64_inplace(sg_ctx* ctx, uint64_t* data, uint64_t n, char* scratch) {
  // exclusive in-place scan of n u64 values (used for tile sums)
  if (n == 0) return SG_OK;
  uint64_t nt = (n + kScanTile - 1) / kScanTile;
  uint64_t* sums = (uint64_t*)scratch;
  char* next = scratch + ((nt * 8 + 255) & ~255ull);
  hipLaunchKernelGGL(k_scan_u64_tile, dim3((uint32_t)nt), dim3(kBlock), 0, ctx->stream, data, n, sums);
  if (nt > 1) {
    int rc = scan_u64_inplace(ctx, sums, nt, next);
    if (rc) return rc;
    hipLaunchKernelGGL(k_scan_add, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, data, n, sums);
  }
  return SG_OK;
}

int scan_counts(sg_ctx* ctx, const uint32_t* d_in, uint64_t* d_out, uint64_t n, size_t ws_used) {
  ScopedTimer tm(ctx, "scan");
  char* scratch = (char*)ctx->ws + ws_used;
  uint64_t nt = n ? (n + kScanTile - 1) / kScanTile : 0;
  uint64_t* sums = (uint64_t*)scratch;
  uint64_t* bases = (uint64_t*)(scratch + ((nt * 8 + 255) & ~255ull));
  char* next = (char*)bases + ((nt * 8 + 255) & ~255ull);
  if (n == 0) {
    SG_HIP(hipMemsetAsync(d_out, 0, 8, ctx->stream));
    return SG_OK;
  }
  hipLaunchKernelGGL(k_scan_tile, dim3((uint32_t)nt), dim3(kBlock), 0, ctx->stream, d_in, n, d_out, sums);
  // (a copy kernel: a device-to-device hipMemcpyAsync between two kernels
  // leaves the stream idle around it)
  hipLaunchKernelGGL(k_copy_u64, dim3(div_up(nt, 256)), dim3(256), 0, ctx->stream, (const uint64_t*)sums, nt, bases);
  int rc = scan_u64_inplace(ctx, bases, nt, next);
  if (rc) return rc;
  if (nt > 1) hipLaunchKernelGGL(k_scan_add, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, d_out, n, bases);
  hipLaunchKernelGGL(k_scan_total, dim3(1), dim3(1), 0, ctx->stream, d_out, n, bases, sums, nt);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

// ---- set kernels -----------------------------------------------------------
__global__ void k_set_add(uint32_t* __restrict__ words, const uint32_t* __restrict__ sig, uint64_t n) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    sgd::set_bit(words, sig[i]);
}

// kOrU quads of `other` per thread in flight (one at a time left the 512 MiB
// pass latency-bound: 0.28 ms on a nearly empty `other`)
constexpr int kOrU = 4;
__global__ __launch_bounds__(256) void k_set_or(uint32_t* __restrict__ words, const uint32_t* __restrict__ other) {
  constexpr uint64_t q = kSetWords / 4;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * kOrU;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x * kOrU + threadIdx.x; i0 < q; i0 += stride) {
    uint4 b[kOrU];
#pragma unroll
    for (int u = 0; u < kOrU; u++) b[u] = reinterpret_cast<const uint4*>(other)[i0 + u * blockDim.x];
#pragma unroll
    for (int u = 0; u < kOrU; u++) {
      if (!(b[u].x | b[u].y | b[u].z | b[u].w)) continue;  // (a sparse `other` reads little else)
      uint4* p = reinterpret_cast<uint4*>(words) + i0 + u * blockDim.x;
      uint4 a = *p;
      a.x |= b[u].x;
      a.y |= b[u].y;
      a.z |= b[u].z;
      a.w |= b[u].w;
      *p = a;
    }
  }
}

// words |= other & ~exclude
__global__ __launch_bounds__(256) void k_set_or_new(uint32_t* __restrict__ words, const uint32_t* __restrict__ other,
                                                    const uint32_t* __restrict__ exclude) {
  constexpr uint64_t q = kSetWords / 4;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * kOrU;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x * kOrU + threadIdx.x; i0 < q; i0 += stride) {
    uint4 b[kOrU];
#pragma unroll
    for (int u = 0; u < kOrU; u++) b[u] = reinterpret_cast<const uint4*>(other)[i0 + u * blockDim.x];
#pragma unroll
    for (int u = 0; u < kOrU; u++) {
      if (!(b[u].x | b[u].y | b[u].z | b[u].w)) continue;
      const uint64_t i = i0 + u * blockDim.x;
      uint4 a = reinterpret_cast<uint4*>(words)[i];
      const uint4 x = reinterpret_cast<const uint4*>(exclude)[i];
      a.x |= b[u].x & ~x.x;
      a.y |= b[u].y & ~x.y;
      a.z |= b[u].z & ~x.z;
      a.w |= b[u].w & ~x.w;
      reinterpret_cast<uint4*>(words)[i] = a;
    }
  }
}

// newsig |= other & ~maxsig; maxsig |= other (newsig nullable)
__global__ __launch_bounds__(256) void k_set_or_new_or(uint32_t* __restrict__ newsig, uint32_t* __restrict__ maxsig,
                                                       const uint32_t* __restrict__ other) {
  constexpr uint64_t q = kSetWords / 4;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * kOrU;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x * kOrU + threadIdx.x; i0 < q; i0 += stride) {
    uint4 b[kOrU];
#pragma unroll
    for (int u = 0; u < kOrU; u++) b[u] = reinterpret_cast<const uint4*>(other)[i0 + u * blockDim.x];
#pragma unroll
    for (int u = 0; u < kOrU; u++) {
      if (!(b[u].x | b[u].y | b[u].z | b[u].w)) continue;
      const uint64_t i = i0 + u * blockDim.x;
      uint4 m = reinterpret_cast<uint4*>(maxsig)[i];
      if (newsig) {
        uint4 n = reinterpret_cast<uint4*>(newsig)[i];
        n.x |= b[u].x & ~m.x;
        n.y |= b[u].y & ~m.y;
        n.z |= b[u].z & ~m.z;
        n.w |= b[u].w & ~m.w;
        reinterpret_cast<uint4*>(newsig)[i] = n;
      }
      m.x |= b[u].x;
      m.y |= b[u].y;
      m.z |= b[u].z;
      m.w |= b[u].w;
      reinterpret_cast<uint4*>(maxsig)[i] = m;
    }
  }
}

__global__ void k_set_new(const uint32_t* __restrict__ words, const uint32_t* __restrict__ sig, uint64_t n,
                          uint64_t* __restrict__ flag) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  bool miss = false;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    miss |= !sgd::test_bit(words, sig[i]);
  if (__any(miss) && (threadIdx.x & 63) == 0) *flag = 1;
}

__global__ void k_count_missing(const uint32_t* __restrict__ words, const uint32_t* __restrict__ v, uint64_t n,
                                unsigned long long* __restrict__ out) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint32_t c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    c += !sgd::test_bit(words, v[i]);
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, (unsigned long long)c);
}

// popcount of the bitmap, per 4096-word tile (for count and export)
__global__ __launch_bounds__(kBlock) void k_set_tile_pop(const uint32_t* __restrict__ words,
                                                         uint32_t* __restrict__ tile_cnt) {
  __shared__ uint32_t red[kBlock / 64];
  // tiles of 4096 words in signal order (sgd::set_word), as the export walks them
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kTile / 4 / kBlock; j++) {
    const uint32_t ws = (uint32_t)blockIdx.x * kTile + (j * kBlock + threadIdx.x) * 4;
    const uint4 v = *reinterpret_cast<const uint4*>(words + sgd::set_word(ws));
    c += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x / 64] = c;
  __syncthreads();
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// each thread owns 16 consecutive words of the tile; block-scan of their
// popcounts gives each thread's first output slot.
__global__ __launch_bounds__(kBlock) void k_set_export(const uint32_t* __restrict__ words,
                                                       const uint64_t* __restrict__ tile_base,
                                                       uint32_t* __restrict__ out, uint64_t cap) {
  __shared__ uint32_t part[kBlock];
  uint64_t w0 = (uint64_t)blockIdx.x * kTile + (uint64_t)threadIdx.x * 16;
  uint64_t tb = tile_base[blockIdx.x];
  if (tile_base[blockIdx.x + 1] == tb) return;  // empty tile (block-uniform)
  // signal-order words w0 .. w0+15: two runs of 8 consecutive bitmap words
  const uint4* r0 = reinterpret_cast<const uint4*>(words + sgd::set_word((uint32_t)w0));
  const uint4* r1 = reinterpret_cast<const uint4*>(words + sgd::set_word((uint32_t)w0 + 8));
  uint32_t w[16];
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    uint4 v = j < 2 ? r0[j] : r1[j - 2];
    w[4 * j] = v.x;
    w[4 * j + 1] = v.y;
    w[4 * j + 2] = v.z;
    w[4 * j + 3] = v.w;
    c += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
  }
  part[threadIdx.x] = c;
  __syncthreads();
  for (int d = 1; d < kBlock; d <<= 1) {
    uint32_t x = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += x;
    __syncthreads();
  }
  uint64_t pos = tb + part[threadIdx.x] - c;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    uint32_t x = w[j];
    while (x) {
      int b = __ffs(x) - 1;
      x &= x - 1;
      if (pos < cap) out[pos] = (uint32_t)((w0 + j) * 32 + b);
      pos++;
    }
  }
}

}  // namespace sg

using namespace sg;

// ---- C-ABI -------------------------------------------------------------------
extern "C" {

const char* sg_version(void) { return "syzsig 0.1 gfx950"; }
const char* sg_last_error(void) { return g_err.c_str(); }

int sg_ctx_create(int device, sg_ctx** out) {
  if (!out) {
    set_error("sg_ctx_create: out is NULL");
    return SG_EINVAL;
  }
  *out = nullptr;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) {
    set_error("no HIP device available (libsyzsig has no CPU path)");
    return SG_ENODEV;
  }
  if (device < 0 || device >= ndev) {
    set_error("device %d out of range (%d devices)", device, ndev);
    return SG_EINVAL;
  }
  hipDeviceProp_t prop;
  SG_HIP(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    set_error("device %d is %s; libsyzsig is built for gfx950 (MI355X) only", device, prop.gcnArchName);
    return SG_ENODEV;
  }
  sg_ctx* c = new sg_ctx();
  c->device = device;
  c->max_launch_recs = kMaxLaunchRecords;
  // the diagnostics switches of the GPU scripts, read once here (every other
  // option is set by sg_ctx_set_option; nothing reads the environment later)
  c->debug_part = getenv("SG_DEBUG_PART") != nullptr;
  if (const char* e = getenv("SG_BUCKET_BLOCKS")) c->opt[kOptBucketBlocks] = strtoll(e, nullptr, 10);
  if (const char* e = getenv("SG_PREFIX_PAIRS")) c->opt[kOptPrefixPairs] = strtoll(e, nullptr, 10) != 0;
  c->cpu_quota = host_cpu_quota();
  int rc = ensure_device(c);
  if (rc) {
    delete c;
    return rc;
  }
  e = hipStreamCreateWithFlags(&c->own_stream, hipStreamDefault);  // blocking: ordered with the null stream
  if (e != hipSuccess) {
    delete c;
    return hip_fail(e, "hipStreamCreate");
  }
  c->stream = c->own_stream;
  e = hipMalloc(&c->dscal, 256);
  if (e != hipSuccess) {
    hipStreamDestroy(c->own_stream);
    delete c;
    return hip_fail(e, "hipMalloc(dscal)");
  }
  *out = c;
  return SG_OK;
}

void sg_ctx_destroy(sg_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  if (ctx->copy_stream) hipStreamSynchronize(ctx->copy_stream);  // (before the buffers its DMAs use go)
  for (auto& r : ctx->timer.pending) {
    hipEventDestroy(r.a);
    hipEventDestroy(r.b);
  }
  for (auto ev : ctx->timer.pool) hipEventDestroy(ev);
  if (ctx->ws) hipFree(ctx->ws);
  for (auto& s : ctx->prefix)
    if (s.ws) hipFree(s.ws);
  if (ctx->pin) hipHostFree(ctx->pin);
  if (ctx->dstage) hipFree(ctx->dstage);
  if (ctx->owner) hipFree(ctx->owner);
  if (ctx->m0f) hipFree(ctx->m0f);
  if (ctx->m0f_host) hipHostFree(ctx->m0f_host);
  if (ctx->m0f_ev) hipEventDestroy(ctx->m0f_ev);
  if (ctx->slice_off) hipFree(ctx->slice_off);
  if (ctx->slice_cuts) hipFree(ctx->slice_cuts);
  if (ctx->dscal) hipFree(ctx->dscal);
  if (ctx->gen_prob) hipFree(ctx->gen_prob);
  if (ctx->gen_alias) hipFree(ctx->gen_alias);
  if (ctx->gen_perm) hipFree(ctx->gen_perm);
  if (ctx->copy_stream) {
    hipStreamSynchronize(ctx->copy_stream);
    for (auto e : ctx->pipe_ev)
      if (e) hipEventDestroy(e);
    hipStreamDestroy(ctx->copy_stream);
  }
  if (ctx->own_stream) hipStreamDestroy(ctx->own_stream);
  delete ctx;
}

int sg_ctx_sync(sg_ctx* ctx) {
  if (!ctx) return SG_EINVAL;
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

int sg_ctx_set_stream(sg_ctx* ctx, void* hip_stream) {
  if (!ctx) return SG_EINVAL;
  ctx->stream = (hipStream_t)hip_stream;  // NULL: the device's legacy default stream
  return SG_OK;
}

int sg_ctx_reset_stream(sg_ctx* ctx) {
  if (!ctx) return SG_EINVAL;
  ctx->stream = ctx->own_stream;
  return SG_OK;
}

void* sg_ctx_stream(sg_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int sg_ctx_timing(sg_ctx* ctx, int enable) {
  if (!ctx) return SG_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  timer_collect(ctx);
  KernelTimer& t = ctx->timer;
  for (auto& v : t.ms) v = 0;
  for (auto& v : t.count) v = 0;
  t.enabled = enable != 0;
  return SG_OK;
}

int sg_ctx_kernel_time(sg_ctx* ctx, const char* name, double* ms, uint64_t* launches) {
  if (!ctx || !name) return SG_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  timer_collect(ctx);
  KernelTimer& t = ctx->timer;
  auto it = t.ids.find(name);
  if (ms) *ms = it == t.ids.end() ? 0 : t.ms[it->second];
  if (launches) *launches = it == t.ids.end() ? 0 : t.count[it->second];
  return SG_OK;
}

}  // extern "C"

namespace sg {
// one-thread kernels that only mark a point of the stream in kernel traces
__global__ void k_mark_begin(uint32_t* sink, uint32_t tag) {
  if (tag == 0xFFFFFFFFu) *sink = tag;  // never taken: keeps the launch from being elided
}
__global__ void k_mark_end(uint32_t* sink, uint32_t tag) {
  if (tag == 0xFFFFFFFFu) *sink = tag;
}
}  // namespace sg

extern "C" {

int sg_ctx_marker(sg_ctx* ctx, int end, uint32_t tag) {
  if (!ctx || tag == 0xFFFFFFFFu) return SG_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  if (end)
    hipLaunchKernelGGL(k_mark_end, dim3(1), dim3(1), 0, ctx->stream, (uint32_t*)ctx->dscal, tag);
  else
    hipLaunchKernelGGL(k_mark_begin, dim3(1), dim3(1), 0, ctx->stream, (uint32_t*)ctx->dscal, tag);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

static const char* const kOptNames[kOptCount] = {
    "bucket_blocks",      "prefix_pairs",       "fold_map",         "minimize_filter",   "minimize_filter_ranks",
    "report_direct",      "rpc_encode_elems",   "rpc_decode_blocks", "host_slice",       "host_copy_threads",
    "m0_filter",          "m0_filter_halves"};

int sg_ctx_set_option(sg_ctx* ctx, const char* key, int64_t value) {
  if (!ctx || !key) return SG_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!strcmp(key, "max_launch_records")) {  // records per partitioned launch (lowered for slicing tests)
    if (value < 0 || (uint64_t)value > kMaxLaunchRecords) {
      set_error("sg_ctx_set_option: max_launch_records in 1..%llu (0: the default)",
                (unsigned long long)kMaxLaunchRecords);
      return SG_EINVAL;
    }
    ctx->max_launch_recs = value ? (uint64_t)value : kMaxLaunchRecords;
    return SG_OK;
  }
  if (!strcmp(key, "owner_key_space")) {  // Minimize's key space (lowered to reach the generation reset)
    if (ctx->owner) {
      set_error("sg_ctx_set_option: owner_key_space is set before the first-owner table exists");
      return SG_EINVAL;
    }
    if (value < 0 || (uint64_t)value > 0xFFFFFFFFull) {
      set_error("sg_ctx_set_option: owner_key_space in 1..2^32-1 (0: the default)");
      return SG_EINVAL;
    }
    ctx->owner_key_space = value ? (uint64_t)value : 0xFFFFFFFFull;
    return SG_OK;
  }
  if (!strcmp(key, "debug_part")) {
    ctx->debug_part = value != 0;
    return SG_OK;
  }
  // value ranges, in kOptNames' order (tri-state options: -1 the regime's choice)
  static const int64_t kLo[kOptCount] = {0, 0, -1, 0, 0, 0, -1, -1, 0, 0, -1, -1};
  static const int64_t kHi[kOptCount] = {1 << 20, 1, 1, 1, 1 << 20, 1, 1, 1, 1ll << 40, 64, 1, 2};
  for (int i = 0; i < kOptCount; i++)
    if (!strcmp(key, kOptNames[i])) {
      if (value < kLo[i] || value > kHi[i]) {
        set_error("sg_ctx_set_option: %s in %lld..%lld", key, (long long)kLo[i], (long long)kHi[i]);
        return SG_EINVAL;
      }
      ctx->opt[i] = value;
      return SG_OK;
    }
  set_error("sg_ctx_set_option: unknown option '%s'", key);
  return SG_EINVAL;
}

int sg_ctx_get_option(sg_ctx* ctx, const char* key, int64_t* out) {
  if (!ctx || !key || !out) return SG_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!strcmp(key, "max_launch_records")) {
    *out = (int64_t)ctx->max_launch_recs;
    return SG_OK;
  }
  if (!strcmp(key, "owner_key_space")) {
    *out = (int64_t)ctx->owner_key_space;
    return SG_OK;
  }
  if (!strcmp(key, "debug_part")) {
    *out = ctx->debug_part;
    return SG_OK;
  }
  for (int i = 0; i < kOptCount; i++)
    if (!strcmp(key, kOptNames[i])) {
      *out = ctx->opt[i];
      return SG_OK;
    }
  set_error("sg_ctx_get_option: unknown option '%s'", key);
  return SG_EINVAL;
}

int sg_ctx_counter(sg_ctx* ctx, const char* name, uint64_t* out) {
  if (!ctx || !name || !out) return SG_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!strcmp(name, "owner_resets"))
    *out = ctx->owner_resets;
  else if (!strcmp(name, "owner_floor"))
    *out = ctx->owner ? ctx->owner_floor : ctx->owner_key_space;
  else if (!strcmp(name, "owner_key_space"))
    *out = ctx->owner_key_space;
  else if (!strcmp(name, "max_launch_records"))
    *out = ctx->max_launch_recs;
  else if (!strcmp(name, "host_copy_bytes"))  // the host ingest's last call (sg_host.hip)
    *out = ctx->host_copy_bytes;
  else if (!strcmp(name, "host_copy_ns"))
    *out = ctx->host_copy_ns;
  else if (!strcmp(name, "host_wait_ns"))
    *out = ctx->host_wait_ns;
  else if (!strcmp(name, "host_copy_threads"))
    *out = ctx->host_threads;
  else if (!strcmp(name, "m0_filter_used"))  // record slices the M0 filter finished (sg_bucket.hip)
    *out = ctx->m0f_used;
  else if (!strcmp(name, "m0_filter_fallback"))  // ... and those whose survivors overflowed (the partition went on)
    *out = ctx->m0f_fallback;
  else if (!strcmp(name, "m0_filter_survivors"))  // survivors of the last filtered slice
    *out = ctx->m0f_survivors;
  else if (!strcmp(name, "m0_filter_queued_milli"))  // queued fraction x1000 of the last partitioned slice
    *out = ctx->m0f_queued < 0 ? ~0ull : (uint64_t)(ctx->m0f_queued * 1000.0 + 0.5);
  else if (!strcmp(name, "m0_filter_halves_log"))  // the index's parts per slice (log2) the auto regime uses now
    *out = (uint64_t)ctx->m0f_logh;
  else if (!strcmp(name, "cpu_quota_milli"))
    *out = (uint64_t)(ctx->cpu_quota * 1000.0 + 0.5);
  else {
    set_error("sg_ctx_counter: unknown counter '%s'", name);
    return SG_EINVAL;
  }
  return SG_OK;
}

int sg_set_create(sg_ctx* ctx, sg_set** out) {
  if (!ctx || !out) return SG_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  sg_set* s = new sg_set();
  s->ctx = ctx;
  hipError_t e = hipMalloc(&s->words, kSetBytes);
  if (e != hipSuccess) {
    delete s;
    return hip_fail(e, "hipMalloc(set)");
  }
  e = hipMemsetAsync(s->words, 0, kSetBytes, ctx->stream);
  if (e != hipSuccess) {
    hipFree(s->words);
    delete s;
    return hip_fail(e, "hipMemset(set)");
  }
  *out = s;
  return SG_OK;
}

void sg_set_destroy(sg_set* set) {
  if (!set) return;
  hipSetDevice(set->ctx->device);
  hipStreamSynchronize(set->ctx->stream);
  if (set->owned) hipFree(set->words);
  delete set;
}

int sg_set_clear(sg_set* set) {
  if (!set) return SG_EINVAL;
  sg_ctx* ctx = set->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  SG_HIP(hipMemsetAsync(set->words, 0, kSetBytes, ctx->stream));
  return SG_OK;
}

void* sg_set_device_words(sg_set* set) { return set ? set->words : nullptr; }

int sg_set_wrap_dev(sg_ctx* ctx, void* d_words, sg_set** out) {
  if (!ctx || !d_words || !out || ((uintptr_t)d_words & 15)) {
    set_error("sg_set_wrap_dev: invalid argument (words must be 16-B aligned device memory)");
    return SG_EINVAL;
  }
  sg_set* s = new sg_set();
  s->ctx = ctx;
  s->words = (uint32_t*)d_words;
  s->owned = false;
  *out = s;
  return SG_OK;
}

int sg_set_copy(sg_set* dst, sg_set* src) {
  if (!dst || !src || dst->ctx != src->ctx) return SG_EINVAL;
  sg_ctx* ctx = dst->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  if (dst != src) SG_HIP(hipMemcpyAsync(dst->words, src->words, kSetBytes, hipMemcpyDeviceToDevice, ctx->stream));
  return SG_OK;
}

int sg_set_count_missing_dev(sg_set* set, const uint32_t* d_vals, uint64_t n, uint64_t* out) {
  if (!set || !out || (n && !d_vals)) return SG_EINVAL;
  *out = 0;
  if (n == 0) return SG_OK;
  sg_ctx* ctx = set->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  SG_HIP(hipMemsetAsync(ctx->dscal, 0, 8, ctx->stream));
  hipLaunchKernelGGL(k_count_missing, dim3(2048), dim3(256), 0, ctx->stream, set->words, d_vals, n,
                     (unsigned long long*)ctx->dscal);
  SG_HIP(hipGetLastError());
  SG_HIP(hipMemcpyAsync(out, ctx->dscal, 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

int sg_set_or_dev(sg_set* set, const uint32_t* d_words) {
  if (!set || !d_words) return SG_EINVAL;
  sg_ctx* ctx = set->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  ScopedTimer tm(ctx, "set_or");
  hipLaunchKernelGGL(k_set_or, dim3(4096), dim3(256), 0, ctx->stream, set->words, d_words);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

int sg_set_or_new_or_dev(sg_set* newsig, sg_set* maxsig, const uint32_t* d_words) {
  if (!maxsig || !d_words || (newsig && (newsig->ctx != maxsig->ctx || newsig == maxsig ||
                                         d_words == (const uint32_t*)newsig->words)) ||
      d_words == (const uint32_t*)maxsig->words) {
    // k_set_or_new_or takes all three __restrict__: no aliasing
    set_error("sg_set_or_new_or_dev: invalid argument (null, another context's set, or aliasing sets / words)");
    return SG_EINVAL;
  }
  sg_ctx* ctx = maxsig->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  ScopedTimer tm(ctx, "set_or_new_or");
  hipLaunchKernelGGL(k_set_or_new_or, dim3(4096), dim3(256), 0, ctx->stream, newsig ? newsig->words : nullptr,
                     maxsig->words, d_words);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

int sg_set_or_new_dev(sg_set* set, const uint32_t* d_words, sg_set* exclude) {
  if (!set || !d_words || !exclude || exclude->ctx != set->ctx || exclude == set ||
      d_words == (const uint32_t*)set->words) {
    // k_set_or_new takes words and exclude __restrict__: no aliasing
    set_error("sg_set_or_new_dev: invalid argument (null, another context's set, or exclude/words aliasing set)");
    return SG_EINVAL;
  }
  sg_ctx* ctx = set->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  ScopedTimer tm(ctx, "set_or_new");
  hipLaunchKernelGGL(k_set_or_new, dim3(4096), dim3(256), 0, ctx->stream, set->words, d_words, exclude->words);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

static int set_tile_bases(sg_set* set, uint64_t** bases_out, uint64_t* total) {
  sg_ctx* ctx = set->ctx;
  const uint64_t ntile = kSetWords / kTile;  // 32768
  WsPlan p;
  size_t o_cnt = p.add(ntile * 4);
  size_t o_base = p.add((ntile + 1) * 8);
  int rc = ws_reserve(ctx, p.total + scan_ws_bytes(ntile));
  if (rc) return rc;
  uint32_t* cnt = (uint32_t*)ws_at(ctx, o_cnt);
  uint64_t* base = (uint64_t*)ws_at(ctx, o_base);
  hipLaunchKernelGGL(k_set_tile_pop, dim3((uint32_t)ntile), dim3(kBlock), 0, ctx->stream, set->words, cnt);
  rc = scan_counts(ctx, cnt, base, ntile, p.total);
  if (rc) return rc;
  SG_HIP(hipMemcpyAsync(total, base + ntile, 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  *bases_out = base;
  return SG_OK;
}

int sg_set_count(sg_set* set, uint64_t* out) {
  if (!set || !out) return SG_EINVAL;
  sg_ctx* ctx = set->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  uint64_t* bases;
  return set_tile_bases(set, &bases, out);
}

}  // extern "C"

namespace sg {
// The members of `set`, ascending, into device memory d_out (capacity cap);
// *total = count (ctx lock held; syncs).
int set_export_dev(sg_set* set, uint32_t* d_out, uint64_t cap, uint64_t* total) {
  sg_ctx* ctx = set->ctx;
  uint64_t* bases;
  int rc = set_tile_bases(set, &bases, total);
  if (rc) return rc;
  const uint64_t m = *total < cap ? *total : cap;
  if (m == 0) return SG_OK;
  hipLaunchKernelGGL(k_set_export, dim3((uint32_t)(kSetWords / kTile)), dim3(kBlock), 0, ctx->stream, set->words,
                     bases, d_out, m);
  SG_HIP(hipGetLastError());
  return SG_OK;
}

// SignalAdd of n device-resident values (ctx lock held, stream-ordered).
int set_add_dev_locked(sg_set* set, const uint32_t* d_vals, uint64_t n) {
  if (n == 0) return SG_OK;
  ScopedTimer tm(set->ctx, "set_add");
  hipLaunchKernelGGL(k_set_add, dim3(std::min<uint64_t>(div_up(n, 256), 8192)), dim3(256), 0, set->ctx->stream,
                     set->words, d_vals, n);
  SG_HIP(hipGetLastError());
  return SG_OK;
}
}  // namespace sg

extern "C" {

int sg_set_export(sg_set* set, uint32_t* out, size_t cap, size_t* n) {
  if (!set || !n || (cap && !out)) return SG_EINVAL;
  sg_ctx* ctx = set->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  uint64_t* bases;
  uint64_t total = 0;
  rc = set_tile_bases(set, &bases, &total);
  if (rc) return rc;
  *n = (size_t)total;
  uint64_t m = total < cap ? total : cap;
  if (m == 0) return SG_OK;
  // output staged in the workspace after the scan area
  size_t used = ((kSetWords / kTile) * 4 + 255) / 256 * 256 + (((kSetWords / kTile) + 1) * 8 + 255) / 256 * 256;
  size_t o_out = used + scan_ws_bytes(kSetWords / kTile);
  o_out = (o_out + 255) & ~size_t(255);
  rc = ws_reserve(ctx, o_out + m * 4);
  if (rc) return rc;
  // ws may have been reallocated: recompute the tile bases if so
  rc = set_tile_bases(set, &bases, &total);
  if (rc) return rc;
  uint32_t* dout = (uint32_t*)ws_at(ctx, o_out);
  hipLaunchKernelGGL(k_set_export, dim3((uint32_t)(kSetWords / kTile)), dim3(kBlock), 0, ctx->stream, set->words,
                     bases, dout, (uint64_t)m);
  SG_HIP(hipGetLastError());
  SG_HIP(hipMemcpyAsync(out, dout, m * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

int sg_set_add(sg_set* set, const uint32_t* sig, size_t n) {
  if (!set || (n && !sig)) return SG_EINVAL;
  if (n == 0) return SG_OK;
  sg_ctx* ctx = set->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  rc = ws_reserve(ctx, n * 4);
  if (rc) return rc;
  uint32_t* d = (uint32_t*)ctx->ws;
  SG_HIP(hipMemcpyAsync(d, sig, n * 4, hipMemcpyHostToDevice, ctx->stream));
  {
    ScopedTimer tm(ctx, "set_add");
    hipLaunchKernelGGL(k_set_add, dim3(std::min<uint64_t>(div_up(n, 256), 8192)), dim3(256), 0, ctx->stream,
                       set->words, d, (uint64_t)n);
  }
  SG_HIP(hipGetLastError());
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

int sg_set_new(sg_set* set, const uint32_t* sig, size_t n, int* out) {
  if (!set || !out || (n && !sig)) return SG_EINVAL;
  *out = 0;
  if (n == 0) return SG_OK;
  sg_ctx* ctx = set->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  rc = ws_reserve(ctx, n * 4);
  if (rc) return rc;
  uint32_t* d = (uint32_t*)ctx->ws;
  SG_HIP(hipMemcpyAsync(d, sig, n * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemsetAsync(ctx->dscal, 0, 8, ctx->stream));
  hipLaunchKernelGGL(k_set_new, dim3(std::min<uint64_t>(div_up(n, 256), 8192)), dim3(256), 0, ctx->stream,
                     set->words, d, (uint64_t)n, ctx->dscal);
  SG_HIP(hipGetLastError());
  uint64_t flag = 0;
  SG_HIP(hipMemcpyAsync(&flag, ctx->dscal, 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  *out = flag ? 1 : 0;
  return SG_OK;
}

}  // extern "C"
