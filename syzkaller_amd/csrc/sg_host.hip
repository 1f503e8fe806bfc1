// sg_host.hip -- the host entry points' ingest of a batch that lives in host
// memory.
//
// In the reference the call signal is born in host memory: the executor's
// shared-memory output, sliced by pkg/ipc/ipc_linux.go:247 (info[i].Signal =
// out[:n:n]) and consumed by syz-fuzzer/fuzzer.go:661-666.  So every batch the
// Go adapter hands to sg_triage_batch / sg_triage_traces crosses PCIe; at C2
// size that is 3.5 GB against 6.7 ms of kernels.  One pageable
// hipMemcpyAsync of the whole batch runs at the runtime's staging rate (21-23
// GB/s on the MI355X box, profiles/r04_micro_h2d.txt) and leaves the GPU idle
// meanwhile.  Here the batch goes through in record slices:
//
//   host    slice i's values copied by host_copy_threads() threads into
//           pinned buffer i % 2 (pageable -> pinned at 72-88 GB/s with 4
//           threads on an idle box; half the cgroup CPU share by default),
//           its record offsets rebased to the slice;
//   copy    DMA of pinned buffer i % 2 into device buffer i % 2 on the
//           context's copy stream (57.5 GB/s from pinned memory);
//   compute the slice's triage on the context's stream.
//
// Slice i+1's host copy and DMA overlap slice i's triage, so the call runs at
// about the DMA rate.  Cutting a batch between two records is exact: the
// sequential loop (fuzzer.go:665) sees the same maxSignal at every record
// whether or not the batch is cut there.
#include "sg_internal.h"

#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>

namespace sg {

constexpr uint64_t kHostSliceDefault = 64ull << 20;  // entries per slice (256 MB of values)
constexpr int kCopyThreadsMax = 16;

// CPUs this process may use: the cgroup v2 quota (cpu.max), else the
// affinity mask (read once, at context creation)
double host_cpu_quota() {
  double q = 0;
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char a[32] = {0};
    unsigned long long per = 0;
    if (fscanf(f, "%31s %llu", a, &per) == 2 && strcmp(a, "max") != 0 && per) q = strtod(a, nullptr) / (double)per;
    fclose(f);
  }
  cpu_set_t cs;
  if (sched_getaffinity(0, sizeof(cs), &cs) == 0) {
    const double n = (double)CPU_COUNT(&cs);
    if (q <= 0 || n < q) q = n;
  }
  return q > 0 ? q : 1;
}

// pageable -> pinned copy threads: the option, else half the CPU share (the
// other half stays with the caller's own threads), 2..16
int host_copy_threads(const sg_ctx* ctx) {
  if (ctx->opt[kOptHostCopyThreads] > 0) return (int)std::min<int64_t>(64, ctx->opt[kOptHostCopyThreads]);
  return std::max(2, std::min(kCopyThreadsMax, (int)(ctx->cpu_quota / 2)));
}

static uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// memcpy by up to `threads` host threads (the calling one included)
static void par_copy(void* dst, const void* src, size_t bytes, int threads) {
  const size_t kMin = 8u << 20;  // below this one thread is faster than starting others
  int t = (int)std::min<size_t>((size_t)threads, std::max<size_t>(1, bytes / kMin));
  if (t <= 1) {
    memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> th;
  const size_t part = (bytes / t + 4095) & ~size_t(4095);
  for (int i = 1; i < t; i++) {
    const size_t lo = part * i;
    if (lo >= bytes) break;
    const size_t n = std::min(part, bytes - lo);
    th.emplace_back([=] { memcpy((char*)dst + lo, (const char*)src + lo, n); });
  }
  memcpy(dst, src, std::min(part, bytes));
  for (auto& x : th) x.join();
}

struct HostSlice {
  uint64_t r0, r1, e0, e1;
};

int host_pipeline(sg_ctx* ctx, uint32_t* mwords, uint32_t* nwords, const uint32_t* vals, const uint64_t* rec_off,
                  uint64_t nrec, uint8_t* rec_new, bool trace) {
  const uint64_t S = ctx->opt[kOptHostSlice] > 0 ? (uint64_t)ctx->opt[kOptHostSlice] : kHostSliceDefault;
  const int threads = host_copy_threads(ctx);
  // record slices of <= S entries (or one record, when it alone holds more)
  std::vector<HostSlice> sl;
  uint64_t max_n = 1, max_r = 1;
  for (uint64_t r0 = 0; r0 < nrec;) {
    const uint64_t e0 = rec_off[r0];
    // largest r1 with rec_off[r1] - e0 <= S, at least r0 + 1
    uint64_t r1 = (uint64_t)(std::upper_bound(rec_off + r0 + 1, rec_off + nrec + 1, e0 + S) - rec_off) - 1;
    if (r1 <= r0) r1 = r0 + 1;
    r1 = std::min(r1, r0 + ctx->max_launch_recs);  // one partitioned launch per slice (no host syncs inside)
    sl.push_back({r0, r1, e0, rec_off[r1]});
    max_n = std::max(max_n, rec_off[r1] - e0);
    max_r = std::max(max_r, r1 - r0);
    r0 = r1;
  }
  const size_t b_vals = (max_n * 4 + 255) & ~size_t(255), b_off = ((max_r + 1) * 8 + 255) & ~size_t(255);
  const size_t b_slot = b_vals + b_off, b_flag = (nrec + 256) & ~size_t(255);
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  // (the staging buffers may still be read by an earlier call's copies)
  if (ctx->copy_stream) SG_HIP(hipStreamSynchronize(ctx->copy_stream));
  rc = pin_reserve(ctx, 2 * b_slot);
  if (rc) return rc;
  rc = dstage_reserve(ctx, 2 * b_slot + b_flag);
  if (rc) return rc;
  if (!ctx->copy_stream) {
    SG_HIP(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    for (auto& e : ctx->pipe_ev) SG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  ctx->host_copy_bytes = ctx->host_copy_ns = ctx->host_wait_ns = 0;
  ctx->host_threads = (uint64_t)threads;
  char* pin = (char*)ctx->pin;
  char* dst = (char*)ctx->dstage;
  uint8_t* dflag = (uint8_t*)(dst + 2 * b_slot);
  hipEvent_t* ev_dma = ctx->pipe_ev;      // slot k's DMA done (pinned k free, device k filled)
  hipEvent_t* ev_tri = ctx->pipe_ev + 2;  // slot k's triage done (device k free)
  for (size_t i = 0; i < sl.size(); i++) {
    const HostSlice& s = sl[i];
    const int k = (int)(i & 1);
    char* pv = pin + k * b_slot;
    uint64_t* po = (uint64_t*)(pv + b_vals);
    char* dv = dst + k * b_slot;
    uint64_t* dof = (uint64_t*)(dv + b_vals);
    const uint64_t n = s.e1 - s.e0, nr = s.r1 - s.r0;
    const uint64_t t0 = now_ns();
    if (i >= 2) SG_HIP(hipEventSynchronize(ev_dma[k]));  // slice i-2's DMA has read pinned k
    const uint64_t t1 = now_ns();
    par_copy(pv, vals + s.e0, n * 4, threads);
    for (uint64_t r = 0; r <= nr; r++) po[r] = rec_off[s.r0 + r] - s.e0;
    const uint64_t t2 = now_ns();
    ctx->host_wait_ns += t1 - t0;
    ctx->host_copy_ns += t2 - t1;
    ctx->host_copy_bytes += n * 4 + (nr + 1) * 8;
    if (i >= 2) SG_HIP(hipStreamWaitEvent(ctx->copy_stream, ev_tri[k], 0));  // slice i-2's triage has read device k
    if (n) SG_HIP(hipMemcpyAsync(dv, pv, n * 4, hipMemcpyHostToDevice, ctx->copy_stream));
    SG_HIP(hipMemcpyAsync(dof, po, (nr + 1) * 8, hipMemcpyHostToDevice, ctx->copy_stream));
    SG_HIP(hipEventRecord(ev_dma[k], ctx->copy_stream));
    SG_HIP(hipStreamWaitEvent(ctx->stream, ev_dma[k], 0));
    rc = bucket_triage(ctx, mwords, nwords, (const uint32_t*)dv, dof, n, nr, dflag + s.r0, trace);
    if (rc) {  // (no DMA may still be reading pinned or writing device staging when this call returns)
      hipStreamSynchronize(ctx->copy_stream);
      return rc;
    }
    SG_HIP(hipEventRecord(ev_tri[k], ctx->stream));
  }
  if (nrec) SG_HIP(hipMemcpyAsync(rec_new, dflag, nrec, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

}  // namespace sg
