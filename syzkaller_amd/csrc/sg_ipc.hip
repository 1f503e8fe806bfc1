// Executor output ingest: the reader of pkg/ipc/ipc_linux.go:168-307
// (readOutCoverage) over a batch of programs, straight from their output
// regions in HBM into the per-record signal / cover CSR that the triage
// kernels consume.  The layout is the one
// executor/executor.h:369-427 writes: ncmd, then per completed call
//   callIndex, callNum, errno, faultInjected, nsig, ncover, ncomps,
//   nsig signal words, ncover cover words, ncomps comparisons
// (a comparison is its type word and two operands, 2 or 4 words).
//
// Two kernels and a scan:
//  - k_ipc_walk: one thread per program follows the record headers (the walk
//    is a chain of dependent loads by nature; ~16 headers per program) and
//    writes, per record, where its signal and cover words start and how many
//    there are, its errno and fault flag, and the program's status;
//  - scan of the counts -> sig_off / cov_off (records program-major, call
//    index ascending: the fuzzer.go:665 record order);
//  - k_ipc_gather: a wave per record copies its words into the CSR.
// Bytes: the headers (28 B per record), the signal and cover words read once
// and written once.
#include "sg_internal.h"

namespace sg {

// program status codes (include/syzsig.h SG_IPC_*), one per Go error path
enum : int32_t {
  kIpcOk = 0,
  kIpcNoNcmd = 1,        // ipc_linux.go:197-200
  kIpcShortHeader = 2,   // :216-219
  kIpcBadIndex = 3,      // :220-224
  kIpcBadCallNum = 4,    // :225-230
  kIpcDouble = 5,        // :231-235
  kIpcSignalSize = 6,    // :238-242
  kIpcCoverSize = 7,     // :247-251
  kIpcCompsShort = 8,    // :258-290 (a readOut that ran out)
  kIpcCompsType = 9,     // :266-270
};

struct IpcArgs {
  const uint32_t* out;       // all programs' output words
  const uint64_t* out_off;   // [nprog+1] word offsets of each program's region
  const uint64_t* call_off;  // [nprog+1] record offsets (len(p.Calls) per program)
  const uint32_t* call_nums; // [nrec] c.Meta.ID per record, or null (no check)
  uint64_t nprog;
  int64_t* err;              // [nrec] Errno: -1 = not executed, else the u32 errno
  uint8_t* fault;            // [nrec] FaultInjected
  int32_t* status;           // [nprog]
  uint64_t* sig_src;         // [nrec] word position of the record's signal
  uint32_t* sig_cnt;         // [nrec]
  uint64_t* cov_src;         // [nrec]
  uint32_t* cov_cnt;         // [nrec]
  uint8_t* seen;             // [nrec] workspace: Signal != nil
};

__global__ void k_ipc_walk(IpcArgs a) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.nprog) return;
  const uint64_t r0 = a.call_off[p], r1 = a.call_off[p + 1], ncalls = r1 - r0;
  for (uint64_t r = r0; r < r1; r++) {  // ipc_linux.go:202-205: Errno -1, not executed
    a.err[r] = -1;
    a.fault[r] = 0;
    a.sig_cnt[r] = 0;
    a.cov_cnt[r] = 0;
    a.sig_src[r] = 0;
    a.cov_src[r] = 0;
    a.seen[r] = 0;
  }
  uint64_t pos = a.out_off[p];
  const uint64_t end = a.out_off[p + 1];
  const uint32_t* w = a.out;
  int32_t st = kIpcOk;
  if (pos >= end) {
    a.status[p] = kIpcNoNcmd;
    return;
  }
  const uint32_t ncmd = w[pos++];
  for (uint32_t i = 0; i < ncmd && st == kIpcOk; i++) {
    if (end - pos < 7) {
      st = kIpcShortHeader;
      break;
    }
    const uint32_t idx = w[pos], num = w[pos + 1], errno_ = w[pos + 2], fi = w[pos + 3], nsig = w[pos + 4],
                   ncov = w[pos + 5], ncomps = w[pos + 6];
    pos += 7;
    if (idx >= ncalls) {
      st = kIpcBadIndex;
      break;
    }
    const uint64_t r = r0 + idx;
    if (a.call_nums && a.call_nums[r] != num) {
      st = kIpcBadCallNum;
      break;
    }
    if (a.seen[r]) {
      st = kIpcDouble;
      break;
    }
    a.err[r] = (int64_t)errno_;
    a.fault[r] = fi != 0;
    if (nsig > end - pos) {
      st = kIpcSignalSize;
      break;
    }
    a.seen[r] = 1;
    a.sig_src[r] = pos;
    a.sig_cnt[r] = nsig;
    pos += nsig;
    if (ncov > end - pos) {
      st = kIpcCoverSize;
      break;
    }
    a.cov_src[r] = pos;
    a.cov_cnt[r] = ncov;
    pos += ncov;
    // comparisons: walked, not decoded (hints are outside the signal path).
    // The widths are the reader's (ipc_linux.go:272-287): two words when
    // (typ & 6) == 6, four otherwise.
    for (uint32_t j = 0; j < ncomps; j++) {
      if (pos >= end) {
        st = kIpcCompsShort;
        break;
      }
      const uint32_t typ = w[pos++];
      if (typ > 7u) {
        st = kIpcCompsType;
        break;
      }
      const uint64_t k = (typ & 6u) == 6u ? 2 : 4;
      if (end - pos < k) {
        st = kIpcCompsShort;
        break;
      }
      pos += k;
    }
  }
  a.status[p] = st;
  // A program whose output failed to parse contributes no signal or cover:
  // execute1 retries it or panics, and never hands its info to the triage
  // loop (syz-fuzzer/fuzzer.go:752-768).  Its records keep their errno /
  // fault (the reader's partial state) but get empty CSR slices, so the CSR
  // is sg_triage_batch's input as is.
  if (st != kIpcOk)
    for (uint64_t r = r0; r < r1; r++) {
      a.sig_cnt[r] = 0;
      a.cov_cnt[r] = 0;
    }
}

// a wave per record: its words from the output region into the CSR
__global__ __launch_bounds__(256) void k_ipc_gather(const uint32_t* __restrict__ out, const uint64_t* __restrict__ src,
                                                    const uint64_t* __restrict__ off, uint64_t nrec,
                                                    uint32_t* __restrict__ vals) {
  const uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nrec) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t n = off[r + 1] - off[r], s = src[r], d = off[r];
  uint64_t i = lane;
  // eight loads in flight per lane before their stores
  for (; i + 7 * 64 < n; i += 8 * 64) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = __builtin_nontemporal_load(out + s + i + 64 * k);
#pragma unroll
    for (int k = 0; k < 8; k++) vals[d + i + 64 * k] = v[k];
  }
  for (; i < n; i += 64) vals[d + i] = out[s + i];
}

}  // namespace sg

using namespace sg;

extern "C" {

int sg_ipc_parse_dev(sg_ctx* ctx, const uint32_t* d_out, const uint64_t* d_out_off, const uint64_t* d_call_off,
                     const uint32_t* d_call_nums, uint64_t nprog, uint64_t nrec, int64_t* d_errno, uint8_t* d_fault,
                     int32_t* d_status, uint64_t* d_sig_off, uint32_t* d_sig_vals, uint64_t* d_cov_off,
                     uint32_t* d_cov_vals) {
  if (!ctx || !d_out_off || !d_call_off || !d_sig_off || !d_sig_vals || (nprog && !d_status) ||
      (nrec && (!d_errno || !d_fault)) || (!d_cov_off != !d_cov_vals))
    return SG_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  if (nrec == 0) {
    SG_HIP(hipMemsetAsync(d_sig_off, 0, 8, ctx->stream));
    if (d_cov_off) SG_HIP(hipMemsetAsync(d_cov_off, 0, 8, ctx->stream));
  }
  WsPlan p;
  const size_t o_ss = p.add(nrec * 8), o_sc = p.add(nrec * 4), o_cs = p.add(nrec * 8), o_cc = p.add(nrec * 4),
               o_seen = p.add(nrec);
  const size_t scan_off = p.total;
  rc = ws_reserve(ctx, p.total + scan_ws_bytes(nrec ? nrec : 1));
  if (rc) return rc;
  IpcArgs a{};
  a.out = d_out;
  a.out_off = d_out_off;
  a.call_off = d_call_off;
  a.call_nums = d_call_nums;
  a.nprog = nprog;
  a.err = d_errno;
  a.fault = d_fault;
  a.status = d_status;
  a.sig_src = (uint64_t*)ws_at(ctx, o_ss);
  a.sig_cnt = (uint32_t*)ws_at(ctx, o_sc);
  a.cov_src = (uint64_t*)ws_at(ctx, o_cs);
  a.cov_cnt = (uint32_t*)ws_at(ctx, o_cc);
  a.seen = (uint8_t*)ws_at(ctx, o_seen);
  if (nprog) {
    ScopedTimer tm(ctx, "ipc_walk");
    hipLaunchKernelGGL(k_ipc_walk, dim3(div_up(nprog, 64)), dim3(64), 0, ctx->stream, a);
  }
  SG_HIP(hipGetLastError());
  if (nrec == 0) return SG_OK;
  rc = scan_counts(ctx, a.sig_cnt, d_sig_off, nrec, scan_off);
  if (rc) return rc;
  {
    ScopedTimer tm(ctx, "ipc_gather");
    hipLaunchKernelGGL(k_ipc_gather, dim3(div_up(nrec, 4)), dim3(256), 0, ctx->stream, d_out, a.sig_src, d_sig_off,
                       nrec, d_sig_vals);
  }
  SG_HIP(hipGetLastError());
  if (d_cov_off) {
    rc = scan_counts(ctx, a.cov_cnt, d_cov_off, nrec, scan_off);
    if (rc) return rc;
    ScopedTimer tm(ctx, "ipc_gather");
    hipLaunchKernelGGL(k_ipc_gather, dim3(div_up(nrec, 4)), dim3(256), 0, ctx->stream, d_out, a.cov_src, d_cov_off,
                       nrec, d_cov_vals);
  }
  SG_HIP(hipGetLastError());
  return SG_OK;
}

int sg_ipc_parse(sg_ctx* ctx, const uint32_t* out, const uint64_t* out_off, const uint64_t* call_off,
                 const uint32_t* call_nums, size_t nprog, int64_t* err, uint8_t* fault, int32_t* status,
                 uint64_t* sig_off, uint32_t* sig_vals, uint64_t* cov_off, uint32_t* cov_vals) {
  if (!ctx || !out_off || !call_off || !sig_off || (!cov_off != !cov_vals)) return SG_EINVAL;
  const uint64_t nwords = out_off[nprog], nrec = call_off[nprog];
  if (out_off[0] != 0 || call_off[0] != 0 || (nwords && (!out || !sig_vals || (cov_off && !cov_vals))) ||
      (nprog && !status) || (nrec && (!err || !fault)))
    return SG_EINVAL;
  for (size_t q = 0; q < nprog; q++)
    if (out_off[q + 1] < out_off[q] || call_off[q + 1] < call_off[q]) return SG_EINVAL;
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t bw = al(nwords * 4 + 4), bo = al((nprog + 1) * 8), br8 = al((nrec + 1) * 8), br4 = al(nrec * 4 + 4),
               br1 = al(nrec + 1), bp = al(nprog * 4 + 4);
  char* st = nullptr;
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    int rc = ensure_device(ctx);
    if (rc) return rc;
    rc = dstage_reserve(ctx, 3 * bw + 2 * bo + 3 * br8 + br4 + br1 + bp + 256);
    if (rc) return rc;
    st = (char*)ctx->dstage;
  }
  uint32_t* dw = (uint32_t*)st;
  uint32_t* dsv = (uint32_t*)(st + bw);
  uint32_t* dcv = (uint32_t*)(st + 2 * bw);
  char* q = st + 3 * bw;
  uint64_t* doo = (uint64_t*)q;
  uint64_t* dco = (uint64_t*)(q + bo);
  uint64_t* derr = (uint64_t*)(q + 2 * bo);
  uint64_t* dso = (uint64_t*)(q + 2 * bo + br8);
  uint64_t* dcvo = (uint64_t*)(q + 2 * bo + 2 * br8);
  uint32_t* dnum = (uint32_t*)(q + 2 * bo + 3 * br8);
  uint8_t* dfi = (uint8_t*)(q + 2 * bo + 3 * br8 + br4);
  int32_t* dst = (int32_t*)(q + 2 * bo + 3 * br8 + br4 + br1);
  if (nwords) SG_HIP(hipMemcpyAsync(dw, out, nwords * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(doo, out_off, (nprog + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dco, call_off, (nprog + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  if (call_nums && nrec) SG_HIP(hipMemcpyAsync(dnum, call_nums, nrec * 4, hipMemcpyHostToDevice, ctx->stream));
  int rc = sg_ipc_parse_dev(ctx, dw, doo, dco, call_nums ? dnum : nullptr, nprog, nrec, (int64_t*)derr, dfi, dst, dso,
                            dsv, cov_off ? dcvo : nullptr, cov_off ? dcv : nullptr);
  if (rc) return rc;
  SG_HIP(hipMemcpyAsync(sig_off, dso, (nrec + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  if (cov_off) SG_HIP(hipMemcpyAsync(cov_off, dcvo, (nrec + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  if (nrec) {
    SG_HIP(hipMemcpyAsync(err, derr, nrec * 8, hipMemcpyDeviceToHost, ctx->stream));
    SG_HIP(hipMemcpyAsync(fault, dfi, nrec, hipMemcpyDeviceToHost, ctx->stream));
  }
  if (nprog) SG_HIP(hipMemcpyAsync(status, dst, nprog * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (sig_off[nrec]) SG_HIP(hipMemcpyAsync(sig_vals, dsv, sig_off[nrec] * 4, hipMemcpyDeviceToHost, ctx->stream));
  if (cov_off && cov_off[nrec])
    SG_HIP(hipMemcpyAsync(cov_vals, dcv, cov_off[nrec] * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

}  // extern "C"
