// syzsig_cover.hpp -- C++ host mirror of syzkaller's pkg/cover API and the
// fuzzer / manager signal loops, on top of the libsyzsig.so C-ABI (syzsig.h).
//
// Same names, argument meaning and results as the reference Go code:
//   pkg/cover/cover.go:11-182        Cover, Copy, RestorePC, Canonicalize,
//                                    Difference, SymmetricDifference, Union,
//                                    Intersection, HasDifference, Minimize,
//                                    SignalNew, SignalDiff, SignalAdd
//   syz-fuzzer/fuzzer.go:645-693     fuzzer::Execute (batched new-signal check)
//   syz-fuzzer/fuzzer.go:467-489     fuzzer::AddInputs
//   syz-manager/manager.go:907-912   manager::NewInputs
//   syz-manager/manager.go:949-956   manager::Poll
// Error behaviour: the Go callers panic on infrastructure failure
// (fuzzer.go:389-391); here every failed call throws syz::Error.
// Header-only; link with -lsyzsig.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "syzsig.h"

namespace syz {

struct Error : std::runtime_error {
  int rc;
  Error(const char* fn, int r) : std::runtime_error(std::string(fn) + ": " + sg_last_error()), rc(r) {}
};

inline void check(const char* fn, int rc) {
  if (rc != SG_OK) throw Error(fn, rc);
}

class Context {
 public:
  explicit Context(int device = 0) { check("sg_ctx_create", sg_ctx_create(device, &h_)); }
  ~Context() { sg_ctx_destroy(h_); }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  sg_ctx* get() const { return h_; }
  void Sync() { check("sg_ctx_sync", sg_ctx_sync(h_)); }
  // Process-wide default context on device 0 (what the package-level
  // functions below use, like Go's package functions).
  static Context& Default() {
    static Context c(0);
    return c;
  }

 private:
  sg_ctx* h_ = nullptr;
};

namespace cover {

using Cover = std::vector<uint32_t>;  // cover.go:11

// map[uint32]struct{} (fuzzer.go:65-68, manager.go:71-73)
class SignalMap {
 public:
  explicit SignalMap(Context& ctx = Context::Default()) : ctx_(&ctx) {
    check("sg_set_create", sg_set_create(ctx.get(), &h_));
  }
  ~SignalMap() { sg_set_destroy(h_); }
  SignalMap(const SignalMap&) = delete;
  SignalMap& operator=(const SignalMap&) = delete;
  sg_set* get() const { return h_; }
  Context& ctx() const { return *ctx_; }
  size_t size() const {
    uint64_t n = 0;
    check("sg_set_count", sg_set_count(h_, &n));
    return (size_t)n;
  }
  void clear() { check("sg_set_clear", sg_set_clear(h_)); }
  // members ascending (Go iterates in map order)
  std::vector<uint32_t> Export() const {
    size_t n = 0;
    check("sg_set_export", sg_set_export(h_, nullptr, 0, &n));
    std::vector<uint32_t> out(n);
    if (n) check("sg_set_export", sg_set_export(h_, out.data(), out.size(), &n));
    return out;
  }

 private:
  Context* ctx_;
  sg_set* h_ = nullptr;
};

inline Cover Copy(const Cover& cov) { return Cover(cov); }  // cover.go:19-21

inline uint64_t RestorePC(uint32_t pc, uint32_t base) { return ((uint64_t)base << 32) + (uint64_t)pc; }  // :23-25

// cover.go:28-40: sorts and uniques `cov` in place (its tail keeps the sorted
// values, as in Go) and returns the canonical prefix.
inline Cover Canonicalize(std::vector<uint32_t>& cov, Context& ctx = Context::Default()) {
  size_t n = 0;
  check("sg_canonicalize", sg_canonicalize(ctx.get(), cov.data(), cov.size(), &n));
  return Cover(cov.begin(), cov.begin() + n);
}

namespace detail {
inline Cover merge(int op, const Cover& a, const Cover& b, Context& ctx) {
  Cover out(a.size() + b.size());
  size_t n = 0;
  check("sg_merge", sg_merge(ctx.get(), op, a.data(), a.size(), b.data(), b.size(), out.data(), &n));
  out.resize(n);
  return out;
}
}  // namespace detail

inline Cover Difference(const Cover& a, const Cover& b, Context& ctx = Context::Default()) {  // :42-49
  return detail::merge(SG_OP_DIFFERENCE, a, b, ctx);
}
inline Cover SymmetricDifference(const Cover& a, const Cover& b, Context& ctx = Context::Default()) {  // :51-61
  return detail::merge(SG_OP_SYMDIFF, a, b, ctx);
}
inline Cover Union(const Cover& a, const Cover& b, Context& ctx = Context::Default()) {  // :63-70
  return detail::merge(SG_OP_UNION, a, b, ctx);
}
inline Cover Intersection(const Cover& a, const Cover& b, Context& ctx = Context::Default()) {  // :72-79
  return detail::merge(SG_OP_INTERSECT, a, b, ctx);
}

inline bool HasDifference(const Cover& a, const Cover& b, Context& ctx = Context::Default()) {  // :106-117
  int out = 0;
  check("sg_has_difference", sg_has_difference(ctx.get(), a.data(), a.size(), b.data(), b.size(), &out));
  return out != 0;
}

// cover.go:120-146, including its sort.Sort processing order (cover.go:128).
inline std::vector<int> Minimize(const std::vector<Cover>& corpus, Context& ctx = Context::Default()) {
  std::vector<uint64_t> off(corpus.size() + 1, 0);
  for (size_t i = 0; i < corpus.size(); i++) off[i + 1] = off[i] + corpus[i].size();
  std::vector<uint32_t> vals;
  vals.reserve(off.back());
  for (const Cover& c : corpus) vals.insert(vals.end(), c.begin(), c.end());
  std::vector<uint32_t> order(corpus.size()), sel(corpus.size());
  check("sg_minimize_order", sg_minimize_order(off.data(), corpus.size(), order.data()));
  size_t n = 0;
  check("sg_minimize", sg_minimize(ctx.get(), vals.data(), off.data(), corpus.size(), order.data(), sel.data(), &n));
  return std::vector<int>(sel.begin(), sel.begin() + n);
}

inline bool SignalNew(SignalMap& base, const std::vector<uint32_t>& signal) {  // :160-167
  int out = 0;
  check("sg_set_new", sg_set_new(base.get(), signal.data(), signal.size(), &out));
  return out != 0;
}

inline std::vector<uint32_t> SignalDiff(SignalMap& base, const std::vector<uint32_t>& signal) {  // :169-176
  std::vector<uint32_t> out(signal.size());
  size_t n = 0;
  check("sg_set_diff", sg_set_diff(base.get(), signal.data(), signal.size(), out.data(), &n));
  out.resize(n);
  return out;
}

inline void SignalAdd(SignalMap& base, const std::vector<uint32_t>& signal) {  // :178-182
  check("sg_set_add", sg_set_add(base.get(), signal.data(), signal.size()));
}

}  // namespace cover

// A batch of call records in sequential (program-major, call-index) order:
// record r's signal is vals[off[r] .. off[r+1]).
struct Records {
  std::vector<uint32_t> vals;
  std::vector<uint64_t> off{0};
  void Append(const std::vector<uint32_t>& sig) {
    vals.insert(vals.end(), sig.begin(), sig.end());
    off.push_back(vals.size());
  }
  size_t size() const { return off.size() - 1; }
};

namespace fuzzer {

// Result of execute()'s per-call loop over a batch (fuzzer.go:665-691).
struct Triage {
  std::vector<uint8_t> queued;  // record r goes to the triage queue (fuzzer.go:678-690)
  std::vector<uint32_t> diff;   // diffs (fuzzer.go:669) of all queued records, concatenated
  std::vector<uint64_t> diff_off;
};

inline Triage Execute(cover::SignalMap& maxSignal, cover::SignalMap* newSignal, const Records& recs) {
  Triage t;
  t.queued.resize(recs.size());
  t.diff.resize(recs.vals.size());
  t.diff_off.resize(recs.size() + 1);
  uint64_t nd = 0;
  check("sg_triage_batch", sg_triage_batch(maxSignal.ctx().get(), maxSignal.get(),
                                           newSignal ? newSignal->get() : nullptr, recs.vals.data(), recs.off.data(),
                                           recs.size(), t.queued.data(), t.diff.data(), t.diff_off.data(), &nd));
  t.diff.resize(nd);
  return t;
}

// fuzzer.go:467-489 addInput over a batch of inputs
inline void AddInputs(cover::SignalMap& corpusSignal, cover::SignalMap& maxSignal, const Records& inputs) {
  check("sg_add_inputs", sg_add_inputs(maxSignal.ctx().get(), corpusSignal.get(), maxSignal.get(),
                                       inputs.vals.data(), inputs.off.data(), inputs.size()));
}

}  // namespace fuzzer

namespace manager {

// manager.go:907-912 NewInput acceptance over a batch of RPCs in arrival order
inline std::vector<uint8_t> NewInputs(cover::SignalMap& corpusSignal, cover::SignalMap* corpusCover,
                                      const Records& signal, const Records* cover) {
  std::vector<uint8_t> acc(signal.size());
  check("sg_accept_batch",
        sg_accept_batch(corpusSignal.ctx().get(), corpusSignal.get(), corpusCover ? corpusCover->get() : nullptr,
                        signal.vals.data(), signal.off.data(), cover ? cover->vals.data() : nullptr,
                        cover ? cover->off.data() : nullptr, signal.size(), acc.data()));
  return acc;
}

// manager.go:949-956: newMaxSignal of each poll, in arrival order
inline Records Poll(cover::SignalMap& maxSignal, const Records& polls) {
  Records out;
  out.vals.resize(polls.vals.size());
  out.off.resize(polls.size() + 1);
  check("sg_merge_poll", sg_merge_poll(maxSignal.ctx().get(), maxSignal.get(), polls.vals.data(), polls.off.data(),
                                       polls.size(), out.vals.data(), out.off.data()));
  out.vals.resize(out.off.back());
  return out;
}

}  // namespace manager

namespace ipc {

// readOutCoverage (pkg/ipc/ipc_linux.go:168-307) over a batch of programs:
// program p's output words are out[out_off[p] .. out_off[p+1]), its calls
// records call_off[p] .. call_off[p+1]; call_nums (c.Meta.ID per record) may
// be empty to skip that check.  status[p] is SG_IPC_OK or the Go error path.
struct CallInfos {
  std::vector<int64_t> errno_;  // Errno: -1 = not executed
  std::vector<uint8_t> fault;   // FaultInjected
  std::vector<int32_t> status;  // per program
  Records signal, cover;        // per record, in record order
};

inline CallInfos ReadOutBatch(const std::vector<uint32_t>& out, const std::vector<uint64_t>& out_off,
                              const std::vector<uint64_t>& call_off, const std::vector<uint32_t>& call_nums = {},
                              Context& ctx = Context::Default()) {
  const size_t nprog = out_off.size() - 1, nrec = call_off.back();
  CallInfos r;
  r.errno_.resize(nrec);
  r.fault.resize(nrec);
  r.status.resize(nprog);
  r.signal.vals.resize(out.size());
  r.signal.off.resize(nrec + 1);
  r.cover.vals.resize(out.size());
  r.cover.off.resize(nrec + 1);
  check("sg_ipc_parse",
        sg_ipc_parse(ctx.get(), out.data(), out_off.data(), call_off.data(), call_nums.empty() ? nullptr : call_nums.data(),
                     nprog, r.errno_.data(), r.fault.data(), r.status.data(), r.signal.off.data(), r.signal.vals.data(),
                     r.cover.off.data(), r.cover.vals.data()));
  r.signal.vals.resize(r.signal.off.back());
  r.cover.vals.resize(r.cover.off.back());
  return r;
}

}  // namespace ipc
}  // namespace syz
