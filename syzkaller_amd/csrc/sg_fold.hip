// sg_fold.hip -- the manager's corpus / cover aggregation.
//
// Reference: the cover.Union folds of syz-manager, all of the shape
//   var cov cover.Cover
//   for _, inp := range <inputs> { cov = cover.Union(cov, inp.Cover) }
// at syz-manager/html.go:84 (per syscall: the corpus grouped by inp.Call),
// :94 (over those per-call covers), :184 (/cover: the corpus, or one call's
// inputs) and :306 (/rawcover: the whole corpus), and the same-hash merge
// manager.go:916-917.  Union (cover.go:63-70) keeps max(a, b) copies of a value
// seen a and b times and drops 0xFFFFFFFF (cover.go:97), so a fold is: every
// value with its largest count over the folded lists, ascending, sentinel
// dropped -- associative and commutative.  The reference walks the inputs one
// after another, O(inputs x |cov|) element copies; here the lists of every
// group are merged pairwise in a balanced tree, one batched Union launch per
// level over all groups (merge_dev, sg_merge.hip), O(N log inputs).
#include "sg_internal.h"

#include <algorithm>

namespace sg {

int merge_dev(sg_ctx* ctx, int op, const uint32_t* da, const uint32_t* db, uint32_t* dout, const uint64_t* a_beg,
              const uint64_t* a_len, const uint64_t* b_beg, const uint64_t* b_len, const uint64_t* out_beg,
              size_t npair, uint64_t* out_len);

namespace {

// dst[dst_off[k] ..] = src[src_beg[k] .. + len[k]), one wave per segment
__global__ void k_fold_pack(const uint32_t* __restrict__ src, const uint64_t* __restrict__ src_beg,
                            const uint64_t* __restrict__ len, const uint64_t* __restrict__ dst_off, uint64_t n,
                            uint32_t* __restrict__ dst) {
  const uint64_t k = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (k >= n) return;
  const uint64_t s = src_beg[k], d = dst_off[k], L = len[k];
  for (uint64_t i = threadIdx.x & 63; i < L; i += 64) dst[d + i] = src[s + i];
}

struct Item {
  uint64_t beg, len;
};

}  // namespace
}  // namespace sg

using namespace sg;

extern "C" {

int sg_union_fold(sg_ctx* ctx, const uint32_t* vals, const uint64_t* off, size_t n, const uint32_t* group,
                  size_t ngroups, uint32_t* out_vals, size_t cap, uint64_t* out_off) {
  if (!ctx || !off || !out_off || ngroups == 0 || (off[n] && !vals)) {
    set_error("sg_union_fold: invalid argument");
    return SG_EINVAL;
  }
  if (off[0] != 0) {
    set_error("sg_union_fold: off[0] != 0");
    return SG_EINVAL;
  }
  for (size_t k = 0; k < n; k++) {
    if (off[k + 1] < off[k] || (group && group[k] >= ngroups)) {
      set_error("sg_union_fold: list %zu: bad offsets or group", k);
      return SG_EINVAL;
    }
  }
  const uint64_t N = off[n];
  // the lists of each group, in input order (the order does not change the result)
  std::vector<std::vector<Item>> items(ngroups);
  for (size_t k = 0; k < n; k++) items[group ? group[k] : 0].push_back({off[k], off[k + 1] - off[k]});
  std::fill(out_off, out_off + ngroups + 1, 0);
  if (N == 0) return SG_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  // two ping-pong buffers of N values: a level's results never exceed its inputs
  const size_t b_v = (N * 4 + 255) & ~size_t(255);
  rc = dstage_reserve(ctx, 2 * b_v + 4 * ((ngroups + 1) * 8 + 256));
  if (rc) return rc;
  uint32_t* buf[2] = {(uint32_t*)ctx->dstage, (uint32_t*)((char*)ctx->dstage + b_v)};
  SG_HIP(hipMemcpyAsync(buf[0], vals, N * 4, hipMemcpyHostToDevice, ctx->stream));
  int cur = 0;
  std::vector<uint64_t> ab, al, bb, bl, ob, ol;
  std::vector<std::pair<size_t, size_t>> who;  // (group, new item index) of each pair
  // level 0 puts every list through one Union (Union(nil, c) drops 0xFFFFFFFF,
  // as the reference's first step does); later levels pair the survivors
  for (bool first = true;; first = false) {
    ab.clear(), al.clear(), bb.clear(), bl.clear(), ob.clear(), who.clear();
    uint64_t pos = 0;
    std::vector<std::vector<Item>> next(ngroups);
    for (size_t gi = 0; gi < ngroups; gi++) {
      const auto& it = items[gi];
      if (it.empty() || (!first && it.size() == 1)) {
        if (!it.empty()) {  // carried over: copied to the other buffer below
          ab.push_back(it[0].beg), al.push_back(it[0].len), bb.push_back(0), bl.push_back(0), ob.push_back(pos);
          who.push_back({gi, next[gi].size()});
          next[gi].push_back({pos, 0});
          pos += it[0].len;
        }
        continue;
      }
      for (size_t i = 0; i < it.size(); i += 2) {
        const Item a = it[i], b = i + 1 < it.size() ? it[i + 1] : Item{0, 0};
        ab.push_back(a.beg), al.push_back(a.len), bb.push_back(b.beg), bl.push_back(b.len), ob.push_back(pos);
        who.push_back({gi, next[gi].size()});
        next[gi].push_back({pos, 0});
        pos += a.len + b.len;
      }
    }
    bool more = false;
    for (size_t gi = 0; gi < ngroups; gi++) more |= items[gi].size() > 1;
    if (!first && !more) break;  // every group is down to its fold
    ol.assign(ab.size(), 0);
    if (!ab.empty()) {
      ScopedTimer tm(ctx, "union_fold");
      rc = merge_dev(ctx, SG_OP_UNION, buf[cur], buf[cur], buf[1 - cur], ab.data(), al.data(), bb.data(), bl.data(),
                     ob.data(), ab.size(), ol.data());
      if (rc) return rc;
    }
    for (size_t p = 0; p < who.size(); p++) next[who[p].first][who[p].second].len = ol[p];
    items.swap(next);
    cur = 1 - cur;
  }
  // pack the folds: group g at out_off[g]
  std::vector<uint64_t> beg(ngroups, 0), len(ngroups, 0);
  for (size_t gi = 0; gi < ngroups; gi++) {
    if (!items[gi].empty()) beg[gi] = items[gi][0].beg, len[gi] = items[gi][0].len;
    out_off[gi + 1] = out_off[gi] + len[gi];
  }
  if (out_off[ngroups] > cap) {
    set_error("sg_union_fold: %llu values, capacity %zu", (unsigned long long)out_off[ngroups], cap);
    return SG_EINVAL;
  }
  if (out_off[ngroups] == 0) return SG_OK;
  if (!out_vals) return SG_EINVAL;
  const size_t b_o = ((ngroups + 1) * 8 + 255) & ~size_t(255);
  uint64_t* dmeta = (uint64_t*)((char*)ctx->dstage + 2 * b_v);
  uint64_t *dbeg = dmeta, *dlen = (uint64_t*)((char*)dmeta + b_o), *doff = (uint64_t*)((char*)dmeta + 2 * b_o);
  SG_HIP(hipMemcpyAsync(dbeg, beg.data(), ngroups * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dlen, len.data(), ngroups * 8, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(doff, out_off, ngroups * 8, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_fold_pack, dim3(div_up(ngroups, 4)), dim3(256), 0, ctx->stream, buf[cur], dbeg, dlen, doff,
                     (uint64_t)ngroups, buf[1 - cur]);
  SG_HIP(hipGetLastError());
  SG_HIP(hipMemcpyAsync(out_vals, buf[1 - cur], out_off[ngroups] * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

}  // extern "C"
