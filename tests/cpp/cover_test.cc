// tests/cpp/cover_test.cc -- pkg/cover/cover_test.go restated against the C++
// host mirror (include/syzsig_cover.hpp) running on the MI355X.
//
// runTest (cover_test.go:31-58): inputs/outputs sorted, symmetric cases
// mirrored, the empty case added, two empty results equal.  The known-answer
// tables come from tests/golden/cover_kats.json (converted to a line format by
// tests/test_gpu_cpp.py, argv[1]); the random tests mirror TestMinimizeRandom
// (:178-208) and TestHasDifference (:210-221) with a fixed seed.
#include <algorithm>
#include <cstdio>
#include <fstream>
#include <map>
#include <random>
#include <sstream>
#include <string>

#include "syzsig_cover.hpp"

using syz::cover::Cover;
namespace cv = syz::cover;

static int failures = 0;
#define EXPECT(cond, ...)                \
  do {                                   \
    if (!(cond)) {                       \
      std::fprintf(stderr, __VA_ARGS__); \
      std::fprintf(stderr, "\n");        \
      failures++;                        \
    }                                    \
  } while (0)

static std::vector<uint32_t> nums(const std::string& s) {
  std::vector<uint32_t> v;
  std::istringstream in(s);
  uint64_t x;
  while (in >> x) v.push_back((uint32_t)x);
  return v;
}

static std::string show(const Cover& c) {
  std::string s = "{";
  for (size_t i = 0; i < c.size(); i++) s += (i ? " " : "") + std::to_string(c[i]);
  return s + "}";
}

struct Case {
  Cover v0, v1, r;
};

static void runTest(const std::string& name, Cover (*f)(const Cover&, const Cover&), bool sorted, bool symmetric,
                    std::vector<Case> tests) {
  if (symmetric) {
    size_t n = tests.size();
    for (size_t i = 0; i < n; i++) tests.push_back({tests[i].v1, tests[i].v0, tests[i].r});
  }
  tests.push_back({{}, {}, {}});
  for (const Case& t : tests) {
    if (sorted) {
      EXPECT(std::is_sorted(t.v0.begin(), t.v0.end()), "%s: input is not sorted", name.c_str());
      EXPECT(std::is_sorted(t.v1.begin(), t.v1.end()), "%s: input is not sorted", name.c_str());
    }
    Cover res = f(t.v0, t.v1);
    EXPECT(std::is_sorted(res.begin(), res.end()), "%s: output is not sorted", name.c_str());
    EXPECT((res.empty() && t.r.empty()) || res == t.r, "%s: f(%s, %s) = %s (expect: %s)", name.c_str(),
           show(t.v0).c_str(), show(t.v1).c_str(), show(res).c_str(), show(t.r).c_str());
  }
}

static Cover canon(const Cover& a, const Cover&) {
  std::vector<uint32_t> v(a);
  return cv::Canonicalize(v);
}
static Cover diff(const Cover& a, const Cover& b) { return cv::Difference(a, b); }
static Cover symdiff(const Cover& a, const Cover& b) { return cv::SymmetricDifference(a, b); }
static Cover uni(const Cover& a, const Cover& b) { return cv::Union(a, b); }
static Cover inter(const Cover& a, const Cover& b) { return cv::Intersection(a, b); }

static Cover randCover(std::mt19937_64& rnd, int maxLen) {  // cover_test.go:170-176
  std::vector<uint32_t> tmp(rnd() % (uint64_t)maxLen);
  for (auto& x : tmp) x = (uint32_t)(rnd() % 100);
  return cv::Canonicalize(tmp);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: cover_test <kats.txt>\n");
    return 2;
  }
  std::map<std::string, Cover (*)(const Cover&, const Cover&)> fns = {
      {"TestCanonicalize", canon}, {"TestDifference", diff}, {"TestSymmetricDifference", symdiff},
      {"TestUnion", uni}, {"TestIntersection", inter}};
  std::map<std::string, std::vector<Case>> tables;
  std::map<std::string, std::pair<bool, bool>> flags;
  std::vector<std::pair<std::vector<Cover>, std::vector<int>>> minimize;
  std::ifstream in(argv[1]);
  std::string line;
  while (std::getline(in, line)) {
    std::vector<std::string> f;
    size_t p = 0, q;
    while ((q = line.find('|', p)) != std::string::npos) {
      f.push_back(line.substr(p, q - p));
      p = q + 1;
    }
    f.push_back(line.substr(p));
    std::istringstream head(f[0]);
    std::string name;
    int so = 0, sy = 0;
    head >> name >> so >> sy;
    if (name == "TestMinimize") {
      std::vector<Cover> covs;
      std::string c;
      std::istringstream cs(f[1]);
      while (std::getline(cs, c, ';')) covs.push_back(nums(c));
      auto out = nums(f[2]);
      minimize.push_back({covs, std::vector<int>(out.begin(), out.end())});
      continue;
    }
    tables[name].push_back({nums(f[1]), nums(f[2]), nums(f[3])});
    flags[name] = {so != 0, sy != 0};
  }
  for (auto& [name, cases] : tables) runTest(name, fns.at(name), flags[name].first, flags[name].second, cases);
  for (auto& [inp, out] : minimize) {  // TestMinimize, cover_test.go:158-167
    auto res = cv::Minimize(inp);
    EXPECT(res == out, "Minimize: got %zu indices, expect %zu", res.size(), out.size());
  }
  std::mt19937_64 rnd(20171012);
  for (int i = 0; i < 300; i++) {  // TestMinimizeRandom
    int n = (int)(rnd() % 20);
    std::vector<Cover> cov(n);
    for (auto& c : cov) c = randCover(rnd, 10);
    Cover total, minimized;
    for (auto& c : cov) total = cv::Union(total, c);
    for (int idx : cv::Minimize(cov)) minimized = cv::Union(minimized, cov[idx]);
    EXPECT(total == minimized, "MinimizeRandom: better luck next time");
  }
  for (int i = 0; i < 300; i++) {  // TestHasDifference
    Cover c1 = randCover(rnd, 20), c2 = randCover(rnd, 20);
    EXPECT((cv::Difference(c1, c2).size() != 0) == cv::HasDifference(c1, c2), "HasDifference mismatch");
  }
  // signal maps (cover.go:160-182) and the batched execute() loop
  cv::SignalMap maxSignal, newSignal;
  cv::SignalAdd(maxSignal, {1, 2, 3});
  EXPECT(!cv::SignalNew(maxSignal, {3, 2, 1, 1}), "SignalNew on known signal");
  EXPECT(cv::SignalNew(maxSignal, {3, 9}), "SignalNew on new signal");
  EXPECT((cv::SignalDiff(maxSignal, {9, 3, 9, 4}) == std::vector<uint32_t>{9, 9, 4}), "SignalDiff order/dups");
  syz::Records recs;
  recs.Append({1, 5, 5});
  recs.Append({5, 6});
  recs.Append({});
  recs.Append({6, 7, 1});
  auto t = syz::fuzzer::Execute(maxSignal, &newSignal, recs);
  EXPECT((t.queued == std::vector<uint8_t>{1, 1, 0, 1}), "Execute queued");
  EXPECT((t.diff == std::vector<uint32_t>{5, 5, 6, 7}), "Execute diff");
  EXPECT((newSignal.Export() == std::vector<uint32_t>{5, 6, 7}), "newSignal");
  EXPECT(maxSignal.size() == 6, "maxSignal size");
  // executor output reader (ipc_linux.go:168-307): program 0 runs call 1 then
  // call 0; program 1 claims call index 5 of 2 (the Go reader's index error)
  std::vector<uint32_t> out = {2, 1, 20, 14, 1, 2, 1, 0, 7, 8, 0x81000010,
                               0, 10, 0, 0, 1, 0, 0, 9,
                               1, 5, 0, 0, 0, 0, 0, 0};
  auto ci = syz::ipc::ReadOutBatch(out, {0, 19, 27}, {0, 2, 4}, {10, 20, 0, 0});
  EXPECT((ci.status == std::vector<int32_t>{SG_IPC_OK, SG_IPC_BAD_INDEX}), "ReadOutBatch status");
  EXPECT((ci.errno_ == std::vector<int64_t>{0, 14, -1, -1}), "ReadOutBatch errno");
  EXPECT((ci.fault == std::vector<uint8_t>{0, 1, 0, 0}), "ReadOutBatch fault");
  EXPECT((ci.signal.vals == std::vector<uint32_t>{9, 7, 8}), "ReadOutBatch signal");
  EXPECT((ci.signal.off == std::vector<uint64_t>{0, 1, 3, 3, 3}), "ReadOutBatch signal offsets");
  EXPECT((ci.cover.vals == std::vector<uint32_t>{0x81000010}), "ReadOutBatch cover");
  if (failures) {
    std::fprintf(stderr, "FAIL: %d\n", failures);
    return 1;
  }
  std::printf("PASS\n");
  return 0;
}
