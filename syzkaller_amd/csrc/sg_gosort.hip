// sg_gosort.hip -- the processing order of cover.Minimize (host side).
//
// pkg/cover/cover.go:128 sorts minInputArray with sort.Sort, Less = "longer
// cover first" (cover.go:157).  sort.Sort is not stable, so for inputs of
// equal length the order (and therefore which input Minimize selects) is
// whatever Go's algorithm produces.  This reproduces the Go 1.8/1.9 `sort`
// package algorithm (introsort: median-of-three / Tukey ninther pivoting with
// a duplicate-protecting partition, ShellSort gap 6 + insertion sort below 13
// elements, heapsort past depth 2*ceil(lg(n+1))) over an index permutation,
// so sg_minimize can be fed exactly the reference's order.  Host-side
// O(n log n) on lengths only; the set work stays on the GPU (sg_minimize).
#include "sg_internal.h"

#include <vector>

namespace sg {
namespace {

class MinOrder {
 public:
  MinOrder(uint32_t* idx, const std::vector<uint64_t>& len) : p_(idx), len_(len) {}

  void sort(long n) {
    int depth = 0;
    for (long i = n; i > 0; i >>= 1) depth++;
    quick(0, n, 2 * depth);
  }

 private:
  bool less(long i, long j) const { return len_[p_[i]] > len_[p_[j]]; }
  void swap(long i, long j) { std::swap(p_[i], p_[j]); }

  void insertion(long a, long b) {
    for (long i = a + 1; i < b; i++)
      for (long j = i; j > a && less(j, j - 1); j--) swap(j, j - 1);
  }

  void sift(long lo, long hi, long first) {
    for (long root = lo;;) {
      long child = 2 * root + 1;
      if (child >= hi) return;
      if (child + 1 < hi && less(first + child, first + child + 1)) child++;
      if (!less(first + root, first + child)) return;
      swap(first + root, first + child);
      root = child;
    }
  }

  void heap(long a, long b) {
    long first = a, hi = b - a;
    for (long i = (hi - 1) / 2; i >= 0; i--) sift(i, hi, first);
    for (long i = hi - 1; i >= 0; i--) {
      swap(first, first + i);
      sift(0, i, first);
    }
  }

  void median3(long m1, long m0, long m2) {
    if (less(m1, m0)) swap(m1, m0);
    if (less(m2, m1)) {
      swap(m2, m1);
      if (less(m1, m0)) swap(m1, m0);
    }
  }

  void pivot(long lo, long hi, long& midlo, long& midhi) {
    long m = (long)((unsigned long)(lo + hi) >> 1);
    if (hi - lo > 40) {
      long s = (hi - lo) / 8;
      median3(lo, lo + s, lo + 2 * s);
      median3(m, m - s, m + s);
      median3(hi - 1, hi - 1 - s, hi - 1 - 2 * s);
    }
    median3(lo, m, hi - 1);
    const long pv = lo;
    long a = lo + 1, c = hi - 1;
    while (a < c && less(a, pv)) a++;
    long b = a;
    for (;;) {
      while (b < c && !less(pv, b)) b++;
      while (b < c && less(pv, c - 1)) c--;
      if (b >= c) break;
      swap(b, c - 1);
      b++;
      c--;
    }
    bool protect = hi - c < 5;
    if (!protect && hi - c < (hi - lo) / 4) {
      int dups = 0;
      if (!less(pv, hi - 1)) {
        swap(c, hi - 1);
        c++;
        dups++;
      }
      if (!less(b - 1, pv)) {
        b--;
        dups++;
      }
      if (!less(m, pv)) {
        swap(m, b - 1);
        b--;
        dups++;
      }
      protect = dups > 1;
    }
    if (protect) {
      for (;;) {
        while (a < b && !less(b - 1, pv)) b--;
        while (a < b && less(a, pv)) a++;
        if (a >= b) break;
        swap(a, b - 1);
        a++;
        b--;
      }
    }
    swap(pv, b - 1);
    midlo = b - 1;
    midhi = c;
  }

  void quick(long a, long b, int depth) {
    while (b - a > 12) {
      if (depth == 0) {
        heap(a, b);
        return;
      }
      depth--;
      long mlo, mhi;
      pivot(a, b, mlo, mhi);
      if (mlo - a < b - mhi) {
        quick(a, mlo, depth);
        a = mhi;
      } else {
        quick(mhi, b, depth);
        b = mlo;
      }
    }
    if (b - a > 1) {
      for (long i = a + 6; i < b; i++)
        if (less(i, i - 6)) swap(i, i - 6);
      insertion(a, b);
    }
  }

  uint32_t* p_;
  const std::vector<uint64_t>& len_;
};

}  // namespace
}  // namespace sg

extern "C" int sg_minimize_order(const uint64_t* off, size_t n, uint32_t* order) {
  if ((n && (!off || !order)) || n >= 0xFFFFFFFFull) {
    sg::set_error("sg_minimize_order: invalid argument");
    return SG_EINVAL;
  }
  std::vector<uint64_t> len(n);
  for (size_t i = 0; i < n; i++) {
    if (off[i + 1] < off[i]) {
      sg::set_error("sg_minimize_order: offsets not non-decreasing at %zu", i);
      return SG_EINVAL;
    }
    len[i] = off[i + 1] - off[i];
    order[i] = (uint32_t)i;
  }
  sg::MinOrder(order, len).sort((long)n);
  return SG_OK;
}
