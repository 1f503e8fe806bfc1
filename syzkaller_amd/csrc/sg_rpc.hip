// sg_rpc.hip -- RPC payload forms of signal and cover.
//
// Reference: pkg/rpctype/rpctype.go:8-63.  The fuzzer and the manager ship
// signal as []uint32 (gob: a varint per element, up to 5 bytes each for
// 32-bit edge signal): RpcInput.Signal / .Cover (canonical, ascending),
// ConnectRes.MaxSignal, PollArgs.MaxSignal (the fuzzer's drained newSignal,
// fuzzer.go:358-364) and PollRes.MaxSignal (manager.go:949-962).
//
// Wire form here: each sorted list as Go's binary.PutUvarint of its first
// value, then of each successive difference (LEB128: 7 bits per byte, high
// bit = more bytes follow).  A Go peer decodes it with binary.Uvarint and a
// running sum.  Encoding and decoding run on the GPU straight from / into a
// signal set's bitmap:
//   encode  lengths of the deltas' varints -> exclusive scan -> byte writes;
//   decode  a byte ends a value iff its high bit is clear; the terminators'
//           scan numbers the values, each terminator decodes its (<= 5-byte)
//           run, and a scan of the deltas restores the values.
// The sancov dump of tools/syz-execprog/execprog.go:159-177 (magic
// 0xC0BFFFFFFFFFFF64, then RestorePC(pc, 0xffffffff) per cover PC, all u64
// little-endian) is the interchange form for offline cover tooling.
#include "sg_internal.h"

#include <algorithm>

namespace sg {
namespace {

constexpr uint64_t kSancovMagic = 0xC0BFFFFFFFFFFF64ull;  // execprog.go:166

__device__ __forceinline__ uint32_t varint_len(uint32_t d) {
  return d < (1u << 7) ? 1u : d < (1u << 14) ? 2u : d < (1u << 21) ? 3u : d < (1u << 28) ? 4u : 5u;
}

// list k of the CSR holding global element i (off non-decreasing, off[0] = 0)
__device__ __forceinline__ uint64_t list_of(const uint64_t* off, uint64_t n, uint64_t i) {
  uint64_t lo = 0, hi = n - 1;  // last k with off[k] <= i
  while (lo < hi) {
    const uint64_t mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

// kw[w] = list_of(min(32 w + 31, N - 1)) for w < ceil(N / 32).  Element i's
// list lies between its word's bounds kw[w - 1] .. kw[w] (almost always one
// list), so a per-element search of the whole offset table (a chain of ~17
// dependent loads: 3-6 ms per 71M-value batch) becomes two cached loads.
__global__ void k_word_lists(const uint64_t* __restrict__ off, uint64_t n, uint64_t N, uint64_t* __restrict__ kw) {
  const uint64_t nw = (N + 31) / 32;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride)
    kw[w] = list_of(off, n, 32 * w + 31 < N ? 32 * w + 31 : N - 1);
}

__device__ __forceinline__ uint64_t list_of_w(const uint64_t* off, const uint64_t* kw, uint64_t i) {
  const uint64_t w = i >> 5;
  uint64_t lo = w ? kw[w - 1] : 0, hi = kw[w];  // off[lo] <= 32 w - 1 < i (or lo = 0)
  while (lo < hi) {
    const uint64_t mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

// delta of element i within its list (the first one: itself); err on a descent
__device__ __forceinline__ uint32_t elem_delta(const uint32_t* v, const uint64_t* off, const uint64_t* kw, uint64_t i,
                                               uint32_t* err) {
  const uint64_t k = list_of_w(off, kw, i);
  const uint32_t x = v[i];
  if (i == off[k]) return x;
  const uint32_t p = v[i - 1];
  if (x < p) *err = 1;
  return x - p;
}

// Encode: per 64-element group (one wave, lanes in element order) the bytes
// of its varints; a scan of the group totals; then each element's byte
// position = its group's base + a wave prefix sum (no per-element position
// array).  The grid-stride loops keep whole waves on whole groups.
__device__ __forceinline__ uint32_t enc_len_at(const uint32_t* v, const uint64_t* off, const uint64_t* kw, uint64_t N,
                                               uint64_t i, uint32_t* err) {
  return i < N ? varint_len(elem_delta(v, off, kw, i, err)) : 0u;
}

__global__ __launch_bounds__(256) void k_enc_len(const uint32_t* __restrict__ v, const uint64_t* __restrict__ off,
                                                 const uint64_t* __restrict__ kw, uint64_t N,
                                                 uint32_t* __restrict__ gsum, uint32_t* __restrict__ err) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); g0 < N; g0 += stride) {
    const uint32_t incl = sgd::wave_incl_add(enc_len_at(v, off, kw, N, g0 + lane, err));
    if (lane == 63) gsum[g0 >> 6] = incl;
  }
}

__global__ __launch_bounds__(256) void k_enc_write(const uint32_t* __restrict__ v, const uint64_t* __restrict__ off,
                                                   const uint64_t* __restrict__ kw, uint64_t N,
                                                   const uint64_t* __restrict__ gbase, uint8_t* __restrict__ out,
                                                   uint32_t* __restrict__ err) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); g0 < N; g0 += stride) {
    const uint64_t i = g0 + lane;
    uint32_t d = i < N ? elem_delta(v, off, kw, i, err) : 0u;
    const uint32_t len = i < N ? varint_len(d) : 0u;
    const uint32_t incl = sgd::wave_incl_add(len);
    if (i >= N) continue;
    uint8_t* o = out + gbase[g0 >> 6] + (incl - len);
    while (d >= 0x80u) {  // binary.PutUvarint
      *o++ = (uint8_t)(d | 0x80u);
      d >>= 7;
    }
    *o = (uint8_t)d;
  }
}

// Encode, one wave per list (four per workgroup): the list in steps of
// kEncRows rows of 64 values, lane L holding value 64 r + L of the step (one
// coalesced dword load per row, all of a step's rows in flight), each value's
// delta against the one before it (the lane before's by DPP; lane 0: the row
// before's lane 63, carried) and its varint length.  Pass A: the list's byte
// count (and the sortedness check); pass B, after a scan of the counts: a
// wave prefix of the row's lengths places each value's bytes, stored straight
// to the payload (store k writes byte k of every value that long: a row's
// stores cover one contiguous run).  No per-value list search.
constexpr int kEncRows = 8;
struct EncRow {
  uint32_t d, len;
};

__device__ __forceinline__ void enc_rows(const uint32_t* __restrict__ v, uint64_t cb, uint64_t e0, uint64_t e1,
                                         uint32_t lane, uint32_t& carry, EncRow (&row)[kEncRows], uint32_t& bad) {
  uint32_t x[kEncRows];
#pragma unroll
  for (int r = 0; r < kEncRows; r++) {
    const uint64_t i = cb + 64 * r + lane;
    x[r] = i < e1 ? v[i] : 0u;
  }
#pragma unroll
  for (int r = 0; r < kEncRows; r++) {
    const uint64_t i = cb + 64 * r + lane;
    const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)carry, (int)x[r], 0x138 /* wave_shr:1 */, 0xF, 0xF, false);
    carry = __builtin_amdgcn_readlane(x[r], 63);
    const bool ok = i < e1, first = i == e0;
    bad |= (uint32_t)(ok && !first && x[r] < prev);
    const uint32_t dd = first ? x[r] : x[r] - prev;
    row[r].d = ok ? dd : 0u;
    row[r].len = ok ? varint_len(dd) : 0u;
  }
}

__global__ __launch_bounds__(256) void k_enc_list_len(const uint32_t* __restrict__ v, const uint64_t* __restrict__ off,
                                                      uint64_t n, uint32_t* __restrict__ lbytes,
                                                      uint32_t* __restrict__ err) {
  const uint64_t k = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= n) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t e0 = off[k], e1 = off[k + 1];
  uint32_t carry = 0, tot = 0, bad = 0;
  for (uint64_t cb = e0; cb < e1; cb += 64 * kEncRows) {
    EncRow row[kEncRows];
    enc_rows(v, cb, e0, e1, lane, carry, row, bad);
#pragma unroll
    for (int r = 0; r < kEncRows; r++) tot += row[r].len;
  }
  tot = __builtin_amdgcn_readlane(sgd::wave_incl_add(tot), 63);
  if (lane == 0) lbytes[k] = tot;
  if (__any(bad != 0) && lane == 0) atomicOr(err, 1u);
}

__global__ __launch_bounds__(256) void k_enc_list_write(const uint32_t* __restrict__ v, const uint64_t* __restrict__ off,
                                                        uint64_t n, const uint64_t* __restrict__ boff,
                                                        uint8_t* __restrict__ out) {
  const uint64_t k = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= n) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t e0 = off[k], e1 = off[k + 1];
  uint8_t* o = out + boff[k];
  uint32_t carry = 0, bad = 0;  // (checked by pass A)
  for (uint64_t cb = e0; cb < e1; cb += 64 * kEncRows) {
    EncRow row[kEncRows];
    enc_rows(v, cb, e0, e1, lane, carry, row, bad);
#pragma unroll
    for (int r = 0; r < kEncRows; r++) {
      const uint32_t len = row[r].len, incl = sgd::wave_incl_add(len);
      uint8_t* p = o + (incl - len);
      uint32_t x = row[r].d;
#pragma unroll
      for (int b = 0; b < 5; b++)  // binary.PutUvarint
        if ((uint32_t)b < len) {
          p[b] = (uint8_t)((uint32_t)b + 1 < len ? (x | 0x80u) : x);
          x >>= 7;
        }
      o += __builtin_amdgcn_readlane(incl, 63);
    }
  }
}

// byte offsets of the lists: out_off[k] = gbase[g] + the bytes of group g's
// elements before off[k] (g = off[k] / 64)
__global__ void k_list_bpos(const uint32_t* __restrict__ v, const uint64_t* __restrict__ off,
                            const uint64_t* __restrict__ kw, uint64_t n, uint64_t N,
                            const uint64_t* __restrict__ gbase, uint32_t* __restrict__ err,
                            uint64_t* __restrict__ out_off) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > n) return;
  const uint64_t o = off[k];
  uint64_t p = gbase[o >> 6];
  for (uint64_t i = o & ~63ull; i < o; i++) p += enc_len_at(v, off, kw, N, i, err);
  out_off[k] = p;
}

// heads bit j <=> byte j starts a non-empty list (the bitmap is zeroed first)
__global__ void k_byte_heads(const uint64_t* __restrict__ in_off, uint64_t n, uint32_t* __restrict__ heads) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    const uint64_t b = in_off[k];
    if (b < in_off[k + 1]) atomicOr(&heads[b >> 5], 1u << (b & 31));
  }
}

__device__ __forceinline__ bool is_head(const uint32_t* heads, uint64_t j) { return (heads[j >> 5] >> (j & 31)) & 1u; }

// Decode works on 32-byte blocks (block b = bytes 32 b .. 32 b + 31; its
// head bits are the word heads[b]).  Pass 1: each block's terminators (bytes
// with the high bit clear end a value) as a mask and a count.
__device__ __forceinline__ void load_block(const uint8_t* in, uint64_t nb, uint64_t b, uint32_t (&w)[8]) {
  const uint64_t j0 = 32 * b;
  if (j0 + 32 <= nb) {
    const uint4* q = reinterpret_cast<const uint4*>(in + j0);
    const uint4 x = q[0], y = q[1];
    w[0] = x.x, w[1] = x.y, w[2] = x.z, w[3] = x.w, w[4] = y.x, w[5] = y.y, w[6] = y.z, w[7] = y.w;
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = 0x80808080u;  // past nb: continuation bytes (never terminators)
    for (uint64_t j = j0; j < nb; j++) {
      const uint32_t i = (uint32_t)(j - j0), sh = 8 * (i & 3);
      w[i >> 2] = (w[i >> 2] & ~(0xFFu << sh)) | ((uint32_t)in[j] << sh);
    }
  }
}

__device__ __forceinline__ uint32_t block_terms(const uint32_t (&w)[8]) {
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) m |= (((w[i >> 2] >> (8 * (i & 3) + 7)) & 1u) ^ 1u) << i;
  return m;
}

__global__ void k_dec_count(const uint8_t* __restrict__ in, uint64_t nb, uint32_t* __restrict__ tmask,
                            uint32_t* __restrict__ tcnt) {
  const uint64_t nblk = (nb + 31) / 32, stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nblk; b += stride) {
    uint32_t w[8];
    load_block(in, nb, b, w);
    const uint32_t m = block_terms(w);
    tmask[b] = m;
    tcnt[b] = __popc(m);
  }
}

// value offsets of the lists: voff[k] = terminators before byte in_off[k]
__global__ void k_list_vpos(const uint64_t* __restrict__ in_off, uint64_t n, const uint64_t* __restrict__ vbase,
                            const uint32_t* __restrict__ tmask, uint64_t* __restrict__ voff) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > n) return;
  const uint64_t o = in_off[k], b = o >> 5;
  const uint32_t r = (uint32_t)(o & 31);
  voff[k] = vbase[b] + (r ? __popc(tmask[b] & ((1u << r) - 1u)) : 0u);
}

// Pass 2: each block walks its bytes in order.  A run starts after a
// terminator or at a list start; the run the block opens inside is found by
// looking back at most 4 bytes.  Checks (as binary.Uvarint): a run must be <=
// 5 bytes and fit 32 bits, and a list must end on a terminator.
__global__ void k_dec_runs(const uint8_t* __restrict__ in, const uint32_t* __restrict__ heads, uint64_t nb,
                           const uint64_t* __restrict__ vbase, uint32_t* __restrict__ delta,
                           uint32_t* __restrict__ err) {
  const uint64_t nblk = (nb + 31) / 32, stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nblk; b += stride) {
    const uint64_t j0 = 32 * b;
    uint32_t w[8];
    load_block(in, nb, b, w);
    const uint32_t hm = heads[b];
    const uint32_t hnext = j0 + 32 < nb ? heads[b + 1] & 1u : 0u;  // does the next block start a list
    // the run open at j0: its start s and the value bits so far
    uint64_t s = j0;
    while (s > 0 && !is_head(heads, s) && (in[s - 1] & 0x80u) && j0 - s < 5) s--;
    uint64_t d = 0;
    for (uint64_t q = s; q < j0; q++) d |= (uint64_t)(in[q] & 0x7Fu) << (7 * (q - s));
    uint64_t vi = vbase[b];
    bool bad = false;
    const uint32_t len = j0 + 32 <= nb ? 32u : (uint32_t)(nb - j0);
    for (uint32_t i = 0; i < len; i++) {
      const uint64_t j = j0 + i;
      if ((hm >> i) & 1u) {
        s = j;
        d = 0;
      }
      const uint32_t c = (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
      const uint64_t r = j - s;  // position in the run
      if (r < 5) d |= (uint64_t)(c & 0x7Fu) << (7 * r);
      if (c & 0x80u) {
        // the list ends inside a value
        const bool last = j + 1 == nb || (i < 31 ? ((hm >> (i + 1)) & 1u) : hnext);
        bad |= last;
      } else {
        bad |= r >= 5 || d > 0xFFFFFFFFull;  // more than 32 bits
        delta[vi++] = (uint32_t)d;
        s = j + 1;
        d = 0;
      }
    }
    if (bad) *err = 1;
  }
}

// values of each list: running sums of its deltas (u64 scan), range-checked
__global__ void k_dec_values(const uint32_t* __restrict__ delta, const uint64_t* __restrict__ excl,
                             const uint64_t* __restrict__ voff, const uint64_t* __restrict__ kw, uint64_t N,
                             uint32_t* __restrict__ out, uint32_t* __restrict__ err) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += stride) {
    const uint64_t k = list_of_w(voff, kw, i);
    const uint64_t v = excl[i] + delta[i] - excl[voff[k]];
    if (v > 0xFFFFFFFFull) *err = 1;
    out[i] = (uint32_t)v;
  }
}

// Per-list decode, pass 1 (one wave per list, four per workgroup): the list's
// terminators, counted over 16-B loads (bytes outside the list masked off);
// a scan of the n counts gives the lists' value offsets.
__global__ __launch_bounds__(256) void k_dec_list_cnt(const uint8_t* __restrict__ in,
                                                      const uint64_t* __restrict__ in_off, uint64_t n,
                                                      uint32_t* __restrict__ lcnt) {
  const uint64_t k = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= n) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b0 = in_off[k], b1 = in_off[k + 1];
  uint32_t c = 0;
  for (uint64_t cb = b0 & ~15ull; cb < b1; cb += 64 * 16) {
    const uint64_t base = cb + (uint64_t)lane * 16;
    if (base >= b1) continue;
    const uint4 q = *reinterpret_cast<const uint4*>(in + base);
    const int64_t lo = (int64_t)b0 - (int64_t)base, hi = (int64_t)b1 - (int64_t)base;  // bytes [lo, hi) are the list's
    const uint32_t m = (hi >= 16 ? 0xFFFFu : (1u << hi) - 1u) & ~(lo <= 0 ? 0u : (1u << lo) - 1u);
    const uint32_t x[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const uint32_t bm = m >> (4 * d);
      const uint32_t e = ((bm & 1u) << 7) | ((bm & 2u) << 14) | ((bm & 4u) << 21) | ((bm & 8u) << 28);
      c += __popc(~x[d] & e);
    }
  }
  c = __builtin_amdgcn_readlane(sgd::wave_incl_add(c), 63);
  if (lane == 0) lcnt[k] = c;
}

// Pass 2 (one wave per list, four per workgroup): the list's bytes in steps of
// kDecRows rows of 256 bytes, lane L holding the row's dword at 4 L (one
// coalesced load per row, all of a step's rows in flight; steps start at the
// list's first byte rounded down to 4).  The 5 bytes before a lane's 4 come
// from the two lanes before (DPP wave shifts; lanes 0 and 1 from the row
// before, carried).  Each terminator decodes its run backwards (LEB128: the
// earlier byte holds the lower bits); the lanes' value counts and delta sums
// are scanned across the wave (32-bit DPP scans), so byte order = (row, lane)
// order = value order, and each value is stored straight to its slot: the
// stores of a row land in one contiguous run, and nothing is staged in LDS.
// Checks (binary.Uvarint, then the running sum): a run of <= 5 bytes fitting
// 32 bits, the list ending on a terminator, every sum within 32 bits (the sum
// is kept mod 2^32; a value whose add wraps it is the first past 2^32 - 1).
// The input buffer is padded to 16 bytes.
constexpr int kDecRows = 8;

// bits 7, 15, 23, 31 of x to bits 0-3 (one multiply: the four terms land on
// distinct bit positions, so nothing carries)
__device__ __forceinline__ int clamp9(int64_t x) { return x < 0 ? 0 : x > 9 ? 9 : (int)x; }

__device__ __forceinline__ uint32_t gather_hi(uint32_t x) { return (((x >> 7) & 0x01010101u) * 0x204081u >> 21) & 0xFu; }
__global__ __launch_bounds__(256) void k_dec_lists(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                                   const uint64_t* __restrict__ voff, uint64_t n, uint64_t cap,
                                                   uint32_t* __restrict__ out, uint32_t* __restrict__ err) {
  const uint64_t k = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= n) return;  // (a wave leaves whole)
  if (voff[n] > cap) {  // the values would not fit: the host reports it, nothing is written
    if (k == 0 && (threadIdx.x & 63) == 0) atomicOr(err, 2u);
    return;
  }
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t b0 = in_off[k], b1 = in_off[k + 1];
  uint32_t* o = out + voff[k];
  uint32_t run = 0, p63 = 0, p62 = 0;  // the running sum; the row before's dwords of lanes 63 and 62
  uint32_t badv = 0;
  for (uint64_t cb = b0 & ~3ull; cb < b1; cb += 256 * kDecRows) {
    uint32_t q[kDecRows];
#pragma unroll
    for (int r = 0; r < kDecRows; r++) {
      const uint64_t base = cb + 256 * r + 4 * lane;
      q[r] = base < b1 ? *reinterpret_cast<const uint32_t*>(in + base) : 0x80808080u;  // past: never terminators
    }
#pragma unroll
    for (int r = 0; r < kDecRows; r++) {
      if (cb + 256 * r >= b1) break;  // (uniform)
      const int64_t base = (int64_t)(cb + 256 * r + 4 * lane);
      const uint32_t s1 = (uint32_t)__builtin_amdgcn_update_dpp((int)p63, (int)q[r], 0x138 /* wave_shr:1 */, 0xF, 0xF, false);
      const uint32_t s2 = (uint32_t)__builtin_amdgcn_update_dpp((int)p62, (int)s1, 0x138, 0xF, 0xF, false);
      p63 = __builtin_amdgcn_readlane(q[r], 63);
      p62 = __builtin_amdgcn_readlane(q[r], 62);
      // the 9 bytes base - 5 .. base + 3 as bit masks (bit i = byte base - 5 + i):
      // cm = continuation bytes (high bit set); bytes before the list count as
      // value ends (they stop a walk back), bytes past it as continuations
      const int lo = clamp9((int64_t)b0 - base + 5), hi = clamp9((int64_t)b1 - base + 5);
      const uint32_t before = (1u << lo) - 1u, past = 0x1FFu & ~((1u << hi) - 1u);
      const uint32_t cm = (((s2 >> 31) | (gather_hi(s1) << 1) | (gather_hi(q[r]) << 5)) & ~before) | past;
      const uint32_t tm = (~cm >> 5) & (~before >> 5) & 0xFu;  // terminators in the lane's 4 bytes
      uint32_t c7[9];  // low 7 bits of each byte
      c7[0] = (s2 >> 24) & 0x7Fu;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        c7[1 + j] = __builtin_amdgcn_ubfe(s1, 8 * j, 7);
        c7[5 + j] = __builtin_amdgcn_ubfe(q[r], 8 * j, 7);
      }
      uint32_t d[4], t = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        // a value ends at byte P = 5 + j: its run is the L continuation bytes
        // before P (LEB128: the earlier byte holds the lower bits)
        constexpr uint32_t one = 1;
        const int P = 5 + j;
        const uint32_t stops = ~cm & ((one << P) - 1u);
        const int L = P - 1 - (stops ? 31 - __builtin_clz(stops) : -1);
        uint32_t v = c7[P];
#pragma unroll
        for (int k = 1; k <= 4; k++) v = k <= L ? (v << 7) | c7[P - k] : v;
        // a sixth byte, or a fifth whose last byte has bits past 32: over
        // binary.Uvarint's 32-bit range here
        const uint32_t is_t = (tm >> j) & 1u;
        badv |= is_t & ((uint32_t)(L >= 5) | ((uint32_t)(L == 4) & (uint32_t)((c7[P] & 0x70u) != 0)));
        d[j] = is_t ? v : 0u;
        t += d[j];
      }
      const uint32_t cnt = __popc(tm), ic = sgd::wave_incl_add(cnt), it = sgd::wave_incl_add(t);
      // (d = 0 off the terminators: the sum only moves at values; an add
      // that wraps it is the first value past 2^32 - 1)
      uint32_t acc = run + (it - t);
      const uint32_t ex = ic - cnt;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t a = acc + d[j];
        badv |= (uint32_t)(a < acc);
        acc = a;
        if ((tm >> j) & 1u) o[ex + __popc(tm & ((1u << j) - 1u))] = a;
      }
      o += __builtin_amdgcn_readlane(ic, 63);
      run += __builtin_amdgcn_readlane(it, 63);
    }
  }
  bool bad = badv != 0;
  if (lane == 0 && b1 > b0 && (in[b1 - 1] & 0x80u)) bad = true;  // the list ends inside a value
  if (__any(bad) && lane == 0) atomicOr(err, 1u);
}

__global__ void k_sancov(const uint32_t* __restrict__ cov, const uint64_t* __restrict__ off,
                         const uint64_t* __restrict__ kw, uint64_t n, uint64_t N, uint64_t* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N + n; i += stride) {
    if (i < n) {
      out[i + off[i]] = kSancovMagic;  // file i's header (execprog.go:166)
    } else {
      const uint64_t e = i - n, k = list_of_w(off, kw, e);
      out[k + 1 + e] = (0xFFFFFFFFull << 32) + cov[e];  // RestorePC(pc, 0xffffffff), cover.go:23-25
    }
  }
}

// One wave per list walks each list in order: right for many lists of
// moderate length (per-call signal), wrong for a few long ones (a set's
// members as one payload: one wave would walk all of it).  The per-element /
// per-block forms spread any list over the whole chip; they take batches of
// fewer than 256 lists or more than 64 Ki values (bytes) per list on average.
constexpr uint64_t kWaveListsMin = 256, kWaveListAvg = 65536;

static bool enc_elems(const sg_ctx* ctx, uint64_t n, uint64_t N) {  // (option rpc_encode_elems forces a form)
  if (ctx->opt[kOptRpcEncodeElems] >= 0) return ctx->opt[kOptRpcEncodeElems] != 0;
  return n < kWaveListsMin || N / n > kWaveListAvg;
}

static bool dec_blocks(const sg_ctx* ctx, uint64_t n, uint64_t nb) {  // (option rpc_decode_blocks forces a form)
  if (ctx->opt[kOptRpcDecodeBlocks] >= 0) return ctx->opt[kOptRpcDecodeBlocks] != 0;
  return n < kWaveListsMin || nb / n > kWaveListAvg;
}

inline uint32_t grid_for(uint64_t n) { return (uint32_t)std::min<uint64_t>(div_up(n ? n : 1, 256), 16384); }

bool offsets_ok(const uint64_t* off, size_t n) {
  if (off[0] != 0) return false;
  for (size_t k = 0; k < n; k++)
    if (off[k + 1] < off[k]) return false;
  return true;
}

// Encode the n lists at device d_v / d_off (N = elements) into device bytes;
// h_out_off (host, n+1) gets the byte offsets.  dstage holds d_v / d_off; the
// scratch and output live in ws from `base`.  Returns the byte buffer.
int encode_dev(sg_ctx* ctx, const uint32_t* d_v, const uint64_t* d_off, uint64_t n, uint64_t N, uint64_t* h_out_off,
               uint8_t** d_bytes) {
  WsPlan p;
  const uint64_t ng = (N + 63) / 64;
  const size_t o_len = p.add(ng * 4 + 4), o_pos = p.add((ng + 1) * 8), o_lo = p.add((n + 1) * 8), o_err = p.add(8),
               o_out = p.add(N * 5 + 8), o_kw = p.add((N + 31) / 32 * 8), o_lb = p.add(n * 4 + 4);
  const size_t scan_off = p.total;
  int rc = ws_reserve(ctx, p.total + scan_ws_bytes(std::max(N, n)));
  if (rc) return rc;
  uint32_t* len = (uint32_t*)ws_at(ctx, o_len);
  uint64_t* pos = (uint64_t*)ws_at(ctx, o_pos);
  uint64_t* lo = (uint64_t*)ws_at(ctx, o_lo);
  uint32_t* err = (uint32_t*)ws_at(ctx, o_err);
  uint8_t* out = (uint8_t*)ws_at(ctx, o_out);
  uint64_t* kw = (uint64_t*)ws_at(ctx, o_kw);
  SG_HIP(hipMemsetAsync(err, 0, 4, ctx->stream));
  // (a list's byte count is a u32: the per-list form when 5 N cannot overflow it)
  if (!enc_elems(ctx, n, N) && N * 5 < (1ull << 32)) {
    ScopedTimer tm(ctx, "rpc_encode");
    uint32_t* lbytes = (uint32_t*)ws_at(ctx, o_lb);
    hipLaunchKernelGGL(k_enc_list_len, dim3((uint32_t)div_up(n, 4)), dim3(256), 0, ctx->stream, d_v, d_off, n, lbytes,
                       err);
    rc = scan_counts(ctx, lbytes, lo, n, scan_off);  // lo = list byte offsets (lo[n] = total)
    if (rc) return rc;
    hipLaunchKernelGGL(k_enc_list_write, dim3((uint32_t)div_up(n, 4)), dim3(256), 0, ctx->stream, d_v, d_off, n,
                       (const uint64_t*)lo, out);
  } else {
    // (option rpc_encode_elems 1: the per-element form)
    ScopedTimer tm(ctx, "rpc_encode");
    if (N) {
      hipLaunchKernelGGL(k_word_lists, dim3(grid_for((N + 31) / 32)), dim3(256), 0, ctx->stream, d_off, n, N, kw);
      hipLaunchKernelGGL(k_enc_len, dim3(grid_for(N)), dim3(256), 0, ctx->stream, d_v, d_off, kw, N, len, err);
    }
    rc = scan_counts(ctx, len, pos, ng, scan_off);  // pos = group byte bases (pos[ng] = total)
    if (rc) return rc;
    if (N)
      hipLaunchKernelGGL(k_enc_write, dim3(grid_for(N)), dim3(256), 0, ctx->stream, d_v, d_off, kw, N, pos, out, err);
    hipLaunchKernelGGL(k_list_bpos, dim3(div_up(n + 1, 256)), dim3(256), 0, ctx->stream, d_v, d_off, kw, n, N, pos, err,
                       lo);
  }
  SG_HIP(hipGetLastError());
  uint32_t herr = 0;
  SG_HIP(hipMemcpyAsync(h_out_off, lo, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (herr) {
    set_error("sg_delta_encode: a list is not sorted (non-decreasing)");
    return SG_EINVAL;
  }
  *d_bytes = out;
  return SG_OK;
}

// Decode n lists of device bytes d_in / d_in_off (nb bytes) into device values
// (capacity cap); h_off (host, n+1) gets the value offsets.  Scratch in ws.
int decode_dev(sg_ctx* ctx, const uint8_t* d_in, const uint64_t* d_in_off, uint64_t n, uint64_t nb, uint32_t* d_vals,
               uint64_t cap, uint64_t* h_off, uint64_t* d_voff) {
  const uint64_t nblk = (nb + 31) / 32;
  WsPlan p;
  const size_t o_tm = p.add(nblk * 4 + 4), o_tc = p.add(std::max(nblk, n) * 4 + 4), o_vb = p.add((nblk + 1) * 8),
               o_d = p.add(nb * 4 + 4), o_x = p.add((nb + 1) * 8), o_err = p.add(8), o_hd = p.add(nblk * 4 + 4),
               o_kwv = p.add(nblk * 8);
  const size_t scan_off = p.total;
  int rc = ws_reserve(ctx, p.total + scan_ws_bytes(std::max(nb, n)));
  if (rc) return rc;
  uint32_t* tmask = (uint32_t*)ws_at(ctx, o_tm);
  uint32_t* tcnt = (uint32_t*)ws_at(ctx, o_tc);  // per block, or per list (the per-list form)
  uint64_t* vbase = (uint64_t*)ws_at(ctx, o_vb);
  uint32_t* delta = (uint32_t*)ws_at(ctx, o_d);
  uint64_t* excl = (uint64_t*)ws_at(ctx, o_x);
  uint32_t* err = (uint32_t*)ws_at(ctx, o_err);
  uint32_t* heads = (uint32_t*)ws_at(ctx, o_hd);
  uint64_t* kwv = (uint64_t*)ws_at(ctx, o_kwv);  // N <= nb
  SG_HIP(hipMemsetAsync(err, 0, 4, ctx->stream));
  ScopedTimer tm(ctx, "rpc_decode");
  // (a list's value count is a u32: the per-list form when nb cannot overflow it)
  const bool lists = nb && nb < (1ull << 32) && !dec_blocks(ctx, n, nb);
  if (lists) {
    // the lists' value counts, their scan; no host wait between the passes:
    // the decode checks the capacity itself (error bit 2: nothing written)
    hipLaunchKernelGGL(k_dec_list_cnt, dim3((uint32_t)div_up(n, 4)), dim3(256), 0, ctx->stream, d_in, d_in_off, n,
                       tcnt);
    rc = scan_counts(ctx, tcnt, d_voff, n, scan_off);
    if (rc) return rc;
    hipLaunchKernelGGL(k_dec_lists, dim3((uint32_t)div_up(n, 4)), dim3(256), 0, ctx->stream, d_in, d_in_off,
                       (const uint64_t*)d_voff, n, cap, d_vals, err);
    SG_HIP(hipMemcpyAsync(h_off, d_voff, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  } else {
    if (nb) hipLaunchKernelGGL(k_dec_count, dim3(grid_for(nblk)), dim3(256), 0, ctx->stream, d_in, nb, tmask, tcnt);
    rc = scan_counts(ctx, tcnt, vbase, nblk, scan_off);
    if (rc) return rc;
    hipLaunchKernelGGL(k_list_vpos, dim3(div_up(n + 1, 256)), dim3(256), 0, ctx->stream, d_in_off, n, vbase, tmask,
                       d_voff);
    SG_HIP(hipMemcpyAsync(h_off, d_voff, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
    SG_HIP(hipStreamSynchronize(ctx->stream));
    const uint64_t N = h_off[n];
    if (N > cap) {
      set_error("sg_delta_decode: %llu values, capacity %llu", (unsigned long long)N, (unsigned long long)cap);
      return SG_EINVAL;
    }
    // (option rpc_decode_blocks 1: the per-block form -- runs per 32-byte block,
    // then a scan of the deltas)
    if (nb) {
      SG_HIP(hipMemsetAsync(heads, 0, nblk * 4 + 4, ctx->stream));
      hipLaunchKernelGGL(k_byte_heads, dim3(grid_for(n)), dim3(256), 0, ctx->stream, d_in_off, n, heads);
      hipLaunchKernelGGL(k_dec_runs, dim3(grid_for(nblk)), dim3(256), 0, ctx->stream, d_in, heads, nb, vbase, delta,
                         err);
    }
    rc = scan_counts(ctx, delta, excl, N, scan_off);
    if (rc) return rc;
    if (N) {
      hipLaunchKernelGGL(k_word_lists, dim3(grid_for((N + 31) / 32)), dim3(256), 0, ctx->stream, d_voff, n, N, kwv);
      hipLaunchKernelGGL(k_dec_values, dim3(grid_for(N)), dim3(256), 0, ctx->stream, delta, excl, d_voff, kwv, N,
                         d_vals, err);
    }
  }
  SG_HIP(hipGetLastError());
  uint32_t herr = 0;
  SG_HIP(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (lists && h_off[n] > cap) {
    set_error("sg_delta_decode: %llu values, capacity %llu", (unsigned long long)h_off[n], (unsigned long long)cap);
    return SG_EINVAL;
  }
  if (herr) {
    set_error("sg_delta_decode: malformed payload (unterminated value, value over 32 bits, or sum over 32 bits)");
    return SG_EINVAL;
  }
  return SG_OK;
}

}  // namespace
}  // namespace sg

using namespace sg;

extern "C" {

int sg_delta_encode_batch(sg_ctx* ctx, const uint32_t* vals, const uint64_t* off, size_t n, uint8_t* out, size_t cap,
                          uint64_t* out_off) {
  if (!ctx || !off || !out_off || !offsets_ok(off, n) || (off[n] && !vals) || (cap && !out)) {
    set_error("sg_delta_encode_batch: invalid argument");
    return SG_EINVAL;
  }
  const uint64_t N = off[n];
  if (n == 0 || N == 0) {
    for (size_t k = 0; k <= n; k++) out_off[k] = 0;
    return SG_OK;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  const size_t b_v = (N * 4 + 255) & ~size_t(255);
  rc = dstage_reserve(ctx, b_v + (n + 1) * 8);
  if (rc) return rc;
  uint32_t* dv = (uint32_t*)ctx->dstage;
  uint64_t* doff = (uint64_t*)((char*)ctx->dstage + b_v);
  SG_HIP(hipMemcpyAsync(dv, vals, N * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(doff, off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  uint8_t* bytes = nullptr;
  rc = encode_dev(ctx, dv, doff, n, N, out_off, &bytes);
  if (rc) return rc;
  if (out_off[n] <= cap) {
    SG_HIP(hipMemcpyAsync(out, bytes, out_off[n], hipMemcpyDeviceToHost, ctx->stream));
    SG_HIP(hipStreamSynchronize(ctx->stream));
  }
  return SG_OK;
}

int sg_delta_decode_batch(sg_ctx* ctx, const uint8_t* in, const uint64_t* in_off, size_t n, uint32_t* vals, size_t cap,
                          uint64_t* off) {
  if (!ctx || !in_off || !off || !offsets_ok(in_off, n) || (in_off[n] && !in) || (cap && !vals)) {
    set_error("sg_delta_decode_batch: invalid argument");
    return SG_EINVAL;
  }
  const uint64_t nb = in_off[n];
  if (n == 0 || nb == 0) {
    for (size_t k = 0; k <= n; k++) off[k] = 0;
    return SG_OK;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  // every byte can end a value: nb values at most
  const size_t b_b = (nb + 255) & ~size_t(255), b_o = ((n + 1) * 8 + 255) & ~size_t(255);
  rc = dstage_reserve(ctx, b_b + 2 * b_o + nb * 4 + 4);
  if (rc) return rc;
  uint8_t* din = (uint8_t*)ctx->dstage;
  uint64_t* dio = (uint64_t*)((char*)ctx->dstage + b_b);
  uint64_t* dvo = (uint64_t*)((char*)ctx->dstage + b_b + b_o);
  uint32_t* dv = (uint32_t*)((char*)ctx->dstage + b_b + 2 * b_o);
  SG_HIP(hipMemcpyAsync(din, in, nb, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dio, in_off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  rc = decode_dev(ctx, din, dio, n, nb, dv, nb, off, dvo);
  if (rc) return rc;
  if (off[n] > cap) {
    set_error("sg_delta_decode_batch: %llu values, capacity %zu", (unsigned long long)off[n], cap);
    return SG_EINVAL;
  }
  if (off[n]) SG_HIP(hipMemcpyAsync(vals, dv, off[n] * 4, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

int sg_set_encode(sg_set* set, uint8_t* out, size_t cap, size_t* nbytes) {
  if (!set || !nbytes || (cap && !out)) return SG_EINVAL;
  sg_ctx* ctx = set->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  uint64_t total = 0;
  {  // count first: the members go to dstage
    rc = set_export_dev(set, nullptr, 0, &total);
    if (rc) return rc;
  }
  *nbytes = 0;
  if (total == 0) return SG_OK;
  const size_t b_v = (total * 4 + 255) & ~size_t(255);
  rc = dstage_reserve(ctx, b_v + 16);
  if (rc) return rc;
  uint32_t* dv = (uint32_t*)ctx->dstage;
  uint64_t* doff = (uint64_t*)((char*)ctx->dstage + b_v);
  rc = set_export_dev(set, dv, total, &total);
  if (rc) return rc;
  const uint64_t hoff[2] = {0, total};
  SG_HIP(hipMemcpyAsync(doff, hoff, 16, hipMemcpyHostToDevice, ctx->stream));
  uint64_t bo[2] = {0, 0};
  uint8_t* bytes = nullptr;
  rc = encode_dev(ctx, dv, doff, 1, total, bo, &bytes);
  if (rc) return rc;
  *nbytes = bo[1];
  if (bo[1] <= cap) {
    SG_HIP(hipMemcpyAsync(out, bytes, bo[1], hipMemcpyDeviceToHost, ctx->stream));
    SG_HIP(hipStreamSynchronize(ctx->stream));
  }
  return SG_OK;
}

int sg_set_decode_add(sg_set* set, const uint8_t* in, size_t nbytes, uint64_t* count) {
  if (!set || (nbytes && !in)) return SG_EINVAL;
  if (count) *count = 0;
  if (nbytes == 0) return SG_OK;
  sg_ctx* ctx = set->ctx;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  const size_t b_b = (nbytes + 255) & ~size_t(255);
  rc = dstage_reserve(ctx, b_b + 512 + nbytes * 4 + 4);
  if (rc) return rc;
  uint8_t* din = (uint8_t*)ctx->dstage;
  uint64_t* dio = (uint64_t*)((char*)ctx->dstage + b_b);
  uint64_t* dvo = dio + 32;
  uint32_t* dv = (uint32_t*)((char*)ctx->dstage + b_b + 512);
  const uint64_t hio[2] = {0, nbytes};
  SG_HIP(hipMemcpyAsync(din, in, nbytes, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(dio, hio, 16, hipMemcpyHostToDevice, ctx->stream));
  uint64_t hoff[2] = {0, 0};
  rc = decode_dev(ctx, din, dio, 1, nbytes, dv, nbytes, hoff, dvo);
  if (rc) return rc;
  rc = set_add_dev_locked(set, dv, hoff[1]);  // fuzzer.go:392-398 / :146-151 (SignalAdd of the payload)
  if (rc) return rc;
  SG_HIP(hipStreamSynchronize(ctx->stream));
  if (count) *count = hoff[1];
  return SG_OK;
}

int sg_sancov_batch(sg_ctx* ctx, const uint32_t* cov, const uint64_t* cov_off, size_t n, uint8_t* out) {
  if (!ctx || !cov_off || !offsets_ok(cov_off, n) || (cov_off[n] && !cov) || (n && !out)) {
    set_error("sg_sancov_batch: invalid argument");
    return SG_EINVAL;
  }
  if (n == 0) return SG_OK;
  const uint64_t N = cov_off[n];
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc = ensure_device(ctx);
  if (rc) return rc;
  const size_t b_v = (N * 4 + 255) & ~size_t(255), b_o = ((n + 1) * 8 + 255) & ~size_t(255);
  const size_t b_w = ((N + 31) / 32 * 8 + 255) & ~size_t(255);
  rc = dstage_reserve(ctx, b_v + b_o + b_w + (N + n) * 8);
  if (rc) return rc;
  uint32_t* dv = (uint32_t*)ctx->dstage;
  uint64_t* doff = (uint64_t*)((char*)ctx->dstage + b_v);
  uint64_t* kw = (uint64_t*)((char*)ctx->dstage + b_v + b_o);
  uint64_t* dout = (uint64_t*)((char*)ctx->dstage + b_v + b_o + b_w);
  if (N) SG_HIP(hipMemcpyAsync(dv, cov, N * 4, hipMemcpyHostToDevice, ctx->stream));
  SG_HIP(hipMemcpyAsync(doff, cov_off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  {
    ScopedTimer tm(ctx, "sancov");
    if (N)
      hipLaunchKernelGGL(k_word_lists, dim3(grid_for((N + 31) / 32)), dim3(256), 0, ctx->stream, doff, (uint64_t)n, N,
                         kw);
    hipLaunchKernelGGL(k_sancov, dim3(grid_for(N + n)), dim3(256), 0, ctx->stream, dv, doff, kw, (uint64_t)n, N, dout);
  }
  SG_HIP(hipGetLastError());
  SG_HIP(hipMemcpyAsync(out, dout, (N + n) * 8, hipMemcpyDeviceToHost, ctx->stream));
  SG_HIP(hipStreamSynchronize(ctx->stream));
  return SG_OK;
}

}  // extern "C"
