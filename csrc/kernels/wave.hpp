// wave64 helpers for gfx950 (CDNA4).  A wave is 64 lanes: ballots are 64-bit,
// one bitmap word (64 vertices) maps to one wave ballot.
#pragma once

#include <hip/hip_runtime.h>

#include "dbfs/common.hpp"

namespace dbfs {
namespace dev {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return static_cast<int>(__lane_id()); }

// Number of set bits of `m` strictly below this lane (v_mbcnt_lo/hi).
__device__ __forceinline__ unsigned mask_rank(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(m >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(m), 0u));
}

__device__ __forceinline__ unsigned long long readlane64(unsigned long long x, int l) {
  const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(x & 0xffffffffull), l));
  const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(x >> 32), l));
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}

__device__ __forceinline__ long long readlane_i64(long long x, int l) {
  return static_cast<long long>(readlane64(static_cast<unsigned long long>(x), l));
}

// Inclusive wave64 scans on DPP lane moves (VALU, no LDS crossbar): a
// Hillis-Steele scan inside each 16-lane row (row_shr 1 / 2 / 4 / 8, lanes
// shifted in from outside the row read 0: bound_ctrl), then the row totals
// carried across rows with the gfx9 row broadcasts (row_bcast:15 into rows 1
// and 3, row_bcast:31 into rows 2 and 3).  A lane a DPP move does not write
// (row / bank mask) reads `old` = 0, so every step is x += move(x).
constexpr int kDppRowShr1 = 0x111, kDppRowShr2 = 0x112, kDppRowShr4 = 0x114, kDppRowShr8 = 0x118;
constexpr int kDppRowBcast15 = 0x142, kDppRowBcast31 = 0x143;

template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ unsigned dpp_u32(unsigned x) {
  return static_cast<unsigned>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(x), kCtrl, kRowMask, 0xf, true));
}
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ unsigned long long dpp_u64(unsigned long long x) {
  const unsigned lo = dpp_u32<kCtrl, kRowMask>(static_cast<unsigned>(x));
  const unsigned hi = dpp_u32<kCtrl, kRowMask>(static_cast<unsigned>(x >> 32));
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}

__device__ __forceinline__ unsigned wave_incl_scan_u32(unsigned x) {
  x += dpp_u32<kDppRowShr1>(x);
  x += dpp_u32<kDppRowShr2>(x);
  x += dpp_u32<kDppRowShr4>(x);
  x += dpp_u32<kDppRowShr8>(x);
  x += dpp_u32<kDppRowBcast15, 0xa>(x);
  x += dpp_u32<kDppRowBcast31, 0xc>(x);
  return x;
}

__device__ __forceinline__ long long wave_incl_scan(long long x) {
  unsigned long long v = static_cast<unsigned long long>(x);
  v += dpp_u64<kDppRowShr1>(v);
  v += dpp_u64<kDppRowShr2>(v);
  v += dpp_u64<kDppRowShr4>(v);
  v += dpp_u64<kDppRowShr8>(v);
  v += dpp_u64<kDppRowBcast15, 0xa>(v);
  v += dpp_u64<kDppRowBcast31, 0xc>(v);
  return static_cast<long long>(v);
}

__device__ __forceinline__ int wave_incl_max(int x) {
  const int l = lane_id();
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int y = __shfl_up(x, off, kWave);
    if (l >= off) x = max(x, y);
  }
  return x;
}

__device__ __forceinline__ long long wave_sum(long long x) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) x += __shfl_xor(x, off, kWave);
  return x;
}

__device__ __forceinline__ bool test_bit(const word_t* bm, unsigned v) {
  return (bm[v >> 6] >> (v & 63)) & 1ull;
}

// Position of the r-th (0-based) set bit of x (r < popcount(x)).
__device__ __forceinline__ int select_bit(unsigned long long x, int r) {
  int pos = 0;
#pragma unroll
  for (int width = 32; width >= 1; width >>= 1) {
    const int c = __popcll(x & ((1ull << width) - 1ull));
    if (r >= c) {
      r -= c;
      x >>= width;
      pos += width;
    }
  }
  return pos;
}

// Compaction of a wave's bit set: lane l holds word l's bits `m` (64 words,
// 4096 positions) and `incl` = inclusive prefix of popcounts over the lanes.
// Element idx (< total) of the set -> position 64 j + bit.  Binary search over
// the lanes' prefixes (6 shuffles) + select in the word.
__device__ __forceinline__ int wave_set_position(unsigned long long m, int incl, int idx) {
  int j = 0;
#pragma unroll
  for (int step = 32; step >= 1; step >>= 1)
    if (__shfl(incl, j + step - 1, kWave) <= idx) j += step;
  // (every lane shuffles: a source lane must be active for its value to be read)
  const int prev = __shfl(incl, j > 0 ? j - 1 : 0, kWave);
  const int ex = j > 0 ? prev : 0;
  const unsigned long long mj = static_cast<unsigned long long>(__shfl(static_cast<long long>(m), j, kWave));
  return j * 64 + select_bit(mj, idx - ex);
}

}  // namespace dev
}  // namespace dbfs
