// Counter-based synthetic graph generators, bit-identical on host and device.
//
// The reference's only generator is the dead `readGraph` uniform multigraph
// (bfs.cu:882-920, srand(12345)).  Here every edge i is a pure function of
// (seed, i), so each rank (or each GPU thread) can regenerate any edge without
// storing the edge list: a rank builds its CSR shard in two passes (degree
// count, then fill) over the same counter stream.
//
//   RMAT (Graph500 Kronecker): a=0.57 b=0.19 c=0.19 d=0.05, edge factor 16,
//   followed by a seeded bijective scramble of vertex labels so hubs are spread
//   over the 1D block partition.
//   Uniform: u, v uniform in [0, n) (the reference's dead generator).
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define DBFS_HD __host__ __device__ __forceinline__
#else
#define DBFS_HD inline
#endif

namespace dbfs {

struct GenParams {
  int scale = 16;             // n = 2^scale (RMAT); for uniform, n given explicitly
  int64_t n = 0;              // vertices
  int64_t m = 0;              // undirected input edges
  uint64_t seed = 1;
  bool uniform = false;       // uniform random instead of RMAT
  bool scramble = true;       // permute RMAT vertex labels
  // RMAT quadrant thresholds in 32-bit fixed point: a, a+b, a+b+c.
  uint32_t t_a = 2448131359u;     // floor(0.57 * 2^32)
  uint32_t t_ab = 3264175145u;    // floor(0.76 * 2^32)
  uint32_t t_abc = 4080218931u;   // floor(0.95 * 2^32)
};

DBFS_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return static_cast<uint64_t>((static_cast<unsigned __int128>(a) * b) >> 64);
#endif
}

DBFS_HD uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Bijective scramble of [0, 2^scale): odd-multiply-add then xorshift, 3 rounds.
DBFS_HD uint64_t scramble_vertex(uint64_t x, int scale, uint64_t seed) {
  const uint64_t mask = (scale >= 64) ? ~0ull : ((1ull << scale) - 1ull);
  const int sh = (scale + 1) / 2;
  uint64_t k1 = mix64(seed ^ 0x5851F42D4C957F2Dull) | 1ull;
  uint64_t k2 = mix64(seed ^ 0x14057B7EF767814Full);
  uint64_t k3 = mix64(seed ^ 0x2545F4914F6CDD1Dull) | 1ull;
  x = (x * k1 + k2) & mask;
  x ^= x >> sh;
  x = (x * k3 + k1) & mask;
  x ^= x >> sh;
  x = (x * k1 + k3) & mask;
  x ^= x >> sh;
  return x & mask;
}

// Edge i of the stream described by p.
DBFS_HD void gen_edge(const GenParams& p, uint64_t i, uint64_t& u, uint64_t& v) {
  const uint64_t base = mix64(p.seed * 0xD1B54A32D192ED03ull ^ mix64(i));
  if (p.uniform) {
    const uint64_t r0 = mix64(base + 1);
    const uint64_t r1 = mix64(base + 2);
    const uint64_t n = static_cast<uint64_t>(p.n);
    // multiply-shift range reduction (unbiased enough for synthetic graphs)
    u = mulhi64(r0, n);
    v = mulhi64(r1, n);
    return;
  }
  uint64_t uu = 0, vv = 0;
  uint64_t r = 0;
  for (int k = 0; k < p.scale; ++k) {
    uint32_t draw;
    if ((k & 1) == 0) {
      r = mix64(base + static_cast<uint64_t>(k / 2 + 1) * 0x9E3779B97F4A7C15ull);
      draw = static_cast<uint32_t>(r);
    } else {
      draw = static_cast<uint32_t>(r >> 32);
    }
    uint64_t bu, bv;
    if (draw < p.t_a) { bu = 0; bv = 0; }
    else if (draw < p.t_ab) { bu = 0; bv = 1; }
    else if (draw < p.t_abc) { bu = 1; bv = 0; }
    else { bu = 1; bv = 1; }
    uu = (uu << 1) | bu;
    vv = (vv << 1) | bv;
  }
  if (p.scramble) {
    uu = scramble_vertex(uu, p.scale, p.seed);
    vv = scramble_vertex(vv, p.scale, p.seed);
  }
  u = uu;
  v = vv;
}

inline GenParams rmat_params(int scale, int edge_factor, uint64_t seed) {
  GenParams p;
  p.scale = scale;
  p.n = int64_t(1) << scale;
  p.m = p.n * edge_factor;
  p.seed = seed;
  return p;
}

inline GenParams uniform_params(int64_t n, int64_t m, uint64_t seed) {
  GenParams p;
  p.uniform = true;
  p.scramble = false;
  p.n = n;
  p.m = m;
  p.seed = seed;
  return p;
}

}  // namespace dbfs
