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
//   Power law (Chung-Lu): both endpoints drawn with probability proportional
//   to the weight w_i = (i + i0)^(-2/3) -- a degree distribution with a
//   power-law tail of exponent 2.5 (social networks: 2-3), the largest
//   expected degree set through i0 -- then a seeded bijective scramble of the
//   labels (hubs spread over the partition).  The stand-in for
//   soc-LiveJournal1 and Friendster at their real vertex / edge counts (the
//   datasets are not on the pool; parity with them stays unpinned).
#pragma once

#include <cmath>
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
  bool power_law = false;     // Chung-Lu power law instead of RMAT (below)
  bool scramble = true;       // permute RMAT / power-law vertex labels
  // > 0: a 2-D grid of grid_w columns and n / grid_w rows, each vertex joined
  // to its right and lower neighbour -- road-like (degree <= 4, diameter
  // grid_w + n / grid_w - 2), the high-diameter case; labels row-major
  int64_t grid_w = 0;
  // Power law, inverse-CDF sampling in 32.32 fixed point (integer arithmetic
  // only, so host and device agree bit for bit): an endpoint is
  // floor(t^3) - pl_i0 with t = pl_a + r * pl_span (r uniform in [0, 1)),
  // pl_a = cbrt(i0), pl_a + pl_span = cbrt(n + i0); labels scrambled over
  // [0, 2^pl_bits) with cycle walking into [0, n).
  uint64_t pl_a = 0, pl_span = 0;
  int64_t pl_i0 = 0;
  int pl_bits = 0;
  int64_t pl_dmax = 0;  // the largest expected degree asked for (information)
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

// (x * y) >> 32 of 64-bit fixed-point values (the product below 2^96).
DBFS_HD uint64_t mul_shr32(uint64_t x, uint64_t y) { return (mulhi64(x, y) << 32) | ((x * y) >> 32); }

// A power-law endpoint from 64 random bits (GenParams::power_law).
DBFS_HD uint64_t power_law_vertex(const GenParams& p, uint64_t r) {
  const uint64_t t = p.pl_a + mulhi64(r, p.pl_span);          // t * 2^32, t < 2^10
  const uint64_t t3 = mul_shr32(mul_shr32(t, t), t);          // t^3 * 2^32
  int64_t x = static_cast<int64_t>(t3 >> 32) - p.pl_i0;
  const int64_t n = p.n;
  x = x < 0 ? 0 : (x >= n ? n - 1 : x);
  if (!p.scramble) return static_cast<uint64_t>(x);
  uint64_t y = static_cast<uint64_t>(x);
  do {
    y = scramble_vertex(y, p.pl_bits, p.seed);  // (a bijection of [0, 2^bits): the walk ends in < 2 steps on average)
  } while (y >= static_cast<uint64_t>(n));
  return y;
}

// Edge i of the stream described by p.
DBFS_HD void gen_edge(const GenParams& p, uint64_t i, uint64_t& u, uint64_t& v) {
  if (p.grid_w > 0) {
    // edges [0, (w - 1) h) horizontal, row-major; the rest vertical
    const uint64_t w = static_cast<uint64_t>(p.grid_w), h = static_cast<uint64_t>(p.n) / w;
    const uint64_t he = (w - 1) * h;
    if (i < he) {
      const uint64_t r = i / (w - 1);
      u = r * w + (i - r * (w - 1));
      v = u + 1;
    } else {
      u = i - he;
      v = u + w;
    }
    return;
  }
  const uint64_t base = mix64(p.seed * 0xD1B54A32D192ED03ull ^ mix64(i));
  if (p.power_law) {
    u = power_law_vertex(p, mix64(base + 1));
    v = power_law_vertex(p, mix64(base + 2));
    return;
  }
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

// The w x h grid (GenParams::grid_w): n = w h vertices, (w - 1) h + w (h - 1)
// edges.
inline GenParams grid_params(int64_t w, int64_t h) {
  GenParams p;
  p.grid_w = w;
  p.scramble = false;
  p.n = w * h;
  p.m = (w - 1) * h + w * (h - 1);
  return p;
}

// Power-law graph of n vertices and m input edges whose largest expected
// degree is about dmax (Chung-Lu, weight exponent -2/3: degree tail exponent
// 2.5).  i0 is found by bisection on the host: the expected degree of vertex
// 0 is 2m (cbrt(1 + i0) - cbrt(i0)) / (cbrt(n + i0) - cbrt(i0)).
inline GenParams power_law_params(int64_t n, int64_t m, int64_t dmax, uint64_t seed) {
  GenParams p;
  p.power_law = true;
  p.scramble = true;
  p.n = n;
  p.m = m;
  p.seed = seed;
  p.pl_dmax = dmax;
  auto d0 = [&](double i0) {
    return 2.0 * static_cast<double>(m) * (std::cbrt(1.0 + i0) - std::cbrt(i0)) /
           (std::cbrt(static_cast<double>(n) + i0) - std::cbrt(i0));
  };
  double lo = 0.0, hi = static_cast<double>(n);
  if (d0(0.0) > static_cast<double>(dmax)) {
    for (int it = 0; it < 200; ++it) {
      const double mid = 0.5 * (lo + hi);
      if (d0(mid) > static_cast<double>(dmax)) lo = mid;
      else hi = mid;
    }
  } else {
    hi = 0.0;
  }
  p.pl_i0 = static_cast<int64_t>(std::llround(hi));
  const double a = std::cbrt(static_cast<double>(p.pl_i0));
  const double b = std::cbrt(static_cast<double>(n + p.pl_i0));
  p.pl_a = static_cast<uint64_t>(std::llround(a * 4294967296.0));
  p.pl_span = static_cast<uint64_t>(std::llround(b * 4294967296.0)) - p.pl_a;
  int bits = 1;
  while ((int64_t(1) << bits) < n) ++bits;
  p.pl_bits = bits;
  return p;
}

}  // namespace dbfs
