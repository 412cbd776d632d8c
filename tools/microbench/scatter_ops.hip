// Microbenchmark: the scattered-update primitives a top-down BFS step can use
// on MI355X, at the sizes of an RMAT-26 level (67 M vertices, 8 MiB bitmap).
//
//   agent-or      64-bit atomicOr, agent scope, random word of an 8 MiB bitmap
//   agent-or-nr   same, result unused (no-return atomic)
//   xcd-or        64-bit atomicOr, WORKGROUP scope, random word of the calling
//                 XCD's own 1 MiB slice (XCC id from HW_REG_XCC_ID): performed
//                 in that XCD's L2 if the scope allows it; correctness checked
//                 (every claimed bit must be in memory after the kernel)
//   byte-store    plain byte store, random vertex of a 64 MiB byte map
//   xcd-byte      plain byte store into the calling XCD's 8 MiB slice
//   rand-load     8-B load of a random word of the 8 MiB bitmap (dependent use)
//   probe-store   visited-bit probe, then the byte store (a direct top-down edge)
//   xcd-probe-st  the same with targets in the calling XCD's 1/8 of the range
//   agent-or32    32-bit atomicOr (returning), agent scope, random 32-bit word of the same bitmap
//   agent-or32-nr same, result unused
//
// Build: hipcc -O3 --offload-arch=gfx950 -o build/scatter_ops tools/microbench/scatter_ops.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

constexpr int kThreads = 256;
constexpr int kPerThread = 16;

__device__ __forceinline__ unsigned xcc_id() {
  // HW_REG_XCC_ID (id 20), bits [3:0]
  return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 7u;
}

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

template <int kMode>
__global__ __launch_bounds__(kThreads) void scatter_kernel(unsigned long long* words, unsigned char* bytes,
                                                           unsigned long long nwords, unsigned long long* claims,
                                                           unsigned long long* sink, unsigned seed) {
  const unsigned long long tid = static_cast<unsigned long long>(blockIdx.x) * kThreads + threadIdx.x;
  unsigned long long local = 0, acc = 0;
  const unsigned x = xcc_id();
#pragma unroll 4
  for (int k = 0; k < kPerThread; ++k) {
    const unsigned long long r = mix(tid * kPerThread + k + (static_cast<unsigned long long>(seed) << 40));
    const unsigned long long bit = 1ull << (r & 63);
    if constexpr (kMode == 0) {
      const unsigned long long w = (r >> 6) % nwords;
      const unsigned long long old = __hip_atomic_fetch_or(words + w, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      local += !(old & bit);
    } else if constexpr (kMode == 1) {
      const unsigned long long w = (r >> 6) % nwords;
      __hip_atomic_fetch_or(words + w, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if constexpr (kMode == 2) {
      const unsigned long long slice = nwords / 8;
      const unsigned long long w = x * slice + (r >> 6) % slice;
      const unsigned long long old =
          __hip_atomic_fetch_or(words + w, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      local += !(old & bit);
    } else if constexpr (kMode == 3) {
      const unsigned long long v = (r >> 6) % (nwords * 64);
      bytes[v] = 1;
    } else if constexpr (kMode == 4) {
      const unsigned long long slice = nwords * 8;
      const unsigned long long v = x * slice + (r >> 6) % slice;
      bytes[v] = 1;
    } else if constexpr (kMode == 6) {
      // byte store only where a probe of the (static) bitmap says unvisited
      const unsigned long long v = (r >> 6) % (nwords * 64);
      if (!(words[v >> 6] & (1ull << (v & 63)))) bytes[v] = 1;
    } else if constexpr (kMode == 7) {
      // the same, targets in the calling XCD's slice
      const unsigned long long slice = nwords * 8;
      const unsigned long long v = x * slice + (r >> 6) % slice;
      if (!(words[v >> 6] & (1ull << (v & 63)))) bytes[v] = 1;
    } else if constexpr (kMode == 8 || kMode == 9) {
      unsigned* w32 = reinterpret_cast<unsigned*>(words);
      const unsigned long long w = (r >> 5) % (nwords * 2);
      const unsigned b32 = 1u << (r & 31);
      if constexpr (kMode == 8) {
        const unsigned old = __hip_atomic_fetch_or(w32 + w, b32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        local += !(old & b32);
      } else {
        __hip_atomic_fetch_or(w32 + w, b32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      const unsigned long long w = (r >> 6) % nwords;
      acc += words[w];
    }
  }
  if (kMode == 0 || kMode == 2 || kMode == 8) atomicAdd(claims, local);
  if (kMode == 5 && acc == 0x123456789ull) sink[0] = acc;
}

__global__ void popcount_kernel(const unsigned long long* w, unsigned long long n, unsigned long long* out) {
  unsigned long long c = 0;
  for (unsigned long long i = static_cast<unsigned long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<unsigned long long>(gridDim.x) * blockDim.x)
    c += __popcll(w[i]);
  atomicAdd(out, c);
}

template <int kMode>
double run(const char* name, unsigned long long* words, unsigned char* bytes, unsigned long long nwords,
           unsigned long long* dev_scalars, unsigned blocks, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  double best = 1e30;
  bool ok = true;
  for (int rep = 0; rep < reps; ++rep) {
    CK(hipMemset(words, 0, nwords * 8));
    CK(hipMemset(dev_scalars, 0, 32));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    scatter_kernel<kMode><<<blocks, kThreads>>>(words, bytes, nwords, dev_scalars, dev_scalars + 2, rep);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
    if (kMode == 0 || kMode == 2 || kMode == 8) {
      popcount_kernel<<<1024, 256>>>(words, nwords, dev_scalars + 1);
      unsigned long long h[2];
      CK(hipMemcpy(h, dev_scalars, 16, hipMemcpyDeviceToHost));
      if (h[0] != h[1]) ok = false;
      if (rep == 0) std::printf("  %-12s claims %llu popcount %llu\n", name, h[0], h[1]);
    }
  }
  const double ops = static_cast<double>(blocks) * kThreads * kPerThread;
  std::printf("%-12s %8.3f ms  %7.2f G ops/s  %s\n", name, best, ops / (best * 1e6), ok ? "ok" : "MISMATCH");
  return best;
}

int main(int argc, char** argv) {
  // argv[2]: vertices (default 64 Mi: an 8 MiB bitmap); 4847616 = soc-LiveJournal1's size
  const unsigned long long nverts = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : (1ull << 26);
  const unsigned long long nwords = (nverts + 511) / 512 * 8;
  const unsigned blocks = argc > 1 ? static_cast<unsigned>(std::atoi(argv[1])) : 24576;  // 100 M ops
  unsigned long long *words, *scal;
  unsigned char* bytes;
  CK(hipMalloc(&words, nwords * 8));
  CK(hipMalloc(&bytes, nwords * 64));
  CK(hipMalloc(&scal, 64));
  CK(hipMemset(bytes, 0, nwords * 64));
  std::printf("ops per kernel: %.1f M\n", blocks * double(kThreads) * kPerThread / 1e6);
  run<0>("agent-or", words, bytes, nwords, scal, blocks, 3);
  run<1>("agent-or-nr", words, bytes, nwords, scal, blocks, 3);
  run<2>("xcd-or", words, bytes, nwords, scal, blocks, 3);
  run<3>("byte-store", words, bytes, nwords, scal, blocks, 3);
  run<4>("xcd-byte", words, bytes, nwords, scal, blocks, 3);
  run<5>("rand-load", words, bytes, nwords, scal, blocks, 3);
  run<6>("probe-store", words, bytes, nwords, scal, blocks, 3);
  run<7>("xcd-probe-st", words, bytes, nwords, scal, blocks, 3);
  run<8>("agent-or32", words, bytes, nwords, scal, blocks, 3);
  run<9>("agent-or32-nr", words, bytes, nwords, scal, blocks, 3);
  return 0;
}
