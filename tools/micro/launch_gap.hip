// Launch-gap micro benchmark: how long does the GPU idle between a kernel and
// its stream successor when the successor (a) was submitted back to back,
// (b) in a later host batch, (c) in a later batch that the host submitted only
// after spinning on a host-mapped mailbox the GPU stamps (the device level
// loop's pattern, engine.cpp run_bitmap_device)?  Start/end read from the
// 100 MHz wall clock inside the kernels.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/launch_gap.hip -o bin/launch_gap
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

struct Big {
  unsigned long long* ts;
  int* mailbox;  // host-mapped; last kernel of a chain stamps its chain index
  int slot, chain, stamp;
  long pad[40];
};

__global__ void spin_kernel(long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (static_cast<long>(wall_clock64() - t0) < ticks) {
  }
}
__global__ void stamp_kernel(Big a) {
  if (threadIdx.x == 0 && blockIdx.x == 0) a.ts[2 * a.slot] = wall_clock64();
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == gridDim.x - 1) {
    a.ts[2 * a.slot + 1] = wall_clock64();
    if (a.stamp) __hip_atomic_store(a.mailbox, a.chain, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

#define CK(x) do { if ((x) != hipSuccess) { std::printf("HIP error %s\n", #x); return 1; } } while (0)

int main() {
  const int chains = 8, per = 4;
  unsigned long long* ts;
  CK(hipMalloc(&ts, sizeof(unsigned long long) * 2 * chains * per));
  int *mb_h, *mb_d;
  CK(hipHostMalloc(reinterpret_cast<void**>(&mb_h), 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&mb_d), mb_h, 0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int rate_khz = 0;
  CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
  const double us_per_tick = 1000.0 / rate_khz;
  const char* names[] = {"back to back", "host gap 30us", "mailbox-driven (enqueue c+1 after stamp c-1)",
                         "mailbox-driven, stamps without waiting"};
  for (int g : {1, 1024})
    for (int mode = 0; mode < 4; ++mode) {
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemsetAsync(ts, 0, sizeof(unsigned long long) * 2 * chains * per, st));
        CK(hipStreamSynchronize(st));
        __atomic_store_n(mb_h, -1, __ATOMIC_RELEASE);
        if (mode < 2) hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, st, static_cast<long>(2000 / us_per_tick));
        auto chain = [&](int c) {
          for (int k = 0; k < per; ++k) {
            Big b{};
            b.ts = ts;
            b.mailbox = mb_d;
            b.slot = c * per + k;
            b.chain = c;
            b.stamp = mode >= 2 && k == per - 1;
            hipLaunchKernelGGL(stamp_kernel, dim3(g), dim3(256), 0, st, b);
          }
        };
        if (mode >= 2) {
          chain(0);
          chain(1);
          for (int c = 2; c < chains; ++c) {
            if (mode == 2)
              while (__atomic_load_n(mb_h, __ATOMIC_ACQUIRE) < c - 2) {
              }
            chain(c);
          }
        } else {
          for (int c = 0; c < chains; ++c) {
            chain(c);
            const auto t0 = std::chrono::steady_clock::now();
            while (mode == 1 &&
                   std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() < 30) {
            }
          }
        }
        CK(hipStreamSynchronize(st));
        std::vector<unsigned long long> h(2 * chains * per);
        CK(hipMemcpy(h.data(), ts, h.size() * 8, hipMemcpyDeviceToHost));
        if (rep < 2) continue;
        double within = 0, between = 0, dur = 0;
        int nw = 0, nb = 0;
        for (int i = 1; i < chains * per; ++i) {
          const double gap = (static_cast<double>(h[2 * i]) - static_cast<double>(h[2 * i - 1])) * us_per_tick;
          if (i % per == 0) between += gap, ++nb;
          else within += gap, ++nw;
        }
        for (int i = 0; i < chains * per; ++i) dur += (h[2 * i + 1] - h[2 * i]) * us_per_tick;
        std::printf("grid %5d %-46s: gap within chain %.2f us, between chains %.2f us, kernel %.2f us\n", g,
                    names[mode], within / nw, between / nb, dur / (chains * per));
      }
    }
  return 0;
}
