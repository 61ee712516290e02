// launch_ubench.hip — host cost of hipLaunchKernel on gfx950: one or several
// host threads, each launching back to back on its own stream, kernels that
// are empty or spin for a fixed time (one workgroup).  Answers whether a
// launch blocks once a stream has work queued (queue depth) and whether
// threads of one process slow each other's launches.
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/launch_ubench.hip -o tools/launch_ubench -lpthread
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

// spin for `ticks` of the 100 MHz constant clock (bounded: always exits)
__global__ void k_spin(uint64_t ticks, uint64_t *sink) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t x = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x++;
  if (threadIdx.x == 0 && x == 0xFFFFFFFFFFFFull) sink[blockIdx.x] = x;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Res {
  double per_launch_us = 0, max_launch_us = 0, wall_us = 0;
};

static Res run_thread(hipStream_t s, uint64_t *sink, int n, uint64_t ticks) {
  Res r;
  // warm-up
  hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, (uint64_t)0, sink);
  (void)hipStreamSynchronize(s);
  const double t0 = now_us();
  for (int i = 0; i < n; i++) {
    const double a = now_us();
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, ticks, sink);
    const double d = now_us() - a;
    if (d > r.max_launch_us) r.max_launch_us = d;
  }
  const double t1 = now_us();
  (void)hipStreamSynchronize(s);
  r.per_launch_us = (t1 - t0) / n;
  r.wall_us = now_us() - t0;
  return r;
}

int main() {
  uint64_t *sink = nullptr;
  if (hipMalloc(&sink, 4096) != hipSuccess) return 1;
  const int N = 2000;
  for (int nthreads : {1, 2, 4, 8}) {
    for (uint64_t us : {0, 20, 60}) {
      std::vector<hipStream_t> st(nthreads);
      for (auto &s : st)
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
      std::vector<Res> res(nthreads);
      std::vector<std::thread> th;
      const double t0 = now_us();
      for (int i = 0; i < nthreads; i++)
        th.emplace_back([&, i] { res[i] = run_thread(st[i], sink, N, us * 100); });
      for (auto &t : th) t.join();
      const double wall = now_us() - t0;
      double avg = 0, mx = 0;
      for (auto &r : res) {
        avg += r.per_launch_us / nthreads;
        mx = r.max_launch_us > mx ? r.max_launch_us : mx;
      }
      printf("threads %d  kernel %3llu us  host us per launch %7.1f  max %8.1f  wall ms %8.1f  (GPU-bound wall %6.1f ms)\n",
             nthreads, (unsigned long long)us, avg, mx, wall / 1e3, (double)N * us / 1e3);
      fflush(stdout);
      for (auto &s : st) (void)hipStreamDestroy(s);
    }
  }
  (void)hipFree(sink);
  return 0;
}
