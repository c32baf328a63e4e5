// Host cost of the HIP runtime calls on the close path's zero-copy post
// (measurement only): hipPointerGetAttributes (is_pinned_host), hipHostGetDevicePointer
// hipEventQuery and hipSetDevice, per call, from 1 and from 8 threads at once.
//
//   hipcc -O2 -std=c++17 tools/hipcall_cost.cpp -o tools/hipcall_cost && tools/hipcall_cost
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

static double per_call_ns(int nthreads, int iters, int which, void* pinned, hipEvent_t ev) {
  std::atomic<int> go{0};
  std::vector<std::thread> ts;
  std::vector<double> ns(size_t(nthreads), 0.0);
  for (int t = 0; t < nthreads; ++t)
    ts.emplace_back([&, t] {
      while (!go.load()) {
      }
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < iters; ++i) {
        if (which == 0) {
          hipPointerAttribute_t a;
          (void)hipPointerGetAttributes(&a, static_cast<char*>(pinned) + 64 * (i & 1023));
        } else if (which == 1) {
          void* d = nullptr;
          (void)hipHostGetDevicePointer(&d, static_cast<char*>(pinned) + 64 * (i & 1023), 0);
        } else if (which == 2) {
          (void)hipEventQuery(ev);
        } else {
          (void)hipSetDevice(0);
        }
      }
      ns[size_t(t)] = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() / iters;
    });
  go = 1;
  for (auto& th : ts) th.join();
  double m = 0;
  for (double v : ns) m = v > m ? v : m;
  return m;
}

int main() {
  void* pinned = nullptr;
  if (hipHostMalloc(&pinned, 4u << 20, hipHostMallocDefault) != hipSuccess) return 1;
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  (void)hipEventRecord(ev, nullptr);
  (void)hipDeviceSynchronize();
  const char* names[4] = {"hipPointerGetAttributes", "hipHostGetDevicePointer", "hipEventQuery", "hipSetDevice"};
  printf("{");
  for (int w = 0; w < 4; ++w) {
    (void)per_call_ns(1, 1000, w, pinned, ev);
    const double one = per_call_ns(1, 20000, w, pinned, ev);
    const double eight = per_call_ns(8, 20000, w, pinned, ev);
    printf("%s\"%s\": {\"ns_1_thread\": %.1f, \"ns_8_threads\": %.1f}", w ? ", " : "", names[w], one, eight);
  }
  printf("}\n");
  (void)hipHostFree(pinned);
  return 0;
}
