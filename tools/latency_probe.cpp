// latency_probe.cpp -- per-call latency of the small-batch paths of the C ABI
// (the dataserver's close path: one lease or a CloseBatcher batch per call).
// Build (CPU side, no HIP headers needed):
//   g++ -O2 -std=c++17 tools/latency_probe.cpp -Ltfs_amd -ltfs_crc -Wl,-rpath,$PWD/tfs_amd -o tools/latency_probe
// Prints one JSON object: p50/p99 microseconds per case.
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "../include/tfs_crc.h"
#include "../include/tfs_crc_testing.h"

// Keep the probe's threads on the GPU's NUMA node (as bench.py's lines and the
// device group's workers are): across the socket link every PCIe round trip is
// longer, and an unbound probe lands on either side from run to run.
static void bind_numa(int device) {
  const int node = tfs_crc32_device_numa_node(device);
  if (node < 0) return;
  char path[96];
  snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = fopen(path, "r");
  if (!f) return;
  char buf[4096] = {0};
  const size_t got = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[got] = 0;
  cpu_set_t cur, want;
  CPU_ZERO(&want);
  if (sched_getaffinity(0, sizeof cur, &cur) != 0) return;
  for (char* tok = strtok(buf, ",\n"); tok; tok = strtok(nullptr, ",\n")) {
    int a = 0, b = 0;
    const int k = sscanf(tok, "%d-%d", &a, &b);
    if (k < 1) continue;
    if (k == 1) b = a;
    for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &cur)) CPU_SET(c, &want);
  }
  if (CPU_COUNT(&want) > 0) sched_setaffinity(0, sizeof want, &want);
}

static double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, size_t(p * double(v.size())))];
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 300;
  bind_numa(0);
  tfs_crc_ctx* ctx = nullptr;
  if (tfs_crc32_ctx_create(0, &ctx) != TFS_SUCCESS) {
    fprintf(stderr, "ctx: %s\n", ctx ? tfs_crc32_last_error(ctx) : "?");
    return 1;
  }
  const uint32_t kFile = 65536, kMax = 64;
  void* pinned = nullptr;
  tfs_crc32_host_malloc_pinned(ctx, size_t(kMax) * kFile + 64, &pinned);
  std::vector<char> pageable(size_t(kMax) * kFile + 64);
  for (size_t i = 0; i < pageable.size(); ++i) pageable[i] = char(i * 2654435761u >> 13);
  memcpy(pinned, pageable.data(), pageable.size());
  void* dbuf = nullptr;
  tfs_crc32_dev_malloc(ctx, pageable.size(), &dbuf);
  tfs_crc32_memcpy(ctx, dbuf, pageable.data(), pageable.size(), nullptr);
  void *d_desc = nullptr, *d_ok = nullptr, *d_bad = nullptr;
  tfs_crc32_dev_malloc(ctx, 16 * kMax, &d_desc);
  tfs_crc32_dev_malloc(ctx, kMax, &d_ok);
  tfs_crc32_dev_malloc(ctx, 4, &d_bad);

  std::vector<tfs_crc_vdesc> vd(kMax);
  std::vector<uint32_t> crc(kMax);
  std::vector<uint8_t> ok(kMax);
  for (uint32_t i = 0; i < kMax; ++i) {
    tfs_crc_desc d{uint64_t(i) * kFile, kFile, 0};
    tfs_crc32_batch(ctx, &d, 1, pageable.data(), pageable.size(), &crc[i]);
    vd[i] = tfs_crc_vdesc{uint64_t(i) * kFile, kFile, crc[i]};
  }
  tfs_crc32_memcpy(ctx, d_desc, vd.data(), 16 * kMax, nullptr);

  std::string out = "{";
  auto run = [&](const char* name, std::function<int()> fn) {
    for (int i = 0; i < 20; ++i) fn();
    std::vector<double> us;
    us.reserve(iters);
    int bad = 0;
    for (int i = 0; i < iters; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      bad |= fn();
      const auto t1 = std::chrono::steady_clock::now();
      us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    char b[256];
    snprintf(b, sizeof b, "%s\"%s\": {\"p50_us\": %.1f, \"p99_us\": %.1f, \"status\": %d}", out.size() > 1 ? ", " : "",
             name, pct(us, 0.5), pct(us, 0.99), bad);
    out += b;
  };
  uint32_t nbad = 0;
  run("scalar_64k_pageable", [&] { return int(tfs_crc32(0, pageable.data(), kFile) != crc[0]); });
  // lone small bodies (the drop-in's floor): 16-80 B (in the
  // ring unit itself since round 6), 96 B, 1 KiB, 4 KiB from pageable memory
  for (uint32_t len : {16u, 32u, 64u, 80u, 96u, 1024u, 4096u, 16384u}) {
    uint32_t want = 0;
    tfs_crc_desc d{0, len, 0};
    tfs_crc32_batch(ctx, &d, 1, pageable.data(), len, &want);
    const std::string s = "scalar_" + std::to_string(len) + "B_pageable";
    run(s.c_str(), [&, len, want] { return int(tfs_crc32(0, pageable.data(), int32_t(len)) != want); });
  }
  run("memset_sync", [&] { return tfs_crc32_memset_device(ctx, d_bad, 0, 4, nullptr) | tfs_crc32_sync(ctx); });
  for (uint32_t n : {1u, 8u, 16u, 32u, 64u}) {
    std::string s = "verify_pinned_n" + std::to_string(n);
    run(s.c_str(), [&, n] {
      return tfs_crc32_verify(ctx, vd.data(), n, pinned, size_t(kMax) * kFile, crc.data(), ok.data(), &nbad);
    });
    s = "verify_pageable_n" + std::to_string(n);
    run(s.c_str(), [&, n] {
      return tfs_crc32_verify(ctx, vd.data(), n, pageable.data(), size_t(kMax) * kFile, crc.data(), ok.data(), &nbad);
    });
    s = "verify_device_n" + std::to_string(n);
    run(s.c_str(), [&, n] {
      return tfs_crc32_verify_device(ctx, static_cast<tfs_crc_vdesc*>(d_desc), n, dbuf, nullptr,
                                     static_cast<uint8_t*>(d_ok), nullptr, nullptr) |
             tfs_crc32_sync(ctx);
    });
  }
  tfs_crc_vdesc tiny{0, 4, 0};
  {
    tfs_crc_desc d{0, 4, 0};
    tfs_crc32_batch(ctx, &d, 1, pageable.data(), 4, &tiny.expected);
  }
  run("verify_pinned_4B", [&] { return tfs_crc32_verify(ctx, &tiny, 1, pinned, 4, nullptr, ok.data(), &nbad); });
  // A call after 1 ms without work: the resident kernel has left (idle exit)
  // and is relaunched by this call.
  {
    std::vector<double> us;
    int bad = 0;
    for (int i = 0; i < iters / 4; ++i) {
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
      const auto t0 = std::chrono::steady_clock::now();
      bad |= tfs_crc32_verify(ctx, vd.data(), 1, pinned, size_t(kMax) * kFile, crc.data(), ok.data(), &nbad);
      const auto t1 = std::chrono::steady_clock::now();
      us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    char b[256];
    snprintf(b, sizeof b, ", \"verify_pinned_n1_after_1ms_idle\": {\"p50_us\": %.1f, \"p99_us\": %.1f, \"status\": %d}",
             pct(us, 0.5), pct(us, 0.99), bad);
    out += b;
  }
  // One V1 RPC frame of a 64 KiB write (header: flag, length, type, version, id,
  // crc; base_packet.h:92-162), sealed, then verified as BasePacket::decode does.
  {
    std::vector<char> frame(24 + kFile);
    const uint32_t flag = TFS_PACKET_FLAG_V1, blen = kFile;
    const int16_t type = 1, version = 1;
    const uint64_t id = 7;
    memcpy(&frame[0], &flag, 4);
    memcpy(&frame[4], &blen, 4);
    memcpy(&frame[8], &type, 2);
    memcpy(&frame[10], &version, 2);
    memcpy(&frame[12], &id, 8);
    memcpy(&frame[24], pageable.data(), kFile);
    tfs_packet_desc pd{0, uint32_t(frame.size()), 0};
    int32_t pst = 0;
    uint32_t pcrc = 0, pbad = 0;
    tfs_packet_seal(ctx, &pd, 1, frame.data(), frame.size(), &pcrc, &pst);
    run("packet_verify_64k_pageable", [&] {
      return tfs_packet_verify(ctx, &pd, 1, frame.data(), frame.size(), &pcrc, &pst, &pbad) | pst;
    });
    memcpy(pinned, frame.data(), frame.size());
    run("packet_verify_64k_pinned", [&] {
      return tfs_packet_verify(ctx, &pd, 1, pinned, frame.size(), &pcrc, &pst, &pbad) | pst;
    });
  }
  uint64_t launches = 0, files = 0;
  tfs_crc32_resident_stats(ctx, &launches, &files);
  {
    char b[160];
    snprintf(b, sizeof b, ", \"resident\": {\"launches\": %llu, \"files\": %llu}", (unsigned long long)launches,
             (unsigned long long)files);
    out += b;
  }
  out += "}";
  printf("%s\n", out.c_str());
  tfs_crc32_host_free_pinned(ctx, pinned);
  tfs_crc32_ctx_destroy(ctx);
  return 0;
}
