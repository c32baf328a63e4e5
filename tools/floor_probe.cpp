// floor_probe.cpp -- where the ~9 us of one lone small call goes.
// Measurement build only: links libtfs_crc_measure.so, whose resident kernel stamps
// each ring unit with the GPU's 100 MHz wall clock (tfs_crc32_res_trace) and whose
// synchronous path stamps the host side (tfs_crc32_res_trace_last).
//   (no HIP headers needed)
//   g++ -O2 -std=c++17 tools/floor_probe.cpp -Ltfs_amd -ltfs_crc_measure -Wl,-rpath,$PWD/tfs_amd -o tools/floor_probe
//   tools/floor_probe [iters]   -> one JSON object on stdout (TFS_FLOOR_FENCE=1: a second
//   pass with the resident kernel's acquire fence before each payload, TFS_CRC_RES_FENCE)
// Per call (a lone body through tfs_crc32_batch from page-locked memory, and the
// scalar drop-in tfs_crc32 from pageable memory) it splits the host's wall time into
//   host_pre     call entry -> the unit published (lock, slot, descriptor, staging copy)
//   post_to_go   published -> the GPU's poll returns with it   (needs the clock offset)
//   poll_rtt     the issue of that poll -> its return        (GPU clock: one PCIe read)
//   unit_rtt     the unit's four words back                   (GPU clock: one PCIe read)
//   fence        the kernel's acquire fence                   (GPU clock)
//   payload_loads wave 0's payload loads back                 (GPU clock: one PCIe read)
//   compute      the CRC (chains, wave and workgroup combine)  (GPU clock)
//   crc_to_seen  result store -> the host sees it             (needs the clock offset)
//   host_post    result seen -> the call returns
// post_to_go + crc_to_seen is measured without any offset ((seen - posted) - (crc - go));
// its split uses the offset estimate min(a) - min(b) over the calls, halved
// (a = go - posted, b = seen - crc: the fastest up and down legs taken as equal).
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
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
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, size_t(p * double(v.size())))];
}

struct Rec {
  double total, host_pre, host_post, poll_rtt, unit_rtt, fence, loads, compute, legs, a, b;
};

// One pass over the forms and sizes on a fresh context (its resident kernel reads
// TFS_CRC_RES_FENCE when tfs_crc32_res_trace arms the stamps).  crcs: every call's
// result, in order (compared across passes).
static int pass(int iters, std::string& out, const char* tag, std::vector<uint32_t>& crcs) {
  tfs_crc_ctx* ctx = nullptr;
  if (tfs_crc32_ctx_create(0, &ctx) != TFS_SUCCESS) {
    fprintf(stderr, "ctx: %s\n", ctx ? tfs_crc32_last_error(ctx) : "?");
    return 1;
  }
  void* trace = nullptr;
  if (tfs_crc32_host_malloc_pinned(ctx, 4096 * 64, &trace) != TFS_SUCCESS) return 1;
  memset(trace, 0, 4096 * 64);
  if (tfs_crc32_res_trace(ctx, trace) != TFS_SUCCESS) {
    fprintf(stderr, "res_trace: %s\n", tfs_crc32_last_error(ctx));
    return 1;
  }
  tfs_crc32_bind_thread(ctx);
  const size_t kBuf = 1 << 20;
  void* pinned = nullptr;
  tfs_crc32_host_malloc_pinned(ctx, kBuf, &pinned);
  std::vector<char> pageable(kBuf);
  for (size_t i = 0; i < kBuf; ++i) pageable[i] = char(i * 2654435761u >> 13);
  memcpy(pinned, pageable.data(), kBuf);
  volatile uint64_t* tr = static_cast<volatile uint64_t*>(trace);
  for (int form = 0; form < 2; ++form) {
    for (uint32_t len : {32u, 80u, 96u, 1024u, 4096u}) {
      std::vector<Rec> recs;
      int resident = 0, lost = 0;
      for (int it = -50; it < iters; ++it) {
        const uint64_t off = (uint64_t(it + 50) * 4099u) % (kBuf - len);
        uint32_t crc = 0;
        if (form == 0) {
          tfs_crc_desc d{off, len, 0u};
          if (tfs_crc32_batch(ctx, &d, 1, static_cast<char*>(pinned), kBuf, &crc) != TFS_SUCCESS) return 2;
        } else {
          int err = 0;
          crc = tfs_crc32_e(0, pageable.data() + off, int32_t(len), &err);
          if (err) return 2;
        }
        crcs.push_back(crc);
        uint64_t h[8];
        tfs_crc32_res_trace_last(ctx, h);
        if (it < 0) continue;
        if (!h[5]) continue;  // launched, not through the ring
        ++resident;
        volatile uint64_t* u = tr + 8u * (h[4] % 4096u);
        // the stamps are stored just before the result: give them a moment to land
        for (int spin = 0; spin < 100000 && u[5] == 0; ++spin) std::this_thread::yield();
        if (u[5] == 0) {
          ++lost;
          continue;
        }
        const double tick = 1e6 / double(h[6] ? h[6] : 100000);  // ns per wall-clock tick
        const double gi = double(u[0]) * tick, gg = double(u[1]) * tick, gu = double(u[2]) * tick,
                     gf = double(u[3]) * tick, gl = double(u[4]) * tick, gc = double(u[5]) * tick;
        const double enter = double(h[0]), posted = double(h[1]), seen = double(h[2]), done = double(h[3]);
        Rec r;
        r.total = (done - enter) / 1e3;
        r.host_pre = (posted - enter) / 1e3;
        r.host_post = (done - seen) / 1e3;
        r.poll_rtt = (gg - gi) / 1e3;
        r.unit_rtt = (gu - gg) / 1e3;
        r.fence = (gf - gu) / 1e3;
        r.loads = (gl - gf) / 1e3;
        r.compute = (gc - gl) / 1e3;
        r.legs = ((seen - posted) - (gc - gg)) / 1e3;
        r.a = (gg - posted) / 1e3;  // offset + up leg
        r.b = (seen - gc) / 1e3;    // down leg - offset
        recs.push_back(r);
        for (int w = 0; w < 8; ++w) u[w] = 0;
      }
      double amin = 1e300, bmin = 1e300;
      for (auto& r : recs) amin = std::min(amin, r.a), bmin = std::min(bmin, r.b);
      const double off_us = (amin - bmin) / 2;  // the fastest up and down legs taken as equal
      auto p50 = [&](auto f) {
        std::vector<double> v;
        for (auto& r : recs) v.push_back(f(r));
        return pct(v, 0.5);
      };
      std::vector<double> tot;
      for (auto& r : recs) tot.push_back(r.total);
      char b[1400];
      snprintf(b, sizeof b,
               ", \"%s%s_%u\": {\"calls\": %zu, \"resident\": %d, \"stamps_lost\": %d, \"p50_us\": {\"total\": %.2f, "
               "\"host_pre\": %.2f, \"post_to_go\": %.2f, \"poll_rtt\": %.2f, \"unit_rtt\": %.2f, \"fence\": %.2f, "
               "\"payload_loads\": %.2f, \"compute\": %.2f, \"crc_to_seen\": %.2f, \"host_post\": %.2f, "
               "\"legs_offset_free\": %.2f}, \"p99_total_us\": %.2f}",
               tag, form == 0 ? "batch_pinned" : "scalar_pageable", len, recs.size(), resident, lost,
               p50([](const Rec& r) { return r.total; }), p50([](const Rec& r) { return r.host_pre; }),
               p50([&](const Rec& r) { return r.a - off_us; }), p50([](const Rec& r) { return r.poll_rtt; }),
               p50([](const Rec& r) { return r.unit_rtt; }), p50([](const Rec& r) { return r.fence; }),
               p50([](const Rec& r) { return r.loads; }), p50([](const Rec& r) { return r.compute; }),
               p50([&](const Rec& r) { return r.b + off_us; }), p50([](const Rec& r) { return r.host_post; }),
               p50([](const Rec& r) { return r.legs; }), pct(tot, 0.99));
      out += b;
    }
  }
  tfs_crc32_bind_thread(nullptr);
  // no unit is outstanding: the idle resident kernel writes no more stamps
  tfs_crc32_host_free_pinned(ctx, pinned);
  tfs_crc32_host_free_pinned(ctx, trace);
  tfs_crc32_ctx_destroy(ctx);
  return 0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 400;
  bind_numa(0);
  std::string out = "{\"tool\": \"floor_probe\", \"iters\": " + std::to_string(iters);
  std::vector<uint32_t> crcs;
  if (int rc = pass(iters, out, "", crcs)) return rc;
  // TFS_FLOOR_FENCE=1 (measurement build): a second pass with the kernel's acquire
  // fence before each payload read (the form before its system-coherent loads) --
  // the fence's cost, and that no result changes
  const char* fe = getenv("TFS_FLOOR_FENCE");
  if (fe && atoi(fe)) {
    std::vector<uint32_t> fenced;
    setenv("TFS_CRC_RES_FENCE", "1", 1);
    if (int rc = pass(iters, out, "fenced_", fenced)) return rc;
    size_t diff = 0;
    for (size_t i = 0; i < crcs.size() && i < fenced.size(); ++i) diff += crcs[i] != fenced[i];
    out += ", \"fenced_results_differing\": " + std::to_string(diff) + ", \"calls_compared\": " +
           std::to_string(std::min(crcs.size(), fenced.size()));
    unsetenv("TFS_CRC_RES_FENCE");
  }
  out += "}";
  printf("%s\n", out.c_str());
  return 0;
}
