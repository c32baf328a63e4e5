// tfs_crc_group.cpp -- the multi-GPU side of the C ABI (include/tfs_crc.h,
// "device group"): one context per local GPU, blocks routed by block id.
//
// The reference dataserver is one process with N PacketQueueThread workers
// (base_service.cpp:163-166,187-192) and a task thread; DataService::initialize
// (dataservice.cpp:151-377) is where it would create this group.  Files are
// independent and a block never straddles GPUs, so routing is
// block_id % size with no collective: each member owns a context (device
// tables, streams, pinned staging), a host worker thread bound to its GPU's
// NUMA node, and page-locked memory allocated from that node.  Batched group
// calls split their jobs by member and run the members concurrently.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tfs_crc.h"
#include "pin_registry.h"

namespace {

// NUMA node of a HIP device (its PCI function's numa_node), -1 when unknown.
int device_numa_node(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  for (char* p = bus; *p; ++p) *p = char(tolower(*p));
  char path[160];
  snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE* f = fopen(path, "r");
  if (!f) return -1;
  int node = -1;
  if (fscanf(f, "%d", &node) != 1) node = -1;
  fclose(f);
  return node;
}

// CPUs of NUMA node `node` that this process may run on.
bool node_cpus(int node, cpu_set_t* out) {
  CPU_ZERO(out);
  if (node < 0) return false;
  char path[96];
  snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = fopen(path, "r");
  if (!f) return false;
  char buf[4096] = {0};
  const size_t got = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[got] = 0;
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return false;
  for (char* p = buf; *p;) {  // "0-63,128-191"
    char* e = nullptr;
    const long a = strtol(p, &e, 10);
    if (e == p) break;
    long b = a;
    if (*e == '-') b = strtol(e + 1, &e, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &allowed)) CPU_SET(c, out);
    p = (*e == ',') ? e + 1 : e;
    if (*p == '\n') break;
  }
  return CPU_COUNT(out) > 0;
}

// One member: a context and the host thread that drives it.
struct Member {
  int device = -1;
  int numa = -1;
  tfs_crc_ctx* ctx = nullptr;
  std::thread worker;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> tasks;
  bool stop = false;
  std::atomic<bool> bound{false};  // worker runs on the GPU's NUMA node

  void run() {
    cpu_set_t cpus;
    if (node_cpus(numa, &cpus)) bound = sched_setaffinity(0, sizeof cpus, &cpus) == 0;  // this thread only
    (void)hipSetDevice(device);
    for (;;) {
      std::function<void()> t;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || !tasks.empty(); });
        if (tasks.empty()) return;
        t = std::move(tasks.front());
        tasks.pop_front();
      }
      t();
    }
  }
  void post(std::function<void()> t) {
    {
      std::lock_guard<std::mutex> g(mu);
      tasks.push_back(std::move(t));
    }
    cv.notify_one();
  }
};

// Run fn(member_index) on every member's worker and wait for all of them.
void run_on_members(std::vector<Member*>& ms, const std::function<void(uint32_t)>& fn) {
  std::mutex mu;
  std::condition_variable cv;
  uint32_t left = uint32_t(ms.size());
  for (uint32_t i = 0; i < ms.size(); ++i)
    ms[i]->post([&, i] {
      fn(i);
      std::lock_guard<std::mutex> g(mu);
      if (--left == 0) cv.notify_all();
    });
  std::unique_lock<std::mutex> lk(mu);
  cv.wait(lk, [&] { return left == 0; });
}

int worst_of(int a, int b) {
  if (a == TFS_SUCCESS) return b;
  if (a == TFS_EXIT_CHECK_CRC_ERROR && b != TFS_SUCCESS) return b;
  return a;
}

}  // namespace

struct tfs_crc_group {
  std::vector<Member*> members;
  std::mutex err_mu;  // members' workers report errors concurrently
  std::string last_error = "no error";
  void set_error(const std::string& e) {
    std::lock_guard<std::mutex> g(err_mu);
    last_error = e;
  }
};

extern "C" {

int tfs_crc32_device_numa_node(int device) { return device_numa_node(device); }

int tfs_crc_group_create(const int* devices, uint32_t n, tfs_crc_group** out) {
  if (!out) return TFS_EXIT_PARAMETER_ERROR;
  *out = nullptr;
  const int ndev = tfs_crc32_device_count();
  if (ndev <= 0) return TFS_CRC_EXIT_NO_DEVICE;
  std::vector<int> devs;
  if (devices) {
    if (n == 0) return TFS_EXIT_PARAMETER_ERROR;
    devs.assign(devices, devices + n);
  } else {
    for (int d = 0; d < ndev; ++d) devs.push_back(d);
  }
  auto* g = new tfs_crc_group();
  int rc = TFS_SUCCESS;
  for (int d : devs) {
    auto* m = new Member();
    m->device = d;
    rc = tfs_crc32_ctx_create(d, &m->ctx);
    if (rc != TFS_SUCCESS) {
      g->last_error = m->ctx ? tfs_crc32_last_error(m->ctx) : "tfs_crc32_ctx_create failed";
      if (m->ctx) tfs_crc32_ctx_destroy(m->ctx);
      delete m;
      break;
    }
    m->numa = device_numa_node(d);
    m->worker = std::thread([m] { m->run(); });
    g->members.push_back(m);
  }
  *out = g;  // returned even on failure so the caller can read the error; destroy it
  return rc;
}

int tfs_crc_group_destroy(tfs_crc_group* g) {
  if (!g) return TFS_EXIT_PARAMETER_ERROR;
  for (Member* m : g->members) {
    {
      std::lock_guard<std::mutex> lk(m->mu);
      m->stop = true;
    }
    m->cv.notify_all();
    m->worker.join();
    tfs_crc32_ctx_destroy(m->ctx);
    delete m;
  }
  delete g;
  return TFS_SUCCESS;
}

const char* tfs_crc_group_last_error(const tfs_crc_group* g) { return g ? g->last_error.c_str() : "null group"; }

uint32_t tfs_crc_group_size(const tfs_crc_group* g) { return g ? uint32_t(g->members.size()) : 0u; }

tfs_crc_ctx* tfs_crc_group_ctx(tfs_crc_group* g, uint32_t i) {
  return g && i < g->members.size() ? g->members[i]->ctx : nullptr;
}

uint32_t tfs_crc_group_member_of(const tfs_crc_group* g, uint32_t block_id) {
  return g && !g->members.empty() ? block_id % uint32_t(g->members.size()) : 0u;
}

tfs_crc_ctx* tfs_crc_group_ctx_for_block(tfs_crc_group* g, uint32_t block_id) {
  return tfs_crc_group_ctx(g, tfs_crc_group_member_of(g, block_id));
}

int tfs_crc_group_numa_node(const tfs_crc_group* g, uint32_t i) {
  return g && i < g->members.size() ? g->members[i]->numa : -1;
}

int tfs_crc_group_host_malloc(tfs_crc_group* g, uint32_t i, uint64_t bytes, void** p) {
  if (!g || i >= g->members.size() || !p) return TFS_EXIT_PARAMETER_ERROR;
  *p = nullptr;
  Member* m = g->members[i];
  int rc = TFS_SUCCESS;
  std::vector<Member*> one{m};
  // Allocated on the member's worker (bound to the GPU's NUMA node), following
  // that thread's local-node policy.
  run_on_members(one, [&](uint32_t) {
    hipError_t e = hipSetDevice(m->device);
    if (e == hipSuccess) e = hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocNumaUser | hipHostMallocPortable);
    void* dev = nullptr;
    if (e == hipSuccess && hipHostGetDevicePointer(&dev, *p, 0) == hipSuccess) tfscrc::pin_register(*p, bytes ? bytes : 1, dev);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      *p = nullptr;
      rc = TFS_CRC_EXIT_DEVICE_ERROR;
      g->set_error(std::string("hipHostMalloc: ") + hipGetErrorString(e));
    }
  });
  return rc;
}

int tfs_crc_group_host_free(tfs_crc_group* g, uint32_t i, void* p) {
  if (!g || i >= g->members.size()) return TFS_EXIT_PARAMETER_ERROR;
  if (p) tfscrc::pin_unregister(p);
  if (p && hipHostFree(p) != hipSuccess) return TFS_CRC_EXIT_DEVICE_ERROR;
  return TFS_SUCCESS;
}

int tfs_crc_group_blocks_verify(tfs_crc_group* g, tfs_block_verify_job* jobs, uint32_t njobs) {
  if (!g || g->members.empty() || (njobs && !jobs)) return TFS_EXIT_PARAMETER_ERROR;
  const uint32_t nm = uint32_t(g->members.size());
  std::vector<std::vector<uint32_t>> mine(nm);
  for (uint32_t j = 0; j < njobs; ++j) mine[jobs[j].block_id % nm].push_back(j);
  std::vector<int> worst(nm, TFS_SUCCESS);
  run_on_members(g->members, [&](uint32_t m) {
    tfs_crc_ctx* ctx = g->members[m]->ctx;
    for (uint32_t j : mine[m]) {
      tfs_block_verify_job& b = jobs[j];
      b.n_bad = 0;
      b.status = tfs_block_verify(ctx, b.image, b.image_len, b.metas, b.n, b.out_crc, b.out_status, &b.n_bad);
      worst[m] = worst_of(worst[m], b.status);
      if (b.status != TFS_SUCCESS && b.status != TFS_EXIT_CHECK_CRC_ERROR)
        g->set_error(tfs_crc32_last_error(ctx));
    }
  });
  int rc = TFS_SUCCESS;
  for (int w : worst) rc = worst_of(rc, w);
  return rc;
}

int tfs_crc_group_blocks_compact(tfs_crc_group* g, const uint32_t* block_ids, tfs_block_job* jobs, uint32_t njobs) {
  if (!g || g->members.empty() || (njobs && (!jobs || !block_ids))) return TFS_EXIT_PARAMETER_ERROR;
  const uint32_t nm = uint32_t(g->members.size());
  std::vector<std::vector<tfs_block_job>> mine(nm);
  std::vector<std::vector<uint32_t>> where(nm);
  for (uint32_t j = 0; j < njobs; ++j) {
    mine[block_ids[j] % nm].push_back(jobs[j]);
    where[block_ids[j] % nm].push_back(j);
  }
  std::vector<int> rcs(nm, TFS_SUCCESS);
  run_on_members(g->members, [&](uint32_t m) {
    if (mine[m].empty()) return;
    rcs[m] = tfs_blocks_compact(g->members[m]->ctx, mine[m].data(), uint32_t(mine[m].size()));
    if (rcs[m] != TFS_SUCCESS && rcs[m] != TFS_EXIT_CHECK_CRC_ERROR)
      g->set_error(tfs_crc32_last_error(g->members[m]->ctx));
  });
  int rc = TFS_SUCCESS;
  for (uint32_t m = 0; m < nm; ++m) {
    for (size_t k = 0; k < where[m].size(); ++k) jobs[where[m][k]] = mine[m][k];
    rc = worst_of(rc, rcs[m]);
  }
  return rc;
}

int tfs_crc_group_member_bound(const tfs_crc_group* g, uint32_t i) {
  return g && i < g->members.size() ? (g->members[i]->bound ? 1 : 0) : 0;
}

}  // extern "C"
