// tfs_crc_abi.cpp -- host side of the C ABI declared in include/tfs_crc.h.
//
// Owns per-GPU contexts (stream, device-resident tables, device scratch and
// pinned staging pools) and drives the gfx950 kernels in tfs_crc_kernels.hip.
// There is deliberately no CPU CRC here: if a device call fails the error is
// returned (TFS_CRC_EXIT_DEVICE_ERROR / TFS_CRC_EXIT_NO_DEVICE), never computed
// on the host instead.
#include <emmintrin.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/tfs_crc.h"
#include "../../include/tfs_crc_testing.h"
#include "crc_math.h"
#include "pin_registry.h"
#include "tfs_crc_device.h"

namespace tfscrc {
hipError_t launch_crc_files(int mode, const uint8_t* base, const Desc* desc, uint32_t n, const Tables* tg,
                            uint32_t* out_crc, uint8_t* out_ok, uint32_t* n_bad, uint32_t* sched, hipStream_t stream,
                            int variant, uint32_t vseed, uint32_t* done_flag, uint32_t seq, unsigned cap,
                            const SplitArgs* split);
hipError_t launch_packet_parse(const uint8_t* base, const PacketDesc* pd, uint32_t n, int mode, Desc* desc,
                               int32_t* pre, hipStream_t stream);
hipError_t launch_packet_files(uint8_t* base, const PacketDesc* pd, uint32_t n, int mode, const Tables* tg,
                               uint32_t* crc, int32_t* status, uint32_t* n_bad, uint32_t* sched, hipStream_t stream,
                               unsigned cap);
hipError_t launch_packet_finish(uint8_t* base, const PacketDesc* pd, const Desc* desc, uint32_t n, int mode,
                                const int32_t* pre, const uint8_t* ok, uint32_t* crc, int32_t* status,
                                uint32_t* n_bad, hipStream_t stream);
hipError_t launch_block_verify_pipe(const uint8_t* image, uint64_t image_len, const RawMeta* metas,
                                    const CompactJob* jobs, uint32_t n, const Tables* tg, uint32_t* out_crc,
                                    int32_t* out_status, uint32_t* n_bad, uint32_t* sched, hipStream_t stream,
                                    int variant, unsigned cap);
hipError_t launch_compact_fused(const uint8_t* src, uint64_t src_len, const RawMeta* metas, const int32_t* flags,
                                const int64_t* dest_off, uint32_t n, uint8_t* dst, const Tables* tg, uint32_t* out_crc,
                                int32_t* out_status, uint32_t* n_bad, uint32_t* sched, hipStream_t stream,
                                int variant, unsigned cap);
hipError_t launch_compact_jobs(const uint8_t* src, uint64_t src_len, const CompactJob* jobs, uint32_t n, uint8_t* dst,
                               const Tables* tg, uint32_t* out_crc, int32_t* out_status, uint32_t* n_bad,
                               uint32_t* sched, hipStream_t stream, int variant, unsigned cap, const CSegArgs* seg);
hipError_t launch_synth_fill(uint64_t* dst, uint64_t nwords, uint64_t seed, uint64_t first_word, hipStream_t stream);
hipError_t launch_write_headers(uint8_t* image, const uint64_t* rec_off, const uint32_t* len, const uint32_t* crc,
                                uint64_t first_id, uint32_t n, hipStream_t stream);
hipError_t launch_write_packet_headers(uint8_t* base, const uint64_t* rec_off, const uint32_t* len, uint32_t n,
                                       int32_t pcode, int32_t version, uint64_t first_id, hipStream_t stream);
#ifdef TFS_CRC_MEASURE
hipError_t set_res_fence(uint32_t v);
hipError_t launch_membench(int pattern, const uint8_t* base, const Desc* desc, uint32_t n, uint64_t nbytes,
                           uint32_t* out, unsigned grid, hipStream_t stream);
#endif
hipError_t launch_resident(const Tables* tg, const ResHost* hs, uint32_t* left, uint32_t* dstate, unsigned grid,
                           uint32_t idle_ticks,
                           uint32_t life_ticks, uint32_t gen, hipStream_t stream, uint64_t* trace);
}  // namespace tfscrc

namespace tfscrc {

namespace {
struct PinRange {
  uintptr_t end;
  uintptr_t dev;
};
std::shared_mutex g_pin_mu;
std::map<uintptr_t, PinRange> g_pins;  // keyed by the allocation's first byte
}  // namespace

void pin_register(void* host, size_t bytes, void* dev) {
  if (!host || !dev) return;
  const uintptr_t h = reinterpret_cast<uintptr_t>(host);
  std::unique_lock<std::shared_mutex> g(g_pin_mu);
  g_pins[h] = PinRange{h + (bytes ? bytes : 1), reinterpret_cast<uintptr_t>(dev)};
}

void pin_unregister(void* host) {
  if (!host) return;
  std::unique_lock<std::shared_mutex> g(g_pin_mu);
  g_pins.erase(reinterpret_cast<uintptr_t>(host));
}

bool pin_lookup(const void* p, void** dev) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  std::shared_lock<std::shared_mutex> g(g_pin_mu);
  auto it = g_pins.upper_bound(a);
  if (it == g_pins.begin()) return false;
  --it;
  if (a >= it->second.end) return false;
  if (dev) *dev = reinterpret_cast<void*>(it->second.dev + (a - it->first));
  return true;
}

}  // namespace tfscrc

static_assert(sizeof(tfs_crc_desc) == 16 && sizeof(tfs_crc_vdesc) == 16, "descriptor ABI");
static_assert(sizeof(tfs_raw_meta) == sizeof(tfscrc::RawMeta), "RawMeta ABI");
static_assert(sizeof(tfs_file_info) == 36, "FileInfo ABI");
static_assert(sizeof(tfs_crc_stats) == 64, "stats ABI");
static_assert(sizeof(tfs_packet_desc) == sizeof(tfscrc::PacketDesc), "packet descriptor ABI");
static_assert(sizeof(tfs_compact_job) == sizeof(tfscrc::CompactJob) && sizeof(tfs_compact_job) == 40, "compact job ABI");

namespace {

using namespace tfscrc;

// Growable device allocation.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t reserve(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 4096);
    want = (want + 0xFFFF) & ~size_t(0xFFFF);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Growable pinned host allocation.  `coherent`: fine-grained memory for words
// the GPU writes while the host polls them (verdicts, completion flags).
struct PinBuf {
  void* p = nullptr;
  void* dev = nullptr;  // its device-visible address (looked up once per allocation)
  size_t cap = 0;
  bool coherent = false;
  hipError_t reserve(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    release();
    size_t want = std::max<size_t>(bytes, 4096);
    want = (want + 0xFFFF) & ~size_t(0xFFFF);
    hipError_t e = hipHostMalloc(&p, want, coherent ? hipHostMallocCoherent : hipHostMallocDefault);
    if (e == hipSuccess) {
      cap = want;
      // Completion words are compared with sequence numbers: recycled memory
      // must not hold one (0 is never a sequence number).
      if (coherent) memset(p, 0, want);
      if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess) {
        dev = nullptr;
        (void)hipGetLastError();
      }
      pin_register(p, cap, dev);
    }
    return e;
  }
  void release() {
    if (p) {
      pin_unregister(p);
      (void)hipHostFree(p);
    }
    p = nullptr;
    dev = nullptr;
    cap = 0;
  }
};

// One in-flight host-memory submission (async API) or the scratch of a sync call.
struct Slot {
  DevBuf d_data, d_desc, d_crc, d_ok, d_bad, d_aux;
  PinBuf h_data, h_crc, h_ok, h_bad, h_desc, h_flag;
  PinBuf h_res;  // resident form: one {crc, seq} result word per file
  hipEvent_t done = nullptr;
  // A synchronous slot's own stream for wide in-place launches (no copies): the
  // launches of concurrent calls overlap, so the next buffer's waves fill the
  // link while the last waves of the previous one drain (made on first use).
  hipStream_t wide_stream = nullptr;
  bool busy = false;
  uint64_t ticket = 0;
  int status = TFS_SUCCESS;
  bool count_bad = false;  // zero-copy launch: n_bad is counted from h_ok
  bool spin = false;       // zero-copy launch: completion = h_flag reaching `seq`
  bool resident = false;   // posted to the resident kernel's ring (no launch, no s.done)
  uint32_t res_first = 0;  // ... as units [res_first, res_first + n)
  uint32_t seq = 0;
  Slot() { h_crc.coherent = h_ok.coherent = h_bad.coherent = h_flag.coherent = h_res.coherent = true; }
  // user outputs for the async path
  uint32_t n = 0;
  uint32_t* out_crc = nullptr;
  uint8_t* out_ok = nullptr;
  uint32_t* n_bad = nullptr;
  void release() {
    d_data.release(); d_desc.release(); d_crc.release(); d_ok.release(); d_bad.release(); d_aux.release();
    h_data.release(); h_crc.release(); h_ok.release(); h_bad.release(); h_desc.release(); h_flag.release();
    h_res.release();
    if (done) (void)hipEventDestroy(done);
    done = nullptr;
    if (wide_stream) (void)hipStreamDestroy(wide_stream);  // (synchronized by the caller)
    wide_stream = nullptr;
  }
};

// Sequence numbers of zero-copy submissions (completion flags, resident result
// words): process-wide, so a word in page-locked memory recycled from another
// context can never carry the value a new submission waits for.
std::atomic<uint32_t> g_flag_seq{0};

constexpr int kSlots = 4;
constexpr int kSyncSlots = 16;  // synchronous host calls in flight at once (CloseBatcher kMaxInFlight)

struct CompactSlot {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  DevBuf d_src, d_dst, d_aux;
  PinBuf h_aux, h_status, h_stage;
  std::vector<uint32_t> live_idx;
  tfs_block_job* job = nullptr;
  // A zero-copy group (compact_enqueue_group): its jobs and, per job, where its
  // records start in live_idx / the status array.
  std::vector<tfs_block_job*> gjobs;
  std::vector<uint32_t> gstart;
  std::vector<CompactJob> gjob_list;
  bool busy = false;
  void release() {
    d_src.release(); d_dst.release(); d_aux.release();
    h_aux.release(); h_status.release(); h_stage.release();
    if (done) (void)hipEventDestroy(done);
    if (stream) (void)hipStreamDestroy(stream);
    done = nullptr;
    stream = nullptr;
  }
};
constexpr int kCompactSlots = 8;          // slots allocated; ctx->compact_slots of them are used
constexpr uint32_t kSchedSlots = 256;
constexpr uint32_t kForeignSlots = 64;    // the last 64 scheduler slots: launches on streams the ctx does not own
constexpr uint32_t kOwnedSlots = kSchedSlots - kForeignSlots;
// Measurement build only (TFS_CRC_VARIANT; the product's ctx->variant is a constant 0):
constexpr int kVariantDmaCompact = 8;      // DMA staging for host compaction / block verify / small batches
#ifdef TFS_CRC_MEASURE
constexpr int kVariantStagedWide = 52;     // wide page-locked host batches staged by DMA (the round-4 form; A/B)
constexpr int kVariantWideCtxStream = 53;  // wide in-place launches on the ctx stream (the round-5 form; A/B)
#else
constexpr int kVariantStagedWide = -1;
constexpr int kVariantWideCtxStream = -1;
#endif
// A context that posted a close batch this recently keeps the resident kernel's
// CUs out of its device's throughput launches even while the kernel is between
// lifetimes.
constexpr int64_t kResRecentNs = 50'000'000;
constexpr uint64_t kZeroCopySpan = 8ull << 20;  // page-locked batches up to this span are read in place
constexpr uint32_t kZeroCopyOutFiles = 65536;   // staged batches up to this many files: verdicts written to host

}  // namespace

struct tfs_crc_ctx {
  int device = -1;
  uint64_t id = 0;  // process-unique (live-context registry)
  hipStream_t stream = nullptr;
  // The latency path's streams (zero-copy small batches; the resident kernel's
  // res_stream) have the device's greatest priority: they never queue behind
  // a throughput launch on `stream`, and their workgroups are dispatched first.
  hipStream_t lat_stream = nullptr;
  int lat_prio = 0;
  Tables* d_tables = nullptr;
  std::mutex mu;
  std::mutex err_mu;
  char last_error[512] = "no error";
  Slot slots[kSlots];  // async submissions, block verify, packets
  // Synchronous host calls (tfs_crc32_batch / _verify and the scalar drop-in):
  // their own slots, taken and launched under `mu`, waited on outside it.
  Slot sync_slots[kSyncSlots];
  std::condition_variable sync_cv;
  CompactSlot cslots[kCompactSlots];
  uint64_t next_ticket = 1;
  // Work-distribution counters: kSchedSlots slots of 8 ticket counters and a
  // finished-waves counter (one 256-byte line each).  The first kOwnedSlots
  // belong to streams this ctx owns (slot 0 = ctx->stream, the compaction
  // streams, tfs_crc32_stream_create), so the launches sharing one are ordered
  // and each leaves it zeroed (launch_exit in the kernels).  Launches on any
  // other stream take a slot of the foreign pool per launch (sched_acquire).
  uint32_t* d_sched = nullptr;
  std::mutex sched_mu;
  std::vector<hipStream_t> sched_streams;  // owned stream of slot k (nullptr = free)
  hipEvent_t foreign_done[kForeignSlots] = {};  // behind the last launch on foreign slot k
  bool foreign_busy[kForeignSlots] = {};
  uint32_t foreign_next = 0;
  uint64_t foreign_launches = 0;
  int compact_slots = 8;  // blocks in flight in tfs_blocks_compact (TFS_CRC_COMPACT_SLOTS, 1..8)
  uint32_t compact_group = 64;  // page-locked blocks per launch in tfs_blocks_compact (TFS_CRC_COMPACT_GROUP, 1..256)
#ifdef TFS_CRC_MEASURE
  int variant = 0;  // kernel variant (TFS_CRC_VARIANT; measurement build only)
#else
  static constexpr int variant = 0;  // the product library holds one form of each kernel
#endif
  unsigned cus = kMaxGrid;  // compute units of the device: throughput grids are at most this
  // Split files (tfs_crc_device.h SplitArgs): one plan per owned scheduler slot,
  // so a launch orders only behind the earlier launches of its own stream, and
  // split launches on different owned streams overlap; the foreign
  // slots share the plan at index kOwnedSlots, ordered by plan_done (plan_index,
  // ADVICE r4).  plan_mu[k] is held from the plan's setup to the launch.
  DevBuf plans[kSchedSlots];
  hipEvent_t plan_done[kSchedSlots] = {};  // behind the latest split launch of slot k
  std::mutex plan_mu[kSchedSlots];
  // The latest split launch (tfs_crc32_split_stats): its slot, stream, files and grid.
  std::mutex last_split_mu;
  int last_split_slot = -1;
  uint32_t last_split_n = 0, last_split_cap = 0, last_split_grid = 0;
  uint64_t split_launches = 0;
  std::atomic<bool> cu_reserve{true};   // leave a live resident kernel's CUs out of throughput launches
  std::atomic<int> split_files{1};  // throughput launches split files > kSplitMin (tfs_crc32_set_split): 0 off
  std::atomic<uint32_t> cseg_lg{0};  // segmented compaction: 1 KiB << cseg_lg segments, 0 = whole records
  std::atomic<bool> cseg_auto{true};  // the default rule (cseg_lg()) until tfs_crc32_set_compact_segment
  std::atomic<uint32_t> inject_skip{0}, inject_count{0};  // tfs_crc32_inject_device_error
  DevBuf packet_scratch;  // device-resident packet calls (parse descriptors, verdicts)
  hipStream_t packet_scratch_stream = nullptr;
  // Resident form for the synchronous zero-copy batches of at
  // most kWgMaxFiles files: ring in page-locked fine-grained memory, device
  // cursor/counters, its own stream.  All fields under `mu`.
  bool resident = true;  // TFS_CRC_RESIDENT=0 launches every batch instead
  unsigned res_grid = 16;  // workgroups of the resident kernel (TFS_CRC_RESIDENT_WGS)
  uint32_t res_idle_us = 200, res_life_us = 10000;  // TFS_CRC_RESIDENT_IDLE_US / _LIFE_US
  ResHost* res_host = nullptr;
  ResHost* res_host_d = nullptr;  // its device-visible address
  // The ring in device memory the host writes through the PCIe BAR (fine-grained,
  // CPU-mapped, on a large-BAR device): the workgroups poll
  // HBM instead of host memory (0.44 against 1.48 us a poll), and bodies of up to
  // kResLandMax bytes land there too.  `left` (GPU-written, host-read) stays in
  // host memory.  Without a large BAR the ring is in page-locked host memory.
  bool res_vram = false;
  bool res_vram_want = true;  // TFS_CRC_RESIDENT_VRAM=0: the ring in page-locked host memory
  void* res_left_block = nullptr;  // the page-locked ResHost holding `left` (and the ring, unless res_vram)
  int64_t res_bar_ns = -1;         // 4 KiB written through the BAR at setup (calibration), -1: not tried
  uint8_t* res_land = nullptr;     // landing slots in device memory (res_vram only), kResUnits x kResLandMax
  uint32_t* res_left = nullptr;    // host address of the `left` word
  uint32_t* res_left_d = nullptr;  // its device-visible address
  uint32_t* res_state = nullptr;
  hipStream_t res_stream = nullptr;
  hipEvent_t res_event = nullptr;
  bool res_running = false;  // a launch was made and res_event recorded behind it
  uint32_t res_published = 0;
  uint32_t res_idle_ticks = 0, res_life_ticks = 0;
  uint64_t res_launches = 0, res_files = 0;
  uint64_t res_ring_full = 0;  // batches launched because the ring had no room (tfs_crc32_stats)
  uint64_t* res_trace_dev = nullptr;  // measurement build: per-unit stamps (tfs_crc32_res_trace); null in the product
#ifdef TFS_CRC_MEASURE
  // tfs_crc32_res_trace_last: host stamps (steady clock ns) of the last synchronous call
  std::atomic<int64_t> tr_enter{0}, tr_posted{0}, tr_seen{0}, tr_done{0};
  std::atomic<uint32_t> tr_first{0}, tr_resident{0};
  int tr_khz = 0;
#endif
  // tfs_crc32_stats: synchronous host calls, their bodies, lone calls, lone calls
  // under TFS_CRC_LONE_CROSSOVER and their bytes
  std::atomic<uint64_t> st_calls{0}, st_files{0}, st_lone{0}, st_lone_small{0}, st_lone_small_bytes{0};
  // Read without ctx->mu by other contexts' throughput launches (throughput_cap):
  std::atomic<uint32_t> res_gen{0};           // generation of the latest resident launch
  std::atomic<int64_t> res_last_post_ns{0};   // steady-clock time of the latest post
  std::atomic<bool> res_ring{false};          // ring set up (res_host valid)
};

namespace {

int set_err(tfs_crc_ctx* ctx, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (ctx) {
    std::lock_guard<std::mutex> g(ctx->err_mu);
    memcpy(ctx->last_error, buf, sizeof buf);
  }
  return code;
}

#define HIP_TRY(ctx, expr)                                                                                   \
  do {                                                                                                       \
    hipError_t e_ = (expr);                                                                                  \
    if (e_ != hipSuccess)                                                                                    \
      return set_err((ctx), TFS_CRC_EXIT_DEVICE_ERROR, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                     __FILE__, __LINE__);                                                                    \
  } while (0)

void build_tables(Tables* t) {
  make_slice_tables(t->slice, 4);
  for (int ri = 0; ri < kNumRuns; ++ri) {
    const uint64_t run = uint64_t(16) << ri;
    make_shift_table5(t->stripe[ri], 63 * run);
    make_shift_table5(t->stripe64[ri], 64 * run);
    for (int j = 0; j < kLevels; ++j) make_shift_table5(t->level[ri][j], run << j);
    make_shift_table(t->stripe8[ri], 63 * run);
    make_shift_table(t->stripe64_8[ri], 64 * run);
    for (int j = 0; j < kLevels; ++j) make_shift_table(t->level8[ri][j], run << j);
  }
  make_shift_table5(t->wg_jump, 16ull * (64ull * kWgWaves - 1ull));
  make_shift_table5(t->seg_shift, kSegBytes);
  for (uint32_t lg = kCSegLgMin; lg <= kCSegLgMax; ++lg) make_shift_table5(t->cseg_shift[lg - kCSegLgMin], 1024ull << lg);
  for (int j = 0; j < kWgLevels; ++j) make_shift_table5(t->wg_level[j], 16ull << j);
}

bool is_pinned_host(const void* p) {
  if (pin_lookup(p, nullptr)) return true;  // allocated here: no runtime query
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// Device-visible address of page-locked host address p: the registry, else the
// runtime.
bool host_dev_ptr(const void* p, void** dev) {
  if (pin_lookup(p, dev)) return true;
  if (hipHostGetDevicePointer(dev, const_cast<void*>(p), 0) == hipSuccess) return true;
  (void)hipGetLastError();
  *dev = nullptr;
  return false;
}

// Range of base actually touched by n descriptors (offset, len pairs).
template <typename D>
bool span_of(const D* d, uint32_t n, uint64_t base_len, uint64_t* lo, uint64_t* hi) {
  uint64_t a = UINT64_MAX, b = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t e = d[i].offset + d[i].len;
    if (e < d[i].offset || e > base_len) return false;
    if (d[i].len == 0) continue;
    a = std::min(a, d[i].offset);
    b = std::max(b, e);
  }
  if (a == UINT64_MAX) a = b = 0;
  *lo = a & ~uint64_t(255);  // keep the device copy 256-aligned modulo the host offset
  *hi = b;
  return true;
}

// Stage the touched span of a host buffer onto the device in slot s.  Returns
// the device pointer that corresponds to host `base` (may point before the
// allocation; only [lo, hi) is valid).
int stage_span(tfs_crc_ctx* ctx, Slot& s, const void* base, uint64_t lo, uint64_t hi, const uint8_t** d_base,
               hipStream_t st = nullptr) {
  if (!st) st = ctx->stream;
  const uint64_t bytes = hi - lo;
  HIP_TRY(ctx, s.d_data.reserve(bytes + 16));
  const uint8_t* src = static_cast<const uint8_t*>(base) + lo;
  if (bytes) {
    if (is_pinned_host(base)) {
      HIP_TRY(ctx, hipMemcpyAsync(s.d_data.p, src, bytes, hipMemcpyHostToDevice, st));
    } else {
      HIP_TRY(ctx, s.h_data.reserve(bytes));
      memcpy(s.h_data.p, src, bytes);
      HIP_TRY(ctx, hipMemcpyAsync(s.d_data.p, s.h_data.p, bytes, hipMemcpyHostToDevice, st));
    }
  }
  *d_base = static_cast<const uint8_t*>(s.d_data.p) - lo;
  return TFS_SUCCESS;
}

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// (Caller holds sched_mu.)  Give stream `st` its own self-resetting slot.
hipError_t bind_owned_stream_locked(tfs_crc_ctx* ctx, hipStream_t st) {
  size_t k = 0;
  while (k < ctx->sched_streams.size() && ctx->sched_streams[k] != st && ctx->sched_streams[k] != nullptr) ++k;
  if (k < ctx->sched_streams.size()) {
    ctx->sched_streams[k] = st;
    return hipSuccess;
  }
  if (k >= kOwnedSlots) return hipErrorOutOfMemory;  // more than 192 live ctx-owned streams
  ctx->sched_streams.push_back(st);
  return hipSuccess;
}

hipError_t bind_owned_stream(tfs_crc_ctx* ctx, hipStream_t st) {
  std::lock_guard<std::mutex> g(ctx->sched_mu);
  return bind_owned_stream_locked(ctx, st);
}

// The scheduler slot one launch on stream `st` uses (see tfs_crc_ctx::d_sched).
// A ctx-owned stream has its own slot: launches on one stream are ordered and
// each leaves its slot zeroed, so no memset launch is needed.  Any other stream
// (a caller's hipStream_t) takes the next slot of the foreign pool: the launch
// that used it last is waited for, and the slot is zeroed on `st` before the
// kernel -- so a caller's stream never depends on another launch having left a
// slot clean, and two unordered streams never share counters.  hipStreamPerThread
// is refused: it is one handle for a different queue on every thread.
struct SchedLease {
  uint32_t* slot = nullptr;
  int foreign = -1;
};

int sched_acquire(tfs_crc_ctx* ctx, hipStream_t st, SchedLease* L) {
  if (st == hipStreamPerThread)
    return set_err(ctx, TFS_EXIT_PARAMETER_ERROR,
                   "hipStreamPerThread is not accepted (a different queue per thread behind one handle); pass NULL, a "
                   "tfs_crc32_stream_create stream or a stream of your own");
  std::unique_lock<std::mutex> lk(ctx->sched_mu);
  for (size_t k = 0; k < ctx->sched_streams.size(); ++k)
    if (ctx->sched_streams[k] == st) {
      L->slot = ctx->d_sched + (kSchedSlotBytes / 4u) * k;
      L->foreign = -1;
      return TFS_SUCCESS;
    }
  int k = -1;
  for (uint32_t i = 0; i < kForeignSlots && k < 0; ++i) {
    const uint32_t c = (ctx->foreign_next + i) % kForeignSlots;
    if (!ctx->foreign_busy[c]) k = int(c);
  }
  if (k < 0) return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "all %u foreign-stream slots in use", kForeignSlots);
  ctx->foreign_next = uint32_t(k + 1) % kForeignSlots;
  ctx->foreign_busy[k] = true;
  ++ctx->foreign_launches;
  hipEvent_t prev = ctx->foreign_done[k];
  lk.unlock();
  uint32_t* slot = ctx->d_sched + (kSchedSlotBytes / 4u) * (kOwnedSlots + uint32_t(k));
  hipError_t e = hipSuccess;
  if (prev) e = hipEventSynchronize(prev);  // the slot's previous launch (normally long finished)
  if (e == hipSuccess) e = hipMemsetAsync(slot, 0, kSchedSlotBytes, st);
  if (e != hipSuccess) {
    std::lock_guard<std::mutex> g(ctx->sched_mu);
    ctx->foreign_busy[k] = false;
    return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "foreign-stream slot: %s", hipGetErrorString(e));
  }
  L->slot = slot;
  L->foreign = k;
  return TFS_SUCCESS;
}

// After the launch that used lease L on `st` (launch_rc its result).  A launch
// that failed leaves an owned slot zeroed again on its stream (launch_exit never
// ran); a foreign slot gets the event its next user waits for.
int sched_release(tfs_crc_ctx* ctx, hipStream_t st, const SchedLease& L, hipError_t launch_rc, const char* what) {
  hipError_t e = hipSuccess;
  if (launch_rc != hipSuccess) (void)hipMemsetAsync(L.slot, 0, kSchedSlotBytes, st);
  if (L.foreign >= 0) {
    std::lock_guard<std::mutex> g(ctx->sched_mu);
    hipEvent_t& ev = ctx->foreign_done[L.foreign];
    if (!ev) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ev, st);
    if (e != hipSuccess && ev) {
      (void)hipEventDestroy(ev);  // no stale event: the next user of the slot synchronises the stream instead
      ev = nullptr;
      (void)hipStreamSynchronize(st);
    }
    ctx->foreign_busy[L.foreign] = false;
  }
  if (launch_rc != hipSuccess)
    return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "%s launch failed: %s", what, hipGetErrorString(launch_rc));
  if (e != hipSuccess) return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "%s: %s", what, hipGetErrorString(e));
  return TFS_SUCCESS;
}

// Workgroups of a throughput launch (crc_files_kernel, compact_pipe_kernel: one
// persistent workgroup per CU).  A resident kernel (§3.7 of DESIGN.md) holds
// res_grid CUs of its device while it lives; a throughput launch that asked
// for every CU would then wait with res_grid workgroups until it leaves (up to
// its lifetime, 10 ms), and a resident kernel launched behind a full-grid launch
// waits for CUs until that launch ends.  So while any context on this device
// has a resident kernel alive or posted a batch within kResRecentNs, throughput
// launches leave its CUs free.
bool resident_live(const tfs_crc_ctx* c, int64_t now) {
  if (!c->res_ring.load(std::memory_order_acquire)) return false;
  const uint32_t gen = c->res_gen.load(std::memory_order_acquire);
  const bool alive = gen != 0 && __atomic_load_n(c->res_left, __ATOMIC_ACQUIRE) != gen;
  return alive || now - c->res_last_post_ns.load(std::memory_order_relaxed) < kResRecentNs;
}

// Host side of a zero-copy launch's completion: spin on the page-locked flag
// the kernel's last workgroup stores (launch_exit); the event recorded behind
// the kernel is polled now and then so a failed launch is reported, never
// waited on forever.
int wait_flag(tfs_crc_ctx* ctx, Slot& s) {
  volatile uint32_t* fl = static_cast<volatile uint32_t*>(s.h_flag.p);
  for (uint32_t spins = 1; *fl != s.seq; ++spins) {
    __builtin_ia32_pause();
    if ((spins & 255u) == 0) {
      const hipError_t e = hipEventQuery(s.done);
      if (e == hipSuccess) {
        if (*fl == s.seq) break;
        return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "kernel completed without its completion flag (seq %u)",
                       s.seq);
      }
      if (e != hipErrorNotReady)
        return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "zero-copy launch failed: %s", hipGetErrorString(e));
    }
  }
  return TFS_SUCCESS;
}

// ---- resident form -------------------------------------------------------------
// Contexts whose resident kernel may be running.  At process exit (a caller that
// never destroys its context -- the scalar drop-in's default context) every such
// kernel is stopped and waited for through host memory only, before the HIP
// runtime tears down and unmaps its ring.
std::mutex g_res_mu;
std::vector<tfs_crc_ctx*> g_res_ctxs;

void resident_atexit() {
  std::lock_guard<std::mutex> g(g_res_mu);
  for (tfs_crc_ctx* c : g_res_ctxs) {
    ResHost* H = c->res_host;
    if (!H || !c->res_running) continue;
    const uint32_t gen = uint32_t(c->res_launches);
    __atomic_store_n(&H->published, uint64_t(c->res_published) | (uint64_t(1) << 32), __ATOMIC_RELEASE);
    _mm_sfence();  // a ring in device memory: the store leaves the write-combining buffer now
    for (int i = 0; i < 200000 && __atomic_load_n(c->res_left, __ATOMIC_ACQUIRE) != gen; ++i) __builtin_ia32_pause();
  }
}

// A BAR the host writes slower than this (4 KiB, write-combined: ~100 ns) is not
// used for the ring.
constexpr int64_t kResBarMaxNs = 2000;

// (Caller holds ctx->mu.)  Ring, device state, stream and event, made on first use.
int resident_setup(tfs_crc_ctx* ctx) {
  if (ctx->res_host) return TFS_SUCCESS;
  static std::once_flag atexit_once;
  std::call_once(atexit_once, [] { std::atexit(resident_atexit); });
  int khz = 0;
  HIP_TRY(ctx, hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device));
  if (khz <= 0) khz = 100000;
  ctx->res_idle_ticks = uint32_t(uint64_t(ctx->res_idle_us) * uint64_t(khz) / 1000u);
  ctx->res_life_ticks = uint32_t(std::min<uint64_t>(uint64_t(ctx->res_life_us) * uint64_t(khz) / 1000u, 0x7fffffffu));
  void* h = nullptr;
  HIP_TRY(ctx, hipHostMalloc(&h, sizeof(ResHost), hipHostMallocCoherent | hipHostMallocMapped));
  memset(h, 0, sizeof(ResHost));
  void* hd = nullptr;
  if (hipHostGetDevicePointer(&hd, h, 0) != hipSuccess) {
    (void)hipHostFree(h);
    return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "resident ring: hipHostGetDevicePointer failed");
  }
  ctx->res_left = &static_cast<ResHost*>(h)->left;
  ctx->res_left_d = &static_cast<ResHost*>(hd)->left;
  // The ring itself in fine-grained device memory the CPU writes through the BAR
  // (a large-BAR device only: every byte of device memory CPU-mapped).
  void* dv = nullptr;
  int large_bar = 0;
  if (ctx->res_vram_want && hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, ctx->device) == hipSuccess &&
      large_bar) {
    void* land = nullptr;
    if (hipExtMallocWithFlags(&dv, sizeof(ResHost), hipDeviceMallocFinegrained) != hipSuccess ||
        hipExtMallocWithFlags(&land, size_t(kResUnits) * kResLandMax, hipDeviceMallocFinegrained) != hipSuccess) {
      (void)hipGetLastError();
      if (dv) (void)hipFree(dv);
      dv = nullptr;
    } else {
      ctx->res_land = static_cast<uint8_t*>(land);
    }
  }
  void* st = nullptr;
  // The device state (done counts, exit line) is zeroed on the kernel's own stream
  // and waited for: a recycled allocation may hold a previous context's counts,
  // and a plain hipMemset on the null stream is not ordered before a kernel on a
  // non-blocking stream (a stale done count makes a workgroup wait for a unit
  // that is never posted while the host relaunches the kernel for its batch).
  if (hipMalloc(&st, kResStateBytes) != hipSuccess ||
      hipStreamCreateWithPriority(&ctx->res_stream, hipStreamNonBlocking, ctx->lat_prio) != hipSuccess ||
      hipMemsetAsync(st, 0, kResStateBytes, ctx->res_stream) != hipSuccess ||
      hipStreamSynchronize(ctx->res_stream) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->res_event, hipEventDisableTiming) != hipSuccess ||
      (dv && (hipMemsetAsync(dv, 0, sizeof(ResHost), ctx->res_stream) != hipSuccess ||
              hipStreamSynchronize(ctx->res_stream) != hipSuccess))) {
    (void)hipHostFree(h);
    if (dv) (void)hipFree(dv);
    if (ctx->res_land) (void)hipFree(ctx->res_land);
    ctx->res_land = nullptr;
    if (st) (void)hipFree(st);
    if (ctx->res_stream) (void)hipStreamDestroy(ctx->res_stream);
    ctx->res_stream = nullptr;
    return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "resident ring: device state allocation failed");
  }
  // Calibrate the host's writes through the BAR: 4 KiB of zeros over the (zeroed)
  // ring, best of three.  Write-combined, that is ~0.1 us; a box whose BAR the
  // CPU maps uncached takes microseconds per 16-byte store (one such mapping was
  // seen, 96-byte calls 2.5 us slower), and the ring then stays in host memory.
  if (dv) {
    alignas(64) static const uint8_t zeros[4096] = {};
    int64_t best = INT64_MAX;
    for (int k = 0; k < 3; ++k) {
      const int64_t t0 = now_ns();
      memcpy(static_cast<ResHost*>(dv)->units, zeros, sizeof zeros);
      _mm_sfence();
      best = std::min(best, now_ns() - t0);
    }
    ctx->res_bar_ns = best;
    if (best > kResBarMaxNs) {
      (void)hipFree(dv);
      if (ctx->res_land) (void)hipFree(ctx->res_land);
      dv = nullptr;
      ctx->res_land = nullptr;
    }
  }
  ctx->res_vram = dv != nullptr;
  ctx->res_host = static_cast<ResHost*>(dv ? dv : h);  // the ring the host posts into
  ctx->res_host_d = static_cast<ResHost*>(dv ? dv : hd);
  ctx->res_left_block = h;
  ctx->res_state = static_cast<uint32_t*>(st);
  ctx->res_published = 0;
  std::lock_guard<std::mutex> g(g_res_mu);
  g_res_ctxs.push_back(ctx);
  ctx->res_ring.store(true, std::memory_order_release);
  return TFS_SUCCESS;
}

// Workgroups for a throughput launch of ctx: its device's CUs minus those of
// the live resident kernels on that device (resident_live), in multiples of 8
// (one per XCD).
unsigned throughput_cap(const tfs_crc_ctx* ctx) {
  const unsigned cap = ctx->cus < kMaxGrid ? ctx->cus : kMaxGrid;
  if (!ctx->cu_reserve.load(std::memory_order_relaxed)) return cap;
  const int64_t now = now_ns();
  unsigned held = 0;
  {
    std::lock_guard<std::mutex> g(g_res_mu);
    for (const tfs_crc_ctx* c : g_res_ctxs)
      if (c->device == ctx->device && resident_live(c, now)) held += c->res_grid;
  }
  if (held == 0) return cap;
  const unsigned left = held + 8u < cap ? cap - held : 8u;
  return left & ~7u ? left & ~7u : 8u;
}

// Grid cap for a crc_files launch of n files (batches of at most kWgMaxFiles
// take the latency form, one workgroup per file: no cap to compute).
unsigned cap_for(const tfs_crc_ctx* ctx, uint32_t n) { return n <= kWgMaxFiles ? kMaxGrid : throughput_cap(ctx); }

// One launch on stream `st` with a scheduler slot leased for it (`sched` in
// LAUNCH); returns from the caller on failure.
#define SCHED_LAUNCH(ctx, st, what, LAUNCH)                                       \
  do {                                                                           \
    SchedLease lease_;                                                           \
    if (const int r_ = sched_acquire((ctx), (st), &lease_)) return r_;          \
    uint32_t* sched = lease_.slot;                                               \
    const hipError_t le_ = (LAUNCH);                                             \
    if (const int r2_ = sched_release((ctx), (st), lease_, le_, (what))) return r2_; \
  } while (0)

// Scheduler slot index of a lease.
uint32_t slot_index(const tfs_crc_ctx* ctx, const SchedLease& L) {
  return uint32_t((L.slot - ctx->d_sched) / (kSchedSlotBytes / 4u));
}

// The plan a lease uses: an owned slot's own, or ONE plan shared by every foreign
// slot (a plan per foreign slot let 64 caller-stream launches keep
// 64 plans -- ~7 GB at 1 M files -- alive per context).  A launch on the shared
// plan waits on its stream for the plan's previous user, which may be on any other
// stream (plan_done); the caller holds plan_mu[index] from here to the launch.
uint32_t plan_index(const SchedLease& L, uint32_t k) { return L.foreign >= 0 ? kOwnedSlots : k; }
int plan_order(tfs_crc_ctx* ctx, hipStream_t st, const SchedLease& L, uint32_t pk) {
  if (L.foreign >= 0 && ctx->plan_done[pk]) HIP_TRY(ctx, hipStreamWaitEvent(st, ctx->plan_done[pk], 0));
  return TFS_SUCCESS;
}

// (Caller holds plan_mu[k], right after a launch on st that reads plan k.)  Record
// plan_done[k] behind it.  When the event cannot be created or recorded, the
// next user of a shared plan would not wait for this launch, so the launch is
// drained here, under the lock, instead.
int plan_mark(tfs_crc_ctx* ctx, hipStream_t st, uint32_t k) {
  hipEvent_t& ev = ctx->plan_done[k];
  if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ev = nullptr;
  if (ev && hipEventRecord(ev, st) == hipSuccess) return TFS_SUCCESS;
  if (ev) (void)hipEventDestroy(ev);
  ev = nullptr;
  HIP_TRY(ctx, hipStreamSynchronize(st));
  return TFS_SUCCESS;
}

// (Caller holds plan_mu[k].)  Slot k's split plan for a throughput crc_files
// launch of n files on st (tfs_crc_device.h: one allocation, up to cap ext
// units).  The earlier launches using this plan are ordered before st's: they
// ran on st itself (owned slot) or were waited for when the slot was leased
// (foreign slot).  Growing frees the plan, so st is drained first.
int split_prepare(tfs_crc_ctx* ctx, hipStream_t st, uint32_t k, uint32_t n, SplitArgs* sa) {
  // room for max(2n, 65,536) segments (at most 4 M); the plan's capacity counts
  // every unit of the address-ordered list (files + segments)
  const uint32_t cap = uint32_t(std::min<uint64_t>(std::max<uint64_t>(2ull * n, 65536ull), kSplitMaxUnits));
  const uint32_t ucap = uint32_t(std::min<uint64_t>(uint64_t(n) + cap, 0xffffffffull));
  const uint64_t bytes = ao_bytes(n, ucap);
  DevBuf& plan = ctx->plans[k];
  if (bytes > plan.cap && plan.p) HIP_TRY(ctx, hipStreamSynchronize(st));
  HIP_TRY(ctx, plan.reserve(bytes));
  *sa = SplitArgs{static_cast<uint8_t*>(plan.p), ucap};
  return TFS_SUCCESS;
}

// A crc_files launch of n files on st (no completion flag): throughput launches
// (n > kWgMaxFiles) get a scheduler slot, that slot's split plan and the CU cap
// of their device; batches of at most kWgMaxFiles files take the latency form.
int files_launch(tfs_crc_ctx* ctx, hipStream_t st, int mode, const uint8_t* base, const Desc* desc, uint32_t n,
                 uint32_t* out_crc, uint8_t* out_ok, uint32_t* n_bad, uint32_t vseed, bool may_split = true) {
  SchedLease lease;
  if (const int r = sched_acquire(ctx, st, &lease)) return r;
  const uint32_t k = plan_index(lease, slot_index(ctx, lease));
  std::unique_lock<std::mutex> lk(ctx->plan_mu[k], std::defer_lock);
  SplitArgs sa{nullptr, 0u};
  const SplitArgs* split = nullptr;
  int rc = TFS_SUCCESS;
  if (may_split && n > kWgMaxFiles && ctx->split_files.load(std::memory_order_relaxed) != 0) {
    lk.lock();
    rc = plan_order(ctx, st, lease, k);
    if (rc == TFS_SUCCESS) rc = split_prepare(ctx, st, k, n, &sa);
    if (rc == TFS_SUCCESS) split = &sa;
  }
  const unsigned cap = cap_for(ctx, n);
  const hipError_t le = rc == TFS_SUCCESS ? launch_crc_files(mode, base, desc, n, ctx->d_tables, out_crc, out_ok, n_bad,
                                                             lease.slot, st, ctx->variant, vseed, nullptr, 0u, cap, split)
                                          : hipSuccess;
  if (split && le == hipSuccess) {
    rc = plan_mark(ctx, st, k);
    std::lock_guard<std::mutex> g(ctx->last_split_mu);
    ctx->last_split_slot = int(k);
    ctx->last_split_n = n;
    ctx->last_split_cap = sa.cap - n;  // segments the plan had room for
    ctx->last_split_grid = cap;  // a split launch takes the whole capped grid (launch_variant)
    ++ctx->split_launches;
  }
  const int r2 = sched_release(ctx, st, lease, le, "crc_files");
  return rc != TFS_SUCCESS ? rc : r2;
}

// Segment size of the segmented compaction (tfs_crc_device.h CSegArgs) for ctx:
// 1 KiB << lg, 0 = records stay whole.
// The product default (cseg_auto): whole records.  Round 4 first made 32 KiB segments
// the default for launches of at least 65,536 records; over seven boxes they averaged
// -0.4 % against whole records (+2.0 % to -1.7 %), while the hybrid record order the
// product now launches (kCompactHS) gained 1.4 % on average.
// Segments stay selectable per context (tfs_crc32_set_compact_segment).
uint32_t cseg_lg(const tfs_crc_ctx* ctx, uint32_t n) {
  (void)n;
  if (ctx->variant != 0) return 0u;  // the measurement variants: whole records
  if (ctx->cseg_auto.load(std::memory_order_relaxed)) return 0u;  // the default: whole records
  return ctx->cseg_lg.load(std::memory_order_relaxed);
}

// (Caller holds plan_mu[k].)  Slot k's segmented-compaction plan for n jobs on st
// (the same per-slot allocation and ordering rules as split_prepare).
int cseg_prepare(tfs_crc_ctx* ctx, hipStream_t st, uint32_t k, uint32_t n, uint32_t lg, CSegArgs* cs) {
  // room for 64 KiB records cut into segments, at least 64 K units, at most 16 M
  const uint64_t per = std::max<uint64_t>(1u, 65536u >> (10u + lg));
  const uint32_t cap = uint32_t(std::min<uint64_t>(std::max<uint64_t>(uint64_t(n) * per, 65536ull), 16ull << 20));
  const uint64_t bytes = cseg_bytes(n, cap);
  DevBuf& plan = ctx->plans[k];
  if (bytes > plan.cap && plan.p) HIP_TRY(ctx, hipStreamSynchronize(st));
  HIP_TRY(ctx, plan.reserve(bytes));
  HIP_TRY(ctx, hipMemsetAsync(plan.p, 0, 8u, st));  // `used`
  *cs = CSegArgs{static_cast<uint8_t*>(plan.p), cap, lg};
  return TFS_SUCCESS;
}

// (Caller holds ctx->mu.)  Launch the resident kernel unless one is running.
// Only one is ever in flight: a new one is launched only after the event behind
// the previous one has completed, i.e. every workgroup of it has left.
// `post`: called right after a post -- while the running launch's last
// workgroup has not signed out through ResHost::left it is taken as running with
// no HIP call (the host reads its own memory); a launch that ended in a fault is
// still found by wait_resident's periodic event query.
int resident_ensure_running(tfs_crc_ctx* ctx, bool post = false) {
  if (ctx->res_running && post &&
      __atomic_load_n(ctx->res_left, __ATOMIC_ACQUIRE) != ctx->res_gen.load(std::memory_order_relaxed))
    return TFS_SUCCESS;
  if (ctx->res_running) {
    const hipError_t e = hipEventQuery(ctx->res_event);
    if (e == hipErrorNotReady) return TFS_SUCCESS;
    if (e != hipSuccess) return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "resident kernel failed: %s", hipGetErrorString(e));
    ctx->res_running = false;
  }
  const uint32_t gen = uint32_t(ctx->res_launches + 1u);
  HIP_TRY(ctx, launch_resident(ctx->d_tables, ctx->res_host_d, ctx->res_left_d, ctx->res_state, ctx->res_grid,
                               ctx->res_idle_ticks, ctx->res_life_ticks, gen, ctx->res_stream, ctx->res_trace_dev));
  HIP_TRY(ctx, hipEventRecord(ctx->res_event, ctx->res_stream));
  ctx->res_running = true;
  ++ctx->res_launches;
  ctx->res_gen.store(gen, std::memory_order_release);
  return TFS_SUCCESS;
}

// (Caller holds ctx->mu.)  Post a zero-copy batch (device-visible base `zb`, the
// same bytes host-readable at `hb`) as units [P, P + n), one per file, each with
// its result word in s.h_res; then `published`; the kernel is (re)launched if
// gone.  A body of at most kResInline bytes is copied into its unit (the kernel
// reads no payload for it; `zb` may be null when every body is such).  Returns 1 (nothing posted) when the ring has no
// room: a unit of a batch still outstanding would be rewritten.
int resident_post(tfs_crc_ctx* ctx, Slot& s, int mode, const uint8_t* zb, const uint8_t* hb, const Desc* d,
                  uint32_t n) {
  if (const int rc = resident_setup(ctx)) return rc;
  ResHost* H = ctx->res_host;
  const uint32_t P = ctx->res_published;
  for (const Slot& x : ctx->sync_slots)
    if (&x != &s && x.busy && x.resident && int32_t(P + n - kResUnits - x.res_first) > 0) return 1;
  HIP_TRY(ctx, s.h_res.reserve(size_t(n) * 8));
  void* zres = s.h_res.dev;
  if (!zres) return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "resident result words are not mapped");
  // Bodies landed in device memory (ring in device memory, up to kResLandMax bytes)
  // and bodies in the unit are not read over PCIe.
  // (at most kResLandBatch landed per batch: a larger batch's bodies are read over PCIe)
  auto landable = [&](uint32_t len) { return ctx->res_land && len > kResInline && len <= kResLandMax; };
  uint64_t land_total = 0;
  for (uint32_t i = 0; i < n; ++i) land_total += landable(d[i].len) ? d[i].len : 0u;
  const bool land_ok = land_total <= kResLandBatch;
  auto landed = [&](uint32_t len) { return land_ok && landable(len); };
  uint64_t pcie_bytes = 0;  // what the kernel reads over PCIe for this batch
  for (uint32_t i = 0; i < n; ++i)
    if (d[i].len > kResInline && !landed(d[i].len)) {
      // (the caller's fast path passes no device-visible base: every body must then be
      // in the unit or landed -- enqueue_host_batch's rule, checked here too)
      if (!zb) return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "resident ring: a body to read over PCIe has no device address");
      pcie_bytes += d[i].len;
    }
  // Landed bodies go through the BAR first, then one store fence, so the device
  // memory holds them before any unit naming them leaves the write-combining buffers.
  bool any_landed = false;
  for (uint32_t i = 0; i < n; ++i)
    if (landed(d[i].len)) {
      memcpy(ctx->res_land + size_t((P + i) % kResUnits) * kResLandMax, hb + d[i].offset, d[i].len);
      any_landed = true;
    }
  if (any_landed) _mm_sfence();
  const uint32_t bulk = pcie_bytes > kResBulkBytes ? kResBulk : 0u;  // tfs_crc_device.h

  for (uint32_t i = 0; i < n; ++i) {
    // each part in one 16-byte store (never torn for the kernel's 16-byte read)
    ResUnit* u = &H->units[(P + i) % kResUnits];
    const uint32_t tag = P + i + 1u;
    uint64_t addr = 0;
    if (landed(d[i].len)) {  // copied into the unit's landing slot above
      addr = uint64_t(reinterpret_cast<uintptr_t>(ctx->res_land + size_t((P + i) % kResUnits) * kResLandMax));
    } else if (d[i].len > kResInline) {
      addr = uint64_t(reinterpret_cast<uintptr_t>(zb + d[i].offset));
    } else {  // the body travels in the unit
      alignas(16) uint32_t w[2 + 6 * 3] = {};
      memcpy(w, hb + d[i].offset, d[i].len);
      addr = uint64_t(w[0]) | uint64_t(w[1]) << 32;
      for (uint32_t k = 0; 8u + 12u * k < d[i].len; ++k)
        _mm_store_si128(reinterpret_cast<__m128i*>(u->body[k]),
                        _mm_set_epi32(int(tag), int(w[2 + 3 * k + 2]), int(w[2 + 3 * k + 1]), int(w[2 + 3 * k])));
    }
    const uint64_t out = uint64_t(reinterpret_cast<uintptr_t>(zres)) + 8u * i;
    _mm_store_si128(reinterpret_cast<__m128i*>(&u->addr),
                    _mm_set_epi32(int(tag), int(d[i].len | (d[i].len > kResInline ? bulk : 0u)),
                                  int(uint32_t(addr >> 32)), int(uint32_t(addr))));
    _mm_store_si128(reinterpret_cast<__m128i*>(&u->out),
                    _mm_set_epi32(int(tag), int(mode == 0 ? d[i].aux : 0u), int(uint32_t(out >> 32)),
                                  int(uint32_t(out))));
  }
  s.res_first = P;
  ctx->res_published = P + n;
  ctx->res_files += n;
  ctx->res_last_post_ns.store(now_ns(), std::memory_order_relaxed);
  if (ctx->res_vram) _mm_sfence();  // the units' write-combined stores leave before `published`
  __atomic_store_n(&H->published, uint64_t(ctx->res_published), __ATOMIC_RELEASE);
  if (ctx->res_vram) _mm_sfence();  // and `published` leaves now
  const int rc = resident_ensure_running(ctx, true);
  // A launch that fails leaves units published that no kernel may ever take (or
  // one taking them late, into result words since reused): the context stops
  // using the ring and launches from then on.
  if (rc) ctx->resident = false;
  return rc;
}

// Completion of a resident batch: spin until every file's result word carries
// its unit's tag; now and then check that the kernel is still there, and
// relaunch it (under mu) when it left with this batch outstanding (idle or
// lifetime exit racing the post).  Then the CRCs and verdicts go where
// finish_slot reads them (the expected CRCs are in s.h_desc).
// A workgroup takes its units in ring order, so units of other threads' batches
// ahead of ours (at most kResUnits / grid per workgroup) may take a relaunch each.
constexpr uint32_t kResMaxIdleRelaunches = 4u * kResUnits;

int wait_resident(tfs_crc_ctx* ctx, Slot& s, int mode, uint32_t n) {
  const volatile uint64_t* res = static_cast<const volatile uint64_t*>(s.h_res.p);
  // Every launch finishes at least one pending unit of each workgroup that has
  // one before it can leave, so relaunches without a new result of this batch
  // are bounded by the units queued ahead of it; past kResMaxIdleRelaunches in a
  // row the wait ends with a device error.
  uint32_t i = 0, relaunches = 0;
  for (uint32_t spins = 1;; ++spins) {
    const uint32_t i0 = i;
    while (i < n && uint32_t(res[i] >> 32) == s.res_first + i + 1u) ++i;  // {crc, unit tag}
    if (i == n) {
#ifdef TFS_CRC_MEASURE
      ctx->tr_seen.store(now_ns(), std::memory_order_relaxed);
#endif
      break;
    }
    if (i != i0) relaunches = 0;
    __builtin_ia32_pause();
    if ((spins & 255u) == 0) {
      // While the launch's last workgroup has not signed out it is running: no
      // HIP call (every closing thread spins here, and the runtime serialises
      // event queries: 38 ns alone, 2.3 us each from 8 threads at once,
      // tools/hipcall_cost.cpp); a faulted launch, which never signs out, is
      // still found by the query every 65,536 spins.
      if (__atomic_load_n(ctx->res_left, __ATOMIC_ACQUIRE) != ctx->res_gen.load(std::memory_order_acquire) &&
          (spins & 65535u) != 0)
        continue;
      const hipError_t e = hipEventQuery(ctx->res_event);
      if (e == hipErrorNotReady) continue;
      std::lock_guard<std::mutex> g(ctx->mu);
      const uint64_t before = ctx->res_launches;
      if (const int rc = resident_ensure_running(ctx)) {
        ctx->resident = false;  // as in resident_post
        return rc;
      }
      if (ctx->res_launches != before && ++relaunches > kResMaxIdleRelaunches) {
        ctx->resident = false;
        return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "resident kernel makes no progress (seq %u)", s.seq);
      }
    }
  }
  uint32_t* crc = static_cast<uint32_t*>(s.h_crc.p);
  uint8_t* ok = static_cast<uint8_t*>(s.h_ok.p);
  const Desc* d = static_cast<const Desc*>(s.h_desc.p);
  for (uint32_t k = 0; k < n; ++k) {
    crc[k] = uint32_t(res[k]);
    if (mode == 1) ok[k] = crc[k] == d[k].aux ? 1 : 0;
  }
  return TFS_SUCCESS;
}

// (Caller holds no lock.)  Stop the resident kernel and free its ring.
void resident_teardown(tfs_crc_ctx* ctx) {
  if (!ctx->res_host) return;
  {
    std::lock_guard<std::mutex> g(g_res_mu);
    g_res_ctxs.erase(std::remove(g_res_ctxs.begin(), g_res_ctxs.end(), ctx), g_res_ctxs.end());
    ctx->res_ring.store(false, std::memory_order_release);
  }
  __atomic_store_n(&ctx->res_host->published, uint64_t(ctx->res_published) | (uint64_t(1) << 32), __ATOMIC_RELEASE);
  _mm_sfence();
  if (ctx->res_stream) (void)hipStreamSynchronize(ctx->res_stream);
  if (ctx->res_event) (void)hipEventDestroy(ctx->res_event);
  if (ctx->res_stream) (void)hipStreamDestroy(ctx->res_stream);
  if (ctx->res_state) (void)hipFree(ctx->res_state);
  if (ctx->res_vram) (void)hipFree(ctx->res_host);
  if (ctx->res_land) (void)hipFree(ctx->res_land);
  ctx->res_land = nullptr;
  (void)hipHostFree(ctx->res_left_block);
  ctx->res_host = ctx->res_host_d = nullptr;
  ctx->res_left = ctx->res_left_d = nullptr;
  ctx->res_left_block = nullptr;
  ctx->res_vram = false;
  ctx->res_state = nullptr;
  ctx->res_stream = nullptr;
  ctx->res_event = nullptr;
}

// An armed tfs_crc32_inject_device_error: this submission fails as a device error would.
int injected_fault(tfs_crc_ctx* ctx) {
  if (ctx->inject_count.load() == 0) return TFS_SUCCESS;
  uint32_t k = ctx->inject_skip.load();
  while (k > 0)
    if (ctx->inject_skip.compare_exchange_weak(k, k - 1)) return TFS_SUCCESS;
  uint32_t c = ctx->inject_count.load();
  while (c > 0)
    if (ctx->inject_count.compare_exchange_weak(c, c - 1))
      return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "injected device error (tfs_crc32_inject_device_error)");
  return TFS_SUCCESS;
}

Slot* free_slot(tfs_crc_ctx* ctx) {
  for (auto& s : ctx->slots)
    if (!s.busy) return &s;
  return nullptr;
}

// Enqueue a host-memory batch on slot s (mode 0 compute, 1 verify).  Outputs
// land in the slot's pinned buffers when s.done fires (or, s.spin, when the
// completion flag reaches s.seq).  `job` >= 0: a synchronous slot whose small
// zero-copy batch may go to the resident kernel as that job slot.
int enqueue_host_batch(tfs_crc_ctx* ctx, Slot& s, int mode, const void* d, uint32_t n, const void* base,
                       uint64_t base_len, int job = -1) {
  s.resident = false;
  if (const int f = injected_fault(ctx)) return f;
  uint64_t lo = 0, hi = 0;
  const Desc* dd = static_cast<const Desc*>(d);
  if (!span_of(dd, n, base_len, &lo, &hi))
    return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "descriptor range exceeds base_len %llu",
                   (unsigned long long)base_len);
  HIP_TRY(ctx, s.h_crc.reserve(size_t(n) * 4));
  HIP_TRY(ctx, s.h_ok.reserve(n));
  HIP_TRY(ctx, s.h_bad.reserve(4));
  HIP_TRY(ctx, s.h_flag.reserve(64));
  if (!s.done) HIP_TRY(ctx, hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  s.spin = false;
  // A small batch (a CloseBatcher batch, one scalar Func::crc, one file read):
  // the kernel reads payloads and descriptors from page-locked memory and writes
  // its verdicts and a completion flag there -- one launch, no copies, and the
  // host spins on the flag instead of an event.  Pageable payloads are first
  // copied into the slot's page-locked staging buffer.  Such calls are bound by
  // latency, not bandwidth.
  // A few files far apart in one page-locked buffer (a CloseBatcher batch of
  // leases in a LeaseBufferPool) are read in place too: only their bytes cross
  // PCIe, however wide the span.
  // Bodies that all fit in their ring units (kResInline bytes or fewer: one
  // scalar Func::crc of a small RPC body, a packet header check): the host copies
  // them into the units from wherever they are -- no page-lock lookup, no staging
  // copy, and the kernel reads no payload.
  bool ring_full = false;
  if (job >= 0 && ctx->resident && ctx->variant == 0 && n <= kWgMaxFiles) {
    // (with the ring in device memory, bodies of up to kResLandMax bytes too: they
    // are copied into landing slots there)
    if (const int rc = resident_setup(ctx)) return rc;
    const uint32_t host_copied = ctx->res_land ? kResLandMax : kResInline;
    bool all_inline = true;
    uint64_t copied = 0;
    for (uint32_t i = 0; i < n && all_inline; ++i) {
      all_inline = dd[i].len <= host_copied;
      copied += dd[i].len;
    }
    if (all_inline && (!ctx->res_land || copied <= kResLandBatch)) {
      HIP_TRY(ctx, s.h_desc.reserve(size_t(n) * sizeof(Desc)));
      memcpy(s.h_desc.p, d, size_t(n) * sizeof(Desc));
      const int rc = resident_post(ctx, s, mode, nullptr, static_cast<const uint8_t*>(base), dd, n);
      if (rc < 0) return rc;
      if (rc == 0) {
        s.count_bad = true;
        s.spin = true;
        s.resident = true;
        return TFS_SUCCESS;
      }
      ++ctx->res_ring_full;  // no room in the ring: the paths below launch it
      ring_full = true;
    }
  }
  const bool wide = hi - lo > kZeroCopySpan;
  const bool pinned = ctx->variant != kVariantDmaCompact && (!wide || n <= kWgMaxFiles) && is_pinned_host(base);
  uint64_t wide_bytes = 0;
  if (wide && pinned)
    for (uint32_t i = 0; i < n; ++i) wide_bytes += dd[i].len;
  if (ctx->variant != kVariantDmaCompact && (!wide || (pinned && wide_bytes <= kZeroCopySpan))) {
    void* host_span = nullptr;  // page-locked host address of base + lo
    if (pinned) {
      host_span = const_cast<uint8_t*>(static_cast<const uint8_t*>(base) + lo);
    } else {
      (void)hipGetLastError();
      HIP_TRY(ctx, s.h_data.reserve(hi - lo + 16));
      if (hi > lo) memcpy(s.h_data.p, static_cast<const uint8_t*>(base) + lo, hi - lo);
      host_span = s.h_data.p;
    }
    HIP_TRY(ctx, s.h_desc.reserve(size_t(n) * sizeof(Desc)));
    memcpy(s.h_desc.p, d, size_t(n) * sizeof(Desc));
    void *zb = nullptr, *zd = s.h_desc.dev, *zcrc = s.h_crc.dev, *zok = s.h_ok.dev, *zflag = s.h_flag.dev;
    if (host_span == s.h_data.p) zb = s.h_data.dev;
    else if (!host_dev_ptr(host_span, &zb)) zb = nullptr;
    if (zb && zd && zcrc && zok && zflag) {
      s.seq = g_flag_seq.fetch_add(1) + 1u;
      if (s.seq == 0) s.seq = g_flag_seq.fetch_add(1) + 1u;  // 0 is the words' initial value
      if (job >= 0 && ctx->resident && ctx->variant == 0 && n <= kWgMaxFiles && !ring_full) {
        const int rc = resident_post(ctx, s, mode, static_cast<const uint8_t*>(zb) - lo,
                                     static_cast<const uint8_t*>(host_span) - lo, static_cast<const Desc*>(d), n);
        if (rc < 0) return rc;
        if (rc == 0) {
          s.count_bad = true;
          s.spin = true;
          s.resident = true;
          return TFS_SUCCESS;
        }
        ++ctx->res_ring_full;  // no room in the ring: launch this batch
      }
      // n_bad is counted from the verdicts on the host (no atomics on host memory)
      SCHED_LAUNCH(ctx, ctx->lat_stream, "crc_files",
                   launch_crc_files(mode, static_cast<const uint8_t*>(zb) - lo, static_cast<const Desc*>(zd), n,
                                    ctx->d_tables, static_cast<uint32_t*>(zcrc), static_cast<uint8_t*>(zok), nullptr,
                                    sched, ctx->lat_stream, ctx->variant, 0u, static_cast<uint32_t*>(zflag), s.seq,
                                    cap_for(ctx, n), nullptr));
      HIP_TRY(ctx, hipEventRecord(s.done, ctx->lat_stream));
      s.count_bad = true;
      s.spin = true;
      return TFS_SUCCESS;
    }
    (void)hipGetLastError();  // not mappable: stage it
  }
  // No file over kSplitMin (a block image of 64 KiB files): no split plan, so no
  // plan kernels ahead of the CRC launch (their descriptors are on the host here).
  uint32_t max_len = 0;
  for (uint32_t i = 0; i < n; ++i) max_len = std::max(max_len, dd[i].len);
  const bool may_split = max_len > kSplitMin;
  s.count_bad = false;
  // On the context stream.  (A stream per slot, so that one block's launch overlaps
  // the next block's copy, measured 0.8 % faster on one box but halved the
  // context stream's copies on another -- 30 against 57 GB/s)
  hipStream_t st = ctx->stream;
  // A wide page-locked batch (a 64 MiB block image read back for verify, configs[4]'s
  // end-to-end leg): the throughput kernel reads the files in place over PCIe, its
  // descriptors from the slot's page-locked words, and writes its verdicts there --
  // one launch per batch, no copy-engine work at all.  A zero-copy read of a whole
  // block image runs at the link's DMA rate (58.1 against 57.5 GB/s).
  // Measurement build: TFS_CRC_VARIANT=52 stages it as before (A/B).
  if (wide && n <= kZeroCopyOutFiles && ctx->variant != kVariantDmaCompact && ctx->variant != kVariantStagedWide &&
      is_pinned_host(base)) {
    void* zb = nullptr;
    HIP_TRY(ctx, s.h_desc.reserve(size_t(n) * sizeof(Desc)));
    if (host_dev_ptr(static_cast<const uint8_t*>(base) + lo, &zb) && s.h_desc.dev && s.h_crc.dev && s.h_ok.dev) {
      memcpy(s.h_desc.p, d, size_t(n) * sizeof(Desc));
      s.count_bad = true;
      // A synchronous call launches on its slot's own stream, so the launches of
      // concurrent calls overlap: the next batch's waves fill the link while the
      // last waves of the previous one drain (round 6, DESIGN.md section 5.5:
      // configs[2]'s receive-buffer leg 0.934 -> 0.965 of H2D).  Async submissions
      // stay on the context stream in submission order (the same A/B on configs[4]'s
      // block images: 0.964 / 0.965 on slot streams against 0.973 / 0.926).
      hipStream_t wst = st;
      if (job >= 0 && ctx->variant != kVariantWideCtxStream) {
        if (!s.wide_stream) {
          HIP_TRY(ctx, hipStreamCreateWithFlags(&s.wide_stream, hipStreamNonBlocking));
          if (bind_owned_stream(ctx, s.wide_stream) != hipSuccess) {
            (void)hipStreamDestroy(s.wide_stream);
            s.wide_stream = nullptr;
          }
        }
        if (s.wide_stream) wst = s.wide_stream;
      }
      if (const int rc2 = files_launch(ctx, wst, mode, static_cast<const uint8_t*>(zb) - lo,
                                       static_cast<const Desc*>(s.h_desc.dev), n, static_cast<uint32_t*>(s.h_crc.dev),
                                       static_cast<uint8_t*>(s.h_ok.dev), nullptr, 0u, may_split))
        return rc2;
      HIP_TRY(ctx, hipEventRecord(s.done, wst));
      return TFS_SUCCESS;
    }
    (void)hipGetLastError();
  }
  const uint8_t* d_base = nullptr;
  int rc = stage_span(ctx, s, base, lo, hi, &d_base, st);
  if (rc) return rc;
  HIP_TRY(ctx, s.d_desc.reserve(size_t(n) * sizeof(Desc)));
  HIP_TRY(ctx, hipMemcpyAsync(s.d_desc.p, d, size_t(n) * sizeof(Desc), hipMemcpyHostToDevice, st));
  // Up to kZeroCopyOutFiles files the kernel writes its CRCs and verdicts straight
  // into the slot's page-locked words (n_bad is counted from them on the host):
  // three D2H copies and a memset less on the stream, ~10 us of DMA set-up each,
  // behind every staged block (a 64 MiB block image: a 1.2 ms copy).
  void* zcrc = s.h_crc.dev;
  void* zok = s.h_ok.dev;
  if (n <= kZeroCopyOutFiles && zcrc && zok) {
    s.count_bad = true;
    if (const int rc2 = files_launch(ctx, st, mode, d_base, static_cast<const Desc*>(s.d_desc.p), n,
                                     static_cast<uint32_t*>(zcrc), static_cast<uint8_t*>(zok), nullptr, 0u, may_split))
      return rc2;
    HIP_TRY(ctx, hipEventRecord(s.done, st));
    return TFS_SUCCESS;
  }
  HIP_TRY(ctx, s.d_crc.reserve(size_t(n) * 4));
  HIP_TRY(ctx, s.d_ok.reserve(n));
  HIP_TRY(ctx, s.d_bad.reserve(4));
  HIP_TRY(ctx, hipMemsetAsync(s.d_bad.p, 0, 4, st));
  if (const int rc2 = files_launch(ctx, st, mode, d_base, static_cast<const Desc*>(s.d_desc.p), n,
                                   static_cast<uint32_t*>(s.d_crc.p), static_cast<uint8_t*>(s.d_ok.p),
                                   static_cast<uint32_t*>(s.d_bad.p), 0u, may_split))
    return rc2;
  HIP_TRY(ctx, hipMemcpyAsync(s.h_crc.p, s.d_crc.p, size_t(n) * 4, hipMemcpyDeviceToHost, st));
  if (mode == 1) {
    HIP_TRY(ctx, hipMemcpyAsync(s.h_ok.p, s.d_ok.p, n, hipMemcpyDeviceToHost, st));
    HIP_TRY(ctx, hipMemcpyAsync(s.h_bad.p, s.d_bad.p, 4, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(ctx, hipEventRecord(s.done, st));
  return TFS_SUCCESS;
}

int finish_slot(tfs_crc_ctx* ctx, Slot& s, int mode, uint32_t n, uint32_t* out_crc, uint8_t* out_ok,
                uint32_t* n_bad) {
  if (s.spin) {
    const int rc = s.resident ? wait_resident(ctx, s, mode, n) : wait_flag(ctx, s);
    if (rc) return rc;
  } else {
    HIP_TRY(ctx, hipEventSynchronize(s.done));
  }
  if (out_crc && n) memcpy(out_crc, s.h_crc.p, size_t(n) * 4);
  if (mode == 1 && s.count_bad) {
    const uint8_t* ok = static_cast<const uint8_t*>(s.h_ok.p);
    uint32_t bad = 0;
    for (uint32_t i = 0; i < n; ++i) bad += ok[i] ? 0u : 1u;
    *static_cast<uint32_t*>(s.h_bad.p) = bad;
  }
  if (mode == 1) {
    if (out_ok && n) memcpy(out_ok, s.h_ok.p, n);
    const uint32_t bad = n ? *static_cast<uint32_t*>(s.h_bad.p) : 0u;
    if (n_bad) *n_bad = bad;
    return bad ? TFS_EXIT_CHECK_CRC_ERROR : TFS_SUCCESS;
  }
  return TFS_SUCCESS;
}

std::once_flag g_default_once;
tfs_crc_ctx* g_default = nullptr;
int g_default_rc = TFS_CRC_EXIT_NO_DEVICE;
std::string g_default_err = "default context not created";

tfs_crc_ctx* default_ctx(int* rc) {
  std::call_once(g_default_once, [] {
    tfs_crc_ctx* c = nullptr;
    g_default_rc = tfs_crc32_ctx_create(0, &c);
    if (g_default_rc == TFS_SUCCESS) g_default = c;
    else g_default_err = c ? c->last_error : "tfs_crc32_ctx_create(0) failed";
  });
  if (rc) *rc = g_default_rc;
  return g_default;
}

// The scalar drop-in's context: the calling thread's binding
// (tfs_crc32_bind_thread), else the process default the caller chose
// (tfs_crc32_set_default_ctx), else a context on device 0 created on first use.
thread_local tfs_crc_ctx* t_scalar_ctx = nullptr;
std::atomic<tfs_crc_ctx*> g_scalar_ctx{nullptr};

// Live contexts and their ids: a thread binding names its context by
// pointer and id, so a binding to a destroyed context is dropped on the thread's
// next scalar call instead of being used, even if a new context reuses the
// address.  The registry is consulted only after some context was destroyed
// since the binding was last checked (one relaxed load on the common path).
std::mutex g_live_mu;
std::map<const tfs_crc_ctx*, uint64_t> g_live;
std::atomic<uint64_t> g_ctx_ids{0}, g_destroy_epoch{0};
thread_local uint64_t t_scalar_id = 0, t_scalar_epoch = 0;

void live_add(const tfs_crc_ctx* c, uint64_t id) {
  std::lock_guard<std::mutex> g(g_live_mu);
  g_live[c] = id;
}

void live_remove(const tfs_crc_ctx* c) {
  std::lock_guard<std::mutex> g(g_live_mu);
  g_live.erase(c);
  g_destroy_epoch.fetch_add(1, std::memory_order_release);
}

uint64_t live_id(const tfs_crc_ctx* c) {
  std::lock_guard<std::mutex> g(g_live_mu);
  auto it = g_live.find(c);
  return it == g_live.end() ? 0 : it->second;
}

tfs_crc_ctx* scalar_ctx(int* rc) {
  if (rc) *rc = TFS_SUCCESS;
  if (t_scalar_ctx) {
    const uint64_t e = g_destroy_epoch.load(std::memory_order_acquire);
    if (e != t_scalar_epoch) {
      if (live_id(t_scalar_ctx) != t_scalar_id) t_scalar_ctx = nullptr;  // destroyed since it was bound
      t_scalar_epoch = e;
    }
    if (t_scalar_ctx) return t_scalar_ctx;
  }
  if (tfs_crc_ctx* c = g_scalar_ctx.load(std::memory_order_acquire)) return c;
  return default_ctx(rc);
}

// Failures of the scalar drop-in (Func::crc has no error channel): counted for
// the whole process and reported on stderr once, so a device fault never passes
// as a plain CRC mismatch unseen (tfs_crc32_error_count).
std::atomic<uint64_t> g_scalar_errors{0};
std::atomic<bool> g_scalar_logged{false};

void scalar_failed(tfs_crc_ctx* ctx, int rc) {
  g_scalar_errors.fetch_add(1, std::memory_order_relaxed);
  if (!g_scalar_logged.exchange(true))
    fprintf(stderr,
            "tfs_crc32: the scalar Func::crc drop-in failed (%d: %s) and returned its seed; callers that can act on "
            "an error use tfs_crc32_e (tfs_crc32_error_count counts every such failure; reported once)\n",
            rc, ctx ? ctx->last_error : g_default_err.c_str());
}

}  // namespace

extern "C" {

int tfs_crc32_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

int tfs_crc32_ctx_create(int device, tfs_crc_ctx** out) {
  if (!out) return TFS_EXIT_PARAMETER_ERROR;
  *out = nullptr;
  int ndev = tfs_crc32_device_count();
  if (ndev <= 0) return TFS_CRC_EXIT_NO_DEVICE;
  if (device < 0 || device >= ndev) return TFS_EXIT_PARAMETER_ERROR;
  auto* ctx = new tfs_crc_ctx();
  ctx->device = device;
  ctx->id = g_ctx_ids.fetch_add(1, std::memory_order_relaxed) + 1;
  live_add(ctx, ctx->id);
#ifdef TFS_CRC_MEASURE
  if (const char* v = getenv("TFS_CRC_VARIANT")) ctx->variant = atoi(v);
  // measurement: the synchronous slots stage pageable bytes in fine-grained
  // (coherent) page-locked memory instead of the default (tools/floor_probe.cpp)
  if (const char* v = getenv("TFS_CRC_STAGE_COHERENT"))
    if (atoi(v))
      for (Slot& x : ctx->sync_slots) x.h_data.coherent = true;
#endif
  if (const char* v = getenv("TFS_CRC_COMPACT_SLOTS")) ctx->compact_slots = std::min(std::max(atoi(v), 1), kCompactSlots);
  if (const char* v = getenv("TFS_CRC_COMPACT_GROUP")) ctx->compact_group = uint32_t(std::min(std::max(atoi(v), 1), 256));
  if (const char* v = getenv("TFS_CRC_RESIDENT")) ctx->resident = atoi(v) != 0;
  if (const char* v = getenv("TFS_CRC_RESIDENT_VRAM")) ctx->res_vram_want = atoi(v) != 0;
  if (const char* v = getenv("TFS_CRC_RESIDENT_WGS")) ctx->res_grid = unsigned(std::min(std::max(atoi(v), 1), 256));
  if (const char* v = getenv("TFS_CRC_RESIDENT_IDLE_US")) ctx->res_idle_us = uint32_t(std::min(std::max(atoi(v), 1), 1000000));
  if (const char* v = getenv("TFS_CRC_RESIDENT_LIFE_US")) ctx->res_life_us = uint32_t(std::min(std::max(atoi(v), 1), 10000000));
  int rc = TFS_SUCCESS;
  do {
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) { rc = set_err(ctx, TFS_CRC_EXIT_NO_DEVICE, "hipSetDevice(%d): %s", device, hipGetErrorString(e)); break; }
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) { rc = set_err(ctx, TFS_CRC_EXIT_NO_DEVICE, "hipGetDeviceProperties: %s", hipGetErrorString(e)); break; }
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
      rc = set_err(ctx, TFS_CRC_EXIT_NO_DEVICE, "device %d is %s; kernels are built for gfx950 only", device, prop.gcnArchName);
      break;
    }
    if (prop.multiProcessorCount > 0) ctx->cus = unsigned(prop.multiProcessorCount);
    e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { rc = set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "hipStreamCreate: %s", hipGetErrorString(e)); break; }
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess) ctx->lat_prio = greatest;
    else (void)hipGetLastError();
    e = hipStreamCreateWithPriority(&ctx->lat_stream, hipStreamNonBlocking, ctx->lat_prio);
    if (e != hipSuccess) { rc = set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "hipStreamCreateWithPriority: %s", hipGetErrorString(e)); break; }
    std::vector<Tables> host(1);
    build_tables(host.data());
    e = hipMalloc(reinterpret_cast<void**>(&ctx->d_tables), sizeof(Tables));
    if (e != hipSuccess) { rc = set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "hipMalloc(tables): %s", hipGetErrorString(e)); break; }
    // The tables and the zeroed scheduler slots are written on the context's
    // stream and waited for: the kernels run on non-blocking streams, which do
    // not wait for work on the null stream, and a recycled allocation may still
    // hold another context's counters.
    e = hipMemcpyAsync(ctx->d_tables, host.data(), sizeof(Tables), hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) { rc = set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "hipMemcpy(tables): %s", hipGetErrorString(e)); break; }
    e = hipMalloc(reinterpret_cast<void**>(&ctx->d_sched), size_t(kSchedSlots) * kSchedSlotBytes);
    if (e != hipSuccess) { rc = set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "hipMalloc(sched): %s", hipGetErrorString(e)); break; }
    e = hipMemsetAsync(ctx->d_sched, 0, size_t(kSchedSlots) * kSchedSlotBytes, ctx->stream);  // then kept zero by the kernels
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) { rc = set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "hipMemset(sched): %s", hipGetErrorString(e)); break; }
    ctx->sched_streams.push_back(ctx->stream);
    ctx->sched_streams.push_back(ctx->lat_stream);
  } while (0);
  *out = ctx;  // returned even on failure so the caller can read last_error; destroy it
  return rc;
}

int tfs_crc32_ctx_destroy(tfs_crc_ctx* ctx) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  {
    tfs_crc_ctx* expect = ctx;  // no longer the scalar default; other threads' bindings drop it on next use
    g_scalar_ctx.compare_exchange_strong(expect, nullptr);
    if (t_scalar_ctx == ctx) t_scalar_ctx = nullptr;
    live_remove(ctx);
  }
  if (ctx->device >= 0) (void)hipSetDevice(ctx->device);
  resident_teardown(ctx);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->lat_stream) (void)hipStreamSynchronize(ctx->lat_stream);
  for (auto& s : ctx->slots) {
    if (s.wide_stream) (void)hipStreamSynchronize(s.wide_stream);
    s.release();
  }
  for (auto& s : ctx->sync_slots) {
    if (s.wide_stream) (void)hipStreamSynchronize(s.wide_stream);
    s.release();
  }
  for (auto& cs : ctx->cslots) {
    if (cs.stream) (void)hipStreamSynchronize(cs.stream);
    cs.release();
  }
  for (hipEvent_t& ev : ctx->foreign_done) {
    if (ev) (void)hipEventSynchronize(ev);
    if (ev) (void)hipEventDestroy(ev);
    ev = nullptr;
  }
  ctx->packet_scratch.release();
  for (uint32_t k = 0; k < kSchedSlots; ++k) {  // split launches on any stream, callers' included
    if (ctx->plan_done[k]) {
      (void)hipEventSynchronize(ctx->plan_done[k]);
      (void)hipEventDestroy(ctx->plan_done[k]);
    }
    ctx->plans[k].release();
  }
  if (ctx->d_tables) (void)hipFree(ctx->d_tables);
  if (ctx->d_sched) (void)hipFree(ctx->d_sched);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->lat_stream) (void)hipStreamDestroy(ctx->lat_stream);
  delete ctx;
  return TFS_SUCCESS;
}

const char* tfs_crc32_last_error(const tfs_crc_ctx* ctx) {
  if (!ctx) {
    if (t_scalar_ctx && live_id(t_scalar_ctx) == t_scalar_id) return t_scalar_ctx->last_error;
    if (const tfs_crc_ctx* c = g_scalar_ctx.load()) return c->last_error;
    if (g_default) return g_default->last_error;
    return g_default_err.c_str();
  }
  return ctx->last_error;
}

uint64_t tfs_crc32_error_count(void) { return g_scalar_errors.load(); }

int tfs_crc32_set_default_ctx(tfs_crc_ctx* ctx) {
  g_scalar_ctx.store(ctx, std::memory_order_release);
  return TFS_SUCCESS;
}

int tfs_crc32_bind_thread(tfs_crc_ctx* ctx) {
  const uint64_t id = ctx ? live_id(ctx) : 0;
  if (ctx && id == 0) return TFS_EXIT_PARAMETER_ERROR;  // not a live context
  t_scalar_ctx = ctx;
  t_scalar_id = id;
  t_scalar_epoch = g_destroy_epoch.load(std::memory_order_acquire);
  return TFS_SUCCESS;
}

tfs_crc_ctx* tfs_crc32_default_ctx(void) { return scalar_ctx(nullptr); }

namespace {

// tfs_crc32_stats: every synchronous host call, and the lone ones under the crossover.
void count_host_call(tfs_crc_ctx* ctx, const Desc* d, uint32_t n) {
  ctx->st_calls.fetch_add(1, std::memory_order_relaxed);
  ctx->st_files.fetch_add(n, std::memory_order_relaxed);
  if (n != 1) return;
  ctx->st_lone.fetch_add(1, std::memory_order_relaxed);
  if (d[0].len < TFS_CRC_LONE_CROSSOVER) {
    ctx->st_lone_small.fetch_add(1, std::memory_order_relaxed);
    ctx->st_lone_small_bytes.fetch_add(d[0].len, std::memory_order_relaxed);
  }
}

// A synchronous host call: its slot is taken and its launch queued under
// ctx->mu, and the wait for the result (the completion-flag spin of a
// zero-copy batch) runs outside it, so calls from several threads -- the
// close path's batches -- overlap their round trips; their kernels queue back
// to back on the ctx stream.
int sync_host_call(tfs_crc_ctx* ctx, int mode, const void* d, uint32_t n, const void* base, uint64_t base_len,
                   uint32_t* out_crc, uint8_t* out_ok, uint32_t* n_bad) {
  count_host_call(ctx, static_cast<const Desc*>(d), n);
#ifdef TFS_CRC_MEASURE
  ctx->tr_enter.store(now_ns(), std::memory_order_relaxed);
#endif
  Slot* s = nullptr;
  {
    std::unique_lock<std::mutex> lk(ctx->mu);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    for (;;) {
      for (Slot& x : ctx->sync_slots)
        if (!x.busy) {
          s = &x;
          break;
        }
      if (s) break;
      ctx->sync_cv.wait(lk);
    }
    s->busy = true;
    const int rc = enqueue_host_batch(ctx, *s, mode, d, n, base, base_len, int(s - ctx->sync_slots));
    if (rc) {
      s->busy = false;
      ctx->sync_cv.notify_one();
      return rc;
    }
#ifdef TFS_CRC_MEASURE
    ctx->tr_posted.store(now_ns(), std::memory_order_relaxed);
    ctx->tr_first.store(s->res_first, std::memory_order_relaxed);
    ctx->tr_resident.store(s->resident ? 1u : 0u, std::memory_order_relaxed);
#endif
  }
  const int rc = finish_slot(ctx, *s, mode, n, out_crc, out_ok, n_bad);
#ifdef TFS_CRC_MEASURE
  ctx->tr_done.store(now_ns(), std::memory_order_relaxed);
#endif
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    s->busy = false;
  }
  ctx->sync_cv.notify_one();
  return rc;
}

}  // namespace

int tfs_crc32_batch(tfs_crc_ctx* ctx, const tfs_crc_desc* d, uint32_t n, const void* base, uint64_t base_len,
                    uint32_t* out_crc) {
  if (!ctx || (n && (!d || !out_crc || !base))) return TFS_EXIT_PARAMETER_ERROR;
  if (n == 0) return TFS_SUCCESS;
  return sync_host_call(ctx, 0, d, n, base, base_len, out_crc, nullptr, nullptr);
}

int tfs_crc32_verify(tfs_crc_ctx* ctx, const tfs_crc_vdesc* d, uint32_t n, const void* base, uint64_t base_len,
                     uint32_t* out_crc, uint8_t* out_ok, uint32_t* n_bad) {
  if (!ctx || (n && (!d || !base))) return TFS_EXIT_PARAMETER_ERROR;
  if (n == 0) {
    if (n_bad) *n_bad = 0;
    return TFS_SUCCESS;
  }
  return sync_host_call(ctx, 1, d, n, base, base_len, out_crc, out_ok, n_bad);
}

int tfs_crc32_submit_verify(tfs_crc_ctx* ctx, const tfs_crc_vdesc* d, uint32_t n, const void* base,
                            uint64_t base_len, uint32_t* out_crc, uint8_t* out_ok, uint32_t* n_bad,
                            tfs_crc_ticket* ticket) {
  if (!ctx || !ticket || (n && (!d || !base))) return TFS_EXIT_PARAMETER_ERROR;
  std::lock_guard<std::mutex> g(ctx->mu);
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  Slot* s = free_slot(ctx);
  if (!s) return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "all %d slots busy; wait on a ticket first", kSlots);
  if (n) {
    int rc = enqueue_host_batch(ctx, *s, 1, d, n, base, base_len);
    if (rc) return rc;
  } else {
    if (!s->done) HIP_TRY(ctx, hipEventCreateWithFlags(&s->done, hipEventDisableTiming));
    HIP_TRY(ctx, hipEventRecord(s->done, ctx->stream));
  }
  s->busy = true;
  s->ticket = ctx->next_ticket++;
  s->n = n;
  s->out_crc = out_crc;
  s->out_ok = out_ok;
  s->n_bad = n_bad;
  ticket->id = s->ticket;
  return TFS_SUCCESS;
}

int tfs_crc32_wait(tfs_crc_ctx* ctx, tfs_crc_ticket ticket) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  std::lock_guard<std::mutex> g(ctx->mu);
  for (auto& s : ctx->slots) {
    if (s.busy && s.ticket == ticket.id) {
      HIP_TRY(ctx, hipSetDevice(ctx->device));
      int rc = finish_slot(ctx, s, 1, s.n, s.out_crc, s.out_ok, s.n_bad);
      s.busy = false;
      return rc;
    }
  }
  return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "unknown ticket %llu", (unsigned long long)ticket.id);
}

int tfs_crc32_batch_device(tfs_crc_ctx* ctx, const tfs_crc_desc* d_desc, uint32_t n, const void* d_base,
                           uint32_t* d_out_crc, void* stream) {
  if (!ctx || (n && (!d_desc || !d_base || !d_out_crc))) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  return files_launch(ctx, st, 0, static_cast<const uint8_t*>(d_base), reinterpret_cast<const Desc*>(d_desc), n,
                      d_out_crc, nullptr, nullptr, 0u);
}

int tfs_crc32_verify_device(tfs_crc_ctx* ctx, const tfs_crc_vdesc* d_desc, uint32_t n, const void* d_base,
                            uint32_t* d_out_crc, uint8_t* d_out_ok, uint32_t* d_n_bad, void* stream) {
  if (!ctx || (n && (!d_desc || !d_base))) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  return files_launch(ctx, st, 1, static_cast<const uint8_t*>(d_base), reinterpret_cast<const Desc*>(d_desc), n,
                      d_out_crc, d_out_ok, d_n_bad, 0u);
}

uint32_t tfs_crc32_e(uint32_t crc, const char* data, int32_t len, int* err) {
  if (err) *err = TFS_SUCCESS;
  if (len <= 0) return crc;  // func.cpp:429: the loop does not run
  if (!data) {
    if (err) *err = TFS_EXIT_PARAMETER_ERROR;
    return crc;
  }
  int rc = 0;
  tfs_crc_ctx* ctx = scalar_ctx(&rc);
  if (!ctx) {
    scalar_failed(nullptr, rc);
    if (err) *err = rc;
    return crc;
  }
  tfs_crc_desc d{0, uint32_t(len), crc};
  uint32_t out = crc;
  rc = tfs_crc32_batch(ctx, &d, 1, data, uint64_t(len), &out);
  if (rc) {
    scalar_failed(ctx, rc);
    if (err) *err = rc;
    return crc;
  }
  return out;
}

uint32_t tfs_crc32(uint32_t crc, const char* data, int32_t len) { return tfs_crc32_e(crc, data, len, nullptr); }

int tfs_datafile_get_crc(tfs_crc_ctx* ctx, const char* data, int32_t length, uint32_t* out_crc) {
  if (!out_crc) return TFS_EXIT_PARAMETER_ERROR;
  if (length <= 0) {
    *out_crc = 0;
    return TFS_SUCCESS;
  }
  if (!ctx) {
    int rc = 0;
    ctx = scalar_ctx(&rc);
    if (!ctx) return rc;
  }
  tfs_crc_desc d{0, uint32_t(length), 0u};
  return tfs_crc32_batch(ctx, &d, 1, data, uint64_t(length), out_crc);
}

int tfs_block_verify_device(tfs_crc_ctx* ctx, const void* d_image, uint64_t image_len, const tfs_raw_meta* d_metas,
                            uint32_t n, uint32_t* d_out_crc, int32_t* d_out_status, uint32_t* d_n_bad, void* stream) {
  if (!ctx || (n && (!d_image || !d_metas))) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  SCHED_LAUNCH(ctx, st, "block_verify_pipe", launch_block_verify_pipe(static_cast<const uint8_t*>(d_image), image_len,
                                        reinterpret_cast<const RawMeta*>(d_metas), nullptr, n, ctx->d_tables, d_out_crc,
                                        d_out_status, d_n_bad, sched, st, ctx->variant, throughput_cap(ctx)));
  return TFS_SUCCESS;
}

int tfs_blocks_verify_device(tfs_crc_ctx* ctx, const void* d_src, uint64_t src_len, const tfs_compact_job* d_jobs,
                             uint32_t n, uint32_t* d_out_crc, int32_t* d_out_status, uint32_t* d_n_bad, void* stream) {
  if (!ctx || (n && (!d_src || !d_jobs))) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  SCHED_LAUNCH(ctx, st, "block_verify_pipe", launch_block_verify_pipe(static_cast<const uint8_t*>(d_src), src_len, nullptr,
                                        reinterpret_cast<const CompactJob*>(d_jobs), n, ctx->d_tables, d_out_crc,
                                        d_out_status, d_n_bad, sched, st, ctx->variant, throughput_cap(ctx)));
  return TFS_SUCCESS;
}

namespace {
// (Caller holds ctx->mu.)  Launch the in-place verify of a page-locked image's
// records on synchronous slot s's own stream, metas / CRCs / statuses in the
// slot's page-locked words; s->done is recorded behind it.
int block_verify_inplace_enqueue(tfs_crc_ctx* ctx, Slot* s, const uint8_t* d_base, uint64_t image_len,
                                 const tfs_raw_meta* metas, uint32_t n) {
  HIP_TRY(ctx, s->h_desc.reserve(size_t(n) * sizeof(RawMeta)));
  HIP_TRY(ctx, s->h_crc.reserve(size_t(n) * 4));
  HIP_TRY(ctx, s->h_ok.reserve(size_t(n) * 4));
  if (!s->h_desc.dev || !s->h_crc.dev || !s->h_ok.dev)
    return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "block_verify: page-locked words not mapped");
  if (!s->wide_stream) {
    HIP_TRY(ctx, hipStreamCreateWithFlags(&s->wide_stream, hipStreamNonBlocking));
    if (bind_owned_stream(ctx, s->wide_stream) != hipSuccess) {
      (void)hipStreamDestroy(s->wide_stream);
      s->wide_stream = nullptr;
      return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "block_verify: no scheduler slot for a stream");
    }
  }
  if (!s->done) HIP_TRY(ctx, hipEventCreateWithFlags(&s->done, hipEventDisableTiming));
  memcpy(s->h_desc.p, metas, size_t(n) * sizeof(RawMeta));
  hipStream_t st = s->wide_stream;
  SCHED_LAUNCH(ctx, st, "block_verify_pipe",
               launch_block_verify_pipe(d_base, image_len, static_cast<const RawMeta*>(s->h_desc.dev), nullptr, n,
                                        ctx->d_tables, static_cast<uint32_t*>(s->h_crc.dev),
                                        static_cast<int32_t*>(s->h_ok.dev), nullptr, sched, st, ctx->variant,
                                        throughput_cap(ctx)));
  HIP_TRY(ctx, hipEventRecord(s->done, st));
  return TFS_SUCCESS;
}
}  // namespace

int tfs_block_verify(tfs_crc_ctx* ctx, const void* image, uint64_t image_len, const tfs_raw_meta* metas, uint32_t n,
                     uint32_t* out_crc, int32_t* out_status, uint32_t* n_bad) {
  if (!ctx || (n && (!image || !metas))) return TFS_EXIT_PARAMETER_ERROR;
  if (n == 0) {
    if (n_bad) *n_bad = 0;
    return TFS_SUCCESS;
  }
  // A page-locked image is read in place on a synchronous slot's own stream, the
  // wait outside the context lock (round 6): verifies from several threads -- the
  // mirror, repair and checker call sites -- run side by side, the next block's
  // waves filling the link while the last waves of another drain.
  void* zc = nullptr;
  if (ctx->variant != kVariantDmaCompact && ctx->variant != kVariantStagedWide && is_pinned_host(image) &&
      host_dev_ptr(image, &zc)) {
    Slot* s = nullptr;
    {
      std::unique_lock<std::mutex> lk(ctx->mu);
      if (const int f = injected_fault(ctx)) return f;
      HIP_TRY(ctx, hipSetDevice(ctx->device));
      for (;;) {
        for (Slot& x : ctx->sync_slots)
          if (!x.busy) {
            s = &x;
            break;
          }
        if (s) break;
        ctx->sync_cv.wait(lk);
      }
      s->busy = true;
      s->resident = false;
      const int rc = block_verify_inplace_enqueue(ctx, s, static_cast<const uint8_t*>(zc), image_len, metas, n);
      if (rc) {
        s->busy = false;
        ctx->sync_cv.notify_one();
        return rc;
      }
    }
    const hipError_t e = hipEventSynchronize(s->done);
    int rc = TFS_SUCCESS;
    uint32_t bad = 0;
    if (e != hipSuccess) {
      std::lock_guard<std::mutex> g(ctx->mu);
      rc = set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "block_verify: %s", hipGetErrorString(e));
    } else {
      const int32_t* st = static_cast<const int32_t*>(s->h_ok.p);
      for (uint32_t i = 0; i < n; ++i) bad += st[i] != TFS_SUCCESS ? 1u : 0u;
      if (out_crc) memcpy(out_crc, s->h_crc.p, size_t(n) * 4);
      if (out_status) memcpy(out_status, st, size_t(n) * 4);
      if (n_bad) *n_bad = bad;
      rc = bad ? TFS_EXIT_CHECK_CRC_ERROR : TFS_SUCCESS;
    }
    {
      std::lock_guard<std::mutex> g(ctx->mu);
      s->busy = false;
    }
    ctx->sync_cv.notify_one();
    return rc;
  }
  (void)hipGetLastError();
  std::lock_guard<std::mutex> g(ctx->mu);
  if (const int f = injected_fault(ctx)) return f;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  Slot* s = free_slot(ctx);
  if (!s) return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "all %d slots busy", kSlots);
  // Pageable images (and the measurement build's staged forms) are staged: one
  // whole-image copy, then the launch on the context stream.
  const uint8_t* d_base = nullptr;
  if (ctx->variant == kVariantStagedWide && is_pinned_host(image) && host_dev_ptr(image, &zc)) {
    d_base = static_cast<const uint8_t*>(zc);  // the round-5 form: in place, copies through DMA
  } else {
    (void)hipGetLastError();
    const int rc = stage_span(ctx, *s, image, 0, image_len, &d_base);
    if (rc) return rc;
  }
  HIP_TRY(ctx, s->d_desc.reserve(size_t(n) * sizeof(RawMeta)));
  HIP_TRY(ctx, s->d_crc.reserve(size_t(n) * 4));
  HIP_TRY(ctx, s->d_ok.reserve(size_t(n) * 4));
  HIP_TRY(ctx, s->d_bad.reserve(4));
  HIP_TRY(ctx, s->h_crc.reserve(size_t(n) * 4));
  HIP_TRY(ctx, s->h_ok.reserve(size_t(n) * 4));
  HIP_TRY(ctx, s->h_bad.reserve(4));
  HIP_TRY(ctx, hipMemcpyAsync(s->d_desc.p, metas, size_t(n) * sizeof(RawMeta), hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(ctx, hipMemsetAsync(s->d_bad.p, 0, 4, ctx->stream));
  SCHED_LAUNCH(ctx, ctx->stream, "block_verify_pipe", launch_block_verify_pipe(d_base, image_len, static_cast<const RawMeta*>(s->d_desc.p), nullptr, n,
                                        ctx->d_tables, static_cast<uint32_t*>(s->d_crc.p),
                                        static_cast<int32_t*>(s->d_ok.p), static_cast<uint32_t*>(s->d_bad.p), sched,
                                        ctx->stream, ctx->variant, throughput_cap(ctx)));
  HIP_TRY(ctx, hipMemcpyAsync(s->h_crc.p, s->d_crc.p, size_t(n) * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(s->h_ok.p, s->d_ok.p, size_t(n) * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(s->h_bad.p, s->d_bad.p, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  if (out_crc) memcpy(out_crc, s->h_crc.p, size_t(n) * 4);
  if (out_status) memcpy(out_status, s->h_ok.p, size_t(n) * 4);
  const uint32_t bad = *static_cast<uint32_t*>(s->h_bad.p);
  if (n_bad) *n_bad = bad;
  return bad ? TFS_EXIT_CHECK_CRC_ERROR : TFS_SUCCESS;
}

// ---- compaction pipeline --------------------------------------------------
// Each block goes through its own slot/stream: H2D of the source image, verify
// of the live files, repack kernel, D2H of the new image.  With kCompactSlots
// slots the H2D of block i+1, the kernels of block i and the D2H of block i-1
// overlap (PCIe is full duplex; the copy engines run beside the kernels).

static int compact_dma(tfs_crc_ctx* ctx, CompactSlot& cs, tfs_block_job* job, uint32_t nl, int64_t w, uint8_t* da,
                       const uint8_t* ha, size_t aux_h2d, const RawMeta* d_metas, const int32_t* d_flags,
                       const int64_t* d_doff, uint32_t* d_crc, int32_t* d_status);

static int compact_enqueue(tfs_crc_ctx* ctx, CompactSlot& cs, tfs_block_job* job) {
  const uint32_t n = job->n;
  cs.job = job;
  // A slot that last carried a group must not finish this block as one.
  cs.gjobs.clear();
  cs.gstart.clear();
  cs.live_idx.clear();
  job->status = TFS_SUCCESS;
  job->dest_len = 0;
  job->n_live = 0;
  if (const int f = injected_fault(ctx)) return f;
  if (n && (!job->src_image || !job->metas || !job->flags || !job->dest_image))
    return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "null block job pointer");
  // Host: new offsets in iteration order (task.cpp:753-768).
  int64_t w = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const tfs_raw_meta& m = job->metas[i];
    if (m.size < TFS_FILEINFO_SIZE || m.offset < 0 || uint64_t(m.offset) + uint64_t(m.size) > job->src_len)
      return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "meta %u out of range", i);
    if (job->flags[i] & (TFS_FI_DELETED | TFS_FI_INVALID)) continue;
    cs.live_idx.push_back(i);
    w += m.size;
  }
  if (uint64_t(w) > job->dest_cap)
    return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "dest_cap %llu < %lld", (unsigned long long)job->dest_cap,
                   (long long)w);
  const uint32_t nl = uint32_t(cs.live_idx.size());
  const size_t mb = size_t(nl) * sizeof(RawMeta), fb = size_t(nl) * 4, ob = size_t(nl) * 8;
  const size_t aux_bytes = ob + mb + fb + 64;
  HIP_TRY(ctx, cs.h_aux.reserve(aux_bytes));
  HIP_TRY(ctx, cs.d_aux.reserve(aux_bytes + 2 * fb + 64));
  uint8_t* ha = static_cast<uint8_t*>(cs.h_aux.p);
  int64_t* h_doff = reinterpret_cast<int64_t*>(ha);
  RawMeta* h_metas = reinterpret_cast<RawMeta*>(ha + ob);
  int32_t* h_flags = reinterpret_cast<int32_t*>(ha + ob + mb);
  // Zero-copy form: when both images are page-locked, the fused kernel reads the
  // live records straight out of the source image over PCIe and writes the new
  // block straight into the destination image, so only live bytes cross the
  // link (the deleted records of a fragmented block never leave host memory).
  // Every destination shift copies through the kernel's CRC chain (only payloads
  // shorter than one stripe are read a second time), so any layout qualifies.
  bool zc = nl && ctx->variant != kVariantDmaCompact && is_pinned_host(job->src_image) &&
            is_pinned_host(job->dest_image);
  int64_t off = 0;
  for (uint32_t k = 0; k < nl; ++k) {
    const uint32_t i = cs.live_idx[k];
    h_doff[k] = off;
    h_metas[k] = RawMeta{job->metas[i].file_id, job->metas[i].offset, job->metas[i].size};
    h_flags[k] = job->flags[i];
    if (job->dest_metas) job->dest_metas[k] = tfs_raw_meta{job->metas[i].file_id, int32_t(off), job->metas[i].size};
    off += job->metas[i].size;
  }
  void* zc_src = nullptr;
  void* zc_dst = nullptr;
  if (zc && (!host_dev_ptr(job->src_image, &zc_src) || !host_dev_ptr(job->dest_image, &zc_dst))) zc = false;
  uint8_t* da = static_cast<uint8_t*>(cs.d_aux.p);
  int64_t* d_doff = reinterpret_cast<int64_t*>(da);
  RawMeta* d_metas = reinterpret_cast<RawMeta*>(da + ob);
  int32_t* d_flags = reinterpret_cast<int32_t*>(da + ob + mb);
  uint32_t* d_crc = reinterpret_cast<uint32_t*>(da + ((aux_bytes + 15) & ~size_t(15)));
  int32_t* d_status = reinterpret_cast<int32_t*>(d_crc + nl);
  HIP_TRY(ctx, cs.h_status.reserve(fb + 4));
  if (zc) {
    HIP_TRY(ctx, hipMemcpyAsync(da, ha, ob + mb + fb, hipMemcpyHostToDevice, cs.stream));
    uint8_t* kdst = static_cast<uint8_t*>(zc_dst);
    SCHED_LAUNCH(ctx, cs.stream, "compact_fused", launch_compact_fused(static_cast<const uint8_t*>(zc_src), job->src_len, d_metas, d_flags, d_doff, nl,
                                      kdst, ctx->d_tables, d_crc, d_status, nullptr, sched, cs.stream, ctx->variant, throughput_cap(ctx)));
    HIP_TRY(ctx, hipMemcpyAsync(cs.h_status.p, d_status, fb, hipMemcpyDeviceToHost, cs.stream));
  } else {
    const int rc = compact_dma(ctx, cs, job, nl, w, da, ha, ob + mb + fb, d_metas, d_flags, d_doff, d_crc, d_status);
    if (rc != TFS_SUCCESS) return rc;
  }
  if (!cs.done) HIP_TRY(ctx, hipEventCreateWithFlags(&cs.done, hipEventDisableTiming));
  HIP_TRY(ctx, hipEventRecord(cs.done, cs.stream));
  job->dest_len = uint64_t(w);
  job->n_live = nl;
  cs.busy = true;
  return TFS_SUCCESS;
}

// Whole-block form: H2D of the source image, fused kernel device to device,
// D2H of the new block.
static int compact_dma(tfs_crc_ctx* ctx, CompactSlot& cs, tfs_block_job* job, uint32_t nl, int64_t w, uint8_t* da,
                       const uint8_t* ha, size_t aux_h2d, const RawMeta* d_metas, const int32_t* d_flags,
                       const int64_t* d_doff, uint32_t* d_crc, int32_t* d_status) {
  const size_t fb = size_t(nl) * 4;
  HIP_TRY(ctx, cs.d_src.reserve(job->src_len + 16));
  HIP_TRY(ctx, cs.d_dst.reserve(uint64_t(w) + 16));
  HIP_TRY(ctx, cs.h_status.reserve(fb + 4));
  if (job->src_len) {
    if (is_pinned_host(job->src_image)) {
      HIP_TRY(ctx, hipMemcpyAsync(cs.d_src.p, job->src_image, job->src_len, hipMemcpyHostToDevice, cs.stream));
    } else {
      HIP_TRY(ctx, cs.h_stage.reserve(job->src_len));
      memcpy(cs.h_stage.p, job->src_image, job->src_len);
      HIP_TRY(ctx, hipMemcpyAsync(cs.d_src.p, cs.h_stage.p, job->src_len, hipMemcpyHostToDevice, cs.stream));
    }
  }
  if (nl) {
    HIP_TRY(ctx, hipMemcpyAsync(da, ha, aux_h2d, hipMemcpyHostToDevice, cs.stream));
    const uint8_t* d_src = static_cast<const uint8_t*>(cs.d_src.p);
    // One read of every live record: re-CRC (the verify the reference's
    // real_compact does not do) and repack from the same registers.
    SCHED_LAUNCH(ctx, cs.stream, "compact_fused", launch_compact_fused(d_src, job->src_len, d_metas, d_flags, d_doff, nl,
                                      static_cast<uint8_t*>(cs.d_dst.p), ctx->d_tables, d_crc, d_status, nullptr, sched,
                                      cs.stream, ctx->variant, throughput_cap(ctx)));
    HIP_TRY(ctx, hipMemcpyAsync(cs.h_status.p, d_status, fb, hipMemcpyDeviceToHost, cs.stream));
    if (w) HIP_TRY(ctx, hipMemcpyAsync(job->dest_image, cs.d_dst.p, size_t(w), hipMemcpyDeviceToHost, cs.stream));
  }
  return TFS_SUCCESS;
}

// Zero-copy groups (round 5).  Blocks whose source and
// destination images are both page-locked go to the GPU compact_group (64) at a time
// as ONE multi-block record launch (tfs_compact_jobs_device's kernel, offsets
// taken from the lowest image address of the group), instead of one launch per
// block: a block is only ~341 live records, so per-block launches kept at most
// 8 x 341 waves (176 workgroups) reading over PCIe, with a copy-engine hop
// before and after each kernel.  Blocks per launch, measured in one process
// (tools/compact_group_probe.py, profiles/r05/host_compact_groups/): 1 -> 0.88 of
// the link's measured duplex rate, 8 -> 0.93, 16 -> 0.94, 32 -> 0.95, 64 -> 0.96.

bool zc_eligible(const tfs_crc_ctx* ctx, const tfs_block_job& job) {
  return job.n && ctx->variant != kVariantDmaCompact && job.src_image && job.dest_image && job.metas && job.flags &&
         is_pinned_host(job.src_image) && is_pinned_host(job.dest_image);
}

static int compact_enqueue_group_body(tfs_crc_ctx* ctx, CompactSlot& cs, tfs_block_job* jobs, uint32_t count);

// Any failure leaves the slot idle and empty: no job pointer of this call may
// survive into a later compact_finish of the same slot.
static int compact_enqueue_group(tfs_crc_ctx* ctx, CompactSlot& cs, tfs_block_job* jobs, uint32_t count) {
  const int rc = compact_enqueue_group_body(ctx, cs, jobs, count);
  if (rc != TFS_SUCCESS) {
    cs.busy = false;
    cs.job = nullptr;
    cs.gjobs.clear();
    cs.gstart.clear();
    cs.live_idx.clear();
  }
  return rc;
}

static int compact_enqueue_group_body(tfs_crc_ctx* ctx, CompactSlot& cs, tfs_block_job* jobs, uint32_t count) {
  cs.job = nullptr;
  cs.gjobs.clear();
  cs.gstart.clear();
  cs.live_idx.clear();
  struct Span {
    uintptr_t src, dst;
  };
  std::vector<Span> sp(count);
  uintptr_t sbase = UINTPTR_MAX, send = 0, dbase = UINTPTR_MAX;
  for (uint32_t k = 0; k < count; ++k) {
    tfs_block_job* job = &jobs[k];
    job->status = TFS_SUCCESS;
    job->dest_len = 0;
    job->n_live = 0;
    if (const int f = injected_fault(ctx)) {
      job->status = f;
      return f;
    }
    // Validate the whole job before anything of the group is recorded.
    int64_t w = 0;
    for (uint32_t i = 0; i < job->n; ++i) {
      const tfs_raw_meta& m = job->metas[i];
      if (m.size < TFS_FILEINFO_SIZE || m.offset < 0 || uint64_t(m.offset) + uint64_t(m.size) > job->src_len) {
        job->status = TFS_EXIT_PARAMETER_ERROR;
        return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "meta %u out of range", i);
      }
      if (job->flags[i] & (TFS_FI_DELETED | TFS_FI_INVALID)) continue;
      w += m.size;
    }
    if (uint64_t(w) > job->dest_cap) {
      job->status = TFS_EXIT_PARAMETER_ERROR;
      return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "dest_cap %llu too small", (unsigned long long)job->dest_cap);
    }
    void *zs = nullptr, *zd = nullptr;
    if (!host_dev_ptr(job->src_image, &zs) || !host_dev_ptr(job->dest_image, &zd))
      return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "page-locked image without a device address");
    sp[k] = Span{reinterpret_cast<uintptr_t>(zs), reinterpret_cast<uintptr_t>(zd)};
    sbase = std::min(sbase, sp[k].src);
    send = std::max<uintptr_t>(send, sp[k].src + job->src_len);
    dbase = std::min(dbase, sp[k].dst);
  }
  // Host: each block's new offsets in iteration order (task.cpp:753-768), its
  // RawMeta list, and one CompactJob per live record with group-relative offsets.
  std::vector<CompactJob>& cj = cs.gjob_list;
  cj.clear();
  for (uint32_t k = 0; k < count; ++k) {
    tfs_block_job* job = &jobs[k];
    cs.gjobs.push_back(job);
    cs.gstart.push_back(uint32_t(cs.live_idx.size()));
    int64_t w = 0;
    for (uint32_t i = 0; i < job->n; ++i) {
      const tfs_raw_meta& m = job->metas[i];  // validated above
      if (job->flags[i] & (TFS_FI_DELETED | TFS_FI_INVALID)) continue;
      if (job->dest_metas) job->dest_metas[cs.live_idx.size() - cs.gstart.back()] =
          tfs_raw_meta{m.file_id, int32_t(w), m.size};
      const bool edge = uint64_t(m.offset) + uint64_t(m.size) + 128u > job->src_len;
      cj.push_back(CompactJob{sp[k].src - sbase + uint64_t(m.offset), sp[k].dst - dbase + uint64_t(w), m.file_id,
                              m.size, job->flags[i], int32_t(w), edge ? TFS_COMPACT_JOB_EDGE : 0});
      cs.live_idx.push_back(i);
      w += m.size;
    }
    job->dest_len = uint64_t(w);
    job->n_live = uint32_t(cs.live_idx.size()) - cs.gstart.back();
  }
  const uint32_t nl = uint32_t(cj.size());
  const size_t jb = size_t(nl) * sizeof(CompactJob), fb = size_t(nl) * 4;
  HIP_TRY(ctx, cs.h_aux.reserve(jb + 64));
  HIP_TRY(ctx, cs.d_aux.reserve(jb + 2 * fb + 128));
  HIP_TRY(ctx, cs.h_status.reserve(fb + 4));
  if (nl) {
    memcpy(cs.h_aux.p, cj.data(), jb);
    uint8_t* da = static_cast<uint8_t*>(cs.d_aux.p);
    const CompactJob* d_jobs = reinterpret_cast<const CompactJob*>(da);
    uint32_t* d_crc = reinterpret_cast<uint32_t*>(da + ((jb + 63) & ~size_t(63)));
    int32_t* d_status = reinterpret_cast<int32_t*>(d_crc + nl);
    HIP_TRY(ctx, hipMemcpyAsync(da, cs.h_aux.p, jb, hipMemcpyHostToDevice, cs.stream));
    SCHED_LAUNCH(ctx, cs.stream, "compact_group",
                 launch_compact_jobs(reinterpret_cast<const uint8_t*>(sbase), uint64_t(send - sbase), d_jobs, nl,
                                     reinterpret_cast<uint8_t*>(dbase), ctx->d_tables, d_crc, d_status, nullptr, sched,
                                     cs.stream, ctx->variant, throughput_cap(ctx), nullptr));
    HIP_TRY(ctx, hipMemcpyAsync(cs.h_status.p, d_status, fb, hipMemcpyDeviceToHost, cs.stream));
  }
  if (!cs.done) HIP_TRY(ctx, hipEventCreateWithFlags(&cs.done, hipEventDisableTiming));
  HIP_TRY(ctx, hipEventRecord(cs.done, cs.stream));
  cs.busy = true;
  return TFS_SUCCESS;
}

static int compact_finish(tfs_crc_ctx* ctx, CompactSlot& cs) {
  if (!cs.busy) return TFS_SUCCESS;
  cs.busy = false;
  HIP_TRY(ctx, hipEventSynchronize(cs.done));
  if (!cs.gjobs.empty()) {  // a zero-copy group: statuses per job
    const int32_t* st = static_cast<const int32_t*>(cs.h_status.p);
    int worst = TFS_SUCCESS;
    for (size_t k = 0; k < cs.gjobs.size(); ++k) {
      tfs_block_job* job = cs.gjobs[k];
      const uint32_t a = cs.gstart[k], e = k + 1 < cs.gjobs.size() ? cs.gstart[k + 1] : uint32_t(cs.live_idx.size());
      if (job->crc_ok)
        for (uint32_t i = 0; i < job->n; ++i) job->crc_ok[i] = 2;  // skipped unless live
      uint32_t bad = 0;
      for (uint32_t q = a; q < e; ++q) {
        const bool ok = st[q] == TFS_SUCCESS;
        bad += ok ? 0u : 1u;
        if (job->crc_ok) job->crc_ok[cs.live_idx[q]] = ok ? 1 : 0;
      }
      job->status = bad ? TFS_EXIT_CHECK_CRC_ERROR : TFS_SUCCESS;
      if (bad) worst = TFS_EXIT_CHECK_CRC_ERROR;
    }
    cs.gjobs.clear();
    return worst;
  }
  tfs_block_job* job = cs.job;
  const int32_t* st = static_cast<const int32_t*>(cs.h_status.p);
  if (job->crc_ok)
    for (uint32_t i = 0; i < job->n; ++i) job->crc_ok[i] = 2;  // skipped unless live
  uint32_t bad = 0;
  for (uint32_t k = 0; k < uint32_t(cs.live_idx.size()); ++k) {
    const bool ok = st[k] == TFS_SUCCESS;
    bad += ok ? 0u : 1u;
    if (job->crc_ok) job->crc_ok[cs.live_idx[k]] = ok ? 1 : 0;
  }
  job->status = bad ? TFS_EXIT_CHECK_CRC_ERROR : TFS_SUCCESS;
  return job->status;
}

int tfs_blocks_compact(tfs_crc_ctx* ctx, tfs_block_job* jobs, uint32_t njobs) {
  if (!ctx || (njobs && !jobs)) return TFS_EXIT_PARAMETER_ERROR;
  std::lock_guard<std::mutex> g(ctx->mu);
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  for (auto& cs : ctx->cslots)
    if (!cs.stream) {
      HIP_TRY(ctx, hipStreamCreateWithFlags(&cs.stream, hipStreamNonBlocking));
      HIP_TRY(ctx, bind_owned_stream(ctx, cs.stream));
    }
  int worst = TFS_SUCCESS;
  auto note = [&](int rc) {
    if (rc != TFS_SUCCESS && (worst == TFS_SUCCESS || worst == TFS_EXIT_CHECK_CRC_ERROR)) worst = rc;
  };
  uint32_t slot = 0;
  uint32_t unissued = njobs;  // first job never enqueued after a device error
  int stop_rc = TFS_SUCCESS;  // that device error
  for (uint32_t j = 0; j < njobs && unissued == njobs;) {
    CompactSlot& cs = ctx->cslots[slot++ % uint32_t(ctx->compact_slots)];
    note(compact_finish(ctx, cs));
    // a run of up to compact_group zero-copy blocks goes as one launch
    uint32_t g = 0;
    while (g < ctx->compact_group && j + g < njobs && zc_eligible(ctx, jobs[j + g])) ++g;
    const int rc = g >= 2 ? compact_enqueue_group(ctx, cs, &jobs[j], g) : compact_enqueue(ctx, cs, &jobs[j]);
    const uint32_t took = g >= 2 ? g : 1u;
    if (rc != TFS_SUCCESS) {
      if (took == 1) jobs[j].status = rc;
      note(rc);
      if (rc != TFS_EXIT_PARAMETER_ERROR) {  // device error: stop issuing, drain below
        unissued = j;
        stop_rc = rc;
        break;
      }
      if (took > 1) {  // a bad job inside a group: run the group's jobs one by one instead
        for (uint32_t q = 0; q < took; ++q) {
          CompactSlot& c1 = ctx->cslots[slot++ % uint32_t(ctx->compact_slots)];
          note(compact_finish(ctx, c1));
          const int r1 = compact_enqueue(ctx, c1, &jobs[j + q]);
          if (r1 != TFS_SUCCESS) {
            jobs[j + q].status = r1;
            note(r1);
            if (r1 != TFS_EXIT_PARAMETER_ERROR) {
              unissued = j + q;
              stop_rc = r1;
              break;
            }
          }
        }
      }
    }
    j += took;
  }
  // Jobs never issued carry the error that stopped the call, not a stale status.
  for (uint32_t j = unissued; j < njobs; ++j) {
    if (j > unissued || jobs[j].status == TFS_SUCCESS) jobs[j].status = stop_rc;
    jobs[j].dest_len = 0;
    jobs[j].n_live = 0;
  }
  for (auto& cs : ctx->cslots) note(compact_finish(ctx, cs));
  return worst;
}

int tfs_block_compact_device(tfs_crc_ctx* ctx, const void* d_src, uint64_t src_len, const tfs_raw_meta* d_live_metas,
                             const int32_t* d_flags, const int64_t* d_dest_off, uint32_t n, void* d_dest,
                             uint32_t* d_out_crc, int32_t* d_out_status, uint32_t* d_n_bad, void* stream) {
  if (!ctx || (n && (!d_src || !d_live_metas || !d_flags || !d_dest_off || !d_dest))) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  SCHED_LAUNCH(ctx, st, "compact_fused", launch_compact_fused(static_cast<const uint8_t*>(d_src), src_len,
                                    reinterpret_cast<const RawMeta*>(d_live_metas), d_flags, d_dest_off, n,
                                    static_cast<uint8_t*>(d_dest), ctx->d_tables, d_out_crc, d_out_status, d_n_bad,
                                    sched, st, ctx->variant, throughput_cap(ctx)));
  return TFS_SUCCESS;
}

int tfs_compact_jobs_device(tfs_crc_ctx* ctx, const void* d_src, uint64_t src_len, const tfs_compact_job* d_jobs,
                            uint32_t n, void* d_dest, uint32_t* d_out_crc, int32_t* d_out_status, uint32_t* d_n_bad,
                            void* stream) {
  if (!ctx || (n && (!d_src || !d_jobs || !d_dest))) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if (n == 0) return TFS_SUCCESS;
  SchedLease lease;
  if (const int r = sched_acquire(ctx, st, &lease)) return r;
  const uint32_t k = plan_index(lease, slot_index(ctx, lease));
  std::unique_lock<std::mutex> lk(ctx->plan_mu[k], std::defer_lock);
  CSegArgs cs{nullptr, 0u, 0u};
  int rc = TFS_SUCCESS;
  const uint32_t lg = cseg_lg(ctx, n);
  if (lg) {
    lk.lock();
    rc = plan_order(ctx, st, lease, k);
    if (rc == TFS_SUCCESS) rc = cseg_prepare(ctx, st, k, n, lg, &cs);
  }
  const hipError_t le =
      rc == TFS_SUCCESS ? launch_compact_jobs(static_cast<const uint8_t*>(d_src), src_len,
                                              reinterpret_cast<const CompactJob*>(d_jobs), n,
                                              static_cast<uint8_t*>(d_dest), ctx->d_tables, d_out_crc, d_out_status,
                                              d_n_bad, lease.slot, st, ctx->variant, throughput_cap(ctx),
                                              cs.plan ? &cs : nullptr)
                        : hipSuccess;
  if (cs.plan && le == hipSuccess) {
    rc = plan_mark(ctx, st, k);
  }
  const int r2 = sched_release(ctx, st, lease, le, "compact_jobs");
  return rc != TFS_SUCCESS ? rc : r2;
}

int tfs_block_compact(tfs_crc_ctx* ctx, const void* src_image, uint64_t src_len, const tfs_raw_meta* metas,
                      const int32_t* flags, uint32_t n, void* dest_image, uint64_t dest_cap, tfs_raw_meta* dest_metas,
                      uint8_t* crc_ok, uint64_t* dest_len, uint32_t* n_live) {
  tfs_block_job job;
  memset(&job, 0, sizeof job);
  job.src_image = src_image;
  job.src_len = src_len;
  job.metas = metas;
  job.flags = flags;
  job.n = n;
  job.dest_image = dest_image;
  job.dest_cap = dest_cap;
  job.dest_metas = dest_metas;
  job.crc_ok = crc_ok;
  const int rc = tfs_blocks_compact(ctx, &job, 1);
  if (dest_len) *dest_len = job.dest_len;
  if (n_live) *n_live = job.n_live;
  return rc;
}

// ---- packet CRC ------------------------------------------------------------
// Throughput launches (more than kWgMaxFiles frames): one pass,
// packet_files_kernel (round 5).  Smaller launches, and the measurement build's
// TFS_CRC_VARIANT=51: parse (frame -> body descriptor + pre-status) -> CRC kernel
// over the bodies (verify: seed TFS_PACKET_FLAG_V1 vs the header crc; seal:
// compute) -> finish (statuses, seal writes the header crc).  `scratch` holds n
// Desc, n pre-status and n ok bytes.
#ifdef TFS_CRC_MEASURE
constexpr int kVariantPacket3 = 51;  // the three-launch packet form for throughput launches (A/B)
#endif

static size_t packet_scratch_bytes(uint32_t n) { return size_t(n) * (sizeof(Desc) + 4 + 4 + 1) + 64; }

static int packet_enqueue(tfs_crc_ctx* ctx, int mode, const PacketDesc* d_pd, uint32_t n, uint8_t* d_base,
                          void* scratch, uint32_t* d_crc, int32_t* d_status, uint32_t* d_n_bad, hipStream_t st) {
  uint8_t* sp = static_cast<uint8_t*>(scratch);
  Desc* d_desc = reinterpret_cast<Desc*>(sp);
  int32_t* d_pre = reinterpret_cast<int32_t*>(sp + size_t(n) * sizeof(Desc));
  uint32_t* d_tmp_crc = reinterpret_cast<uint32_t*>(sp + size_t(n) * (sizeof(Desc) + 4));
  uint8_t* d_ok = sp + size_t(n) * (sizeof(Desc) + 8);
  uint32_t* crc = d_crc ? d_crc : d_tmp_crc;
  bool one_pass = n > kWgMaxFiles;
#ifdef TFS_CRC_MEASURE
  if (ctx->variant == kVariantPacket3) one_pass = false;
#endif
  if (one_pass) {
    SCHED_LAUNCH(ctx, st, "packet_files",
                 launch_packet_files(d_base, d_pd, n, mode, ctx->d_tables, d_crc, d_status, d_n_bad, sched, st,
                                     throughput_cap(ctx)));
    return TFS_SUCCESS;
  }
  HIP_TRY(ctx, launch_packet_parse(d_base, d_pd, n, mode, d_desc, d_pre, st));
  if (const int rc = files_launch(ctx, st, mode, d_base, d_desc, n, crc, mode == 1 ? d_ok : nullptr, nullptr,
                                  kPacketFlagV1))
    return rc;
  HIP_TRY(ctx, launch_packet_finish(d_base, d_pd, d_desc, n, mode, d_pre, d_ok, crc, d_status, d_n_bad, st));
  return TFS_SUCCESS;
}

// Device-resident: scratch comes from slot 0's d_aux under the ctx mutex.
static int packet_device(tfs_crc_ctx* ctx, int mode, const tfs_packet_desc* d_desc, uint32_t n, void* d_base,
                         uint32_t* d_out_crc, int32_t* d_out_status, uint32_t* d_n_bad, void* stream) {
  if (!ctx || (n && (!d_desc || !d_base || !d_out_status))) return TFS_EXIT_PARAMETER_ERROR;
  if (n == 0) return TFS_SUCCESS;
  std::lock_guard<std::mutex> g(ctx->mu);
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  // The scratch buffer is shared by device-resident packet calls: calls on one
  // stream are ordered by the stream; switching streams waits for the last one.
  if (ctx->packet_scratch_stream && ctx->packet_scratch_stream != st)
    HIP_TRY(ctx, hipStreamSynchronize(ctx->packet_scratch_stream));
  if (packet_scratch_bytes(n) > ctx->packet_scratch.cap && ctx->packet_scratch_stream)
    HIP_TRY(ctx, hipStreamSynchronize(ctx->packet_scratch_stream));  // growing frees the old buffer
  HIP_TRY(ctx, ctx->packet_scratch.reserve(packet_scratch_bytes(n)));
  ctx->packet_scratch_stream = st;
  return packet_enqueue(ctx, mode, reinterpret_cast<const PacketDesc*>(d_desc), n, static_cast<uint8_t*>(d_base),
                        ctx->packet_scratch.p, d_out_crc, d_out_status, d_n_bad, st);
}

static uint32_t le32(const uint8_t* p) {
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}

// A frame's header as packet_parse_kernel reads it (getPacketInfo, base_packet_
// streamer.cpp:43-124, and the version decode() sees, base_packet.cpp:100-141):
// the body descriptor (seed TFS_PACKET_FLAG_V1; aux = the stored crc for a
// verify) and the pre-status -- kPacketPending when the body CRC decides.
static void packet_parse_host(const uint8_t* base, const tfs_packet_desc& f, int mode, Desc* d, int32_t* pre) {
  *d = Desc{f.offset, 0u, kPacketFlagV1};
  const uint8_t* p = base + f.offset;
  if (f.len < uint32_t(kPacketHeaderV0Size)) {
    *pre = kPacketIncomplete;
    return;
  }
  const uint32_t flag = le32(p);
  const int32_t length = int32_t(le32(p + 4));
  const int32_t type = int16_t(uint16_t(p[8] | p[9] << 8)), check = int16_t(uint16_t(p[10] | p[11] << 8));
  const bool v1 = flag == kPacketFlagV1;
  if (v1 && f.len < uint32_t(kPacketHeaderV0Size + kPacketHeaderDiffSize)) {
    *pre = kPacketIncomplete;
  } else if ((flag != kPacketFlagV0 && !v1) || length <= 0 || length > kPacketMaxDataLen) {
    *pre = kTfsError;
  } else {
    const int64_t data_len = int64_t(length) + (v1 ? kPacketHeaderDiffSize : 0);
    const uint32_t version = ((type < 0) ? 0xFFFFu : 0u) | (v1 ? uint32_t(uint16_t(check)) : 0u);
    if (uint64_t(kPacketHeaderV0Size) + uint64_t(data_len) > f.len) {
      *pre = kPacketIncomplete;
    } else if (version >= 1u) {
      if (data_len < kPacketHeaderDiffSize) {
        *pre = kTfsError;
      } else {
        d->offset = f.offset + kPacketHeaderV0Size + kPacketHeaderDiffSize;
        d->len = uint32_t(data_len - kPacketHeaderDiffSize);
        d->aux = mode == 1 ? le32(p + kPacketHeaderV0Size + 8) : kPacketFlagV1;
        *pre = kPacketPending;
      }
    } else {
      *pre = kSuccess;
    }
  }
}

// Small host batches (a connection's read, a send queue's few packets): the
// headers are walked on the host as the streamer does and the bodies' CRCs go
// through the synchronous small-batch path (read in place, the resident kernel)
// -- one GPU round trip instead of parse, CRC and finish launches with their
// copies.  Same statuses, CRCs and sealed bytes as the launched path.
static int packet_host_small(tfs_crc_ctx* ctx, int mode, const tfs_packet_desc* d, uint32_t n, void* base,
                             uint64_t base_len, uint32_t* out_crc, int32_t* out_status, uint32_t* n_bad) {
  std::vector<Desc> body;
  std::vector<uint32_t> idx;
  std::vector<int32_t> pre(n);
  std::vector<uint32_t> stored(n, 0u);
  body.reserve(n);
  idx.reserve(n);
  const uint8_t* b8 = static_cast<const uint8_t*>(base);
  for (uint32_t i = 0; i < n; ++i) {
    Desc x;
    packet_parse_host(b8, d[i], mode, &x, &pre[i]);
    if (pre[i] != kPacketPending) continue;
    stored[i] = x.aux;
    x.aux = kPacketFlagV1;  // computed with the packet seed, compared here
    idx.push_back(i);
    body.push_back(x);
  }
  std::vector<uint32_t> crc(body.size());
  if (body.empty()) {
    if (const int f = injected_fault(ctx)) return f;  // as the launched path (no GPU call to fail here)
  } else {
    const int rc = tfs_crc32_batch(ctx, reinterpret_cast<const tfs_crc_desc*>(body.data()), uint32_t(body.size()),
                                   base, base_len, crc.data());
    if (rc) return rc;
  }
  uint32_t bad = 0;
  if (out_crc) memset(out_crc, 0, size_t(n) * 4);
  for (size_t k = 0; k < idx.size(); ++k) {
    const uint32_t i = idx[k];
    if (out_crc) out_crc[i] = crc[k];
    if (mode == 1) {
      pre[i] = crc[k] == stored[i] ? kSuccess : kExitCheckCrcError;  // decode (base_packet.cpp:142-148)
    } else {
      pre[i] = kSuccess;
      uint8_t* p = static_cast<uint8_t*>(base) + d[i].offset;
      if (le32(p) == TFS_PACKET_FLAG_V1)  // seal: only V1 headers carry a crc (base_packet_streamer.cpp:166-175)
        for (int b = 0; b < 4; ++b) p[TFS_PACKET_HEADER_V0_SIZE + 8 + b] = uint8_t(crc[k] >> (8 * b));
    }
  }
  for (uint32_t i = 0; i < n; ++i) bad += pre[i] != kSuccess ? 1u : 0u;
  if (out_status) memcpy(out_status, pre.data(), size_t(n) * 4);
  if (n_bad) *n_bad = bad;
  if (mode == 0) return TFS_SUCCESS;
  return bad ? TFS_EXIT_CHECK_CRC_ERROR : TFS_SUCCESS;
}

static int packet_host(tfs_crc_ctx* ctx, int mode, const tfs_packet_desc* d, uint32_t n, void* base,
                       uint64_t base_len, uint32_t* out_crc, int32_t* out_status, uint32_t* n_bad) {
  if (!ctx || (n && (!d || !base))) return TFS_EXIT_PARAMETER_ERROR;
  if (n_bad) *n_bad = 0;
  if (n == 0) return TFS_SUCCESS;
  {
    uint64_t lo = 0, hi = 0;
    if (ctx->variant == 0 && n <= kWgMaxFiles && span_of(d, n, base_len, &lo, &hi) && hi - lo <= kZeroCopySpan)
      return packet_host_small(ctx, mode, d, n, base, base_len, out_crc, out_status, n_bad);
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  if (const int f = injected_fault(ctx)) return f;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  Slot* s = free_slot(ctx);
  if (!s) return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "all %d slots busy with async submissions", kSlots);
  uint64_t lo = 0, hi = 0;
  if (!span_of(d, n, base_len, &lo, &hi))
    return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "frame range exceeds base_len %llu", (unsigned long long)base_len);
  const uint8_t* d_base = nullptr;
  int rc = stage_span(ctx, *s, base, lo, hi, &d_base);
  if (rc) return rc;
  HIP_TRY(ctx, s->d_desc.reserve(size_t(n) * sizeof(PacketDesc)));
  HIP_TRY(ctx, s->d_aux.reserve(packet_scratch_bytes(n)));
  HIP_TRY(ctx, s->d_crc.reserve(size_t(n) * 4));
  HIP_TRY(ctx, s->d_ok.reserve(size_t(n) * 4));  // statuses
  HIP_TRY(ctx, s->d_bad.reserve(4));
  HIP_TRY(ctx, s->h_crc.reserve(size_t(n) * 4));
  HIP_TRY(ctx, s->h_ok.reserve(size_t(n) * 4));  // statuses
  HIP_TRY(ctx, s->h_bad.reserve(4));
  HIP_TRY(ctx, hipMemcpyAsync(s->d_desc.p, d, size_t(n) * sizeof(PacketDesc), hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(ctx, hipMemsetAsync(s->d_bad.p, 0, 4, ctx->stream));
  rc = packet_enqueue(ctx, mode, static_cast<const PacketDesc*>(s->d_desc.p), n, const_cast<uint8_t*>(d_base),
                      s->d_aux.p, static_cast<uint32_t*>(s->d_crc.p), static_cast<int32_t*>(s->d_ok.p),
                      static_cast<uint32_t*>(s->d_bad.p), ctx->stream);
  if (rc) return rc;
  HIP_TRY(ctx, hipMemcpyAsync(s->h_crc.p, s->d_crc.p, size_t(n) * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(s->h_ok.p, s->d_ok.p, size_t(n) * 4, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(s->h_bad.p, s->d_bad.p, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  const uint32_t* hc = static_cast<const uint32_t*>(s->h_crc.p);
  const int32_t* hs = static_cast<const int32_t*>(s->h_ok.p);
  if (out_crc) memcpy(out_crc, hc, size_t(n) * 4);
  if (out_status) memcpy(out_status, hs, size_t(n) * 4);
  const uint32_t bad = *static_cast<const uint32_t*>(s->h_bad.p);
  if (n_bad) *n_bad = bad;
  if (mode == 0) {
    // Seal: the device wrote the crc into its copy of each checked V1 header;
    // store the same four bytes into the caller's frames (the frames it checked:
    // the same header rules on the host bytes, packet_parse_host).
    uint8_t* hb = static_cast<uint8_t*>(base);
    for (uint32_t i = 0; i < n; ++i) {
      Desc x;
      int32_t pre;
      packet_parse_host(hb, d[i], mode, &x, &pre);
      if (pre != kPacketPending) continue;
      uint8_t* p = hb + d[i].offset;
      const uint32_t flag = uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
      if (flag != TFS_PACKET_FLAG_V1) continue;
      for (int b = 0; b < 4; ++b) p[TFS_PACKET_HEADER_V0_SIZE + 8 + b] = uint8_t(hc[i] >> (8 * b));
    }
    return TFS_SUCCESS;
  }
  return bad ? TFS_EXIT_CHECK_CRC_ERROR : TFS_SUCCESS;
}

int tfs_packet_verify(tfs_crc_ctx* ctx, const tfs_packet_desc* d, uint32_t n, const void* base, uint64_t base_len,
                      uint32_t* out_crc, int32_t* out_status, uint32_t* n_bad) {
  return packet_host(ctx, 1, d, n, const_cast<void*>(base), base_len, out_crc, out_status, n_bad);
}

int tfs_packet_seal(tfs_crc_ctx* ctx, const tfs_packet_desc* d, uint32_t n, void* base, uint64_t base_len,
                    uint32_t* out_crc, int32_t* out_status) {
  return packet_host(ctx, 0, d, n, base, base_len, out_crc, out_status, nullptr);
}

int tfs_packet_verify_device(tfs_crc_ctx* ctx, const tfs_packet_desc* d_desc, uint32_t n, const void* d_base,
                             uint32_t* d_out_crc, int32_t* d_out_status, uint32_t* d_n_bad, void* stream) {
  return packet_device(ctx, 1, d_desc, n, const_cast<void*>(d_base), d_out_crc, d_out_status, d_n_bad, stream);
}

int tfs_packet_seal_device(tfs_crc_ctx* ctx, const tfs_packet_desc* d_desc, uint32_t n, void* d_base,
                           uint32_t* d_out_crc, int32_t* d_out_status, void* stream) {
  return packet_device(ctx, 0, d_desc, n, d_base, d_out_crc, d_out_status, nullptr, stream);
}

// ---- test / bench helpers (not part of the dataserver boundary) ----------

int tfs_crc32_synth_fill_device(tfs_crc_ctx* ctx, void* d_dst, uint64_t nbytes, uint64_t seed, uint64_t first_word,
                                void* stream) {
  if (!ctx || !d_dst || (nbytes & 7)) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  HIP_TRY(ctx, launch_synth_fill(static_cast<uint64_t*>(d_dst), nbytes / 8, seed, first_word, st));
  return TFS_SUCCESS;
}

int tfs_crc32_write_headers_device(tfs_crc_ctx* ctx, void* d_image, const uint64_t* d_rec_off, const uint32_t* d_len,
                                   const uint32_t* d_crc, uint64_t first_id, uint32_t n, void* stream) {
  if (!ctx || !d_image) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  HIP_TRY(ctx, launch_write_headers(static_cast<uint8_t*>(d_image), d_rec_off, d_len, d_crc, first_id, n, st));
  return TFS_SUCCESS;
}

int tfs_crc32_write_packet_headers_device(tfs_crc_ctx* ctx, void* d_base, const uint64_t* d_frame_off,
                                          const uint32_t* d_body_len, uint32_t n, int32_t pcode, int32_t version,
                                          uint64_t first_id, void* stream) {
  if (!ctx || (n && (!d_base || !d_frame_off || !d_body_len))) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  HIP_TRY(ctx, launch_write_packet_headers(static_cast<uint8_t*>(d_base), d_frame_off, d_body_len, n, pcode, version,
                                           first_id, st));
  return TFS_SUCCESS;
}

int tfs_crc32_membench_device(tfs_crc_ctx* ctx, int pattern, const void* d_base, const tfs_crc_desc* d_desc,
                              uint32_t n, uint64_t nbytes, uint32_t* d_out, unsigned grid, void* stream) {
  if (!ctx || !d_base || !d_out) return TFS_EXIT_PARAMETER_ERROR;
#ifdef TFS_CRC_MEASURE
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  HIP_TRY(ctx, launch_membench(pattern, static_cast<const uint8_t*>(d_base), reinterpret_cast<const Desc*>(d_desc), n,
                               nbytes, d_out, grid, st));
  return TFS_SUCCESS;
#else
  (void)pattern, (void)d_desc, (void)n, (void)nbytes, (void)grid, (void)stream;
  return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "calibration kernels are in the measurement build only "
                 "(tfs_amd/libtfs_crc_measure.so)");
#endif
}

int tfs_crc32_dev_malloc(tfs_crc_ctx* ctx, uint64_t bytes, void** d_ptr) {
  if (!ctx || !d_ptr) return TFS_EXIT_PARAMETER_ERROR;
  *d_ptr = nullptr;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  // TFS_CRC_DEV_CONTIG=1 (measurement): physically contiguous memory, so the
  // page tables can map it with the largest fragments (fewer address-translation
  // misses for a scan over tens of GiB); ordinary memory when that fails.
  static const bool contig = [] {
    const char* v = getenv("TFS_CRC_DEV_CONTIG");
    return v && atoi(v) != 0;
  }();
  if (contig && bytes >= (64ull << 20)) {
    if (hipExtMallocWithFlags(d_ptr, bytes, hipDeviceMallocContiguous) == hipSuccess) return TFS_SUCCESS;
    (void)hipGetLastError();
    *d_ptr = nullptr;
  }
  HIP_TRY(ctx, hipMalloc(d_ptr, bytes ? bytes : 1));
  return TFS_SUCCESS;
}

int tfs_crc32_dev_free(tfs_crc_ctx* ctx, void* d_ptr) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  if (!d_ptr) return TFS_SUCCESS;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipFree(d_ptr));
  return TFS_SUCCESS;
}

int tfs_crc32_host_malloc_pinned(tfs_crc_ctx* ctx, uint64_t bytes, void** h_ptr) {
  if (!ctx || !h_ptr) return TFS_EXIT_PARAMETER_ERROR;
  *h_ptr = nullptr;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipHostMalloc(h_ptr, bytes ? bytes : 1, hipHostMallocDefault));
  void* dev = nullptr;
  if (hipHostGetDevicePointer(&dev, *h_ptr, 0) == hipSuccess) pin_register(*h_ptr, bytes ? bytes : 1, dev);
  else (void)hipGetLastError();
  return TFS_SUCCESS;
}

int tfs_crc32_host_free_pinned(tfs_crc_ctx* ctx, void* h_ptr) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  if (!h_ptr) return TFS_SUCCESS;
  pin_unregister(h_ptr);
  HIP_TRY(ctx, hipHostFree(h_ptr));
  return TFS_SUCCESS;
}

int tfs_crc32_host_device_ptr(tfs_crc_ctx* ctx, const void* h_ptr, void** d_ptr) {
  if (!ctx || !h_ptr || !d_ptr) return TFS_EXIT_PARAMETER_ERROR;
  *d_ptr = nullptr;
  if (pin_lookup(h_ptr, d_ptr)) return TFS_SUCCESS;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipHostGetDevicePointer(d_ptr, const_cast<void*>(h_ptr), 0));
  return TFS_SUCCESS;
}

int tfs_crc32_memcpy(tfs_crc_ctx* ctx, void* dst, const void* src, uint64_t bytes, void* stream) {
  if (!ctx || (bytes && (!dst || !src))) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if (bytes) HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, st));
  if (!stream) HIP_TRY(ctx, hipStreamSynchronize(st));
  return TFS_SUCCESS;
}

int tfs_crc32_memset_device(tfs_crc_ctx* ctx, void* d_ptr, int value, uint64_t bytes, void* stream) {
  if (!ctx || (bytes && !d_ptr)) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  if (bytes) HIP_TRY(ctx, hipMemsetAsync(d_ptr, value, bytes, st));
  return TFS_SUCCESS;
}

int tfs_crc32_event_create(tfs_crc_ctx* ctx, void** ev) {
  if (!ctx || !ev) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipEvent_t e;
  HIP_TRY(ctx, hipEventCreate(&e));
  *ev = e;
  return TFS_SUCCESS;
}

int tfs_crc32_event_record(tfs_crc_ctx* ctx, void* ev, void* stream) {
  if (!ctx || !ev) return TFS_EXIT_PARAMETER_ERROR;
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
  HIP_TRY(ctx, hipEventRecord(static_cast<hipEvent_t>(ev), st));
  return TFS_SUCCESS;
}

int tfs_crc32_event_elapsed_ms(tfs_crc_ctx* ctx, void* ev_start, void* ev_end, float* ms) {
  if (!ctx || !ev_start || !ev_end || !ms) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipEventSynchronize(static_cast<hipEvent_t>(ev_end)));
  HIP_TRY(ctx, hipEventElapsedTime(ms, static_cast<hipEvent_t>(ev_start), static_cast<hipEvent_t>(ev_end)));
  return TFS_SUCCESS;
}

int tfs_crc32_event_destroy(tfs_crc_ctx* ctx, void* ev) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  if (ev) HIP_TRY(ctx, hipEventDestroy(static_cast<hipEvent_t>(ev)));
  return TFS_SUCCESS;
}

void* tfs_crc32_stream(tfs_crc_ctx* ctx) { return ctx ? static_cast<void*>(ctx->stream) : nullptr; }

int tfs_crc32_sync(tfs_crc_ctx* ctx) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  // the zero-copy small batches launched on the latency stream
  HIP_TRY(ctx, hipStreamSynchronize(ctx->lat_stream));
  // and the wide in-place launches on the slots' own streams (round 6)
  std::vector<hipStream_t> wide;
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    for (const Slot& x : ctx->slots)
      if (x.wide_stream) wide.push_back(x.wide_stream);
    for (const Slot& x : ctx->sync_slots)
      if (x.wide_stream) wide.push_back(x.wide_stream);
  }
  for (hipStream_t w : wide) HIP_TRY(ctx, hipStreamSynchronize(w));
  return TFS_SUCCESS;
}

int tfs_crc32_inject_device_error(tfs_crc_ctx* ctx, uint32_t skip, uint32_t count) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  ctx->inject_count = 0;
  ctx->inject_skip = skip;
  ctx->inject_count = count;
  return TFS_SUCCESS;
}

int tfs_crc32_set_resident(tfs_crc_ctx* ctx, int on) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  std::lock_guard<std::mutex> g(ctx->mu);
  ctx->resident = on != 0;
  return TFS_SUCCESS;
}

int tfs_crc32_debug_state(tfs_crc_ctx* ctx, void** d_sched, uint64_t* sched_bytes, void** d_res_state,
                          uint64_t* res_state_bytes) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (d_sched) *d_sched = ctx->d_sched;
  if (sched_bytes) *sched_bytes = uint64_t(kSchedSlots) * kSchedSlotBytes;
  if (d_res_state) *d_res_state = ctx->res_state;
  if (res_state_bytes) *res_state_bytes = kResStateBytes;
  return TFS_SUCCESS;
}

int tfs_crc32_debug_poison_resident(tfs_crc_ctx* ctx, uint32_t done) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  std::lock_guard<std::mutex> g(ctx->mu);
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  if (const int rc = resident_setup(ctx)) return rc;
  if (ctx->res_running) {  // only between lifetimes: a live kernel owns its lines
    const hipError_t e = hipEventQuery(ctx->res_event);
    if (e == hipErrorNotReady) return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "resident kernel is running");
  }
  std::vector<uint32_t> lines(size_t(kResMaxGrid) * kSchedStride, 0u);
  for (uint32_t w = 0; w < kResMaxGrid; ++w) lines[size_t(w) * kSchedStride] = done;
  HIP_TRY(ctx, hipMemcpyAsync(ctx->res_state, lines.data(), lines.size() * 4, hipMemcpyHostToDevice, ctx->res_stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->res_stream));
  return TFS_SUCCESS;
}

int tfs_crc32_set_cu_reserve(tfs_crc_ctx* ctx, int on) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  ctx->cu_reserve.store(on != 0, std::memory_order_relaxed);
  return TFS_SUCCESS;
}

int tfs_crc32_set_split(tfs_crc_ctx* ctx, int on) {
  if (!ctx || on < 0 || on > 1) return TFS_EXIT_PARAMETER_ERROR;
  ctx->split_files.store(on, std::memory_order_relaxed);
  return TFS_SUCCESS;
}

int tfs_crc32_set_compact_segment(tfs_crc_ctx* ctx, uint32_t seg_bytes) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  if (seg_bytes == 1u) {  // back to the default rule
    ctx->cseg_auto.store(true, std::memory_order_relaxed);
    return TFS_SUCCESS;
  }
  uint32_t lg = 0;
  if (seg_bytes == 8192u) lg = 3;
  else if (seg_bytes == 16384u) lg = 4;
  else if (seg_bytes == 32768u) lg = 5;
  else if (seg_bytes != 0u) return TFS_EXIT_PARAMETER_ERROR;
  ctx->cseg_lg.store(lg, std::memory_order_relaxed);
  ctx->cseg_auto.store(false, std::memory_order_relaxed);
  return TFS_SUCCESS;
}

int tfs_crc32_split_stats(tfs_crc_ctx* ctx, uint64_t* launches, uint64_t* used, uint32_t* files, uint32_t* cap,
                          uint32_t* grid) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  int k;
  uint32_t n, c, g;
  uint64_t nl;
  {
    std::lock_guard<std::mutex> lg(ctx->last_split_mu);
    k = ctx->last_split_slot;
    n = ctx->last_split_n;
    c = ctx->last_split_cap;
    g = ctx->last_split_grid;
    nl = ctx->split_launches;
  }
  uint64_t u = 0;
  if (k >= 0) {
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    std::lock_guard<std::mutex> pg(ctx->plan_mu[k]);
    if (!ctx->plan_done[k]) return set_err(ctx, TFS_CRC_EXIT_DEVICE_ERROR, "split_stats: no event behind the plan");
    HIP_TRY(ctx, hipEventSynchronize(ctx->plan_done[k]));
    uint32_t hdr[4] = {0u, 0u, 0u, 0u};  // {units, nosplit, ext, cut}
    HIP_TRY(ctx, hipMemcpy(hdr, ctx->plans[k].p, 16, hipMemcpyDeviceToHost));
    u = hdr[1] ? 0u : hdr[2];
  }
  if (launches) *launches = nl;
  if (used) *used = u;
  if (files) *files = n;
  if (cap) *cap = c;
  if (grid) *grid = g;
  return TFS_SUCCESS;
}

int tfs_crc32_plan_stats(tfs_crc_ctx* ctx, uint32_t* plans, uint64_t* bytes) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  uint32_t np = 0;
  uint64_t nb = 0;
  for (uint32_t k = 0; k < kSchedSlots; ++k) {
    std::lock_guard<std::mutex> g(ctx->plan_mu[k]);
    if (ctx->plans[k].p) {
      ++np;
      nb += ctx->plans[k].cap;
    }
  }
  if (plans) *plans = np;
  if (bytes) *bytes = nb;
  return TFS_SUCCESS;
}

int tfs_crc32_throughput_grid(tfs_crc_ctx* ctx) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  return int(throughput_cap(ctx));
}

int tfs_crc32_sched_stats(tfs_crc_ctx* ctx, uint32_t* owned_streams, uint64_t* foreign_launches) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  std::lock_guard<std::mutex> g(ctx->sched_mu);
  uint32_t k = 0;
  for (hipStream_t st : ctx->sched_streams) k += st ? 1u : 0u;
  if (owned_streams) *owned_streams = k;
  if (foreign_launches) *foreign_launches = ctx->foreign_launches;
  return TFS_SUCCESS;
}

int tfs_crc32_res_trace(tfs_crc_ctx* ctx, void* pinned) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
#ifdef TFS_CRC_MEASURE
  std::lock_guard<std::mutex> g(ctx->mu);
  if (ctx->res_running) return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "res_trace: set it before the first resident call");
  void* dev = nullptr;
  if (pinned && !host_dev_ptr(pinned, &dev)) return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "res_trace: not page-locked");
  ctx->res_trace_dev = static_cast<uint64_t*>(dev);
  HIP_TRY(ctx, hipDeviceGetAttribute(&ctx->tr_khz, hipDeviceAttributeWallClockRate, ctx->device));
  // TFS_CRC_RES_FENCE=1: the resident kernel also fences before each payload read
  // over PCIe, as it did before its system-coherent loads (the A/B of round 6)
  const char* fe = getenv("TFS_CRC_RES_FENCE");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, set_res_fence(fe && atoi(fe) ? 1u : 0u));
  return TFS_SUCCESS;
#else
  (void)pinned;
  return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "res_trace: measurement build only (libtfs_crc_measure.so)");
#endif
}

int tfs_crc32_res_trace_last(tfs_crc_ctx* ctx, uint64_t* out) {
  if (!ctx || !out) return TFS_EXIT_PARAMETER_ERROR;
#ifdef TFS_CRC_MEASURE
  out[0] = uint64_t(ctx->tr_enter.load());
  out[1] = uint64_t(ctx->tr_posted.load());
  out[2] = uint64_t(ctx->tr_seen.load());
  out[3] = uint64_t(ctx->tr_done.load());
  out[4] = ctx->tr_first.load();
  out[5] = ctx->tr_resident.load();
  out[6] = uint64_t(ctx->tr_khz);
  out[7] = 0;
  return TFS_SUCCESS;
#else
  return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "res_trace_last: measurement build only (libtfs_crc_measure.so)");
#endif
}

int tfs_crc32_stats(tfs_crc_ctx* ctx, tfs_crc_stats* out) {
  if (!ctx || !out) return TFS_EXIT_PARAMETER_ERROR;
  memset(out, 0, sizeof *out);
  out->host_calls = ctx->st_calls.load(std::memory_order_relaxed);
  out->host_files = ctx->st_files.load(std::memory_order_relaxed);
  out->lone_calls = ctx->st_lone.load(std::memory_order_relaxed);
  out->lone_small_calls = ctx->st_lone_small.load(std::memory_order_relaxed);
  out->lone_small_bytes = ctx->st_lone_small_bytes.load(std::memory_order_relaxed);
  std::lock_guard<std::mutex> g(ctx->mu);
  out->resident_launches = ctx->res_launches;
  out->resident_files = ctx->res_files;
  out->resident_ring_full = ctx->res_ring_full;
  return TFS_SUCCESS;
}

int tfs_crc32_resident_stats(tfs_crc_ctx* ctx, uint64_t* launches, uint64_t* files) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (launches) *launches = ctx->res_launches;
  if (files) *files = ctx->res_files;
  return TFS_SUCCESS;
}

int tfs_crc32_resident_ring_in_device_memory(tfs_crc_ctx* ctx) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!ctx->res_host) return -1;
  return ctx->res_vram ? 1 : 0;
}

int tfs_crc32_stream_create(tfs_crc_ctx* ctx, void** stream) {
  if (!ctx || !stream) return TFS_EXIT_PARAMETER_ERROR;
  *stream = nullptr;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  hipStream_t st = nullptr;
  HIP_TRY(ctx, hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  if (bind_owned_stream(ctx, st) != hipSuccess) {
    (void)hipStreamDestroy(st);
    return set_err(ctx, TFS_EXIT_PARAMETER_ERROR, "more than %u live streams on one context", kOwnedSlots);
  }
  *stream = st;
  return TFS_SUCCESS;
}

int tfs_crc32_stream_sync(tfs_crc_ctx* ctx, void* stream) {
  if (!ctx) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipStreamSynchronize(stream ? static_cast<hipStream_t>(stream) : ctx->stream));
  return TFS_SUCCESS;
}

int tfs_crc32_stream_destroy(tfs_crc_ctx* ctx, void* stream) {
  if (!ctx || !stream || stream == ctx->stream || stream == ctx->lat_stream) return TFS_EXIT_PARAMETER_ERROR;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  {
    // Its scheduler slot is zero (every launch leaves it so, a failed one is
    // zeroed again) and may be rebound.
    std::lock_guard<std::mutex> g(ctx->sched_mu);
    for (auto& s : ctx->sched_streams)
      if (s == static_cast<hipStream_t>(stream)) s = nullptr;
  }
  HIP_TRY(ctx, hipStreamDestroy(static_cast<hipStream_t>(stream)));
  return TFS_SUCCESS;
}

}  // extern "C"
