// ds_capi.cpp -- C entry points over the dataserver-shaped harness, so tests
// can drive the write / close / verify / compact call sites the way the
// reference's gtest programs drive LogicBlock/DataFile directly
// (tests/dataserver/test_logic_block_and_compact.cpp).  Host C++ only.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ds_harness.h"

using namespace tfs::dataserver;

extern "C" {

void* tfs_ds_datafile_new(tfs_crc_ctx* ctx, uint64_t fn, const char* tmp_dir) {
  return new DataFile(fn, tmp_dir ? tmp_dir : "/tmp", ctx);
}
// The same with its buffer from a LeaseBufferPool (tfs_ds_lease_pool_new; the heap
// when the pool is exhausted or NULL).
void* tfs_ds_datafile_new2(tfs_crc_ctx* ctx, uint64_t fn, const char* tmp_dir, void* pool) {
  return new DataFile(fn, tmp_dir ? tmp_dir : "/tmp", ctx, static_cast<LeaseBufferPool*>(pool));
}
int tfs_ds_datafile_pooled(void* df) { return static_cast<DataFile*>(df)->pool() != nullptr; }
void tfs_ds_datafile_free(void* df) { delete static_cast<DataFile*>(df); }
int tfs_ds_datafile_set_data(void* df, const char* data, int32_t len, int32_t offset) {
  return static_cast<DataFile*>(df)->set_data(data, len, offset);
}
int32_t tfs_ds_datafile_length(void* df) { return static_cast<DataFile*>(df)->get_length(); }
uint32_t tfs_ds_datafile_get_crc(void* df, int* status) {
  DataFile* d = static_cast<DataFile*>(df);
  const uint32_t c = d->get_crc();
  if (status) *status = d->last_status();
  return c;
}

void* tfs_ds_block_new(uint32_t block_id, int64_t capacity) { return new LogicBlockImage(block_id, capacity); }
// Page-locked block buffers lent to LogicBlockImages (a dataserver's preallocated blocks).
void* tfs_ds_pool_new(tfs_crc_ctx* ctx, uint32_t count, uint64_t bytes) {
  return new BlockImagePool(ctx, count, size_t(bytes));
}
void tfs_ds_pool_free(void* pool) { delete static_cast<BlockImagePool*>(pool); }
uint32_t tfs_ds_pool_in_use(void* pool) { return uint32_t(static_cast<BlockImagePool*>(pool)->in_use()); }
uint32_t tfs_ds_pool_size(void* pool) { return uint32_t(static_cast<BlockImagePool*>(pool)->size()); }
void* tfs_ds_block_new_in(void* pool, uint32_t block_id, int64_t capacity) {
  return new LogicBlockImage(block_id, capacity, pool ? static_cast<BlockImagePool*>(pool)->take() : nullptr);
}
void tfs_ds_block_free(void* b) { delete static_cast<LogicBlockImage*>(b); }
int64_t tfs_ds_block_size(void* b) { return static_cast<LogicBlockImage*>(b)->data_size(); }
const char* tfs_ds_block_data(void* b) { return static_cast<LogicBlockImage*>(b)->data().data(); }
int tfs_ds_block_set_flag(void* b, uint64_t file_id, int32_t flag) {
  return static_cast<LogicBlockImage*>(b)->set_flag(file_id, flag);
}
int tfs_ds_block_corrupt(void* b, int64_t offset, uint8_t xor_mask) {
  auto& d = static_cast<LogicBlockImage*>(b)->data();
  if (offset < 0 || offset >= int64_t(d.size())) return TFS_EXIT_PARAMETER_ERROR;
  d[size_t(offset)] = char(uint8_t(d[size_t(offset)]) ^ xor_mask);
  return TFS_SUCCESS;
}
int tfs_ds_block_metas(void* b, tfs_raw_meta* out, int32_t* flags, uint32_t cap) {
  const auto m = static_cast<LogicBlockImage*>(b)->sorted_metas();
  const auto f = static_cast<LogicBlockImage*>(b)->sorted_flags();
  for (size_t i = 0; i < m.size() && i < cap; ++i) {
    out[i] = m[i];
    if (flags) flags[i] = f[i];
  }
  return int(m.size());
}

int tfs_ds_close_write_file(void* block, uint64_t file_id, uint32_t client_crc, void* df) {
  CloseFileInfo info;
  info.block_id_ = static_cast<LogicBlockImage*>(block)->block_id();
  info.file_id_ = file_id;
  info.crc_ = client_crc;
  return close_write_file(info, *static_cast<DataFile*>(df), *static_cast<LogicBlockImage*>(block));
}

void* tfs_ds_batcher_new(tfs_crc_ctx* ctx, uint32_t max_batch, int max_wait_us) {
  return new CloseBatcher(ctx, max_batch, max_wait_us);
}
// in_flight: batches in use at once (1..16; the constructor's default is 8).
void* tfs_ds_batcher_new2(tfs_crc_ctx* ctx, uint32_t max_batch, int max_wait_us, int in_flight) {
  return new CloseBatcher(ctx, max_batch, max_wait_us, in_flight);
}
// pool (a tfs_ds_lease_pool_new handle, may be NULL): closes of DataFiles made
// on it are checked where their payload is, with no gather copy.
void* tfs_ds_batcher_new3(tfs_crc_ctx* ctx, uint32_t max_batch, int max_wait_us, int in_flight, void* pool) {
  return new CloseBatcher(ctx, max_batch, max_wait_us, in_flight, static_cast<LeaseBufferPool*>(pool));
}
void* tfs_ds_batcher_pool(void* b) { return static_cast<CloseBatcher*>(b)->pool(); }

// Page-locked DataFile buffers (LeaseBufferPool); NULL when the allocation fails.
void* tfs_ds_lease_pool_new(tfs_crc_ctx* ctx, uint32_t nbuffers) {
  std::unique_ptr<LeaseBufferPool> p(new LeaseBufferPool(ctx, nbuffers));
  return p->ok() ? p.release() : nullptr;
}
void tfs_ds_lease_pool_free(void* p) { delete static_cast<LeaseBufferPool*>(p); }
uint32_t tfs_ds_lease_pool_in_use(void* p) { return static_cast<LeaseBufferPool*>(p)->in_use(); }
void tfs_ds_batcher_free(void* b) { delete static_cast<CloseBatcher*>(b); }
uint64_t tfs_ds_batcher_batches(void* b) { return static_cast<CloseBatcher*>(b)->batches(); }
int tfs_ds_batcher_close(void* batcher, void* block, uint64_t file_id, uint32_t client_crc, void* df) {
  CloseFileInfo info;
  info.block_id_ = static_cast<LogicBlockImage*>(block)->block_id();
  info.file_id_ = file_id;
  info.crc_ = client_crc;
  return static_cast<CloseBatcher*>(batcher)->close(info, *static_cast<DataFile*>(df),
                                                    *static_cast<LogicBlockImage*>(block));
}

void* tfs_ds_checker_new(int max_crc_error_nums) { return new BlockCrcChecker(max_crc_error_nums); }
void tfs_ds_checker_free(void* c) { delete static_cast<BlockCrcChecker*>(c); }
int tfs_ds_checker_errors(void* c, uint32_t block_id) { return static_cast<BlockCrcChecker*>(c)->crc_errors(block_id); }
int tfs_ds_checker_needs_repair(void* c, uint32_t block_id) {
  return static_cast<BlockCrcChecker*>(c)->needs_repair(block_id) ? 1 : 0;
}

int tfs_ds_verify_block(tfs_crc_ctx* ctx, void* block, int32_t* status, uint32_t cap, void* checker) {
  std::vector<int32_t> st;
  const int r = verify_block(ctx, *static_cast<LogicBlockImage*>(block), &st, static_cast<BlockCrcChecker*>(checker));
  for (size_t i = 0; i < st.size() && i < cap; ++i) status[i] = st[i];
  return r;
}

int tfs_ds_recombine_block(tfs_crc_ctx* ctx, void* src, void* dest, int* skipped_crc) {
  return recombine_block(ctx, *static_cast<LogicBlockImage*>(src), *static_cast<LogicBlockImage*>(dest), skipped_crc);
}

// LogicBlock::read_file (logic_block.cpp:374-440) into buf; *nbytes in/out.
int tfs_ds_block_read_file(void* b, uint64_t file_id, char* buf, int32_t* nbytes, int32_t offset, int force) {
  return static_cast<LogicBlockImage*>(b)->read_file(file_id, buf, nbytes, offset, force != 0);
}

// read_data of a whole file + the GPU verify-on-read hook; FileInfo|payload into buf (cap bytes).
int tfs_ds_read_file_verified(tfs_crc_ctx* ctx, void* block, uint64_t file_id, char* buf, int32_t cap, int32_t* len,
                              void* checker) {
  std::vector<char> out;
  const int rc = read_file_verified(ctx, *static_cast<LogicBlockImage*>(block), file_id, &out,
                                    static_cast<BlockCrcChecker*>(checker));
  *len = int32_t(out.size());
  if (buf && !out.empty()) memcpy(buf, out.data(), std::min(out.size(), size_t(cap > 0 ? cap : 0)));
  return rc;
}

int tfs_ds_compact_block(tfs_crc_ctx* ctx, void* src, void* dest, uint8_t* crc_ok, uint32_t cap) {
  std::vector<uint8_t> ok;
  const int r = compact_block(ctx, *static_cast<LogicBlockImage*>(src), *static_cast<LogicBlockImage*>(dest), &ok);
  for (size_t i = 0; i < ok.size() && i < cap; ++i) crc_ok[i] = ok[i];
  return r;
}

// BASELINE.json configs[0] through the dataserver-shaped code: n payloads of
// `len` bytes written into `block` by `nthreads` worker threads (DataService's
// PacketQueueThreads, base_service.cpp:187-192).  Per file: DataFile::set_data
// (the staging memcpy, data_file.cpp:104), then close through the CloseBatcher
// (one GPU verify of every pending lease's client CRC, data_management.cpp:
// 196-198, then FileInfo|payload appended, logic_block.cpp:171-178).  Then
// verify-on-read of the whole block (sync_backup.cpp:383-429).  Returns the
// number of files that failed either check, or a negative status.
int tfs_ds_loopback_block_with(tfs_crc_ctx* ctx, void* batcher, const char* payloads, uint32_t n, int32_t len,
                               const uint32_t* client_crc, int nthreads, void* block);
int tfs_ds_loopback_block(tfs_crc_ctx* ctx, const char* payloads, uint32_t n, int32_t len, const uint32_t* client_crc,
                          int nthreads, void* block) {
  return tfs_ds_loopback_block_with(ctx, nullptr, payloads, n, len, client_crc, nthreads, block);
}

// The same with a long-lived CloseBatcher (DataService creates it once, at
// initialize); NULL = one for this call.
int tfs_ds_loopback_block_with(tfs_crc_ctx* ctx, void* batcher, const char* payloads, uint32_t n, int32_t len,
                               const uint32_t* client_crc, int nthreads, void* block) {
  if (!ctx || !block || len < 0 || (n && (!payloads || !client_crc))) return TFS_EXIT_PARAMETER_ERROR;
  LogicBlockImage& blk = *static_cast<LogicBlockImage*>(block);
  if (nthreads < 1) nthreads = 1;
  blk.reserve(blk.data_size() + int64_t(n) * (int64_t(len) + TFS_FILEINFO_SIZE));
  std::atomic<int> bad{0}, err{0};
  // TFS_DS_TRACE=1: per-phase thread-time totals on stderr (diagnostics only)
  const bool trace = getenv("TFS_DS_TRACE") != nullptr;
  std::atomic<int64_t> t_new{0}, t_set{0}, t_close{0}, t_free{0};
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto us = [](auto a, auto b) { return int64_t(std::chrono::duration_cast<std::chrono::microseconds>(b - a).count()); };
  const auto t_begin = now();
  {
    std::unique_ptr<CloseBatcher> own;
    if (!batcher) own.reset(new CloseBatcher(ctx, CloseBatcher::batch_for(size_t(nthreads)), 100));
    CloseBatcher& bat = batcher ? *static_cast<CloseBatcher*>(batcher) : *own;
    std::vector<std::thread> workers;
    for (int t = 0; t < nthreads; ++t)
      workers.emplace_back([&, t] {
        for (uint32_t i = uint32_t(t); i < n; i += uint32_t(nthreads)) {
          const auto t0 = now();
          std::unique_ptr<DataFile> df(new DataFile(i + 1, "/tmp", ctx, bat.pool()));
          const auto t1 = now();
          if (df->set_data(payloads + size_t(i) * size_t(len), len, 0) < 0) {
            err = TFS_EXIT_PARAMETER_ERROR;
            continue;
          }
          const auto t2 = now();
          CloseFileInfo info;
          info.block_id_ = blk.block_id();
          info.file_id_ = i + 1;
          info.crc_ = client_crc[i];
          const int rc = bat.close(info, *df, blk);
          const auto t3 = now();
          df.reset();
          if (trace) {
            t_new += us(t0, t1);
            t_set += us(t1, t2);
            t_close += us(t2, t3);
            t_free += us(t3, now());
          }
          if (rc == TFS_EXIT_DATA_FILE_ERROR) ++bad;
          else if (rc != TFS_SUCCESS) err = rc;
        }
      });
    for (auto& w : workers) w.join();
  }
  if (err.load() != 0) return err.load();
  const auto t_writes = now();
  const int nb = verify_block(ctx, blk, nullptr, nullptr);
  if (trace)
    fprintf(stderr, "loopback trace: writes %lld us wall, verify %lld us; thread-us new %lld set %lld close %lld free %lld\n",
            (long long)us(t_begin, t_writes), (long long)us(t_writes, now()), (long long)t_new.load(),
            (long long)t_set.load(), (long long)t_close.load(), (long long)t_free.load());
  return nb < 0 ? nb : bad.load() + nb;
}

// ---- write-path latency (SURVEY §7 "Batching vs. latency") ------------------

// Per-close latency of DataManagement::close_write_file through the CloseBatcher:
// `nleases` worker threads (concurrent leases) each close `iters` files of `len`
// bytes; a close is timed from the call to its return (GPU check of the client
// CRC + FileInfo|payload append).  out_us receives nleases*iters microseconds.
// out_phase (may be NULL): kClosePhases doubles per close, in out_us's order --
// CloseTiming's claim, copy, wait, append, lead_wait, verify (us), leader,
// batch_n, relaunches, ring_full.
constexpr int kClosePhases = 10;
int tfs_ds_close_latency_phases(tfs_crc_ctx* ctx, int nleases, int iters, int32_t len, double* out_us,
                                double* out_phase) {
  if (!ctx || nleases < 1 || iters < 1 || len < 0 || !out_us) return TFS_EXIT_PARAMETER_ERROR;
  std::vector<char> payload(size_t(len) + 1);
  for (int32_t i = 0; i < len; ++i) payload[size_t(i)] = char((i * 2654435761u) >> 11);
  uint32_t client = 0;
  int rc = tfs_datafile_get_crc(ctx, payload.data(), len, &client);  // the client's Func::crc
  if (rc != TFS_SUCCESS) return rc;
  LogicBlockImage blk(1, int64_t(INT32_MAX));
  constexpr int kWarm = 8;  // untimed closes per lease first: steady state, not first-use allocations
  const int64_t total = int64_t(nleases) * (iters + kWarm) * (int64_t(len) + TFS_FILEINFO_SIZE);
  if (total > int64_t(INT32_MAX)) return TFS_EXIT_PARAMETER_ERROR;
  blk.reserve(total);
  std::atomic<int> err{0};
  {
    CloseBatcher batcher(ctx, CloseBatcher::batch_for(size_t(nleases)), 100);
    std::vector<std::thread> workers;
    for (int t = 0; t < nleases; ++t)
      workers.emplace_back([&, t] {
        for (int k = -kWarm; k < iters; ++k) {
          const uint64_t fid = uint64_t(t) * uint64_t(iters + kWarm) + uint64_t(k + kWarm) + 1;
          DataFile df(fid, "/tmp", ctx);
          df.set_data(payload.data(), len, 0);
          CloseFileInfo info;
          info.block_id_ = 1;
          info.file_id_ = fid;
          info.crc_ = client;
          CloseTiming ph;
          const auto t0 = std::chrono::steady_clock::now();
          const int r = batcher.close(info, df, blk, out_phase ? &ph : nullptr);
          const auto t1 = std::chrono::steady_clock::now();
          const size_t at = size_t(t) * size_t(iters) + size_t(k);
          if (k >= 0) out_us[at] = std::chrono::duration<double, std::micro>(t1 - t0).count();
          if (k >= 0 && out_phase) {
            double* o = out_phase + at * kClosePhases;
            o[0] = ph.claim_us, o[1] = ph.copy_us, o[2] = ph.wait_us, o[3] = ph.append_us;
            o[4] = ph.lead_wait_us, o[5] = ph.verify_us, o[6] = ph.leader, o[7] = ph.batch_n;
            o[8] = ph.relaunches, o[9] = ph.ring_full;
          }
          if (r != TFS_SUCCESS) err = r;
        }
      });
    for (auto& w : workers) w.join();
  }
  return err.load();
}

int tfs_ds_close_latency(tfs_crc_ctx* ctx, int nleases, int iters, int32_t len, double* out_us) {
  return tfs_ds_close_latency_phases(ctx, nleases, iters, len, out_us, nullptr);
}

// A stream of closes (DataManagement::close_write_file, data_management.cpp:
// 173-236) from `nleases` worker threads through one CloseBatcher, running until
// *stop is set: the dataserver's packet workers closing 64 KiB writes while a
// throughput launch (a compaction on the task thread, dataservice.cpp:2915-2918,
// or a block verify) runs on the same GPU.  Each thread appends to a block of its
// own, replaced when full.  Latencies of up to `cap` closes (in completion order
// per thread, threads interleaved by slot) go to out_us; *count = closes done.
int tfs_ds_close_stream(tfs_crc_ctx* ctx, int nleases, int32_t len, const volatile int* stop, double* out_us,
                        uint64_t cap, uint64_t* count) {
  if (!ctx || nleases < 1 || len < 0 || !stop || !count) return TFS_EXIT_PARAMETER_ERROR;
  std::vector<char> payload(size_t(len) + 1);
  for (int32_t i = 0; i < len; ++i) payload[size_t(i)] = char((i * 2654435761u) >> 13);
  uint32_t client = 0;
  int rc = tfs_datafile_get_crc(ctx, payload.data(), len, &client);
  if (rc != TFS_SUCCESS) return rc;
  constexpr int64_t kBlockBytes = 64ll << 20;
  const int64_t per_block = std::max<int64_t>(1, kBlockBytes / (int64_t(len) + TFS_FILEINFO_SIZE));
  std::atomic<int> err{0};
  std::atomic<uint64_t> done{0};
  {
    CloseBatcher batcher(ctx, CloseBatcher::batch_for(size_t(nleases)), 100);
    std::vector<std::thread> workers;
    for (int t = 0; t < nleases; ++t)
      workers.emplace_back([&, t] {
        std::unique_ptr<LogicBlockImage> blk;
        int64_t in_blk = per_block;
        for (uint64_t k = 0; !*stop && err.load() == TFS_SUCCESS; ++k) {
          if (in_blk == per_block) {
            blk.reset(new LogicBlockImage(uint32_t(t + 1), kBlockBytes));
            blk->reserve(kBlockBytes);
            in_blk = 0;
          }
          ++in_blk;
          const uint64_t fid = k + 1;
          DataFile df(fid, "/tmp", ctx);
          df.set_data(payload.data(), len, 0);
          CloseFileInfo info;
          info.block_id_ = uint32_t(t + 1);
          info.file_id_ = fid;
          info.crc_ = client;
          const auto t0 = std::chrono::steady_clock::now();
          const int r = batcher.close(info, df, *blk);
          const auto t1 = std::chrono::steady_clock::now();
          const uint64_t slot = k * uint64_t(nleases) + uint64_t(t);
          if (out_us && slot < cap) out_us[slot] = std::chrono::duration<double, std::micro>(t1 - t0).count();
          if (r != TFS_SUCCESS) err = r;
          done.fetch_add(1);
        }
      });
    for (auto& w : workers) w.join();
  }
  *count = done.load();
  return err.load();
}

// The scalar drop-in: tfs_crc32(0, data, len) on a pageable buffer, timed per call.
int tfs_ds_scalar_latency(int iters, int32_t len, double* out_us) {
  if (iters < 1 || len < 0 || !out_us) return TFS_EXIT_PARAMETER_ERROR;
  std::vector<char> payload(size_t(len) + 1);
  for (int32_t i = 0; i < len; ++i) payload[size_t(i)] = char((i * 40503u) >> 5);
  int err = TFS_SUCCESS;
  for (int k = 0; k < 8 && err == TFS_SUCCESS; ++k) (void)tfs_crc32_e(0, payload.data(), len, &err);  // untimed
  for (int k = 0; k < iters; ++k) {
    const auto t0 = std::chrono::steady_clock::now();
    (void)tfs_crc32_e(0, payload.data(), len, &err);
    const auto t1 = std::chrono::steady_clock::now();
    out_us[k] = std::chrono::duration<double, std::micro>(t1 - t0).count();
    if (err != TFS_SUCCESS) return err;
  }
  return TFS_SUCCESS;
}

// ---- multi-GPU service (CrcService over a tfs_crc_group) --------------------

void* tfs_ds_service_new(tfs_crc_group* group, uint32_t max_batch, int max_wait_us) {
  return group ? new CrcService(group, max_batch, max_wait_us) : nullptr;
}
void tfs_ds_service_free(void* s) { delete static_cast<CrcService*>(s); }
tfs_crc_ctx* tfs_ds_service_ctx_for_block(void* s, uint32_t block_id) {
  return static_cast<CrcService*>(s)->ctx_for_block(block_id);
}
int tfs_ds_service_close(void* s, void* block, uint64_t file_id, uint32_t client_crc, void* df) {
  CloseFileInfo info;
  info.block_id_ = static_cast<LogicBlockImage*>(block)->block_id();
  info.file_id_ = file_id;
  info.crc_ = client_crc;
  return static_cast<CrcService*>(s)->close_write_file(info, *static_cast<DataFile*>(df),
                                                       *static_cast<LogicBlockImage*>(block));
}
int tfs_ds_service_verify_blocks(void* s, void** blocks, uint32_t n, uint32_t* nbad) {
  std::vector<const LogicBlockImage*> b(n);
  for (uint32_t i = 0; i < n; ++i) b[i] = static_cast<const LogicBlockImage*>(blocks[i]);
  std::vector<uint32_t> nb;
  const int rc = static_cast<CrcService*>(s)->verify_blocks(b, &nb);
  for (uint32_t i = 0; nbad && i < n; ++i) nbad[i] = nb[i];
  return rc;
}

// BASELINE configs[0]'s loop over several blocks on a multi-GPU node: worker
// threads write file k of block b (block ids blocks[b]->block_id()) through a
// DataFile on that block's GPU and close it through the service (routed by
// block id), then every block is verified on its GPU, members concurrently.
// Returns the number of files that failed either check, or a negative status.
int tfs_ds_service_loopback(void* service, const char* payloads, uint32_t nblocks, uint32_t files_per_block,
                            int32_t len, const uint32_t* client_crc, int nthreads, void** blocks) {
  auto* svc = static_cast<CrcService*>(service);
  if (!svc || !blocks || len < 0) return TFS_EXIT_PARAMETER_ERROR;
  if (nthreads < 1) nthreads = 1;
  const uint32_t n = nblocks * files_per_block;
  for (uint32_t b = 0; b < nblocks; ++b) {
    auto* blk = static_cast<LogicBlockImage*>(blocks[b]);
    blk->reserve(blk->data_size() + int64_t(files_per_block) * (int64_t(len) + TFS_FILEINFO_SIZE));
  }
  std::atomic<int> bad{0}, err{0};
  std::vector<std::thread> workers;
  for (int t = 0; t < nthreads; ++t)
    workers.emplace_back([&, t] {
      for (uint32_t i = uint32_t(t); i < n; i += uint32_t(nthreads)) {
        auto* blk = static_cast<LogicBlockImage*>(blocks[i % nblocks]);
        DataFile df(i + 1, "/tmp", svc->ctx_for_block(blk->block_id()));
        if (df.set_data(payloads + size_t(i) * size_t(len), len, 0) < 0) {
          err = TFS_EXIT_PARAMETER_ERROR;
          continue;
        }
        CloseFileInfo info;
        info.block_id_ = blk->block_id();
        info.file_id_ = i + 1;
        info.crc_ = client_crc[i];
        const int rc = svc->close_write_file(info, df, *blk);
        if (rc == TFS_EXIT_DATA_FILE_ERROR) ++bad;
        else if (rc != TFS_SUCCESS) err = rc;
      }
    });
  for (auto& w : workers) w.join();
  if (err.load() != 0) return err.load();
  std::vector<const LogicBlockImage*> all(nblocks);
  for (uint32_t b = 0; b < nblocks; ++b) all[b] = static_cast<const LogicBlockImage*>(blocks[b]);
  std::vector<uint32_t> nb;
  const int rc = svc->verify_blocks(all, &nb);
  if (rc != TFS_SUCCESS && rc != TFS_EXIT_CHECK_CRC_ERROR) return rc;
  int total = bad.load();
  for (uint32_t x : nb) total += int(x);
  return total;
}

}  // extern "C"

// ---- packet codec (packet_codec.h) ----------------------------------------
#include "packet_codec.h"

extern "C" {

void* tfs_ds_encoder_new(tfs_crc_ctx* ctx) { return new tfs::common::PacketEncoder(ctx); }
void tfs_ds_encoder_free(void* e) { delete static_cast<tfs::common::PacketEncoder*>(e); }
void tfs_ds_encoder_add(void* e, int16_t pcode, int16_t version, uint64_t id, const char* body, int32_t len) {
  static_cast<tfs::common::PacketEncoder*>(e)->add(pcode, version, id, body, len);
}
int tfs_ds_encoder_flush(void* e) { return static_cast<tfs::common::PacketEncoder*>(e)->flush(); }
int64_t tfs_ds_encoder_size(void* e) { return int64_t(static_cast<tfs::common::PacketEncoder*>(e)->output().size()); }
const char* tfs_ds_encoder_data(void* e) { return static_cast<tfs::common::PacketEncoder*>(e)->output().data(); }

// Decode a received buffer: per frame offset/status/crc (cap entries), *nframes, *consumed.
int tfs_ds_decode(tfs_crc_ctx* ctx, const char* data, int64_t len, int64_t* offsets, int32_t* status, uint32_t* crc,
                  uint32_t cap, uint32_t* nframes, int64_t* consumed) {
  tfs::common::PacketDecoder dec(ctx);
  std::vector<tfs::common::PacketDecoder::Frame> fr;
  const int rc = dec.decode(data, len, &fr, consumed);
  *nframes = uint32_t(fr.size());
  for (size_t i = 0; i < fr.size() && i < cap; ++i) {
    if (offsets) offsets[i] = fr[i].offset;
    if (status) status[i] = fr[i].status;
    if (crc) crc[i] = fr[i].crc;
  }
  return rc;
}

}  // extern "C"

// ---- on-disk blocks (block_store.h) ----------------------------------------
#include "block_store.h"

extern "C" {

static tfs::dataserver::BlockStore make_store(const char* mount, int32_t main_size, int32_t ext_size) {
  tfs::dataserver::BlockStore st;
  st.mount = mount;
  st.main_block_size = main_size;
  st.ext_block_size = ext_size;
  return st;
}

int tfs_ds_block_write_files(void* block, const char* mount, int32_t main_size, int32_t ext_size, uint32_t main_id,
                             uint32_t first_ext_id, int32_t bucket_size, uint32_t* ext_ids, uint32_t cap,
                             uint32_t* n_ext) {
  std::vector<uint32_t> ids;
  const int rc = tfs::dataserver::write_logic_block(make_store(mount, main_size, ext_size), main_id, first_ext_id,
                                                    *static_cast<LogicBlockImage*>(block), bucket_size, &ids);
  if (n_ext) *n_ext = uint32_t(ids.size());
  for (size_t i = 0; ext_ids && i < ids.size() && i < cap; ++i) ext_ids[i] = ids[i];
  return rc;
}

int tfs_ds_block_append(void* b, uint64_t file_id, const char* payload, int32_t len, uint32_t crc) {
  return static_cast<LogicBlockImage*>(b)->append_record(file_id, payload, len, crc);
}

void* tfs_ds_loaded_new(tfs_crc_ctx* ctx) { return new tfs::dataserver::LoadedBlock(ctx); }
void tfs_ds_loaded_free(void* b) { delete static_cast<tfs::dataserver::LoadedBlock*>(b); }
int tfs_ds_loaded_load(void* b, const char* mount, int32_t main_size, int32_t ext_size, uint32_t main_id) {
  return static_cast<tfs::dataserver::LoadedBlock*>(b)->load(make_store(mount, main_size, ext_size), main_id);
}
int64_t tfs_ds_loaded_size(void* b) { return static_cast<tfs::dataserver::LoadedBlock*>(b)->size(); }
const char* tfs_ds_loaded_data(void* b) { return static_cast<tfs::dataserver::LoadedBlock*>(b)->data(); }
uint32_t tfs_ds_loaded_logic_id(void* b) { return static_cast<tfs::dataserver::LoadedBlock*>(b)->logic_block_id; }
// Copy metas/flags (cap entries) and the chain (chain_cap); returns the meta count.
uint32_t tfs_ds_loaded_metas(void* b, tfs_raw_meta* metas, int32_t* flags, uint32_t cap, uint32_t* chain,
                             uint32_t chain_cap, uint32_t* chain_len, void* header48) {
  auto* lb = static_cast<tfs::dataserver::LoadedBlock*>(b);
  for (size_t i = 0; i < lb->metas.size() && i < cap; ++i) {
    if (metas) metas[i] = lb->metas[i];
    if (flags) flags[i] = lb->flags[i];
  }
  if (chain_len) *chain_len = uint32_t(lb->chain.size());
  for (size_t i = 0; chain && i < lb->chain.size() && i < chain_cap; ++i) chain[i] = lb->chain[i];
  if (header48) memcpy(header48, &lb->header, sizeof lb->header);
  return uint32_t(lb->metas.size());
}

namespace {
int export_compact_result(int rc, const tfs::dataserver::CompactFilesResult& r, tfs_raw_meta* dest_metas,
                          int32_t* status, uint32_t cap, uint32_t* ext_ids, uint32_t ext_cap, uint32_t* n_ext,
                          int64_t* counters) {
  for (size_t i = 0; i < r.dest_metas.size() && i < cap; ++i) {
    if (dest_metas) dest_metas[i] = r.dest_metas[i];
    if (status) status[i] = r.status[i];
  }
  if (n_ext) *n_ext = uint32_t(r.ext_ids.size());
  for (size_t i = 0; ext_ids && i < r.ext_ids.size() && i < ext_cap; ++i) ext_ids[i] = r.ext_ids[i];
  if (counters) {
    counters[0] = int64_t(r.dest_metas.size());
    counters[1] = r.dest_size;
    counters[2] = r.windows;
    counters[3] = r.launches;
    counters[4] = r.big_files;
    counters[5] = r.n_bad;
    counters[6] = int64_t(r.dropped.size());
  }
  return rc;
}
}  // namespace

// compact_block_files: the new block's metas / statuses (cap entries), ext ids
// (ext_cap), and counters[7] = {n_live, dest_size, windows, launches, big_files, n_bad, n_dropped}.
int tfs_ds_compact_block_files(tfs_crc_ctx* ctx, const char* src_mount, const char* dst_mount, int32_t main_size,
                               int32_t ext_size, uint32_t src_main_id, uint32_t dst_main_id, uint32_t first_ext_id,
                               int32_t bucket_size, int windows_per_launch, tfs_raw_meta* dest_metas,
                               int32_t* status, uint32_t cap, uint32_t* ext_ids, uint32_t ext_cap, uint32_t* n_ext,
                               int64_t* counters) {
  tfs::dataserver::CompactFilesResult r;
  const int rc = tfs::dataserver::compact_block_files(ctx, make_store(src_mount, main_size, ext_size), src_main_id,
                                                      make_store(dst_mount, main_size, ext_size), dst_main_id,
                                                      first_ext_id, bucket_size, windows_per_launch, &r);
  return export_compact_result(rc, r, dest_metas, status, cap, ext_ids, ext_cap, n_ext, counters);
}

// A BlockFileCompactor kept across blocks (window buffers and streams allocated once).
void* tfs_ds_compactor_new(tfs_crc_ctx* ctx, int windows_per_launch) {
  return ctx ? new tfs::dataserver::BlockFileCompactor(ctx, windows_per_launch) : nullptr;
}
void tfs_ds_compactor_free(void* h) { delete static_cast<tfs::dataserver::BlockFileCompactor*>(h); }
int tfs_ds_compactor_compact(void* h, const char* src_mount, const char* dst_mount, int32_t main_size,
                             int32_t ext_size, uint32_t src_main_id, uint32_t dst_main_id, uint32_t first_ext_id,
                             int32_t bucket_size, tfs_raw_meta* dest_metas, int32_t* status, uint32_t cap,
                             uint32_t* ext_ids, uint32_t ext_cap, uint32_t* n_ext, int64_t* counters) {
  if (!h) return TFS_EXIT_PARAMETER_ERROR;
  tfs::dataserver::CompactFilesResult r;
  const int rc = static_cast<tfs::dataserver::BlockFileCompactor*>(h)->compact(
      make_store(src_mount, main_size, ext_size), src_main_id, make_store(dst_mount, main_size, ext_size), dst_main_id,
      first_ext_id, bucket_size, &r);
  return export_compact_result(rc, r, dest_metas, status, cap, ext_ids, ext_cap, n_ext, counters);
}

int tfs_ds_verify_block_files(tfs_crc_ctx* ctx, const char* mount, int32_t main_size, int32_t ext_size,
                              uint32_t main_id, int32_t* status, uint32_t cap, uint32_t* n_live, void* checker) {
  std::vector<int32_t> st;
  const int rc = tfs::dataserver::verify_block_files(ctx, make_store(mount, main_size, ext_size), main_id, &st,
                                                     static_cast<BlockCrcChecker*>(checker));
  if (n_live) *n_live = uint32_t(st.size());
  for (size_t i = 0; status && i < st.size() && i < cap; ++i) status[i] = st[i];
  return rc;
}

}  // extern "C"
