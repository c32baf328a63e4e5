// ds_harness.cpp -- see ds_harness.h.  Everything CRC goes through the C ABI.
#include "ds_harness.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <ctime>

namespace tfs {
namespace dataserver {

namespace {
constexpr int32_t kFileInfoSize = TFS_FILEINFO_SIZE;
constexpr int32_t kExitReadOffset = -8002;    // EXIT_READ_OFFSET_ERROR, error_msg.h:138
constexpr int32_t kExitMetaNotFound = -8025;  // EXIT_META_NOT_FOUND_ERROR, error_msg.h:161
constexpr int32_t kExitBlockExhaust = -8004;  // EXIT_BLOCK_EXHAUST_ERROR, error_msg.h:140
constexpr int32_t kTfsError = -1;             // TFS_ERROR: DataFile::get_data failed (logic_block.cpp:264-270)

void put_file_info(char* dst, const tfs_file_info& fi) { memcpy(dst, &fi, kFileInfoSize); }
}  // namespace

// ---------------- DataFile (data_file.cpp) ----------------

DataFile::DataFile(uint64_t fn, const std::string& tmp_dir, tfs_crc_ctx* ctx, LeaseBufferPool* pool)
    : ctx_(ctx) {
  if (pool && (data_ = pool->take()) != nullptr) pool_ = pool;
  else data_ = new char[WRITE_DATA_TMPBUF_SIZE];
  char name[512];
  snprintf(name, sizeof name, "%s/%llu.dat", tmp_dir.c_str(), static_cast<unsigned long long>(fn));
  tmp_file_name_ = name;
}

DataFile::~DataFile() {
  set_over();
  if (pool_) pool_->give(data_);
  else delete[] data_;
}

// ---------------- LeaseBufferPool ----------------

LeaseBufferPool::LeaseBufferPool(tfs_crc_ctx* ctx, uint32_t nbuffers) : ctx_(ctx) {
  void* p = nullptr;
  if (nbuffers && tfs_crc32_host_malloc_pinned(ctx_, uint64_t(nbuffers) * uint64_t(DataFile::WRITE_DATA_TMPBUF_SIZE),
                                               &p) == TFS_SUCCESS) {
    base_ = static_cast<char*>(p);
    n_ = nbuffers;
    free_.reserve(n_);
    for (uint32_t i = n_; i-- > 0;) free_.push_back(base_ + size_t(i) * size_t(DataFile::WRITE_DATA_TMPBUF_SIZE));
  }
}

LeaseBufferPool::~LeaseBufferPool() {
  if (base_) tfs_crc32_host_free_pinned(ctx_, base_);
}

char* LeaseBufferPool::take() {
  std::lock_guard<std::mutex> g(mu_);
  if (free_.empty()) return nullptr;
  char* p = free_.back();
  free_.pop_back();
  return p;
}

void LeaseBufferPool::give(char* p) {
  std::lock_guard<std::mutex> g(mu_);
  free_.push_back(p);
}

uint32_t LeaseBufferPool::in_use() const {
  std::lock_guard<std::mutex> g(mu_);
  return n_ - uint32_t(free_.size());
}

void DataFile::set_over() {
  length_ = 0;
  if (fd_ != -1) {
    close(fd_);
    unlink(tmp_file_name_.c_str());
    fd_ = -1;
  }
}

int DataFile::set_data(const char* data, int32_t len, int32_t offset) {
  if (len <= 0) return TFS_SUCCESS;
  const int32_t length = offset + len;
  if (length > WRITE_DATA_TMPBUF_SIZE || length_ > WRITE_DATA_TMPBUF_SIZE) {  // spill (data_file.cpp:73-101)
    if (fd_ == -1) {
      fd_ = open(tmp_file_name_.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0600);
      if (fd_ == -1) return -1;
      if (write(fd_, data_, length_) != length_) return -1;
    }
    if (lseek(fd_, offset, SEEK_SET) == -1) return -1;
    if (write(fd_, data, len) != len) return -1;
  } else {
    memcpy(data_ + offset, data, len);
  }
  if (length > length_) length_ = length;
  return len;
}

char* DataFile::get_data(char* data, int32_t* len, int32_t offset) {
  if (offset >= length_) {
    *len = -1;
    return nullptr;
  }
  if (length_ > WRITE_DATA_TMPBUF_SIZE) {
    if (fd_ == -1 || lseek(fd_, offset, SEEK_SET) == -1) {
      *len = -1;
      return nullptr;
    }
    if (data == nullptr) {
      data = data_;
      *len = WRITE_DATA_TMPBUF_SIZE;
    }
    const ssize_t r = read(fd_, data, *len);
    if (r < 0) {
      *len = -1;
      return nullptr;
    }
    *len = int32_t(r);
    return data;
  }
  if (data == nullptr) {
    data = data_ + offset;
    *len = length_ - offset;
  } else {
    if (*len > length_ - offset) *len = length_ - offset;
    memcpy(data, data_ + offset, *len);
  }
  return data;
}

uint32_t DataFile::get_crc() {
  status_ = TFS_SUCCESS;
  if (crc_ != 0) return crc_;
  // The running CRC stays local until every chunk has been computed: a device
  // failure part-way leaves crc_ at 0 ("not computed", recomputed on the next
  // call, :170) instead of caching a partial value, and last_status() tells the
  // close path it was the device, not the client's data.
  if (length_ > WRITE_DATA_TMPBUF_SIZE) {  // data_file.cpp:172-187: re-read in 2 MiB chunks, running seed
    if (fd_ == -1 || lseek(fd_, 0, SEEK_SET) == -1) return crc_;
    uint32_t run = 0;
    ssize_t rlen;
    while ((rlen = read(fd_, data_, WRITE_DATA_TMPBUF_SIZE)) > 0) {
      tfs_crc_desc d{0, uint32_t(rlen), run};
      uint32_t out = 0;
      status_ = tfs_crc32_batch(ctx_, &d, 1, data_, uint64_t(rlen), &out);
      if (status_ != TFS_SUCCESS) return 0;
      run = out;
    }
    crc_ = run;
  } else {
    uint32_t out = 0;
    status_ = tfs_datafile_get_crc(ctx_, data_, length_, &out);
    if (status_ != TFS_SUCCESS) return 0;
    crc_ = out;
  }
  return crc_;
}

// ---------------- LogicBlockImage (logic_block.cpp) ----------------

LogicBlockImage::LogicBlockImage(uint32_t block_id, int64_t capacity, ImageArena* arena)
    : block_id_(block_id), capacity_(capacity), data_(ImageAlloc<char>(arena)) {
  // A pooled image takes its whole arena now and never grows past it: a growth
  // would move the image to pageable memory and give the arena back, and the
  // in-place verify of a page-locked image would silently stop applying.
  if (arena && arena->cap) {
    capacity_ = std::min<int64_t>(capacity_, int64_t(arena->cap));
    data_.reserve(arena->cap);
  }
}

BlockImagePool::BlockImagePool(tfs_crc_ctx* ctx, size_t count, size_t bytes) : ctx_(ctx) {
  for (size_t i = 0; i < count; ++i) {
    void* p = nullptr;
    if (tfs_crc32_host_malloc_pinned(ctx, bytes, &p) != TFS_SUCCESS) break;
    arenas_.emplace_back(new ImageArena());
    arenas_.back()->p = static_cast<char*>(p);
    arenas_.back()->cap = bytes;
  }
}

BlockImagePool::~BlockImagePool() {
  // An arena still lent to a live image is not freed under it (that image would
  // write to freed page-locked memory); the caller frees the pool after its
  // blocks (tfs_amd/dataserver.py refuses otherwise).
  for (auto& a : arenas_)
    if (!a->in_use.load()) tfs_crc32_host_free_pinned(ctx_, a->p);
}

size_t BlockImagePool::in_use() const {
  size_t k = 0;
  for (const auto& a : arenas_) k += a->in_use.load() ? 1u : 0u;
  return k;
}

ImageArena* BlockImagePool::take() {
  for (auto& a : arenas_)
    if (!a->in_use.load()) return a.get();  // claimed by the image's first allocation
  return nullptr;
}

int LogicBlockImage::append_record(uint64_t file_id, const char* payload, int32_t len, uint32_t crc) {
  if (len < 0) return TFS_EXIT_PARAMETER_ERROR;
  tfs_file_info fi;
  memset(&fi, 0, sizeof fi);
  fi.id_ = file_id;
  fi.size_ = len + kFileInfoSize;   // logic_block.cpp:173
  fi.usize_ = fi.size_;             // :235
  fi.modify_time_ = int32_t(time(nullptr));
  fi.create_time_ = fi.modify_time_;
  fi.flag_ = 0;
  fi.crc_ = crc;                    // :177
  int64_t off;
  {
    // The record's range and index entry are taken under a short lock; the bytes
    // are copied outside it, beside other writers (records are disjoint).
    std::lock_guard<std::mutex> g(mu_);
    off = used_.load();
    // Capacity and the int32 FileInfo/RawMeta offset are checked under the lock
    // that reserves the range, so batched and unbatched closes accept the same
    // writes and concurrent appends cannot overrun the block together.
    if (off + int64_t(fi.size_) > capacity_ || off + int64_t(fi.size_) > int64_t(INT32_MAX))
      return kExitBlockExhaust;
    fi.offset_ = int32_t(off);
    if (size_t(off + fi.size_) > data_.capacity()) {  // moves the image: no copy may be in flight
      std::unique_lock<std::shared_mutex> w(grow_mu_);
      data_.reserve(std::max(data_.capacity() * 2, size_t(off + fi.size_)));
    }
    data_.resize(size_t(off + fi.size_));
    used_.store(off + fi.size_, std::memory_order_release);
    index_[file_id] = tfs_raw_meta{file_id, int32_t(off), fi.size_};
    flags_[file_id] = 0;
  }
  std::shared_lock<std::shared_mutex> g(grow_mu_);
  put_file_info(data_.data() + off, fi);
  if (len) memcpy(data_.data() + off + kFileInfoSize, payload, size_t(len));
  return TFS_SUCCESS;
}

void LogicBlockImage::reserve(int64_t bytes) {
  std::lock_guard<std::mutex> g(mu_);
  std::unique_lock<std::shared_mutex> w(grow_mu_);
  if (bytes <= int64_t(data_.capacity())) return;
  data_.reserve(size_t(bytes));
  const uintptr_t a = (reinterpret_cast<uintptr_t>(data_.data()) + (2u << 20) - 1) & ~uintptr_t((2u << 20) - 1);
  const uintptr_t e = (reinterpret_cast<uintptr_t>(data_.data()) + data_.capacity()) & ~uintptr_t((2u << 20) - 1);
  if (e > a) madvise(reinterpret_cast<void*>(a), e - a, MADV_HUGEPAGE);  // advisory; failure is harmless
  // Fault the reservation in now, as the dataserver's block files are allocated at
  // full size before any write (BlockFileManager::create_block_prefix formats each
  // block file, blockfile_manager.cpp:1307-1372, blockfile_format.h:63-87 fallocate):
  // left to the appends, every 2 MiB of records paid one huge-page zeroing on
  // the close path (~100 us; the close tail of round 5).
  // A page-locked arena is resident already.
  // TFS_DS_PREFAULT=0 leaves the faults to the appends (the round-5 behaviour, A/B).
  static const bool prefault = [] {
    const char* v = getenv("TFS_DS_PREFAULT");
    return !(v && atoi(v) == 0);
  }();
  const ImageArena* ar = data_.get_allocator().arena;
  if (prefault && !(ar && data_.data() == ar->p)) {
    volatile char* p = data_.data();
    for (size_t o = data_.size(); o < data_.capacity(); o += 4096) p[o] = 0;
  }
}

int LogicBlockImage::close_write_file(uint64_t file_id, DataFile& df, uint32_t crc) {
  const int32_t file_size = df.get_length();
  if (const char* p = df.in_memory_payload()) return append_record(file_id, p, file_size, crc);
  std::vector<char> payload(static_cast<size_t>(file_size));
  int32_t off = 0;
  while (off < file_size) {  // logic_block.cpp:258-306: drain the DataFile
    int32_t rl = file_size - off;
    if (!df.get_data(payload.data() + off, &rl, off) || rl <= 0) return kTfsError;
    off += rl;
  }
  return append_record(file_id, payload.data(), file_size, crc);
}

int LogicBlockImage::read_file(uint64_t file_id, std::vector<char>& out) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = index_.find(file_id);
  if (it == index_.end()) return TFS_EXIT_FILE_INFO_ERROR;
  out.assign(data_.begin() + it->second.offset, data_.begin() + it->second.offset + it->second.size);
  return TFS_SUCCESS;
}

int LogicBlockImage::read_file(uint64_t file_id, char* buf, int32_t* nbytes, int32_t offset, bool force) const {
  tfs_raw_meta m;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(file_id);
    if (it == index_.end()) return kExitMetaNotFound;
    m = it->second;
  }
  if (offset + *nbytes > m.size) *nbytes = m.size - offset;  // truncate to the record (:388-391)
  if (*nbytes < 0) return kExitReadOffset;
  if (int64_t(m.offset) + offset + *nbytes > data_size()) return TFS_EXIT_PARAMETER_ERROR;
  memcpy(buf, data_.data() + m.offset + offset, size_t(*nbytes));
  if (offset == 0) {  // :414-435
    if (*nbytes < kFileInfoSize) return TFS_EXIT_READ_FILE_SIZE_ERROR;
    tfs_file_info fi;
    memcpy(&fi, buf, sizeof fi);
    const int32_t real = flag_of(file_id);  // get_real_flag: the index keeps the unlink flag
    const int32_t reject = force ? TFS_FI_INVALID : (TFS_FI_DELETED | TFS_FI_INVALID | TFS_FI_CONCEAL);
    if (fi.id_ != file_id || (real & reject)) return TFS_EXIT_FILE_INFO_ERROR;
  }
  return TFS_SUCCESS;
}

int LogicBlockImage::set_flag(uint64_t file_id, int32_t flag) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = flags_.find(file_id);
  if (it == flags_.end()) return TFS_EXIT_FILE_INFO_ERROR;
  it->second = flag;
  return TFS_SUCCESS;
}

int32_t LogicBlockImage::flag_of(uint64_t file_id) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = flags_.find(file_id);
  return it == flags_.end() ? TFS_FI_INVALID : it->second;
}

std::vector<tfs_raw_meta> LogicBlockImage::sorted_metas() const {
  std::vector<tfs_raw_meta> v;
  {
    std::lock_guard<std::mutex> g(mu_);
    v.reserve(index_.size());
    for (auto& kv : index_) v.push_back(kv.second);
  }
  std::sort(v.begin(), v.end(), [](const tfs_raw_meta& a, const tfs_raw_meta& b) { return a.offset < b.offset; });
  return v;
}

std::vector<int32_t> LogicBlockImage::sorted_flags() const {
  std::vector<int32_t> f;
  for (auto& m : sorted_metas()) f.push_back(flag_of(m.file_id));
  return f;
}

void LogicBlockImage::replace(ByteImage&& data, const std::vector<tfs_raw_meta>& metas,
                              const std::vector<int32_t>& flags) {
  std::lock_guard<std::mutex> g(mu_);
  std::unique_lock<std::shared_mutex> w(grow_mu_);
  data_ = std::move(data);
  used_ = int64_t(data_.size());
  index_.clear();
  flags_.clear();
  for (size_t i = 0; i < metas.size(); ++i) {
    index_[metas[i].file_id] = metas[i];
    flags_[metas[i].file_id] = i < flags.size() ? flags[i] : 0;
  }
}

// ---------------- close path (data_management.cpp:173-236) ----------------

int close_write_file(const CloseFileInfo& info, DataFile& df, LogicBlockImage& block) {
  const uint32_t datafile_crc = df.get_crc();
  if (df.last_status() != TFS_SUCCESS) return df.last_status();
  if (info.crc_ != datafile_crc) return TFS_EXIT_DATA_FILE_ERROR;  // :197-198
  return block.close_write_file(info.file_id_, df, datafile_crc);
}

namespace {
// Wait for `pred` spinning (the verdict of a batch arrives in tens of
// microseconds), yielding the CPU once the wait grows long.
template <typename P>
void spin_until(P pred) {
  for (uint32_t i = 0; !pred(); ++i) {
    if (i < 4096) __builtin_ia32_pause();
    else std::this_thread::yield();
  }
}
}  // namespace

CloseBatcher::CloseBatcher(tfs_crc_ctx* ctx, size_t max_batch, int max_wait_us, int in_flight,
                           LeaseBufferPool* pool)
    : ctx_(ctx), max_batch_(max_batch ? max_batch : 1), max_wait_us_(max_wait_us),
      gather_cap_(std::min<size_t>(std::max<size_t>(max_batch_ * (256u << 10), 4u << 20), 16u << 20)),
      pool_(pool && pool->ok() ? pool : nullptr),
      nbatches_(std::min(std::max(in_flight, 1), kMaxInFlight)),
      batches_buf_(new Batch[size_t(nbatches_)]),
      trace_(getenv("TFS_DS_TRACE") != nullptr) {
  // The gather buffers are page-locked once, here (DataService::initialize),
  // never on a close.  A batcher on a lease pool gathers nothing.
  for (Batch& b : all_batches()) {
    b.desc.resize(max_batch_);
    b.crc.resize(max_batch_);
    b.ok.resize(max_batch_);
    if (pool_) continue;
    void* p = nullptr;
    if (tfs_crc32_host_malloc_pinned(ctx_, gather_cap_, &p) == TFS_SUCCESS) {
      b.gather = static_cast<char*>(p);
    } else {
      b.fallback.resize(gather_cap_);
      b.gather = b.fallback.data();
    }
  }
}

CloseBatcher::~CloseBatcher() {
  for (Batch& b : all_batches())
    if (b.gather && b.fallback.empty()) tfs_crc32_host_free_pinned(ctx_, b.gather);
  if (getenv("TFS_DS_TRACE"))
    fprintf(stderr,
            "close batcher: %llu batches, verify %lld us; thread-us claim %lld copy %lld wait %lld (leader "
            "pre-verify %lld) append %lld\n",
            (unsigned long long)batches_.load(), (long long)verify_us_.load(), (long long)t_claim_.load(),
            (long long)t_copy_.load(), (long long)t_wait_.load(), (long long)t_lead_wait_.load(),
            (long long)t_append_.load());
}

CloseBatcher::Batch* CloseBatcher::take_batch(std::unique_lock<std::mutex>& lk) {
  for (;;) {
    for (Batch& b : all_batches()) {
      if (!b.free) continue;
      b.free = false;
      b.n = 0;
      b.bytes = 0;
      b.closed = false;
      b.ready = 0;
      b.left = 0;
      b.done = 0;
      b.rc = TFS_SUCCESS;
      b.opened = std::chrono::steady_clock::now();
      return &b;
    }
    free_cv_.wait(lk);
  }
}

// The first member of a batch: close it (full, or max_wait_us after it opened),
// wait for every member's payload, run the GPU verify, publish the verdicts.
void CloseBatcher::lead(Batch* b) {
  const auto deadline = b->opened + std::chrono::microseconds(max_wait_us_);
  spin_until([&] { return b->closed.load(std::memory_order_acquire) || std::chrono::steady_clock::now() >= deadline; });
  uint32_t n;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!b->closed.load()) {
      b->closed = true;
      if (cur_ == b) cur_ = nullptr;
    }
    n = b->n;
  }
  spin_until([&] { return b->ready.load(std::memory_order_acquire) == n; });
  tfs_crc_stats s0{};
  if (b->timed) tfs_crc32_stats(ctx_, &s0);
  const auto t0 = std::chrono::steady_clock::now();
  if (trace_) t_lead_wait_ += std::chrono::duration_cast<std::chrono::microseconds>(t0 - b->opened).count();
  uint32_t nbad = 0;
  // Pooled batches: each member's payload is read in its own lease buffer.
  b->rc = pool_ ? tfs_crc32_verify(ctx_, b->desc.data(), n, pool_->base(), pool_->bytes(), b->crc.data(),
                                   b->ok.data(), &nbad)
                : tfs_crc32_verify(ctx_, b->desc.data(), n, b->gather, b->bytes, b->crc.data(), b->ok.data(), &nbad);
  const auto t1 = std::chrono::steady_clock::now();
  verify_us_ += std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count();
  if (b->timed) {
    tfs_crc_stats s1{};
    tfs_crc32_stats(ctx_, &s1);
    b->lead_wait_us = std::chrono::duration<double, std::micro>(t0 - b->opened).count();
    b->verify_us = std::chrono::duration<double, std::micro>(t1 - t0).count();
    b->relaunches = uint32_t(s1.resident_launches - s0.resident_launches);
    b->ring_full = uint32_t(s1.resident_ring_full - s0.resident_ring_full);
  }
  ++batches_;
  b->done.store(1, std::memory_order_release);
}

int CloseBatcher::close(const CloseFileInfo& info, DataFile& df, LogicBlockImage& block, CloseTiming* t) {
  const int32_t len = df.get_length();
  const char* own = df.in_memory_payload();
  const bool pooled = pool_ && own && pool_->owns(own);
  if (len > kMaxBatched || (pool_ ? !pooled : size_t(len) > gather_cap_))
    return close_write_file(info, df, block);  // unbatched
  using clk = std::chrono::steady_clock;
  auto us = [](clk::time_point a, clk::time_point b2) {
    return int64_t(std::chrono::duration_cast<std::chrono::microseconds>(b2 - a).count());
  };
  const bool timed = trace_ || t;
  const auto c0 = timed ? clk::now() : clk::time_point();
  Batch* b;
  uint32_t slot;
  uint64_t off;
  {
    std::unique_lock<std::mutex> lk(mu_);
    if (cur_ && !pooled && cur_->bytes + uint64_t(len) > gather_cap_) {  // no room: close it, its leader fires it
      cur_->closed = true;
      cur_ = nullptr;
    }
    if (!cur_) cur_ = take_batch(lk);
    b = cur_;
    slot = b->n++;
    if (slot == 0) b->timed = t != nullptr;
    off = b->bytes;
    b->bytes += uint64_t(len);
    b->left.fetch_add(1);
    if (b->n == max_batch_) {
      b->closed.store(true, std::memory_order_release);
      cur_ = nullptr;
    }
  }
  const auto c1 = timed ? clk::now() : clk::time_point();
  // This lease's payload into the batch's gather buffer (data_file.cpp:115-166),
  // or, from a lease pool, read where it is.
  int32_t got = 0;
  if (pooled) {
    got = len;
    off = uint64_t(own - pool_->base());
  }
  while (got < len) {
    int32_t rl = len - got;
    if (!df.get_data(b->gather + off + got, &rl, got) || rl <= 0) break;
    got += rl;
  }
  // An unreadable lease (spill-file I/O error) gets an empty descriptor and fails
  // with TFS_ERROR as LogicBlock::close_write_file would (logic_block.cpp:264-270).
  const bool readable = got == len;
  b->desc[slot] = tfs_crc_vdesc{off, readable ? uint32_t(len) : 0u, info.crc_};
  b->ready.fetch_add(1, std::memory_order_release);
  const auto c2 = timed ? clk::now() : clk::time_point();
  if (slot == 0) lead(b);
  else spin_until([&] { return b->done.load(std::memory_order_acquire) != 0; });
  if (timed) {
    const auto c3 = clk::now();
    if (trace_) {
      t_claim_ += us(c0, c1);
      t_copy_ += us(c1, c2);
      t_wait_ += us(c2, c3);
    }
    if (t) {
      auto fus = [](clk::time_point a, clk::time_point b2) { return std::chrono::duration<double, std::micro>(b2 - a).count(); };
      t->claim_us = fus(c0, c1);
      t->copy_us = fus(c1, c2);
      t->wait_us = fus(c2, c3);
      t->leader = slot == 0;
      t->batch_n = b->n;
      if (b->timed) {
        t->lead_wait_us = b->lead_wait_us;
        t->verify_us = b->verify_us;
        t->relaunches = b->relaunches;
        t->ring_full = b->ring_full;
      }
    }
  }
  int status;
  uint32_t crc = 0;
  if (!readable) {
    status = kTfsError;
  } else if (b->rc != TFS_SUCCESS && b->rc != TFS_EXIT_CHECK_CRC_ERROR) {
    status = b->rc;  // device failure: reported as such, never as client corruption
  } else if (!b->ok[slot]) {
    status = TFS_EXIT_DATA_FILE_ERROR;  // data_management.cpp:198
  } else {
    status = kAppend;
    crc = b->crc[slot];
  }
  if (b->left.fetch_sub(1) == 1) {  // last reader: the batch is free again
    std::lock_guard<std::mutex> g(mu_);
    b->free = true;
    free_cv_.notify_one();
  }
  if (status != kAppend) return status;
  // Checked: persist from this thread (LogicBlock::close_write_file runs on the
  // worker, logic_block.cpp:156-372), so the appends of a batch run side by side.
  const auto c4 = timed ? clk::now() : clk::time_point();
  const int rc = block.close_write_file(info.file_id_, df, crc);
  if (timed) {
    const auto c5 = clk::now();
    if (trace_) t_append_ += us(c4, c5);
    if (t) t->append_us = std::chrono::duration<double, std::micro>(c5 - c4).count();
  }
  return rc;
}

// ---------------- CrcService (DataService's CRC side, multi-GPU) ----------------

CrcService::CrcService(tfs_crc_group* group, size_t max_batch, int max_wait_us) : group_(group) {
  for (uint32_t i = 0; i < tfs_crc_group_size(group); ++i)
    batchers_.emplace_back(new CloseBatcher(tfs_crc_group_ctx(group, i), max_batch, max_wait_us));
}

CrcService::~CrcService() = default;

int CrcService::close_write_file(const CloseFileInfo& info, DataFile& df, LogicBlockImage& block) {
  if (batchers_.empty()) return TFS_EXIT_PARAMETER_ERROR;
  return batchers_[tfs_crc_group_member_of(group_, info.block_id_)]->close(info, df, block);
}

int CrcService::verify_blocks(const std::vector<const LogicBlockImage*>& blocks, std::vector<uint32_t>* nbad) {
  std::vector<std::vector<tfs_raw_meta>> live(blocks.size());
  std::vector<tfs_block_verify_job> jobs(blocks.size());
  for (size_t i = 0; i < blocks.size(); ++i) {
    const LogicBlockImage& b = *blocks[i];
    for (auto& m : b.sorted_metas())
      if (!(b.flag_of(m.file_id) & (TFS_FI_DELETED | TFS_FI_INVALID))) live[i].push_back(m);
    tfs_block_verify_job& j = jobs[i];
    memset(&j, 0, sizeof j);
    j.block_id = b.block_id();
    j.image = b.data().data();
    j.image_len = uint64_t(b.data_size());
    j.metas = live[i].data();
    j.n = uint32_t(live[i].size());
  }
  const int rc = tfs_crc_group_blocks_verify(group_, jobs.data(), uint32_t(jobs.size()));
  if (nbad) {
    nbad->resize(blocks.size());
    for (size_t i = 0; i < blocks.size(); ++i) (*nbad)[i] = jobs[i].n_bad;
  }
  return rc;
}

// ---------------- verify / checker / compact ----------------

void BlockCrcChecker::add_crc_error(uint32_t block_id, uint64_t file_id) {
  ++errors_[block_id];
  repair_.emplace_back(block_id, file_id);
}

int BlockCrcChecker::crc_errors(uint32_t block_id) const {
  auto it = errors_.find(block_id);
  return it == errors_.end() ? 0 : it->second;
}

int read_file_verified(tfs_crc_ctx* ctx, const LogicBlockImage& block, uint64_t file_id, std::vector<char>* out,
                       BlockCrcChecker* checker) {
  std::vector<tfs_raw_meta> metas = block.sorted_metas();
  int32_t size = -1;
  for (auto& m : metas)
    if (m.file_id == file_id) size = m.size;
  if (size < 0) return kExitMetaNotFound;
  out->assign(size_t(size), 0);
  int32_t nbytes = size;
  int rc = block.read_file(file_id, out->data(), &nbytes, 0, false);
  if (rc != TFS_SUCCESS) return rc;
  tfs_file_info fi;
  memcpy(&fi, out->data(), sizeof fi);
  const tfs_crc_vdesc d{uint64_t(kFileInfoSize), uint32_t(nbytes - kFileInfoSize), fi.crc_};
  rc = tfs_crc32_verify(ctx, &d, 1, out->data(), uint64_t(nbytes), nullptr, nullptr, nullptr);
  if (rc == TFS_EXIT_CHECK_CRC_ERROR && checker) checker->add_crc_error(block.block_id(), file_id);
  return rc;
}

int verify_block(tfs_crc_ctx* ctx, const LogicBlockImage& block, std::vector<int32_t>* status,
                 BlockCrcChecker* checker) {
  std::vector<tfs_raw_meta> metas;
  for (auto& m : block.sorted_metas())
    if (!(block.flag_of(m.file_id) & (TFS_FI_DELETED | TFS_FI_INVALID))) metas.push_back(m);
  std::vector<uint32_t> crc(metas.size());
  std::vector<int32_t> st(metas.size());
  uint32_t nbad = 0;
  const int rc = tfs_block_verify(ctx, block.data().data(), uint64_t(block.data_size()), metas.data(),
                                  uint32_t(metas.size()), crc.data(), st.data(), &nbad);
  if (rc != TFS_SUCCESS && rc != TFS_EXIT_CHECK_CRC_ERROR) return rc;
  if (checker)
    for (size_t i = 0; i < metas.size(); ++i)
      if (st[i] == TFS_EXIT_CHECK_CRC_ERROR) checker->add_crc_error(block.block_id(), metas[i].file_id);
  if (status) *status = st;
  return int(nbad);
}

int recombine_block(tfs_crc_ctx* ctx, const LogicBlockImage& src, LogicBlockImage& dest, int* skipped_crc) {
  const std::vector<tfs_raw_meta> metas = src.sorted_metas();
  std::vector<int32_t> flags = src.sorted_flags();
  std::vector<tfs_raw_meta> check;
  std::vector<size_t> where;
  for (size_t i = 0; i < metas.size(); ++i) {
    if ((flags[i] & (TFS_FI_DELETED | TFS_FI_INVALID)) || metas[i].file_id == 0) {
      flags[i] |= TFS_FI_INVALID;
      continue;
    }
    uint32_t id_lo = 0;  // memcmp(&finfo, data_finfo, sizeof(FILEINFO_SIZE)): 4 bytes
    if (metas[i].offset < 0 || int64_t(metas[i].offset) + kFileInfoSize > src.data_size()) {
      flags[i] |= TFS_FI_INVALID;
      continue;
    }
    memcpy(&id_lo, src.data().data() + metas[i].offset, 4);
    if (id_lo != uint32_t(metas[i].file_id)) {
      flags[i] |= TFS_FI_INVALID;
      continue;
    }
    check.push_back(metas[i]);
    where.push_back(i);
  }
  std::vector<int32_t> st(check.size());
  uint32_t nbad = 0;
  int rc = tfs_block_verify(ctx, src.data().data(), uint64_t(src.data_size()), check.data(), uint32_t(check.size()),
                            nullptr, st.data(), &nbad);
  if (rc != TFS_SUCCESS && rc != TFS_EXIT_CHECK_CRC_ERROR) return rc;
  int dropped = 0;
  for (size_t k = 0; k < check.size(); ++k) {
    if (st[k] == TFS_SUCCESS) continue;
    dropped += st[k] == TFS_EXIT_CHECK_CRC_ERROR ? 1 : 0;
    flags[where[k]] |= TFS_FI_INVALID;  // not copied
  }
  if (skipped_crc) *skipped_crc = dropped;
  uint64_t cap = 16;
  for (auto& m : metas) cap += uint64_t(m.size);
  ByteImage out(static_cast<size_t>(cap));
  std::vector<tfs_raw_meta> dmetas(metas.size());
  uint64_t dlen = 0;
  uint32_t nlive = 0;
  rc = tfs_block_compact(ctx, src.data().data(), uint64_t(src.data_size()), metas.data(), flags.data(),
                         uint32_t(metas.size()), out.data(), cap, dmetas.data(), nullptr, &dlen, &nlive);
  if (rc != TFS_SUCCESS) return rc;  // every survivor was verified: a mismatch here is an error
  out.resize(size_t(dlen));
  dmetas.resize(nlive);
  std::vector<int32_t> dflags;
  for (size_t i = 0; i < metas.size(); ++i)
    if (!(flags[i] & (TFS_FI_DELETED | TFS_FI_INVALID))) dflags.push_back(flags[i]);
  dest.replace(std::move(out), dmetas, dflags);
  return TFS_SUCCESS;
}

int compact_block(tfs_crc_ctx* ctx, const LogicBlockImage& src, LogicBlockImage& dest, std::vector<uint8_t>* crc_ok) {
  const std::vector<tfs_raw_meta> metas = src.sorted_metas();
  const std::vector<int32_t> flags = src.sorted_flags();
  uint64_t cap = 16;
  for (auto& m : metas) cap += uint64_t(m.size);
  ByteImage out(static_cast<size_t>(cap));
  std::vector<tfs_raw_meta> dmetas(metas.size());
  std::vector<uint8_t> ok(metas.size());
  uint64_t dlen = 0;
  uint32_t nlive = 0;
  const int rc = tfs_block_compact(ctx, src.data().data(), uint64_t(src.data_size()), metas.data(), flags.data(),
                                   uint32_t(metas.size()), out.data(), cap, dmetas.data(), ok.data(), &dlen, &nlive);
  if (rc != TFS_SUCCESS && rc != TFS_EXIT_CHECK_CRC_ERROR) return rc;
  out.resize(size_t(dlen));
  dmetas.resize(nlive);
  std::vector<int32_t> dflags;
  for (size_t i = 0; i < metas.size(); ++i)
    if (!(flags[i] & (TFS_FI_DELETED | TFS_FI_INVALID))) dflags.push_back(flags[i]);
  dest.replace(std::move(out), dmetas, dflags);
  if (crc_ok) *crc_ok = ok;
  return rc;
}

}  // namespace dataserver
}  // namespace tfs
