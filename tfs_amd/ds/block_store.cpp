// block_store.cpp -- see block_store.h.  Host C++ (POSIX I/O); CRC work goes
// through the C ABI.
#include "block_store.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <set>
#include <thread>
#include <utility>

namespace tfs {
namespace dataserver {
namespace {

constexpr int32_t kReserve = TFS_BLOCK_RESERVER_LENGTH;  // physical_block.h:31
constexpr int kMaxChain = 64;

std::string main_path(const BlockStore& st, uint32_t id) { return st.mount + "/" + std::to_string(id); }
std::string ext_path(const BlockStore& st, uint32_t id) { return st.mount + "/extend/" + std::to_string(id); }
std::string index_path(const BlockStore& st, uint32_t id) { return st.mount + "/index/" + std::to_string(id); }

int pread_all(int fd, void* buf, size_t n, off_t off) {
  char* p = static_cast<char*>(buf);
  while (n) {
    const ssize_t r = pread(fd, p, n, off);
    if (r <= 0) return TFS_ERROR;
    p += r;
    n -= size_t(r);
    off += r;
  }
  return TFS_SUCCESS;
}
int pwrite_all(int fd, const void* buf, size_t n, off_t off) {
  const char* p = static_cast<const char*>(buf);
  while (n) {
    const ssize_t r = pwrite(fd, p, n, off);
    if (r <= 0) return TFS_ERROR;
    p += r;
    n -= size_t(r);
    off += r;
  }
  return TFS_SUCCESS;
}

struct Fd {
  int fd = -1;
  explicit Fd(int f) : fd(f) {}
  ~Fd() {
    if (fd >= 0) close(fd);
  }
};

// Prefix of a physical block: <mount>/block_prefix when present, else the
// block file's first 24 bytes (PhysicalBlock::load_block_prefix).
int read_prefix(const BlockStore& st, uint32_t id, bool main, BlockPrefix* out) {
  const std::string pf = st.mount + "/block_prefix";
  Fd f(open(pf.c_str(), O_RDONLY));
  if (f.fd >= 0) return pread_all(f.fd, out, sizeof *out, off_t(id - 1) * off_t(sizeof(BlockPrefix)));
  Fd b(open((main ? main_path(st, id) : ext_path(st, id)).c_str(), O_RDONLY));
  if (b.fd < 0) return TFS_ERROR;
  return pread_all(b.fd, out, sizeof *out, 0);
}

}  // namespace

// ---- writing ----------------------------------------------------------------

ChainWriter::ChainWriter(const BlockStore& st, uint32_t main_id, uint32_t first_ext_id, uint32_t logic_id)
    : st_(st), first_ext_id_(first_ext_id), logic_id_(logic_id) {
  mkdir(st.mount.c_str(), 0755);
  mkdir((st.mount + "/extend").c_str(), 0755);
  mkdir((st.mount + "/index").c_str(), 0755);
  rc_ = add_block(main_id);
}

ChainWriter::~ChainWriter() {
  for (int fd : fds_)
    if (fd >= 0) close(fd);
}

// A new physical block at the end of the chain (LogicBlock::extend_block): the
// file preallocated to its block length, its prefix in the reserved area, and
// the previous block's prefix pointed at it.
int ChainWriter::add_block(uint32_t id) {
  if (int(chain_.size()) >= kMaxChain) return TFS_EXIT_PARAMETER_ERROR;
  const bool main = chain_.empty();
  const int32_t blen = main ? st_.main_block_size : st_.ext_block_size;
  if (blen <= kReserve) return TFS_EXIT_PARAMETER_ERROR;
  const int fd = open((main ? main_path(st_, id) : ext_path(st_, id)).c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return TFS_ERROR;
  fds_.push_back(fd);
  std::vector<char> reserve(kReserve, 0);
  BlockPrefix bp{logic_id_, main ? 0u : chain_.back(), 0u, 0u, 0u};
  memcpy(reserve.data(), &bp, sizeof bp);
  if (pwrite_all(fd, reserve.data(), reserve.size(), 0) || ftruncate(fd, blen)) return TFS_ERROR;
  if (!main) {
    BlockPrefix prev;
    if (pread_all(fds_[fds_.size() - 2], &prev, sizeof prev, 0)) return TFS_ERROR;
    prev.next_physic_blockid_ = id;
    if (pwrite_all(fds_[fds_.size() - 2], &prev, sizeof prev, 0)) return TFS_ERROR;
  }
  chain_.push_back(id);
  return TFS_SUCCESS;
}

int ChainWriter::write(const char* src, int64_t len, int64_t off) {
  if (rc_) return rc_;
  if (off < 0 || len < 0) return TFS_EXIT_PARAMETER_ERROR;
  while (len > 0) {
    // physical block k holding logic offset `off` (DataHandle::choose_physic_block)
    size_t k = 0;
    int64_t base = 0;
    for (;; ++k) {
      const int64_t area = (k == 0 ? st_.main_block_size : st_.ext_block_size) - kReserve;
      if (off < base + area) break;
      base += area;
    }
    while (chain_.size() <= k) {
      rc_ = add_block(first_ext_id_ + uint32_t(chain_.size() - 1));
      if (rc_) return rc_;
    }
    const int64_t area = (k == 0 ? st_.main_block_size : st_.ext_block_size) - kReserve;
    const int64_t n = std::min(len, base + area - off);
    if (pwrite_all(fds_[k], src, size_t(n), off_t(kReserve + off - base))) return rc_ = TFS_ERROR;
    src += n;
    off += n;
    len -= n;
  }
  return TFS_SUCCESS;
}

int write_index(const BlockStore& st, uint32_t main_id, const BlockInfo& info, const std::vector<tfs_raw_meta>& metas,
                const std::vector<int32_t>& unlink_flags, int32_t bucket_size, int32_t data_size) {
  if (bucket_size <= 0 || (!unlink_flags.empty() && unlink_flags.size() != metas.size()))
    return TFS_EXIT_PARAMETER_ERROR;
  mkdir(st.mount.c_str(), 0755);
  mkdir((st.mount + "/index").c_str(), 0755);
  // Header, zeroed buckets, then one MetaInfo per file in write order.
  IndexHeader h;
  memset(&h, 0, sizeof h);
  h.block_info_ = info;
  h.bucket_size_ = bucket_size;
  h.index_file_size_ = int32_t(sizeof(IndexHeader) + size_t(bucket_size) * 4);
  h.data_file_offset_ = data_size;
  std::vector<char> idx(size_t(h.index_file_size_) + metas.size() * sizeof(MetaInfo), 0);
  int32_t* slots = reinterpret_cast<int32_t*>(idx.data() + sizeof(IndexHeader));
  for (size_t i = 0; i < metas.size(); ++i) {
    const int32_t slot = int32_t(uint32_t(metas[i].file_id) % uint32_t(bucket_size));
    const int32_t at = h.index_file_size_;
    h.index_file_size_ += int32_t(sizeof(MetaInfo));  // hash_insert: expand the index file
    MetaInfo mi{metas[i], 0};
    const int32_t fl = unlink_flags.empty() ? 0 : unlink_flags[i];
    if (fl) {
      // LogicBlock::unlink_file: the flag goes into the index entry
      // (RawMeta::set_unlink_flag, internal.h:610-614 -- bits 28-30 plus the
      // use-index bit 27); the FileInfo on disk keeps its old flag_.
      mi.raw_meta_.size = (mi.raw_meta_.size & kFileSizeMask) | ((fl << kUnlinkShift) & kUnlinkMask) | kUseIndexFlag;
    }
    memcpy(idx.data() + at, &mi, sizeof mi);
    // link at the tail of the slot's chain
    if (slots[slot] == 0) {
      slots[slot] = at;
    } else {
      int32_t pos = slots[slot];
      for (;;) {
        MetaInfo* node = reinterpret_cast<MetaInfo*>(idx.data() + pos);
        if (node->next_meta_offset_ == 0) {
          node->next_meta_offset_ = at;
          break;
        }
        pos = node->next_meta_offset_;
      }
    }
  }
  memcpy(idx.data(), &h, sizeof h);
  Fd f(open(index_path(st, main_id).c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644));
  if (f.fd < 0) return TFS_ERROR;
  return pwrite_all(f.fd, idx.data(), idx.size(), 0);
}

int write_logic_block(const BlockStore& st, uint32_t main_id, uint32_t first_ext_id, const LogicBlockImage& img,
                      int32_t bucket_size, std::vector<uint32_t>* ext_ids) {
  if (bucket_size <= 0 || st.main_block_size <= kReserve || st.ext_block_size <= kReserve)
    return TFS_EXIT_PARAMETER_ERROR;
  const int64_t size = img.data_size();
  ChainWriter w(st, main_id, first_ext_id, img.block_id());
  int rc = w.write(img.data().data(), size, 0);
  if (rc) return rc;
  if (ext_ids) ext_ids->assign(w.chain().begin() + 1, w.chain().end());
  const std::vector<tfs_raw_meta> metas = img.sorted_metas();
  const std::vector<int32_t> flags = img.sorted_flags();
  BlockInfo info;
  memset(&info, 0, sizeof info);
  info.block_id_ = img.block_id();
  info.seq_no_ = 1;
  info.version_ = int32_t(metas.size());
  for (size_t i = 0; i < metas.size(); ++i) {
    info.file_count_ += 1;
    info.size_ += metas[i].size;
    if (flags[i] & TFS_FI_DELETED) {
      info.del_file_count_ += 1;
      info.del_size_ += metas[i].size;
    }
    if (uint32_t(metas[i].file_id) >= info.seq_no_) info.seq_no_ = uint32_t(metas[i].file_id) + 1;
  }
  return write_index(st, main_id, info, metas, flags, bucket_size, int32_t(size));
}

int load_chain(const BlockStore& st, uint32_t main_id, std::vector<uint32_t>* chain, uint32_t* logic_block_id) {
  chain->clear();
  BlockPrefix bp;
  if (read_prefix(st, main_id, true, &bp)) return TFS_ERROR;
  if (logic_block_id) *logic_block_id = bp.logic_blockid_;
  chain->push_back(main_id);
  uint32_t prev = main_id;
  while (bp.next_physic_blockid_ != 0) {
    const uint32_t id = bp.next_physic_blockid_;
    if (int(chain->size()) >= kMaxChain || std::find(chain->begin(), chain->end(), id) != chain->end())
      return TFS_ERROR;  // loop or runaway chain
    if (read_prefix(st, id, false, &bp)) return TFS_ERROR;
    if (bp.prev_physic_blockid_ != prev) return TFS_ERROR;  // broken back link
    chain->push_back(id);
    prev = id;
  }
  return TFS_SUCCESS;
}

int load_index(const BlockStore& st, uint32_t main_id, IndexHeader* header, std::vector<tfs_raw_meta>* metas) {
  metas->clear();
  Fd f(open(index_path(st, main_id).c_str(), O_RDONLY));
  if (f.fd < 0) return TFS_ERROR;
  struct stat sb;
  if (fstat(f.fd, &sb) || sb.st_size < off_t(sizeof(IndexHeader))) return TFS_ERROR;
  std::vector<char> idx(size_t(sb.st_size));
  if (pread_all(f.fd, idx.data(), idx.size(), 0)) return TFS_ERROR;
  memcpy(header, idx.data(), sizeof *header);
  const int32_t nb = header->bucket_size_;
  if (nb <= 0 || sizeof(IndexHeader) + size_t(nb) * 4 > idx.size()) return TFS_ERROR;
  const int32_t* slots = reinterpret_cast<const int32_t*>(idx.data() + sizeof(IndexHeader));
  // traverse_segment_meta (index_handle.cpp:844-868)
  for (int32_t s = 0; s < nb; ++s) {
    size_t guard = 0;
    for (int32_t pos = slots[s]; pos != 0;) {
      if (pos < 0 || pos >= header->index_file_size_ || size_t(pos) + sizeof(MetaInfo) > idx.size() ||
          ++guard > idx.size() / sizeof(MetaInfo))
        return TFS_ERROR;  // EXIT_META_OFFSET_ERROR
      MetaInfo mi;
      memcpy(&mi, idx.data() + pos, sizeof mi);
      metas->push_back(mi.raw_meta_);  // size keeps its flag bits; LoadedBlock splits them
      pos = mi.next_meta_offset_;
    }
  }
  std::stable_sort(metas->begin(), metas->end(),
                   [](const tfs_raw_meta& a, const tfs_raw_meta& b) { return a.offset < b.offset; });  // RawMetaSort
  return TFS_SUCCESS;
}

int read_data(const BlockStore& st, const std::vector<uint32_t>& chain, char* dst, int64_t size) {
  int64_t done = 0;
  for (size_t k = 0; k < chain.size() && done < size; ++k) {
    const bool main = k == 0;
    const int64_t area = (main ? st.main_block_size : st.ext_block_size) - kReserve;
    const int64_t n = std::min(area, size - done);
    Fd f(open((main ? main_path(st, chain[k]) : ext_path(st, chain[k])).c_str(), O_RDONLY));
    if (f.fd < 0 || pread_all(f.fd, dst + done, size_t(n), kReserve)) return TFS_ERROR;
    done += n;
  }
  return done == size ? TFS_SUCCESS : TFS_ERROR;  // EXIT_PHYSIC_BLOCK_OFFSET_ERROR
}

int read_range(const BlockStore& st, const std::vector<uint32_t>& chain, char* dst, int64_t off, int64_t len) {
  if (off < 0 || len < 0) return TFS_EXIT_PARAMETER_ERROR;
  int64_t base = 0;
  for (size_t k = 0; k < chain.size() && len > 0; ++k) {
    const bool main = k == 0;
    const int64_t area = (main ? st.main_block_size : st.ext_block_size) - kReserve;
    if (off < base + area) {
      const int64_t n = std::min(len, base + area - off);
      Fd f(open((main ? main_path(st, chain[k]) : ext_path(st, chain[k])).c_str(), O_RDONLY));
      if (f.fd < 0 || pread_all(f.fd, dst, size_t(n), off_t(kReserve + off - base))) return TFS_ERROR;
      dst += n;
      off += n;
      len -= n;
    }
    base += area;
  }
  return len == 0 ? TFS_SUCCESS : TFS_ERROR;  // EXIT_PHYSIC_BLOCK_OFFSET_ERROR
}

// LogicBlock::get_real_flag (logic_block.cpp:996-1009): the index entry's unlink
// bits when its use-index bit is set, the FileInfo's flag_ otherwise.
int32_t index_flag(int32_t raw_size, const tfs_file_info& fi) {
  return (raw_size & kUseIndexFlag) ? (raw_size & kUnlinkMask) >> kUnlinkShift : fi.flag_;
}

// A file's flag as FileIterator::next sees it for a file read from its window
// (logic_block.cpp:1250-1273): FI_INVALID when the FileInfo disagrees with the
// index entry, else index_flag.  (A big file takes index_flag with no such
// check, :1221-1240.)
int32_t real_flag(const tfs_raw_meta& m, int32_t raw_size, const tfs_file_info& fi) {
  if (fi.id_ != m.file_id || fi.size_ != m.size) return TFS_FI_INVALID;
  return index_flag(raw_size, fi);
}

// Pinned when a ctx is given (direct DMA); plain heap memory otherwise
// (host-only tools and tests).
static void free_buf(tfs_crc_ctx* ctx, char* p) {
  if (!p) return;
  if (ctx) tfs_crc32_host_free_pinned(ctx, p);
  else free(p);
}

LoadedBlock::~LoadedBlock() { free_buf(ctx_, data_); }

int LoadedBlock::load(const BlockStore& st, uint32_t main_id) {
  int rc = load_chain(st, main_id, &chain, &logic_block_id);
  if (rc) return rc;
  rc = load_index(st, main_id, &header, &metas);
  if (rc) return rc;
  size_ = header.data_file_offset_;
  if (size_ < 0) return TFS_ERROR;
  if (size_ > cap_) {
    free_buf(ctx_, data_);
    data_ = nullptr;
    void* p = nullptr;
    if (ctx_) {
      rc = tfs_crc32_host_malloc_pinned(ctx_, uint64_t(size_), &p);
      if (rc) return rc;
    } else if (!(p = malloc(size_t(size_ ? size_ : 1)))) {
      return TFS_ERROR;
    }
    data_ = static_cast<char*>(p);
    cap_ = size_;
  }
  rc = read_data(st, chain, data_, size_);
  if (rc) return rc;
  // Real flag of every file as FileIterator sees it (logic_block.cpp:1250-1273):
  // FI_INVALID when the FileInfo disagrees with the index, else
  // LogicBlock::get_real_flag (:996-1009) -- the index entry's unlink bits when
  // its use-index bit is set, the FileInfo's flag_ otherwise.
  flags.assign(metas.size(), 0);
  for (size_t i = 0; i < metas.size(); ++i) {
    tfs_raw_meta& m = metas[i];
    const int32_t raw = m.size;
    m.size = raw & kFileSizeMask;  // RawMeta::get_size
    if (m.offset < 0 || int64_t(m.offset) + TFS_FILEINFO_SIZE > size_) {
      flags[i] = TFS_FI_INVALID;
      continue;
    }
    tfs_file_info fi;
    memcpy(&fi, data_ + m.offset, sizeof fi);
    flags[i] = real_flag(m, raw, fi);
  }
  return TFS_SUCCESS;
}

int verify_block_files(tfs_crc_ctx* ctx, const BlockStore& st, uint32_t main_id, std::vector<int32_t>* status,
                       BlockCrcChecker* checker) {
  LoadedBlock b(ctx);
  int rc = b.load(st, main_id);
  if (rc) return rc;
  std::vector<tfs_raw_meta> live;
  for (size_t i = 0; i < b.metas.size(); ++i)
    if (!(b.flags[i] & (TFS_FI_DELETED | TFS_FI_INVALID))) live.push_back(b.metas[i]);
  status->assign(live.size(), TFS_SUCCESS);
  uint32_t nbad = 0;
  rc = tfs_block_verify(ctx, b.data(), uint64_t(b.size()), live.data(), uint32_t(live.size()), nullptr,
                        status->data(), &nbad);
  if (rc != TFS_SUCCESS && rc != TFS_EXIT_CHECK_CRC_ERROR) return rc;
  if (checker)
    for (size_t i = 0; i < live.size(); ++i)
      if ((*status)[i] == TFS_EXIT_CHECK_CRC_ERROR) checker->add_crc_error(b.logic_block_id, live[i].file_id);
  return int(nbad);
}

// ---- compaction from block files ---------------------------------------------

namespace {

// Page-locked host memory that the GPU addresses directly (zero-copy), or
// (device = true) device memory with no host view.
struct PinnedArena {
  tfs_crc_ctx* ctx = nullptr;
  bool device = false;
  char* p = nullptr;
  char* dev = nullptr;
  uint64_t cap = 0;
  ~PinnedArena() {
    if (device && dev) tfs_crc32_dev_free(ctx, dev);
    if (!device && p) tfs_crc32_host_free_pinned(ctx, p);
  }
  // Grow to at least n bytes, keeping the first `keep` bytes (host arenas).
  int grow(uint64_t n, uint64_t keep = 0) {
    if (n <= cap) return TFS_SUCCESS;
    const uint64_t c = std::max<uint64_t>(n, cap * 2);
    void* q = nullptr;
    if (device) {
      const int rc = tfs_crc32_dev_malloc(ctx, c, &q);
      if (rc) return rc;
      if (dev) tfs_crc32_dev_free(ctx, dev);
      dev = static_cast<char*>(q);
      cap = c;
      return TFS_SUCCESS;
    }
    int rc = tfs_crc32_host_malloc_pinned(ctx, c, &q);
    if (rc) return rc;
    if (p) {
      if (keep) memcpy(q, p, size_t(std::min(keep, cap)));
      tfs_crc32_host_free_pinned(ctx, p);
    }
    p = static_cast<char*>(q);
    cap = c;
    void* d = nullptr;
    rc = tfs_crc32_host_device_ptr(ctx, p, &d);
    dev = static_cast<char*>(d);
    return rc;
  }
};

// One GPU launch worth of windows: source windows back to back in `src`, their
// live records repacked back to back in `dst`.
struct WindowGroup {
  struct Win {
    uint64_t dst_slot;  // offset of the window's new bytes in dst
    int64_t dst_off;    // ... and in the destination logic block
    int64_t dst_len;
  };
  PinnedArena src, dst, jobs, status, d_status;  // statuses: device, then copied to `status`
  void* stream = nullptr;
  std::vector<Win> wins;
  std::vector<size_t> file_idx;  // CompactFilesResult::status slot of each job
  uint64_t src_used = 0, dst_used = 0;
  uint32_t njobs = 0;
  bool inflight = false;
};

// The new block's bytes go to the destination files on a writer thread, in the
// order they were queued, while the compaction thread reads the next windows
// (the reference's task thread does both in turn: task.cpp:753-836).  A group's
// write buffer is refilled by its next launch only after wait_idle().
class AsyncWriter {
 public:
  // threaded = false: post() runs the write at once on the caller's thread.
  explicit AsyncWriter(bool threaded) : threaded_(threaded) {
    if (threaded_) th_ = std::thread([this] { run(); });
  }
  ~AsyncWriter() {
    if (!threaded_) return;
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void post(std::function<int()> f) {
    if (!threaded_) {
      if (!rc_) rc_ = f();
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_all();
  }
  // Every queued write done; the first failure, if any.
  int wait_idle() {
    if (!threaded_) return rc_;
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return q_.empty() && !busy_; });
    return rc_;
  }

 private:
  void run() {
    for (;;) {
      std::function<int()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        f = std::move(q_.front());
        q_.pop_front();
        busy_ = true;
      }
      const int r = rc_ ? rc_ : f();  // after a failure the rest is not written
      {
        std::lock_guard<std::mutex> g(mu_);
        busy_ = false;
        if (r && !rc_) rc_ = r;
      }
      cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<int()>> q_;
  const bool threaded_;
  bool busy_ = false, stop_ = false;
  int rc_ = TFS_SUCCESS;
  std::thread th_;
};

}  // namespace

struct BlockFileCompactor::Impl {
  tfs_crc_ctx* ctx;
  int K;
  int setup_rc = TFS_SUCCESS;
  WindowGroup groups[2];
  Impl(tfs_crc_ctx* c, int windows_per_launch) : ctx(c), K(std::max(1, std::min(windows_per_launch, 64))) {
    if (!ctx) {
      setup_rc = TFS_EXIT_PARAMETER_ERROR;
      return;
    }
    const uint64_t kWin = uint64_t(kMaxCompactReadSize);
    for (WindowGroup& g : groups) {
      g.src.ctx = g.dst.ctx = g.jobs.ctx = g.status.ctx = g.d_status.ctx = ctx;
      g.d_status.device = true;
      // 128 bytes of slack past the last window: the record kernel's stripe grid
      // may read up to 112 bytes past a record's payload (make_geo).
      int rc;
      if ((rc = g.src.grow(uint64_t(K) * kWin + 256)) || (rc = g.dst.grow(uint64_t(K) * kWin + 256)) ||
          (rc = g.jobs.grow(4096 * sizeof(tfs_compact_job))) || (rc = g.status.grow(4096 * 4)) ||
          (rc = g.d_status.grow(4096 * 4)) || (rc = tfs_crc32_stream_create(ctx, &g.stream))) {
        setup_rc = rc;
        return;
      }
    }
  }
  ~Impl() {
    for (WindowGroup& g : groups)
      if (g.stream) tfs_crc32_stream_destroy(ctx, g.stream);
  }
  int compact(const BlockStore& src, uint32_t src_main_id, const BlockStore& dst, uint32_t dst_main_id,
              uint32_t first_ext_id, int32_t bucket_size, CompactFilesResult* out);
};

BlockFileCompactor::BlockFileCompactor(tfs_crc_ctx* ctx, int windows_per_launch)
    : impl_(new Impl(ctx, windows_per_launch)) {}
BlockFileCompactor::~BlockFileCompactor() { delete impl_; }
int BlockFileCompactor::compact(const BlockStore& src, uint32_t src_main_id, const BlockStore& dst,
                                uint32_t dst_main_id, uint32_t first_ext_id, int32_t bucket_size,
                                CompactFilesResult* out) {
  return impl_->compact(src, src_main_id, dst, dst_main_id, first_ext_id, bucket_size, out);
}

int compact_block_files(tfs_crc_ctx* ctx, const BlockStore& src, uint32_t src_main_id, const BlockStore& dst,
                        uint32_t dst_main_id, uint32_t first_ext_id, int32_t bucket_size, int windows_per_launch,
                        CompactFilesResult* out) {
  BlockFileCompactor c(ctx, windows_per_launch);
  return c.compact(src, src_main_id, dst, dst_main_id, first_ext_id, bucket_size, out);
}

int BlockFileCompactor::Impl::compact(const BlockStore& src, uint32_t src_main_id, const BlockStore& dst,
                                      uint32_t dst_main_id, uint32_t first_ext_id, int32_t bucket_size,
                                      CompactFilesResult* out) {
  if (!out) return TFS_EXIT_PARAMETER_ERROR;
  *out = CompactFilesResult();
  if (setup_rc) return setup_rc;
  for (WindowGroup& g : groups) {  // a previous call that failed part-way may have left a group queued
    if (g.inflight) (void)tfs_crc32_stream_sync(ctx, g.stream);
    g.wins.clear();
    g.file_idx.clear();
    g.src_used = g.dst_used = 0;
    g.njobs = 0;
    g.inflight = false;
  }
  std::vector<uint32_t> chain;
  uint32_t logic_id = 0;
  int rc = load_chain(src, src_main_id, &chain, &logic_id);
  if (rc) return rc;
  // The reference always compacts into another logic block.  ChainWriter opens
  // the destination files with O_TRUNC before any source window is read, so a
  // destination file that IS a source file (same inode: the same mount and id,
  // an overlapping extension id, a symlinked or hard-linked path) would destroy
  // the block: refuse that before anything is opened for writing.
  {
    std::set<std::pair<dev_t, ino_t>> src_files;
    auto add = [&](const std::string& p) {
      struct stat sb;
      if (stat(p.c_str(), &sb) == 0) src_files.insert({sb.st_dev, sb.st_ino});
    };
    for (size_t k = 0; k < chain.size(); ++k) add(k == 0 ? main_path(src, chain[k]) : ext_path(src, chain[k]));
    add(index_path(src, src_main_id));
    auto clash = [&](const std::string& p) {
      struct stat sb;
      return stat(p.c_str(), &sb) == 0 && src_files.count({sb.st_dev, sb.st_ino}) != 0;
    };
    bool bad = clash(main_path(dst, dst_main_id)) || clash(index_path(dst, dst_main_id));
    for (int k = 0; k + 1 < kMaxChain && !bad; ++k) bad = clash(ext_path(dst, first_ext_id + uint32_t(k)));
    if (bad) return TFS_EXIT_PARAMETER_ERROR;
  }
  IndexHeader h;
  std::vector<tfs_raw_meta> metas;  // sorted by offset, sizes with their flag bits
  rc = load_index(src, src_main_id, &h, &metas);
  if (rc) return rc;
  const int64_t data_size = h.data_file_offset_;
  const uint64_t kWin = uint64_t(kMaxCompactReadSize);
  ChainWriter w(dst, dst_main_id, first_ext_id, logic_id);
  int64_t dest_off = 0;
  int cur = 0;
  // TFS_DS_COMPACT_WRITER=1 (measurement): the new bytes go out on a writer
  // thread while the next windows are read; default: written in turn by this
  // thread, as the reference's task thread does.
  static const bool kAsyncWrites = getenv("TFS_DS_COMPACT_WRITER") && atoi(getenv("TFS_DS_COMPACT_WRITER")) != 0;
  AsyncWriter writer(kAsyncWrites);  // declared after w: joined (every queued write done) before w goes

  auto submit = [&](WindowGroup& g) -> int {
    if (g.inflight || g.wins.empty()) return TFS_SUCCESS;
    // The launch rewrites g.dst: the writes queued from it must be done.
    if (const int r = writer.wait_idle()) return r;
    g.inflight = true;
    if (g.njobs == 0) return TFS_SUCCESS;
    ++out->launches;
    int r = tfs_compact_jobs_device(ctx, g.src.dev, g.src.cap, reinterpret_cast<const tfs_compact_job*>(g.jobs.dev),
                                    g.njobs, g.dst.dev, nullptr, reinterpret_cast<int32_t*>(g.d_status.dev), nullptr,
                                    g.stream);
    // The verdicts come back by a copy on the same stream, which also orders the
    // kernel's stores into the page-locked write buffer before the host reads it
    // (as tfs_blocks_compact's zero-copy path does).
    if (!r) r = tfs_crc32_memcpy(ctx, g.status.p, g.d_status.dev, uint64_t(g.njobs) * 4, g.stream);
    return r;
  };
  // Wait for a group, append its new bytes to the destination, take its verdicts.
  auto drain = [&](WindowGroup& g) -> int {
    if (!g.inflight) return TFS_SUCCESS;
    int r = tfs_crc32_stream_sync(ctx, g.stream);
    if (r) return r;
    writer.post([&w, wins = g.wins, dp = g.dst.p]() -> int {
      for (const WindowGroup::Win& win : wins)
        if (win.dst_len)
          if (const int wr = w.write(dp + win.dst_slot, win.dst_len, win.dst_off)) return wr;
      return TFS_SUCCESS;
    });
    if (!kAsyncWrites && (r = writer.wait_idle())) return r;  // written in turn: its failure now
    const int32_t* st = reinterpret_cast<const int32_t*>(g.status.p);
    for (uint32_t j = 0; j < g.njobs; ++j) {
      out->status[g.file_idx[j]] = st[j];
      if (st[j] != TFS_SUCCESS) ++out->n_bad;
    }
    g.wins.clear();
    g.file_idx.clear();
    g.src_used = g.dst_used = 0;
    g.njobs = 0;
    g.inflight = false;
    return TFS_SUCCESS;
  };
  // Read source bytes [w0, w1) holding metas [i0, i1) as the next window of the
  // current group and queue its live records.
  auto add_window = [&](int64_t w0, int64_t w1, size_t i0, size_t i1) -> int {
    int r;
    if (groups[cur].wins.size() == size_t(K)) {
      if ((r = submit(groups[cur]))) return r;
      cur ^= 1;
      if ((r = drain(groups[cur]))) return r;
    }
    WindowGroup& g = groups[cur];
    const uint64_t slot = g.src_used;
    char* buf = g.src.p + slot;
    if ((r = read_range(src, chain, buf, w0, w1 - w0))) return r;
    WindowGroup::Win win{g.dst_used, dest_off, 0};
    for (size_t i = i0; i < i1; ++i) {
      tfs_raw_meta m = metas[i];
      const int32_t raw = m.size;
      m.size = raw & kFileSizeMask;  // RawMeta::get_size
      // A record shorter than its FileInfo, or running past the block's data,
      // cannot be read whole.  FileIterator would hand it on with whatever
      // bytes follow the data area (parity unpinned: no fixture covers it);
      // here it is not copied, and reported (out->dropped) so the caller sees it.
      if (m.size < TFS_FILEINFO_SIZE || int64_t(m.offset) + m.size > w1) {
        out->dropped.push_back(m.file_id);
        continue;
      }
      tfs_file_info fi;
      memcpy(&fi, buf + (m.offset - w0), sizeof fi);
      const int32_t flag = real_flag(m, raw, fi);
      if (flag & (TFS_FI_DELETED | TFS_FI_INVALID)) continue;  // task.cpp:747-751
      if ((r = g.jobs.grow(uint64_t(g.njobs + 1) * sizeof(tfs_compact_job), uint64_t(g.njobs) * sizeof(tfs_compact_job))) ||
          (r = g.status.grow(uint64_t(g.njobs + 1) * 4)) || (r = g.d_status.grow(uint64_t(g.njobs + 1) * 4)))
        return r;
      tfs_compact_job& j = reinterpret_cast<tfs_compact_job*>(g.jobs.p)[g.njobs++];
      j.src_offset = slot + uint64_t(m.offset - w0);
      j.dest_offset = g.dst_used + uint64_t(win.dst_len);
      j.file_id = m.file_id;
      j.size = m.size;
      j.flag = flag;
      j.new_offset = int32_t(dest_off);  // FileInfo.offset_ = w_file_offset (task.cpp:755)
      j.reserved = 0;
      g.file_idx.push_back(out->status.size());
      out->status.push_back(TFS_SUCCESS);
      out->dest_metas.push_back(tfs_raw_meta{m.file_id, int32_t(dest_off), m.size});
      dest_off += m.size;
      win.dst_len += m.size;
    }
    g.src_used += uint64_t(w1 - w0);
    g.dst_used += uint64_t(win.dst_len);
    g.wins.push_back(win);
    ++out->windows;
    return TFS_SUCCESS;
  };
  // write_big_file (task.cpp:838-880): FileInfo, then the payload in window-sized
  // pieces, each checksummed with the previous piece's CRC as seed.
  auto big_file = [&](size_t i) -> int {
    int r;
    for (WindowGroup& g : groups)
      if ((r = submit(g)) || (r = drain(g))) return r;
    if ((r = writer.wait_idle())) return r;  // the big file's pieces follow every queued write
    tfs_raw_meta m = metas[i];
    const int32_t raw = m.size;
    m.size = raw & kFileSizeMask;
    tfs_file_info fi;
    if ((r = read_range(src, chain, reinterpret_cast<char*>(&fi), m.offset, sizeof fi))) return r;
    // FileIterator's big-file branch (logic_block.cpp:1221-1240) takes the flag
    // with no id/size check against the index, and write_big_file copies the
    // file whatever its header says (task.cpp:838-880).
    const int32_t flag = index_flag(raw, fi);
    if (flag & (TFS_FI_DELETED | TFS_FI_INVALID)) return TFS_SUCCESS;
    tfs_file_info dfi = fi;
    dfi.offset_ = int32_t(dest_off);
    dfi.size_ = dfi.usize_ = m.size;
    dfi.flag_ = flag;
    if ((r = w.write(reinterpret_cast<const char*>(&dfi), sizeof dfi, dest_off))) return r;
    char* buf = groups[0].src.p;
    uint32_t crc = 0;
    const int64_t len = int64_t(m.size) - TFS_FILEINFO_SIZE;
    for (int64_t done = 0; done < len;) {
      const int64_t n = std::min<int64_t>(int64_t(kWin), len - done);
      if ((r = read_range(src, chain, buf, m.offset + TFS_FILEINFO_SIZE + done, n))) return r;
      const tfs_crc_desc d{0, uint32_t(n), crc};
      if ((r = tfs_crc32_batch(ctx, &d, 1, buf, uint64_t(n), &crc))) return r;
      if ((r = w.write(buf, n, dest_off + TFS_FILEINFO_SIZE + done))) return r;
      done += n;
    }
    const int32_t st = crc == fi.crc_ ? TFS_SUCCESS : TFS_EXIT_CHECK_CRC_ERROR;
    if (st != TFS_SUCCESS) ++out->n_bad;
    out->status.push_back(st);
    out->dest_metas.push_back(tfs_raw_meta{m.file_id, int32_t(dest_off), m.size});
    dest_off += m.size;
    ++out->big_files;
    return TFS_SUCCESS;
  };

  if (!rc) rc = w.status();
  // FileIterator's walk: windows of whole files, each at most 8 MiB.
  int64_t w0 = -1, w1 = -1;
  size_t i0 = 0;
  for (size_t i = 0; i < metas.size() && !rc; ++i) {
    const int64_t off = metas[i].offset;
    const int64_t size = metas[i].size & kFileSizeMask;
    if (off < 0 || off >= data_size) {  // FileIterator::next: EXIT_META_OFFSET_ERROR
      rc = kExitMetaOffsetError;
      break;
    }
    const int64_t end = std::min<int64_t>(data_size, off + std::max<int64_t>(size, TFS_FILEINFO_SIZE));
    if (size > int64_t(kWin)) {  // is_big_file: flush the window, then the file on its own
      if (w0 >= 0 && (rc = add_window(w0, w1, i0, i))) break;
      w0 = -1;
      if ((rc = big_file(i))) break;
      continue;
    }
    if (w0 >= 0 && std::max(w1, end) - w0 > int64_t(kWin)) {
      if ((rc = add_window(w0, w1, i0, i))) break;
      w0 = -1;
    }
    if (w0 < 0) {
      w0 = off;
      w1 = end;
      i0 = i;
    } else {
      w1 = std::max(w1, end);
    }
  }
  if (!rc && w0 >= 0) rc = add_window(w0, w1, i0, metas.size());
  for (int k = 0; k < 2; ++k) {  // in submission order: the current group was filled last
    WindowGroup& g = groups[(cur + 1 + k) & 1];
    const int r = submit(g);
    const int r2 = drain(g);
    if (!rc) rc = r ? r : r2;
  }
  const int rw = writer.wait_idle();
  if (!rc) rc = rw;
  if (rc) return rc;
  out->dest_size = dest_off;
  out->ext_ids.assign(w.chain().begin() + 1, w.chain().end());
  // batch_write_meta (logic_block.cpp:817-857): the new metas and BlockInfo.
  BlockInfo info = h.block_info_;
  info.version_ += 1;  // VERSION_INC_STEP_DEFAULT (internal.h:183)
  info.file_count_ = int32_t(out->dest_metas.size());
  info.size_ = int32_t(dest_off);
  info.del_file_count_ = 0;
  info.del_size_ = 0;
  rc = write_index(dst, dst_main_id, info, out->dest_metas, {}, bucket_size > 0 ? bucket_size : h.bucket_size_,
                   int32_t(dest_off));
  if (rc) return rc;
  return out->n_bad ? TFS_EXIT_CHECK_CRC_ERROR : TFS_SUCCESS;
}

}  // namespace dataserver
}  // namespace tfs
