// block_store.cpp -- see block_store.h.  Host C++ (POSIX I/O); CRC work goes
// through the C ABI.
#include "block_store.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

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

int write_logic_block(const BlockStore& st, uint32_t main_id, uint32_t first_ext_id, const LogicBlockImage& img,
                      int32_t bucket_size, std::vector<uint32_t>* ext_ids) {
  if (bucket_size <= 0 || st.main_block_size <= kReserve || st.ext_block_size <= kReserve)
    return TFS_EXIT_PARAMETER_ERROR;
  mkdir(st.mount.c_str(), 0755);
  mkdir((st.mount + "/extend").c_str(), 0755);
  mkdir((st.mount + "/index").c_str(), 0755);
  const int64_t size = img.data_size();
  const char* data = img.data().data();
  // Physical blocks: main, then extension blocks until the data fits (extend_block).
  std::vector<uint32_t> chain{main_id};
  int64_t avail = st.main_block_size - kReserve;
  while (avail < size) {
    chain.push_back(first_ext_id + uint32_t(chain.size() - 1));
    avail += st.ext_block_size - kReserve;
    if (int(chain.size()) > kMaxChain) return TFS_EXIT_PARAMETER_ERROR;
  }
  if (ext_ids) ext_ids->assign(chain.begin() + 1, chain.end());
  int64_t done = 0;
  for (size_t k = 0; k < chain.size(); ++k) {
    const bool main = k == 0;
    const int32_t blen = main ? st.main_block_size : st.ext_block_size;
    Fd f(open((main ? main_path(st, chain[k]) : ext_path(st, chain[k])).c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644));
    if (f.fd < 0) return TFS_ERROR;
    std::vector<char> reserve(kReserve, 0);
    BlockPrefix bp{img.block_id(), main ? 0u : chain[k - 1], k + 1 < chain.size() ? chain[k + 1] : 0u, 0u, 0u};
    memcpy(reserve.data(), &bp, sizeof bp);
    if (pwrite_all(f.fd, reserve.data(), reserve.size(), 0)) return TFS_ERROR;
    const int64_t n = std::min<int64_t>(blen - kReserve, size - done);
    if (n > 0 && pwrite_all(f.fd, data + done, size_t(n), kReserve)) return TFS_ERROR;
    done += std::max<int64_t>(n, 0);
    if (ftruncate(f.fd, blen)) return TFS_ERROR;  // physical blocks are preallocated files
  }
  // Index: header, zeroed buckets, then one MetaInfo per file in write order.
  const std::vector<tfs_raw_meta> metas = img.sorted_metas();
  IndexHeader h;
  memset(&h, 0, sizeof h);
  h.block_info_.block_id_ = img.block_id();
  h.block_info_.seq_no_ = 1;
  h.block_info_.version_ = int32_t(metas.size());
  h.bucket_size_ = bucket_size;
  h.index_file_size_ = int32_t(sizeof(IndexHeader) + size_t(bucket_size) * 4);
  h.data_file_offset_ = int32_t(size);
  std::vector<char> idx(size_t(h.index_file_size_) + metas.size() * sizeof(MetaInfo), 0);
  int32_t* slots = reinterpret_cast<int32_t*>(idx.data() + sizeof(IndexHeader));
  const std::vector<int32_t> flags = img.sorted_flags();
  for (size_t i = 0; i < metas.size(); ++i) {
    const int32_t slot = int32_t(uint32_t(metas[i].file_id) % uint32_t(bucket_size));
    const int32_t at = h.index_file_size_;
    h.index_file_size_ += int32_t(sizeof(MetaInfo));  // hash_insert: expand the index file
    MetaInfo mi{metas[i], 0};
    if (flags[i]) {
      // LogicBlock::unlink_file: the flag goes into the index entry
      // (RawMeta::set_unlink_flag, internal.h:610-614 -- bits 28-30 plus the
      // use-index bit 27); the FileInfo on disk keeps its old flag_.
      mi.raw_meta_.size = (mi.raw_meta_.size & kFileSizeMask) | ((flags[i] << kUnlinkShift) & kUnlinkMask) |
                          kUseIndexFlag;
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
    h.block_info_.file_count_ += 1;
    h.block_info_.size_ += metas[i].size;
    if (flags[i] & TFS_FI_DELETED) {
      h.block_info_.del_file_count_ += 1;
      h.block_info_.del_size_ += metas[i].size;
    }
    if (uint32_t(metas[i].file_id) >= h.block_info_.seq_no_) h.block_info_.seq_no_ = uint32_t(metas[i].file_id) + 1;
  }
  memcpy(idx.data(), &h, sizeof h);
  Fd f(open(index_path(st, main_id).c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644));
  if (f.fd < 0) return TFS_ERROR;
  return pwrite_all(f.fd, idx.data(), idx.size(), 0);
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
    if (fi.id_ != m.file_id || fi.size_ != m.size) flags[i] = TFS_FI_INVALID;
    else flags[i] = (raw & kUseIndexFlag) ? (raw & kUnlinkMask) >> kUnlinkShift : fi.flag_;
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

}  // namespace dataserver
}  // namespace tfs
