// ds_harness.h -- dataserver-shaped host code that calls the CRC path only
// through the C ABI (include/tfs_crc.h), exactly as TFS's dataserver call sites
// would after the drop-in.  Host C++ only (no HIP): this is what a dataserver
// links.  Names and semantics mirror the reference (simonsysu/tfs, TFS 2.3.0):
//
//   DataFile              src/dataserver/data_file.{h,cpp}        (write staging, get_crc)
//   CloseFileInfo         src/common/internal.h:716-726
//   LogicBlockImage       src/dataserver/logic_block.cpp:156-372  (FileInfo|payload records, index)
//   close_write_file      src/dataserver/data_management.cpp:173-236 (crc compare, persist)
//   CloseBatcher          the async batching queue across leases (SURVEY §7 "Batching vs. latency")
//   verify_file/_block    src/dataserver/sync_backup.cpp:315-472, block_console.cpp:502-613
//   BlockCrcChecker       src/dataserver/block_checker.cpp:58-182, block_status.h:40-52
//   compact_block         src/dataserver/task.cpp:713-836 (+ re-CRC verify)
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/tfs_crc.h"

namespace tfs {
namespace dataserver {

// DataFile (data_file.h:33-96): per-lease payload buffer, 2 MiB in memory,
// spilled to work_dir/tmp/<fn>.dat beyond that (data_file.cpp:73-101).
class LeaseBufferPool;

class DataFile {
 public:
  static const int32_t WRITE_DATA_TMPBUF_SIZE = 2 * 1024 * 1024;  // data_file.h:78

  // pool: the lease's 2 MiB buffer comes from it when one is free (page-locked,
  // so the close's GPU check reads the payload where set_data put it), else from
  // the heap as in the reference.
  DataFile(uint64_t fn, const std::string& tmp_dir, tfs_crc_ctx* ctx, LeaseBufferPool* pool = nullptr);
  ~DataFile();
  DataFile(const DataFile&) = delete;
  DataFile& operator=(const DataFile&) = delete;

  // data_file.cpp:65-113: returns len on success, TFS_SUCCESS for len <= 0, <0 on error.
  int set_data(const char* data, int32_t len, int32_t offset);
  // data_file.cpp:115-166 (data == NULL: return the inner buffer).
  char* get_data(char* data, int32_t* len, int32_t offset);
  int32_t get_length() const { return length_; }
  // data_file.cpp:168-194 on the GPU: seed 0; > 2 MiB re-read in 2 MiB chunks
  // with the running crc as seed (each chunk one C-ABI call).  0 = "not
  // computed" and is recomputed on the next call, as in the reference (:170).
  uint32_t get_crc();
  int last_status() const { return status_; }
  void set_over();
  const char* buffer() const { return data_; }
  // The staged payload when it never spilled to the tmp file (length <= 2 MiB).
  const char* in_memory_payload() const { return fd_ == -1 ? data_ : nullptr; }
  // The pool the buffer came from (nullptr: heap).
  LeaseBufferPool* pool() const { return pool_; }

 private:
  int32_t length_ = 0;
  char* data_ = nullptr;  // data_file.h:83: a plain char array, not zero-filled
  LeaseBufferPool* pool_ = nullptr;
  uint32_t crc_ = 0;
  int fd_ = -1;
  std::string tmp_file_name_;
  tfs_crc_ctx* ctx_;
  int status_ = TFS_SUCCESS;
};

// Page-locked DataFile buffers (WRITE_DATA_TMPBUF_SIZE each) in one allocation,
// made once (DataService::initialize) like the block images of a BlockImagePool:
// a lease's payload stays where set_data copied it (data_file.cpp:104) and the
// close's GPU check reads it there, so a CloseBatcher on this pool has no
// gather copy (each member's descriptor is its buffer's offset in the pool).
// The pool must outlive every DataFile made on it and every CloseBatcher given it.
class LeaseBufferPool {
 public:
  LeaseBufferPool(tfs_crc_ctx* ctx, uint32_t nbuffers);
  ~LeaseBufferPool();
  LeaseBufferPool(const LeaseBufferPool&) = delete;
  LeaseBufferPool& operator=(const LeaseBufferPool&) = delete;
  bool ok() const { return base_ != nullptr; }
  char* take();  // nullptr when every buffer is in use
  void give(char* p);
  bool owns(const char* p) const { return p >= base_ && p < base_ + bytes(); }
  const char* base() const { return base_; }
  uint64_t bytes() const { return uint64_t(n_) * uint64_t(DataFile::WRITE_DATA_TMPBUF_SIZE); }
  uint32_t size() const { return n_; }
  uint32_t in_use() const;

 private:
  tfs_crc_ctx* ctx_;
  char* base_ = nullptr;
  uint32_t n_ = 0;
  mutable std::mutex mu_;
  std::vector<char*> free_;
};

struct CloseFileInfo {  // internal.h:716-726
  uint32_t block_id_ = 0;
  uint64_t file_id_ = 0;
  int32_t mode_ = 0;
  uint32_t crc_ = 0;
  uint64_t file_number_ = 0;
};

// The logical data area of one block (main + extension blocks stitched, as
// DataHandle presents them: data_handle.cpp:103-141) plus its index.
// Block bytes: a vector whose growth does not zero-fill (every byte below size()
// belongs to a record that its writer fills), so appends touch each page once.
// Its storage may be a page-locked arena from a BlockImagePool: a dataserver
// preallocates its blocks (BlockFileManager::bootstrap), and a page-locked image
// is verified in place -- only the named records cross PCIe, no staging copy.
struct ImageArena {
  char* p = nullptr;
  size_t cap = 0;
  std::atomic<bool> in_use{false};
};

template <typename T>
struct ImageAlloc {
  using value_type = T;
  using propagate_on_container_move_assignment = std::true_type;
  using propagate_on_container_swap = std::true_type;
  using propagate_on_container_copy_assignment = std::true_type;
  ImageArena* arena = nullptr;
  ImageAlloc() = default;
  explicit ImageAlloc(ImageArena* a) : arena(a) {}
  template <typename U>
  ImageAlloc(const ImageAlloc<U>& o) noexcept : arena(o.arena) {}
  T* allocate(size_t n) {
    if (arena && n * sizeof(T) <= arena->cap && !arena->in_use.exchange(true)) return reinterpret_cast<T*>(arena->p);
    return static_cast<T*>(::operator new(n * sizeof(T)));
  }
  void deallocate(T* p, size_t) noexcept {
    if (arena && reinterpret_cast<char*>(p) == arena->p) {
      arena->in_use = false;
      return;
    }
    ::operator delete(p);
  }
  template <typename U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <typename U, typename... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
  template <typename U>
  bool operator==(const ImageAlloc<U>& o) const noexcept { return arena == o.arena; }
  template <typename U>
  bool operator!=(const ImageAlloc<U>& o) const noexcept { return arena != o.arena; }
};
using ByteImage = std::vector<char, ImageAlloc<char>>;

// Page-locked block buffers (tfs_crc32_host_malloc_pinned on one context),
// allocated once and lent to LogicBlockImages.
class BlockImagePool {
 public:
  BlockImagePool(tfs_crc_ctx* ctx, size_t count, size_t bytes);
  ~BlockImagePool();
  ImageArena* take();  // a free arena, or nullptr (the image then lives in pageable memory)
  size_t size() const { return arenas_.size(); }
  size_t in_use() const;  // arenas lent to live images

 private:
  tfs_crc_ctx* ctx_;
  std::vector<std::unique_ptr<ImageArena>> arenas_;
};

class LogicBlockImage {
 public:
  explicit LogicBlockImage(uint32_t block_id, int64_t capacity = 64LL * 1024 * 1024, ImageArena* arena = nullptr);
  uint32_t block_id() const { return block_id_; }
  // LogicBlock::close_write_file (logic_block.cpp:156-372), insert path:
  // FileInfo{id, offset=data_offset, size=len+36, usize, mtime, ctime, flag=0, crc}|payload.
  int close_write_file(uint64_t file_id, DataFile& df, uint32_t crc);
  // Thread-safe: the record's range and index entry are taken under the lock, the
  // FileInfo|payload bytes are filled beside other writers (records are disjoint).
  int append_record(uint64_t file_id, const char* payload, int32_t len, uint32_t crc);
  // Size the image for `bytes` of records up front (a block file is preallocated on
  // disk), so appends never move it; huge pages where the kernel offers them.
  void reserve(int64_t bytes);
  // LogicBlock::read_file at offset 0 (logic_block.cpp:374-440): FileInfo|payload.
  int read_file(uint64_t file_id, std::vector<char>& out) const;
  // The full read of logic_block.cpp:374-440: *nbytes truncated to the record,
  // EXIT_META_NOT_FOUND_ERROR / EXIT_READ_OFFSET_ERROR, and on the first
  // fragment the FileInfo checks (id, real flag: FI_DELETED|FI_INVALID|
  // FI_CONCEAL rejected, only FI_INVALID with `force`) -> EXIT_FILE_INFO_ERROR.
  int read_file(uint64_t file_id, char* buf, int32_t* nbytes, int32_t offset, bool force) const;
  int set_flag(uint64_t file_id, int32_t flag);
  int32_t flag_of(uint64_t file_id) const;
  // index in offset order (traverse_sorted_segment_meta, index_handle.cpp:870-878)
  std::vector<tfs_raw_meta> sorted_metas() const;
  std::vector<int32_t> sorted_flags() const;
  const ByteImage& data() const { return data_; }
  ByteImage& data() { return data_; }
  int64_t data_size() const { return used_.load(std::memory_order_acquire); }
  void replace(ByteImage&& data, const std::vector<tfs_raw_meta>& metas, const std::vector<int32_t>& flags);

 private:
  uint32_t block_id_;
  int64_t capacity_;
  ByteImage data_;
  std::atomic<int64_t> used_{0};  // == data_.size() once every append has returned
  std::map<uint64_t, tfs_raw_meta> index_;
  std::map<uint64_t, int32_t> flags_;
  mutable std::mutex mu_;                // record ranges, index and flags
  mutable std::shared_mutex grow_mu_;    // exclusive only to move the image (growth past the reservation)
};

// DataManagement::close_write_file (data_management.cpp:173-236): CRC compare
// then persist with the computed crc.  EXIT_DATA_FILE_ERROR on mismatch.
int close_write_file(const CloseFileInfo& info, DataFile& df, LogicBlockImage& block);

// Batched closes across leases.  Leader-based: the first lease of a batch leads
// it -- it waits until max_batch leases have joined (or max_wait_us passed),
// then runs one GPU verify of every member's client CRC (tfs_crc32_verify, a
// zero-copy launch over the page-locked gather buffer).  Each member copies its
// own payload into the gather buffer (the copies run side by side) and waits
// spinning for the verdict -- no hand-off thread, no condition-variable wake-up
// on the critical path.  Up to `in_flight` batches (default kBatches) are in use
// at once, so the next batch forms while one is on the GPU.  Each member then gets the status
// close_write_file would have returned and persists its own record.  Payloads
// larger than kMaxBatched take the unbatched close.
// One close's phases (CloseBatcher::close with a CloseTiming): where its time went.
struct CloseTiming {
  double claim_us = 0;      // taking a batch slot (the batcher's lock, a free batch)
  double copy_us = 0;       // the lease's payload into the gather buffer
  double wait_us = 0;       // until the batch's verdicts are in (the leader: its verify)
  double append_us = 0;     // the FileInfo|payload append
  double lead_wait_us = 0;  // the batch's leader: from the batch's opening to its verify call
  double verify_us = 0;     // the batch's tfs_crc32_verify call
  uint32_t leader = 0;      // this close led its batch
  uint32_t batch_n = 0;     // members of its batch
  uint32_t relaunches = 0;  // resident kernel launches during the batch's verify call
  uint32_t ring_full = 0;   // ring-full launches during it
};

class CloseBatcher {
 public:
  // pool: closes of DataFiles whose buffers are in it are checked in place (no
  // gather copy); other closes through this batcher then take the unbatched path.
  CloseBatcher(tfs_crc_ctx* ctx, size_t max_batch, int max_wait_us, int in_flight = kBatches,
               LeaseBufferPool* pool = nullptr);
  ~CloseBatcher();
  // Blocks until this close has been checked (and persisted on success).
  // With `t`, the close's phases go there (the leader also reads the context's
  // counters around its verify call: tfs_crc32_stats).
  int close(const CloseFileInfo& info, DataFile& df, LogicBlockImage& block, CloseTiming* t = nullptr);
  uint64_t batches() const { return batches_.load(); }
  LeaseBufferPool* pool() const { return pool_; }

  // Leases per batch for `leases` closing threads: with the resident kernel a
  // batch costs no launch, so up to 8 threads close one file per batch (10.4 vs
  // 9.5 GiB/s in configs[0] against batches of 2 on one box; 9.1 vs 8.1 on
  // another); more threads batch leases/16 (64 -> 4: 9.1-10.4 GiB/s against 8.1-10.3
  // for 2 and 8.4-9.6 for 8), tools/loopback_probe.py, DESIGN.md §5.2.
  static size_t batch_for(size_t leases) { return leases <= 8 ? 1 : std::max<size_t>(1, leases / 16); }
  static constexpr int kBatches = 8;
  static constexpr int kMaxInFlight = 16;  // the context's synchronous slots (tfs_crc_abi.cpp kSyncSlots)
  static constexpr int32_t kMaxBatched = 2 * 1024 * 1024;  // DataFile's in-memory limit (data_file.h:78)

 private:
  struct Batch {
    char* gather = nullptr;  // page-locked (pageable `fallback` if that allocation failed)
    std::vector<char> fallback;
    std::vector<tfs_crc_vdesc> desc;
    std::vector<uint32_t> crc;
    std::vector<uint8_t> ok;
    uint32_t n = 0;           // members (under mu_)
    uint64_t bytes = 0;       // gather bytes claimed (under mu_)
    bool free = true;         // (under mu_)
    std::atomic<bool> closed{false};
    std::atomic<uint32_t> ready{0};  // members whose payload and descriptor are in place
    std::atomic<uint32_t> left{0};   // members that have not read their verdict yet
    std::atomic<int> done{0};
    int rc = TFS_SUCCESS;
    std::chrono::steady_clock::time_point opened;
    bool timed = false;  // the leader asked for timing: the fields below are filled
    double lead_wait_us = 0, verify_us = 0;
    uint32_t relaunches = 0, ring_full = 0;
  };
  static constexpr int kAppend = 1;  // checked, the closing thread persists it
  Batch* take_batch(std::unique_lock<std::mutex>& lk);
  void lead(Batch* b);
  tfs_crc_ctx* ctx_;
  size_t max_batch_;
  int max_wait_us_;
  size_t gather_cap_;  // per batch: max_batch x 256 KiB, within [4 MiB, 16 MiB]
  std::mutex mu_;
  std::condition_variable free_cv_;
  LeaseBufferPool* pool_;
  int nbatches_;
  std::unique_ptr<Batch[]> batches_buf_;
  struct Span {
    Batch *b, *e;
    Batch* begin() const { return b; }
    Batch* end() const { return e; }
  };
  Span all_batches() { return Span{batches_buf_.get(), batches_buf_.get() + nbatches_}; }
  Batch* cur_ = nullptr;  // the batch taking members (under mu_)
  std::atomic<uint64_t> batches_{0};
  std::atomic<int64_t> verify_us_{0};  // TFS_DS_TRACE diagnostics
  std::atomic<int64_t> t_claim_{0}, t_copy_{0}, t_wait_{0}, t_append_{0}, t_lead_wait_{0};
  bool trace_ = false;
};

// The CRC side of DataService on a multi-GPU node (dataservice.cpp:151-377
// creates it): a device group (include/tfs_crc.h, one context per GPU) and one
// CloseBatcher per member.  Every call is routed by block id -- the lease's
// DataFile, its close, a block's verify -- so a block's files stay on one GPU
// and nothing crosses between GPUs.
class CrcService {
 public:
  CrcService(tfs_crc_group* group, size_t max_batch, int max_wait_us);
  ~CrcService();
  tfs_crc_ctx* ctx_for_block(uint32_t block_id) const { return tfs_crc_group_ctx_for_block(group_, block_id); }
  uint32_t members() const { return tfs_crc_group_size(group_); }
  // DataManagement::close_write_file through the block's GPU batcher.
  int close_write_file(const CloseFileInfo& info, DataFile& df, LogicBlockImage& block);
  // Verify-on-read of whole blocks, each on its GPU, members concurrently
  // (tfs_crc_group_blocks_verify).  nbad[i]: bad files of blocks[i].  Returns
  // TFS_SUCCESS, TFS_EXIT_CHECK_CRC_ERROR or a device error.
  int verify_blocks(const std::vector<const LogicBlockImage*>& blocks, std::vector<uint32_t>* nbad);

 private:
  tfs_crc_group* group_;
  std::vector<std::unique_ptr<CloseBatcher>> batchers_;
};

// BlockChecker's CRC-error accounting (block_checker.cpp:58-182, block_status.h:40-52):
// per-block crc_error_ counter; >= max_crc_error_nums_ (parameter.cpp:256, default 4)
// marks the block for repair.
class BlockCrcChecker {
 public:
  explicit BlockCrcChecker(int max_crc_error_nums = 4) : max_(max_crc_error_nums) {}
  void add_crc_error(uint32_t block_id, uint64_t file_id);
  int crc_errors(uint32_t block_id) const;
  bool needs_repair(uint32_t block_id) const { return crc_errors(block_id) >= max_; }
  std::vector<std::pair<uint32_t, uint64_t>> repair_queue() const { return repair_; }

 private:
  int max_;
  std::map<uint32_t, int> errors_;
  std::vector<std::pair<uint32_t, uint64_t>> repair_;
};

// DataManagement::read_data (data_management.cpp:238-268) of a whole file plus
// the verify-on-read hook the build adds at this call site (the reference
// returns FileInfo.crc_ to the client unchecked, dataservice.cpp:1557): the
// payload is re-CRC'd on the GPU against FileInfo.crc_; a mismatch returns
// EXIT_CHECK_CRC_ERROR and is reported to `checker` (may be NULL).  `out`
// receives FileInfo|payload either way.
int read_file_verified(tfs_crc_ctx* ctx, const LogicBlockImage& block, uint64_t file_id, std::vector<char>* out,
                       BlockCrcChecker* checker);

// Verify-on-read of every live file of a block (one GPU batch); per-file status
// as sync_backup.cpp:419-435 / block_console.cpp:543-577.  Mismatches are
// reported to `checker` (may be NULL).  Returns the number of bad files or <0.
int verify_block(tfs_crc_ctx* ctx, const LogicBlockImage& block, std::vector<int32_t>* status,
                 BlockCrcChecker* checker);

// TranBlock::recombine_data (tools/transfer/block_console.cpp:502-613): every file
// of `src` in offset order, skipping FI_DELETED|FI_INVALID, id 0 (:534-539), a
// stored FileInfo that disagrees with the index entry (:543; the tool compares
// sizeof(FILEINFO_SIZE) = 4 bytes, the low half of id_) and a payload whose CRC
// is not crc_ (:569-577); the rest is repacked with offset_/size_/usize_
// rewritten and flag_ kept (FI_CONCEAL survives, :526-531,587).  One GPU verify,
// then the fused compaction pass over the survivors.  *skipped_crc: files
// dropped for their CRC.  Returns TFS_SUCCESS or a negative code.
int recombine_block(tfs_crc_ctx* ctx, const LogicBlockImage& src, LogicBlockImage& dest, int* skipped_crc);

// CompactTask::real_compact with re-CRC (task.cpp:713-836): dest receives the
// live files repacked; crc_ok per source file (1 ok / 0 mismatch / 2 skipped).
int compact_block(tfs_crc_ctx* ctx, const LogicBlockImage& src, LogicBlockImage& dest, std::vector<uint8_t>* crc_ok);

}  // namespace dataserver
}  // namespace tfs
