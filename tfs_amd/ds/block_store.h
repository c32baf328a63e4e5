// block_store.h -- TFS's on-disk block formats, read by host C++ so that
// verify-on-read and compaction can start from real block files
// (disk -> page-locked buffer -> GPU), SURVEY §8 f2.  Writing is provided for
// fixtures and benchmarks and follows the reference's write path.
//
//   physical block  <mount>/<id> (main), <mount>/extend/<id> (ext)
//                   (dataserver_define.h:36-37, physical_block.cpp:30-60):
//                   BLOCK_RESERVER_LENGTH (512) bytes whose first 24 are the
//                   BlockPrefix -- or, when <mount>/block_prefix exists, the
//                   prefix lives there at (id-1)*24 (physical_block.cpp:172-189)
//                   -- followed by block_length - 512 data bytes.
//   chain           BlockPrefix.next_physic_blockid_ from the main block through
//                   its extension blocks (logic_block.cpp:1066-1113); the logic
//                   block's data is their data areas in chain order
//                   (DataHandle::choose_physic_block, data_handle.cpp:103-141).
//   index           <mount>/index/<main id> (index_handle.cpp:30-39): IndexHeader,
//                   bucket_size int32 slots, MetaInfo nodes chained per slot
//                   (slot = uint32(file id) % bucket_size, hash_insert
//                   index_handle.cpp:1015-1060); traverse_sorted_segment_meta
//                   (:870-878) lists every RawMeta sorted by offset.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "ds_harness.h"

namespace tfs {
namespace dataserver {

#pragma pack(push, 4)
struct BlockPrefix {  // dataserver_define.h:95-107
  uint32_t logic_blockid_;
  uint32_t prev_physic_blockid_;
  uint32_t next_physic_blockid_;
  uint32_t flag_;
  uint64_t family_id_;
};
struct MetaInfo {  // dataserver_define.h:109-230
  tfs_raw_meta raw_meta_;
  int32_t next_meta_offset_;
};
#pragma pack(pop)
struct BlockInfo {  // common/internal.h:448-500
  uint32_t block_id_;
  int32_t version_;
  int32_t file_count_;
  int32_t size_;
  int32_t del_file_count_;
  int32_t del_size_;
  uint32_t seq_no_;
};
struct IndexHeader {  // index_handle.h:30-46
  BlockInfo block_info_;
  int32_t flag_;  // DirtyFlag
  int32_t bucket_size_;
  int32_t data_file_offset_;
  int32_t index_file_size_;
  int32_t free_head_offset_;
};
static_assert(sizeof(BlockPrefix) == 24 && sizeof(MetaInfo) == 20, "on-disk layout");
static_assert(sizeof(BlockInfo) == 28 && sizeof(IndexHeader) == 48, "on-disk layout");

constexpr int32_t kFileSizeMask = 0x07FFFFFF;  // internal.h:175-178: RawMeta size bits 0-26,
constexpr int32_t kUseIndexFlag = 0x08000000;  //   use-index-flag bit 27,
constexpr int32_t kUnlinkMask = 0x70000000;    //   unlink flag bits 28-30
constexpr int kUnlinkShift = 28;

struct BlockStore {
  std::string mount;
  int32_t main_block_size = 64 * 1024 * 1024;  // mainblock_size (config_item.h:132)
  int32_t ext_block_size = 32 * 1024 * 1024;   // extblock_size (config_item.h:133)
};

// A logic block being written: physical blocks are created as the data grows
// (main block first, then extension blocks first_ext_id, first_ext_id+1, ...;
// LogicBlock::extend_block, logic_block.cpp:1066-1113), each preallocated to
// its block length with its prefix chained to the previous one.  write() takes
// logic data offsets (DataHandle::write_segment_data, data_handle.cpp:103-141).
class ChainWriter {
 public:
  ChainWriter(const BlockStore& st, uint32_t main_id, uint32_t first_ext_id, uint32_t logic_id);
  ~ChainWriter();
  ChainWriter(const ChainWriter&) = delete;
  ChainWriter& operator=(const ChainWriter&) = delete;
  int write(const char* src, int64_t len, int64_t off);
  int status() const { return rc_; }
  const std::vector<uint32_t>& chain() const { return chain_; }

 private:
  int add_block(uint32_t id);
  BlockStore st_;
  uint32_t first_ext_id_, logic_id_;
  std::vector<uint32_t> chain_;
  std::vector<int> fds_;
  int rc_ = 0;
};

// The index file of a logic block: header with `info`, bucket_size empty slots,
// one MetaInfo per meta in the given order (hash_insert, index_handle.cpp:
// 1015-1060); unlink_flags (empty, or one per meta) go into the index entries.
int write_index(const BlockStore& st, uint32_t main_id, const BlockInfo& info, const std::vector<tfs_raw_meta>& metas,
                const std::vector<int32_t>& unlink_flags, int32_t bucket_size, int32_t data_size);

// Write `img` as logic block `img.block_id()`: main block <main_id>, extension
// blocks first_ext_id, first_ext_id+1, ... as needed (ids returned in
// *ext_ids), prefixes in-file, and the index with every file inserted in offset
// order.  Returns TFS_SUCCESS or a negative code.
int write_logic_block(const BlockStore& st, uint32_t main_id, uint32_t first_ext_id, const LogicBlockImage& img,
                      int32_t bucket_size, std::vector<uint32_t>* ext_ids);

// Physical ids of a logic block, main block first (follows next_physic_blockid_).
int load_chain(const BlockStore& st, uint32_t main_id, std::vector<uint32_t>* chain, uint32_t* logic_block_id);
// IndexHeader and every RawMeta as stored (size with its flag bits), sorted by offset.
int load_index(const BlockStore& st, uint32_t main_id, IndexHeader* header, std::vector<tfs_raw_meta>* metas);
// The logic block's data bytes [0, size) stitched from the chain into dst.
int read_data(const BlockStore& st, const std::vector<uint32_t>& chain, char* dst, int64_t size);
// Data bytes [off, off + len) (LogicBlock::read_raw_data).
int read_range(const BlockStore& st, const std::vector<uint32_t>& chain, char* dst, int64_t off, int64_t len);
// A file's flag as FileIterator reports it (logic_block.cpp:1250-1273):
// FI_INVALID when the FileInfo disagrees with the index entry, else
// LogicBlock::get_real_flag (:996-1009) -- the entry's unlink bits when its
// use-index bit is set, the FileInfo's flag_ otherwise.  m.size already masked.
int32_t real_flag(const tfs_raw_meta& m, int32_t raw_size, const tfs_file_info& fi);

// A block loaded for the GPU: index, chain, the FileInfo flag of every meta
// (FileIterator, logic_block.cpp:1273) and the data in page-locked memory
// (tfs_crc32_host_malloc_pinned) so that the H2D copy runs at full PCIe rate.
class LoadedBlock {
 public:
  explicit LoadedBlock(tfs_crc_ctx* ctx) : ctx_(ctx) {}
  ~LoadedBlock();
  LoadedBlock(const LoadedBlock&) = delete;
  LoadedBlock& operator=(const LoadedBlock&) = delete;
  int load(const BlockStore& st, uint32_t main_id);
  uint32_t logic_block_id = 0;
  IndexHeader header{};
  std::vector<uint32_t> chain;
  std::vector<tfs_raw_meta> metas;
  std::vector<int32_t> flags;
  const char* data() const { return data_; }
  int64_t size() const { return size_; }

 private:
  tfs_crc_ctx* ctx_;
  char* data_ = nullptr;
  int64_t size_ = 0, cap_ = 0;
};

// Verify-on-read of every live file of a block on disk (one GPU batch):
// statuses as tfs_block_verify for live files in offset order; mismatches go to
// `checker` (may be NULL).  Returns the number of bad files or < 0.
int verify_block_files(tfs_crc_ctx* ctx, const BlockStore& st, uint32_t main_id, std::vector<int32_t>* status,
                       BlockCrcChecker* checker);

// CompactTask::real_compact over block files on disk (task.cpp:713-836) with
// the build's re-CRC: the source logic block is walked in offset order through
// windows of MAX_COMPACT_READ_SIZE (8 MiB, dataserver_define.h:41) as
// FileIterator does (logic_block.cpp:1132-1329); each window is read into
// page-locked memory, and its live records are verified and repacked on the GPU
// straight into a page-locked write buffer (tfs_compact_jobs_device, zero-copy)
// whose bytes are then appended to the destination logic block
// (write_raw_data).  `windows_per_launch` windows go to the GPU in one launch,
// and the next group is read from disk while it runs.  Files larger than a
// window take write_big_file's path (task.cpp:838-880): window-sized pieces,
// their CRC chained piece to piece.  Records are copied whatever their CRC (the
// reference copies, it never verifies); status[i] is the verdict of the i-th
// file of the new block (TFS_SUCCESS or TFS_EXIT_CHECK_CRC_ERROR).  The
// destination index gets the new metas and BlockInfo{file_count_, size_ of the
// live files, del_* 0, version_ + 1 (VERSION_INC_STEP_DEFAULT), the rest
// copied} (batch_write_meta, logic_block.cpp:817-857).  Returns TFS_SUCCESS,
// TFS_EXIT_CHECK_CRC_ERROR when some file failed its CRC, or an error
// (EXIT_META_OFFSET_ERROR -8027 for a meta past the data, as FileIterator::next;
// TFS_EXIT_PARAMETER_ERROR, before anything is written, when a destination file
// would be one of the source chain's files).  A record shorter than its FileInfo
// or running past the data area is not copied and its id is listed in `dropped`.
struct CompactFilesResult {
  std::vector<tfs_raw_meta> dest_metas;
  std::vector<int32_t> status;
  std::vector<uint32_t> ext_ids;
  int64_t dest_size = 0;
  uint32_t windows = 0, launches = 0, big_files = 0, n_bad = 0;
  std::vector<uint64_t> dropped;  // ids of records that cannot be read whole (shorter than FileInfo / past the data)
};
constexpr int32_t kMaxCompactReadSize = 8388608;  // MAX_COMPACT_READ_SIZE, dataserver_define.h:41
constexpr int kExitMetaOffsetError = -8027;       // EXIT_META_OFFSET_ERROR, error_msg.h:163
int compact_block_files(tfs_crc_ctx* ctx, const BlockStore& src, uint32_t src_main_id, const BlockStore& dst,
                        uint32_t dst_main_id, uint32_t first_ext_id, int32_t bucket_size, int windows_per_launch,
                        CompactFilesResult* out);

// The same walk with its page-locked window buffers and streams kept across
// blocks (the compaction task thread's state, dataservice.cpp:2915-2918): what
// a dataserver compacting block after block holds.  Not thread-safe; one per
// compacting thread.
class BlockFileCompactor {
 public:
  BlockFileCompactor(tfs_crc_ctx* ctx, int windows_per_launch);
  ~BlockFileCompactor();
  BlockFileCompactor(const BlockFileCompactor&) = delete;
  BlockFileCompactor& operator=(const BlockFileCompactor&) = delete;
  int compact(const BlockStore& src, uint32_t src_main_id, const BlockStore& dst, uint32_t dst_main_id,
              uint32_t first_ext_id, int32_t bucket_size, CompactFilesResult* out);

 private:
  struct Impl;
  Impl* impl_;
};

}  // namespace dataserver
}  // namespace tfs
