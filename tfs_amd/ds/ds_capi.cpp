// ds_capi.cpp -- C entry points over the dataserver-shaped harness, so tests
// can drive the write / close / verify / compact call sites the way the
// reference's gtest programs drive LogicBlock/DataFile directly
// (tests/dataserver/test_logic_block_and_compact.cpp).  Host C++ only.
#include <cstring>
#include <string>

#include "ds_harness.h"

using namespace tfs::dataserver;

extern "C" {

void* tfs_ds_datafile_new(tfs_crc_ctx* ctx, uint64_t fn, const char* tmp_dir) {
  return new DataFile(fn, tmp_dir ? tmp_dir : "/tmp", ctx);
}
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

int tfs_ds_compact_block(tfs_crc_ctx* ctx, void* src, void* dest, uint8_t* crc_ok, uint32_t cap) {
  std::vector<uint8_t> ok;
  const int r = compact_block(ctx, *static_cast<LogicBlockImage*>(src), *static_cast<LogicBlockImage*>(dest), &ok);
  for (size_t i = 0; i < ok.size() && i < cap; ++i) crc_ok[i] = ok[i];
  return r;
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
