// packet_codec.h -- the RPC packet CRC call sites of TFS (src/common/base_packet*.cpp)
// in dataserver-shaped host C++ over the C ABI (include/tfs_crc.h):
//
//   send:    BasePacket::copy / reply compute crc_ = Func::crc(TFS_PACKET_FLAG_V1,
//            stream_) (base_packet.cpp:74,208); BasePacketStreamer::encode writes
//            TfsPacketNewHeaderV1 + body (base_packet_streamer.cpp:155-200).
//            PacketEncoder batches a send queue's packets and seals all their
//            headers with one tfs_packet_seal.
//   receive: BasePacketStreamer::getPacketInfo splits the byte stream
//            (base_packet_streamer.cpp:43-124); BasePacket::decode checks the crc
//            (base_packet.cpp:100-170).  PacketDecoder walks a received buffer and
//            checks every complete frame with one tfs_packet_verify.
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/tfs_crc.h"

namespace tfs {
namespace common {

// base_packet.h:92-162 (serialized little-endian: flag, length, type, version, id, crc).
struct TfsPacketNewHeaderV1 {
  uint64_t id_ = 0;
  uint32_t flag_ = TFS_PACKET_FLAG_V1;
  uint32_t crc_ = 0;
  int32_t length_ = 0;
  int16_t type_ = 0;
  int16_t version_ = 0;
  int serialize(char* data, int64_t data_len, int64_t& pos) const;
  int deserialize(const char* data, int64_t data_len, int64_t& pos);  // all six fields
  static int64_t length() { return TFS_PACKET_HEADER_V1_SIZE; }
};

class PacketEncoder {
 public:
  explicit PacketEncoder(tfs_crc_ctx* ctx) : ctx_(ctx) {}
  // Append one V1 frame (header with crc_ 0 + body).  version >= 1 packets get
  // their crc filled in by flush(); version 0 ones are sent without (as the
  // reference's V0 encode path).
  void add(int16_t pcode, int16_t version, uint64_t id, const char* body, int32_t len);
  // Seal every pending frame (one GPU call).  TFS_SUCCESS or a negative code.
  int flush();
  const std::vector<char>& output() const { return out_; }
  void clear() { out_.clear(); frames_.clear(); }

 private:
  tfs_crc_ctx* ctx_;
  std::vector<char> out_;
  std::vector<tfs_packet_desc> frames_;
};

class PacketDecoder {
 public:
  struct Frame {
    int64_t offset = 0;   // frame start in the input
    int32_t avail = 0;    // frame bytes present
    int32_t status = 0;   // TFS_SUCCESS / TFS_EXIT_CHECK_CRC_ERROR / TFS_ERROR / TFS_PACKET_INCOMPLETE
    uint32_t crc = 0;     // computed body crc (checked frames)
  };
  explicit PacketDecoder(tfs_crc_ctx* ctx) : ctx_(ctx) {}
  // Walk [data, data+len) as getPacketInfo does and verify every frame in one
  // call.  *consumed = bytes of whole frames (a trailing incomplete frame is
  // left for the next read; a broken header ends the walk -- the reference
  // clears the connection's input there, :57-59,84).  Returns TFS_SUCCESS,
  // TFS_EXIT_CHECK_CRC_ERROR when some frame failed its check, TFS_ERROR on a
  // broken stream, or a device error.
  int decode(const char* data, int64_t len, std::vector<Frame>* frames, int64_t* consumed);

 private:
  tfs_crc_ctx* ctx_;
};

}  // namespace common
}  // namespace tfs
