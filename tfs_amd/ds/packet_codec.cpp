// packet_codec.cpp -- see packet_codec.h.  Host C++; the CRC runs on the GPU
// through include/tfs_crc.h.
#include "packet_codec.h"

#include <cstring>

namespace tfs {
namespace common {
namespace {

// Serialization::set_int* / get_int* (serialization.h): little-endian.
void put(char* p, uint64_t v, int n) {
  for (int i = 0; i < n; ++i) p[i] = char(uint8_t(v >> (8 * i)));
}
uint64_t get(const char* p, int n) {
  uint64_t v = 0;
  for (int i = n - 1; i >= 0; --i) v = (v << 8) | uint8_t(p[i]);
  return v;
}

}  // namespace

int TfsPacketNewHeaderV1::serialize(char* data, int64_t data_len, int64_t& pos) const {
  if (!data || data_len - pos < length()) return TFS_ERROR;
  char* p = data + pos;
  put(p, flag_, 4);
  put(p + 4, uint32_t(length_), 4);
  put(p + 8, uint16_t(type_), 2);
  put(p + 10, uint16_t(version_), 2);
  put(p + 12, id_, 8);
  put(p + 20, crc_, 4);
  pos += length();
  return TFS_SUCCESS;
}

int TfsPacketNewHeaderV1::deserialize(const char* data, int64_t data_len, int64_t& pos) {
  if (!data || data_len - pos < length()) return TFS_ERROR;
  const char* p = data + pos;
  flag_ = uint32_t(get(p, 4));
  length_ = int32_t(uint32_t(get(p + 4, 4)));
  type_ = int16_t(uint16_t(get(p + 8, 2)));
  version_ = int16_t(uint16_t(get(p + 10, 2)));
  id_ = get(p + 12, 8);
  crc_ = uint32_t(get(p + 20, 4));
  pos += length();
  return TFS_SUCCESS;
}

void PacketEncoder::add(int16_t pcode, int16_t version, uint64_t id, const char* body, int32_t len) {
  TfsPacketNewHeaderV1 h;
  h.id_ = id;
  h.length_ = len;
  h.type_ = pcode;
  h.version_ = version;
  const size_t at = out_.size();
  out_.resize(at + size_t(h.length()) + size_t(len > 0 ? len : 0));
  int64_t pos = int64_t(at);
  h.serialize(out_.data(), int64_t(out_.size()), pos);
  if (len > 0) memcpy(out_.data() + pos, body, size_t(len));
  frames_.push_back(tfs_packet_desc{uint64_t(at), uint32_t(out_.size() - at), 0u});
}

int PacketEncoder::flush() {
  if (frames_.empty()) return TFS_SUCCESS;
  std::vector<int32_t> st(frames_.size());
  const int rc = tfs_packet_seal(ctx_, frames_.data(), uint32_t(frames_.size()), out_.data(), out_.size(), nullptr,
                                 st.data());
  frames_.clear();
  return rc;
}

int PacketDecoder::decode(const char* data, int64_t len, std::vector<Frame>* frames, int64_t* consumed) {
  frames->clear();
  *consumed = 0;
  std::vector<tfs_packet_desc> d;
  int64_t pos = 0;
  bool broken = false;
  while (pos < len) {
    const int64_t avail = len - pos;
    int64_t size = 0;
    if (avail >= TFS_PACKET_HEADER_V0_SIZE) {
      const uint32_t flag = uint32_t(get(data + pos, 4));
      const int32_t length = int32_t(uint32_t(get(data + pos + 4, 4)));
      if ((flag != TFS_PACKET_FLAG_V0 && flag != TFS_PACKET_FLAG_V1) || length <= 0 || length > 0x4000000) {
        broken = true;  // verify reports TFS_ERROR for it
      } else {
        size = (flag == TFS_PACKET_FLAG_V1 ? TFS_PACKET_HEADER_V1_SIZE : TFS_PACKET_HEADER_V0_SIZE) + int64_t(length);
      }
    }
    const int64_t take = broken || size == 0 || size > avail ? avail : size;
    d.push_back(tfs_packet_desc{uint64_t(pos), uint32_t(take), 0u});
    if (broken || size == 0 || size > avail) break;  // broken, or the tail waits for more bytes
    pos += size;
  }
  if (d.empty()) return TFS_SUCCESS;
  std::vector<uint32_t> crc(d.size());
  std::vector<int32_t> st(d.size());
  uint32_t nbad = 0;
  const int rc = tfs_packet_verify(ctx_, d.data(), uint32_t(d.size()), data, uint64_t(len), crc.data(), st.data(),
                                   &nbad);
  if (rc != TFS_SUCCESS && rc != TFS_EXIT_CHECK_CRC_ERROR) return rc;
  int worst = TFS_SUCCESS;
  for (size_t i = 0; i < d.size(); ++i) {
    Frame f;
    f.offset = int64_t(d[i].offset);
    f.avail = int32_t(d[i].len);
    f.status = st[i];
    f.crc = crc[i];
    frames->push_back(f);
    if (st[i] == TFS_PACKET_INCOMPLETE) break;
    *consumed = f.offset + f.avail;
    if (st[i] == TFS_ERROR) worst = TFS_ERROR;
    else if (st[i] != TFS_SUCCESS && worst == TFS_SUCCESS) worst = st[i];
  }
  return worst;
}

}  // namespace common
}  // namespace tfs
