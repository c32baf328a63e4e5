"""Wire frames of TFS RPC packets (host-side serialization helpers).

Restates the frame layout the packet CRC covers -- byte layout only, the CRC
itself is computed by the GPU through include/tfs_crc.h (tfs_packet_seal /
tfs_packet_verify):

  TfsPacketNewHeaderV1::serialize   src/common/base_packet.h:101-130
      flag u32, length i32, type i16, version i16, id u64, crc u32 (24 B)
  TfsPacketNewHeaderV0              src/common/base_packet.h:33-90 (first 12 B)
  Serialization::set_int*           src/common/serialization.h (little-endian)
  WriteDataMessage::serialize       src/message/write_data_message.cpp:71-96
      WriteDataInfo (internal.cpp:635-667) | vint64 ds_ | data
  BasePacketStreamer::getPacketInfo src/common/base_packet_streamer.cpp:43-124
      (frame boundaries of a received byte stream)
"""
import struct

import numpy as np

TFS_PACKET_FLAG_V0 = 0x4D534654
TFS_PACKET_FLAG_V1 = 0x4E534654
TFS_PACKET_VERSION_V0, TFS_PACKET_VERSION_V1, TFS_PACKET_VERSION_V2 = 0, 1, 2
HEADER_V0_SIZE, HEADER_V1_SIZE = 12, 24
WRITE_DATA_MESSAGE = 9          # base_packet.h:207
MAX_DATA_LEN = 0x4000000        # base_packet_streamer.cpp:81
ULONG_LONG_MAX = (1 << 64) - 1


def header_v1(length, pcode, version, pid, crc=0, flag=TFS_PACKET_FLAG_V1):
    """TfsPacketNewHeaderV1::serialize (base_packet.h:101-130)."""
    return struct.pack("<IihhQI", flag & 0xFFFFFFFF, length, pcode, version, pid & ((1 << 64) - 1),
                       crc & 0xFFFFFFFF)


def header_v0(length, pcode, check=0):
    """TfsPacketNewHeaderV0::serialize (base_packet.h:41-62)."""
    return struct.pack("<Iihh", TFS_PACKET_FLAG_V0, length, pcode, check)


def write_data_body(block_id, file_id, offset, data, is_server=0, file_number=0, ds=(), lease=None):
    """WriteDataMessage::serialize: WriteDataInfo | vint64 ds_ (+ lease triple) | data."""
    ds = list(ds)
    if lease is not None:  # has_lease(): ds_ += {ULONG_LONG_MAX, version, lease_id} (:73-78)
        version, lease_id = lease
        ds += [ULONG_LONG_MAX, version, lease_id]
    data = bytes(data)
    info = struct.pack("<IQiiiQ", block_id, file_id, offset, len(data), is_server, file_number)
    return info + struct.pack("<i", len(ds)) + b"".join(struct.pack("<Q", v) for v in ds) + data


def frame_v1(body, pcode=WRITE_DATA_MESSAGE, version=TFS_PACKET_VERSION_V2, pid=1, crc=0):
    """One V1 wire frame; crc 0 until sealed (tfs_packet_seal)."""
    return header_v1(len(body), pcode, version, pid, crc) + bytes(body)


def split_frames(buf):
    """Frame boundaries of a received stream: (offset, avail) per frame, the way
    getPacketInfo walks it (header, then length_ [+12 for V1] bytes).  Stops at a
    broken header (returned as one frame so that verify reports it) or at the
    end of the buffer (the tail is an incomplete frame)."""
    b = memoryview(bytes(buf)) if not isinstance(buf, np.ndarray) else memoryview(buf.tobytes())
    out, pos, n = [], 0, len(b)
    while pos < n:
        avail = n - pos
        if avail < HEADER_V0_SIZE:
            out.append((pos, avail))
            break
        flag, length = struct.unpack_from("<Ii", b, pos)
        if flag not in (TFS_PACKET_FLAG_V0, TFS_PACKET_FLAG_V1) or length <= 0 or length > MAX_DATA_LEN:
            out.append((pos, avail))
            break
        size = (HEADER_V1_SIZE if flag == TFS_PACKET_FLAG_V1 else HEADER_V0_SIZE) + length
        out.append((pos, min(size, avail)))
        pos += size
    return out
