/*
 * oracle/crc_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's per-file CRC32 integrity path, used
 * as the parity checker for the HIP implementation and as the timed CPU
 * baseline (`cpu_baseline.kind = "port"`).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library; the product path
 * (tfs_amd/, include/) never links or calls it.
 *
 * Parity is pinned: tests/golden/ holds vectors produced by the reference's own
 * Func::crc text compiled in the survey container (oracle/gen_golden.py), and
 * tests/test_oracle.py checks every one of them against this file.
 *
 * What is restated (reference = /root/reference, TFS 2.3.0):
 *   - _crc32tab                      src/common/func.h:128-154
 *       (re-derived here from the reflected polynomial 0xEDB88320; the test
 *        suite pins the derived table against the reference's 256 values)
 *   - Func::crc(crc, data, len)      src/common/func.cpp:426-435
 *       byte loop, caller seed, no pre/post inversion, len <= 0 -> seed.
 *   - DataFile::get_crc()            src/dataserver/data_file.cpp:168-194
 *       seed 0; payloads > 2 MiB are CRC'd in 2 MiB chunks with a running
 *       seed (:183-186); a result of 0 means "not computed" (:170).
 *   - DataManagement::close_write_file CRC compare
 *                                    src/dataserver/data_management.cpp:196-203
 *   - LogicBlock::close_write_file   src/dataserver/logic_block.cpp:171-178,293-300
 *       FileInfo{id, offset, size=len+36, usize, mtime, ctime, flag=0, crc}
 *       followed by the payload.
 *   - verify-on-read                 src/dataserver/sync_backup.cpp:357-435
 *       size check (EXIT_SYNC_FILE_ERROR) before crc check (EXIT_CHECK_CRC_ERROR).
 *   - CompactTask::real_compact      src/dataserver/task.cpp:713-836
 *       skip FI_DELETED|FI_INVALID (:747-751), rewrite offset/size/usize
 *       (:753-759), copy crc_ verbatim, pack FileInfo|payload (:795-798).
 *   - packet frames                  src/common/base_packet_streamer.cpp:43-124
 *       (getPacketInfo), src/common/base_packet.cpp:100-170 (decode),
 *       :74,208 (copy/reply compute), header layout base_packet.h:33-162,
 *       little-endian Serialization (serialization.h:100-140).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define ORACLE_POLY 0xEDB88320u
#define ORACLE_FILEINFO_SIZE 36
#define ORACLE_TMPBUF_SIZE (2 * 1024 * 1024) /* data_file.h:78 WRITE_DATA_TMPBUF_SIZE */

/* TFS error codes (src/common/error_msg.h, src/common/cdefine.h) */
#define ORACLE_TFS_SUCCESS 0
#define ORACLE_EXIT_CHECK_CRC_ERROR (-1010)  /* error_msg.h:35 */
#define ORACLE_EXIT_PARAMETER_ERROR (-1016)  /* error_msg.h:41 */
#define ORACLE_EXIT_SYNC_FILE_ERROR (-8038)  /* error_msg.h:174 */
#define ORACLE_EXIT_DATA_FILE_ERROR (-8013)  /* error_msg.h:149 */

#define ORACLE_FI_DELETED 1
#define ORACLE_FI_INVALID 2

#pragma pack(push, 4)
typedef struct {
  uint64_t id_;
  int32_t offset_;
  int32_t size_;
  int32_t usize_;
  int32_t modify_time_;
  int32_t create_time_;
  int32_t flag_;
  uint32_t crc_;
} oracle_file_info; /* src/common/internal.h:432-446, 36 bytes */
#pragma pack(pop)

typedef struct {
  uint64_t offset;
  uint32_t len;
  uint32_t seed; /* or expected crc for verify */
} oracle_desc;

static uint32_t g_tab[256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void build_table(void) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ ORACLE_POLY : (c >> 1);
    g_tab[i] = c;
  }
}

static inline const uint32_t* tab(void) {
  pthread_once(&g_once, build_table);
  return g_tab;
}

void oracle_table(uint32_t* out256) { memcpy(out256, tab(), sizeof(g_tab)); }

/* Func::crc -- src/common/func.cpp:426-435 */
uint32_t oracle_crc(uint32_t crc, const char* data, int32_t len) {
  const uint32_t* t = tab();
  for (int32_t i = 0; i < len; ++i) {
    crc = (crc >> 8) ^ t[(crc ^ (uint32_t)data[i]) & 0xffu];
  }
  return crc;
}

/* One call of Func::crc per descriptor (the shape of every per-file call site). */
void oracle_crc_batch(const oracle_desc* d, uint32_t n, const char* base, uint32_t* out) {
  for (uint32_t i = 0; i < n; ++i) out[i] = oracle_crc(d[i].seed, base + d[i].offset, (int32_t)d[i].len);
}

/* A Func::crc implementation: this restatement, or the reference's own text
 * (oracle/_ref/libref_crc.so ref_func_crc) passed in by the caller. */
typedef uint32_t (*oracle_crc_fn)(uint32_t, const char*, int32_t);

typedef struct {
  const oracle_desc* d;
  const char* base;
  uint32_t* out;
  uint32_t begin, end;
  oracle_crc_fn fn;
} mt_job;

static void* mt_worker(void* arg) {
  mt_job* j = (mt_job*)arg;
  for (uint32_t i = j->begin; i < j->end; ++i)
    j->out[i] = j->fn(j->d[i].seed, j->base + j->d[i].offset, (int32_t)j->d[i].len);
  return NULL;
}

/* All-core variant with a caller-supplied Func::crc (NULL = this restatement):
 * one file per task, contiguous ranges per thread. */
int oracle_crc_batch_mt_fn(oracle_crc_fn fn, const oracle_desc* d, uint32_t n, const char* base, uint32_t* out,
                           int nthreads) {
  if (!fn) fn = oracle_crc;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  mt_job jobs[256];
  int ok[256];
  uint32_t per = (n + (uint32_t)nthreads - 1) / (uint32_t)nthreads;
  for (int t = 0; t < nthreads; ++t) {
    uint32_t b = (uint32_t)t * per, e = b + per;
    if (b > n) b = n;
    if (e > n) e = n;
    jobs[t] = (mt_job){d, base, out, b, e, fn};
    ok[t] = pthread_create(&th[t], NULL, mt_worker, &jobs[t]) == 0;
    if (!ok[t]) mt_worker(&jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t)
    if (ok[t]) pthread_join(th[t], NULL);
  return 0;
}

/* All-core variant: one file per task, contiguous ranges per thread. */
int oracle_crc_batch_mt(const oracle_desc* d, uint32_t n, const char* base, uint32_t* out, int nthreads) {
  return oracle_crc_batch_mt_fn(oracle_crc, d, n, base, out, nthreads);
}

/* DataFile::get_crc -- src/dataserver/data_file.cpp:168-194.  The >2 MiB branch
 * re-reads the spill file in WRITE_DATA_TMPBUF_SIZE chunks with a running seed. */
uint32_t oracle_datafile_get_crc(const char* data, int32_t length) {
  uint32_t crc = 0;
  if (length > ORACLE_TMPBUF_SIZE) {
    int32_t off = 0;
    while (off < length) {
      int32_t rlen = length - off > ORACLE_TMPBUF_SIZE ? ORACLE_TMPBUF_SIZE : length - off;
      crc = oracle_crc(crc, data + off, rlen);
      off += rlen;
    }
  } else {
    crc = oracle_crc(0, data, length);
  }
  return crc;
}

/*
 * Config 1 (BASELINE.json configs[0]): "src/dataserver write+verify over one 64 MB
 * block of N x len synthetic payloads, single-process loopback".
 *
 * Per file (write path): stage the payload into a DataFile-sized
 * buffer (data_file.cpp:104 memcpy), get_crc (data_file.cpp:190), compare with
 * the client crc (data_management.cpp:197), then append FileInfo|payload to the
 * block image (logic_block.cpp:171-178, 295-300).  Then verify-on-read of every
 * file: re-CRC the payload and compare with the stored FileInfo.crc_
 * (sync_backup.cpp:383, 429).
 *
 * payloads: n payloads of `len` bytes, contiguous.  client_crc: the client's CRC
 * per file (tfs_file.cpp:962-963).  image: out, >= n*(36+len) bytes.
 * Returns the number of files that failed either check.
 */
int32_t oracle_loopback_block_fn(oracle_crc_fn fn, const char* payloads, uint32_t n, int32_t len,
                                 const uint32_t* client_crc, char* stage, char* image, uint32_t* stored_crc);
int32_t oracle_loopback_block(const char* payloads, uint32_t n, int32_t len, const uint32_t* client_crc,
                              char* stage, char* image, uint32_t* stored_crc) {
  return oracle_loopback_block_fn(oracle_crc, payloads, n, len, client_crc, stage, image, stored_crc);
}

/* The same loop with a caller-supplied Func::crc (the reference text for the CPU
 * baseline; NULL = this restatement).  Payloads <= 2 MiB, as in config 1. */
int32_t oracle_loopback_block_fn(oracle_crc_fn fn, const char* payloads, uint32_t n, int32_t len,
                                 const uint32_t* client_crc, char* stage, char* image, uint32_t* stored_crc) {
  if (!fn) fn = oracle_crc;
  int32_t bad = 0;
  int64_t woff = 0;
  uint32_t written = 0;
  for (uint32_t i = 0; i < n; ++i) {
    memcpy(stage, payloads + (int64_t)i * len, (size_t)len);       /* DataFile::set_data */
    uint32_t crc = len > ORACLE_TMPBUF_SIZE ? oracle_datafile_get_crc(stage, len)
                                            : fn(0, stage, len);   /* DataFile::get_crc, data_file.cpp:190 */
    if (crc != client_crc[i]) { ++bad; continue; }                  /* EXIT_DATA_FILE_ERROR */
    oracle_file_info fi;
    memset(&fi, 0, sizeof fi);
    fi.id_ = (uint64_t)i + 1;
    fi.offset_ = (int32_t)woff;
    fi.size_ = len + ORACLE_FILEINFO_SIZE;
    fi.usize_ = fi.size_;
    fi.flag_ = 0;
    fi.crc_ = crc;
    memcpy(image + woff, &fi, ORACLE_FILEINFO_SIZE);
    memcpy(image + woff + ORACLE_FILEINFO_SIZE, stage, (size_t)len);
    if (stored_crc) stored_crc[i] = crc;
    woff += fi.size_;
    ++written;
  }
  /* verify-on-read over the block just written */
  int64_t roff = 0;
  for (uint32_t i = 0; i < written; ++i) {
    oracle_file_info fi;
    memcpy(&fi, image + roff, ORACLE_FILEINFO_SIZE);
    int32_t plen = fi.size_ - ORACLE_FILEINFO_SIZE;
    uint32_t crc = fn(0, image + roff + ORACLE_FILEINFO_SIZE, plen);
    if (crc != fi.crc_) ++bad;
    roff += fi.size_;
  }
  return bad;
}

/*
 * Verify-on-read of one file stored in a block image, with the semantics of
 * TfsMirrorBackup::copy_file (sync_backup.cpp:357-435): the first read returns
 * FileInfo|payload, FileInfo.size_ includes the 36-byte header; size check then
 * crc check.  meta_size is RawMeta.size_ (bytes incl. header) as the index holds it.
 */
int32_t oracle_verify_file(const char* image, int64_t image_len, int64_t offset, int32_t meta_size,
                           uint32_t* out_crc) {
  if (offset < 0 || offset + ORACLE_FILEINFO_SIZE > image_len || meta_size <= ORACLE_FILEINFO_SIZE)
    return ORACLE_EXIT_PARAMETER_ERROR;
  oracle_file_info fi;
  memcpy(&fi, image + offset, ORACLE_FILEINFO_SIZE);
  int32_t plen = meta_size - ORACLE_FILEINFO_SIZE;
  if (offset + meta_size > image_len) return ORACLE_EXIT_PARAMETER_ERROR;
  uint32_t crc = oracle_crc(0, image + offset + ORACLE_FILEINFO_SIZE, plen);
  if (out_crc) *out_crc = crc;
  if (fi.size_ - ORACLE_FILEINFO_SIZE != plen) return ORACLE_EXIT_SYNC_FILE_ERROR;
  return crc != fi.crc_ ? ORACLE_EXIT_CHECK_CRC_ERROR : ORACLE_TFS_SUCCESS;
}

/*
 * Compaction with the added verify: walk the file list in offset
 * order (FileIterator, logic_block.cpp:1132-1329 over traverse_sorted_segment_meta),
 * skip FI_DELETED|FI_INVALID (task.cpp:747-751; flag_ is the real flag the index
 * reports, logic_block.cpp:1272-1274), rewrite offset_/size_/usize_ (task.cpp:753-759),
 * copy crc_ verbatim and pack FileInfo|payload back to back (task.cpp:795-798).
 * The build additionally recomputes the payload CRC and compares it with the
 * stored crc_ (block_console.cpp:569-577 is the reference exemplar of that check).
 *
 * metas: n x {offset, size(incl. header)} sorted by offset; flags: real flag per file.
 * Outputs: dest image, dest_off/dest_size per input file (-1 when skipped),
 * crc_ok per input file (1 ok, 0 mismatch, 2 skipped).  Returns dest length.
 */
int64_t oracle_compact(const char* src, const int64_t* meta_off, const int32_t* meta_size, const int32_t* flags,
                       uint32_t n, char* dest, int64_t* dest_off, int32_t* dest_size, uint8_t* crc_ok) {
  int64_t w = 0;
  for (uint32_t i = 0; i < n; ++i) {
    oracle_file_info fi;
    memcpy(&fi, src + meta_off[i], ORACLE_FILEINFO_SIZE);
    int32_t plen = meta_size[i] - ORACLE_FILEINFO_SIZE;
    if (flags[i] & (ORACLE_FI_DELETED | ORACLE_FI_INVALID)) {
      dest_off[i] = -1;
      dest_size[i] = 0;
      crc_ok[i] = 2;
      continue;
    }
    uint32_t crc = oracle_crc(0, src + meta_off[i] + ORACLE_FILEINFO_SIZE, plen);
    crc_ok[i] = crc == fi.crc_ ? 1 : 0;
    oracle_file_info d = fi;
    d.offset_ = (int32_t)w;
    d.size_ = plen + ORACLE_FILEINFO_SIZE;
    d.usize_ = plen + ORACLE_FILEINFO_SIZE;
    d.flag_ = flags[i];
    memcpy(dest + w, &d, ORACLE_FILEINFO_SIZE);
    memcpy(dest + w + ORACLE_FILEINFO_SIZE, src + meta_off[i] + ORACLE_FILEINFO_SIZE, (size_t)plen);
    dest_off[i] = w;
    dest_size[i] = d.size_;
    w += d.size_;
  }
  return w;
}

/* ---- packet frames ------------------------------------------------------ */
#define ORACLE_PACKET_FLAG_V0 0x4d534654u /* base_packet.h:347 */
#define ORACLE_PACKET_FLAG_V1 0x4e534654u /* base_packet.h:348 */
#define ORACLE_TFS_ERROR (-1)
#define ORACLE_PACKET_INCOMPLETE 1
#define ORACLE_PACKET_CHECKED 2 /* internal: decode's CRC check applies */

static uint32_t le32(const unsigned char* p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

/* Classify one frame of `avail` bytes the way getPacketInfo + decode would.
 * Returns ORACLE_PACKET_CHECKED with *body, *body_len and *stored set when decode
 * checks a CRC, else the final status. */
static int32_t packet_classify(const unsigned char* p, uint32_t avail, uint32_t* body_off, int32_t* body_len,
                               uint32_t* stored) {
  uint32_t flag;
  int32_t length;
  int16_t type, check;
  int64_t data_len;
  uint32_t version;
  if (avail < 12) return ORACLE_PACKET_INCOMPLETE;             /* getPacketInfo:49 */
  flag = le32(p);
  length = (int32_t)le32(p + 4);
  type = (int16_t)(p[8] | p[9] << 8);
  check = (int16_t)(p[10] | p[11] << 8);
  if (flag == ORACLE_PACKET_FLAG_V1 && avail < 24) return ORACLE_PACKET_INCOMPLETE;  /* :65-69 */
  if ((flag != ORACLE_PACKET_FLAG_V0 && flag != ORACLE_PACKET_FLAG_V1) || length <= 0 || length > 0x4000000)
    return ORACLE_TFS_ERROR;                                   /* :78-87 */
  {
    /* header->_pcode = type_ (int16 -> int, sign-extended); V1: |= check_ << 16 (:89) */
    int32_t pcode = (int32_t)type;
    data_len = length;
    if (flag == ORACLE_PACKET_FLAG_V1) {
      pcode |= (int32_t)((uint32_t)(int32_t)check << 16);
      data_len += 12;                                          /* :93 */
    }
    version = ((uint32_t)pcode >> 16) & 0xFFFFu;               /* base_packet.cpp:104 */
  }
  if (12 + (uint64_t)data_len > avail) return ORACLE_PACKET_INCOMPLETE;
  if (version < 1) return ORACLE_TFS_SUCCESS;
  if (data_len < 12) return ORACLE_TFS_ERROR;
  *stored = le32(p + 12 + 8);                                  /* id (8) then crc (4): :117-129 */
  *body_off = 24;
  *body_len = (int32_t)(data_len - 12);                        /* :137 */
  return ORACLE_PACKET_CHECKED;
}

/* tfs_packet_verify's semantics: status per frame, computed crc (0 if none). */
uint32_t oracle_packet_verify(const char* base, const uint64_t* offset, const uint32_t* avail, uint32_t n,
                              uint32_t* out_crc, int32_t* out_status) {
  uint32_t i, bad = 0;
  for (i = 0; i < n; ++i) {
    const unsigned char* p = (const unsigned char*)base + offset[i];
    uint32_t body_off = 0, stored = 0;
    int32_t body_len = 0;
    int32_t st = packet_classify(p, avail[i], &body_off, &body_len, &stored);
    uint32_t c = 0;
    if (st == ORACLE_PACKET_CHECKED) {
      c = oracle_crc(ORACLE_PACKET_FLAG_V1, (const char*)p + body_off, body_len); /* :141 */
      st = c == stored ? ORACLE_TFS_SUCCESS : ORACLE_EXIT_CHECK_CRC_ERROR;
    }
    if (out_crc) out_crc[i] = c;
    if (out_status) out_status[i] = st;
    bad += st != ORACLE_TFS_SUCCESS;
  }
  return bad;
}

/* tfs_packet_seal's semantics: V1 frames that decode would check get their
 * header crc_ set to the body CRC (copy/reply :74,208 + streamer encode). */
void oracle_packet_seal(char* base, const uint64_t* offset, const uint32_t* avail, uint32_t n, uint32_t* out_crc,
                        int32_t* out_status) {
  uint32_t i;
  for (i = 0; i < n; ++i) {
    unsigned char* p = (unsigned char*)base + offset[i];
    uint32_t body_off = 0, stored = 0, c = 0;
    int32_t body_len = 0;
    int32_t st = packet_classify(p, avail[i], &body_off, &body_len, &stored);
    if (st == ORACLE_PACKET_CHECKED) {
      c = oracle_crc(ORACLE_PACKET_FLAG_V1, (const char*)p + body_off, body_len);
      if (le32(p) == ORACLE_PACKET_FLAG_V1) {
        p[20] = (unsigned char)c; p[21] = (unsigned char)(c >> 8);
        p[22] = (unsigned char)(c >> 16); p[23] = (unsigned char)(c >> 24);
      }
      st = ORACLE_TFS_SUCCESS;
    }
    if (out_crc) out_crc[i] = c;
    if (out_status) out_status[i] = st;
  }
}
