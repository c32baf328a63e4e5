/*
 * tfs_ec.h -- C ABI of the MI355X erasure-code region kernels.
 *
 * Drop-in for tfs::dataserver::ErasureCode (src/dataserver/erasure_code.{h,cpp})
 * as MarshallingTask / ReinstateTask / DataManagement use it (task.cpp:1179-1290,
 * 1382-1480; data_management.cpp:293-400): a Cauchy Reed-Solomon code over
 * GF(2^8) (polynomial 0435) in jerasure's bitmatrix form, w = 8, packetsize =
 * 128, so every call works on whole 1 KiB units.  Output bytes are identical to
 * jerasure_bitmatrix_encode / _dotprod (jerasure.cpp:304-348,1345-1364); the
 * byte work runs on the GPU, the matrix setup on the host.
 *
 * Members: dn data + pn parity buffers ("disks"), dn + pn <= 12
 * (MAX_MARSHALLING_NUM, common/internal.h:170).  Status codes as error_msg.h.
 */
#ifndef TFS_EC_H_
#define TFS_EC_H_

#include <stdint.h>

#include "tfs_crc.h"

#ifdef __cplusplus
extern "C" {
#endif

#define TFS_EXIT_NO_MEMORY (-16000)      /* error_msg.h:216 */
#define TFS_EXIT_DATA_INVALID (-16001)   /* error_msg.h:217 */
#define TFS_EXIT_SIZE_INVALID (-16002)   /* error_msg.h:218 */
#define TFS_EXIT_MATRIX_INVALID (-16003) /* error_msg.h:219 */
#define TFS_EXIT_NO_ENOUGH_DATA (-16004) /* error_msg.h:220 */
#define TFS_EC_WORD_SIZE 8               /* ErasureCode::ws_ */
#define TFS_EC_PACKET_SIZE 128           /* ErasureCode::ps_ */
#define TFS_EC_UNIT 1024                 /* ws_ * ps_: sizes must be multiples */
#define TFS_EC_MAX_MEMBERS 12

typedef struct tfs_ec tfs_ec;

/* ErasureCode::config(dn, pn, erased) (erasure_code.cpp:49-119).  erased ==
 * NULL configures encode only; otherwise erased[dn+pn] holds 0 alive, 1 dead,
 * -1 not used, and the decoding plan is built: TFS_EXIT_NO_ENOUGH_DATA when
 * fewer than dn members are alive, TFS_EXIT_MATRIX_INVALID when the surviving
 * rows are singular.  *out is set even on failure (the coder then refuses to
 * decode) and must be released with tfs_ec_free. */
int tfs_ec_config(tfs_crc_ctx* ctx, int dn, int pn, const int* erased, tfs_ec** out);
int tfs_ec_free(tfs_ec* ec);

/* ErasureCode::encode(size) (:141-175): parity members dn..dn+pn-1 get the
 * code of data members 0..dn-1 over [0, size).  Checks in the reference's
 * order: no matrix -> TFS_EXIT_MATRIX_INVALID; size % 1024 ->
 * TFS_EXIT_SIZE_INVALID; a NULL member or sizes[i] < size ->
 * TFS_EXIT_DATA_INVALID.  Device form: members are device pointers of ctx's
 * GPU (host array of dn+pn pointers), sizes may be NULL (all large enough);
 * asynchronous on `stream`.  Host form: host buffers, synchronous. */
int tfs_ec_encode_device(tfs_ec* ec, void* const* d_members, const int* sizes, int size, void* stream);
int tfs_ec_encode(tfs_ec* ec, char* const* members, const int* sizes, int size);

/* ErasureCode::decode(size) (:177-235): rebuild every erased data member
 * (erased != 0) and every dead parity member (erased == 1) from the first dn
 * alive members.  Same checks as encode (a coder configured without `erased`
 * has no decoding matrix -> TFS_EXIT_MATRIX_INVALID). */
int tfs_ec_decode_device(tfs_ec* ec, void* const* d_members, const int* sizes, int size, void* stream);
int tfs_ec_decode(tfs_ec* ec, char* const* members, const int* sizes, int size);

#ifdef __cplusplus
}
#endif
#endif /* TFS_EC_H_ */
