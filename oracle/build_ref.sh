#!/usr/bin/env bash
# oracle/build_ref.sh -- TEST INFRASTRUCTURE ONLY.
#
# Builds oracle/_ref/libref_crc.so from the reference's own CRC source text, so
# the golden vectors (oracle/gen_golden.py) and the CPU baseline can come from
# the reference implementation itself.
#
# The reference dataserver cannot be built here (src/common/func.h:39 pulls in
# <tbsys.h>; tbsys/tbnet are not vendored).  The CRC itself is
# self-contained, so this script compiles exactly these reference lines, read
# from /root/reference at build time and fed to g++ on stdin (no reference
# source is written into the repository or into oracle/_ref/):
#   src/common/func.h:90        static uint32_t crc(uint32_t crc, const char* data, const int32_t len);
#   src/common/func.h:128-154   static const uint32_t _crc32tab[] = {...};
#   src/common/func.cpp:426-435 uint32_t Func::crc(...) { byte loop }
# wrapped only in `namespace tfs { namespace common { struct Func { <:90> }; ... } }`
# and an extern "C" forwarder.  Flags are the reference release flags
# (configure.ac:167: -O2 -finline-functions -fno-strict-aliasing).
#
# Output: oracle/_ref/libref_crc.so (git-ignored; travels to the GPU box with
# the gpurun snapshot like every other built .so).  No-op when /root/reference
# is absent (the GPU box uses the prebuilt file).
set -euo pipefail
REF=${TFS_REFERENCE_ROOT:-/root/reference}
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
OUT="$HERE/_ref"
mkdir -p "$OUT"
if [ ! -f "$REF/src/common/func.h" ] || [ ! -f "$REF/src/common/func.cpp" ]; then
  echo "build_ref: $REF not present; keeping prebuilt $OUT/libref_crc.so if any" >&2
  exit 0
fi
{
  echo '#include <stdint.h>'
  echo 'namespace tfs { namespace common {'
  echo 'struct Func {'
  sed -n '90p' "$REF/src/common/func.h"
  echo '};'
  sed -n '128,154p' "$REF/src/common/func.h"
  sed -n '426,435p' "$REF/src/common/func.cpp"
  echo '} }'
  echo 'extern "C" uint32_t ref_func_crc(uint32_t c, const char* d, int32_t n) { return tfs::common::Func::crc(c, d, n); }'
} | g++ -x c++ -O2 -finline-functions -fno-strict-aliasing -fPIC -shared -o "$OUT/libref_crc.so" -
echo "build_ref: wrote $OUT/libref_crc.so"

# Erasure code: the reference's vendored jerasure + galois
# compile on their own (only libc headers); they are compiled in place from
# /root/reference with oracle/ec_ref_driver.cpp (ErasureCode's glue, restated).
DS="$REF/src/dataserver"
if [ -f "$DS/jerasure.cpp" ] && [ -f "$DS/galois.cpp" ]; then
  g++ -O2 -finline-functions -fno-strict-aliasing -fPIC -shared -w -I"$DS" \
    "$DS/jerasure.cpp" "$DS/galois.cpp" "$HERE/ec_ref_driver.cpp" -o "$OUT/libref_ec.so"
  echo "build_ref: wrote $OUT/libref_ec.so"
fi
