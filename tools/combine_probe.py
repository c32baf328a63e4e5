"""Measurement probe (not product, not a test): time the headline verify launch
(1 M x 64 KiB files, block-image layout) with whatever libtfs_crc.so is in the
package, no result checks.  tools/combine_probe.sh runs it against the product
build and a diagnostic build without the per-file lane combine
(-DTFS_DIAG_SKIP_COMBINE, wrong CRCs), alternating, to price the combine."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tfs_amd.crc as crc  # noqa: E402

FILE, HDR, N = 65536, 36, 1 << 20
ctx = crc.Context(0)
rec = HDR + FILE
img = crc.DeviceBuffer(ctx, N * rec + 4096)
ctx.synth_fill_device(img, N * rec // 8 * 8, 1, 0)
desc = np.zeros(N, crc.DESC_DTYPE)
desc["offset"] = np.arange(N, dtype=np.uint64) * rec + HDR
desc["len"] = FILE
d_desc = crc.DeviceBuffer(ctx, desc.nbytes).upload(desc)
d_ok = crc.DeviceBuffer(ctx, N)
d_bad = crc.DeviceBuffer(ctx, 4)
ctx.verify_device(d_desc, N, img, None, d_ok, d_bad)
ms = []
for _ in range(7):
    e0, e1 = crc.Event(ctx), crc.Event(ctx)
    e0.record()
    for _ in range(3):
        ctx.verify_device(d_desc, N, img, None, d_ok, d_bad)
    e1.record()
    ctx.sync()
    ms.append(e0.elapsed_ms(e1) / 3)
ms.sort()
print(json.dumps({"build": sys.argv[1] if len(sys.argv) > 1 else "?", "median_ms": ms[3], "min_ms": ms[0]}), flush=True)
