"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports
every symbol include/tfs_crc.h declares; the ABI structs have the reference
layouts; without a GPU the library fails loudly instead of computing on the CPU."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HDR = os.path.join(ROOT, "include", "tfs_crc.h")
HDRS = [os.path.join(ROOT, "include", h) for h in sorted(os.listdir(os.path.join(ROOT, "include"))) if h.endswith(".h")]


def declared_functions():
    names = set()
    for h in HDRS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(tfs_\w+)\s*\(", src))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    import tfs_amd.crc as crc
    L = crc.lib()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
    import tfs_amd.ec as ec
    assert sorted(crc.EXPORTED + ec.EXPORTED) == names


def _header_functions(name):
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", name)).read(), flags=re.S)
    return set(re.findall(r"\b(tfs_\w+)\s*\(", src))


# The dataserver boundary: context, scalar, DataFile, batch, verify,
# device-resident, async, block images / compaction, packets (f1), the device
# group (§8e) and the memory / stream / event helpers a caller without a HIP
# runtime needs.  Nothing else may appear in the drop-in header.
PRODUCT_API = {
    "tfs_crc32_ctx_create", "tfs_crc32_ctx_destroy", "tfs_crc32_last_error", "tfs_crc32_device_count",
    "tfs_crc32_device_numa_node",
    "tfs_crc32", "tfs_crc32_e", "tfs_crc32_error_count", "tfs_crc32_set_default_ctx", "tfs_crc32_bind_thread",
    "tfs_crc32_default_ctx", "tfs_datafile_get_crc", "tfs_crc32_stats",
    "tfs_crc32_batch", "tfs_crc32_verify", "tfs_crc32_batch_device", "tfs_crc32_verify_device",
    "tfs_crc32_submit_verify", "tfs_crc32_wait",
    "tfs_block_verify", "tfs_block_verify_device", "tfs_block_compact", "tfs_block_compact_device",
    "tfs_compact_jobs_device", "tfs_blocks_verify_device", "tfs_blocks_compact",
    "tfs_packet_verify", "tfs_packet_verify_device", "tfs_packet_seal", "tfs_packet_seal_device",
    "tfs_crc_group_create", "tfs_crc_group_destroy", "tfs_crc_group_last_error", "tfs_crc_group_size",
    "tfs_crc_group_ctx", "tfs_crc_group_member_of", "tfs_crc_group_ctx_for_block", "tfs_crc_group_numa_node",
    "tfs_crc_group_member_bound", "tfs_crc_group_host_malloc", "tfs_crc_group_host_free",
    "tfs_crc_group_blocks_verify", "tfs_crc_group_blocks_compact",
    "tfs_crc32_dev_malloc", "tfs_crc32_dev_free", "tfs_crc32_host_malloc_pinned", "tfs_crc32_host_free_pinned",
    "tfs_crc32_host_device_ptr", "tfs_crc32_memcpy", "tfs_crc32_memset_device", "tfs_crc32_event_create",
    "tfs_crc32_event_record", "tfs_crc32_event_elapsed_ms", "tfs_crc32_event_destroy", "tfs_crc32_stream",
    "tfs_crc32_sync", "tfs_crc32_stream_create", "tfs_crc32_stream_sync", "tfs_crc32_stream_destroy",
}


def test_product_header_is_the_boundary_only():
    """include/tfs_crc.h declares exactly the §8b families, the device group and the
    memory / stream helpers; the test, calibration and tuning hooks live in
    include/tfs_crc_testing.h, and INTEGRATION.md -- what a
    dataserver maintainer reads -- names only the product header and its symbols."""
    prod = _header_functions("tfs_crc.h")
    test = _header_functions("tfs_crc_testing.h")
    assert prod == PRODUCT_API, (sorted(prod - PRODUCT_API), sorted(PRODUCT_API - prod))
    assert not prod & test
    for hook in ("tfs_crc32_inject_device_error", "tfs_crc32_synth_fill_device", "tfs_crc32_membench_device",
                 "tfs_crc32_debug_state", "tfs_crc32_set_split", "tfs_crc32_set_compact_segment"):
        assert hook in test, hook
    integ = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "tfs_crc_testing.h" not in integ
    for sym in test:
        assert sym not in integ, sym


def test_library_is_gfx950_code_object():
    so = os.path.join(ROOT, "tfs_amd", "libtfs_crc.so")
    blob = open(so, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"crc_files_kernel" in blob


def test_abi_struct_layouts():
    import tfs_amd.crc as crc
    assert crc.DESC_DTYPE.itemsize == 16
    assert crc.META_DTYPE.itemsize == 16
    assert crc.FILEINFO_DTYPE.itemsize == 36          # internal.h:432-446 pack(4)
    assert crc.FILEINFO_DTYPE.fields["crc_"][1] == 32  # crc_ at +32


@pytest.mark.parametrize("hdr", [os.path.basename(h) for h in HDRS])
def test_header_compiles_as_c(hdr):
    r = subprocess.run(["gcc", "-x", "c", "-std=c99", "-Wall", "-Werror", "-fsyntax-only",
                        os.path.join(ROOT, "include", hdr)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_no_device_fails_loudly():
    import tfs_amd.crc as crc
    if crc.device_count() > 0:
        pytest.skip("GPU present; covered by -m gpu")
    with pytest.raises(crc.TfsCrcError) as e:
        crc.Context(0)
    assert e.value.code == crc.TFS_CRC_EXIT_NO_DEVICE
    before = crc.lib().tfs_crc32_error_count()
    with pytest.raises(crc.TfsCrcError) as e2:
        crc.func_crc(0, b"123456789")
    assert e2.value.code == crc.TFS_CRC_EXIT_NO_DEVICE
    # the plain Func::crc drop-in returns its seed (no error channel) but the
    # failure is counted, never silent (include/tfs_crc.h, tfs_crc32_error_count)
    assert crc.lib().tfs_crc32(7, b"123456789", 9) == 7
    assert crc.lib().tfs_crc32_error_count() == before + 2
    assert crc.lib().tfs_crc32_default_ctx() is None
    # len <= 0 never touches the device (func.cpp:429 loop does not run)
    assert crc.func_crc(0x1234, b"", 0) == 0x1234
    assert crc.lib().tfs_crc32_error_count() == before + 2


def test_product_path_does_not_reference_oracle():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "tfs_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in txt.lower(), os.path.join(dirpath, f)


def _kernel_symbols(so):
    out = subprocess.run(["nm", "-C", so], capture_output=True, text=True, check=True).stdout
    return set(re.findall(r"(\w+_kernel(?:<[^>]*>)?)\(", out))


def test_product_library_holds_one_form_of_each_kernel():
    """The A/B kernel forms and calibration kernels live only in the measurement
    build (libtfs_crc_measure.so, -DTFS_CRC_MEASURE): the product library holds
    one crc_files_kernel per mode, no calibration copies, no membench, and never
    names TFS_CRC_VARIANT / TFS_EC_VARIANT, so no environment variable can swap
    a dataserver's kernel."""
    prod = os.path.join(ROOT, "tfs_amd", "libtfs_crc.so")
    meas = os.path.join(ROOT, "tfs_amd", "libtfs_crc_measure.so")
    blob = open(prod, "rb").read()
    assert b"TFS_CRC_VARIANT" not in blob and b"TFS_EC_VARIANT" not in blob
    assert b"TFS_CRC_VARIANT" in open(meas, "rb").read()
    kp, km = _kernel_symbols(prod), _kernel_symbols(meas)
    files_p = {k for k in kp if k.startswith("crc_files_kernel<")}
    assert len(files_p) == 2, files_p  # verify and compute
    assert len({k for k in km if k.startswith("crc_files_kernel<")}) == 4  # + one file per ticket (50)
    for name in ("membench", "compact_probe_copy_kernel", "ec_apply_chunk_kernel"):
        assert not any(name in k for k in kp), name
        assert any(name in k for k in km), name
    # the product's kernels are all in the measurement build too (same sources)
    assert files_p <= km


def test_measurement_library_only_on_request(monkeypatch):
    """Contexts load the product library unless a variant is asked for."""
    import tfs_amd.crc as crc
    monkeypatch.delenv("TFS_CRC_VARIANT", raising=False)
    monkeypatch.delenv("TFS_EC_VARIANT", raising=False)
    assert not crc.measuring()
    monkeypatch.setenv("TFS_CRC_VARIANT", "0")
    assert not crc.measuring()
    monkeypatch.setenv("TFS_CRC_VARIANT", "42")
    assert crc.measuring()
    assert crc.lib(True) is not crc.lib(False)
    for n in crc.EXPORTED:
        assert hasattr(crc.lib(True), n), n
