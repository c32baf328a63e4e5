"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports
every symbol include/tfs_crc.h declares; the ABI structs have the reference
layouts; without a GPU the library fails loudly instead of computing on the CPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
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
    with pytest.raises(crc.TfsCrcError):
        crc.func_crc(0, b"123456789")
    # len <= 0 never touches the device (func.cpp:429 loop does not run)
    assert crc.func_crc(0x1234, b"", 0) == 0x1234


def test_product_path_does_not_reference_oracle():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "tfs_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in txt.lower(), os.path.join(dirpath, f)
