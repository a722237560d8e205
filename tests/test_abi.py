"""The C ABI library loads, exports exactly what include/viterbi_amd.h declares, and its
host-only entry points behave; no GPU compute here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from helpers import CODES, REPO, load_golden

from convolutionalencdec_amd import native
from convolutionalencdec_amd.decoder import ConvCode

HEADER = os.path.join(REPO, "include", "viterbi_amd.h")


def _header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vtb_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_the_exported_list():
    assert _header_functions() == sorted(native.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], capture_output=True, text=True, check=True)
    syms = {line.split()[-1] for line in out.stdout.splitlines() if " T " in line}
    missing = [s for s in _header_functions() if s not in syms]
    assert not missing, missing
    lib = native.lib()
    for s in native.EXPORTED_SYMBOLS:
        assert hasattr(lib, s)


def test_library_carries_gfx950_code_object():
    with open(native.LIB_PATH, "rb") as fh:
        blob = fh.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_version_and_errors():
    lib = native.lib()
    assert b"gfx950" in lib.vtb_version()
    for code in (native.VTB_ERR_INVALID, native.VTB_ERR_CODE, native.VTB_ERR_UNSUPPORTED, native.VTB_ERR_DEVICE):
        assert lib.vtb_strerror(code)


@pytest.mark.parametrize("K", [5, 7, 9])
def test_edge_table_matches_reference(K):
    assert (ConvCode(K, CODES[K]).edge_table() == load_golden("edge_tables.npz")[f"k{K}"]).all()


def test_code_check():
    lib = native.lib()
    ok = native.VtbCode.make(7, CODES[7])
    assert lib.vtb_code_check(ctypes.byref(ok)) == 0
    bad = native.VtbCode.make(3, (0b111, 0b110))  # handTraced config: no symmetry
    assert lib.vtb_code_check(ctypes.byref(bad)) == native.VTB_ERR_CODE
    big = native.VtbCode.make(11, (0o3345, 0o3613))
    assert lib.vtb_code_check(ctypes.byref(big)) == native.VTB_ERR_UNSUPPORTED
    n3 = native.VtbCode.make(7, CODES[7])
    n3.coded_bits = 3
    assert lib.vtb_code_check(ctypes.byref(n3)) == native.VTB_ERR_UNSUPPORTED
    assert lib.vtb_code_check(None) == native.VTB_ERR_INVALID
    with pytest.raises(native.VtbError):
        ConvCode(3, (0b111, 0b110)).check()


def test_frame_sizes():
    lib = native.lib()
    c = native.VtbCode.make(7, CODES[7])
    assert lib.vtb_input_bytes_per_frame(ctypes.byref(c), native.VTB_INPUT_HARD, 1024) == 1030
    assert lib.vtb_input_bytes_per_frame(ctypes.byref(c), native.VTB_INPUT_SOFT8, 1024) == 2060
    assert lib.vtb_output_bytes_per_frame(1024) == 128
    assert lib.vtb_output_bytes_per_frame(1001) == 126
    assert lib.vtb_output_bytes_per_frame(0) == 0


def test_plan_without_gpu_fails_loudly():
    """No silent CPU fallback: without a gfx950 device plan creation is an error."""
    lib = native.lib()
    if lib.vtb_device_count() > 0:
        pytest.skip("a GPU is present")
    c = native.VtbCode.make(7, CODES[7])
    plan = ctypes.c_void_p()
    assert lib.vtb_plan_create(ctypes.byref(plan), ctypes.byref(c), 0, 1024, 0) == native.VTB_ERR_DEVICE
    with pytest.raises(native.VtbError):
        from convolutionalencdec_amd import ViterbiDecoder

        ViterbiDecoder(frame_bits=1024)
    coded = np.zeros(1030, np.uint8)
    out = np.zeros(128, np.uint8)
    assert lib.vtb_decode_frame_legacy(ctypes.byref(c), coded.ctypes.data_as(ctypes.c_void_p), 1030,
                                       out.ctypes.data_as(ctypes.c_void_p)) == native.VTB_ERR_DEVICE
    stream = ctypes.c_void_p()
    assert lib.vtb_stream_create(ctypes.byref(stream), ctypes.byref(c), 0, 8, 0, 0) == native.VTB_ERR_DEVICE
    k9 = native.VtbCode.make(9, CODES[9])
    assert lib.vtb_stream_create(ctypes.byref(stream), ctypes.byref(k9), 0, 8, 0, 0) == native.VTB_ERR_DEVICE
    k5 = native.VtbCode.make(5, CODES[5])
    # every K streams since round 3 (the generic stream kernel): no GPU -> device error, loudly
    assert lib.vtb_stream_create(ctypes.byref(stream), ctypes.byref(k5), 0, 8, 0, 0) == native.VTB_ERR_DEVICE


@pytest.mark.parametrize("F", [0, 1, 2, 3, 7, 100, 1001, 4096, 131072, 2**20, 2**20 + 5, 2**40 + 3])
def test_shard_range_tiles_the_batch(F):
    """The frame split of vtb_decode_host_multi / vtb_decode_peer_multi: contiguous shards that
    tile [0, F) exactly, sizes differing by at most one, for even and uneven F / G."""
    from convolutionalencdec_amd import shard_range

    for G in (1, 2, 3, 4, 5, 7, 8, 9, 16, 64):
        bounds = [shard_range(F, G, i) for i in range(G)]
        assert bounds[0][0] == 0 and bounds[-1][1] == F
        assert all(bounds[i][1] == bounds[i + 1][0] for i in range(G - 1))
        sizes = [hi - lo for lo, hi in bounds]
        assert min(sizes) >= 0 and max(sizes) - min(sizes) <= 1
        assert sum(sizes) == F


def test_shard_range_and_peer_multi_argument_errors():
    lib = native.lib()
    lo, hi = ctypes.c_size_t(), ctypes.c_size_t()
    assert lib.vtb_shard_range(10, 0, 0, ctypes.byref(lo), ctypes.byref(hi)) == native.VTB_ERR_INVALID
    assert lib.vtb_shard_range(10, 4, 4, ctypes.byref(lo), ctypes.byref(hi)) == native.VTB_ERR_INVALID
    assert lib.vtb_shard_range(10, 4, 0, None, ctypes.byref(hi)) == native.VTB_ERR_INVALID
    c = native.VtbCode.make(7, CODES[7])
    devs = (ctypes.c_int * 2)(0, 0)
    buf = ctypes.c_void_p(0x1000)
    args = (ctypes.byref(c), 0, 1024, 0, buf, buf, 16)
    assert lib.vtb_decode_peer_multi(*args, devs, 0, 0, None) == native.VTB_ERR_INVALID  # no devices
    assert lib.vtb_decode_peer_multi(*args, devs, 2, 0x80, None) == native.VTB_ERR_INVALID  # unknown flag
    bad = native.VtbCode.make(7, (0o112, 0o171))
    assert lib.vtb_decode_peer_multi(ctypes.byref(bad), 0, 1024, 0, buf, buf, 16, devs, 2, 0,
                                     None) == native.VTB_ERR_CODE
    if lib.vtb_device_count() == 0:  # no GPU here: the device check fails loudly
        assert lib.vtb_decode_peer_multi(*args, devs, 2, 0, None) == native.VTB_ERR_DEVICE
