"""The legacy C API (include/viterbiDecoder.h, convEncode.h) is layout- and
link-compatible with the reference: struct sizes and offsets match, the reference's own
harness sources compile and link against this build unchanged, and the host-side legacy
encoder reproduces the reference encoder.  CPU only (no decode calls)."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

from helpers import CODES, REPO, golden_sets, manifest

REF = "/root/reference"
LIB_DIR = os.path.join(REPO, "convolutionalencdec_amd", "lib")

PROBE = r"""
#include <stddef.h>
#include <stdio.h>
#include "convEncode.h"
#include "viterbiDecoder.h"
int main(void) {
    printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %lu\n", sizeof(viterbiHardState_t),
           offsetof(viterbiHardState_t, nodeMetricsA), offsetof(viterbiHardState_t, traceBackA),
           offsetof(viterbiHardState_t, nodeMetricsB), offsetof(viterbiHardState_t, nodeMetricsCur),
           offsetof(viterbiHardState_t, iteration), offsetof(viterbiHardState_t, renormCounter),
           offsetof(viterbiHardState_t, decodeCarryOverCount), offsetof(viterbiHardState_t, tracebackBufs),
           sizeof(convEncoderState_t), offsetof(convEncoderState_t, remainingUncodedCount), NUM_STATES);
    return 0;
}
"""


def _probe(tmp_path, inc, params):
    src = tmp_path / "probe.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=gnu11", f"-I{params}", f"-I{inc}", str(src), "-o", str(exe)], check=True,
                   capture_output=True)
    return subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()


@pytest.mark.parametrize("K", [5, 7, 9])
def test_state_struct_size_matches_reference(tmp_path, K):
    got = _probe(tmp_path, os.path.join(REPO, "include"), os.path.join(REPO, "params", f"k{K}"))
    assert int(got[0]) == manifest()["kat"]["viterbiHardState_t_sizeof"][str(K)]
    assert int(got[-1]) == 1 << (K - 1)


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")), reason="reference tree not present")
@pytest.mark.parametrize("K", [7, 9])
def test_struct_layout_identical_to_reference_headers(tmp_path, K):
    params = os.path.join(REPO, "params", f"k{K}")
    ours = _probe(tmp_path, os.path.join(REPO, "include"), params)
    ref = _probe(tmp_path, os.path.join(REF, "src"), params)
    assert ours == ref


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")), reason="reference tree not present")
@pytest.mark.parametrize("harness", ["speedDecode/speedDecode.c", "berTestK7/berTestK7.c",
                                     "speedEncode/speedEncode.c"])
def test_reference_harness_links_unchanged(tmp_path, harness):
    """The reference harness source compiles against include/ and links against the
    legacy library with no unresolved symbols (it is not run: no GPU here)."""
    exe = tmp_path / "harness"
    r = subprocess.run(["gcc", "-std=gnu11", "-O1", "-w", f"-I{os.path.join(REF, 'src', 'defaultParams')}",
                        f"-I{os.path.join(REPO, 'include')}", os.path.join(REF, harness),
                        os.path.join(REF, "src", "defaultParams", "convCodeParams.c"), f"-L{LIB_DIR}",
                        "-lviterbi_legacy_k7", "-lviterbi_amd", f"-Wl,-rpath,{LIB_DIR}", "-pthread", "-lm", "-o",
                        str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


def _legacy(K):
    L = ctypes.CDLL(os.path.join(LIB_DIR, f"libviterbi_legacy_k{K}.so"))
    v = ctypes.c_void_p
    L.resetConvEncoder.argtypes = [v]
    L.initConvEncoder.argtypes = [v]
    L.convEnc.argtypes = [v, v, v, ctypes.c_int, ctypes.c_bool]
    L.calcHammingDist.argtypes = [ctypes.c_uint8, ctypes.c_uint8, ctypes.c_int]
    L.calcHammingDist.restype = ctypes.c_uint8
    return L


@pytest.mark.parametrize("K", [5, 7, 9])
def test_legacy_encoder_matches_reference(K):
    lib = _legacy(K)
    enc = (ctypes.c_uint8 * 64)()
    for key, L, unc, rx, dec in golden_sets(K):
        if not key.endswith("p000"):
            continue
        for f in range(0, unc.shape[0], 7):
            lib.resetConvEncoder(enc)
            lib.initConvEncoder(enc)
            row = np.ascontiguousarray(unc[f])
            out = np.zeros(rx.shape[1], np.uint8)
            n = lib.convEnc(enc, row.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p), len(row),
                            True)
            assert n == rx.shape[1] and (out == rx[f]).all(), (key, f)


def test_legacy_encoder_streams_across_calls():
    """Bytes split over several last=false calls encode like one call (convEnc state)."""
    lib = _legacy(7)
    enc = (ctypes.c_uint8 * 64)()
    key, L, unc, rx, dec = next(s for s in golden_sets(7) if s[0] == "L1024_p000")
    row = np.ascontiguousarray(unc[0])
    out = np.zeros(rx.shape[1], np.uint8)
    lib.resetConvEncoder(enc)
    lib.initConvEncoder(enc)
    start, written = 0, 0
    for cut in (5, 17, 64, len(row)):
        seg = np.ascontiguousarray(row[start:cut])
        dst = out[written:]
        written += lib.convEnc(enc, seg.ctypes.data_as(ctypes.c_void_p), dst.ctypes.data_as(ctypes.c_void_p),
                               len(seg), cut == len(row))
        start = cut
    assert written == rx.shape[1]
    assert (out == rx[0]).all()


@pytest.mark.parametrize("K", [5, 7, 9])
def test_legacy_encoder_random_splits_vs_oracle(K):
    """The drop-in encoder's byte-table path (k = 1, csrc/legacy/convEncode.c) on random
    payloads split over random last=false calls, against the oracle's bit-serial encoder."""
    from helpers import Oracle

    orc = Oracle()
    lib = _legacy(K)
    enc = (ctypes.c_uint8 * 64)()
    rng = np.random.default_rng(K)
    for trial in range(20):
        nb = int(rng.integers(1, 600))
        row = rng.integers(0, 256, nb, dtype=np.uint8)
        want = orc.encode(K, CODES[K], row[None, :])[0]
        out = np.zeros(want.size + 16, np.uint8)
        lib.resetConvEncoder(enc)
        lib.initConvEncoder(enc)
        cuts = sorted(set(int(c) for c in rng.integers(0, nb, int(rng.integers(0, 5))))) + [nb]
        start, written = 0, 0
        for cut in cuts:
            seg = np.ascontiguousarray(row[start:cut])
            dst = out[written:]
            written += lib.convEnc(enc, seg.ctypes.data_as(ctypes.c_void_p), dst.ctypes.data_as(ctypes.c_void_p),
                                   len(seg), cut == nb)
            start = cut
        assert written == want.size and (out[:written] == want).all(), (K, trial, nb, cuts)
        assert (out[written:] == 0).all()


def test_calc_hamming_dist():
    lib = _legacy(7)
    assert lib.calcHammingDist(0b11, 0b00, 2) == 2
    assert lib.calcHammingDist(0xFF, 0x00, 2) == 2  # only the low `bits` bits count
    assert lib.calcHammingDist(0xF0, 0x0F, 8) == 8


LEGACY_CONFIGS = {"k3": (1, 3, 2), "k5": (1, 5, 2), "k7": (1, 7, 2), "k9": (1, 9, 2), "k4_k2n3": (2, 4, 3),
                  "k3_k3n4": (3, 3, 4)}


@pytest.mark.parametrize("name", sorted(LEGACY_CONFIGS))
def test_layout_helper_matches_compiled_struct(tmp_path, name):
    """tests/helpers.legacy_layout (used by the GPU legacy tests to read nodeMetricsCur and
    renormCounter out of the caller's state struct) against the compiler's layout."""
    from helpers import legacy_layout

    got = list(map(int, _probe(tmp_path, os.path.join(REPO, "include"), os.path.join(REPO, "params", name))))
    lay = legacy_layout(*LEGACY_CONFIGS[name])
    assert got[:9] == [lay[f] for f in ("sizeof", "nodeMetricsA", "traceBackA", "nodeMetricsB", "nodeMetricsCur",
                                        "iteration", "renormCounter", "decodeCarryOverCount", "tracebackBufs")]
    assert got[-1] == lay["N"]


def _defined(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {ln.split()[2] for ln in out.splitlines() if len(ln.split()) == 3 and ln.split()[1] == "T"}


@pytest.mark.parametrize("ref,ours", [("libref_k7.so", "k7"), ("libref_k9.so", "k9"),
                                      ("librefgenk_k4_k2n3.so", "k4_k2n3")])
def test_drop_in_exports_every_reference_symbol(ref, ours):
    """Every function the reference library defines (src/*.c compiled by oracle/Makefile,
    minus the test shim's own ref*_ entry points) is exported by the drop-in."""
    path = os.path.join(REPO, "oracle", "_ref", ref)
    if not os.path.exists(path):
        pytest.skip("reference build not present (oracle/Makefile ref)")
    want = {s for s in _defined(path) if not s.startswith(("ref_", "refgenk_", "refenc_"))}
    assert "minMetricGeneric" in want and "viterbiDecoderHard" in want
    missing = want - _defined(os.path.join(LIB_DIR, f"libviterbi_legacy_{ours}.so"))
    assert not missing, sorted(missing)
