"""ctypes binding of the C ABI in include/viterbi_amd.h (libviterbi_amd.so, built in-tree).

Plumbing only: every decode runs in the HIP kernels behind the C ABI.  There is no CPU
fallback -- if the library is missing or the device is not a gfx950, calls raise.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
# $VTB_LIB_PATH points at an alternative build (A/B measurement of kernel variants only): it must
# be a measurement build under lib/exp/ (tools/build_variants.sh, tools/ab_lib.sh), so the public
# API can never be pointed at an arbitrary library.
EXP_DIR = os.path.join(LIB_DIR, "exp")


def _lib_path(environ=os.environ):
    alt = environ.get("VTB_LIB_PATH")
    if not alt:
        return os.path.join(LIB_DIR, "libviterbi_amd.so")
    real = os.path.realpath(alt)
    if os.path.commonpath([real, os.path.realpath(EXP_DIR)]) != os.path.realpath(EXP_DIR):
        raise ImportError(f"VTB_LIB_PATH={alt!r}: only measurement builds under {EXP_DIR} may replace the library")
    return real


LIB_PATH = _lib_path()

VTB_OK = 0
VTB_ERR_INVALID = -1
VTB_ERR_CODE = -2
VTB_ERR_UNSUPPORTED = -3
VTB_ERR_DEVICE = -4
VTB_ERR_NOMEM = -5

VTB_PEER_STAGE_ALL = 1
VTB_GENK_K1_REFERENCE_U8 = 1

VTB_INPUT_HARD = 0
VTB_INPUT_SOFT8 = 1

# Every symbol include/viterbi_amd.h declares (tests/test_abi.py checks the header and the
# library against this list).
EXPORTED_SYMBOLS = (
    "vtb_version",
    "vtb_strerror",
    "vtb_code_check",
    "vtb_edge_table",
    "vtb_input_bytes_per_frame",
    "vtb_output_bytes_per_frame",
    "vtb_plan_create",
    "vtb_plan_destroy",
    "vtb_decode_device",
    "vtb_decode_host",
    "vtb_decode_host_multi",
    "vtb_release_cached_plans",
    "vtb_shard_range",
    "vtb_decode_peer_multi",
    "vtb_decode_frame_sync",
    "vtb_decode_frame_legacy",
    "vtb_stream_create",
    "vtb_stream_destroy",
    "vtb_stream_out_bytes",
    "vtb_stream_decode",
    "vtb_device_count",
    "vtb_rand64",
    "vtb_payload_device",
    "vtb_encode_device",
    "vtb_channel_device",
    "vtb_awgn_kq",
    "vtb_bsc_p32",
    "vtb_genk_decode_device",
    "vtb_legacy_metrics_k1",
    "vtb_legacy_metrics_k1n",
    "vtb_legacy_metrics_genk",
    "vtb_genk_decode_frame_legacy",
)


class VtbGenKCode(ctypes.Structure):
    """vtb_genk_code_t: a rate-k/n code (include/viterbi_amd.h)."""
    _fields_ = [
        ("input_bits", ctypes.c_int32),
        ("constraint_length", ctypes.c_int32),
        ("coded_bits", ctypes.c_int32),
        ("flags", ctypes.c_int32),  # 0 or VTB_GENK_K1_REFERENCE_U8
        ("generators", ctypes.c_uint64 * 8),
    ]

    @classmethod
    def make(cls, k, K, g, flags=0):
        c = cls()
        c.input_bits, c.constraint_length, c.coded_bits, c.flags = int(k), int(K), len(g), int(flags)
        for i, v in enumerate(g):
            c.generators[i] = int(v)
        return c


class VtbCode(ctypes.Structure):
    _fields_ = [
        ("constraint_length", ctypes.c_int32),
        ("coded_bits", ctypes.c_int32),
        ("generators", ctypes.c_uint64 * 2),
    ]

    @classmethod
    def make(cls, K, g):
        c = cls()
        c.constraint_length = int(K)
        c.coded_bits = 2
        c.generators[0] = int(g[0])
        c.generators[1] = int(g[1])
        return c


class VtbError(RuntimeError):
    def __init__(self, code, what):
        self.code = code
        super().__init__(f"{what}: {strerror(code)} ({code})")


_lib = None


def lib():
    """Load libviterbi_amd.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run `make` (or __graft_entry__.build()) first")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, i32, cp = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.POINTER(VtbCode)
    L.vtb_version.restype = ctypes.c_char_p
    L.vtb_version.argtypes = []
    L.vtb_strerror.restype = ctypes.c_char_p
    L.vtb_strerror.argtypes = [ctypes.c_int]
    L.vtb_code_check.argtypes = [cp]
    L.vtb_edge_table.argtypes = [cp, vp]
    L.vtb_input_bytes_per_frame.restype = sz
    L.vtb_input_bytes_per_frame.argtypes = [cp, ctypes.c_int, i32]
    L.vtb_output_bytes_per_frame.restype = sz
    L.vtb_output_bytes_per_frame.argtypes = [i32]
    L.vtb_plan_create.argtypes = [ctypes.POINTER(vp), cp, ctypes.c_int, i32, ctypes.c_int]
    L.vtb_plan_destroy.restype = None
    L.vtb_plan_destroy.argtypes = [vp]
    L.vtb_decode_device.argtypes = [vp, vp, sz, vp, sz, sz, vp]
    L.vtb_decode_host.argtypes = [vp, vp, vp, sz]
    L.vtb_decode_host_multi.argtypes = [cp, ctypes.c_int, i32, vp, vp, sz, ctypes.c_uint32]
    L.vtb_release_cached_plans.restype = None
    L.vtb_release_cached_plans.argtypes = []
    L.vtb_shard_range.argtypes = [sz, sz, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)]
    L.vtb_decode_peer_multi.argtypes = [cp, ctypes.c_int, i32, ctypes.c_int, vp, vp, sz, ctypes.POINTER(ctypes.c_int),
                                        ctypes.c_int, ctypes.c_uint32, vp]
    L.vtb_decode_frame_legacy.argtypes = [cp, vp, i32, vp]
    L.vtb_decode_frame_sync.argtypes = [vp, vp, vp]
    L.vtb_stream_create.argtypes = [ctypes.POINTER(vp), cp, ctypes.c_int, sz, i32, ctypes.c_int]
    L.vtb_stream_destroy.restype = None
    L.vtb_stream_destroy.argtypes = [vp]
    L.vtb_stream_out_bytes.restype = sz
    L.vtb_stream_out_bytes.argtypes = [vp]
    L.vtb_stream_decode.argtypes = [vp, vp, sz, i32, ctypes.c_int, vp, sz, vp, vp]
    L.vtb_device_count.argtypes = []
    u64 = ctypes.c_uint64
    L.vtb_rand64.restype = u64
    L.vtb_rand64.argtypes = [u64, u64, u64]
    L.vtb_payload_device.argtypes = [u64, i32, vp, sz, sz, vp]
    L.vtb_encode_device.argtypes = [cp, i32, vp, sz, vp, sz, sz, vp]
    L.vtb_channel_device.argtypes = [ctypes.c_int, ctypes.c_double, u64, vp, sz, i32, vp, sz, sz, vp]
    L.vtb_awgn_kq.restype = ctypes.c_int64
    L.vtb_awgn_kq.argtypes = [ctypes.c_double]
    L.vtb_bsc_p32.restype = ctypes.c_uint32
    L.vtb_bsc_p32.argtypes = [ctypes.c_double]
    L.vtb_genk_decode_device.argtypes = [ctypes.POINTER(VtbGenKCode), i32, vp, sz, vp, sz, sz, vp]
    for name in ("vtb_code_check", "vtb_edge_table", "vtb_plan_create", "vtb_decode_device", "vtb_decode_host",
                 "vtb_decode_host_multi", "vtb_decode_peer_multi", "vtb_shard_range", "vtb_decode_frame_legacy", "vtb_decode_frame_sync", "vtb_stream_create", "vtb_stream_decode",
                 "vtb_device_count", "vtb_payload_device",
                 "vtb_encode_device", "vtb_channel_device", "vtb_genk_decode_device"):
        getattr(L, name).restype = ctypes.c_int
    _lib = L
    return L


def last_kernel():
    """Kernel instance of this thread's last decode launch (testing: vtb_debug_last_kernel)."""
    f = lib().vtb_debug_last_kernel
    f.restype, f.argtypes = ctypes.c_char_p, []
    return f().decode()


def strerror(code):
    try:
        return lib().vtb_strerror(int(code)).decode()
    except Exception:  # pragma: no cover - used while formatting another error
        return "error"


def check(rc, what):
    if rc < 0:
        raise VtbError(rc, what)
    return rc


def set_guard_counter(ptr):
    """Testing: device address of a uint32 that every traceback completeness guard firing in
    later launches adds 1 to (vtb_debug_set_guard_counter); 0 / None turns it off."""
    f = lib().vtb_debug_set_guard_counter
    f.restype, f.argtypes = None, [ctypes.c_void_p]
    f(ctypes.c_void_p(ptr or 0))


def effective_debug_flags():
    """Testing: the $VTB_DEBUG bits a plan created now carries (the shipped library drops the
    output-corrupting bits 0-4; vtb_debug_effective_flags)."""
    f = lib().vtb_debug_effective_flags
    f.restype, f.argtypes = ctypes.c_int, []
    return int(f())


def measure_build():
    """True for a -DVTB_MEASURE library (tools/build_variants.sh), which honours them."""
    f = lib().vtb_debug_measure_build
    f.restype, f.argtypes = ctypes.c_int, []
    return bool(f())
