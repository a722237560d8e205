"""MI355X-native Viterbi decoder behind the ucb-cyarp/ConvolutionalEncDec C API.

C ABI:      include/viterbi_amd.h            -> lib/libviterbi_amd.so (HIP, gfx950)
Legacy API: include/viterbiDecoder.h, convEncode.h -> lib/libviterbi_legacy_k<K>.so
Python:     plumbing over the C ABI (native.py, decoder.py).
"""
from .decoder import (K7_CODE, K9_CODE, ConvCode, GenKDecoder, ViterbiDecoder, ViterbiStream, decode_multi,  # noqa: F401
                      decode_peer, release_cached_plans, shard_range)
from .native import LIB_DIR, LIB_PATH, VtbError  # noqa: F401

__all__ = ["ConvCode", "ViterbiDecoder", "ViterbiStream", "decode_multi", "decode_peer", "shard_range",
           "release_cached_plans", "K7_CODE", "K9_CODE", "VtbError", "LIB_DIR", "LIB_PATH"]
