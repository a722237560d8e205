#!/bin/bash
# speedDecode protocol on N host threads (one decoder state each): the legacy drop-in (GPU,
# tools/probes/legacy_mt_speed) against the reference decoder (oracle/_ref/libref_k7.so,
# ref_speed), 2,048-bit frames, 2 s per point.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
o=gpurun_out/r02mt; mkdir -p $o
timeout -k 10 120 tools/probes/legacy_mt_speed 2 1 2 4 8 16 > $o/dropin.txt 2>$o/dropin.err || { tail $o/dropin.err; exit 1; }
grep threads $o/dropin.txt | sed 's/^/drop-in /'
timeout -k 10 120 python3 - <<'PY' 2>/dev/null
import ctypes
lib = ctypes.CDLL("oracle/_ref/libref_k7.so")
lib.ref_speed.restype = ctypes.c_double
lib.ref_speed.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_int]
for t in (1, 2, 4, 8, 16):
    print(f"reference threads {t}: {lib.ref_speed(2.0, t, 256):.1f} Mbit/s aggregate", flush=True)
PY
exit 0
