"""Guard for the asm-load hazard (commit 34aeaea): every shipped HIP kernel TU
is compiled to gfx950 assembly and tools/isa_asm_load_lint.py must report no register of an
inline-asm global load read before a vmcnt wait.  CPU only (hipcc cross-compiles)."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import isa_asm_load_lint as lint  # noqa: E402

HIPCC = "/opt/rocm/bin/hipcc"
CSRC = os.path.join(REPO, "convolutionalencdec_amd", "csrc")
SHIPPED = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))


def test_lint_flags_a_read_before_the_wait():
    asm = "\n".join([
        "_Z3fooPi:",
        ";;#ASMSTART",
        "global_load_dwordx2 v[4:5], v1, s[0:1]",
        ";;#ASMEND",
        "v_mov_b32 v9, v5",  # read of an in-flight register: reported
        "s_waitcnt vmcnt(0)",
        "v_add_u32 v2, v4, v4",  # after the wait: fine
    ])
    reps = lint.lint(asm)
    assert [(r[2], r[3]) for r in reps] == [("v5", "v_mov_b32 v9, v5")]


def test_lint_accepts_wait_first():
    asm = "\n".join(["_Z3barv:", ";;#ASMSTART", "global_load_dword v3, v1, s[0:1]", ";;#ASMEND",
                     "s_waitcnt vmcnt(0) lgkmcnt(0)", "v_mov_b32 v9, v3"])
    assert lint.lint(asm) == []


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not present")
def test_shipped_kernels_have_no_asm_load_hazard(tmp_path):
    def compile_one(name):
        out = tmp_path / (name + ".s")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(REPO, "include"),
                        "-I" + CSRC, "--cuda-device-only", "-S", "-o", str(out), os.path.join(CSRC, name)],
                       check=True, capture_output=True)
        return name, out.read_text()

    with ThreadPoolExecutor(max_workers=min(4, os.cpu_count() or 1)) as ex:
        asm = dict(ex.map(compile_one, SHIPPED))
    reports = {n: lint.lint(s) for n, s in asm.items()}
    bad = {n: r[:5] for n, r in reports.items() if r}
    assert not bad, f"asm-load hazard: {bad}"
    # the lint must have had something to check: the K=7 / K=9 kernels issue asm loads
    for name in ("vtb_k7_lds.hip", "vtb_k9.hip"):
        assert asm_global_loads(asm[name]) > 0, name
    # no kernel spills to or indexes into scratch memory (round 6: a select between 64-bit
    # survivor words in the generic traceback compiled to a dynamically indexed scratch array)
    scratch = {n: sum(1 for ln in s.split("\n") if ln.strip().startswith(("scratch_", "buffer_store", "buffer_load")))
               for n, s in asm.items()}
    assert not any(scratch.values()), scratch


def asm_global_loads(text):
    n, inside = 0, False
    for ln in text.split("\n"):
        s = ln.strip()
        if s.startswith(";;#ASMSTART"):
            inside = True
        elif s.startswith(";;#ASMEND"):
            inside = False
        elif inside and s.startswith("global_load"):
            n += 1
    return n
