"""Lint: registers loaded by inline-asm global loads must not be read before a vmcnt wait.

The compiler does not know that a `global_load_*` written in inline asm is asynchronous: it
treats the destination register as ready when the asm statement ends, so it may copy or read
it (e.g. at a control-flow join) before the asm `s_waitcnt vmcnt(...)` that really waits for
it.  That produced wrong frames once (commit 34aeaea).  This lint scans the
gfx950 assembly of one translation unit function by function and reports every read of such a
register that comes before any vmcnt wait in program order.

It is a linear scan: control flow is ignored, so a read on a path that did wait is still
reported (conservative), and a wait on another path still clears the register (the shipped
kernels wait in straight-line code after their prefetches).  Used by
tests/test_isa_lint.py on every shipped .hip file.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Iconvolutionalencdec_amd/csrc \\
        --cuda-device-only -S -o /tmp/k7.s convolutionalencdec_amd/csrc/vtb_k7_lds.hip
    python tools/isa_asm_load_lint.py /tmp/k7.s
"""
import re
import sys

_RANGE = re.compile(r"v\[(\d+):(\d+)\]")
_FUNC = re.compile(r"^(_Z\S*):")
_STORE_LIKE = ("global_store", "ds_write", "buffer_store", "s_")


def _covers(operand, reg):
    """True if `operand` names `reg` (vN), directly or through a v[a:b] range."""
    if operand == reg:
        return True
    m = _RANGE.fullmatch(operand)
    if m and reg.startswith("v") and reg[1:].isdigit():
        return int(m.group(1)) <= int(reg[1:]) <= int(m.group(2))
    return False


def _dest_regs(operand):
    """Registers written by an asm load whose destination operand is `operand`."""
    m = _RANGE.fullmatch(operand)
    if m:
        return [f"v{i}" for i in range(int(m.group(1)), int(m.group(2)) + 1)]
    return [operand]


def lint(asm_text):
    """Return a list of (function, line number, register, instruction) reports."""
    reports = []
    func, in_asm, pending = None, False, {}
    for n, line in enumerate(asm_text.split("\n"), 1):
        m = _FUNC.match(line)
        if m:
            func, pending = m.group(1)[:90], {}
            continue
        s = line.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        if op == "s_waitcnt" and "vmcnt(" in s:
            pending = {}
            continue
        if in_asm and op.startswith("global_load"):
            for r in _dest_regs(s.split()[1].rstrip(",")):
                pending[r] = n
            continue
        if not pending:
            continue
        operands = [p.strip().rstrip(",") for p in s.split()[1:]]
        sources = operands if op.startswith(_STORE_LIKE) else operands[1:]
        for r in list(pending):
            if any(_covers(p, r) for p in sources):
                reports.append((func, n, r, s))
                del pending[r]
    return reports


def main(paths):
    total = 0
    for p in paths:
        with open(p) as fh:
            reps = lint(fh.read())
        for r in reps:
            print(p, *r)
        total += len(reps)
    print(total, "reports")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
