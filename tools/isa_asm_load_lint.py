"""Measurement/debug only: flag reads of registers loaded by inline-asm global loads before any
vmcnt wait (the compiler does not know such loads are asynchronous, so it may copy their
destination registers early).  Linear scan of one function's text, control flow ignored.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Iconvolutionalencdec_amd/csrc \
        --cuda-device-only -S -o /tmp/k7.s convolutionalencdec_amd/csrc/vtb_k7_lds.hip
    python tools/isa_asm_load_lint.py /tmp/k7.s
"""
import re,sys
lines=open(sys.argv[1]).read().split("\n")
kern=None; inasm=False; pending={}  # reg -> line of load
reports=[]
for n,l in enumerate(lines):
    if re.match(r"^_Z\S*:",l): kern=l.split(":")[0][:90]; pending={}; continue
    s=l.strip()
    if s.startswith(";;#ASMSTART"): inasm=True; continue
    if s.startswith(";;#ASMEND"): inasm=False; continue
    if not s or s.startswith(";") or s.startswith("."): continue
    m=re.match(r"s_waitcnt\s+(.*)",s)
    if m and "vmcnt(" in m.group(1): pending={}; continue
    op=s.split()[0]
    if inasm and op.startswith("global_load"):
        dst=s.split()[1].rstrip(",")
        pending[dst]=n; continue
    if pending:
        parts=[p.strip().rstrip(",") for p in s.split()[1:]]
        srcs=parts[1:] if not op.startswith(("global_store","ds_write","buffer_store","s_")) else parts
        for r in list(pending):
            if r in srcs or any(re.fullmatch(r"v\[(\d+):(\d+)\]",p) and int(re.fullmatch(r"v\[(\d+):(\d+)\]",p).group(1))<=int(r[1:])<=int(re.fullmatch(r"v\[(\d+):(\d+)\]",p).group(2)) for p in srcs if r.startswith("v") and r[1:].isdigit()):
                reports.append((kern,n+1,r,s)); del pending[r]
for r in reports: print(r)
print(len(reports),"reports")
