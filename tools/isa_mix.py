"""Issue-priced VALU bound of each decode kernel's ACS loop, from its gfx950 disassembly.

For the kernel instances bench.py measures, find the hot loop (the smallest backward-branch loop
holding exactly one unrolled 48-step ACS chunk: 48 `v_pk_min` per metric register; where the
compiler left no such loop, the loop with the most), classify its VALU instructions and
price them with the issue costs measured by tools/probes/isa_bench*.hip at two waves per SIMD
(profiles/r01/isa_bench*.txt):

  plain 32-bit ops (add/sub/and/or/xor/shift/mov/bitop3, VOP2 or VOP1)   2.8 cycles
  v_pk_* , DPP ops, v_perm, v_bfi, other VOP3 (3-operand / _e64) ops     4.6 cycles
  v_permlane16/32_swap                                                   9.4 cycles

Per wave-step: VALU instructions v and priced cycles p.  A SIMD then issues at most v / p
wave-instructions per cycle for this mix, i.e. 1,024 SIMDs x 2.4 GHz x v / p G/s: bench.py's
roofline.secondary.issue_priced peak (the SIMD-32's 2-cycle rate, 1,228.8 G/s, is the absolute
peak beside it).  Output: profiles/isa_mix.json, keyed "<kernel>/<soft|hard>" as
vtb_debug_last_kernel names them, stamped with the library's sha (bench.py pairs an entry only
with the library it was computed from).

usage: python tools/isa_mix.py [out.json]
"""
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(REPO, "convolutionalencdec_amd", "lib", "obj")
LIB = os.path.join(REPO, "convolutionalencdec_amd", "lib", "libviterbi_amd.so")
B = "/opt/rocm/lib/llvm/bin"

COST_PLAIN, COST_SLOW, COST_SWAP = 2.8, 4.6, 9.4
PLAIN = re.compile(r"^v_(add|sub|subrev|and|or|xor|not|lshlrev|lshrrev|ashrrev|lshl|lshr|mov|bitop3|cndmask|max|min)"
                   r"(_u32|_i32|_b32|_u16|_i16|_b16)?(_e32)?$")

# note_kernel name -> (object, symbol template, metric registers per lane)
K7 = "_ZN3vtb12_GLOBAL__N_113k7_lds_kernelILb{S}ELb{GS}ELb0ELb{LOOP}ELb{SPLIT}ELb0ELi2EEEvPKhmPhmiiiiimiNS_6LaunchES4_mNS_10StreamArgsE"
K9 = "_ZN3vtb12_GLOBAL__N_19k9_kernelILb{S}ELb{LOOP}ELb0ELi2EEEvPKhmPhmiiiiiimiNS_6LaunchES4_mNS_10StreamArgsE"
K9S = "_ZN3vtb12_GLOBAL__N_110k9s_kernelILb{S}EEEvPKhmPhmiiiiiiiNS_6LaunchES4_mj"
KERNELS = {
    "k7_lds": ("vtb_k7_lds.o", K7, dict(GS=0, LOOP=0, SPLIT=0), 1),
    "k7_lds_loop": ("vtb_k7_lds.o", K7, dict(GS=0, LOOP=1, SPLIT=0), 1),
    "k7_lds_split": ("vtb_k7_lds.o", K7, dict(GS=0, LOOP=0, SPLIT=1), 1),
    "k7_split_loop": ("vtb_k7_lds.o", K7, dict(GS=0, LOOP=1, SPLIT=1), 1),
    "k7_global": ("vtb_k7_lds.o", K7, dict(GS=1, LOOP=0, SPLIT=0), 1),
    "k7_global_loop": ("vtb_k7_lds.o", K7, dict(GS=1, LOOP=1, SPLIT=0), 1),
    "k9": ("vtb_k9.o", K9, dict(LOOP=0), 4),
    "k9_loop": ("vtb_k9.o", K9, dict(LOOP=1), 4),
    "k9s": ("vtb_k9.o", K9S, {}, 2),
}


def disassemble(obj):
    with tempfile.TemporaryDirectory() as t:
        subprocess.run([f"{B}/llvm-objcopy", f"--dump-section=.hip_fatbin={t}/fb", obj], check=True)
        subprocess.run([f"{B}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={t}/fb", f"--output={t}/co", "--unbundle"], check=True)
        return subprocess.run([f"{B}/llvm-objdump", "-d", "--no-show-raw-insn", f"{t}/co"], check=True,
                              capture_output=True, text=True).stdout


def functions(dis):
    """symbol -> [(address, mnemonic, branch target address or None)]"""
    out, cur, base = {}, None, 0
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(\S+)>:$", line)
        if m:
            base, cur = int(m.group(1), 16), m.group(2)
            out[cur] = []
            continue
        if cur is None or not line.startswith("\t"):
            continue
        m = re.match(r"^\t(\S+)(.*?)//\s*([0-9A-F]+):", line)
        if not m:
            continue
        tgt = re.search(r"<" + re.escape(cur) + r"\+0x([0-9a-f]+)>", line)
        out[cur].append((int(m.group(3), 16), m.group(1), base + int(tgt.group(1), 16) if tgt else None))
    return out


def price(body):
    n = {"plain": 0, "slow": 0, "swap": 0, "pk_min": 0}
    for _, mn, _ in body:
        if not mn.startswith("v_") or mn.startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
            if mn.startswith("v_readfirstlane"):
                n["slow"] += 1
            continue
        if mn.startswith("v_pk_min"):
            n["pk_min"] += 1
        if "permlane" in mn and "swap" in mn:
            n["swap"] += 1
        elif PLAIN.match(mn):
            n["plain"] += 1
        else:
            n["slow"] += 1
    return n


def hot_loop(insts, regs):
    """The steady-state chunk loop: the smallest backward-branch loop whose body holds exactly
    one 48-step chunk (48 v_pk_min per metric register); else the loop with the most."""
    loops = []
    for addr, mn, tgt in insts:
        if tgt is not None and tgt < addr and mn.startswith(("s_cbranch", "s_branch")):
            body = [x for x in insts if tgt <= x[0] <= addr]
            loops.append((sum(1 for x in body if x[1].startswith("v_pk_min")), len(body), body))
    one = [lp for lp in loops if lp[0] == 48 * regs]
    if one:
        return min(one, key=lambda lp: lp[1])[2]
    return max(loops, key=lambda lp: lp[0])[2] if loops else []


def is_chunk(n, regs):
    return n["pk_min"] == 48 * regs


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "profiles", "isa_mix.json")
    sha = hashlib.sha256(open(LIB, "rb").read()).hexdigest()[:16]
    cache = {}
    res = {"_note": __doc__.strip().split("\n\n")[0], "_costs": {"plain": COST_PLAIN, "slow": COST_SLOW,
                                                                  "swap": COST_SWAP}}
    for name, (obj, tmpl, par, regs) in KERNELS.items():
        if obj not in cache:
            cache[obj] = functions(disassemble(os.path.join(OBJ, obj)))
        for soft in (1, 0):
            sym = tmpl.format(S=soft, **par)
            insts = cache[obj].get(sym)
            if not insts:
                raise SystemExit(f"{sym} not found in {obj}")
            n = price(hot_loop(insts, regs))
            steps = n["pk_min"] / regs
            valu = n["plain"] + n["slow"] + n["swap"]
            cyc = COST_PLAIN * n["plain"] + COST_SLOW * n["slow"] + COST_SWAP * n["swap"]
            res[f"{name}/{'soft' if soft else 'hard'}"] = {
                "lib_sha16": sha, "symbol": sym, "loop_steps": steps, "valu_per_wave_step": round(valu / steps, 3),
                "priced_cycles_per_wave_step": round(cyc / steps, 3), "mix": n,
                "loop": "one 48-step chunk" if is_chunk(n, regs) else "largest loop (no single-chunk loop)",
                "priced_peak_G": round(1024 * 2.4 * valu / cyc, 1)}
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, v in res.items():
        if not k.startswith("_"):
            print(k, v["loop_steps"], v["valu_per_wave_step"], v["priced_cycles_per_wave_step"], v["priced_peak_G"], v["mix"])


if __name__ == "__main__":
    main()
