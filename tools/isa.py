#!/usr/bin/env python3
"""Disassemble the gfx950 code object inside a built .o/.so and summarise one kernel.

    python tools/isa.py <file.o|.so> <kernel-substring> [--dump]
Prints resource usage and an instruction histogram of the kernel's largest loop body
(the longest backward-branch range), so VALU/MFMA counts per stage can be compared.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def disasm(path):
    tmp = tempfile.mkdtemp()
    fb = os.path.join(tmp, "fb.bin")
    co = os.path.join(tmp, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", path], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    asm = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                         capture_output=True, text=True).stdout
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    return asm, notes


def main():
    path, pat = sys.argv[1], sys.argv[2]
    asm, notes = disasm(path)
    funcs = re.split(r"\n(?=[0-9a-f]+ <)", asm)
    cands = [f for f in funcs if re.match(r"[0-9a-f]+ <[^>]*" + re.escape(pat), f)]
    if not cands:
        sys.exit("no kernel matches " + pat)
    f = cands[0]
    name = re.match(r"[0-9a-f]+ <([^>]+)>", f).group(1)
    print(name)
    i = notes.find(name)
    for key in ("vgpr_count", "agpr_count", "sgpr_count", "group_segment_fixed_size", "vgpr_spill_count"):
        m = re.search(r"\." + key + r":\s+(\d+)", notes[i - 2500:i + 2500]) if i >= 0 else None
        print(f"  {key}: {m.group(1) if m else '?'}")
    lines = [l.split("//")[0].strip() for l in f.splitlines()[1:]]
    addrs = [re.search(r"// ([0-9A-F]+):", l) for l in f.splitlines()[1:]]
    # loops: backward branches
    best, best_m = (0, 0, 0), -1
    for k, l in enumerate(f.splitlines()[1:]):
        m = re.search(r"s_cbranch_\w+ (\d+)|s_branch (\d+)", l)
        if m:
            off = int(m.group(1) or m.group(2))
            if off >= 32768:
                back = 65536 - off
                # count instructions back by address: approximate with 1 instr / 6 bytes
                tgt = re.search(r"<[^+]+\+0x([0-9a-f]+)>", l)
                if tgt:
                    t = int(tgt.group(1), 16)
                    for j in range(k, -1, -1):
                        a = addrs[j]
                        if a and int(a.group(1), 16) - int(cands[0].split()[0], 16) <= t:
                            # the loop with the most MFMAs (then the longest) is the main loop
                            nm = sum("mfma" in x for x in lines[j:k + 1])
                            if (nm, k - j) > (best_m, best[0]):
                                best, best_m = (k - j, j, k), nm
                            break
    body = [l for l in lines[best[1]:best[2] + 1] if l]
    marks = [k for k, l in enumerate(lines) if l.startswith("s_nop 15")]
    if len(marks) >= 2:  # -DQMHA_ISA_MARKS build: the first marked region
        body = [l for l in lines[marks[0] + 1:marks[1]] if l]
    hist = collections.Counter(l.split()[0] for l in body)
    print(f"  loop body: {len(body)} instructions")
    cats = collections.Counter()
    for op, n in hist.items():
        c = ("mfma" if "mfma" in op else "ds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_")) else
             "nop" if op == "s_nop" else "salu" if op.startswith("s_") else "valu")
        cats[c] += n
    print("  " + ", ".join(f"{k}={v}" for k, v in cats.most_common()))
    for op, n in hist.most_common(40):
        print(f"    {n:4d} {op}")
    if "--dump" in sys.argv:
        print("\n".join(body))


if __name__ == "__main__":
    main()
