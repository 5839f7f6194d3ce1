"""Identity of the shipped machine code: a hash of one kernel's gfx950 instruction bytes.

bench.py records `isa_sha16` beside every number so that two bench lines (two rounds, two boxes)
can be told apart by code or matched as the same code: the kernel's bytes are read out of the
built library itself -- the `.hip_fatbin` section of the host ELF holds one clang offload bundle
per translation unit, each bundle a gfx950 code object (an AMDGPU ELF) whose symbol table locates
the kernel's instructions.  Pure Python (struct), so it runs wherever the library is loaded.

    python -m quantizedmha_amd.isa_id [lib.so] [kernel-substring ...]
"""
import hashlib
import os
import struct
import sys

_BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf):
    """{name: (offset, size)} of a 64-bit little-endian ELF image, plus the raw section headers."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2 or elf[5] != 1:
        raise ValueError("not a 64-bit little-endian ELF")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    stro = hdrs[shstrndx][4]
    out = {}
    for h in hdrs:
        name = elf[stro + h[0]:elf.index(b"\0", stro + h[0])].decode()
        out[name] = h
    return out, hdrs


def code_objects(lib_path):
    """Yield every gfx950 code object (bytes) bundled in a HIP shared library."""
    with open(lib_path, "rb") as f:
        host = f.read()
    secs, _ = _sections(host)
    if ".hip_fatbin" not in secs:
        return
    h = secs[".hip_fatbin"]
    fat = host[h[4]:h[4] + h[5]]
    pos = fat.find(_BUNDLE_MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fat, pos + 24)
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and size:
                yield fat[pos + off:pos + off + size]
        pos = fat.find(_BUNDLE_MAGIC, pos + 32)


def kernel_bytes(lib_path, pattern):
    """{symbol: instruction bytes} of every kernel symbol whose name contains `pattern`."""
    out = {}
    for co in code_objects(lib_path):
        secs, hdrs = _sections(co)
        if ".symtab" not in secs or ".strtab" not in secs:
            continue
        st, strt = secs[".symtab"], secs[".strtab"]
        for i in range(st[5] // 24):
            name_off, info, _other, shndx, value, size = struct.unpack_from("<IBBHQQ", co, st[4] + 24 * i)
            if (info & 0xF) != 2 or size == 0 or shndx >= len(hdrs):  # STT_FUNC with a body
                continue
            name = co[strt[4] + name_off:co.index(b"\0", strt[4] + name_off)].decode()
            if pattern not in name:
                continue
            sec = hdrs[shndx]  # value is a virtual address inside that section
            start = sec[4] + (value - sec[3])
            out[name] = co[start:start + size]
    return out


def isa_sha16(lib_path, pattern):
    """First 16 hex digits of the SHA-256 of the matching kernels' bytes (sorted by symbol), or None."""
    ks = kernel_bytes(lib_path, pattern)
    if not ks:
        return None
    h = hashlib.sha256()
    for name in sorted(ks):
        h.update(name.encode() + b"\0" + ks[name])
    return h.hexdigest()[:16]


def main(argv):
    root = os.path.dirname(os.path.abspath(__file__))
    lib = argv[1] if len(argv) > 1 else os.path.join(root, "lib", "libqmha.so")
    pats = argv[2:] or ["qmha_"]
    for pat in pats:
        for name, b in sorted(kernel_bytes(lib, pat).items()):
            print(f"{hashlib.sha256(b).hexdigest()[:16]}  {len(b):7d}  {name}")


if __name__ == "__main__":
    main(sys.argv)
