#!/usr/bin/env python3
"""sha256 of one kernel's gfx950 machine code inside a hipcc object or shared
library: the .hip_fatbin section's clang offload bundle -> the gfx950 code
object (an AMDGPU ELF) -> the kernel symbol's bytes in .text.

bench.py ties its PMC traffic figure (profiles/pmc_build_coop_p50.json) to
this hash of the bench's build-kernel instantiation, so a change elsewhere in
the build sources (another instantiation, a comment) does not mark the
measurement stale, and a change of the bench kernel's code does.

usage: kernel_hash.py FILE SYMBOL_SUBSTRING [--out PATH]"""
import hashlib
import struct
import sys

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf: bytes):
    """{name: (offset, size, addr)} of an ELF64 little-endian file."""
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = []
    for i in range(shnum):
        o = shoff + i * shentsize
        name, typ, flags, addr, off, size, link, info, align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", elf, o)
        hdrs.append((name, typ, addr, off, size, link, entsize))
    stroff = hdrs[shstrndx][3]
    out = {}
    for name, typ, addr, off, size, link, entsize in hdrs:
        end = elf.index(b"\0", stroff + name)
        out[elf[stroff + name:end].decode()] = (off, size, addr, typ, link, entsize)
    return out, hdrs


def code_objects(blob: bytes):
    """gfx950 code objects of every offload bundle found in blob."""
    out, pos = [], 0
    while True:
        i = blob.find(MAGIC, pos)
        if i < 0:
            return out
        n, = struct.unpack_from("<Q", blob, i + len(MAGIC))
        p = i + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and size:
                out.append(blob[i + off:i + off + size])
        pos = i + len(MAGIC)


def kernel_bytes(co: bytes, key: str):
    """(symbol, machine code) of the first function symbol containing key."""
    secs, hdrs = _sections(co)
    if ".symtab" not in secs:
        return None
    off, size, _, _, link, entsize = secs[".symtab"]
    stroff = hdrs[link][3]
    for k in range(size // entsize):
        name, info, other, shndx, value, sz = struct.unpack_from("<IBBHQQ", co, off + k * entsize)
        if (info & 0xF) != 2 or not sz:  # STT_FUNC
            continue
        end = co.index(b"\0", stroff + name)
        sym = co[stroff + name:end].decode()
        if key in sym:
            # value is the virtual address; map through the section holding it
            sh = hdrs[shndx]
            faddr = sh[3] + (value - sh[2])
            return sym, co[faddr:faddr + sz]
    return None


def main():
    path, key = sys.argv[1], sys.argv[2]
    blob = open(path, "rb").read()
    for co in code_objects(blob):
        r = kernel_bytes(co, key)
        if r:
            sym, code = r
            h = hashlib.sha256(code).hexdigest()[:16]
            line = f"{h} {len(code)} {sym}\n"
            if "--out" in sys.argv:
                open(sys.argv[sys.argv.index("--out") + 1], "w").write(line)
            sys.stdout.write(line)
            return 0
    sys.exit(f"kernel {key} not found in {path}")


if __name__ == "__main__":
    sys.exit(main())
