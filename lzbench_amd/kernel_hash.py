"""lzbench_amd.kernel_hash -- identity of a kernel's machine code in a built library.

liblzbench_hip.so carries one clang offload bundle per translation unit; each holds a gfx950 code object
(an ELF).  kernel_hashes() reads every bundle's symbol table and returns, per kernel symbol, the sha256 of its
instruction bytes plus its kernel descriptor (`<name>.kd`: LDS size, register counts).  A PMC profile of a
kernel (profiles/traffic*.json) records this hash, and bench.py only reports the profile's traffic for a kernel
whose code is still the same (tools/pmc_traffic.sh writes it; traffic_for checks it).
Measurement tooling only: nothing on the codec path imports it.
"""
import hashlib
import struct

_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _elf_symbols(elf: bytes):
    """(name, section index, value, size, type) of every ELF64 symbol"""
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        return [], []
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    secs = []
    for i in range(shnum):
        name, typ, flags, addr, off, size, link, info, align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", elf, shoff + i * shentsize)
        secs.append((typ, addr, off, size, link, entsize))
    syms = []
    for typ, addr, off, size, link, entsize in secs:
        if typ != 2 or entsize == 0:   # SHT_SYMTAB
            continue
        stroff = secs[link][2]
        for k in range(size // entsize):
            st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", elf,
                                                                                       off + k * entsize)
            end = elf.index(b"\0", stroff + st_name)
            syms.append((elf[stroff + st_name:end].decode(errors="replace"), st_shndx, st_value, st_size,
                         st_info & 15))
    return syms, secs


def _bytes_at(elf, secs, shndx, value, size):
    if shndx == 0 or shndx >= len(secs) or size == 0:
        return b""
    typ, addr, off, ssize, link, entsize = secs[shndx]
    return elf[off + (value - addr): off + (value - addr) + size]


def kernel_hashes(lib_path: str) -> dict:
    """{kernel name: sha256 hex (first 16) of its code bytes + kernel descriptor} over every gfx950 bundle.
    Device functions the compiler kept out of line (no `.kd`: callees such as lz4v3::compress_chunk<..>) are
    hashed into every kernel of their code object -- a conservative identity: a change in a callee changes
    the hash of each kernel that might call it."""
    data = open(lib_path, "rb").read()
    out = {}
    pos = data.find(_MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", data, pos + 24)
        p = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tl]
            p += 24 + tl
            if b"amdgcn" not in triple or size == 0:
                continue
            elf = data[pos + off:pos + off + size]
            syms, secs = _elf_symbols(elf)
            by = {s[0]: s for s in syms}
            funcs = [s for s in syms if s[4] == 2 and not s[0].endswith(".kd")]   # STT_FUNC
            helpers = b"".join(_bytes_at(elf, secs, s[1], s[2], s[3]) for s in sorted(funcs)
                               if s[0] + ".kd" not in by)
            for name, shndx, value, ssize, typ in funcs:
                if name + ".kd" not in by:
                    continue
                h = hashlib.sha256(_bytes_at(elf, secs, shndx, value, ssize))
                h.update(helpers)
                kd = by.get(name + ".kd")
                if kd is not None:
                    h.update(_bytes_at(elf, secs, kd[1], kd[2], kd[3]))
                out[name] = h.hexdigest()[:16]
        pos = data.find(_MAGIC, pos + len(_MAGIC))
    return out


if __name__ == "__main__":
    import sys
    for k, v in sorted(kernel_hashes(sys.argv[1]).items()):
        print(v, k)
