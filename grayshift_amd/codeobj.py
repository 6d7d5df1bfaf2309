"""Identity of the device code that is timed: a hash of the gfx950 code objects.

PMC summaries (profiles/pmc/) are only valid for the binary they were collected on.
``code_object_hash(lib)`` hashes the ``.hip_fatbin`` section of a shared library (the
offload bundle holding the gfx950 code objects), so host-only rebuilds or a different
install path do not change it, and any change of the kernels does.
"""
import hashlib
import struct


def _section(path, name):
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"\x7fELF" or data[4] != 2:  # ELFCLASS64
        raise ValueError("%s: not a 64-bit ELF file" % path)
    end = "<" if data[5] == 1 else ">"
    shoff, = struct.unpack_from(end + "Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from(end + "HHH", data, 0x3A)

    def sh(i):
        # sh_name, sh_type, sh_flags, sh_addr, sh_offset, sh_size
        return struct.unpack_from(end + "IIQQQQ", data, shoff + i * shentsize)

    stroff, strsize = sh(shstrndx)[4], sh(shstrndx)[5]
    strtab = data[stroff:stroff + strsize]
    for i in range(shnum):
        nm, typ, _, _, off, size = sh(i)
        s = strtab[nm:strtab.index(b"\0", nm)].decode()
        if s == name:
            return data[off:off + size] if typ != 8 else b""  # SHT_NOBITS
    raise KeyError("%s: no %s section" % (path, name))


def code_object_hash(path):
    """sha256 (hex, first 16 chars) of the library's .hip_fatbin section."""
    return hashlib.sha256(_section(path, ".hip_fatbin")).hexdigest()[:16]


def _bundles(fatbin):
    """The gfx950 code objects (ELF bytes) of every offload bundle in a .hip_fatbin."""
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out = []
    i = fatbin.find(magic)
    while i >= 0:
        off = i + len(magic)
        n, = struct.unpack_from("<Q", fatbin, off)
        off += 8
        for _ in range(n):
            eo, es, ts = struct.unpack_from("<QQQ", fatbin, off)
            off += 24
            triple = fatbin[off:off + ts].decode()
            off += ts
            if "gfx950" in triple and es:
                out.append(fatbin[i + eo:i + eo + es])
        i = fatbin.find(magic, i + len(magic))
    return out


def kernel_scratch(path):
    """{kernel symbol: private segment bytes per lane} from the kernel descriptors (the
    '.kd' symbols: group_segment_fixed_size, then private_segment_fixed_size) of the
    library's gfx950 code objects -- the scratch each kernel launches with."""
    res = {}
    for co in _bundles(_section(path, ".hip_fatbin")):
        if co[:4] != b"\x7fELF":
            raise ValueError("compressed or unknown code object")
        shoff, = struct.unpack_from("<Q", co, 0x28)
        shentsize, shnum, shstrndx = struct.unpack_from("<HHH", co, 0x3A)
        secs = [struct.unpack_from("<IIQQQQIIQQ", co, shoff + k * shentsize) for k in range(shnum)]
        for sec in secs:
            if sec[1] != 2:  # SHT_SYMTAB
                continue
            strtab = secs[sec[6]]
            names = co[strtab[4]:strtab[4] + strtab[5]]
            for k in range(sec[5] // 24):
                nm, info, other, shndx, value, size = struct.unpack_from("<IBBHQQ", co, sec[4] + k * 24)
                name = names[nm:names.index(b"\0", nm)].decode()
                if not name.endswith(".kd") or shndx == 0 or shndx >= shnum:
                    continue
                tsec = secs[shndx]
                base = tsec[4] + (value - tsec[3])  # file offset of the descriptor
                res[name[:-3]] = struct.unpack_from("<I", co, base + 4)[0]
    return res
