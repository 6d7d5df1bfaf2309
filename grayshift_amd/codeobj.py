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
