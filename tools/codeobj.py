#!/usr/bin/env python3
"""Per-kernel resource metadata of the built HIP library, read on the CPU:
the gfx950 code objects in libcosmomc_amd.so's offload bundles, their
AMDGPU metadata note (msgpack), per kernel the VGPR count, the scratch
(private segment) bytes per lane and the group-segment (LDS) bytes.

  python3 tools/codeobj.py [path/to/libcosmomc_amd.so]
"""
import os
import struct
import sys

import msgpack

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf):
    (shoff,) = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    out = []
    for i in range(shnum):
        name, typ, _flags, _addr, off, size = struct.unpack_from("<IIQQQQ", elf, shoff + i * shentsize)
        out.append((name, typ, off, size))
    return out


def _notes(elf):
    for _name, typ, off, size in _sections(elf):
        if typ != 7:                                      # SHT_NOTE
            continue
        p = off
        while p < off + size:
            namesz, descsz, ntype = struct.unpack_from("<III", elf, p)
            name = elf[p + 12:p + 12 + namesz]
            dp = p + 12 + ((namesz + 3) & ~3)
            yield name.rstrip(b"\0"), ntype, elf[dp:dp + descsz]
            p = dp + ((descsz + 3) & ~3)


def kernels(path):
    """{kernel symbol: {"vgpr": n, "agpr": n, "scratch": bytes/lane, "lds": bytes}} over every gfx950 object."""
    data = open(path, "rb").read()
    out = {}
    pos = data.find(MAGIC)
    while pos >= 0:
        (n,) = struct.unpack_from("<Q", data, pos + 24)
        p = pos + 32
        for _ in range(n):
            off, size, tsz = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tsz].decode()
            p += 24 + tsz
            if "gfx950" not in triple:
                continue
            elf = data[pos + off:pos + off + size]
            for name, ntype, desc in _notes(elf):
                if name != b"AMDGPU" or ntype != 32:
                    continue
                meta = msgpack.unpackb(desc, raw=False, strict_map_key=False)
                for k in meta.get("amdhsa.kernels", []):
                    out[k[".name"]] = {"vgpr": k.get(".vgpr_count"), "agpr": k.get(".agpr_count"),
                                       "scratch": k.get(".private_segment_fixed_size"),
                                       "lds": k.get(".group_segment_fixed_size")}
        pos = data.find(MAGIC, pos + 1)
    return out


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "cosmomc_amd", "lib", "libcosmomc_amd.so")
    ks = kernels(lib)
    for name, k in sorted(ks.items(), key=lambda kv: -kv[1]["scratch"]):
        print(f"{k['scratch']:6d} B scratch  {k['vgpr']:4d} vgpr  {k['lds']:6d} B lds  {name[:100]}")
