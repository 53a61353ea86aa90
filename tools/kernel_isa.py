#!/usr/bin/env python3
"""Machine-code fingerprints of the gfx950 kernels inside libnmz_gpu.so (measurement infrastructure).

A roofline priced from a rocprofv3 profile is only meaningful while the kernel it profiled is the kernel that
runs. tools/profile_r03.sh records these fingerprints next to each profile, tools/valu_per_unit.py stores them
in profiles/valu_per_unit.json, and bench.py recomputes them from the shipped library: an entry whose kernel
code differs is reported as stale (no frac).

Fingerprint of a kernel = sha256 over its .text bytes (st_value .. st_value + st_size of its FUNC symbol) and
its kernel descriptor (`<name>.kd`: register counts, LDS size, launch attributes; without the code entry offset,
which depends on where the linker placed the kernel), first 16 hex digits.
The library holds one uncompressed clang offload bundle per translation unit (`__CLANG_OFFLOAD_BUNDLE__`);
the gfx950 entry of each is an ELF64 code object.

usage: kernel_isa.py [libnmz_gpu.so] [out.json]   -> {demangled kernel name: fingerprint}
"""
import hashlib
import json
import os
import struct
import subprocess
import sys

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB = os.path.join(HERE, "..", "namazu_amd", "libnmz_gpu.so")


def code_objects(blob):
    """gfx950 ELF images of every offload bundle in `blob`."""
    out = []
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and size:
                out.append(blob[pos + off:pos + off + size])
        pos = blob.find(MAGIC, pos + 1)
    return out


def elf_symbols(img):
    """(name, section bytes slice of the symbol) for FUNC and OBJECT symbols of an ELF64 code object."""
    shoff = struct.unpack_from("<Q", img, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", img, 0x3A)
    secs = []
    for i in range(shnum):
        name, typ, flags, addr, off, size, link, info, align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", img, shoff + i * shentsize)
        secs.append(dict(type=typ, addr=addr, off=off, size=size, link=link, entsize=entsize))
    syms = []
    for s in secs:
        if s["type"] != 2:  # SHT_SYMTAB
            continue
        strtab = secs[s["link"]]
        for k in range(s["size"] // 24):
            st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from(
                "<IBBHQQ", img, s["off"] + 24 * k)
            if st_size == 0 or st_shndx == 0 or st_shndx >= len(secs) or (st_info & 0xF) not in (1, 2):
                continue
            end = img.index(b"\0", strtab["off"] + st_name)
            name = img[strtab["off"] + st_name:end].decode()
            sec = secs[st_shndx]
            if sec["type"] == 8:  # NOBITS
                continue
            start = sec["off"] + (st_value - sec["addr"])
            syms.append((name, img[start:start + st_size]))
    return syms


def demangle(names):
    if not names:
        return {}
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names) + "\n", capture_output=True, text=True, check=True)
        return dict(zip(names, r.stdout.splitlines()))
    except (OSError, subprocess.CalledProcessError):
        return {n: n for n in names}


def kernel_fingerprints(lib=DEFAULT_LIB):
    blob = open(lib, "rb").read()
    parts = {}
    for img in code_objects(blob):
        syms = dict(elf_symbols(img))
        for name, code in syms.items():
            if name.endswith(".kd"):
                continue
            kd = syms.get(name + ".kd")
            if kd is None:  # not a kernel entry point
                continue
            # bytes 16..23 of the descriptor are kernel_code_entry_byte_offset (descriptor -> code distance),
            # which moves with the layout of the code object, not with the kernel: left out
            kd = kd[:16] + kd[24:]
            parts[name] = hashlib.sha256(code + b"\0kd\0" + kd).hexdigest()[:16]
    dm = demangle(sorted(parts))
    return {dm[n]: h for n, h in parts.items()}


def lookup(fps, kernel_name):
    """Fingerprint of the kernel rocprofv3 names `kernel_name` (demangled signature), or None."""
    if kernel_name in fps:
        return fps[kernel_name]
    # rocprofv3 may print a demangled name without the return type
    for n, h in fps.items():
        if n.endswith(kernel_name) or kernel_name.endswith(n):
            return h
    return None


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_LIB
    fps = kernel_fingerprints(lib)
    if len(sys.argv) > 2:
        json.dump(fps, open(sys.argv[2], "w"), indent=1, sort_keys=True)
    for n, h in sorted(fps.items()):
        print(h, n)


if __name__ == "__main__":
    main()
