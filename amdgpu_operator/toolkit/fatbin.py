"""Arch-trimmed ROCm libraries: keep only the node's GPU code object.

Why: a stock ROCm library carries device code for every supported GPU in one
zstd-compressed offload bundle.  librccl.so.1 of ROCm 7.2 holds 13 code
objects (gfx1030 ... gfx950) = 5.29 GB uncompressed in a 571 MB bundle, and
the HIP runtime decompresses the WHOLE bundle on the first kernel lookup to
reach the gfx950 entry, which is the last one.  In the validator that lookup
is ncclCommInitRank's kernel set-up: 1.56 s of its 1.65 s on MI355X
(RCCL "Init timings", profiles/r1_bench/rccl_init_probe.json), on the
time-to-Ready critical path of every node with >= 2 GPUs.  The driver /
toolkit images of this operator target gfx950 only, so the validator image
ships an RCCL whose bundle holds just the gfx950 code object, DWARF stripped
(108 MB).  It is stored uncompressed: decoding the 15.5 MB zstd form cost
ncclCommInitRank another ~80 ms (0.44 -> 0.36 s median, interleaved A/B on
MI355X, profiles/r2_ttr/rccl_lib_probe.txt).

How (no relink: the host code and every virtual address stay as they are):

* the new compressed bundle (``CCOB`` v3, zstd, MD5 integrity hash exactly as
  clang-offload-bundler writes it) is placed at the start of the old
  ``.hip_fatbin`` section, so the ``__hip_fatbin_wrapper`` pointers (one per
  translation unit, R_X86_64_RELATIVE relocations) stay valid untouched;
* the read-only PT_LOAD that held the 571 MB section is split in two: the
  part up to the end of the new bundle, and the part from the page holding
  ``.eh_frame_hdr`` on, whose file offset moves down by a whole number of
  pages (offset == vaddr mod page size is kept for every later segment);
* the PT_NOTE entry (build-id; not used for loading) gives up its program
  header slot for the second PT_LOAD, keeping PT_LOADs in ascending order;
* section headers follow their bytes; ``.hip_fatbin`` shrinks.

``verify_library`` re-reads the output and checks that its bundle decodes
to the same code-object bytes as the source's entry for the arch.
"""

from __future__ import annotations

import ctypes
import hashlib
import mmap
import os
import struct
from dataclasses import dataclass

PAGE = 0x1000
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
CCOB_MAGIC = b"CCOB"
CCOB_HDR = struct.Struct("<4sHHQQQ")  # magic, version, method, total size, uncompressed size, hash
HOST_TRIPLE = "host-x86_64-unknown-linux-gnu-"
PT_LOAD, PT_NOTE = 1, 4
EHDR = struct.Struct("<16sHHIQQQIHHHHHH")
PHDR = struct.Struct("<IIQQQQQQ")
SHDR = struct.Struct("<IIQQQQIIQQ")
SHT_NOBITS = 8


def _zstd():
    z = ctypes.CDLL("libzstd.so.1")
    sz, vp = ctypes.c_size_t, ctypes.c_void_p
    for fn, res, args in (("ZSTD_decompress", sz, [vp, sz, vp, sz]), ("ZSTD_compress", sz, [vp, sz, vp, sz, ctypes.c_int]),
                          ("ZSTD_compressBound", sz, [sz]), ("ZSTD_isError", ctypes.c_uint, [sz]),
                          ("ZSTD_getErrorName", ctypes.c_char_p, [sz])):
        getattr(z, fn).restype = res
        getattr(z, fn).argtypes = args
    return z


def _check(z, n: int, what: str) -> int:
    if z.ZSTD_isError(n):
        raise ValueError(f"zstd {what}: {z.ZSTD_getErrorName(n).decode()}")
    return n


@dataclass
class Entry:
    triple: str
    offset: int
    size: int


def parse_bundle(data) -> list[Entry]:
    """Entries of an uncompressed clang offload bundle."""
    if bytes(data[:24]) != BUNDLE_MAGIC:
        raise ValueError("not a clang offload bundle")
    (n,) = struct.unpack_from("<Q", data, 24)
    p, out = 32, []
    for _ in range(n):
        off, size, tl = struct.unpack_from("<QQQ", data, p)
        p += 24
        out.append(Entry(bytes(data[p:p + tl]).decode(), off, size))
        p += tl
    return out


def decompress_ccob(blob) -> bytearray:
    """CCOB v2/v3 (zstd) -> uncompressed bundle bytes, hash-checked."""
    magic, ver, method, total, unc, h = CCOB_HDR.unpack_from(blob, 0)
    if magic != CCOB_MAGIC or ver != 3 or method != 1:
        raise ValueError(f"unsupported compressed bundle (version {ver}, method {method})")
    z = _zstd()
    src = bytes(blob[CCOB_HDR.size:total])
    dst = ctypes.create_string_buffer(unc)
    n = _check(z, z.ZSTD_decompress(dst, unc, src, len(src)), "decompress")
    out = bytearray(memoryview(dst)[:n])
    if _md5_low(out) != h:
        raise ValueError("compressed bundle hash mismatch")
    return out


def _md5_low(data) -> int:
    return struct.unpack("<Q", hashlib.md5(data).digest()[:8])[0]


def build_bundle(code_object: bytes, triple: str) -> bytes:
    """A two-entry uncompressed offload bundle (empty host entry + the code
    object at the first page boundary)."""
    entries = [(HOST_TRIPLE, 0), (triple, len(code_object))]
    hdr = bytearray(BUNDLE_MAGIC + struct.pack("<Q", len(entries)))
    for t, size in entries:
        hdr += struct.pack("<QQQ", PAGE, size, len(t)) + t.encode()
    assert len(hdr) <= PAGE
    return bytes(hdr) + bytes(PAGE - len(hdr)) + code_object


def build_ccob(code_object: bytes, triple: str, level: int = 3) -> bytes:
    """The same bundle compressed the way clang-offload-bundler --compress
    writes format v3."""
    bundle = build_bundle(code_object, triple)
    z = _zstd()
    cap = z.ZSTD_compressBound(len(bundle))
    out = ctypes.create_string_buffer(cap)
    n = _check(z, z.ZSTD_compress(out, cap, bundle, len(bundle), level), "compress")
    return CCOB_HDR.pack(CCOB_MAGIC, 3, 1, CCOB_HDR.size + n, len(bundle), _md5_low(bundle)) + out.raw[:n]


class Elf:
    def __init__(self, data: bytes | bytearray):
        self.data = data
        h = EHDR.unpack_from(data, 0)
        if h[0][:4] != b"\x7fELF" or h[0][4] != 2 or h[0][5] != 1:
            raise ValueError("not a little-endian ELF64 file")
        self.hdr = list(h)
        self.phoff, self.shoff, self.phnum, self.shnum, self.shstrndx = h[5], h[6], h[10], h[12], h[13]
        self.phdrs = [list(PHDR.unpack_from(data, self.phoff + i * PHDR.size)) for i in range(self.phnum)]
        self.shdrs = [list(SHDR.unpack_from(data, self.shoff + i * SHDR.size)) for i in range(self.shnum)]
        st = self.shdrs[self.shstrndx]
        strtab = bytes(data[st[4]:st[4] + st[5]])
        self.names = [strtab[s[0]:strtab.index(b"\0", s[0])].decode() for s in self.shdrs]

    def section(self, name: str) -> list:
        return self.shdrs[self.names.index(name)]


def fatbin_of(path: str):
    """(Elf, bundle entries, uncompressed bundle) of a library's .hip_fatbin."""
    with open(path, "rb") as f:
        data = f.read()
    elf = Elf(data)
    sec = elf.section(".hip_fatbin")
    blob = memoryview(data)[sec[4]:sec[4] + sec[5]]
    bundle = decompress_ccob(blob) if bytes(blob[:4]) == CCOB_MAGIC else bytearray(blob)
    return elf, parse_bundle(bundle), bundle


def code_object(bundle, entries: list[Entry], arch: str) -> tuple[str, bytes]:
    for e in entries:
        if e.triple.endswith("--" + arch):
            return e.triple, bytes(bundle[e.offset:e.offset + e.size])
    raise KeyError(f"no {arch} code object in bundle ({[e.triple for e in entries]})")


SHF_ALLOC = 0x2
OBJCOPY = "/opt/rocm/lib/llvm/bin/llvm-objcopy"


def _alloc_sections(co: bytes) -> list[tuple]:
    e = Elf(co)
    return [(e.names[i], s[3], s[5], bytes(co[s[4]:s[4] + s[5]]) if s[1] != SHT_NOBITS else b"")
            for i, s in enumerate(e.shdrs) if s[2] & SHF_ALLOC]


def strip_debug(co: bytes, objcopy: str = OBJCOPY) -> bytes:
    """Drop the DWARF sections of a device code object (RCCL's gfx950 object
    is 569 MB of which 460 MB is debug info, and the HSA loader's time grows
    with the file it is handed: 1.2 s for hipModuleLoadData of the full
    object on MI355X, tools/native/co_load_probe.cpp).  Every SHF_ALLOC
    section - what the loader maps, i.e. the kernels - is checked to be
    byte-identical afterwards."""
    import subprocess
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.co"), os.path.join(d, "out.co")
        with open(src, "wb") as f:
            f.write(co)
        subprocess.run([objcopy, "--strip-debug", src, dst], check=True, capture_output=True)
        with open(dst, "rb") as f:
            out = f.read()
    if _alloc_sections(out) != _alloc_sections(co):
        raise ValueError("strip-debug changed a loadable section")
    return out


def slim_library(src: str, dst: str, arch: str = "gfx950", level: int = 3, strip: bool = True,
                 compress: bool = True) -> dict:
    """Write ``dst``: ``src`` with a .hip_fatbin holding only ``arch`` (debug
    sections stripped unless ``strip`` is false; an uncompressed bundle with
    ``compress`` false, which the HIP runtime uses without decompressing)."""
    elf, entries, bundle = fatbin_of(src)
    triple, co = code_object(bundle, entries, arch)
    del bundle
    full_bytes = len(co)
    if strip:
        co = strip_debug(co)
    ccob = build_ccob(co, triple, level) if compress else build_bundle(co, triple)
    data = elf.data
    fb = elf.section(".hip_fatbin")
    fb_off, fb_addr, fb_size = fb[4], fb[3], fb[5]
    if len(ccob) > fb_size:
        raise ValueError("trimmed bundle does not fit the old section")
    loads = [i for i, p in enumerate(elf.phdrs) if p[0] == PT_LOAD]
    li = next(i for i in loads if elf.phdrs[i][2] <= fb_off < elf.phdrs[i][2] + elf.phdrs[i][5])
    seg = elf.phdrs[li]
    k = seg[3] - seg[2]  # vaddr - offset of that segment
    if fb_addr - fb_off != k:
        raise ValueError("unexpected .hip_fatbin placement")
    seg_end = seg[2] + seg[5]
    after = [s[4] for s in elf.shdrs if s[4] >= fb_off + fb_size and s[4] < seg_end and s[1] != SHT_NOBITS]
    keep_from = min(after) if after else seg_end  # first byte after the bundle still needed (.eh_frame_hdr)
    cut = keep_from & ~(PAGE - 1)
    new_cut = (fb_off + len(ccob) + PAGE - 1) & ~(PAGE - 1)
    if new_cut >= cut or not any(p[0] == PT_NOTE for p in elf.phdrs):
        # small library (nothing to give back) or no spare program header:
        # rewrite the bundle in place, file layout unchanged
        out = bytearray(data)
        out[fb_off:fb_off + fb_size] = ccob + bytes(fb_size - len(ccob))
        return _finish(out, dst, src, arch, triple, co, full_bytes, entries, ccob, len(data))
    delta = cut - new_cut
    for i, p in enumerate(elf.phdrs):  # nothing else may live in the bytes that go away
        if i != li and p[5] and p[2] < cut and p[2] + p[5] > fb_off + len(ccob):
            raise ValueError("a segment overlaps the removed bundle bytes")
    out = bytearray(data[:fb_off]) + ccob + bytes(new_cut - fb_off - len(ccob)) + data[cut:]
    # program headers: split the bundle's PT_LOAD, drop PT_NOTE, shift the rest
    a = list(seg)
    a[5] = a[6] = fb_off + len(ccob) - seg[2]
    b = list(seg)
    b[2], b[3], b[4] = new_cut, cut + k, cut + k
    b[5] = b[6] = seg_end - cut
    phdrs = []
    for i, p in enumerate(elf.phdrs):
        if i == li:
            phdrs += [a, b]
            continue
        if p[0] == PT_NOTE:
            continue
        q = list(p)
        if q[2] >= cut:
            q[2] -= delta
        phdrs.append(q)
    if len(phdrs) != elf.phnum:
        raise ValueError("no PT_NOTE slot to reuse for the split segment")
    for i, p in enumerate(phdrs):
        PHDR.pack_into(out, elf.phoff + i * PHDR.size, *p)
    # section headers follow their bytes
    shoff = elf.shoff - delta
    for i, s in enumerate(elf.shdrs):
        q = list(s)
        if i == elf.names.index(".hip_fatbin"):
            q[5] = len(ccob)
        elif q[4] >= cut:
            q[4] -= delta
        SHDR.pack_into(out, shoff + i * SHDR.size, *q)
    hdr = list(elf.hdr)
    hdr[6] = shoff
    EHDR.pack_into(out, 0, *hdr)
    return _finish(out, dst, src, arch, triple, co, full_bytes, entries, ccob, len(data))


def _finish(out, dst, src, arch, triple, co, full_bytes, entries, ccob, src_bytes) -> dict:
    tmp = dst + ".tmp"
    with open(tmp, "wb") as f:
        f.write(out)
    os.chmod(tmp, 0o755)
    os.replace(tmp, dst)
    _, entries2, bundle2 = fatbin_of(dst)  # read back: the output decodes to the same code object
    if code_object(bundle2, entries2, arch) != (triple, co) or len(entries2) != 2:
        os.unlink(dst)
        raise ValueError("trimmed library does not decode to the source code object")
    return {"source": src, "output": dst, "arch": arch, "triple": triple, "code_object_bytes": len(co),
            "code_object_bytes_with_debug": full_bytes,
            "source_entries": len(entries), "bundle_bytes": len(ccob), "file_bytes": len(out),
            "source_file_bytes": src_bytes}


def verify_library(path: str, src: str, arch: str = "gfx950") -> dict:
    """The trimmed library's bundle holds exactly the source's ``arch`` code
    object, and every PT_LOAD keeps offset == vaddr mod page."""
    elf, entries, bundle = fatbin_of(path)
    triple, co = code_object(bundle, entries, arch)
    s_elf, s_entries, s_bundle = fatbin_of(src)
    s_triple, s_co = code_object(s_bundle, s_entries, arch)
    loads = [p for p in elf.phdrs if p[0] == PT_LOAD]
    aligned = all((p[2] - p[3]) % PAGE == 0 for p in loads)
    ascending = all(loads[i][3] < loads[i + 1][3] for i in range(len(loads) - 1))
    same = co == s_co or _alloc_sections(co) == _alloc_sections(s_co)  # full, or debug-stripped
    ok = same and triple == s_triple and aligned and ascending and len(entries) == 2
    return {"ok": ok, "entries": [e.triple for e in entries], "same_kernels": same, "stripped": co != s_co,
            "load_segments": len(loads), "aligned": aligned, "ascending": ascending}


def mmap_bundle_header(path: str) -> tuple[int, int, int]:
    """(version, compressed bytes, uncompressed bytes) of a library's bundle, cheaply."""
    with open(path, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as m:
        elf_hdr = EHDR.unpack_from(m, 0)
        shoff, shnum, shstrndx = elf_hdr[6], elf_hdr[12], elf_hdr[13]
        shdrs = [SHDR.unpack_from(m, shoff + i * SHDR.size) for i in range(shnum)]
        st = shdrs[shstrndx]
        strtab = m[st[4]:st[4] + st[5]]
        for s in shdrs:
            if strtab[s[0]:strtab.index(b"\0", s[0])] == b".hip_fatbin":
                if m[s[4]:s[4] + 24] == BUNDLE_MAGIC:  # uncompressed bundle
                    return 0, s[5], s[5]
                _, ver, _, total, unc, _ = CCOB_HDR.unpack_from(m, s[4])
                return ver, total, unc
    raise KeyError(".hip_fatbin")


if __name__ == "__main__":
    import argparse
    import json

    ap = argparse.ArgumentParser(description="trim a ROCm library's device code to one GPU arch")
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--arch", default="gfx950")
    ap.add_argument("--level", type=int, default=3)
    ap.add_argument("--verify", action="store_true")
    ap.add_argument("--keep-debug", action="store_true")
    ap.add_argument("--uncompressed", action="store_true", help="store the bundle without zstd")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(os.path.abspath(a.dst)), exist_ok=True)
    rep = slim_library(a.src, a.dst, a.arch, a.level, strip=not a.keep_debug, compress=not a.uncompressed)
    if a.verify:
        rep["verify"] = verify_library(a.dst, a.src, a.arch)
        if not rep["verify"]["ok"]:
            print(json.dumps(rep))
            raise SystemExit(1)
    print(json.dumps(rep))
