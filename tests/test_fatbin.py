"""Arch-trimmed ROCm libraries (amdgpu_operator/toolkit/fatbin.py).

A synthetic two-arch (gfx942 + gfx950) HIP library with a compressed offload
bundle stands in for librccl on CPU: trimming keeps exactly the gfx950 kernels,
the ELF still loads (host code runs), and both rewrite paths are covered - the
segment split (library with a PT_NOTE slot) and the in-place rewrite.  The GPU
tests run the trimmed kernel on MI355X and the validator's RCCL step on the
trimmed librccl that native/Makefile builds."""

import ctypes
import json
import os
import subprocess

import pytest

from amdgpu_operator import native
from amdgpu_operator.toolkit import fatbin as F

HIPCC = "/opt/rocm/bin/hipcc"
PROBE_SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "native", "testdata",
                         "fatbin_probe.hip")


def _build(tmp, name, build_id):
    out = tmp / name
    cmd = [HIPCC, "-shared", "-fPIC", "-O2", "-g", "--offload-arch=gfx942", "--offload-arch=gfx950",
           "--offload-compress", PROBE_SRC, "-o", str(out)] + (["-Wl,--build-id"] if build_id else [])
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    return str(out)


@pytest.fixture(scope="module")
def libs(tmp_path_factory):
    """The two probe libraries native/Makefile builds (with / without a build-id
    note); compiled here only when the artefacts are missing (CPU tier)."""
    d = tmp_path_factory.mktemp("fatbin")
    built = {k: native.artefact(f"testdata/libfatbin_probe_{k}.so") for k in ("note", "plain")}
    if all(p.exists() for p in built.values()):
        return {"note": str(built["note"]), "plain": str(built["plain"]), "dir": d}
    if not os.path.exists(HIPCC):
        pytest.skip("no hipcc and no prebuilt probe libraries")
    return {"note": _build(d, "libk_note.so", True), "plain": _build(d, "libk_plain.so", False), "dir": d}


def test_source_bundle_has_both_arches(libs):
    _, entries, _ = F.fatbin_of(libs["note"])
    triples = [e.triple for e in entries]
    assert any(t.endswith("--gfx950") for t in triples) and any(t.endswith("--gfx942") for t in triples)


@pytest.mark.parametrize("kind,strip,compress", [("note", True, True), ("note", False, True), ("plain", True, True),
                                                   ("note", True, False)])
def test_trim_keeps_only_gfx950_and_loads(libs, kind, strip, compress):
    src = libs[kind]
    dst = str(libs["dir"] / f"out_{kind}_{strip}_{compress}.so")
    rep = F.slim_library(src, dst, "gfx950", strip=strip, compress=compress)
    if not compress:
        assert F.mmap_bundle_header(dst)[0] == 0  # plain __CLANG_OFFLOAD_BUNDLE__
    v = F.verify_library(dst, src, "gfx950")
    assert v["ok"], v
    assert v["entries"] == [F.HOST_TRIPLE, "hipv4-amdgcn-amd-amdhsa--gfx950"]
    assert v["stripped"] == strip
    if strip:
        assert rep["code_object_bytes"] < rep["code_object_bytes_with_debug"]
    if kind == "note" and strip and compress:  # segment split: the file shrinks, PT_NOTE slot becomes a PT_LOAD
        assert rep["file_bytes"] < rep["source_file_bytes"]
        elf = F.Elf(open(dst, "rb").read())
        assert not any(p[0] == F.PT_NOTE for p in elf.phdrs)
        assert sum(p[0] == F.PT_LOAD for p in elf.phdrs) == sum(p[0] == F.PT_LOAD for p in F.Elf(open(src, "rb").read()).phdrs) + 1
    elif compress:
        assert rep["file_bytes"] == rep["source_file_bytes"]
    # the dynamic loader maps it and the host code runs (static init registered the bundle)
    assert ctypes.CDLL(dst).answer() == 42


def test_ccob_roundtrip_and_hash():
    co = os.urandom(3000) + bytes(5000)
    blob = F.build_ccob(co, "hipv4-amdgcn-amd-amdhsa--gfx950", level=1)
    magic, ver, method, total, unc, _ = F.CCOB_HDR.unpack_from(blob, 0)
    assert (magic, ver, method, total) == (b"CCOB", 3, 1, len(blob))
    bundle = F.decompress_ccob(blob)
    assert len(bundle) == unc
    entries = F.parse_bundle(bundle)
    assert F.code_object(bundle, entries, "gfx950")[1] == co
    bad = bytearray(blob)
    bad[F.CCOB_HDR.size - 1] ^= 1  # hash byte
    with pytest.raises(ValueError, match="hash"):
        F.decompress_ccob(bad)
    with pytest.raises(KeyError):
        F.code_object(bundle, entries, "gfx942")


def test_missing_arch_is_an_error(libs, tmp_path):
    with pytest.raises(KeyError):
        F.slim_library(libs["plain"], str(tmp_path / "x.so"), "gfx1100")


def test_makefile_rccl_artefact_is_trimmed():
    """The validator's RCCL (native/Makefile RCCL_SLIM) holds gfx950 only, without DWARF."""
    path = native.artefact("rccl-gfx950/librccl.so.1")
    if not os.path.exists(path):
        pytest.skip("native artefacts not built")
    ver, total, unc = F.mmap_bundle_header(str(path))
    # stored uncompressed (the runtime skips a 108 MB zstd decode in ncclCommInitRank):
    # one code object instead of ROCm's 571 MB bundle / 5.3 GB uncompressed
    assert ver == 0 and total == unc < 256 << 20
    rep = json.loads(open(os.path.join(os.path.dirname(path), "trim.json")).read())
    assert rep["source_entries"] > 1 and rep["code_object_bytes"] < rep["code_object_bytes_with_debug"]


@pytest.mark.gpu
@pytest.mark.parametrize("compress", [True, False], ids=["zstd", "plain"])
def test_trimmed_kernel_runs_on_mi355x(libs, compress):
    import torch

    dst = str(libs["dir"] / f"gpu_trim_{compress}.so")
    F.slim_library(libs["note"], dst, "gfx950", strip=True, compress=compress)
    x = torch.zeros(1000, device="cuda")
    torch.cuda.synchronize()
    lib = ctypes.CDLL(dst)
    assert lib.launch_add1(ctypes.c_void_p(x.data_ptr()), 1000) == 0
    assert torch.equal(x.cpu(), torch.ones(1000))


@pytest.mark.gpu
@pytest.mark.parametrize("library", ["trimmed", "system"])
def test_validator_rccl_on_trimmed_and_system_library(tmp_path, library):
    env = dict(os.environ)
    if library == "system":
        env["AMDGPU_RCCL_LIBRARY"] = ""
    p = subprocess.run([str(native.binary("amdgpu-validator")), "--rendezvous", str(tmp_path), "--steps", "hip,rccl",
                        "--rccl-elems", str(1 << 20)], capture_output=True, text=True, timeout=120, env=env)
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0 and rep["ok"], rep
    r = {s["name"]: s for s in rep["steps"]}["rccl"]
    assert r["mismatches"] == 0
    if library == "trimmed":
        assert r["library"].endswith("rccl-gfx950/librccl.so.1")
    else:
        assert os.path.basename(r["library"]).startswith("librccl.so")
        assert "rccl-gfx950" not in r["library"]
