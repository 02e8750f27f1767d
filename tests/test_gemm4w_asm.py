"""The 4-wave GEMM's generated main loop (native/validator/gen_gemm4w_asm.py
-> gemm4w_asm.inc): the checked-in file is the generator's output, and the
schedules keep the invariants the kernel's correctness rests on (no GPU: the
instruction text is checked; tests/test_kernels_gpu.py runs the kernels).

Invariants of every schedule, per 64-MFMA slice (sub-slice in schedule 4):
  * 64 MFMAs, 16 fragment reads, 8 LDS-DMA pieces (schedule 3: 16 on even
    slices, none on odd ones);
  * an A fragment register is re-read >= 3 MFMAs after its last use, and B
    reads only go to the other parity's set;
  * each piece's M0 write has >= 1 instruction between it and its load, and
    the next M0 write comes only after that load (M0 is read at issue);
  * consecutive pieces are >= 4 MFMAs apart (back-to-back pieces were
    measured to corrupt the LDS image: round 4's ablation variants 22/23);
  * at most one filler (DS read, M0 write, load) per MFMA gap, but for the
    early B pieces of schedule 4c (a DS read and an M0 write may share);
  * the slice ends with the counted vmcnt, lgkmcnt(0), the exit test and the
    s_barrier (schedule 4b/4c: odd sub-slices end with lgkmcnt(0) only).
Schedule 4c (avk_g4_mainloop4c) is the shipped one (variant 28).
"""

import importlib.util
import os
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parents[1]
GEN = ROOT / "native" / "validator" / "gen_gemm4w_asm.py"
INC = ROOT / "native" / "validator" / "gemm4w_asm.inc"


def _gen():
    spec = importlib.util.spec_from_file_location("gen_gemm4w_asm", GEN)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_checked_in_inc_is_the_generator_output():
    g = _gen()
    assert INC.read_text() == g.render_all(), \
        "run: python3 native/validator/gen_gemm4w_asm.py > " + str(INC)


def _slices(lines):
    """Split the program after the first MFMA into slices ending in s_barrier
    (or the exit branch target)."""
    out, cur, started = [], [], False
    for ln in lines:
        if ln.startswith("v_mfma"):
            started = True
        if not started:
            continue
        cur.append(ln)
        if ln == "s_barrier":
            out.append(cur)
            cur = []
    return out


import pytest  # noqa: E402


@pytest.mark.parametrize("sched", [2, 3])
def test_schedule_slice_invariants(sched):
    g = _gen()
    prog = g.program2() if sched == 2 else g.program3()
    vm = g.VM_INFLIGHT if sched == 2 else g.S3_VM
    spacing = 8 if sched == 2 else 4
    slices = _slices(prog)
    assert len(slices) == 11  # the peeled first slice + the 10-slice body
    for n, sl in enumerate(slices):
        body = [ln for ln in sl if not ln.endswith(":")]
        mfma = [i for i, ln in enumerate(body) if ln.startswith("v_mfma")]
        assert len(mfma) == 64
        assert sum(ln.startswith("ds_read_b128") for ln in body) == 16
        loads = [i for i, ln in enumerate(body) if ln.startswith("global_load_lds_dwordx4")]
        pos = 0 if n == 0 else n - 1  # body position: the peeled slice 0, then 0..9
        assert len(loads) == (8 if sched == 2 else 16 if pos % 2 == 0 else 0)
        assert body[-4:] == [f"s_waitcnt vmcnt({vm}) lgkmcnt(0)", f"s_cmp_eq_u32 {g.S2_CNT}, 0",
                             "s_cbranch_scc1 3f", "s_barrier"]
        # one filler per gap
        for a, b in zip(mfma, mfma[1:]):
            fill = [ln for ln in body[a + 1:b] if ln.startswith(("ds_read", "global_load", "s_add_u32 m0"))]
            assert len(fill) <= 1, body[a:b + 1]
        # M0 write -> its load: at least one instruction between; nothing else writes M0 in between
        m0 = [i for i, ln in enumerate(body) if ln.startswith("s_add_u32 m0")]
        assert len(m0) == len(loads)
        for w, ld in zip(m0, loads):
            assert 1 < ld - w and not any(ln.startswith("s_add_u32 m0") for ln in body[w + 1:ld])
        # pieces spaced (schedule 2: 8 MFMAs; schedule 3: 4, each slice pair's halves back to back)
        at = [sum(1 for i in mfma if i < ld) for ld in loads]
        assert all(b - a >= spacing for a, b in zip(at, at[1:]))
        # A rows re-read in place only >= 3 MFMAs after the last MFMA reading them
        for k, ln in enumerate(body):
            m = re.match(r"ds_read_b128 (v\[\d+:\d+\])", ln)
            if not m:
                continue
            reg = m.group(1)
            before = [i for i in mfma if i < k]
            users = [n for n, i in enumerate(before) if reg in body[i].split(", ")[1:3]]
            if users:
                assert len(before) - 1 - users[-1] >= 2, (ln, len(before), users[-1])
            after = [i for i in mfma if i > k]
            # the register is not an MFMA source again in this slice (it holds the next slice's fragment)
            assert not any(reg in body[i].split(", ")[1:3] for i in after), ln


def test_schedule2_slot_rotation_covers_the_ring():
    g = _gen()
    reads, writes = [], []
    for pos in range(10):
        sl = g.s2_slice(pos)
        m0 = [int(ln.rsplit(", ", 1)[1]) for ln in sl if ln.startswith("s_add_u32 m0")]
        writes.append(min(m0) // g.SLICE_BYTES)
        reads.append((pos + 1) % g.NSLOT)
    assert writes == [p % 5 for p in range(10)]
    # a slot is refilled only in the slice after the one that read it
    for pos in range(10):
        assert writes[pos] == reads[(pos - 1) % 10]


# ds_read_b128 serves a wave in four groups of 16 lanes; a group is conflict
# free when its 16 addresses fall in 16 distinct 16-B slots of the 256-B bank row
_DS_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
              list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
              list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
              list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]


def test_schedule4_image_is_conflict_free_and_a_bijection():
    g = _gen()
    swz = g.S4_SWZ
    assert swz == [((r & 2) << 1) | ((r & 4) >> 1) for r in range(8)]
    for h in (0, 1):  # k-half of the 64-deep stage
        for base in range(0, 256, 16):  # fragment rows base..base+15 (wave tile rows)
            for grp in _DS_GROUPS:
                slots = set()
                for lane in grp:
                    r = base + (lane & 15)
                    p = (4 * h + (lane >> 4)) ^ swz[r % 8]
                    slots.add(((r * 128 + p * 16) % 256) // 16)
                assert len(slots) == 16
    # the LDS-DMA side: lane l of a piece writes physical chunk l & 7 of row l >> 3 and
    # fetches logical chunk (l & 7) ^ swz(row): every logical chunk of every row once
    got = {((lane >> 3), (lane & 7) ^ swz[lane >> 3]) for lane in range(64)}
    assert got == {(r, c) for r in range(8) for c in range(8)}


def test_schedule4_ring_and_counts():
    """Unit u + 4 loads in sub-slice u into a slot whose unit was last read in
    sub-slice u - 1 at the latest; the units of stage s are waited for at the
    barrier ending sub-slice 2s - 2 (vmcnt(8): the 8 pieces issued in it stay
    out) and never earlier than they were issued."""
    g = _gen()
    for pos in range(10):
        sl = g.s4_slice(pos)
        m0 = [int(ln.rsplit(", ", 1)[1]) for ln in sl if ln.startswith("s_add_u32 m0")]
        assert {x // g.UNIT_BYTES for x in m0} == {(pos + 4) % 5}
        assert sorted(x % g.UNIT_BYTES for x in m0) == [j * 1024 for j in range(8)]
        assert any(f"vmcnt({8 if pos % 2 == 0 else 16}) lgkmcnt(0)" in ln for ln in sl)
    # slot reuse: over a long run, the unit in a slot is read (sub-slices 2s-1, 2s for unit of
    # stage s) strictly before the next unit is loaded into it (sub-slice unit + 4 - 5 + ... )
    last_read = {}
    for u in range(0, 200):
        s = (u + 1) >> 1  # stage whose fragments are read in u
        for unit in (2 * s, 2 * s + 1):
            last_read[unit] = u
        loaded = u + 4
        prev = loaded - 5  # the unit that slot held
        if prev >= 0:
            assert last_read.get(prev, -1) < u, (u, prev)


def _subslices(lines):
    """Schedule 4: split after each exit test (every sub-slice has one)."""
    out, cur, started = [], [], False
    for ln in lines:
        if ln.startswith("v_mfma"):
            started = True
        if not started:
            continue
        cur.append(ln)
        if ln == "s_cbranch_scc1 3f":
            out.append(cur)
            cur = []
    return out


@pytest.mark.parametrize("variant", [{}, {"odd_barrier": False}, {"odd_barrier": False, "early_b": True}])
def test_schedule4_subslice_invariants(variant):
    g = _gen()
    g.S4_OPTS.update({"odd_barrier": True, "early_b": False}, **variant)
    try:
        subs = _subslices(g.program4())
    finally:
        g.S4_OPTS.update(odd_barrier=True, early_b=False)
    assert len(subs) == 11
    for n, sl in enumerate(subs):
        pos = 0 if n == 0 else n - 1
        even = pos % 2 == 0
        body = [ln for ln in sl if not ln.endswith(":") and ln != "s_barrier"]
        mfma = [i for i, ln in enumerate(body) if ln.startswith("v_mfma")]
        loads = [i for i, ln in enumerate(body) if ln.startswith("global_load_lds_dwordx4")]
        m0 = [i for i, ln in enumerate(body) if ln.startswith("s_add_u32 m0")]
        assert len(mfma) == 64 and len(loads) == 8 == len(m0)
        assert sum(ln.startswith("ds_read_b128") for ln in body) == 16
        for w, ld in zip(m0, loads):
            assert 1 < ld - w and not any(ln.startswith("s_add_u32 m0") for ln in body[w + 1:ld])
        at = [sum(1 for i in mfma if i < ld) for ld in loads]
        assert all(b - a >= 4 for a, b in zip(at, at[1:]))
        limit = 2 if variant.get("early_b") and not even else 1
        for a, b in zip(mfma, mfma[1:]):
            fill = [ln for ln in body[a + 1:b] if ln.startswith(("ds_read", "global_load", "s_add_u32 m0"))]
            assert len(fill) <= limit, body[a:b + 1]
        assert sl[-1] == "s_cbranch_scc1 3f"
        if even or variant.get("odd_barrier", True):
            assert f"s_waitcnt vmcnt({8 if even else 16}) lgkmcnt(0)" in sl[-3:]
        else:
            assert "s_waitcnt lgkmcnt(0)" in sl[-3:] and not any("vmcnt" in ln for ln in sl[-3:])
    # barriers: 2 in the prologue, then after every even sub-slice (the peeled one and 5 in the
    # body) and, in schedule 4, after the 5 odd ones too
    g.S4_OPTS.update({"odd_barrier": True, "early_b": False}, **variant)
    try:
        prog = g.program4()
    finally:
        g.S4_OPTS.update(odd_barrier=True, early_b=False)
    assert sum(ln == "s_barrier" for ln in prog) == 2 + 6 + (5 if variant.get("odd_barrier", True) else 0)


# ------------------------------------------------------------ schedule 8 (fp8) --

def test_schedule8_image_is_conflict_free_and_a_bijection():
    """fp8 fragments read 32 B per lane (chunks 2g, 2g + 1 of the 128-B row,
    g = lane >> 4) as two ds_read_b128: under S8_SWZ each of the two reads
    meets 16 distinct bank slots per lane group (under S4_SWZ they collide),
    and the LDS-DMA side still moves every logical chunk of every row once."""
    g = _gen()
    for swz, want_free in ((g.S8_SWZ, True), (g.S4_SWZ, False)):
        free = True
        for t in (0, 1):
            for base in range(0, 256, 16):
                for grp in _DS_GROUPS:
                    slots = {(((base + (lane & 15)) * 128 + ((2 * (lane >> 4) + t) ^ swz[lane & 7]) * 16) % 256) // 16
                             for lane in grp}
                    free &= len(slots) == 16
        assert free == want_free
    got = {((lane >> 3), (lane & 7) ^ g.S8_SWZ[lane >> 3]) for lane in range(64)}
    assert got == {(r, c) for r in range(8) for c in range(8)}
    # the two 16-B halves of a lane's 32 B stay a pair of adjacent chunks
    assert all(((2 * q) ^ s) ^ 1 == (2 * q + 1) ^ s for q in range(4) for s in g.S8_SWZ)


def _s8_stream(g):
    """Schedule 8 in execution order: prologue, the two peeled sub-slices,
    body positions 2..9, then two full turns of the body."""
    prog = g.program8()
    i2 = prog.index("2:")
    i1 = prog.index("1:")
    peel_end = prog.index("s_branch 2f")
    body = prog[i1 + 1:prog.index("s_branch 1b")]
    body = [ln for ln in body if ln != "2:"]
    return prog[:peel_end] + prog[i2 + 1:prog.index("s_branch 1b")] + body + body


def test_schedule8_fragment_hazards_and_waits():
    """Every fragment register is overwritten by a DS read only 3 or more MFMAs
    after the last MFMA that read it, and every MFMA reads only registers
    whose DS reads have returned (LDS returns a wave's reads in order:
    ``lgkmcnt(k)`` leaves the last k outstanding)."""
    import re

    g = _gen()
    pending: list[int] = []       # first VGPR of each outstanding DS read, in issue order
    last_use: dict[int, int] = {}  # VGPR -> index of the last MFMA that read it
    n_mfma = 0
    for ln in _s8_stream(g):
        if ln.startswith("s_waitcnt") and "lgkmcnt(" in ln:
            k = int(re.search(r"lgkmcnt\((\d+)\)", ln).group(1))
            pending = pending[len(pending) - k:] if k else []
        elif ln.startswith("ds_read_b128"):
            lo = int(re.match(r"ds_read_b128 v\[(\d+):", ln).group(1))
            for r in range(lo, lo + 4):
                assert n_mfma - last_use.get(r, -99) >= 3, (ln, n_mfma, last_use.get(r))
            pending.append(lo)
        elif ln.startswith("v_mfma"):
            regs = re.findall(r"v\[(\d+):(\d+)\]", ln)
            assert len(regs) == 2
            for a, b in regs:
                busy = [p for p in pending if int(a) <= p <= int(b)]
                assert not busy, (ln, busy)
                for r in range(int(a), int(b) + 1):
                    last_use[r] = n_mfma
            n_mfma += 1
    assert n_mfma == 32 * (2 + 8 + 20)


def test_schedule8_subslice_shape():
    g = _gen()
    for pos in range(10):
        sl = g.s8_slice(pos)
        assert sum(ln.startswith("v_mfma_f32_16x16x128_f8f6f4") for ln in sl) == 32
        assert sum(ln.startswith("ds_read_b128") for ln in sl) == 16
        assert sum(ln.startswith("global_load_lds_dwordx4") for ln in sl) == 8
        m0 = [int(ln.rsplit(", ", 1)[1]) for ln in sl if ln.startswith("s_add_u32 m0")]
        assert {x // g.UNIT_BYTES for x in m0} == {(pos + 4) % 5}  # unit u + 4, as schedule 4
        assert ("s_barrier" in sl) == (pos % 2 == 0)  # only even sub-slices end with a barrier (schedule 4b)
        # E reads this stage's units, O the next stage's (slot = base VGPR group x 2 + offset // unit)
        groups = {b: n for key, bases in g.S8_FBASE.items() for n, b in enumerate(bases)}
        read_slots = set()
        for ln in sl:
            if ln.startswith("ds_read_b128"):
                base, off = re.search(r", (v\d+) offset:(\d+)", ln).groups()
                read_slots.add(2 * groups[base] + int(off) // g.UNIT_BYTES)
        stage = (pos >> 1) + (pos & 1)
        assert read_slots == {(2 * stage) % 5, (2 * stage + 1) % 5}, (pos, read_slots)


def test_agpr_accumulators_live_from_the_main_loop_to_the_epilogue():
    """the epilogue reads the accumulators by AGPR name in asm
    statements the compiler knows nothing of.  In the built code object no
    instruction between a GEMM kernel's last MFMA (the end of the main-loop
    statement) and its end writes an AGPR (no spill, copy or reuse), all 256
    are read there, and nothing spills to scratch."""
    import re
    import shutil
    import subprocess

    from amdgpu_operator import native

    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    assert shutil.which(objdump) or os.path.exists(objdump)
    co = native.artefact("validator_kernels.co")
    text = subprocess.run([objdump, "-d", "--no-show-raw-insn", str(co)], capture_output=True, text=True,
                          check=True).stdout.splitlines()
    starts = [i for i, ln in enumerate(text) if re.match(r"^[0-9a-f]+ <.*>:$", ln)]
    checked = 0
    for k, st in enumerate(starts):
        name = text[st]
        if not ("gemm_fp8_nt_kernel" in name or "gemm_bf16_nt_4wa_kernel" in name):
            continue
        end = starts[k + 1] if k + 1 < len(starts) else len(text)
        body = [ln.strip() for ln in text[st + 1:end] if ln.strip() and not ln.strip().startswith(";")]
        last = max(i for i, ln in enumerate(body) if ln.startswith("v_mfma"))
        tail = body[last + 1:]
        assert not [ln for ln in tail if ln.startswith(("v_accvgpr_write", "v_accvgpr_mov", "v_mfma"))], name
        read = {int(m.group(1)) for ln in tail if (m := re.match(r"v_accvgpr_read_b32 v\d+, a(\d+)", ln))}
        assert read == set(range(256)), (name, len(read))
        assert not any("scratch_" in ln for ln in body), name
        checked += 1
    assert checked >= 4  # the shipped bf16 default (bf16 and f32 out) and the fp8 kernel (both outs)
