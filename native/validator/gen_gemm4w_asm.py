#!/usr/bin/env python3
"""Generate gemm4w_asm.inc: the main loop of the 4-wave 256x256 bf16 GEMM
(validator_kernels.hip, gemm_bf16_nt_4wa_kernel) as ONE inline-asm statement.

Why asm: the kernel keeps 256 fp32 accumulators per lane (a 128x128 wave
tile of v_mfma_f32_16x16x32_bf16) - the whole AGPR half of the register file
- next to ~100 VGPRs of operand fragments.  hipcc (ROCm 7.2) selects VGPR-form
MFMAs and then parks a few dozen accumulators in VGPRs, shuffling them through
v_accvgpr_read/write/mov every slice and spilling to scratch (measured on
every builtin variant of this loop: 44-840 copies per 64 MFMAs).  Written as
one statement, every register is placed once and the instruction stream is
exactly the schedule below; tests/test_gemm4w_asm.py checks this file is
regenerated whenever the generator changes and the schedules' invariants,
tests/test_kernels_gpu.py checks the kernels against an fp32 reference.

Schedules (each a function of this file; profiles/r4_gemm/ has the A/B):
  1  32-deep slices in a 5-slot ring of 64-B rows, slot registers rotated by
     SALU every slice (variant 15)
  2  the same ring, the body unrolled over 10 slices so every address is a
     constant, one filler per MFMA gap (24)
  3  2 with each slice pair's pieces back to back (25)
  4  64-deep stages in 128-B rows: whole-line LDS-DMA pieces, a ring of 5
     operand units (26); 4b drops the barriers the ring does not need (27);
     4c also issues each B unit early in its sub-slice (28, SHIPPED)
The 64-B-row schedules ask L2 for every line twice (TCC_HIT 2.3x hipBLASLt's
at equal misses): the step from 2 to 4 is worth 11 % (1273 -> 1416 TF/s at
4096^3) and takes MFMA utilisation from 0.75 to 0.83.

Register map (all named, all clobbered by the statement):
  a[0:255]   acc tile (i, j) of the wave's 8x8 grid at a[4(8i+j) : 4(8i+j)+3]
  v[0:23]    A fragments of rows 0-5 (re-read in place after their last use)
  v[24:31] / v[32:39]  A fragments of rows 6, 7: two sets, by slice parity
  v[40:71] / v[72:103] B fragments 0-7: two sets, by slice parity
  v104..     addresses (per schedule, see its section)
Per slice (32 deep, 1,024 MFMA cycles on the SIMD), interleaved between its
64 MFMAs: the 16 ds_read_b128 of the next slice's fragments and this wave's
8 LDS-DMA pieces (global_load_lds_dwordx4, 1 KiB each) of a later slice into
a slot the barrier freed; then the counted vmcnt, lgkmcnt(0) and s_barrier.
Hazards handled in the text: M0 write -> LDS-DMA one wait state; the last
MFMA's result -> the epilogue's v_accvgpr_read (s_nop 15 x 2 closes the
statement); a fragment register is re-read 3 MFMAs after its last use
(hipcc's own hazard recognizer pads a DS write after an MFMA source read with
nothing).
"""

from __future__ import annotations

import os
import re
import sys

SLICE_BYTES = 32 * 1024          # one ring slot: A 256x32 + B 256x32 bf16
NSLOT = 5
RING_BYTES = NSLOT * SLICE_BYTES  # 160 KiB
OP_BYTES = 16 * 1024             # one operand's slice
VM_INFLIGHT = 24                 # 3 slices x 8 pieces per wave

B_READ_AT = {3 * j + 1: j for j in range(8)}          # B fragment j of the next slice after MFMA 3j+1
A_READ_AT = {8 * i + 10: i for i in range(6)}         # A rows 0-5 in place, 3 MFMAs after their last use
A_READ_AT.update({25: 6, 28: 7})                      # A rows 6, 7 into the other set
PIECE_AT = {8 * q + 5: q for q in range(8)}           # LDS-DMA piece q


def a_reg(i: int, parity: int) -> str:
    if i < 6:
        return f"v[{4 * i}:{4 * i + 3}]"
    base = 24 + 8 * parity + 4 * (i - 6)
    return f"v[{base}:{base + 3}]"


def b_reg(j: int, parity: int) -> str:
    base = 40 + 32 * parity + 4 * j
    return f"v[{base}:{base + 3}]"


def acc(i: int, j: int) -> str:
    n = 4 * (8 * i + j)
    return f"a[{n}:{n + 3}]"


# named SGPRs (clobbered): the inputs are copied in at the start
SA, SB, ST = "s[80:81]", "s[82:83]", "s[84:85]"
SA_LO, SA_HI, SB_LO, SB_HI, ST_LO, ST_HI = "s80", "s81", "s82", "s83", "s84", "s85"
PS, SR, SW, SWAVE, SADV, SITER, STMP, SINC, SWS, SKEEP = ("s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93",
                                                          "s94", "s95")
SGPRS = range(80, 96)


def piece(q: int) -> list[str]:
    """This wave's piece q of the slice at sA/sB: operand q >> 2, row block
    (wave*4 + (q & 3)) of 16 rows; source = base + (q & 3) * piece stride."""
    lo, hi, base = (SA_LO, SA_HI, SA) if q < 4 else (SB_LO, SB_HI, SB)
    r = q & 3
    out = []
    if r == 0:
        src = base
    else:
        out += [f"s_add_u32 {ST_LO}, {lo if r == 1 else ST_LO}, {PS}",
                f"s_addc_u32 {ST_HI}, {hi if r == 1 else ST_HI}, 0"]
        src = ST
    off = (0 if q < 4 else OP_BYTES) + r * 1024
    if OPTS.get("vgpr_load"):  # ablation: the same load into VGPRs (no LDS write)
        return out + [f"global_load_dwordx4 v[110:113], v106, {src}"]
    if OPTS.get("fixed_m0"):  # ablation: no per-piece M0 set-up
        return out + [f"global_load_lds_dwordx4 v106, {src}"]
    out += [f"s_add_u32 m0, {SWS}, {off}", "s_nop 0", f"global_load_lds_dwordx4 v106, {src}"]
    return out


OPTS = {"glds": True, "barrier": True, "early_rotate": False, "dsread": True}


def rotate() -> list[str]:
    """Advance to the next slice: the load address moves on while slices are
    left to load (past the last one the refills re-read it into slots no one
    reads), the read and refill slots rotate through the ring."""
    lines = [f"s_cmp_gt_i32 {SADV}, 0", f"s_cselect_b32 {SINC}, 64, 0", f"s_sub_i32 {SADV}, {SADV}, 1",
             f"s_add_u32 {SA_LO}, {SA_LO}, {SINC}", f"s_addc_u32 {SA_HI}, {SA_HI}, 0",
             f"s_add_u32 {SB_LO}, {SB_LO}, {SINC}", f"s_addc_u32 {SB_HI}, {SB_HI}, 0"]
    for reg in (SR, SW):
        lines += [f"s_add_u32 {reg}, {reg}, {SLICE_BYTES}", f"s_sub_u32 {STMP}, {reg}, {RING_BYTES}",
                  f"s_cmp_ge_u32 {reg}, {RING_BYTES}", f"s_cselect_b32 {reg}, {STMP}, {reg}"]
    return lines


def slice_body(parity: int, first: bool) -> list[str]:
    """One slice: MFMAs on the fragments of set `parity`, the next slice's
    fragments into set 1 - parity, this wave's pieces of the slice to load."""
    nxt = 1 - parity
    lines = [f"v_add_u32 v107, {SR}, v104", f"v_add_u32 v108, {SR}, v105", f"s_add_u32 {SWS}, {SW}, {SWAVE}"]
    rot = rotate()
    for m in range(64):
        i, j = m >> 3, m & 7
        c = "0" if first else acc(i, j)
        lines.append(f"v_mfma_f32_16x16x32_bf16 {acc(i, j)}, {b_reg(j, parity)}, {a_reg(i, parity)}, {c}")
        if OPTS["early_rotate"]:  # the slice change's SALU work among the last MFMAs (after the last piece)
            if 56 <= m < 60:
                lines += rot[7 + 4 * (m - 56) // 2 * 0 + 2 * (m - 56):7 + 2 * (m - 56) + 2]
            elif m == 62:
                lines += rot[0:4]
            elif m == 63:
                lines += rot[4:7]
        if m in B_READ_AT and OPTS["dsread"]:
            jj = B_READ_AT[m]
            lines.append(f"ds_read_b128 {b_reg(jj, nxt)}, v108 offset:{jj * 1024}")
        if m in A_READ_AT and OPTS["dsread"]:
            ii = A_READ_AT[m]
            lines.append(f"ds_read_b128 {a_reg(ii, nxt)}, v107 offset:{ii * 1024}")
        if OPTS["glds"]:
            at = OPTS.get("piece_at") or PIECE_AT
            for q in at.get(m, ()) if isinstance(at.get(m), tuple) else ([at[m]] if m in at else []):
                lines += piece(q)
    if not OPTS["early_rotate"]:
        lines += rot

    lines += [f"s_waitcnt vmcnt({VM_INFLIGHT if OPTS['glds'] else 0}) lgkmcnt(0)"]
    if OPTS.get("fixed_m0"):
        lines.insert(0, f"s_mov_b32 m0, {SWAVE}")
    if OPTS["barrier"]:
        lines += ["s_barrier"]
    return lines


def stage(slot: int) -> list[str]:
    """Prologue: this wave's 8 pieces of the slice at sA/sB into `slot`, then
    advance the load address one slice."""
    out = [f"s_add_u32 {SWS}, {SWAVE}, {slot * SLICE_BYTES}"]
    for q in range(8):
        out += piece(q)
    out += [f"s_add_u32 {SA_LO}, {SA_LO}, 64", f"s_addc_u32 {SA_HI}, {SA_HI}, 0",
            f"s_add_u32 {SB_LO}, {SB_LO}, 64", f"s_addc_u32 {SB_HI}, {SB_HI}, 0"]
    return out


def program() -> list[str]:
    lines = [f"s_mov_b32 {SKEEP}, m0",
             f"s_mov_b32 {SA_LO}, %[a_lo]", f"s_mov_b32 {SA_HI}, %[a_hi]",
             f"s_mov_b32 {SB_LO}, %[b_lo]", f"s_mov_b32 {SB_HI}, %[b_hi]",
             f"s_mov_b32 {PS}, %[ps]", f"s_mov_b32 {SWAVE}, %[wave_lds]", f"s_mov_b32 {SADV}, %[adv]",
             f"s_mov_b32 {SITER}, %[iters]", f"s_mov_b32 {SR}, {SLICE_BYTES}", f"s_mov_b32 {SW}, 0",
             "v_mov_b32 v104, %[a_off]", "v_mov_b32 v105, %[b_off]", "v_mov_b32 v106, %[g_off]"]
    for s in range(NSLOT):  # slices 0..4 (K >= 256: nk >= 8 slices)
        lines += stage(s)
    # slices 0 and 1 landed (3 in flight), visible to every wave
    lines += [f"s_waitcnt vmcnt({VM_INFLIGHT})", "s_barrier"]
    for i in range(8):  # slice 0's fragments into set 0
        lines.append(f"ds_read_b128 {a_reg(i, 0)}, v104 offset:{i * 1024}")
    for j in range(8):
        lines.append(f"ds_read_b128 {b_reg(j, 0)}, v105 offset:{j * 1024}")
    lines += ["s_waitcnt lgkmcnt(0)", "s_barrier"]  # every wave's reads of slot 0 retired
    lines += slice_body(0, first=True)   # slice 0 (accumulators start from 0)
    lines += slice_body(1, first=False)  # slice 1
    lines += ["1:"]                      # slices 2.. in pairs
    lines += slice_body(0, first=False)
    lines += slice_body(1, first=False)
    lines += [f"s_sub_u32 {SITER}, {SITER}, 1", f"s_cmp_lg_u32 {SITER}, 0", "s_cbranch_scc1 1b"]
    lines += ["s_waitcnt vmcnt(0)",  # no LDS-DMA may outlive the workgroup
              "s_nop 15", "s_nop 15",  # last MFMA results -> the epilogue's accumulator reads
              f"s_mov_b32 m0, {SKEEP}"]
    return lines


HEADER = """// GENERATED by native/validator/gen_gemm4w_asm.py - do not edit; run
//   python3 native/validator/gen_gemm4w_asm.py > native/validator/gemm4w_asm.inc
// The 4-wave GEMM main loop as one asm statement (see the generator's
// docstring for the register map and the schedule).
"""


VARIANTS = {  # function suffix -> options (the shipped loop is "")
    "": {},
    "_noglds": {"glds": False},
    "_nobar": {"barrier": False},
    "_early": {"early_rotate": True},
    "_nods": {"dsread": False},
    "_fixm0": {"fixed_m0": True},
    "_vgpr": {"vgpr_load": True},
    "_pairs": {"piece_at": {16 * p + 5: (2 * p, 2 * p + 1) for p in range(4)}},
    "_burst": {"piece_at": {0: tuple(range(8))}},
}


def render() -> str:
    out = HEADER
    for suffix, opts in VARIANTS.items():
        OPTS.update({"glds": True, "barrier": True, "early_rotate": False, "dsread": True}, **opts)
        out += render_one(suffix)
    return out


def render_one(suffix: str) -> str:
    body = "\\n\\t".join(program())
    clob = ", ".join([f'"v{r}"' for r in range(114)] + [f'"s{r}"' for r in SGPRS] + [f'"a{r}"' for r in range(256)])
    return ("// a_lo/a_hi, b_lo/b_hi: global byte address of this wave's first A / B piece\n"
            "// of slice 0; ps: bytes between pieces (16 rows); wave_lds: LDS byte address of\n"
            "// this wave's first piece in slot 0; adv: nk - 6; iters: (nk - 2) / 2;\n"
            "// a_off / b_off: per-lane LDS byte address of fragment 0 of A / B in slot 0;\n"
            "// g_off: per-lane byte offset of the lane's 16 B within a piece.\n"
            f"__device__ __forceinline__ void avk_g4_mainloop{suffix}(unsigned a_lo, unsigned a_hi, unsigned b_lo, unsigned b_hi,\n"
            "                                                unsigned ps, unsigned wave_lds, int adv, unsigned iters,\n"
            "                                                unsigned a_off, unsigned b_off, unsigned g_off) {\n"
            f'  asm volatile("{body}"\n'
            "               :\n"
            "               : [a_lo] \"s\"(a_lo), [a_hi] \"s\"(a_hi), [b_lo] \"s\"(b_lo), [b_hi] \"s\"(b_hi), [ps] \"s\"(ps),\n"
            "                 [wave_lds] \"s\"(wave_lds), [adv] \"s\"(adv), [iters] \"s\"(iters), [a_off] \"v\"(a_off),\n"
            "                 [b_off] \"v\"(b_off), [g_off] \"v\"(g_off)\n"
            f"               : \"memory\", \"scc\", {clob});\n"
            "}\n")




# ----------------------------------------------------------------- schedule 2 --
# Fewer and better spread fillers between the MFMAs (counters of schedule 1,
# profiles/r4_gemm: MFMA util 0.79 even with the loads removed, SALU issue 2x
# hipBLASLt's): the loop body is unrolled over 10 slices (2 fragment parities
# x 5 ring slots), so every LDS address is a constant of the slice's
# position; each piece has its own global base SGPR pair (the wave's rows
# 16r.. of A or B, set once), the slice's k offset is one VGPR advanced once
# per slice (held on the last slice once the loads are past it: the refills
# then re-read it into slots no one reads).  Each MFMA gap carries at most one
# filler (a DS read, an M0 write or a load) but for the loop's own SALU, the
# M0 write one MFMA ahead of its load.
S2_BASE = [f"s[{64 + 2 * q}:{65 + 2 * q}]" for q in range(8)]  # piece q's global base
S2_WAVE, S2_CNT, S2_KEEP, S2_INC = "s80", "s81", "s82", "s83"
S2_SGPRS = range(64, 84)
S2_VOFF = "v106"
# v104/v105: A/B fragment 0 address in slot 0; v107/v108: + 64 KiB; v109/v110: + 128 KiB
S2_VBASE = {0: ("v104", "v105", 0), 1: ("v104", "v105", SLICE_BYTES), 2: ("v107", "v108", 0),
            3: ("v107", "v108", SLICE_BYTES), 4: ("v109", "v110", 0)}
S2_B_READ = {4 * j + 1: j for j in range(8)}
S2_A_READ = {8 * i + 10: i for i in range(6)}
S2_A_READ.update({37: 6, 45: 7})
S2_M0_AT = {8 * q + 6: q for q in range(8)}
S2_LOAD_AT = {8 * q + 7: q for q in range(8)}
S2_ADVANCE_MIN = NSLOT + 1  # slices left after this one for the refill address to move on


def s2_m0(slot: int, q: int) -> str:
    return f"s_add_u32 m0, {S2_WAVE}, {slot * SLICE_BYTES + (0 if q < 4 else OP_BYTES) + (q & 3) * 1024}"


def s2_slice(pos: int, first: bool = False, label: str | None = None) -> list[str]:
    """Slice at body position `pos` (0..9): fragments of parity pos % 2, reads
    of the next slice from slot (pos + 1) % 5, refill of slot pos % 5."""
    parity, nxt = pos % 2, 1 - pos % 2
    rslot, wslot = (pos + 1) % NSLOT, pos % NSLOT
    va, vb, off = S2_VBASE[rslot]
    lines = [f"{label}:"] if label else []
    for m in range(64):
        i, j = m >> 3, m & 7
        c = "0" if first else acc(i, j)
        lines.append(f"v_mfma_f32_16x16x32_bf16 {acc(i, j)}, {b_reg(j, parity)}, {a_reg(i, parity)}, {c}")
        if m in S2_B_READ:
            jj = S2_B_READ[m]
            lines.append(f"ds_read_b128 {b_reg(jj, nxt)}, {vb} offset:{off + jj * 1024}")
        if m in S2_A_READ:
            ii = S2_A_READ[m]
            lines.append(f"ds_read_b128 {a_reg(ii, nxt)}, {va} offset:{off + ii * 1024}")
        if m in S2_M0_AT:
            lines.append(s2_m0(wslot, S2_M0_AT[m]))
        if m in S2_LOAD_AT:
            lines.append(f"global_load_lds_dwordx4 {S2_VOFF}, {S2_BASE[S2_LOAD_AT[m]]}")
        if m == 40:  # this slice done: slices left; the refill address moves on while one is left to load
            lines += [f"s_sub_u32 {S2_CNT}, {S2_CNT}, 1"]
        if m == 41:
            lines += [f"s_cmp_ge_u32 {S2_CNT}, {S2_ADVANCE_MIN}", f"s_cselect_b32 {S2_INC}, 64, 0"]
    lines += [f"v_add_u32 {S2_VOFF}, {S2_INC}, {S2_VOFF}",
              f"s_waitcnt vmcnt({VM_INFLIGHT}) lgkmcnt(0)", f"s_cmp_eq_u32 {S2_CNT}, 0", "s_cbranch_scc1 3f",
              "s_barrier"]
    return lines


def program2() -> list[str]:
    lines = [f"s_mov_b32 {S2_KEEP}, m0",
             f"s_mov_b32 s64, %[a_lo]", f"s_mov_b32 s65, %[a_hi]",
             f"s_mov_b32 s72, %[b_lo]", f"s_mov_b32 s73, %[b_hi]"]
    for q in range(8):  # piece q's base = operand base + (q & 3) * ps
        if q & 3:
            lo, prev = 64 + 2 * q, 64 + 2 * (q - 1)
            lines += [f"s_add_u32 s{lo}, s{prev}, %[ps]", f"s_addc_u32 s{lo + 1}, s{prev + 1}, 0"]
    lines += [f"s_mov_b32 {S2_WAVE}, %[wave_lds]", f"s_mov_b32 {S2_CNT}, %[nk]",  # slices left, this one included
              "v_mov_b32 v104, %[a_off]", "v_mov_b32 v105, %[b_off]", f"v_mov_b32 {S2_VOFF}, %[g_off]",
              f"v_add_u32 v107, {2 * SLICE_BYTES}, v104", f"v_add_u32 v108, {2 * SLICE_BYTES}, v105",
              f"v_add_u32 v109, {4 * SLICE_BYTES}, v104", f"v_add_u32 v110, {4 * SLICE_BYTES}, v105"]
    for slot in range(NSLOT):  # slices 0..4 (nk >= 8)
        for q in range(8):
            lines += [s2_m0(slot, q), "s_nop 0", f"global_load_lds_dwordx4 {S2_VOFF}, {S2_BASE[q]}"]
        lines.append(f"v_add_u32 {S2_VOFF}, 64, {S2_VOFF}")
    lines += [f"s_waitcnt vmcnt({VM_INFLIGHT})", "s_barrier"]  # slices 0, 1 landed and visible
    for i in range(8):
        lines.append(f"ds_read_b128 {a_reg(i, 0)}, v104 offset:{i * 1024}")
    for j in range(8):
        lines.append(f"ds_read_b128 {b_reg(j, 0)}, v105 offset:{j * 1024}")
    lines += ["s_waitcnt lgkmcnt(0)", "s_barrier"]  # every wave's reads of slot 0 retired
    lines += s2_slice(0, first=True)
    lines += ["s_branch 2f"]
    lines += ["1:"] + s2_slice(0)
    lines += s2_slice(1, label="2")
    for pos in range(2, 10):
        lines += s2_slice(pos)
    lines += ["s_branch 1b", "3:",
              "s_waitcnt vmcnt(0)",  # no LDS-DMA may outlive the workgroup
              "s_nop 15", "s_nop 15",  # last MFMA results -> the epilogue's accumulator reads
              f"s_mov_b32 m0, {S2_KEEP}"]
    return lines


def render2() -> str:
    body = "\\n\\t".join(program2())
    clob = ", ".join([f'"v{r}"' for r in range(111)] + [f'"s{r}"' for r in S2_SGPRS] + [f'"a{r}"' for r in range(256)])
    return ("// Schedule 2: a_lo/a_hi, b_lo/b_hi, ps, wave_lds, a_off, b_off, g_off as above;\n"
            "// nk = K / 32 (a multiple of 8).\n"
            "__device__ __forceinline__ void avk_g4_mainloop2(unsigned a_lo, unsigned a_hi, unsigned b_lo, unsigned b_hi,\n"
            "                                                 unsigned ps, unsigned wave_lds, unsigned nk,\n"
            "                                                 unsigned a_off, unsigned b_off, unsigned g_off) {\n"
            f'  asm volatile("{body}"\n'
            "               :\n"
            "               : [a_lo] \"s\"(a_lo), [a_hi] \"s\"(a_hi), [b_lo] \"s\"(b_lo), [b_hi] \"s\"(b_hi), [ps] \"s\"(ps),\n"
            "                 [wave_lds] \"s\"(wave_lds), [nk] \"s\"(nk), [a_off] \"v\"(a_off), [b_off] \"v\"(b_off),\n"
            "                 [g_off] \"v\"(g_off)\n"
            f"               : \"memory\", \"scc\", {clob});\n"
            "}\n")


# ----------------------------------------------------------------- schedule 3 --
# Schedule 2's loop with the loads issued in slice PAIRS: on every even slice s
# each piece of slice s + 4 is followed at once by the same rows' piece of
# slice s + 5, the other 64 B of the same 128-B lines.  Schedule 2 asks L2
# for each line twice, 64 B a slice apart (TCC_HIT 2.3x hipBLASLt's at equal
# misses, profiles/r4_gemm); back to back, the second half can be served by
# the first request's line (vector L1 / the miss queue).  Slots (s+4) % 5 and
# s % 5 are both free at the start of an even slice s; every slice ends with
# vmcnt(16) (the pair issued last stays in flight).
S3_VOFF2 = "v111"        # S2_VOFF + 64: the pair's second slice
S3_B_READ = {4 * j + 1: j for j in range(8)}
S3_A_READ = {8 * i + 12: i for i in range(6)}
S3_A_READ.update({33: 6, 37: 7})
S3_M0_AT = {4 * p + 2: p for p in range(16)}
S3_LOAD_AT = {4 * p + 3: p for p in range(16)}
S3_VM = 16
S3_ADVANCE_MIN = 7       # slices left after this one for the next pair to exist


def s3_slice(pos: int, first: bool = False, label: str | None = None) -> list[str]:
    """Slice at body position `pos` (0..9); even positions load the pair
    (pos + 4, pos + 5): piece q of the pair's first slice goes to slot
    (pos + 4) % 5, of the second to slot pos % 5."""
    parity, nxt = pos % 2, 1 - pos % 2
    rslot = (pos + 1) % NSLOT
    va, vb, off = S2_VBASE[rslot]
    loads = pos % 2 == 0
    slots = ((pos + 4) % NSLOT, pos % NSLOT)
    lines = [f"{label}:"] if label else []
    for m in range(64):
        i, j = m >> 3, m & 7
        c = "0" if first else acc(i, j)
        lines.append(f"v_mfma_f32_16x16x32_bf16 {acc(i, j)}, {b_reg(j, parity)}, {a_reg(i, parity)}, {c}")
        if m in S3_B_READ:
            jj = S3_B_READ[m]
            lines.append(f"ds_read_b128 {b_reg(jj, nxt)}, {vb} offset:{off + jj * 1024}")
        if m in S3_A_READ:
            ii = S3_A_READ[m]
            lines.append(f"ds_read_b128 {a_reg(ii, nxt)}, {va} offset:{off + ii * 1024}")
        if loads and m in S3_M0_AT:
            p = S3_M0_AT[m]
            lines.append(s2_m0(slots[p & 1], p >> 1))
        if loads and m in S3_LOAD_AT:
            p = S3_LOAD_AT[m]
            lines.append(f"global_load_lds_dwordx4 {(S2_VOFF, S3_VOFF2)[p & 1]}, {S2_BASE[p >> 1]}")
        if m == 40:
            lines += [f"s_sub_u32 {S2_CNT}, {S2_CNT}, 1"]
        if loads and m == 41:
            lines += [f"s_cmp_ge_u32 {S2_CNT}, {S3_ADVANCE_MIN}", f"s_cselect_b32 {S2_INC}, 0x80, 0"]
    if loads:
        lines += [f"v_add_u32 {S2_VOFF}, {S2_INC}, {S2_VOFF}", f"v_add_u32 {S3_VOFF2}, {S2_INC}, {S3_VOFF2}"]
    lines += [f"s_waitcnt vmcnt({S3_VM}) lgkmcnt(0)", f"s_cmp_eq_u32 {S2_CNT}, 0", "s_cbranch_scc1 3f",
              "s_barrier"]
    return lines


def program3() -> list[str]:
    lines = program2()[:program2().index(f"v_add_u32 v110, {4 * SLICE_BYTES}, v105") + 1]
    lines.append(f"v_add_u32 {S3_VOFF2}, 64, {S2_VOFF}")
    for pair in range(2):  # slices 0..3 into slots 0..3, in pairs
        for p in range(16):
            lines += [s2_m0(2 * pair + (p & 1), p >> 1), "s_nop 0",
                      f"global_load_lds_dwordx4 {(S2_VOFF, S3_VOFF2)[p & 1]}, {S2_BASE[p >> 1]}"]
        lines += [f"v_add_u32 {S2_VOFF}, 0x80, {S2_VOFF}", f"v_add_u32 {S3_VOFF2}, 0x80, {S3_VOFF2}"]
    lines += [f"s_waitcnt vmcnt({S3_VM})", "s_barrier"]  # slices 0, 1 landed and visible
    for i in range(8):
        lines.append(f"ds_read_b128 {a_reg(i, 0)}, v104 offset:{i * 1024}")
    for j in range(8):
        lines.append(f"ds_read_b128 {b_reg(j, 0)}, v105 offset:{j * 1024}")
    lines += ["s_waitcnt lgkmcnt(0)", "s_barrier"]
    lines += s3_slice(0, first=True)
    lines += ["s_branch 2f"]
    lines += ["1:"] + s3_slice(0)
    lines += s3_slice(1, label="2")
    for pos in range(2, 10):
        lines += s3_slice(pos)
    lines += ["s_branch 1b", "3:",
              "s_waitcnt vmcnt(0)", "s_nop 15", "s_nop 15", f"s_mov_b32 m0, {S2_KEEP}"]
    return lines


def render3() -> str:
    return render2().replace("avk_g4_mainloop2(", "avk_g4_mainloop3(").replace(
        "// Schedule 2:", "// Schedule 3 (schedule 2, loads in slice pairs):").replace(
        "\\n\\t".join(program2()), "\\n\\t".join(program3())).replace(
        '"v110", ', '"v110", "v111", ')

# ----------------------------------------------------------------- schedule 4 --
# 64-deep K stages in 128-B LDS rows (the shape of hipBLASLt's requests):
# schedules 1-3 move each operand row as two 64-B halves a slice apart, so
# every LDS-DMA instruction touches 16 rows x 64 B (TCC_HIT 2.3x hipBLASLt's;
# the guide's measurement of the same shapes: address-unit busy 2x).  Here a
# piece is 8 rows x 128 B - whole lines - into an XOR-swizzled [rows][128 B]
# image, physical 16-B chunk p of row r holding logical chunk p ^ swz(r),
# swz(r) = ((r & 2) << 1) | ((r & 4) >> 1) (every ds_read_b128 lane group
# meets 16 distinct bank slots, tests/test_gemm4w_asm.py).
# The ring holds 5 units of 32 KiB, a unit = one operand of one stage
# (A_t = unit 2t, B_t = unit 2t + 1, slot = unit % 5).  Sub-slice u (k-half
# u & 1 of stage u >> 1, 64 MFMAs) reads the fragments of u + 1 and loads
# unit u + 4 into the slot the last reader left at the barrier before it;
# units of stage s must be in LDS by the barrier that ends sub-slice 2s - 2:
# vmcnt(8) after even sub-slices, vmcnt(16) after odd ones.
S4_SWZ = [((r & 2) << 1) | ((r & 4) >> 1) for r in range(8)]
UNIT_BYTES = 32 * 1024
S4_SA, S4_SB = "s[64:65]", "s[66:67]"
S4_SA_LO, S4_SA_HI, S4_SB_LO, S4_SB_HI = "s64", "s65", "s66", "s67"
S4_WAVE, S4_CNT, S4_KEEP, S4_INC, S4_ROW = "s68", "s69", "s70", "s71", "s72"
S4_SGPRS = range(64, 73)
# fragment address bases: (operand, h) -> VGPR for slots 0/1, 2/3, 4
S4_FBASE = {("A", 0): ("v104", "v106", "v108"), ("A", 1): ("v105", "v107", "v109"),
            ("B", 0): ("v110", "v112", "v114"), ("B", 1): ("v111", "v113", "v115")}
S4_VOFF = [f"v{116 + j}" for j in range(8)]  # piece j's per-lane global offset (rows 8j..)
S4_VGPRS = 124
S4_B_READ = {4 * j + 1: j for j in range(8)}
S4_A_READ = {8 * i + 10: i for i in range(6)}
S4_A_READ.update({37: 6, 45: 7})
S4_M0_AT = {8 * q + 6: q for q in range(8)}
S4_LOAD_AT = {8 * q + 7: q for q in range(8)}


def s4_addr(op: str, h: int, slot: int, i: int) -> str:
    base = S4_FBASE[(op, h)][slot // 2]
    return f"{base} offset:{(slot % 2) * UNIT_BYTES + i * 2048}"


def s4_m0(slot: int, j: int) -> str:
    return f"s_add_u32 m0, {S4_WAVE}, {slot * UNIT_BYTES + j * 1024}"


S4_OPTS = {"odd_barrier": True, "early_b": False}
S4_M0_EARLY = {4 * q + 2: q for q in range(8)}    # a B unit's pieces in the first half of its sub-slice
S4_LOAD_EARLY = {4 * q + 3: q for q in range(8)}


def s4_slice(pos: int, first: bool = False, label: str | None = None) -> list[str]:
    """Sub-slice at body position `pos` (u mod 10).  Only the barriers that
    end EVEN sub-slices are needed (the slot a sub-slice refills was last read
    at or before the even sub-slice before it, and units become visible at
    even barriers); with S4_OPTS["odd_barrier"] False the odd ones end with
    the wave's own lgkmcnt(0) only."""
    parity, nxt = pos % 2, 1 - pos % 2
    stage = (pos + 1) >> 1                 # stage of the fragments read (mod 5)
    h = (pos + 1) & 1
    aslot, bslot = (2 * stage) % NSLOT, (2 * stage + 1) % NSLOT
    lslot = (pos + 4) % NSLOT              # unit u + 4
    even = pos % 2 == 0                    # the unit loaded is an A unit
    src = S4_SA if even else S4_SB
    lines = [f"{label}:"] if label else []
    for m in range(64):
        i, j = m >> 3, m & 7
        c = "0" if first else acc(i, j)
        lines.append(f"v_mfma_f32_16x16x32_bf16 {acc(i, j)}, {b_reg(j, parity)}, {a_reg(i, parity)}, {c}")
        if m in S4_B_READ:
            jj = S4_B_READ[m]
            lines.append(f"ds_read_b128 {b_reg(jj, nxt)}, {s4_addr('B', h, bslot, jj)}")
        if m in S4_A_READ:
            ii = S4_A_READ[m]
            lines.append(f"ds_read_b128 {a_reg(ii, nxt)}, {s4_addr('A', h, aslot, ii)}")
        m0_at, load_at = ((S4_M0_EARLY, S4_LOAD_EARLY) if S4_OPTS["early_b"] and not even
                          else (S4_M0_AT, S4_LOAD_AT))
        if m in m0_at:
            lines.append(s4_m0(lslot, m0_at[m]))
        if m in load_at:
            lines.append(f"global_load_lds_dwordx4 {S4_VOFF[load_at[m]]}, {src}")
        if m == 40:
            lines += [f"s_sub_u32 {S4_CNT}, {S4_CNT}, 1"]
        if m == 41:  # the next unit of this operand exists: move its base one stage on
            lines += [f"s_cmp_ge_u32 {S4_CNT}, {7 if even else 6}", f"s_cselect_b32 {S4_INC}, 0x80, 0"]
    lo, hi = (S4_SA_LO, S4_SA_HI) if even else (S4_SB_LO, S4_SB_HI)
    lines += [f"s_add_u32 {lo}, {lo}, {S4_INC}", f"s_addc_u32 {hi}, {hi}, 0"]
    if even or S4_OPTS["odd_barrier"]:
        lines += [f"s_waitcnt vmcnt({8 if even else 16}) lgkmcnt(0)", f"s_cmp_eq_u32 {S4_CNT}, 0",
                  "s_cbranch_scc1 3f", "s_barrier"]
    else:
        lines += ["s_waitcnt lgkmcnt(0)", f"s_cmp_eq_u32 {S4_CNT}, 0", "s_cbranch_scc1 3f"]
    return lines


def program4() -> list[str]:
    lines = [f"s_mov_b32 {S4_KEEP}, m0",
             f"s_mov_b32 {S4_SA_LO}, %[a_lo]", f"s_mov_b32 {S4_SA_HI}, %[a_hi]",
             f"s_mov_b32 {S4_SB_LO}, %[b_lo]", f"s_mov_b32 {S4_SB_HI}, %[b_hi]",
             f"s_mov_b32 {S4_WAVE}, %[wave_lds]", f"s_lshl_b32 {S4_CNT}, %[ns], 1",  # sub-slices left, this one included
             f"s_mov_b32 {S4_ROW}, %[ps]",
             "v_mov_b32 v104, %[la0]", "v_mov_b32 v105, %[la1]", "v_mov_b32 v110, %[lb0]", "v_mov_b32 v111, %[lb1]",
             f"v_mov_b32 {S4_VOFF[0]}, %[g_off]"]
    for op in ("A", "B"):
        for h in (0, 1):
            b0, b2, b4 = S4_FBASE[(op, h)]
            lines += [f"v_add_u32 {b2}, {2 * UNIT_BYTES}, {b0}", f"v_add_u32 {b4}, {4 * UNIT_BYTES}, {b0}"]
    for j in range(1, 8):
        lines.append(f"v_add_u32 {S4_VOFF[j]}, {S4_ROW}, {S4_VOFF[j - 1]}")
    for unit in range(4):  # A_0, B_0, A_1, B_1 into slots 0..3
        lo, hi, src = (S4_SA_LO, S4_SA_HI, S4_SA) if unit % 2 == 0 else (S4_SB_LO, S4_SB_HI, S4_SB)
        for j in range(8):
            lines += [s4_m0(unit, j), "s_nop 0", f"global_load_lds_dwordx4 {S4_VOFF[j]}, {src}"]
        lines += ["s_nop 4", f"s_add_u32 {lo}, {lo}, 0x80", f"s_addc_u32 {hi}, {hi}, 0"]
    lines += ["s_waitcnt vmcnt(16)", "s_barrier"]  # A_0, B_0 landed and visible
    for i in range(8):
        lines.append(f"ds_read_b128 {a_reg(i, 0)}, {s4_addr('A', 0, 0, i)}")
    for j in range(8):
        lines.append(f"ds_read_b128 {b_reg(j, 0)}, {s4_addr('B', 0, 1, j)}")
    lines += ["s_waitcnt lgkmcnt(0)", "s_barrier"]
    lines += s4_slice(0, first=True)
    lines += ["s_branch 2f"]
    lines += ["1:"] + s4_slice(0)
    lines += s4_slice(1, label="2")
    for pos in range(2, 10):
        lines += s4_slice(pos)
    lines += ["s_branch 1b", "3:",
              "s_waitcnt vmcnt(0)", "s_nop 15", "s_nop 15", f"s_mov_b32 m0, {S4_KEEP}"]
    return lines


def render4(suffix: str = "", **opts) -> str:
    S4_OPTS.update({"odd_barrier": True, "early_b": False}, **opts)
    body = "\\n\\t".join(program4())
    S4_OPTS.update(odd_barrier=True, early_b=False)
    clob = ", ".join([f'"v{r}"' for r in range(S4_VGPRS)] + [f'"s{r}"' for r in S4_SGPRS]
                     + [f'"a{r}"' for r in range(256)])
    return ("// Schedule 4: 64-deep stages in 128-B rows.  a_lo/a_hi, b_lo/b_hi: global byte\n"
            "// address of this wave's first A / B row (rows wave*64..), stage 0; ps: 8 rows\n"
            "// in bytes; wave_lds: LDS byte address of this wave's first piece (slot 0);\n"
            "// ns = K / 64; la0/la1, lb0/lb1: per-lane LDS byte address of fragment 0 of\n"
            "// A / B, k-half 0 / 1, slot 0; g_off: per-lane byte offset in piece 0.\n"
            f"__device__ __forceinline__ void avk_g4_mainloop4{suffix}(unsigned a_lo, unsigned a_hi, unsigned b_lo, unsigned b_hi,\n"
            "                                                 unsigned ps, unsigned wave_lds, unsigned ns, unsigned la0,\n"
            "                                                 unsigned la1, unsigned lb0, unsigned lb1, unsigned g_off) {\n"
            f'  asm volatile("{body}"\n'
            "               :\n"
            "               : [a_lo] \"s\"(a_lo), [a_hi] \"s\"(a_hi), [b_lo] \"s\"(b_lo), [b_hi] \"s\"(b_hi), [ps] \"s\"(ps),\n"
            "                 [wave_lds] \"s\"(wave_lds), [ns] \"s\"(ns), [la0] \"v\"(la0), [la1] \"v\"(la1),\n"
            "                 [lb0] \"v\"(lb0), [lb1] \"v\"(lb1), [g_off] \"v\"(g_off)\n"
            f"               : \"memory\", \"scc\", {clob});\n"
            "}\n")

# ------------------------------------------------------------ schedule 8 (fp8) --
# The same ring, units, pieces and barriers as schedule 4b (every byte address
# of the data movement is schedule 4's: a 128-B row is 64 bf16 or 128 fp8 k),
# with v_mfma_f32_16x16x128_f8f6f4 (OCP e4m3 A and B: cbsz = blgp = 0) on the
# stage's whole 128-B rows: twice the cycles of the bf16 16x16x32 at 4x its K,
# so 2x its FLOP per cycle (MI355X_MICROARCH.md "FP8" row).  A stage is 64
# MFMAs in two sub-slices of 32 (1,024 MFMA cycles each, as schedule 4's):
# E(s) rows 0-3 and O(s) rows 4-7 of the wave's 8x8 tiles, both in B-major
# order (MFMA m = 4j + i').  A fragment is 16 rows x 32 B: lane l holds row
# l & 15, bytes 32 (l >> 4) .. +31 - two ds_read_b128 into 8 VGPRs.
#
# One register set per fragment (128 VGPRs), each read in place:
#   E(s) reads B4-7(s) (first used at E m = 16: counted lgkmcnt waits) and
#        A4-7(s) (used in O(s)); their registers were last read in O(s-1);
#   O(s) reads B0-3(s+1) three MFMAs after each one's last use in O(s), and
#        A0-3(s+1) (last used in E(s)) - stage s+1's units are visible after
#        the barrier that ends E(s) (vmcnt(8) there, as in schedule 4).
# 16 fragment reads per sub-slice either way.  The image swizzle differs from
# schedule 4's: this read pattern (chunks 2g, 2g + 1 of 16 rows per lane
# group) meets 16 distinct bank slots per ds_read_b128 lane group under
# S8_SWZ (tests/test_gemm4w_asm.py), under S4_SWZ it conflicts.
S8_SWZ = [((r >> 1) & 1) | (((r >> 2) & 1) << 2) for r in range(8)]
# (operand, 16-B half t of the lane's 32 B) -> fragment base VGPR for slots 0/1, 2/3, 4
S8_FBASE = {("A", 0): ("v128", "v130", "v132"), ("A", 1): ("v129", "v131", "v133"),
            ("B", 0): ("v134", "v136", "v138"), ("B", 1): ("v135", "v137", "v139")}
S8_VOFF = [f"v{140 + j}" for j in range(8)]
S8_VGPRS = 148
S8_M0_AT = {4 * q + 2: q for q in range(8)}
S8_LOAD_AT = {4 * q + 3: q for q in range(8)}


def a8(i: int) -> str:
    return f"v[{8 * i}:{8 * i + 7}]"


def b8(j: int) -> str:
    return f"v[{64 + 8 * j}:{64 + 8 * j + 7}]"


def s8_addr(op: str, t: int, slot: int, i: int) -> str:
    base = S8_FBASE[(op, t)][slot // 2]
    return f"{base} offset:{(slot % 2) * UNIT_BYTES + i * 2048}"


def s8_reads(pos: int) -> dict[int, list[tuple[str, str]]]:
    """MFMA index -> the fragment reads issued after it, (register, address)."""
    stage = pos >> 1
    out: dict[int, list[tuple[str, str]]] = {}
    if pos % 2 == 0:  # E: this stage's B4-7 (in place), then A4-7
        aslot, bslot = (2 * stage) % NSLOT, (2 * stage + 1) % NSLOT
        for n, j in enumerate(range(4, 8)):
            for t in (0, 1):
                out.setdefault(2 * n + t, []).append((f"v[{64 + 8 * j + 4 * t}:{64 + 8 * j + 4 * t + 3}]",
                                                      s8_addr("B", t, bslot, j)))
        for n, i in enumerate(range(4, 8)):
            for t in (0, 1):
                out.setdefault(8 + 2 * n + t, []).append((f"v[{8 * i + 4 * t}:{8 * i + 4 * t + 3}]",
                                                          s8_addr("A", t, aslot, i)))
    else:  # O: the next stage's B0-3 after their last use here, and A0-3
        aslot, bslot = (2 * stage + 2) % NSLOT, (2 * stage + 3) % NSLOT
        for j in range(4):
            for t in (0, 1):
                out.setdefault(4 * j + 6 + t, []).append((f"v[{64 + 8 * j + 4 * t}:{64 + 8 * j + 4 * t + 3}]",
                                                          s8_addr("B", t, bslot, j)))
        for i in range(4):
            for t in (0, 1):
                out.setdefault(20 + 2 * i + t, []).append((f"v[{8 * i + 4 * t}:{8 * i + 4 * t + 3}]",
                                                           s8_addr("A", t, aslot, i)))
    return out


def s8_slice(pos: int, first: bool = False, label: str | None = None) -> list[str]:
    """Sub-slice at body position `pos` (u mod 10): E (even) or O (odd) of
    stage pos >> 1 (mod 5); loads unit u + 4 like schedule 4b."""
    even = pos % 2 == 0
    rows = range(0, 4) if even else range(4, 8)
    lslot = (pos + 4) % NSLOT
    src = S4_SA if even else S4_SB
    reads = s8_reads(pos)
    issued: list[str] = []  # registers of the DS reads issued so far in this sub-slice, in order
    lines = [f"{label}:"] if label else []
    for m in range(32):
        j, i = m >> 2, rows[m & 3]
        if even and m % 4 == 0 and j >= 4:
            # B_j of this stage was read in this sub-slice: wait until its two reads are back
            # (LDS returns a wave's reads in order: later reads may stay outstanding)
            last = max(k for k, r in enumerate(issued) if r.startswith(f"v[{64 + 8 * j + 4}:"))
            lines.append(f"s_waitcnt lgkmcnt({len(issued) - 1 - last})")
        c = "0" if first else acc(i, j)
        lines.append(f"v_mfma_f32_16x16x128_f8f6f4 {acc(i, j)}, {b8(j)}, {a8(i)}, {c}")
        for reg, addr in reads.get(m, []):
            lines.append(f"ds_read_b128 {reg}, {addr}")
            issued.append(reg)
        if m in S8_M0_AT:
            lines.append(s4_m0(lslot, S8_M0_AT[m]))
        if m in S8_LOAD_AT:
            lines.append(f"global_load_lds_dwordx4 {S8_VOFF[S8_LOAD_AT[m]]}, {src}")
        if m == 20:
            lines += [f"s_sub_u32 {S4_CNT}, {S4_CNT}, 1"]
        if m == 21:  # the next unit of this operand exists: move its base one stage on
            lines += [f"s_cmp_ge_u32 {S4_CNT}, {7 if even else 6}", f"s_cselect_b32 {S4_INC}, 0x80, 0"]
    lo, hi = (S4_SA_LO, S4_SA_HI) if even else (S4_SB_LO, S4_SB_HI)
    lines += [f"s_add_u32 {lo}, {lo}, {S4_INC}", f"s_addc_u32 {hi}, {hi}, 0"]
    if even:
        lines += ["s_waitcnt vmcnt(8) lgkmcnt(0)", f"s_cmp_eq_u32 {S4_CNT}, 0", "s_cbranch_scc1 3f", "s_barrier"]
    else:
        lines += ["s_waitcnt lgkmcnt(0)", f"s_cmp_eq_u32 {S4_CNT}, 0", "s_cbranch_scc1 3f"]
    return lines


def program8() -> list[str]:
    lines = [f"s_mov_b32 {S4_KEEP}, m0",
             f"s_mov_b32 {S4_SA_LO}, %[a_lo]", f"s_mov_b32 {S4_SA_HI}, %[a_hi]",
             f"s_mov_b32 {S4_SB_LO}, %[b_lo]", f"s_mov_b32 {S4_SB_HI}, %[b_hi]",
             f"s_mov_b32 {S4_WAVE}, %[wave_lds]", f"s_lshl_b32 {S4_CNT}, %[ns], 1",  # sub-slices left, this one included
             f"s_mov_b32 {S4_ROW}, %[ps]",
             "v_mov_b32 v128, %[la0]", "v_mov_b32 v129, %[la1]", "v_mov_b32 v134, %[lb0]", "v_mov_b32 v135, %[lb1]",
             f"v_mov_b32 {S8_VOFF[0]}, %[g_off]"]
    for op in ("A", "B"):
        for t in (0, 1):
            b0, b2, b4 = S8_FBASE[(op, t)]
            lines += [f"v_add_u32 {b2}, {2 * UNIT_BYTES}, {b0}", f"v_add_u32 {b4}, {4 * UNIT_BYTES}, {b0}"]
    for j in range(1, 8):
        lines.append(f"v_add_u32 {S8_VOFF[j]}, {S4_ROW}, {S8_VOFF[j - 1]}")
    # the step to stage 2 only when there is one (K = 256 has stages 0 and 1):
    # the first sub-slices load the stage the pointers hold before their own
    # INC check, so with ns = 2 they re-load stage 1 into the free ring unit
    # instead of reading 128 B past the end of the last row of A / Bt
    lines += [f"s_cmp_gt_u32 %[ns], 2", f"s_cselect_b32 {S4_INC}, 0x80, 0"]
    for unit in range(4):  # A_0, B_0, A_1, B_1 into slots 0..3
        lo, hi, src = (S4_SA_LO, S4_SA_HI, S4_SA) if unit % 2 == 0 else (S4_SB_LO, S4_SB_HI, S4_SB)
        for j in range(8):
            lines += [s4_m0(unit, j), "s_nop 0", f"global_load_lds_dwordx4 {S8_VOFF[j]}, {src}"]
        lines += ["s_nop 4", f"s_add_u32 {lo}, {lo}, {'0x80' if unit < 2 else S4_INC}", f"s_addc_u32 {hi}, {hi}, 0"]
    lines += ["s_waitcnt vmcnt(16)", "s_barrier"]  # A_0, B_0 landed and visible
    for i in range(4):  # E(0)'s A0-3 and B0-3 (it reads its own B4-7 and O(0)'s A4-7)
        for t in (0, 1):
            lines.append(f"ds_read_b128 v[{8 * i + 4 * t}:{8 * i + 4 * t + 3}], {s8_addr('A', t, 0, i)}")
    for j in range(4):
        for t in (0, 1):
            lines.append(f"ds_read_b128 v[{64 + 8 * j + 4 * t}:{64 + 8 * j + 4 * t + 3}], {s8_addr('B', t, 1, j)}")
    lines += ["s_waitcnt lgkmcnt(0)", "s_barrier"]
    lines += s8_slice(0, first=True)   # E(0), O(0): every accumulator starts from 0
    lines += s8_slice(1, first=True)
    lines += ["s_branch 2f"]
    lines += ["1:"] + s8_slice(0) + s8_slice(1)
    lines += s8_slice(2, label="2")
    for pos in range(3, 10):
        lines += s8_slice(pos)
    lines += ["s_branch 1b", "3:",
              "s_waitcnt vmcnt(0)", "s_nop 15", "s_nop 15", f"s_mov_b32 m0, {S4_KEEP}"]
    return lines


def render8() -> str:
    body = "\\n\\t".join(program8())
    clob = ", ".join([f'"v{r}"' for r in range(S8_VGPRS)] + [f'"s{r}"' for r in S4_SGPRS]
                     + [f'"a{r}"' for r in range(256)])
    return ("// Schedule 8 (OCP fp8 e4m3, v_mfma_f32_16x16x128_f8f6f4): schedule 4b's data movement.\n"
            "// a_lo/a_hi, b_lo/b_hi: global byte address of this wave's first A / B row\n"
            "// (rows wave*64..), stage 0; ps: 8 rows in bytes; wave_lds: LDS byte address of\n"
            "// this wave's first piece (slot 0); ns = K / 128; la0/la1, lb0/lb1: per-lane LDS\n"
            "// byte address of 16-B half 0 / 1 of fragment 0 of A / B, slot 0; g_off: per-lane\n"
            "// byte offset in piece 0.\n"
            "__device__ __forceinline__ void avk_g8_mainloop(unsigned a_lo, unsigned a_hi, unsigned b_lo, unsigned b_hi,\n"
            "                                                unsigned ps, unsigned wave_lds, unsigned ns, unsigned la0,\n"
            "                                                unsigned la1, unsigned lb0, unsigned lb1, unsigned g_off) {\n"
            f'  asm volatile("{body}"\n'
            "               :\n"
            "               : [a_lo] \"s\"(a_lo), [a_hi] \"s\"(a_hi), [b_lo] \"s\"(b_lo), [b_hi] \"s\"(b_hi), [ps] \"s\"(ps),\n"
            "                 [wave_lds] \"s\"(wave_lds), [ns] \"s\"(ns), [la0] \"v\"(la0), [la1] \"v\"(la1),\n"
            "                 [lb0] \"v\"(lb0), [lb1] \"v\"(lb1), [g_off] \"v\"(g_off)\n"
            f"               : \"memory\", \"scc\", {clob});\n"
            "}\n")


# ------------------------------------------------------------ schedule 9 (fp4) --
# OCP FP4 (e2m1, two per byte, element 2k in the low nibble) on the same
# instruction with cbsz = blgp = 4: a 16x16x128 step takes 16 B of K per lane
# (4 VGPRs) at half the cycles of the fp8 one.  Schedule 8's data movement
# unchanged: a 128-B row is 256 k, so a stage is two k-steps - the two
# ds_read_b128 of a fragment are its k-step 0 (chunk g, g = lane >> 4) and
# k-step 1 (chunk g + 4); the kernel's per-lane addresses pick them, under
# S4_SWZ (conflict free for this pattern, tests/test_gemm4w_asm.py).  Each
# tile gets two MFMAs per sub-slice: k-step 0 in schedule 8's order, k-step 1
# S9_LAG tiles later (dependent accumulations never back to back), and every
# fragment read that overwrites a register moves S9_LAG slots later with its
# last use; the last S9_LAG k-step-1 MFMAs close the sub-slice.
S9_SWZ = [((r & 2) << 1) | ((r & 4) >> 1) for r in range(8)]
S9_LAG = 4


def a9(i: int, t: int) -> str:
    return f"v[{8 * i + 4 * t}:{8 * i + 4 * t + 3}]"


def b9(j: int, t: int) -> str:
    return f"v[{64 + 8 * j + 4 * t}:{64 + 8 * j + 4 * t + 3}]"


def s9_reads(pos: int) -> dict[int, list[tuple[str, str]]]:
    """Schedule 8's reads; those that overwrite a fragment used in this
    sub-slice (O's next-stage B0-3 and A0-3) S9_LAG slots later."""
    out = s8_reads(pos)
    if pos % 2 == 1:
        out = {m + S9_LAG: rd for m, rd in out.items()}
    return out


def s9_slice(pos: int, first: bool = False, label: str | None = None) -> list[str]:
    even = pos % 2 == 0
    rows = range(0, 4) if even else range(4, 8)
    lslot = (pos + 4) % NSLOT
    src = S4_SA if even else S4_SB
    reads = s9_reads(pos)
    issued: list[str] = []
    lines = [f"{label}:"] if label else []

    def mfma(m: int, t: int) -> str:
        j, i = m >> 2, rows[m & 3]
        c = "0" if first and t == 0 else acc(i, j)
        return f"v_mfma_f32_16x16x128_f8f6f4 {acc(i, j)}, {b9(j, t)}, {a9(i, t)}, {c} cbsz:4 blgp:4"

    for m in range(32 + S9_LAG):
        j = m >> 2
        if m < 32:
            if even and m % 4 == 0 and j >= 4:
                last = max(k for k, r in enumerate(issued) if r.startswith(f"v[{64 + 8 * j + 4}:"))
                lines.append(f"s_waitcnt lgkmcnt({len(issued) - 1 - last})")
            lines.append(mfma(m, 0))
        if m >= S9_LAG:
            lines.append(mfma(m - S9_LAG, 1))
        for reg, addr in reads.get(m, []):
            lines.append(f"ds_read_b128 {reg}, {addr}")
            issued.append(reg)
        if m in S8_M0_AT:
            lines.append(s4_m0(lslot, S8_M0_AT[m]))
        if m in S8_LOAD_AT:
            lines.append(f"global_load_lds_dwordx4 {S8_VOFF[S8_LOAD_AT[m]]}, {src}")
        if m == 20:
            lines += [f"s_sub_u32 {S4_CNT}, {S4_CNT}, 1"]
        if m == 21:
            lines += [f"s_cmp_ge_u32 {S4_CNT}, {7 if even else 6}", f"s_cselect_b32 {S4_INC}, 0x80, 0"]
    lo, hi = (S4_SA_LO, S4_SA_HI) if even else (S4_SB_LO, S4_SB_HI)
    lines += [f"s_add_u32 {lo}, {lo}, {S4_INC}", f"s_addc_u32 {hi}, {hi}, 0"]
    if even:
        lines += ["s_waitcnt vmcnt(8) lgkmcnt(0)", f"s_cmp_eq_u32 {S4_CNT}, 0", "s_cbranch_scc1 3f", "s_barrier"]
    else:
        lines += ["s_waitcnt lgkmcnt(0)", f"s_cmp_eq_u32 {S4_CNT}, 0", "s_cbranch_scc1 3f"]
    return lines


def program9() -> list[str]:
    """program8 with schedule 9's sub-slices (same prologue: the fragment
    reads of stage 0 are layout-agnostic)."""
    prog = program8()
    head = prog[:prog.index("s_waitcnt lgkmcnt(0)") + 2]  # through the prologue's second barrier
    assert head[-1] == "s_barrier"
    lines = list(head)
    lines += s9_slice(0, first=True)
    lines += s9_slice(1, first=True)
    lines += ["s_branch 2f"]
    lines += ["1:"] + s9_slice(0) + s9_slice(1)
    lines += s9_slice(2, label="2")
    for pos in range(3, 10):
        lines += s9_slice(pos)
    lines += ["s_branch 1b", "3:",
              "s_waitcnt vmcnt(0)", "s_nop 15", "s_nop 15", f"s_mov_b32 m0, {S4_KEEP}"]
    return lines


def render9() -> str:
    body = "\\n\\t".join(program9())
    clob = ", ".join([f'"v{r}"' for r in range(S8_VGPRS)] + [f'"s{r}"' for r in S4_SGPRS]
                     + [f'"a{r}"' for r in range(256)])
    return ("// Schedule 9 (OCP fp4 e2m1, v_mfma_f32_16x16x128_f8f6f4 cbsz:4 blgp:4): schedule 8's\n"
            "// data movement, two k-steps per 128-B row.  Arguments as avk_g8_mainloop, with\n"
            "// la0/la1, lb0/lb1 the per-lane LDS byte addresses of k-step 0 / 1 of fragment 0,\n"
            "// slot 0, and ns = K / 256.\n"
            "__device__ __forceinline__ void avk_g9_mainloop(unsigned a_lo, unsigned a_hi, unsigned b_lo, unsigned b_hi,\n"
            "                                                unsigned ps, unsigned wave_lds, unsigned ns, unsigned la0,\n"
            "                                                unsigned la1, unsigned lb0, unsigned lb1, unsigned g_off) {\n"
            f'  asm volatile("{body}"\n'
            "               :\n"
            "               : [a_lo] \"s\"(a_lo), [a_hi] \"s\"(a_hi), [b_lo] \"s\"(b_lo), [b_hi] \"s\"(b_hi), [ps] \"s\"(ps),\n"
            "                 [wave_lds] \"s\"(wave_lds), [ns] \"s\"(ns), [la0] \"v\"(la0), [la1] \"v\"(la1),\n"
            "                 [lb0] \"v\"(lb0), [lb1] \"v\"(lb1), [g_off] \"v\"(g_off)\n"
            f"               : \"memory\", \"scc\", {clob});\n"
            "}\n")


# ------------------------------------------------------------ schedule 10 (fp6) --
# OCP FP6 (e2m3: cbsz = blgp = 2) on schedule 8 unchanged: a lane's fragment
# of 32 fp6 is 24 B packed + 8 B of padding, so a 32-element block takes a
# 32-B slot and a row of K fp6 the K bytes of an fp8 row (the validator's
# storage layout for its synthetic fp6 operands, gemm_fp6_nt_kernel).  The
# instruction reads the first six VGPRs of each eight-VGPR fragment, at the
# fp4 rate: half the cycles of the fp8 step on the same bytes.
S10_FMT = {"e2m3": 2, "e3m2": 3}


def s10_slice(pos: int, first: bool = False, label: str | None = None, fmt: int = 2) -> list[str]:
    out = []
    for ln in s8_slice(pos, first, label):
        if ln.startswith("v_mfma_f32_16x16x128_f8f6f4 "):
            dst, b, a, c = [x.strip() for x in ln.split(" ", 1)[1].split(",")]
            six = [re.sub(r"\[(\d+):(\d+)\]", lambda mm: f"[{mm.group(1)}:{int(mm.group(1)) + 5}]", r) for r in (b, a)]
            ln = f"v_mfma_f32_16x16x128_f8f6f4 {dst}, {six[0]}, {six[1]}, {c} cbsz:{fmt} blgp:{fmt}"
        out.append(ln)
    return out


def program10(fmt: int = 2) -> list[str]:
    prog = program8()
    head = prog[:prog.index("s_waitcnt lgkmcnt(0)") + 2]
    assert head[-1] == "s_barrier"
    lines = list(head)
    lines += s10_slice(0, first=True, fmt=fmt)
    lines += s10_slice(1, first=True, fmt=fmt)
    lines += ["s_branch 2f"]
    lines += ["1:"] + s10_slice(0, fmt=fmt) + s10_slice(1, fmt=fmt)
    lines += s10_slice(2, label="2", fmt=fmt)
    for pos in range(3, 10):
        lines += s10_slice(pos, fmt=fmt)
    lines += ["s_branch 1b", "3:",
              "s_waitcnt vmcnt(0)", "s_nop 15", "s_nop 15", f"s_mov_b32 m0, {S4_KEEP}"]
    return lines


_MAINLOOP_ARGS = ("(unsigned a_lo, unsigned a_hi, unsigned b_lo, unsigned b_hi,\n"
                  "                                                 unsigned ps, unsigned wave_lds, unsigned ns, unsigned la0,\n"
                  "                                                 unsigned la1, unsigned lb0, unsigned lb1, unsigned g_off")
_MAINLOOP_IN = ("               : [a_lo] \"s\"(a_lo), [a_hi] \"s\"(a_hi), [b_lo] \"s\"(b_lo), [b_hi] \"s\"(b_hi), [ps] \"s\"(ps),\n"
                "                 [wave_lds] \"s\"(wave_lds), [ns] \"s\"(ns), [la0] \"v\"(la0), [la1] \"v\"(la1),\n"
                "                 [lb0] \"v\"(lb0), [lb1] \"v\"(lb1), [g_off] \"v\"(g_off)")


def render10() -> str:
    body = "\\n\\t".join(program10(S10_FMT["e2m3"]))
    clob = ", ".join([f'"v{r}"' for r in range(S8_VGPRS)] + [f'"s{r}"' for r in S4_SGPRS]
                     + [f'"a{r}"' for r in range(256)])
    return ("// Schedule 10 (OCP fp6 e2m3 in 32-B slots per 32 elements, v_mfma_f32_16x16x128_f8f6f4\n"
            "// cbsz:2 blgp:2): schedule 8's data movement and arguments (ns = K / 128).\n"
            "__device__ __forceinline__ void avk_g10_mainloop" + _MAINLOOP_ARGS + ") {\n"
            f'  asm volatile("{body}"\n'
            "               :\n" + _MAINLOOP_IN + "\n"
            f"               : \"memory\", \"scc\", {clob});\n"
            "}\n")


# ------------------------------------------------- schedule 11 (MX-scaled fp4) --
# Block-scaled OCP MXFP4 on schedule 9: v_mfma_scale_f32_16x16x128_f8f6f4 with
# one E8M0 scale per operand per lane per MFMA - the scale of the lane's
# 32-element k-block (a 16-B chunk of the 128-B row).  The validator's MX
# operands carry a scale per (row, k-block mod 8): a lane's scales are then
# the same in every stage, 16 bytes per operand (fragment i or j, k-step t ->
# byte 2i + t), loaded by the kernel into four VGPRs per operand before the
# loop and picked per MFMA by op_sel / op_sel_hi (byte = op_sel + 2 op_sel_hi).
# The instruction's first source is the B fragment (the product is computed
# transposed, as in every schedule here), so its scale is B's.
def s11_scale(op: str, idx: int, t: int) -> tuple[str, int]:
    byte = 2 * idx + t
    return f"%[s{op.lower()}{byte // 4}]", byte % 4


def s11_slice(pos: int, first: bool = False, label: str | None = None) -> list[str]:
    even = pos % 2 == 0
    rows = range(0, 4) if even else range(4, 8)
    out = []
    for ln in s9_slice(pos, first, label):
        if ln.startswith("v_mfma_f32_16x16x128_f8f6f4 "):
            ops = [x.strip() for x in ln.split(" ", 1)[1].split(" cbsz")[0].split(",")]
            dst, b, a, c = ops
            j = (int(re.match(r"v\[(\d+):", b).group(1)) - 64) // 8
            t = ((int(re.match(r"v\[(\d+):", b).group(1)) - 64) % 8) // 4
            i = int(re.match(r"v\[(\d+):", a).group(1)) // 8
            assert i in rows and t == (int(re.match(r"v\[(\d+):", a).group(1)) % 8) // 4
            sb, bb = s11_scale("B", j, t)
            sa, ba = s11_scale("A", i, t)
            ln = (f"v_mfma_scale_f32_16x16x128_f8f6f4 {dst}, {b}, {a}, {c}, {sb}, {sa} "
                  f"op_sel:[{bb & 1},{ba & 1},0] op_sel_hi:[{bb >> 1},{ba >> 1},0] cbsz:4 blgp:4")
        out.append(ln)
    return out


def program11() -> list[str]:
    prog = program8()
    head = prog[:prog.index("s_waitcnt lgkmcnt(0)") + 2]
    assert head[-1] == "s_barrier"
    lines = list(head)
    lines += s11_slice(0, first=True)
    lines += s11_slice(1, first=True)
    lines += ["s_branch 2f"]
    lines += ["1:"] + s11_slice(0) + s11_slice(1)
    lines += s11_slice(2, label="2")
    for pos in range(3, 10):
        lines += s11_slice(pos)
    lines += ["s_branch 1b", "3:",
              "s_waitcnt vmcnt(0)", "s_nop 15", "s_nop 15", f"s_mov_b32 m0, {S4_KEEP}"]
    return lines


def render11() -> str:
    body = "\\n\\t".join(program11())
    clob = ", ".join([f'"v{r}"' for r in range(S8_VGPRS)] + [f'"s{r}"' for r in S4_SGPRS]
                     + [f'"a{r}"' for r in range(256)])
    scales = ", ".join(f"unsigned s{op}{q}" for op in "ab" for q in range(4))
    scale_in = ", ".join(f'[s{op}{q}] "v"(s{op}{q})' for op in "ab" for q in range(4))
    return ("// Schedule 11 (MXFP4: v_mfma_scale_f32_16x16x128_f8f6f4 cbsz:4 blgp:4 with E8M0 block\n"
            "// scales): schedule 9's data movement and arguments (ns = K / 256), plus the lane's\n"
            "// scale bytes of A (sa0..sa3: fragment i, k-step t at byte 2i + t) and of B (sb0..sb3).\n"
            "__device__ __forceinline__ void avk_g11_mainloop" + _MAINLOOP_ARGS + ",\n"
            "                                                 " + scales + ") {\n"
            f'  asm volatile("{body}"\n'
            "               :\n" + _MAINLOOP_IN + ",\n"
            "                 " + scale_in + "\n"
            f"               : \"memory\", \"scc\", {clob});\n"
            "}\n")


def render_all() -> str:
    return (render() + render2() + render3() + render4() + render4("b", odd_barrier=False)
            + render4("c", odd_barrier=False, early_b=True) + render8() + render9() + render10() + render11())


if __name__ == "__main__":
    sys.stdout.write(render_all())
