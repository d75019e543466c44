#!/usr/bin/env python3
"""Generate the hand-scheduled gfx950 assembly body of the f8a fp8 (OCP e4m3) GEMM kernel.

Writes ``k8s_nvidia_gpus_amd/ops/csrc/gemm_fp8_gfx950_f8a_kloop.inc`` — the fp8 counterpart of
``tools/gen_gemm_w4a_kloop.py`` (same LDS image, DMA pieces, buffer-resource advance, exact
lgkmcnt simulation and C-image epilogue; read that file's docstring first).

What differs for fp8: a K-tile is 128 fp8 deep (the same 128 B per row), and one
``v_mfma_scale_f32_16x16x128_f8f6f4`` (unit E8M0 scales) consumes a whole K-tile of a fragment
pair — the 16-B chunk fq (read at the K-half-0 offset) and chunk 4+fq (K-half-1 offset) of row frow
as one 8-VGPR operand. So a K-tile is 64 MFMAs of 32 cycles over ONE fragment set, and the
next K-tile's fragments cannot wait for a free K-half: B fragments (used by every row of MFMAs) and
A fragments 6, 7 are double-buffered by K-tile parity, A fragments 0-5 are re-read in place after
their last MFMA (8·I + 7). Per K-tile (buffer cur = t & 1), as in the hipcc fp8 kernel:
  top:       lgkmcnt(0) + barrier #1 — every wave holds tile t in registers, cur may be restaged —
             and the clamped DMA-source advance;
  slots 1, 3 … 31: the 16 DMA pieces of tile t+2 into cur (one per 64 cycles);
  slot 31:   vmcnt(16) + barrier #2 — tile t+1 (issued a K-tile earlier) landed everywhere;
  slots 32-63: the 32 reads of tile t+1 from the other buffer, one per MFMA gap, in first-use order
             — A'0, B'0..7, A'1..7 — each in-place A'I no earlier than the slot after MFMA 8·I + 7.

Register map:
  v[0:63]    A fragments (A[i] = v[8i:8i+7]: lo = chunk fq, hi = chunk 4+fq); v[204:219] A[6], A[7]
             of odd K-tiles
  v[64:127]  B fragments, set 0      v[128:191] B fragments, set 1
  v192..v195 LDS read bases, buffer 0: A lo, A hi, B lo, B hi     v196..v199 buffer 1
  v200/v201  DMA lane offsets A/B     v202 C-image base     v203 E8M0 scales (0x7f7f7f7f)
  a[4n:4n+3] accumulator tile n = 8·I + J; SGPRs as in the w4a generator.

usage: python tools/gen_gemm_f8a_kloop.py   (rerun after editing; the .inc is committed)
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
from gen_gemm_w4a_kloop import C_STRIDE, TILE, piece  # noqa: E402

OUT = os.path.join(os.path.dirname(__file__), "..", "k8s_nvidia_gpus_amd", "ops", "csrc",
                   "gemm_fp8_gfx950_f8a_kloop.inc")

# next-tile read order (first use in the next K-tile) and earliest slot of each A re-read
READS = [("a", 0)] + [("b", j) for j in range(8)] + [("a", i) for i in range(1, 8)]
BAR2 = 31                                                  # after the last DMA piece
DMA_SLOTS = [1 + 2 * i for i in range(16)]                 # 1, 3, … 31: one per 64 cycles
A_DOUBLE = (6, 7)      # A fragments re-read too late to stay in place: double-buffered by parity


def a_reg(i: int, half: int, s: int = 0) -> str:
    b = (204 + 8 * (i - A_DOUBLE[0]) if (s and i in A_DOUBLE) else 8 * i) + 4 * half
    return f"v[{b}:{b + 3}]"


def atag(i: int, half: int, s: int) -> str:
    """LDS-queue tag of an A fragment read (double-buffered fragments carry their set)."""
    return f"a{i}{half}" + (f"s{s}" if i in A_DOUBLE else "")


def b_reg(s: int, j: int, half: int) -> str:
    b = 64 + 64 * s + 8 * j + 4 * half
    return f"v[{b}:{b + 3}]"


def read_slots(per_slot: int = 1):
    """(slot, operand, index, half) for the 32 next-tile reads after barrier #2, `per_slot` per MFMA
    gap, each in-place A'I no earlier than the slot after MFMA 8·I + 7."""
    out, slot, used = [], BAR2 + 1, 0
    for opnd, idx in READS:
        if opnd == "a" and idx > 0 and idx not in A_DOUBLE and slot < 8 * idx + 8:
            slot, used = 8 * idx + 8, 0
        for half in (0, 1):
            out.append((min(slot, 63), opnd, idx, half))
            used += 1
            if used == per_slot:
                slot, used = slot + 1, 0
    assert all(BAR2 < s <= 63 for s, *_ in out)
    return out


# schedules: name → reads per MFMA gap after barrier #2
SCHEDULES = {"spread": 1, "dense": 2}
DEFAULT = "dense"


def body(parity: int, queue: list, per_slot: int = 1) -> list:
    """One K-tile: barrier #1 (lgkmcnt(0): every wave holds tile t) and the clamped DMA-source
    advance sit before MFMA 0; op lists after[k] issue right after MFMA k."""
    after = [[] for _ in range(64)]
    nxt = 1 - parity
    top = ["s_waitcnt lgkmcnt(0)", "s_barrier", "s_add_u32 s75, s73, 2", "s_cmp_lt_u32 s75, s72",
           "s_cselect_b32 s76, 0x80, 0", "s_add_u32 s64, s64, s76", "s_addc_u32 s65, s65, 0",
           "s_add_u32 s68, s68, s76", "s_addc_u32 s69, s69, 0"]
    queue.clear()
    for p, slot in enumerate(DMA_SLOTS):
        opnd, row, off = piece(p)
        rs, voff = ("s[64:67]", "v200") if opnd == "A" else ("s[68:71]", "v201")
        assert slot >= 1
        after[slot - 1].append(("salu", None, f"s_add_u32 m0, s74, {parity * TILE + off}"))
        after[slot].append(("vmem", None, f"buffer_load_dwordx4 {voff}, {rs}, {row} offen lds"))
    after[BAR2] += [("waitv", None, "s_waitcnt vmcnt(16)"), ("bar", None, "s_barrier")]
    for slot, opnd, idx, half in read_slots(per_slot):
        base = f"v{192 + 4 * nxt + (0 if opnd == 'a' else 2) + half}"
        dst = a_reg(idx, half, nxt) if opnd == "a" else b_reg(nxt, idx, half)
        tag = atag(idx, half, nxt) if opnd == "a" else f"b{nxt}{idx}{half}"
        after[slot].append(("lds", tag, f"ds_read_b128 {dst}, {base} offset:{idx * 2048}"))
    out = list(top)
    for k in range(64):
        I, J = k >> 3, k & 7
        needed = {atag(I, 0, parity), atag(I, 1, parity), f"b{parity}{J}0", f"b{parity}{J}1"}
        need = [i for i, tag in enumerate(queue) if tag in needed]
        if need:
            keep = min(len(queue) - need[-1] - 1, 15)
            out.append(f"s_waitcnt lgkmcnt({keep})")
            del queue[: len(queue) - keep]
        n = 8 * I + J
        a_lo = int(a_reg(I, 0, parity)[2:].split(":")[0])
        # the unscaled f8f6f4 MFMA (operand formats cbsz = blgp = 0: OCP e4m3) — what the unit E8M0
        # scales of the _scale form compute, in an 8-byte encoding instead of 16
        out.append(f"v_mfma_f32_16x16x128_f8f6f4 a[{4 * n}:{4 * n + 3}], "
                   f"v[{64 + 64 * parity + 8 * J}:{64 + 64 * parity + 8 * J + 7}], "
                   f"v[{a_lo}:{a_lo + 7}], a[{4 * n}:{4 * n + 3}]")
        for kind, tag, ins in after[k]:
            if kind == "lds":
                queue.append(tag)
            elif kind == "wait0":
                queue.clear()
            out.append(ins)
    return out


def prologue() -> list:
    out = ["s_mov_b32 s72, %0", "s_mov_b32 s64, %1", "s_and_b32 s65, %2, 0xffff",
           "s_mov_b32 s66, %3", "s_mov_b32 s67, 0x20000", "s_mov_b32 s68, %4",
           "s_and_b32 s69, %5, 0xffff", "s_mov_b32 s70, %6", "s_mov_b32 s71, 0x20000",
           "s_mov_b32 s74, %9"]
    for e in range(8):
        rows = (e >> 1) * 32 + (e & 1) * 128
        out.append(f"s_mul_i32 s{80 + e}, %7, {rows}")
        out.append(f"s_mul_i32 s{88 + e}, %8, {rows}")
    for i in range(4):                  # v192 A lo, v193 A hi, v194 B lo, v195 B hi; +64 KiB: buf 1
        out.append(f"v_mov_b32 v{192 + i}, %{10 + i}")
        out.append(f"v_add_u32 v{196 + i}, {TILE}, %{10 + i}")
    out += ["v_mov_b32 v200, %14", "v_mov_b32 v201, %15", "v_mov_b32 v202, %16",
            "v_mov_b32 v203, 0x7f7f7f7f"]
    # the 256 accumulator zero-writes fill the gaps between the 32 prologue DMA issues (8 per gap:
    # they also cover the M0 → LDS-DMA hazard) instead of delaying the first DMA
    zero = [f"v_accvgpr_write_b32 a{r}, 0" for r in range(256)]
    for buf in range(2):
        if buf == 1:
            out += ["s_cmp_gt_u32 s72, 1", "s_cselect_b32 s76, 0x80, 0",
                    "s_add_u32 s64, s64, s76", "s_addc_u32 s65, s65, 0",
                    "s_add_u32 s68, s68, s76", "s_addc_u32 s69, s69, 0"]
        for p in range(16):
            opnd, row, off = piece(p)
            rs, voff = ("s[64:67]", "v200") if opnd == "A" else ("s[68:71]", "v201")
            gap = zero[(buf * 16 + p) * 8:(buf * 16 + p + 1) * 8]
            out += [f"s_add_u32 m0, s74, {buf * TILE + off}", *gap,
                    f"buffer_load_dwordx4 {voff}, {rs}, {row} offen lds"]
    out += ["s_waitcnt vmcnt(16)", "s_barrier"]
    for opnd, idx in READS:             # tile 0 into A and B set 0, in the loop's read order
        for half in (0, 1):
            base = f"v{192 + (0 if opnd == 'a' else 2) + half}"
            dst = a_reg(idx, half) if opnd == "a" else b_reg(0, idx, half)
            out.append(f"ds_read_b128 {dst}, {base} offset:{idx * 2048}")
    out.append("s_mov_b32 s73, 0")
    return out


def epilogue() -> list:
    out = ["s_waitcnt vmcnt(0) lgkmcnt(0)", "s_nop 15", "s_nop 15", "s_barrier"]
    for i in range(8):
        bank = 64 + 16 * (i & 1)
        if i >= 2:
            out.append("s_waitcnt lgkmcnt(8)")
        for j in range(8):
            n = 8 * i + j
            for c in range(4):
                out.append(f"v_accvgpr_read_b32 v{4 * j + c}, a{4 * n + c}")
        for j in range(8):
            out.append(f"v_cvt_pk_bf16_f32 v{bank + 2 * j}, v{4 * j}, v{4 * j + 1}")
            out.append(f"v_cvt_pk_bf16_f32 v{bank + 2 * j + 1}, v{4 * j + 2}, v{4 * j + 3}")
        for j in range(8):
            out.append(f"ds_write_b64 v202, v[{bank + 2 * j}:{bank + 2 * j + 1}] "
                       f"offset:{i * 16 * C_STRIDE + j * 32}")
    out.append("s_waitcnt lgkmcnt(0)")
    return out


def kernel_asm(per_slot: int) -> list:
    lines = prologue()
    bodies = []
    # LDS reads outstanding at the top of a K-tile of parity p: the 32 next-tile reads of the
    # previous K-tile, which wrote B set p (tile 0's prologue reads fill set 0 in the same order)
    q_start = {p: [atag(i, h, p) if o == "a" else f"b{p}{i}{h}" for o, i in READS for h in (0, 1)]
               for p in (0, 1)}
    for parity in (0, 1):
        q = list(q_start[parity])
        bodies.append(body(parity, q, per_slot))
        assert q == q_start[1 - parity], q
    lines.append("amdk8s_f8a_loop_%=:")
    lines += bodies[0]
    lines += ["s_add_u32 s73, s73, 1", "s_cmp_ge_u32 s73, s72", "s_cbranch_scc1 amdk8s_f8a_end_%="]
    lines += bodies[1]
    lines += ["s_add_u32 s73, s73, 1", "s_cmp_lt_u32 s73, s72", "s_cbranch_scc1 amdk8s_f8a_loop_%="]
    lines.append("amdk8s_f8a_end_%=:")
    lines += epilogue()
    return lines


def main():
    names = list(SCHEDULES)
    clob = ([f'"v{i}"' for i in range(204 + 8 * len(A_DOUBLE))] + [f'"a{i}"' for i in range(256)]
            + [f'"s{i}"' for i in range(64, 96)] + ['"scc"', '"memory"'])
    with open(OUT, "w") as f:
        f.write("// GENERATED by tools/gen_gemm_f8a_kloop.py — do not edit by hand.\n")
        f.write(f"// schedules: {', '.join(f'{i} = {n}' for i, n in enumerate(names))}; "
                f"default {DEFAULT}\n")
        f.write(f"#define AMDK8S_F8A_NUM_SCHEDULES {len(names)}\n")
        f.write(f"#define AMDK8S_F8A_DEFAULT_SCHEDULE {names.index(DEFAULT)}\n")
        f.write("#define AMDK8S_F8A_SCHEDULE_NAMES {" + ", ".join(f'"{n}"' for n in names) + "}\n")
        for i, n in enumerate(names):
            lines = kernel_asm(SCHEDULES[n])
            f.write(f"\n// {n}: {sum(1 for l in lines if 'v_mfma' in l)} MFMAs, "
                    f"{len(lines)} instructions\n#define AMDK8S_F8A_ASM_{i} \\\n")
            for ln in lines:
                f.write(f'  "{ln}\\n" \\\n')
            f.write("  \"\"\n")
        f.write("\n#define AMDK8S_F8A_CLOBBERS \\\n")
        for i in range(0, len(clob), 12):
            f.write("  " + ", ".join(clob[i:i + 12]) + (", \\\n" if i + 12 < len(clob) else "\n"))
    print(f"wrote {OUT}: schedules {names}")


if __name__ == "__main__":
    main()
