#!/usr/bin/env python3
"""Generate the hand-scheduled gfx950 assembly body of the w4a bf16 GEMM kernel.

Writes ``k8s_nvidia_gpus_amd/ops/csrc/gemm_bf16_gfx950_w4a_kloop.inc``: one ``asm volatile`` body
(prologue DMA, the K-loop unrolled by two LDS-buffer parities, the accumulator → bf16 → LDS
C-image epilogue) with every register explicit, so no compiler-inserted instruction sits between
the MFMAs. Op placement is the REGION schedule of ``gemm_bf16_gfx950_w4.hip`` (one op per MFMA
gap, three barriers per K-tile); the counted ``s_waitcnt lgkmcnt`` before each MFMA is computed
here by simulating the in-order LDS return queue, instead of hipcc's conservative counting.

Register map (kernel side passes operands; the asm copies them into these):
  v[0:31]  a0 fragments (a0[i] = v[4i:4i+3])      v[32:63] b0      v[64:95] a1      v[96:127] b1
  v128..v131  LDS read bases, buffer 0: A K-half 0, A K-half 1, B K-half 0, B K-half 1
  v132..v135  same for buffer 1 (+64 KiB)         v136/v137 DMA lane offsets A/B   v138 C-image base
  a[4n:4n+3]  accumulator tile n = 8·I + J (I: A fragment, J: B fragment)
  s[64:67] / s[68:71]  buffer resources A / B (base advanced one K-tile at a time, clamped)
  s72 T   s73 t   s74 LDS DMA base of this wave   s75/s76 scratch   s[80:87] / s[88:95] row offsets

usage: python tools/gen_gemm_w4a_kloop.py   (rerun after editing; the .inc is committed)
"""
from __future__ import annotations

import os

OUT = os.path.join(os.path.dirname(__file__), "..", "k8s_nvidia_gpus_amd", "ops", "csrc",
                   "gemm_bf16_gfx950_w4a_kloop.inc")

HALF = 16384          # bytes of one 128-row operand half in a K-tile buffer
TILE = 4 * HALF       # A0 A1 B0 B1
C_STRIDE = 528        # padded C-image row (bytes)


def frag(kind: str, idx: int) -> str:
    base = {"a0": 0, "b0": 32, "a1": 64, "b1": 96}[kind] + 4 * idx
    return f"v[{base}:{base + 3}]"


def read_order(x: int):
    """x-th fragment read of a K-half in first-use order: b[0..3], a[0], b[4..7], a[1..7]."""
    if x < 4:
        return "b", x
    if x == 4:
        return "a", 0
    if x < 9:
        return "b", x - 1
    return "a", x - 8


def piece(p: int):
    """DMA piece p: (operand, row-register, LDS byte offset inside a K-tile buffer)."""
    j, h = p >> 2, (p >> 1) & 1
    e = p >> 1                                  # index among the 8 pieces of this operand
    if p % 2 == 0:
        return "A", f"s{80 + e}", j * 4096 + h * HALF
    return "B", f"s{88 + e}", j * 4096 + (2 + h) * HALF


class Body:
    """One K-tile (128 MFMA slots) with ops attached after MFMA k, plus the lgkm simulation."""

    def __init__(self, parity: int):
        self.P = parity
        self.after = [[] for _ in range(128)]

    # LDS read bases for this parity
    def rd_base(self, which: str, operand: str, khalf: int) -> str:
        buf = self.P if which == "cur" else 1 - self.P
        return f"v{128 + 4 * buf + (0 if operand == 'a' else 2) + khalf}"

    def read(self, which: str, khalf: int, x: int):
        op, idx = read_order(x)
        dst = frag(f"{op}{'1' if khalf else '0'}", idx)
        base = self.rd_base(which, op, khalf)
        return ("lds", f"{op}{'1' if khalf else '0'}{idx}",
                f"ds_read_b128 {dst}, {base} offset:{idx * 2048}")

    def dma(self, p: int):
        opnd, row, off = piece(p)
        rs = "s[64:67]" if opnd == "A" else "s[68:71]"
        voff = "v136" if opnd == "A" else "v137"
        m0 = ("salu", None, f"s_add_u32 m0, s74, {self.P * TILE + off}")
        ld = ("vmem", None, f"buffer_load_dwordx4 {voff}, {rs}, {row} offen lds")
        return m0, ld

    def build(self):
        A = self.after
        # K-half 0 (a0, b0): K-half-1 reads of cur, B DMA pieces after barrier #1
        for g in range(16):
            for q in range(4):
                k = 4 * g + q
                if q == 0:
                    if g < 4:
                        A[k].append(self.read("cur", 1, 2 * g))
                    if g == 4:
                        A[k].append(self.read("cur", 1, 8))
                    if 6 <= g < 13:
                        A[k].append(self.read("cur", 1, g + 3))
                if q == 2 and g < 4:
                    A[k].append(self.read("cur", 1, 2 * g + 1))
                if q == 1 and 6 <= g < 14:
                    m0, ld = self.dma(2 * (g - 6) + 1)
                    A[k - 1].append(m0)
                    A[k].append(ld)
                if q == 3 and g == 5:
                    A[k].append(("wait0", None, "s_waitcnt lgkmcnt(0)"))
                    A[k].append(("bar", None, "s_barrier"))
        # K-half 1 (a1, b1): A DMA pieces after barrier #2, next K-tile's K-half-0 reads after #3
        for g in range(16):
            for q in range(4):
                k = 64 + 4 * g + q
                if q == 1 and 2 <= g < 10:
                    m0, ld = self.dma(2 * (g - 2))
                    A[k - 1].append(m0)
                    A[k].append(ld)
                if g >= 10:
                    x0, x1 = (g - 10) * 16 // 6, (g - 9) * 16 // 6
                    if q == 0:
                        A[k].append(self.read("nxt", 0, x0))
                    if q == 2 and x0 + 1 < x1:
                        A[k].append(self.read("nxt", 0, x0 + 1))
                    if q == 3 and x0 + 2 < x1:
                        A[k].append(self.read("nxt", 0, x0 + 2))
                if q == 3 and g == 1:
                    A[k].append(("wait0", None, "s_waitcnt lgkmcnt(0)"))
                    A[k].append(("bar", None, "s_barrier"))
                if q == 3 and g == 9:
                    A[k].append(("waitv", None, "s_waitcnt vmcnt(16)"))
                    A[k].append(("bar", None, "s_barrier"))
        # clamp-advance the DMA source one K-tile (before the first piece, one SALU per gap)
        step = ["s_add_u32 s75, s73, 2", "s_cmp_lt_u32 s75, s72", "s_cselect_b32 s76, 0x80, 0",
                "s_add_u32 s64, s64, s76", "s_addc_u32 s65, s65, 0",
                "s_add_u32 s68, s68, s76", "s_addc_u32 s69, s69, 0"]
        for i, ins in enumerate(step):
            A[1 + 2 * i].append(("salu", None, ins))

    def emit(self, lgkm_queue: list) -> list:
        """Instructions of the body; lgkm_queue = outstanding LDS reads (oldest first), updated."""
        out = []
        for k in range(128):
            khalf = k >= 64
            I, J = (k % 64) >> 3, k & 7
            fa, fb = (f"a1{I}", f"b1{J}") if khalf else (f"a0{I}", f"b0{J}")
            need = [n for n, tag in enumerate(lgkm_queue) if tag in (fa, fb)]
            if need:
                keep = len(lgkm_queue) - need[-1] - 1
                out.append(f"s_waitcnt lgkmcnt({min(keep, 15)})")
                del lgkm_queue[: len(lgkm_queue) - min(keep, 15)]
            n = 8 * I + J
            src_a = frag("a1" if khalf else "a0", I)
            src_b = frag("b1" if khalf else "b0", J)
            out.append(f"v_mfma_f32_16x16x32_bf16 a[{4 * n}:{4 * n + 3}], {src_b}, {src_a}, "
                       f"a[{4 * n}:{4 * n + 3}]")
            for kind, tag, ins in self.after[k]:
                if kind == "lds":
                    lgkm_queue.append(tag)
                elif kind == "wait0":
                    lgkm_queue.clear()
                out.append(ins)
        return out


def prologue() -> list:
    out = []
    # operands → fixed registers (%0.. order must match the kernel's operand list)
    out += ["s_mov_b32 s72, %0", "s_mov_b32 s64, %1", "s_and_b32 s65, %2, 0xffff",
            "s_mov_b32 s66, %3", "s_mov_b32 s67, 0x20000", "s_mov_b32 s68, %4",
            "s_and_b32 s69, %5, 0xffff", "s_mov_b32 s70, %6", "s_mov_b32 s71, 0x20000",
            "s_mov_b32 s74, %9"]
    for e in range(8):
        rows = (e >> 1) * 32 + (e & 1) * 128
        out.append(f"s_mul_i32 s{80 + e}, %7, {rows}")
        out.append(f"s_mul_i32 s{88 + e}, %8, {rows}")
    for i in range(4):                  # v128 rA0, v129 rA1, v130 rB0, v131 rB1; +64 KiB: buffer 1
        out.append(f"v_mov_b32 v{128 + i}, %{10 + i}")
        out.append(f"v_add_u32 v{132 + i}, {TILE}, %{10 + i}")
    out += ["v_mov_b32 v136, %14", "v_mov_b32 v137, %15", "v_mov_b32 v138, %16"]
    out += [f"v_accvgpr_write_b32 a{r}, 0" for r in range(256)]
    # K-tiles 0 and min(1, T-1) in flight (buffers 0 and 1)
    for buf in range(2):
        if buf == 1:
            out += ["s_cmp_gt_u32 s72, 1", "s_cselect_b32 s76, 0x80, 0",
                    "s_add_u32 s64, s64, s76", "s_addc_u32 s65, s65, 0",
                    "s_add_u32 s68, s68, s76", "s_addc_u32 s69, s69, 0"]
        for p in range(16):
            opnd, row, off = piece(p)
            rs, voff = ("s[64:67]", "v136") if opnd == "A" else ("s[68:71]", "v137")
            out += [f"s_add_u32 m0, s74, {buf * TILE + off}", "s_nop 0",
                    f"buffer_load_dwordx4 {voff}, {rs}, {row} offen lds"]
    out += ["s_waitcnt vmcnt(16)", "s_barrier"]
    b = Body(1)   # reads "nxt" of parity 1 = buffer 0
    for x in range(16):
        out.append(b.read("nxt", 0, x)[2])
    out.append("s_mov_b32 s73, 0")
    return out


def epilogue() -> list:
    out = ["s_waitcnt vmcnt(0) lgkmcnt(0)", "s_nop 15", "s_nop 15", "s_barrier"]
    for i in range(8):
        bank = 32 + 16 * (i & 1)
        if i >= 2:
            out.append("s_waitcnt lgkmcnt(8)")     # the ds_writes of i-2 read this bank
        for j in range(8):
            n = 8 * i + j
            for c in range(4):
                out.append(f"v_accvgpr_read_b32 v{4 * j + c}, a{4 * n + c}")
        for j in range(8):
            out.append(f"v_cvt_pk_bf16_f32 v{bank + 2 * j}, v{4 * j}, v{4 * j + 1}")
            out.append(f"v_cvt_pk_bf16_f32 v{bank + 2 * j + 1}, v{4 * j + 2}, v{4 * j + 3}")
        for j in range(8):
            out.append(f"ds_write_b64 v138, v[{bank + 2 * j}:{bank + 2 * j + 1}] "
                       f"offset:{i * 16 * C_STRIDE + j * 32}")
    out.append("s_waitcnt lgkmcnt(0)")
    return out


def main():
    lines = prologue()
    queue = [f"{read_order(x)[0]}0{read_order(x)[1]}" for x in range(16)]
    bodies = []
    for P in (0, 1):
        b = Body(P)
        b.build()
        q = list(queue)
        bodies.append(b.emit(q))
        assert q == queue, "LDS read queue at the end of a K-tile must match its start"
    lines.append("amdk8s_w4a_loop_%=:")
    lines += bodies[0]
    lines += ["s_add_u32 s73, s73, 1", "s_cmp_ge_u32 s73, s72", "s_cbranch_scc1 amdk8s_w4a_end_%="]
    lines += bodies[1]
    lines += ["s_add_u32 s73, s73, 1", "s_cmp_lt_u32 s73, s72", "s_cbranch_scc1 amdk8s_w4a_loop_%="]
    lines.append("amdk8s_w4a_end_%=:")
    lines += epilogue()
    clob = ([f'"v{i}"' for i in range(139)] + [f'"a{i}"' for i in range(256)]
            + [f'"s{i}"' for i in range(64, 96)] + ['"scc"', '"memory"'])  # M0: reserved; no M0 user follows the asm
    with open(OUT, "w") as f:
        f.write("// GENERATED by tools/gen_gemm_w4a_kloop.py — do not edit by hand.\n")
        f.write(f"// {sum(1 for l in lines if 'v_mfma' in l)} MFMAs, {len(lines)} instructions.\n")
        f.write("#define AMDK8S_W4A_ASM \\\n")
        for ln in lines:
            f.write(f'  "{ln}\\n" \\\n')
        f.write("  \"\"\n\n#define AMDK8S_W4A_CLOBBERS \\\n")
        for i in range(0, len(clob), 12):
            f.write("  " + ", ".join(clob[i:i + 12]) + (", \\\n" if i + 12 < len(clob) else "\n"))
    print(f"wrote {OUT}: {len(lines)} lines")


if __name__ == "__main__":
    main()
