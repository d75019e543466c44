"""CPU tests for the generated-assembly GEMM K-loops (tools/gen_gemm_w4a_kloop.py, gen_gemm_f8a_kloop.py).

The committed .inc files must be exactly what the generators produce (they are build inputs), every
built-in schedule must pass the buffer-discipline checks, a schedule that breaks the discipline
must be rejected, and the lgkmcnt simulation must wait for exactly the reads an MFMA consumes.
"""
import importlib
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

w4a = importlib.import_module("gen_gemm_w4a_kloop")
f8a = importlib.import_module("gen_gemm_f8a_kloop")


@pytest.mark.parametrize("gen", [w4a, f8a], ids=["w4a", "f8a"])
def test_committed_inc_matches_generator(gen, tmp_path, monkeypatch):
    committed = open(gen.OUT).read()
    out = tmp_path / "kloop.inc"
    monkeypatch.setattr(gen, "OUT", str(out))
    gen.main()
    assert out.read_text() == committed, f"rerun {gen.__name__}.py and commit its .inc"


@pytest.mark.parametrize("name", list(w4a.SCHEDULES) + list(w4a.EXPERIMENTS))
def test_w4a_schedules_pass_discipline_checks(name):
    sched = {**w4a.SCHEDULES, **w4a.EXPERIMENTS}[name]()
    w4a.check(name, sched)
    lines = w4a.kernel_asm(name)
    assert sum("v_mfma_f32_16x16x32_bf16" in ln for ln in lines) == 256  # 2 parities x 128
    per_tile = 2 if any(op == ("bar", 12) for _, op in sched) else 3       # twobar merges #1/#2
    assert sum(ln == "s_barrier" for ln in lines) == 2 * per_tile + 2    # + prologue, epilogue


def test_w4a_rejects_dma_before_its_barrier():
    sched = w4a.sched_region()
    # move B piece 1 (after barrier #1 at slot 23) in front of the barrier
    bad = [(10, op) if op == ("dma", 1) else (slot, op) for slot, op in sched]
    with pytest.raises(AssertionError):
        w4a.check("bad", bad)


def test_w4a_rejects_next_tile_read_before_barrier3():
    sched = w4a.sched_region()
    first_r0 = next((slot, op) for slot, op in sched if op[0] == "r0")
    bad = [(70, op) if (slot, op) == first_r0 else (slot, op) for slot, op in sched]
    with pytest.raises(AssertionError):
        w4a.check("bad", bad)


def test_w4a_lgkm_waits_are_exact():
    """Before MFMA 0 of a K-tile the queue holds the 16 next-tile reads in first-use order; MFMA 0
    needs b0[0] and a0[0] (the 5th read), so exactly 11 later reads may stay outstanding."""
    queue = [f"{o}0{i}" for o, i in w4a.FIRST_USE]
    lines = w4a.body("region", w4a.sched_region(), 0, queue)
    assert lines[0] == "s_waitcnt lgkmcnt(11)"
    assert lines[1].startswith("v_mfma_f32_16x16x32_bf16 a[0:3]")


def test_f8a_read_slots_respect_in_place_reuse():
    for per_slot in f8a.SCHEDULES.values():
        for slot, opnd, idx, _ in f8a.read_slots(per_slot):
            assert slot > f8a.BAR2
            if opnd == "a" and idx not in f8a.A_DOUBLE:
                assert slot >= 8 * idx + 8, (per_slot, slot, idx)  # after A[idx]'s last MFMA


def test_f8a_mfmas_use_parity_fragment_sets():
    q0 = [f8a.atag(i, h, 0) if o == "a" else f"b0{i}{h}" for o, i in f8a.READS for h in (0, 1)]
    even = f8a.body(0, list(q0), 2)
    odd_q = [f8a.atag(i, h, 1) if o == "a" else f"b1{i}{h}" for o, i in f8a.READS for h in (0, 1)]
    odd = f8a.body(1, list(odd_q), 2)
    mf_even = [ln for ln in even if ln.startswith("v_mfma")]
    mf_odd = [ln for ln in odd if ln.startswith("v_mfma")]
    assert len(mf_even) == len(mf_odd) == 64
    assert "v[64:71]" in mf_even[0] and "v[128:135]" in mf_odd[0]      # B set by parity
    assert "v[48:55]" in mf_even[48] and "v[204:211]" in mf_odd[48]    # A6 double-buffered
