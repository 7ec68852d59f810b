"""tools/isa_check.py (the build-time ISA hazard check, DESIGN.md §3 "MFMA
hazards") on synthetic gfx950 instruction sequences: each rule fires on the
pattern it names and stays quiet on the shape the hazard-safe tile emits."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
import isa_check as ic  # noqa: E402

MF = "v_mfma_i32_16x16x64_i8"


def kinds(lines):
    body = [(None, t) for t in lines]
    return sorted({k for k, _, _ in ic.check_kernel(body, 0)})


def test_safe_tile_shape_is_clean():
    # the asm tile: operands 2 states old, early-clobber D, 8 states of pad
    lines = ["v_xor_b32_e32 v90, 0x80808080, v0", "s_nop 1",
             f"{MF} v[0:3], v[10:13], v[90:93], v[20:23]", f"{MF} v[4:7], v[14:17], v[90:93], 0",
             f"{MF} v[30:33], v[18:21], v[90:93], 0", f"{MF} v[34:37], v[22:25], v[90:93], 0", "s_nop 7",
             "v_lshl_add_u32 v40, v34, 8, v30", "v_mov_b32_e32 v90, 0"]
    assert kinds(lines) == []


def test_d_overlapping_b_is_flagged():
    lines = ["s_nop 1", f"{MF} v[88:91], v[10:13], v[88:91], 0", "s_nop 7"]
    assert "M3" in kinds(lines)


def test_early_read_of_d_is_flagged():
    lines = ["s_nop 1", f"{MF} v[0:3], v[10:13], v[90:93], 0", "s_nop 2", "v_add_u32_e32 v5, v0, v1"]
    assert "M1" in kinds(lines)


def test_write_of_in_flight_operand_is_flagged():
    lines = ["s_nop 1", f"{MF} v[0:3], v[10:13], v[90:93], 0", "s_nop 5", "v_mov_b64_e32 v[90:91], s[10:11]"]
    assert "M2" in kinds(lines)


def test_fresh_operand_is_flagged():
    lines = ["v_xor_b32_e32 v90, 0x80808080, v0", f"{MF} v[0:3], v[10:13], v[90:93], 0", "s_nop 7"]
    assert "M4" in kinds(lines)


def test_unwaited_load_register_is_flagged_and_waited_one_is_not():
    bad = ["ds_read_b32 v5, v1 offset:64", "v_mov_b32_e32 v6, v5", "s_waitcnt lgkmcnt(0)"]
    good = ["ds_read_b32 v5, v1 offset:64", "s_waitcnt lgkmcnt(0)", "v_mov_b32_e32 v6, v5"]
    assert kinds(bad) == ["L1"]
    assert kinds(good) == []
    # in-order VMEM returns: vmcnt(1) retires the older of two loads
    two = ["buffer_load_dword v5, v1, s[4:7], 0 offen", "buffer_load_dword v6, v1, s[4:7], 0 offen",
           "s_waitcnt vmcnt(1)", "v_mov_b32_e32 v7, v5", "v_mov_b32_e32 v8, v6"]
    assert kinds(two) == ["L1"]


def test_lds_dma_has_no_register_destination():
    lines = ["global_load_lds_dword v20, s[44:45]", "v_mov_b32_e32 v20, 0"]
    assert kinds(lines) == []


def test_overwrite_of_wide_store_data_is_flagged():
    # the r05 pattern: a 128-bit buffer store with an SGPR soffset, its data
    # register rewritten by the next instruction (hipcc pads nothing here)
    st = "buffer_store_dwordx4 v[0:3], v94, s[20:23], s78 offen"
    assert kinds([st, "v_mov_b32_e32 v0, v126"]) == ["S1"]
    assert kinds([st, "v_writelane_b32 v1, s78, 39"]) == ["S1"]
    assert kinds([st, "s_nop 0", "v_mov_b32_e32 v3, v126"]) == ["S1"]
    # two wait states on, or a register outside the data, or 64-bit data: clean
    assert kinds([st, "s_nop 1", "v_mov_b32_e32 v0, v126"]) == []
    assert kinds([st, "v_mov_b32_e32 v4, v126"]) == []
    assert kinds(["buffer_store_dwordx2 v[0:1], v94, s[20:23], s78 offen", "v_mov_b32_e32 v0, v126"]) == []
    assert kinds(["global_store_dwordx4 v[8:9], v[0:3], off", "v_mov_b32_e32 v2, 0"]) == ["S1"]


def kinds_at(lines):
    """Lines with addresses (4 bytes apart from 0x100) so branch targets
    `<k+0xADDR>` resolve; function base 0."""
    body = [(0x100 + 4 * i, t) for i, t in enumerate(lines)]
    return sorted({k for k, _, _ in ic.check_kernel(body, 0)})


def test_loop_carried_wide_store_hazard_is_caught():
    # the store is the last instruction of the loop body; the loop head's
    # first instruction rewrites its data: a hazard only along the back edge
    loop = ["v_mov_b32_e32 v0, v126",                                  # 0x100: loop head
            "v_add_u32_e32 v5, v5, v6",
            "buffer_store_dwordx4 v[0:3], v94, s[20:23], s78 offen",   # 0x108
            "s_cbranch_scc1 65533 <k+0x100>",                          # back to the head
            "s_endpgm"]
    assert kinds_at(loop) == ["S1"]
    # two wait states at the loop head: clean
    safe = ["s_nop 1", "v_mov_b32_e32 v0, v126", "buffer_store_dwordx4 v[0:3], v94, s[20:23], s78 offen",
            "s_cbranch_scc1 65533 <k+0x100>", "s_endpgm"]
    assert kinds_at(safe) == []


def test_loop_carried_mfma_and_load_hazards_are_caught():
    # an MFMA issued at the loop's end, its D read at the head
    mf = ["v_add_u32_e32 v40, v0, v1", "s_nop 7", "s_nop 1",
          f"{MF} v[0:3], v[10:13], v[90:93], 0",
          "s_cbranch_scc1 65532 <k+0x100>", "s_endpgm"]
    assert "M1" in kinds_at(mf)
    # a load issued at the loop's end and waited for only after the head read it
    ld = ["v_mov_b32_e32 v6, v5", "s_waitcnt vmcnt(0)", "buffer_load_dword v5, v1, s[4:7], 0 offen",
          "s_cbranch_scc1 65533 <k+0x100>", "s_endpgm"]
    assert kinds_at(ld) == ["L1"]
    ld_ok = ["s_waitcnt vmcnt(0)", "v_mov_b32_e32 v6, v5", "buffer_load_dword v5, v1, s[4:7], 0 offen",
             "s_cbranch_scc1 65533 <k+0x100>", "s_endpgm"]
    assert kinds_at(ld_ok) == []


def test_loop_states_converge_with_a_load_issued_every_iteration():
    # a load re-issued each iteration and waited at the head: a fixpoint,
    # no X1 and no finding
    lines = ["s_waitcnt vmcnt(0)", "v_add_u32_e32 v6, v5, v6", "buffer_load_dword v5, v1, s[4:7], 0 offen",
             "buffer_store_dword v6, v1, s[4:7], 0 offen", "s_cbranch_scc1 65532 <k+0x100>", "s_endpgm"]
    assert kinds_at(lines) == []
