"""CPU check of the built library's gfx950 machine code: no > 64-bit vector-memory store has its
data VGPRs overwritten by a VALU instruction inside the store-data hazard's wait states
(tools/isa_hazards.py; DESIGN.md section 4 -- the round-2 layer3 tail corruption)."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'tools'))

import isa_hazards  # noqa: E402

LIB = os.path.join(REPO, 'pose-unsupervised_amd', 'lib', 'posu', 'libposeu.so')

BAD = """
0000000000001000 <kernel_a>:
	buffer_store_dwordx4 v[154:157], v144, s[16:19], s7 offen   // 000000001000: E07C1000
	v_mov_b32_e32 v154, v23                                      // 000000001008: 7F340317
"""
SWAP = """
0000000000001000 <kernel_b>:
	global_store_dwordx4 v[68:69], v[158:161], off
	v_mov_b32_e32 v3, v4
	v_permlane16_swap_b32_e32 v7, v160
"""
GOOD = """
0000000000001000 <kernel_c>:
	buffer_store_dwordx4 v[154:157], v144, s[16:19], 0 offen
	s_nop 1
	v_mov_b32_e32 v154, v23
	buffer_store_dwordx4 v[10:13], v144, s[16:19], 0 offen
	v_mov_b32_e32 v9, v23
	v_add_u32_e32 v14, v1, v2
	v_mov_b32_e32 v10, v23
"""

# the offending VALU sits at a branch target (a loop head reached through the back-edge, and the
# target of a forward conditional branch): the straight-line window after the store is clean
BRANCH_BACK = """
0000000000002000 <kernel_d>:
	v_mov_b32_e32 v20, v1                                        // 000000002000: 7E280301
	v_add_u32_e32 v5, v1, v2                                     // 000000002004: 680A0501
	buffer_store_dwordx4 v[20:23], v144, s[16:19], 0 offen       // 000000002008: E07C1000 80031490
	s_cbranch_scc1 65531                                         // 000000002010: BF85FFFB
	s_endpgm                                                     // 000000002014: BF810000
"""
BRANCH_FWD = """
0000000000003000 <kernel_e>:
	global_store_dwordx4 v[68:69], v[158:161], off               // 000000003000: DC7C8000 009E0044
	s_cbranch_execz 2                                            // 000000003008: BF880002
	v_mov_b32_e32 v3, v4                                         // 00000000300C: 7E060304
	s_nop 1                                                      // 000000003010: BF800001
	v_mov_b32_e32 v159, v4                                       // 000000003014: 7F3E0304
	s_endpgm                                                     // 000000003018: BF810000
"""
# the same shapes with the hazard waited out on every path
BRANCH_OK = """
0000000000004000 <kernel_f>:
	s_nop 1                                                      // 000000004000: BF800001
	v_mov_b32_e32 v20, v1                                        // 000000004004: 7E280301
	v_add_u32_e32 v5, v1, v2                                     // 000000004008: 680A0501
	buffer_store_dwordx4 v[20:23], v144, s[16:19], 0 offen       // 00000000400C: E07C1000 80031490
	s_cbranch_scc1 65530                                         // 000000004014: BF85FFFA
	s_endpgm                                                     // 000000004018: BF810000
"""


def test_scanner_flags_the_hazard_pattern():
    assert len(isa_hazards.scan(BAD)) == 1
    assert len(isa_hazards.scan(SWAP)) == 1      # the swap writes both of its operands
    assert isa_hazards.scan(GOOD) == []          # waited out / other registers / past the window


def test_scanner_follows_branches():
    assert len(isa_hazards.scan(BRANCH_BACK)) == 1   # VALU at the loop head, reached by the back-edge
    assert len(isa_hazards.scan(BRANCH_FWD)) == 1    # VALU at a forward branch target
    assert isa_hazards.scan(BRANCH_OK) == []


def test_built_library_has_no_store_data_hazard():
    if not os.path.exists(LIB):
        pytest.fail('libposeu.so is not built (run __graft_entry__.build())')
    text = isa_hazards.disassemble(LIB)
    found = isa_hazards.scan(text)
    assert sum(1 for line in text.splitlines() if isa_hazards._STORE.match(line.strip())) > 100
    assert found == [], found[:4]
