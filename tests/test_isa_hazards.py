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


def test_scanner_flags_the_hazard_pattern():
    assert len(isa_hazards.scan(BAD)) == 1
    assert len(isa_hazards.scan(SWAP)) == 1      # the swap writes both of its operands
    assert isa_hazards.scan(GOOD) == []          # waited out / other registers / past the window


def test_built_library_has_no_store_data_hazard():
    if not os.path.exists(LIB):
        pytest.fail('libposeu.so is not built (run __graft_entry__.build())')
    text = isa_hazards.disassemble(LIB)
    found = isa_hazards.scan(text)
    assert sum(1 for line in text.splitlines() if isa_hazards._STORE.match(line.strip())) > 100
    assert found == [], found[:4]
