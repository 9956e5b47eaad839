"""Static check of libposeu.so's gfx950 machine code for the VMEM store-data hazard.

A vector-memory store of more than 64 bits of data per lane (buffer_/global_store_dwordx3/x4)
reads its data VGPRs after it issues; a VALU instruction that writes one of those VGPRs within
the next wait states corrupts the stored value.  hipcc's hazard recognizer inserts the wait
states for global stores and for buffer stores with an immediate soffset, but treats a buffer
store whose soffset is an SGPR as hazard-free -- on gfx950 it is not: the round-2 layer3 tail
kernel with `__builtin_amdgcn_raw_buffer_store_b128(..., soffset = row offset)` stored wrong
values into a few hundred 16-B chunks per launch (pixel columns 12-15 of the first rows of
a tile; profiles/r03/store_order.txt, measured by tools removed in round 4 with the kernel).  This scanner disassembles the
built library and reports every store whose data VGPRs a VALU instruction overwrites within
WAIT_STATES instructions (s_nop n counts n + 1).

    python tools/isa_hazards.py [path/to/libposeu.so]      (exit status 1 on a finding)
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

OBJDUMP = '/opt/rocm/lib/llvm/bin/llvm-objdump'
WAIT_STATES = 2
_STORE = re.compile(r'^(buffer|global|flat|scratch)_store_dwordx([34])\b')
_VREG = re.compile(r'v\[(\d+):(\d+)\]|v(\d+)\b')


def _regs(op):
    m = _VREG.match(op.strip())
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def _split(line):
    code = line.split('//')[0].strip()
    if not code or code.endswith(':') or code.startswith(';') or code.startswith('.'):
        return None, []
    parts = code.split(None, 1)
    ops = [o.strip() for o in parts[1].split(',')] if len(parts) > 1 else []
    return parts[0], ops


def _written(mn, ops):
    """VGPRs a VALU instruction writes (both operands of the permlane swaps)."""
    if not mn.startswith('v_') or not ops:
        return set()
    w = _regs(ops[0])
    if mn.startswith('v_permlane16_swap') or mn.startswith('v_permlane32_swap'):
        w |= _regs(ops[1])
    return w


_ADDR = re.compile(r'//\s*([0-9A-Fa-f]+):')
_END = ('s_endpgm', 's_setpc_b64', 's_trap', 's_rfe_b64')


def _branch_target(addr, ops):
    """Target address of an s_branch / s_cbranch_* at addr: PC + 4 + 4 * simm16."""
    imm = int(ops[0], 0) & 0xFFFF
    if imm & 0x8000:
        imm -= 0x10000
    return addr[0], addr[1] + 4 + 4 * imm


def scan(text):
    """-> list of (function, store instruction, offending instruction).

    From every > 64-bit store, every control-flow path is followed for WAIT_STATES wait states:
    s_nop n counts n + 1, any other instruction 1 (a branch too: it issues, as LLVM's hazard
    recognizer counts it); s_branch continues at its target, s_cbranch_* at its target AND its
    fall-through, so a VALU at a branch target or at a loop head reached through a back-edge is
    checked too, not only the straight-line successors."""
    out, fn, obj = [], '?', 0
    insts, at = [], {}
    for line in text.splitlines():
        s = line.strip()
        if 'file format' in s:   # a new code object: addresses restart
            obj += 1
            continue
        if s.endswith('>:'):
            fn = s
            insts.append((fn, None, [], s, None))
            continue
        mn, ops = _split(line)
        if mn is not None:
            m = _ADDR.search(line)
            addr = int(m.group(1), 16) if m else None
            if addr is not None:
                addr = (obj, addr)
                at[addr] = len(insts)
            insts.append((fn, mn, ops, s, addr))
    for i, (f, mn, ops, s, _) in enumerate(insts):
        if mn is None:
            continue
        m = _STORE.match(mn)
        if not m:
            continue
        # operands: global_store v[addr], v[data], ... ; buffer_store v[data], voffset, ...
        data = _regs(ops[1] if m.group(1) in ('global', 'flat', 'scratch') else ops[0])
        hit, seen, todo = None, set(), [(i + 1, 0)]
        while todo and hit is None:
            j, waits = todo.pop()
            while j < len(insts) and waits < WAIT_STATES and (j, waits) not in seen:
                seen.add((j, waits))
                f2, mn2, ops2, s2, a2 = insts[j]
                if mn2 is None or mn2 in _END:
                    break
                if mn2 == 's_nop':
                    waits += int(ops2[0], 0) + 1 if ops2 else 1
                    j += 1
                    continue
                if mn2 == 's_branch' or mn2.startswith('s_cbranch'):
                    tgt = at.get(_branch_target(a2, ops2)) if a2 is not None and ops2 else None
                    if tgt is None:            # unresolved target: a hazard unless waited out
                        hit = s2 + '  (unresolved branch target inside the window)'
                        break
                    waits += 1
                    if mn2 == 's_branch':
                        j = tgt
                        continue
                    todo.append((tgt, waits))
                    j += 1
                    continue
                if _written(mn2, ops2) & data:
                    hit = s2
                    break
                waits += 1
                j += 1
        if hit is not None:
            out.append((f, s, hit))
    return out


def disassemble(lib):
    tmp = tempfile.mkdtemp(prefix='posu_isa_')
    try:
        dst = os.path.join(tmp, 'lib.so')
        shutil.copy(lib, dst)
        subprocess.run([OBJDUMP, '--offloading', dst], cwd=tmp, check=True, capture_output=True)
        text = []
        for name in sorted(os.listdir(tmp)):
            if name.endswith('gfx950'):
                r = subprocess.run([OBJDUMP, '-d', '--mcpu=gfx950', os.path.join(tmp, name)], check=True,
                                   capture_output=True, text=True)
                text.append(r.stdout)
        return '\n'.join(text)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'pose-unsupervised_amd', 'lib', 'posu',
        'libposeu.so')
    text = disassemble(lib)
    found = scan(text)
    nst = sum(1 for l in text.splitlines() if _STORE.match(l.strip()))
    for f, s, s2 in found:
        print('%s\n    %s\n    %s' % (f, s.split('//')[0].strip(), s2.split('//')[0].strip()))
    print('%s: %d stores of > 64 bits, %d with a VALU overwrite of their data inside %d wait states'
          % (os.path.basename(lib), nst, len(found), WAIT_STATES))
    return 1 if found else 0


if __name__ == '__main__':
    sys.exit(main())
