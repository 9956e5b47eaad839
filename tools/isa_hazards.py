"""Static check of libposeu.so's gfx950 machine code for the VMEM store-data hazard.

A vector-memory store of more than 64 bits of data per lane (buffer_/global_store_dwordx3/x4)
reads its data VGPRs after it issues; a VALU instruction that writes one of those VGPRs within
the next wait states corrupts the stored value.  hipcc's hazard recognizer inserts the wait
states for global stores and for buffer stores with an immediate soffset, but treats a buffer
store whose soffset is an SGPR as hazard-free -- on gfx950 it is not: the round-2 layer3 tail
kernel with `__builtin_amdgcn_raw_buffer_store_b128(..., soffset = row offset)` stored wrong
values into a few hundred 16-B chunks per launch (pixel columns 12-15 of the first rows of
a tile; tools/store_check.py, profiles/r03/store_order.txt).  This scanner disassembles the
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


def scan(text):
    """-> list of (function, store instruction, offending instruction)."""
    out, fn = [], '?'
    insts = []
    for line in text.splitlines():
        s = line.strip()
        if s.endswith('>:'):
            fn = s
            insts.append((fn, None, [], s))
            continue
        mn, ops = _split(line)
        if mn is not None:
            insts.append((fn, mn, ops, s))
    for i, (f, mn, ops, s) in enumerate(insts):
        if mn is None:
            continue
        m = _STORE.match(mn)
        if not m:
            continue
        # operands: global_store v[addr], v[data], ... ; buffer_store v[data], voffset, ...
        data = _regs(ops[1] if m.group(1) in ('global', 'flat', 'scratch') else ops[0])
        waits = 0
        for f2, mn2, ops2, s2 in insts[i + 1:]:
            if mn2 is None or waits >= WAIT_STATES:
                break
            if mn2 == 's_nop':
                waits += int(ops2[0], 0) + 1 if ops2 else 1
                continue
            if _written(mn2, ops2) & data:
                out.append((f, s, s2))
                break
            waits += 1
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
