"""Summarise kernels in a hipcc -save-temps .s file: VGPR/AGPR/SGPR/LDS/scratch from the
metadata and, per kernel body, counts of MFMA, barriers, waitcnt forms and scratch accesses.

    python tools/isa_stats.py file.s [name-substring ...]
"""
import re
import sys


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    s = open(path).read()
    for m in re.finditer(r'^(_Z\S+):\s', s, re.M):
        name = m.group(1)
        if pats and not all(p in name for p in pats):
            continue
        i = m.end()
        j = s.find('.Lfunc_end', i)
        body = s[i:j]
        meta = {}
        md = s[s.find('amdhsa.kernels'):]
        for blk in re.split(r'\n  - ', md):  # one YAML entry per kernel
            if re.search(r'\.name:\s+' + re.escape(name) + r'\s', blk):
                for key in ('vgpr_count', 'agpr_count', 'sgpr_count', 'group_segment_fixed_size',
                            'private_segment_fixed_size', 'vgpr_spill_count'):
                    mm = re.search(r'\.' + key + r':\s+(\d+)', blk)
                    meta[key] = mm.group(1) if mm else '?'
                break
        waits = re.findall(r's_waitcnt\s+(.*)', body)
        vm = {}
        for w in waits:
            for x in re.findall(r'vmcnt\((\d+)\)', w):
                vm[x] = vm.get(x, 0) + 1
        print(name[:110])
        print('   meta', meta)
        print('   mfma %d  s_barrier %d  buffer_load..lds %d  ds_read %d  scratch %d  vmcnt %s' % (
            len(re.findall(r'v_mfma', body)), len(re.findall(r's_barrier', body)),
            len(re.findall(r'buffer_load_dwordx4.*lds', body)), len(re.findall(r'ds_read', body)),
            len(re.findall(r'scratch_', body)), dict(sorted(vm.items()))))


if __name__ == '__main__':
    main()
