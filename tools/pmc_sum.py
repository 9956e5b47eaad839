"""Sum rocprofv3 counter_collection.csv values per (kernel, grid, dispatch order) group.

    python tools/pmc_sum.py run_counter_collection.csv [kernel-substring]
"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    pat = sys.argv[2] if len(sys.argv) > 2 else 'posu'
    per = collections.OrderedDict()
    for r in rows:
        if pat not in r['Kernel_Name']:
            continue
        d = int(r['Dispatch_Id'])
        per.setdefault(d, {'name': r['Kernel_Name'], 'grid': r['Grid_Size'], 'lds': r['LDS_Block_Size'],
                           'vgpr': r.get('VGPR_Count'), 'agpr': r.get('Accum_VGPR_Count')})
        per[d][r['Counter_Name']] = per[d].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    for d, v in per.items():
        name = v.pop('name')
        tag = name[name.find('kernel'):][:70]
        print(d, tag, ' '.join('%s=%s' % (k, ('%.4g' % x) if isinstance(x, float) else x) for k, x in v.items()))


if __name__ == '__main__':
    main()
