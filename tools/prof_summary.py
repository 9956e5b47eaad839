"""Per-kernel time summary of a rocprofv3 rocpd database (kernel-trace run).

    python tools/prof_summary.py gpurun_out/prof/run_results.db [--top 40] [--csv out.csv]
"""
import argparse
import collections
import glob
import re
import sqlite3


def load(db):
    con = sqlite3.connect(db)
    names = [r[0] for r in con.execute("select name from sqlite_master where type='table'")]
    suf = re.search(r'rocpd_metadata(_.*)', [n for n in names if n.startswith('rocpd_metadata')][0]).group(1)
    rows = con.execute(f"select s.display_name, d.start, d.end, d.grid_size_x, d.workgroup_size_x "
                       f"from rocpd_kernel_dispatch{suf} d join rocpd_info_kernel_symbol{suf} s "
                       f"on d.kernel_id = s.id order by d.start").fetchall()
    return rows


def short(name):
    name = name.replace('(anonymous namespace)::', '').replace('posu::', '')
    name = re.sub(r'\(.*', '', name)
    return name[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--top', type=int, default=40)
    ap.add_argument('--csv')
    a = ap.parse_args()
    rows = load(glob.glob(a.db)[0])
    agg = collections.defaultdict(lambda: [0, 0.0])
    for name, s, e, _, _ in rows:
        k = short(name)
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e3
    total = sum(v[1] for v in agg.values())
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    lines = ['"Name","Calls","TotalDurationUs","AverageUs","Percentage"']
    for k, (n, t) in out:
        lines.append('"%s",%d,%.1f,%.2f,%.2f' % (k, n, t, t / n, 100 * t / total))
    print('total kernel time %.1f us over %d dispatches' % (total, len(rows)))
    for ln in lines[:a.top + 1]:
        print(ln)
    if a.csv:
        open(a.csv, 'w').write('\n'.join(lines) + '\n')


if __name__ == '__main__':
    main()
