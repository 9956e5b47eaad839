"""CPU tests of the profile reducers behind profiles/<round>/ (tools/replay_breakdown.py,
tools/pmc_traffic.py) on synthetic rocprofv3 CSVs: a forward run depth-first over two chunks
starts two stem runs, and the reducers must still take whole forwards (--per / --stems)."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(REPO, 'tools')

# one chunked forward: chunk 0's early stage, chunk 1's early stage, then the whole-batch rest
EARLY = ['stem_pool_kernel<f16_t>', 'tail_stream_kernel<a>', 'tail_stream_kernel<b>']
REST = ['conv_igemm_kernel<l3>', 'conv_igemm_kernel<l4>', 'conv_igemm_kernel<head>']


def _forward_names():
    return EARLY + EARLY + REST


def _write_trace(path, forwards):
    t = 1_000_000
    with open(path, 'w', newline='') as f:
        w = csv.DictWriter(f, fieldnames=['Kernel_Name', 'Start_Timestamp', 'End_Timestamp'])
        w.writeheader()
        for k in range(forwards):
            for i, n in enumerate(_forward_names()):
                d = 10_000 + 1_000 * i          # launch i of a forward lasts 10 + i us
                w.writerow({'Kernel_Name': n, 'Start_Timestamp': t, 'End_Timestamp': t + d})
                t += d
            w.writerow({'Kernel_Name': 'softargmax_kernel', 'Start_Timestamp': t, 'End_Timestamp': t + 5_000})
            t += 100_000                        # the next replay after a gap


def _write_pmc(path, counter, forwards, value_of):
    with open(path, 'w', newline='') as f:
        w = csv.DictWriter(f, fieldnames=['Dispatch_Id', 'Kernel_Name', 'Counter_Name', 'Counter_Value'])
        w.writeheader()
        d = 0
        for k in range(forwards):
            for i, n in enumerate(_forward_names()):
                d += 1
                w.writerow({'Dispatch_Id': d, 'Kernel_Name': n, 'Counter_Name': counter,
                            'Counter_Value': value_of(k, i)})


def test_replay_breakdown_merges_chunked_forwards(tmp_path):
    trace = tmp_path / 'trace.csv'
    _write_trace(trace, forwards=4)
    out = subprocess.run([sys.executable, os.path.join(TOOLS, 'replay_breakdown.py'), str(trace), '--last', '3',
                          '--per', '2'], capture_output=True, text=True, check=True).stdout
    n = len(_forward_names())
    assert out.splitlines()[0] == '3 replays of %d launches' % n
    total = sum(10 + i for i in range(n))
    assert 'sum of launches %.1f us' % total in out
    # without --per, each stem run starts a replay: the chunked forward is cut in two
    one = subprocess.run([sys.executable, os.path.join(TOOLS, 'replay_breakdown.py'), str(trace), '--last', '3'],
                         capture_output=True, text=True, check=True).stdout
    assert ' of %d launches' % n not in one.splitlines()[0]


def test_pmc_traffic_takes_the_last_whole_chunked_forward(tmp_path):
    fetch, write = tmp_path / 'fetch.csv', tmp_path / 'write.csv'
    # KiB per launch; the last forward's values are distinct (forward index k in the thousands)
    _write_pmc(fetch, 'FETCH_SIZE', 3, lambda k, i: 1000 * k + i + 1)
    _write_pmc(write, 'WRITE_SIZE', 3, lambda k, i: 1000 * k + 2 * i + 1)
    out = subprocess.run([sys.executable, os.path.join(TOOLS, 'pmc_traffic.py'), str(fetch), str(write),
                          '--stems', '2'], capture_output=True, text=True, check=True).stdout
    line = json.loads(out.splitlines()[0])
    n = len(_forward_names())
    assert line['launches'] == n
    k = 2
    # FETCH_SIZE doubled (gfx950 correction; the stem's scale is 2 by default too), KiB -> bytes
    assert line['fetch_bytes_corrected'] == sum(2 * (1000 * k + i + 1) * 1024 for i in range(n))
    assert line['write_bytes'] == sum((1000 * k + 2 * i + 1) * 1024 for i in range(n))
    # one stem run back only: the tail of the forward from its second chunk's stem
    out1 = subprocess.run([sys.executable, os.path.join(TOOLS, 'pmc_traffic.py'), str(fetch), str(write)],
                          capture_output=True, text=True, check=True).stdout
    assert json.loads(out1.splitlines()[0])['launches'] == len(EARLY) + len(REST)
