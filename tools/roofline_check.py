"""Cross-check bench.py's roofline against a rocprofv3 kernel trace of the same command.

    python tools/roofline_check.py <dir>/infer/run_kernel_trace.csv <bench log> [launches_per_forward]

Groups the trace into network forwards (input pack or fused stem .. fused deconv+head; the
launch count per forward is found from the gaps between forward starts unless given), sums kernel durations per forward for the last timed forwards, and prints them next
to bench.py's HIP-event network time and the implied TFLOP/s.
"""
import csv
import json
import sys

NET = ('conv_igemm_kernel', 'conv_persist_kernel', 'bottleneck', 'tail_stream_kernel', 'stem_pool_kernel', 'maxpool_kernel',
       'pack_s2d_kernel', 'pack_kernel')


def forwards(trace, per_fwd):
    tr = sorted(csv.DictReader(open(trace)), key=lambda r: int(r['Start_Timestamp']))
    net = [r for r in tr if any(k in r['Kernel_Name'] for k in NET)]
    first = ('pack', 'stem_pool')  # a forward opens with its input pack / fused stem launches

    def is_first(r):
        return any(k in r['Kernel_Name'] for k in first)

    starts = [i for i, r in enumerate(net) if is_first(r) and (i == 0 or not is_first(net[i - 1]))]
    if per_fwd <= 0:  # launches per forward = the common gap between forward starts
        gaps = sorted(b - a for a, b in zip(starts, starts[1:]))
        per_fwd = gaps[len(gaps) // 2]
    out = []
    for a in starts:
        seq = net[a:a + per_fwd]
        if len(seq) == per_fwd:
            out.append((sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in seq) / 1e6,
                        (int(seq[-1]['End_Timestamp']) - int(seq[0]['Start_Timestamp'])) / 1e6))
    return out


def main():
    per_fwd = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    fw = forwards(sys.argv[1], per_fwd)[-10:]
    line = next(json.loads(l) for l in open(sys.argv[2]) if l.startswith('{"metric"'))
    gf = 14.47 * line['config']['frames_per_gpu_step']
    busy = sum(f[0] for f in fw) / len(fw)
    print('bench: network_ms %.4f  achieved %.1f TFLOP/s  (value %.1f frames/s)'
          % (line['network_ms'], line['roofline']['achieved'], line['value']))
    print('trace: %d forwards, kernel-busy %.4f ms/forward (span %.4f ms) -> %.1f TFLOP/s'
          % (len(fw), busy, sum(f[1] for f in fw) / len(fw), gf / busy))
    print('agreement: trace / events = %.3f' % (busy / line['network_ms']))


if __name__ == '__main__':
    main()
