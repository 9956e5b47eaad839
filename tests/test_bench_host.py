"""CPU-side pieces of bench.py's default line: the CPU baseline leg (the oracle chain on the host
cores) returns plain JSON values -- a leaked numpy meta dict once made the whole default line fail
at json.dumps on the GPU box -- and the line's serializer handles numpy scalars."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def test_cpu_baseline_entry_is_plain_json():
    cpu, ref = bench.cpu_baseline(18, 128, 1, 0.0)
    s = json.dumps(cpu)       # no default= hook: every value must already be a JSON type
    d = json.loads(s)
    assert d['kind'] == 'port' and d['cores'] >= 1 and isinstance(d['host_cpus'], int)
    assert d['value'] > 0 and d['batch1_forward_ms'] > 0
    assert 'X' in ref and 'host' in ref


def test_line_serializer_converts_numpy_values():
    line = {'a': np.float32(1.5), 'b': np.int64(3), 'c': np.arange(3)}
    d = json.loads(json.dumps(line, default=bench._json_default))
    assert d == {'a': 1.5, 'b': 3, 'c': [0, 1, 2]}
