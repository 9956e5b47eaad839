"""Run a repo script (bench.py, a tools/ micro-benchmark) against another build of libposeu.so, for
A/B timings inside one GPU call:

    python tools/with_lib.py pose-unsupervised_amd/build/abl/libposeu_X.so bench.py --mode train ...
"""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

from posu import _native  # noqa: E402

_native._LIB_PATH = os.path.abspath(sys.argv[1])
script = sys.argv[2]
sys.argv = sys.argv[2:]
runpy.run_path(script, run_name='__main__')
