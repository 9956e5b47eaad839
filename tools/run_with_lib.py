"""Run a repo script against another build of libposeu.so (A/B experiments only):
    python tools/run_with_lib.py LIB SCRIPT [args...]"""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

from posu import _native  # noqa: E402

_native._LIB_PATH = os.path.abspath(sys.argv[1])
sys.argv = sys.argv[2:]
runpy.run_path(sys.argv[0], run_name='__main__')
