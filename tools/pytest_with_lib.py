"""pytest against another build of libposeu.so (A/B variants before one becomes the product build):

    python tools/pytest_with_lib.py pose-unsupervised_amd/build/ab6/libposeu_X.so tests/test_gpu_bottleneck.py -k w24
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

from posu import _native  # noqa: E402

_native._LIB_PATH = os.path.abspath(sys.argv[1])

import pytest  # noqa: E402

sys.exit(pytest.main(['-m', 'gpu', '-x', '-v', '--timeout', '200', '--timeout-method', 'thread'] + sys.argv[2:]))
