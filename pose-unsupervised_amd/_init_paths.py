"""Put this build's ``lib`` on sys.path, like the reference's run/*/_init_paths.py, so
``import models.pose_resnet``, ``multiviews.triangulate`` ... resolve to the HIP build."""
import os.path as osp
import sys

LIB = osp.join(osp.dirname(osp.abspath(__file__)), 'lib')
if LIB not in sys.path:
    sys.path.insert(0, LIB)
