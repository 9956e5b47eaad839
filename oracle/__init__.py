"""CPU ORACLE -- test infrastructure only.

A plain CPU restatement (torch-CPU fp32 / numpy fp64) of the reference's hot path,
used ONLY as the checker by tests/, __graft_entry__.smoke() and bench.py's
``cpu_baseline`` leg.  The product (pose-unsupervised_amd/) never imports it.

Pinning: every function here is checked against golden vectors produced by importing
the reference itself (tests/golden/make_golden.py -> tests/golden/*.npz):
PoseResNet heatmaps / features, soft-argmax + transform_back, argmax decoding,
FundamentalLoss and JointsMSELoss values and gradients, camera projection.  The
triangulation restates pymvg (not vendored by the reference, not installed): it is
pinned by exact known-answer tests (noise-free pinhole projections of known 3-D
points, produced with the reference's own projection code), and is otherwise
"parity unpinned" for the distorted / noisy case.
"""
