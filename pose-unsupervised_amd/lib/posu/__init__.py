"""posu: Python side of the MI355X-native pose-unsupervised hot path.

_native  -- ctypes binding of libposeu.so (include/posu.h)
ops      -- tensor wrappers + autograd Functions over the kernels
packing  -- reference NCHW parameters -> kernel layouts, BN folding
plan     -- PoseResNet forward as a launch sequence (hipGraph-capturable)
pipeline -- the batched 4-view path: forward -> soft-argmax -> epipolar -> DLT
synthetic-- deterministic synthetic weights / cameras / batches (tests, bench)
"""
