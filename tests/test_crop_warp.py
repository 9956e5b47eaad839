"""The data path's crop: JointsDatasetCompatible.__getitem__'s
cv2.warpAffine(INTER_LINEAR) + ToTensor + Normalize (lib/dataset/joints_dataset_compatible.py
:161-172).  OpenCV is absent here, so the oracle (oracle/geometry_ref.warp_affine_linear)
restates OpenCV 3.4's fixed-point algorithm and is pinned only by the exact cases below:
PARITY UNPINNED against cv2 itself.  The HIP kernel (posu_crop_warp) must match the oracle bit
for bit (GPU tests)."""
import numpy as np
import pytest
import torch

from oracle import geometry_ref as G


def _img(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def _getitem_trans(rng, h, w, size=256):
    """A crop affine as __getitem__ builds it: centre / scale (x 200 px) / rotation."""
    from utils.transforms import get_affine_transform
    c = np.array([rng.uniform(-0.1, 1.1) * w, rng.uniform(-0.1, 1.1) * h])
    s = np.array([rng.uniform(0.3, 2.5)] * 2)
    r = float(rng.choice([0.0, rng.uniform(-60, 60)]))
    return get_affine_transform(c, s, r, [size, size])


def test_oracle_exact_cases():
    img = _img(40, 50, 0)
    assert np.array_equal(G.warp_affine_linear(img, [[1, 0, 0], [0, 1, 0]], (50, 40)), img)        # identity
    o = G.warp_affine_linear(img, [[1, 0, 3], [0, 1, 2]], (50, 40))                               # integer shift
    assert np.array_equal(o[2:, 3:], img[:-2, :-3]) and not o[:2].any() and not o[:, :3].any()
    o = G.warp_affine_linear(img, [[1, 0, -0.5], [0, 1, 0]], (50, 40))                            # half pixel
    a, b = img[:, :-1].astype(int), img[:, 1:].astype(int)
    assert np.array_equal(o[:, :-1], (a + b + 1) >> 1)
    assert np.array_equal(o[:, -1], (img[:, -1].astype(int) + 1) >> 1)    # the last tap is the 0 border
    o = G.warp_affine_linear(img, [[1, 0, 100], [0, 1, 0]], (50, 40))                             # all outside
    assert not o.any()
    # horizontal flip about the centre column (x' = W - 1 - x): exact
    o = G.warp_affine_linear(img, [[-1, 0, 49], [0, 1, 0]], (50, 40))
    assert np.array_equal(o, img[:, ::-1])


def test_oracle_is_bilinear_within_the_fixed_point_error():
    """Against float bilinear interpolation with the same constant-0 border: within 2 grey levels
    (1/32-px coordinates, 15-bit weights)."""
    rng = np.random.default_rng(1)
    img = (np.add.outer(np.arange(60), np.arange(70)) * 1.5 % 256).astype(np.uint8)[:, :, None].repeat(3, 2)
    for _ in range(4):
        M = _getitem_trans(rng, 60, 70, 48)
        o = G.warp_affine_linear(img, M, (48, 48)).astype(float)
        Mi = np.linalg.inv(np.vstack([M, [0, 0, 1]]))[:2]
        yy, xx = np.meshgrid(np.arange(48), np.arange(48), indexing='ij')
        sx = Mi[0, 0] * xx + Mi[0, 1] * yy + Mi[0, 2]
        sy = Mi[1, 0] * xx + Mi[1, 1] * yy + Mi[1, 2]
        x0, y0 = np.floor(sx).astype(int), np.floor(sy).astype(int)
        fx, fy = sx - x0, sy - y0
        ref = np.zeros((48, 48))
        for ox, oy, wt in ((0, 0, (1 - fx) * (1 - fy)), (1, 0, fx * (1 - fy)), (0, 1, (1 - fx) * fy), (1, 1, fx * fy)):
            tx, ty = x0 + ox, y0 + oy
            ok = (tx >= 0) & (tx < 70) & (ty >= 0) & (ty < 60)
            ref += np.where(ok, img[np.clip(ty, 0, 59), np.clip(tx, 0, 69), 0], 0) * wt
        inside = (x0 >= 0) & (x0 < 69) & (y0 >= 0) & (y0 < 59)
        assert np.abs(o[..., 0] - ref)[inside].max() <= 2.0


@pytest.mark.gpu
@pytest.mark.parametrize('out', ['u8', 'f32'])
def test_crop_warp_kernel_matches_the_oracle_bit_for_bit(cuda, out):
    from posu import datapath
    rng = np.random.default_rng(7)
    sizes = [(1002, 1000), (480, 640), (37, 53), (256, 256), (1000, 1000), (300, 200)]
    imgs = [_img(h, w, k) for k, (h, w) in enumerate(sizes)]
    trans = np.stack([_getitem_trans(rng, h, w) for (h, w) in sizes] +
                     [np.array([[1.0, 0, 0], [0, 1.0, 0]]), np.array([[1.0, 0, -0.5], [0, 1.0, 0.25]])])
    imgs += [imgs[3], imgs[3]]
    got = datapath.crop_warp(imgs, trans, (256, 256), cuda, out=out).cpu().numpy()
    for k, (im, M) in enumerate(zip(imgs, trans)):
        ref = G.warp_affine_linear(im, M, (256, 256))
        if out == 'u8':
            np.testing.assert_array_equal(got[k], ref)
        else:
            np.testing.assert_array_equal(got[k], G.to_tensor_normalize(ref, datapath.IMAGENET_MEAN,
                                                                        datapath.IMAGENET_STD))


@pytest.mark.gpu
def test_crop_batch_is_getitem_crop(cuda):
    """crop_batch = get_affine_transform per sample + the warp: the network input __getitem__
    hands the model (ToTensor + Normalize)."""
    from posu import datapath
    from utils.transforms import get_affine_transform
    imgs = [_img(500, 600, 11), _img(500, 600, 12)]
    centers = [np.array([300.0, 250.0]), np.array([100.0, 480.0])]
    scales = [np.array([1.2, 1.2]), np.array([2.0, 2.0])]
    x, trans = datapath.crop_batch(imgs, centers, scales, [0.0, 30.0], (256, 256), cuda)
    assert x.shape == (2, 3, 256, 256) and x.dtype == torch.float32
    for k in range(2):
        M = get_affine_transform(centers[k], scales[k], [0.0, 30.0][k], [256, 256])
        np.testing.assert_array_equal(trans[k], M)
        ref = G.to_tensor_normalize(G.warp_affine_linear(imgs[k], M, (256, 256)), datapath.IMAGENET_MEAN,
                                    datapath.IMAGENET_STD)
        np.testing.assert_array_equal(x[k].cpu().numpy(), ref)
