"""CPU checks of the preprocessing restatement's invariants (cv2 absent:
parity with cv2 itself is unpinned; these pin the stated algorithm)."""
import numpy as np

from oracle import preprocess as pre


def test_cubic_weights_partition_of_unity():
    t = np.linspace(0, 1, 11)
    w = pre.cubic_weights(t)
    np.testing.assert_allclose(w.sum(-1), 1.0, atol=1e-12)
    np.testing.assert_allclose(pre.cubic_weights(0.0), [0, 1, 0, 0], atol=1e-12)


def test_constant_image_stays_constant():
    im = np.full((128, 64, 3), 77, np.uint8)
    out = pre.prep_im_for_blob(im)
    np.testing.assert_allclose(out, np.broadcast_to(77 - pre.PIXEL_MEANS, out.shape), rtol=0, atol=1e-4)
    assert out.shape == (384, 128, 3)


def test_identity_resize():
    rng = np.random.RandomState(0)
    im = rng.rand(20, 12, 3)
    np.testing.assert_allclose(pre.resize_cubic(im, 12, 20), im, atol=1e-12)


def test_weights_symmetric_at_half():
    w = pre.cubic_weights(0.5)
    np.testing.assert_allclose(w, w[::-1], atol=1e-15)
    np.testing.assert_allclose(w, [-0.09375, 0.59375, 0.59375, -0.09375], atol=1e-15)


def test_matches_an_independent_bicubic_implementation():
    """torch's upsample_bicubic2d (align_corners=False) implements the same
    published cubic convolution (a = -0.75, half-pixel centres, clamped
    border taps) as OpenCV's INTER_CUBIC: a second, independent
    implementation of the stated algorithm agrees with the restatement at
    the reference's scale (Market 64x128 -> 128x384).  Not a cv2 pin."""
    import torch
    import torch.nn.functional as F
    rng = np.random.RandomState(1)
    im = rng.randint(0, 256, (128, 64, 3)).astype(np.uint8)
    ours = pre.prep_im_for_blob(im)
    x = torch.from_numpy((im.astype(np.float32) - pre.PIXEL_MEANS).transpose(2, 0, 1)[None])
    ref = F.interpolate(x.double(), size=(384, 128), mode='bicubic', align_corners=False)
    np.testing.assert_allclose(ours, ref[0].numpy().transpose(1, 2, 0), rtol=0, atol=1e-3)
