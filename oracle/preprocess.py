"""ORACLE (test infrastructure only) -- NumPy restatement of the reference's
image preprocessing, detectron/utils/blob.py:97-117 `prep_im_for_blob` and
:65-94 `im_list_to_blob`:

  im = im.astype(float32) - PIXEL_MEANS            (:105-106)
  im = cv2.resize(im, REID.SCALE, INTER_CUBIC)      (:112)
  blob = NCHW stack                                 (:85-93)

cv2 is not installed here and the reference pins no opencv version
(requirements.txt:4), so the resize is restated from OpenCV's published
INTER_CUBIC definition: Keys cubic with a = -0.75, source coordinate
(dst + 0.5) * (src / dst) - 0.5, separable (horizontal pass first), border
taps clamped to the edge.  Parity vs cv2 itself: UNPINNED (no cv2, no
fixture in the reference).
"""
import numpy as np

PIXEL_MEANS = np.array([102.9801, 115.9465, 122.7717], np.float32)


def cubic_weights(t):
    A = -0.75
    t = np.asarray(t, np.float64)
    w0 = ((A * (t + 1) - 5 * A) * (t + 1) + 8 * A) * (t + 1) - 4 * A
    w1 = ((A + 2) * t - (A + 3)) * t * t + 1
    w2 = ((A + 2) * (1 - t) - (A + 3)) * (1 - t) * (1 - t) + 1
    w3 = 1 - w0 - w1 - w2
    return np.stack([w0, w1, w2, w3], -1)


def _taps(n_src, n_dst):
    f = (np.arange(n_dst) + 0.5) * (n_src / n_dst) - 0.5
    i0 = np.floor(f).astype(np.int64)
    w = cubic_weights(f - i0)
    idx = np.clip(i0[:, None] + np.arange(-1, 3)[None, :], 0, n_src - 1)
    return idx, w


def resize_cubic(im, out_w, out_h):
    """im float [H, W, C] -> [out_h, out_w, C] (float64 accumulation)."""
    H, W = im.shape[:2]
    xi, xw = _taps(W, out_w)
    yi, yw = _taps(H, out_h)
    tmp = np.einsum('hxkc,xk->hxc', im[:, xi, :].astype(np.float64), xw)
    return np.einsum('ykxc,yk->yxc', tmp[yi, :, :], yw)


def prep_im_for_blob(im_bgr_u8, target_wh=(128, 384), means=PIXEL_MEANS):
    im = im_bgr_u8.astype(np.float32) - means
    return resize_cubic(im, target_wh[0], target_wh[1]).astype(np.float32)


def im_list_to_blob(ims):
    """HWC float images of equal size -> NCHW float32 (FPN padding off)."""
    return np.stack(ims).transpose(0, 3, 1, 2).astype(np.float32)
