"""Statistics for comparing a render with the reference's own render (examples/sdl_quadrics.jpg).

Shared by tests/test_reference_render_pin.py, tests/golden/make_coplanar_delta.py and
tools/pin_variants.py. Test infrastructure only.

Per-block z-score. A 25x25-pixel block mean of a render at N spp has a Monte Carlo standard error
sigma_pix / 25, where sigma_pix is estimated from the render itself as the RMS of horizontal
neighbour differences / sqrt(2) inside the block (pixels are independent samples; at edges the
estimate includes the edge and is conservative). The reference's render has the same spp (121,
raysnail.rs CLI conventions), i.e. sqrt(spp_ours / 121) times ours; the JPEG adds quantisation of the
DC term and 4:2:0 chroma (measured ~0.5/255 on a block mean). So

    sigma_block^2 = (sigma_pix / 25)^2 * (1 + spp_ours / 121) + JPEG_SIGMA^2

and z = (ours - reference) / sigma_block per block and channel. The model has no term for the
spp-dependent bias of the per-pixel gamma sqrt and the u8 floor (Jensen: dark, noisy blocks come out
low at few spp), so compare renders at >= ~49 spp (measured max |z| 2.3 at 49 spp, 5.4 at 16).
"""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
JPEG_SIGMA = 0.002
REF_SPP = 121


def pin():
    return json.load(open(os.path.join(GOLDEN, "sdl_quadrics_pin.json")))


def quantize(rgba):
    """raysnail.rs:437-439: (clamp(c, 0..1) * 255.5) as u8, then / 255 like the decoded JPEG."""
    q = np.floor(np.clip(np.asarray(rgba)[..., :3].astype(np.float64), 0.0, 1.0) * 255.5)
    return np.minimum(q, 255.0) / 255.0


def _blocks(a, B):
    h, w = a.shape[:2]
    return a[: h // B * B, : w // B * B].reshape(h // B, B, w // B, B, -1)


def block_means(img01, B):
    return _blocks(img01, B).mean(axis=(1, 3))


def block_sigma(img01, B, spp):
    """Standard error of (our block mean - the reference's block mean), per block and channel."""
    dx = img01[:, 1:] - img01[:, :-1]
    dx = np.concatenate([dx, dx[:, -1:]], axis=1)
    s_pix = np.sqrt(_blocks(dx ** 2, B).mean(axis=(1, 3)) / 2.0)
    s_ours = s_pix / B
    s_ref = s_ours * np.sqrt(spp / REF_SPP)       # the reference render's noise at 121 spp
    return np.sqrt(s_ours ** 2 + s_ref ** 2 + JPEG_SIGMA ** 2)


def zmap(img01, spp, delta=None, p=None):
    """z-scores (blocks_y, blocks_x, 3) of a quantised render against the pin; `delta` (same shape)
    is added to our block means first (the coplanar-face correction, make_coplanar_delta.py)."""
    p = p or pin()
    B = p["block"]
    m = block_means(img01, B)
    if delta is not None:
        m = m + np.asarray(delta)
    return (m - np.array(p["block_mean"])) / block_sigma(img01, B, spp)


def global_gap(img01, p=None):
    p = p or pin()
    return np.abs(img01.mean(axis=(0, 1)) - np.array(p["global_mean_rgb"]))
