"""numpy restatements of the CLI's per-pass helpers (src/bin/raysnail.rs), used as test oracles.

TEST INFRASTRUCTURE ONLY."""
import numpy as np


def combine_pixels(old, new, p):
    """raysnail.rs:176-208 (f32)."""
    old = old.astype(np.float32)
    new = new.astype(np.float32)
    p = np.float32(p)
    keep = np.all(new == 0, axis=-1, keepdims=True)
    mixed = (old * p + new) / (p + np.float32(1.0))
    return np.where(keep, old, mixed).astype(np.float32)


def calc_noise(px):
    """raysnail.rs:150-173 for every pixel, including `let x = y`: the 5x5 window's columns are
    centred on y. f32, accumulation in window order (rows outer, columns inner)."""
    h, w, _ = px.shape
    px = px.astype(np.float32)
    ys, xs = np.mgrid[0:h, 0:w]
    dflt = px[ys, xs, :3]
    diff = np.zeros((h, w), np.float32)
    for dy in range(-2, 3):
        for dx in range(-2, 3):
            yy = ys + dy
            xx = ys + dx           # columns around y, not x (upstream shadows x)
            inside = (xx >= 0) & (yy >= 0) & (xx < w) & (yy < h)
            q = np.where(inside[..., None], px[np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1), :3], dflt)
            d = dflt - q
            diff = diff + ((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2])
    return diff


def noise_stats(px, t=0.01):
    n = calc_noise(px)
    valid = n[n == n]
    mn = min(np.float32(3.0), valid.min()) if valid.size else np.float32(3.0)
    mx = max(np.float32(1.0), valid.max()) if valid.size else np.float32(1.0)
    return float(mn), float(mx), int(np.count_nonzero(n >= np.float32(t))), (n >= np.float32(t)).astype(np.uint8)


def quantize_rgb8(px):
    """raysnail.rs:429-441: clamp(c as f64, 0..1) * 255.5 -> u8."""
    v = np.clip(px[..., :3].astype(np.float64), 0.0, 1.0)
    v = np.where(np.isnan(v), 0.0, v)
    return np.minimum(np.floor(v * 255.5), 255).astype(np.uint8)
