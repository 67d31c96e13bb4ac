"""Generate tests/golden/sdl_quadrics_pin.json from the reference's one integrator output.

/root/reference/examples/sdl_quadrics.jpg (README.md:7) is raysnail's own 800x500 render of
sdl/quadric.sdl through the CLI (src/bin/raysnail.rs:311-445: CLI camera / light conventions, depth 8,
clamp * 255.5 -> u8, then saved by the author as a JPEG). This script decodes it with PIL and stores
only derived numbers -- the global mean RGB and 25x25-pixel block means (32 x 20 blocks) plus each
block's pixel standard deviation -- so the GPU test on the box (where /root/reference does not
exist) can compare a fresh render of the same scene against the reference's render.

usage: python tests/golden/make_quadric_pin.py [path/to/sdl_quadrics.jpg]
"""
import json
import os
import sys

import numpy as np

BLOCK = 25
HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT = "/root/reference/examples/sdl_quadrics.jpg"


def block_stats(rgb01: np.ndarray, block: int = BLOCK):
    h, w, _ = rgb01.shape
    by, bx = h // block, w // block
    a = rgb01[: by * block, : bx * block].reshape(by, block, bx, block, 3)
    return a.mean(axis=(1, 3)), a.std(axis=(1, 3))


def main():
    from PIL import Image
    path = sys.argv[1] if len(sys.argv) > 1 else DEFAULT
    im = Image.open(path).convert("RGB")
    a = np.asarray(im, dtype=np.float64) / 255.0
    mean, std = block_stats(a)
    out = {
        "source": "examples/sdl_quadrics.jpg (Varkalandar/raysnail README.md:7), decoded with PIL",
        "size": [im.size[0], im.size[1]],
        "block": BLOCK,
        "global_mean_rgb": [round(float(x), 6) for x in a.mean(axis=(0, 1))],
        "block_mean": np.round(mean, 5).tolist(),
        "block_std": np.round(std, 5).tolist(),
    }
    with open(os.path.join(HERE, "sdl_quadrics_pin.json"), "w") as f:
        json.dump(out, f)
    print("global mean", out["global_mean_rgb"])


if __name__ == "__main__":
    main()
