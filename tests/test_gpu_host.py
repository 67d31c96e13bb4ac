"""GPU: the C++ host layer end to end (SDL front end and the raysnail-shaped object API) against
the CPU oracle, bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from raysnail_amd import _abi as A
from raysnail_amd import host_lib

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN_SDL = os.path.join(HERE, "golden", "sdl")


@pytest.mark.parametrize("mode", [A.RS_MODE_AUTO, A.RS_MODE_MEGAKERNEL, A.RS_MODE_WAVEFRONT])
@pytest.mark.parametrize("name", ["features", "loops"])
def test_sdl_render_matches_oracle(gpu, oracle_lib, name, mode):
    from oracle.binding import OracleScene
    path = os.path.join(GOLDEN_SDL, name + ".sdl")
    W, H = 96, 60
    st = A.rs_render_settings()
    st.samples, st.depth, st.gamma, st.seed, st.mode, st.row_step = 16, 12, 1, 9, mode, 1
    img, stats = host_lib.sdl_render(path, W, H, st)
    sc = OracleScene(fill=lambda api, h: host_lib.sdl_build(path, W, H, api, h))
    ref, rstats = sc.render(sc.fill_result, st, threads=16)
    assert stats.segments == rstats.segments
    assert np.array_equal(img, ref), f"{np.mean(np.all(img == ref, axis=-1)):.4f} of pixels equal"


def test_cpp_api_driver(gpu, oracle_lib):
    """tests/cpp/test_api.cpp: every material / geometry kind through the C++ classes, PainterTarget
    rows + sentinel, PixelController mask, progressive passes, error paths; vs the oracle."""
    from oracle.binding import LIB_PATH
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "cpp")], check=True)
    r = subprocess.run([os.path.join(HERE, "cpp", "build", "test_api"), LIB_PATH], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout + r.stderr
