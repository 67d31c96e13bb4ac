"""The CLI's progressive passes and output (src/bin/raysnail.rs:123-208, 311-445): PNG output on
the CPU; the GPU noise map and the C++ pass loop against numpy / oracle restatements."""
import os
import struct
import zlib

import numpy as np
import pytest

from raysnail_amd import _abi as A
from raysnail_amd import host_lib

HERE = os.path.dirname(os.path.abspath(__file__))
import sys
sys.path.insert(0, HERE)
import passes_ref as R  # noqa: E402


def read_png_rgb8(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat = 8, b""
    w = h = None
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        crc = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0]
        assert crc == zlib.crc32(typ + body) & 0xFFFFFFFF
        if typ == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", body[:10])
            assert depth == 8 and ctype == 2
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    rows = np.frombuffer(raw, np.uint8).reshape(h, 1 + 3 * w)
    assert (rows[:, 0] == 0).all()
    return rows[:, 1:].reshape(h, w, 3)


def test_png_output_quantisation(tmp_path):
    rng = np.random.default_rng(3)
    px = rng.uniform(-0.2, 1.3, (37, 53, 4)).astype(np.float32)
    px[0, 0, :3] = np.nan
    px[1, 1, :3] = [1.0, 0.5, 0.0]
    path = str(tmp_path / "out.png")
    host_lib.write_png(path, px)
    got = read_png_rgb8(path)
    assert np.array_equal(got, R.quantize_rgb8(px))
    assert list(got[1, 1]) == [255, 127, 0]


def test_png_large_frame_multiple_stored_blocks(tmp_path):
    px = np.linspace(0, 1, 300 * 200 * 4, dtype=np.float32).reshape(200, 300, 4)
    path = str(tmp_path / "big.png")
    host_lib.write_png(path, px)
    assert np.array_equal(read_png_rgb8(path), R.quantize_rgb8(px))


def test_noise_reference_quirk():
    """calc_noise's window follows the row index: a pixel's noise only sees column y's neighbourhood."""
    px = np.zeros((6, 9, 4), np.float32)
    px[..., 3] = 1
    px[2, 8, :3] = 1.0             # far from column 2's window for row 2
    n = R.calc_noise(px)
    assert n[2, 8] > 0 and n[2, 2] == 0   # (8,2) differs from its window; (2,2)'s window is all zero


@pytest.mark.gpu
def test_noise_map_kernel_matches_restatement(gpu):
    torch = gpu
    rng = np.random.default_rng(7)
    for (h, w) in ((31, 47), (200, 160)):
        px = rng.uniform(0, 1, (h, w, 4)).astype(np.float32) ** 3
        px[rng.uniform(size=(h, w)) < 0.5] = px[0, 0]
        lib = A.load()
        d = torch.from_numpy(px).cuda()
        redo = torch.zeros((h, w), dtype=torch.uint8, device="cuda")
        st = A.rs_noise_stats()
        assert lib.rs_noise_map_device(d.data_ptr(), w, h, 0.01, redo.data_ptr(), None, st) == 0
        mn, mx, cnt, ref_map = R.noise_stats(px)
        assert (st.min, st.max, st.count) == (np.float32(mn), np.float32(mx), cnt)
        assert np.array_equal(redo.cpu().numpy(), ref_map)


@pytest.mark.gpu
def test_combine_kernel_matches_restatement(gpu):
    torch = gpu
    rng = np.random.default_rng(8)
    old = rng.uniform(0, 2, (40, 30, 4)).astype(np.float32)
    new = rng.uniform(0, 2, (40, 30, 4)).astype(np.float32)
    new[rng.uniform(size=(40, 30)) < 0.3] = 0
    d_old, d_new = torch.from_numpy(old).cuda(), torch.from_numpy(new).cuda()
    assert A.load().rs_combine_pixels_device(d_old.data_ptr(), d_new.data_ptr(), 40 * 30, 2.0, None) == 0
    assert np.array_equal(d_old.cpu().numpy(), R.combine_pixels(old, new, 2.0))


@pytest.mark.gpu
@pytest.mark.parametrize("adaptive", [False, True])
def test_pass_loop_matches_oracle(gpu, oracle_lib, adaptive):
    """render_passes (C++) vs the oracle's passes folded and measured in numpy, pass by pass."""
    from oracle.binding import OracleScene
    path = os.path.join(HERE, "golden", "sdl", "features.sdl")
    W, H, spp, passes, seed = 64, 40, 4, 3, 12
    img, noise = host_lib.sdl_render_passes(path, W, H, spp, passes, seed, adaptive)
    sc = OracleScene(fill=lambda api, h: host_lib.sdl_build(path, W, H, api, h))
    acc = np.zeros((H, W, 4), np.float32)
    acc[..., 3] = 1
    redo = np.ones((H, W), np.uint8)
    for p in range(passes):
        st = A.rs_render_settings()
        st.samples, st.depth, st.gamma, st.seed, st.row_step = spp, 8, 1, seed, 1
        st.pass_ = p
        frame, _ = sc.render(sc.fill_result, st, threads=16, mask=redo if adaptive else None)
        acc = R.combine_pixels(acc, frame, p)
        mn, mx, cnt, m = R.noise_stats(acc)
        assert tuple(noise[p]) == (np.float32(mn), np.float32(mx), np.float32(cnt))
        redo = m
    assert np.array_equal(img, acc)
