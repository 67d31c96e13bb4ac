"""GPU: the BASELINE configs (C2-C5) at their depth and image sizes, checked against the oracle.

* depth-50 parity for the SDL scenes (C2 example.sdl, C4 quadric.sdl + Cornell emitter) on small
  frames, bit for bit (the depth-8 frames are in test_gpu_parity.py);
* C3 at its full 1920x1080 size, 256 spp, depth 50: the oracle re-renders every 90th row;
* C5 (71.4k-triangle mesh) at 1920x1080, depth 50 at a reduced 16 spp: every 120th row;
* C4 at 1024x1024, depth 50 at a reduced 16 spp: every 128th row;
* the configs at full size, spp and depth: C2 every 10th row, C4 (1024 spp) every 256th, C5 (484 spp)
  every 540th.
Whole-frame properties (finite, alpha 1, sample count) are checked on every full-size frame.
"""
import numpy as np
import pytest

from raysnail_amd import scenes

pytestmark = pytest.mark.gpu


def _oracle(world):
    from oracle.binding import OracleScene
    return OracleScene(world)


def _check(img, ref, rows=slice(None)):
    g, r = img[rows], ref[rows]
    d = np.abs(g[..., :3].astype(np.float64) - r[..., :3].astype(np.float64))
    rmse = float(np.sqrt(np.mean(d * d)))
    exact = float(np.mean(np.all(g == r, axis=-1)))
    assert rmse < 1e-4 and exact >= 0.999, (rmse, exact, float(d.max()))


@pytest.mark.parametrize("name,build", [("example_sdl", lambda: scenes.example_sdl(64, 40)),
                                        ("quadric_sdl", lambda: scenes.quadric_sdl(48, 48))])
@pytest.mark.parametrize("spp", [4, 9])
def test_sdl_scenes_depth50(gpu, name, build, spp):
    cam, world = build()
    photo = cam.take_photo().samples(spp).depth(50).seed(21)
    img = photo.shot(None, world)
    ref, rs = _oracle(world).render(cam.desc, photo.settings(), threads=16)
    assert photo.last_stats.segments == rs.segments
    _check(img, ref)


@pytest.mark.parametrize("key,build,spp,k", [
    ("C3", lambda: scenes.rtow_13_1(1920, 1080)[:2], 256, 90),
    ("C5", lambda: scenes.mesh_scene(1920, 1080), 16, 120),
    ("C4", lambda: scenes.quadric_sdl(1024, 1024), 16, 128),
])
def test_full_size_config_rows_match_oracle(gpu, key, build, spp, k):
    cam, world = build()
    photo = cam.take_photo().samples(spp).depth(50).seed(1)
    img = photo.shot(None, world)
    H, W = cam.desc.height, cam.desc.width
    n = int(spp ** 0.5) ** 2
    assert photo.last_stats.samples == W * H * n
    assert np.isfinite(img).all() and (img[..., 3] == 1.0).all()
    ref, rs = _oracle(world).render(cam.desc, photo.rows(0, 0, k).settings(), threads=16)
    assert rs.samples == len(range(0, H, k)) * W * n
    _check(img, ref, slice(0, H, k))


@pytest.mark.parametrize("key,build,spp,k", [
    ("C2", lambda: scenes.example_sdl(800, 500), 64, 10),          # full size, spp and depth
    ("C4", lambda: scenes.quadric_sdl(1024, 1024), 1024, 256),     # full 1024 spp, every 256th row
    ("C5", lambda: scenes.mesh_scene(1920, 1080), 512, 540),       # 512 -> 484 spp (painter.rs:110-118)
])
def test_full_config_spp_rows_match_oracle(gpu, key, build, spp, k):
    """The configs at their full size, spp and depth 50 (BASELINE.json configs[1], [3], [4]): the
    whole frame on the GPU, the oracle on every k-th row (bounded CPU time: C5's mesh costs the
    oracle ~0.15 Msamples/s)."""
    cam, world = build()
    photo = cam.take_photo().samples(spp).depth(50).seed(1)
    img = photo.shot(None, world)
    H, W = cam.desc.height, cam.desc.width
    n = int(spp ** 0.5) ** 2
    assert photo.last_stats.samples == W * H * n
    assert np.isfinite(img).all() and (img[..., 3] == 1.0).all()
    ref, rs = _oracle(world).render(cam.desc, photo.rows(0, 0, k).settings(), threads=16)
    assert rs.samples == len(range(0, H, k)) * W * n
    _check(img, ref, slice(0, H, k))


def test_pool_sized_from_free_memory(gpu):
    """A C3-shaped frame (RTIOW 1920x1080, 256 spp, depth 50) rendered by a scene whose device is shared: a
    torch tensor holds half the device (after the reference scene's own pool), so the three frame slots' full
    256 Mi-path pools (~65 GB each) no longer fit. The pools are sized from the memory free when a slot
    allocates (rs_host.cpp pool_limit_free): three asynchronous frames, one per slot, and a two-lane frame
    equal the unconstrained frame bit for bit, or the call returns an RS_E_* code; it never aborts."""
    import gc
    import torch
    from raysnail_amd import _abi as A
    from raysnail_amd.api import RaysnailError
    gc.collect()  # the scenes of earlier tests give their pools back (rs_scene_destroy)
    torch.cuda.empty_cache()
    cam, world = scenes.rtow_13_1(1920, 1080)[:2]
    st = cam.take_photo().samples(256).depth(50).seed(1).settings()
    ref, rstats = world.device_scene().render(cam.desc, st)
    free, total = torch.cuda.mem_get_info()
    # half the device, leaving the second scene at least 48 GiB (three slots' pools then get ~13 GB each)
    hold = torch.empty(max(0, min(total // 2, free - (48 << 30))), dtype=torch.uint8, device="cuda")
    try:
        cam2, world2 = scenes.rtow_13_1(1920, 1080)[:2]
        ds = world2.device_scene()
        outs = [torch.zeros((1080, 1920, 4), dtype=torch.float32, device="cuda") for _ in range(3)]
        s = torch.cuda.current_stream().cuda_stream
        ok, errs = 0, []
        try:
            for o in outs:  # one frame per frame slot, back to back: each slot allocates its own pool
                ds.render_device(cam2.desc, st, o.data_ptr(), s, stats=False)
            torch.cuda.synchronize()
            for o in outs:
                assert np.array_equal(o.cpu().numpy(), ref)
            ok += 1
        except RaysnailError as e:
            assert e.code in (A.RS_E_NOMEM, A.RS_E_HIP), e
            errs.append(str(e))
        del outs
        ds.set_lanes(2)
        try:
            img, stats = ds.render(cam2.desc, st)
            assert stats.segments == rstats.segments
            assert np.array_equal(img, ref)
            ok += 1
        except RaysnailError as e:
            assert e.code in (A.RS_E_NOMEM, A.RS_E_HIP), e
            errs.append(str(e))
        # on a 288 GB device both renders are expected to succeed with the shrunken pools
        assert ok == 2, errs
    finally:
        del hold
        torch.cuda.empty_cache()
