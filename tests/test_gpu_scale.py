"""GPU: large trees (4-wide BVH past the LDS stack, HBM stack overflow) and the multi-device C-ABI.

* C5's full-size mesh (~71.4k triangles) and a ~1M-triangle mesh commit with the 4-wide tree
  (rs_render_stats.tree_arity == 4) although their worst-case traversal stack exceeds the LDS part;
  their frames match the oracle (whose BVH is the reference's binary recursion).
* rs_scene_commit_devices: the row lattice split over devices (painter.rs:248 over GPUs) gives the
  1-device frame bit for bit, through rs_render (host) and rs_render_device (into a torch tensor);
  virtual devices ({0, 0}, {0, 0, 0}) exercise the split, the per-device streams and the frame-end
  row gather on the one GPU of the box.
"""
import numpy as np
import pytest

from raysnail_amd import _abi as A
from raysnail_amd import api, scenes

pytestmark = pytest.mark.gpu
KSTACK_LDS = 16  # the flat mode's LDS stack entries (rs_internal.h stack_lds)


def _oracle(world):
    from oracle.binding import OracleScene
    return OracleScene(world)


def _match(img, ref):
    d = np.abs(img[..., :3].astype(np.float64) - ref[..., :3].astype(np.float64))
    rmse = float(np.sqrt(np.mean(d * d)))
    exact = float(np.mean(np.all(img == ref, axis=-1)))
    return rmse, exact


@pytest.mark.parametrize("mode", [A.RS_MODE_WAVEFRONT, A.RS_MODE_MEGAKERNEL])
def test_full_c5_mesh_uses_bvh4_and_matches_oracle(gpu, mode):
    cam, world = scenes.mesh_scene(64, 36)          # 120 x 300 -> 71,402 objects (C5 mesh)
    ds = world.device_scene()
    info = ds.info()
    assert info.n_objects > 70000
    assert info.tree_arity == 4, "C5 must traverse the 4-wide tree"
    assert info.stack_need > KSTACK_LDS == info.stack_lds   # the HBM overflow is exercised
    photo = cam.take_photo().samples(4).depth(8).seed(5).mode(mode)
    img = photo.shot(None, world)
    assert photo.last_stats.tree_arity == 4
    ref, rs = _oracle(world).render(cam.desc, photo.settings(), threads=16)
    assert photo.last_stats.segments == rs.segments
    rmse, exact = _match(img, ref)
    assert rmse < 1e-4 and exact >= 0.999, (rmse, exact)


def test_million_triangle_mesh(gpu):
    cam, world = scenes.mesh_scene(48, 27, 500, 1000)   # 998,002 objects
    ds = world.device_scene()
    info = ds.info()
    assert info.n_objects > 990000 and info.tree_arity == 4 and info.stack_need > KSTACK_LDS
    photo = cam.take_photo().samples(4).depth(6).seed(2)
    img = photo.shot(None, world)
    assert photo.last_stats.tree_arity == 4
    ref, rs = _oracle(world).render(cam.desc, photo.settings(), threads=16)
    assert photo.last_stats.segments == rs.segments
    rmse, exact = _match(img, ref)
    assert rmse < 1e-4 and exact >= 0.999, (rmse, exact)


def _frame(world, cam, st, devices, mask=None):
    ds = api.DeviceScene(world, devices=devices)
    assert ds.info().n_devices == len(devices)
    out, stats = ds.render(cam.desc, st, mask)
    return out, stats, ds


@pytest.mark.parametrize("build", ["rtow", "mesh", "quadric"])
def test_virtual_devices_equal_one_device(gpu, build):
    cam, world = {"rtow": lambda: scenes.rtow_13_1(72, 45)[:2],
                  "mesh": lambda: scenes.mesh_scene(64, 36, 40, 80),
                  "quadric": lambda: scenes.quadric_sdl(48, 48)}[build]()
    st = cam.take_photo().samples(9).depth(8).seed(4).settings()
    one, s1, _ = _frame(world, cam, st, [0])
    for devs in ([0, 0], [0, 0, 0]):
        many, sn, _ = _frame(world, cam, st, devs)
        assert np.array_equal(one, many), devs
        assert sn.segments == s1.segments and sn.samples == s1.samples
        assert sn.kernel_launches >= s1.kernel_launches


def test_virtual_devices_rows_mask_and_untouched(gpu):
    cam, world = scenes.example_sdl(50, 31)
    photo = cam.take_photo().samples(4).depth(8).seed(6)
    st = photo.rows(3, 29, 2).settings()            # a sparse lattice: odd rows 3..27
    mask = (np.indices((31, 50)).sum(0) % 5 != 0).astype(np.uint8)
    sentinel = np.full((31, 50, 4), -7.0, dtype=np.float32)
    a, _, _ = _frame(world, cam, st, [0], mask)
    ds3 = api.DeviceScene(world, devices=[0, 0, 0])
    b, _ = ds3.render(cam.desc, st, mask, out=sentinel.copy())
    rows = np.arange(3, 29, 2)
    assert np.array_equal(a[rows], b[rows])
    others = np.setdiff1d(np.arange(31), rows)
    assert np.all(b[others] == -7.0)                 # rows off the lattice keep the caller's values
    assert np.all(b[rows][mask[rows] == 0] == 0.0)


def test_virtual_devices_render_device(gpu):
    torch = gpu
    cam, world, _, _ = scenes.rtow_13_1(64, 40)
    st = cam.take_photo().samples(4).depth(8).seed(9).settings()
    host, _, _ = _frame(world, cam, st, [0])
    ds = api.DeviceScene(world, devices=[0, 0])
    t = torch.zeros((40, 64, 4), dtype=torch.float32, device="cuda")
    stats = ds.render_device(cam.desc, st, t.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert stats.samples == 64 * 40 * 4 and stats.kernel_launches > 0
    assert np.array_equal(t.cpu().numpy(), host)
    # asynchronous (no stats): the second device's rows are ordered after the caller's stream by the
    # frame's entry event and copied into the first device's buffer; two frames in flight on a side
    # stream, the buffers reset on the caller's stream first
    side = torch.cuda.Stream()
    for k in range(3):
        t.fill_(-1.0)
        side.wait_stream(torch.cuda.current_stream())
        assert ds.render_device(cam.desc, st, t.data_ptr(), side.cuda_stream, stats=False) is None
        torch.cuda.current_stream().wait_stream(side)
        assert np.array_equal(t.cpu().numpy(), host), k


def test_host_only_commit_refuses_render(gpu):
    cam, world, _, _ = scenes.rtow_13_1(16, 10)
    ds = api.DeviceScene(world, devices=[])
    assert ds.info().n_devices == 0
    with pytest.raises(api.RaysnailError):
        ds.render(cam.desc, cam.take_photo().samples(1).settings())


def test_virtual_devices_render_device_passes(gpu):
    """rs_render_device_passes on a scene committed to virtual devices {0, 0} (one-pass calls over the devices) and
    on one device with passes too large for the sample stream (1.2 M samples at depth 8: one-pass calls): every pass
    equals its one-pass frame on one device."""
    torch = gpu
    s = torch.cuda.current_stream().cuda_stream
    for w, h, spp, devs in ((64, 40, 4, [0, 0]), (1200, 1000, 1, [0])):
        cam, world, _, _ = scenes.rtow_13_1(w, h)
        one = api.DeviceScene(world, devices=[0])
        ds = api.DeviceScene(world, devices=devs)
        photo = cam.take_photo().samples(spp).depth(8).seed(9).pass_index(5)
        outs = [torch.full((h, w, 4), -1.0, dtype=torch.float32, device="cuda") for _ in range(3)]
        stats = ds.render_device_passes(cam.desc, photo.settings(), [o.data_ptr() for o in outs], s)
        assert stats.samples == 3 * w * h * spp
        for k in range(3):
            ref = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
            one.render_device(cam.desc, cam.take_photo().samples(spp).depth(8).seed(9).pass_index(5 + k).settings(),
                              ref.data_ptr(), s)
            assert np.array_equal(outs[k].cpu().numpy(), ref.cpu().numpy(), equal_nan=True), (w, devs, k)
