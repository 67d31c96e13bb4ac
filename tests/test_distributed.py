"""N > 1 path on CPU: world_size-2 gloo ranks render their shard with the CPU oracle (the GPU
renderer is swapped for the checker, the sharding/exchange code is the product's), then the
gathered frame is compared with a single-process render."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, split, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.binding import OracleScene
    from raysnail_amd import scenes
    from raysnail_amd.distributed import render_sharded
    cam, w = scenes.example_sdl(40, 23)
    photo = cam.take_photo().samples(4).depth(6).seed(5)
    orc = OracleScene(w)

    def render(rb, re, rs, p):
        st = photo.rows(rb, re, rs).pass_index(p).settings()
        img, _ = orc.render(cam.desc, st, threads=2)
        return torch.from_numpy(img)

    out = render_sharded(render, rank, world, split)
    if rank == 0:
        q.put(out.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _run(split, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, split, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def _single(pass_index=0):
    from oracle.binding import OracleScene
    from raysnail_amd import scenes
    cam, w = scenes.example_sdl(40, 23)
    photo = cam.take_photo().samples(4).depth(6).seed(5).pass_index(pass_index)
    img, _ = OracleScene(w).render(cam.desc, photo.settings(), threads=4)
    return img


def test_rows_split_world2_equals_single_frame():
    out = _run("rows", 2)
    assert np.array_equal(out, _single())


def test_rows_split_world3_uneven_rows():
    out = _run("rows", 3)   # 23 rows over 3 ranks: 8/8/7
    assert np.array_equal(out, _single())


def test_passes_split_world2_folds_like_cli():
    out = _run("passes", 2)
    p0, p1 = _single(0), _single(1)
    init = np.zeros_like(p0)
    init[..., 3] = 1
    acc = (init * np.float32(0) + p0) / np.float32(1)
    acc = (acc * np.float32(1) + p1) / np.float32(2)
    assert np.allclose(out, acc, rtol=0, atol=1e-7)
