"""Measure BASELINE.json's configs C2-C5 on one GPU (the bench line itself is C1-shaped, bench.py): after one
full host-output frame (warm-up + the image checked against the oracle), the median of 3 device-resident frames
(1 when a frame takes over a second), plus the CPU oracle on a bounded row subset of the same frame (num_cpus + 1
threads like Painter::draw), scaled by samples. Writes one JSON object per config to stdout.

usage: python tools/bench_configs.py [--only C3,C4] [--cpu-seconds 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def configs():
    from raysnail_amd import scenes
    return {
        "C2": ("sdl/example.sdl + CLI lights, 800x500, 64 spp, depth 50",
               lambda: scenes.example_sdl(800, 500), 64, 50),
        "C3": ("RTIOW final scene (balls_scene seed 7 + light), 1920x1080, 256 spp, depth 50",
               lambda: scenes.rtow_13_1(1920, 1080)[:2], 256, 50),
        "C4": ("sdl/quadric.sdl + Cornell xz emitter, 1024x1024, 1024 spp, depth 50",
               lambda: scenes.quadric_sdl(1024, 1024), 1024, 50),
        "C5": ("synthetic 72k-triangle mesh + ground + light, 1920x1080, 512 -> 484 spp, depth 50",
               lambda: scenes.mesh_scene(1920, 1080), 512, 50),
        # not BASELINE configs: the §8(f)3 features (rich scene mode) at a bench-like size
        "X1": ("all_feature_scene (boxes, media, Image + Perlin spheres, moving sphere), 800x800, 64 spp, depth 50",
               lambda: scenes.all_feature_scene(800, 800), 64, 50),
        "X2": ("cornell_smoke (two ConstantMedium boxes), 600x600, 64 spp, depth 50",
               lambda: scenes.cornell_smoke(600, 600), 64, 50),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=len(os.sched_getaffinity(0)) + 1,
                    help="default num_cpus + 1 like Painter::draw (painter.rs:321-325)")
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--inproc", action="store_true", help="run the configs in this process (default: one process each)")
    args = ap.parse_args()
    if not args.inproc:
        # one process per config: a config's frame slots size their pools from the memory free when they allocate
        # (rs_host.cpp pool_limit_free), so nothing of the previous config's scene may still be held
        import subprocess
        keys = [k for k in configs() if not args.only or k in set(filter(None, args.only.split(",")))]
        for key in keys:
            cmd = [sys.executable, os.path.abspath(__file__), "--inproc", "--only", key, "--cpu-seconds", str(args.cpu_seconds),
                   "--cpu-threads", str(args.cpu_threads), "--mode", str(args.mode)]
            r = subprocess.run(cmd)
            if r.returncode != 0:
                sys.exit(r.returncode)
        return
    import torch
    torch.cuda.set_device(0)
    from oracle.binding import OracleScene
    only = set(filter(None, args.only.split(",")))
    for key, (desc, build, spp, depth) in configs().items():
        if only and key not in only:
            continue
        cam, world = build()
        t0 = time.perf_counter()
        ds = world.device_scene()
        t_commit = time.perf_counter() - t0
        H, W = cam.desc.height, cam.desc.width
        photo = cam.take_photo().samples(spp).depth(depth).seed(1).mode(args.mode)
        # the full frame once: kernel load and the frame's workspace (path pool, radiance ring: a few-row warm-up
        # left their allocation inside the timed frame), and the image the oracle rows are checked against
        t0 = time.perf_counter()
        img = photo.shot(None, world)
        t_first = time.perf_counter() - t0
        st = photo.last_stats
        # timed like bench.py: frames into a device buffer (inputs resident, no PCIe), the median of 3 frames (1
        # for frames over a second)
        frame = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        # one device frame per frame slot first (each slot allocates its own path pool and radiance ring on its
        # first frame: for C4's 256 Mi-path pool that alone took ~0.9 s)
        for _ in range(2):
            ds.render_device(cam.desc, photo.settings(), frame.data_ptr(), stream, stats=False)
        torch.cuda.synchronize()
        reps = 3 if t_first < 1.0 else 1
        times = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ds.render_device(cam.desc, photo.settings(), frame.data_ptr(), stream, stats=False)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        dt = sorted(times)[len(times) // 2]
        assert np.array_equal(frame.cpu().numpy(), img, equal_nan=True), "device frame differs from the host frame"
        gpu_msps = st.samples / dt / 1e6
        # CPU oracle: rows 0::k with k chosen from a probe so the run takes ~cpu_seconds
        orc = OracleScene(world)
        probe_rows = max(1, H // 64)
        ps = photo.rows(0, 0, H // probe_rows).settings()
        t0 = time.perf_counter()
        _, pst = orc.render(cam.desc, ps, threads=args.cpu_threads)
        tp = time.perf_counter() - t0
        per_sample = tp / max(1, pst.samples)
        want = args.cpu_seconds / per_sample
        k = max(1, int(round(st.samples / max(1.0, want))))
        cs = photo.rows(0, 0, k).settings()
        t0 = time.perf_counter()
        ref, cst = orc.render(cam.desc, cs, threads=args.cpu_threads)
        tc = time.perf_counter() - t0
        cpu_msps = cst.samples / tc / 1e6
        same_rows = bool((img[::k] == ref[::k]).all())
        # roofline (bench.py's fields): the dominant kernel's launches event-timed in the host-output frame above
        # (its extends -- and the streaming finish, which traces the frame's last segments -- or the bounce-synchronous
        # extends), SURVEY 8(d)'s 44 B per segment; and the frame model 212 B/segment + 124 B/sample over the
        # device-resident frame time
        from raysnail_amd._abi import KERNEL_NAMES
        kl = max(1, st.kernel_launches)
        alg = 44.0 * st.segments / kl
        avg_s = st.kernel_ms / kl / 1e3
        ach = alg / avg_s / 1e9 if avg_s > 0 else 0.0
        fbytes = 212.0 * st.segments + 124.0 * st.samples
        roof = {"bound": "hbm", "kernel": KERNEL_NAMES.get(st.kernel_id), "launches": st.kernel_launches,
                "avg_launch_ms": round(avg_s * 1e3, 4), "alg_bytes_per_launch": int(alg),
                "achieved": round(ach, 2), "peak": 8000.0, "unit": "GB/s", "frac": round(ach / 8000.0, 5),
                "kernel_share_of_frame": round(st.kernel_ms / (dt * 1e3), 4),
                "frame_bytes": int(fbytes), "achieved_frame": round(fbytes / dt / 1e9, 2),
                "frac_frame": round(fbytes / dt / 1e9 / 8000.0, 5)}
        out = {"config": key, "workload": desc, "width": W, "height": H, "spp": int(spp ** 0.5) ** 2,
               "depth": depth, "gpu": {"Msamples_per_s": round(gpu_msps, 2), "ms_per_frame": round(dt * 1e3, 2),
                                       "frames_timed": reps, "Gseg_per_s": round(st.segments / dt / 1e9, 3),
                                       "kernel_ms": round(st.kernel_ms, 2), "segments": st.segments,
                                       "segments_per_sample": round(st.segments / st.samples, 4),
                                       "launches": st.launches, "commit_s": round(t_commit, 3)},
               "roofline": roof,
               "cpu_baseline": {"Msamples_per_s": round(cpu_msps, 4), "threads": args.cpu_threads, "kind": "port",
                                "sample": f"rows 0::{k} ({cst.samples} samples) in {tc:.1f} s"},
               "speedup": round(gpu_msps / cpu_msps, 1), "sampled_rows_bit_identical": same_rows}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
