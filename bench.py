"""bench.py — BASELINE metric: Msamples/s (whole node) + ms/frame on the RTIOW-13.1 scene
(examples/rtow_13_1.rs: balls_scene seed 7 + light sphere) at 800x500, 64 spp, depth 8.

A step = one frame of that workload (inputs resident in HBM: the scene is committed before timing,
the frame lands in a device buffer). --split rows (default, strong scaling): the frame's rows are
interleaved over ranks like render_rows (painter.rs:248) and gathered to rank 0 at frame end (one
RCCL gather), so N = 1 and N = 8 render the same frame; --split passes (weak scaling): rank r renders
progressive pass r of the whole frame and rank 0 folds the passes (raysnail.rs:379-427).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 the driver uses
torch.distributed.run with one rank per GPU. Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
LANES = int(os.environ.get("RS_LANES", "0"))  # wavefront lanes of the timed region (rs_scene_set_lanes; 0 = defaults)
FRAMES = int(os.environ.get("RS_FRAMES", "0"))  # frames in flight (rs_scene_set_frames_in_flight; 0 = default 3)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpus():
    """What raysnail's thread count sees on this host: num_cpus 1.13.0 get() (Cargo.lock:345-347) =
    the CPUs in the process's affinity mask; Painter::draw uses get() + 1 threads (painter.rs:321-325).
    Also the CPU model and the cgroup CPU quota (which caps the threads' combined throughput)."""
    n = len(os.sched_getaffinity(0))
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return n, model, quota


def cpu_baseline(cam, world, spp, depth, seed, row_step, threads):
    """The oracle (C++ restatement of Painter::draw, f64, row-interleaved threads) on a bounded row
    subset of the same frame. kind = 'port'."""
    from oracle.binding import OracleScene
    from raysnail_amd import _abi as A
    st = A.rs_render_settings()
    st.samples, st.depth, st.gamma, st.seed = spp, depth, 1, seed
    st.row_begin, st.row_end, st.row_step = 0, 0, row_step
    sc = OracleScene(world)
    t0 = time.perf_counter()
    _, stats = sc.render(cam.desc, st, threads=threads)
    dt = time.perf_counter() - t0
    n, model, quota = host_cpus()
    cores = min(threads, n, int(quota) if quota else n)  # CPUs the threads can actually occupy at once
    return {"value": stats.samples / dt / 1e6, "unit": "Msamples/s", "cores": cores, "kind": "port",
            "threads": threads, "nproc": n, "cpu_model": model, "cgroup_cpu_quota": quota,
            "sample": f"rows 0::{row_step} of the frame ({stats.samples} samples, {stats.segments} segments) "
                      f"in {dt:.1f} s, {threads} threads (num_cpus {n} + 1, painter.rs:321-325) on {model}"
                      + (f" under a {quota}-CPU cgroup quota" if quota else "") + ", oracle/oracle.cpp f64"}


def frame_model_bytes(segments, samples):
    """SURVEY 8(d)'s frame-level algorithmic bytes: 212 B per path segment (extend: 28 B ray in,
    16 B hit out; shade: 76 B state + 16 B hit in, 76 B state out) + 124 B per camera sample (generate: 76 B
    state out; finalize: 16 B radiance + pixel in, 32 B float4 framebuffer read-modify-write)."""
    return 212.0 * segments + 124.0 * samples


class GatherProxy:
    """Rank 0's share of distributed.gather_rows on one GPU, per frame: the pack copy of its rows, the arrival
    of all `world` ranks' packed rows (a device copy of the same size stands in for the RCCL gather's writes
    into rank 0's receive buffer) and the de-interleave into the full frame -- on the current stream, like
    the real gather. The views are built once, so a frame costs three copy launches of host time."""

    def __init__(self, frame, world):
        import torch
        H = frame.shape[0]
        rest = tuple(frame.shape[1:])
        per = (H + world - 1) // world
        n = len(range(0, H, world))
        self.packed = torch.zeros((per,) + rest, dtype=frame.dtype, device=frame.device)
        self.allp = torch.zeros((world, per) + rest, dtype=frame.dtype, device=frame.device)
        self.src = torch.zeros_like(self.allp)
        self.full = torch.empty((per * world,) + rest, dtype=frame.dtype, device=frame.device)
        self.pack_dst, self.pack_src = self.packed[:n], frame[0::world]
        self.full_v, self.allp_t = self.full.view((per, world) + rest), self.allp.transpose(0, 1)

    def __call__(self):
        self.pack_dst.copy_(self.pack_src)
        self.allp.copy_(self.src)  # the gather's bytes landing in rank 0's receive buffer
        self.full_v.copy_(self.allp_t)


def load_pmc(kernel_prefix):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary (tools/collect_pmc.py) and the
    profile round it was measured in (the field is only valid while the kernels are unchanged)."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
        k = d.get(kernel_prefix)
        return (None if k is None else float(k["hbm_bytes_per_launch"])), d.get("_round")
    except Exception:
        return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--height", type=int, default=500)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--split", choices=["passes", "rows"], default="rows")
    ap.add_argument("--mode", type=int, default=0, help="RS_MODE_* (0 auto)")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-row-step", type=int, default=1)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = num_cpus + 1 like Painter::draw")
    ap.add_argument("--row-share", type=int, default=8,
                    help="at N = 1 also time rows 0::K of the frame (one rank's share at N = K) and report "
                         "the predicted strong-scaling efficiency T(full) / (K * T(share)); 0 = off")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from raysnail_amd import scenes
    from raysnail_amd.distributed import render_sharded

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    cam, scene_world, _, _ = scenes.rtow_13_1(args.width, args.height)
    photo = cam.take_photo().samples(args.spp).depth(args.depth).seed(args.seed).mode(args.mode)
    ds = scene_world.device_scene()  # BVH build + upload: outside the timed region
    ds.set_lanes(LANES)
    if FRAMES:
        ds.set_frames_in_flight(FRAMES)
    H, W = args.height, args.width
    frame = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    last = {}

    timed = {"on": False}
    n_eff = int(args.spp ** 0.5) ** 2

    def render(rb, re, rs, pass_index):
        st = photo.rows(rb, re, rs).pass_index(pass_index).settings()
        # asynchronous frames (rs_render_device without stats) in the timed region; the kernel
        # timing / byte statistics come from the same frames rendered with stats (synchronous) below
        stats = ds.render_device(cam.desc, st, frame.data_ptr(), torch.cuda.current_stream().cuda_stream,
                                 stats=timed["on"])
        if stats is not None:
            last["stats"] = stats
        rows = len(range(rb, re or H, rs))
        last["samples"] = last.get("samples", 0) + rows * W * n_eff
        return frame

    def step():
        return render_sharded(render, rank, world, args.split)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    last["samples"] = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    samples = last["samples"]
    # the frame latency: frames one at a time, each waited for (the timed region above is the pipelined
    # throughput of back-to-back asynchronous frames, rs_scene_set_frames_in_flight)
    lat = []
    for _ in range(min(args.steps, 5)):
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t2)
    latency_ms = sorted(lat)[len(lat) // 2] * 1e3
    # the dominant kernel's launches, event-timed (the events ride on the dispatches themselves), and
    # the library's byte / segment counts: the same K frames again with stats, synchronous and on ONE
    # wavefront lane, so that no launch shares the GPU with another lane's or frame's kernels
    # (concurrent launches would stretch every duration)
    ds.set_lanes(1)
    timed["on"] = True
    kern_ms = 0.0
    kern_launches = 0
    kern_bytes = 0
    segs = 0
    stat_samples = 0
    for _ in range(args.steps):
        step()
        st = last["stats"]
        kern_ms += st.kernel_ms
        kern_launches += st.kernel_launches
        kern_bytes += st.kernel_bytes
        segs += st.segments
        stat_samples += st.samples
    timed["on"] = False
    ds.set_lanes(LANES)
    if stat_samples != samples:
        log(f"warning: stats counted {stat_samples} samples, the timed loop {samples}")
    t = torch.tensor([dt], dtype=torch.float64, device="cuda")
    tot = torch.tensor([float(samples), float(segs)], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    dt = float(t.item())
    all_samples, all_segs = float(tot[0].item()), float(tot[1].item())

    share = None
    if world == 1 and args.row_share > 1:
        # one rank's work at N = K: the row lattice 0::K of the same frame (render_sharded's split)
        K = args.row_share
        ns = max(args.steps, 30)  # share frames are ~1 ms: more of them for a steadier clock
        # the share frames alone and with rank 0's gather work after each (distributed.gather_rows: pack copy,
        # the world's packed rows arriving -- a same-size device copy stands in for RCCL's writes --,
        # de-interleave), pipelined like the real job's: the gather of frame f overlaps frame f+1's path kernels.
        # The two loops alternate, 3 runs each, and each reports its median run: timed one after the other, the
        # second loop also paid for whatever state the first left (round 6 read 40-54 us of "gather" that way,
        # against 7 us for the three copies in a pipelined probe, profiles/r6/ab/gather_probe_r6d.txt)
        gather = GatherProxy(frame, K)

        def share_loop(with_gather):
            for _ in range(args.warmup):
                render(0, 0, K, 0)
                if with_gather:
                    gather()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(ns):
                render(0, 0, K, 0)
                if with_gather:
                    gather()
            torch.cuda.synchronize()
            return (time.perf_counter() - t1) / ns * 1e3

        runs = {False: [], True: []}
        for _ in range(3):
            for g in (False, True):
                runs[g].append(share_loop(g))
        sh_ms = sorted(runs[False])[1]
        shg_ms = sorted(runs[True])[1]
        ds.set_lanes(1)
        timed["on"] = True
        sh_launch_ms = 0.0
        for _ in range(ns):
            render(0, 0, K, 0)
            sh_launch_ms += last["stats"].kernel_ms
        timed["on"] = False
        ds.set_lanes(LANES)
        # the xGMI leg the proxy's device copy cannot show: each peer's packed rows over its own link into rank
        # 0 (links in parallel), at the per-link figure the task states (7 links x ~153 GB/s per GPU)
        per_rank_bytes = len(range(0, H, K)) * W * 16
        xgmi_ms = per_rank_bytes / 153e9 * 1e3
        full_ms = dt / args.steps * 1e3
        eff_g = full_ms / (K * (shg_ms + xgmi_ms))
        share = {"K": K, "rows": f"0::{K}", "ms_per_share": round(sh_ms, 4), "ms_full_frame": round(full_ms, 4),
                 "predicted_efficiency_no_gather": round(full_ms / (K * sh_ms), 4),
                 "ms_per_share_with_gather": round(shg_ms, 4), "gather_ms": round(shg_ms - sh_ms + xgmi_ms, 4),
                 "gather_model": "rank-0 pack + same-size device copy + de-interleave, measured pipelined; plus "
                                 f"{per_rank_bytes} B per peer over one xGMI link at 153 GB/s ({xgmi_ms:.4f} ms)",
                 "predicted_efficiency": round(eff_g, 4),
                 "predicted_speedup": round(K * eff_g, 3),
                 "runs_ms": [round(x, 4) for x in runs[False]],
                 "runs_with_gather_ms": [round(x, 4) for x in runs[True]],
                 "extend_ms_per_share": round(sh_launch_ms / ns, 4), "share_frames_timed": ns,
                 "samples_per_share": int(last["stats"].samples), "launches_per_share": int(last["stats"].launches)}

    if rank == 0:
        value = all_samples / dt / 1e6
        # roofline of the dominant kernel, rank 0's launches: algorithmic bytes per launch (library
        # model from the queue counts, DESIGN.md Roofline) / mean event-timed launch duration
        from raysnail_amd._abi import KERNEL_NAMES
        kname = KERNEL_NAMES.get(last["stats"].kernel_id)
        avg_launch_s = kern_ms / max(1, kern_launches) / 1e3
        bytes_per_launch = kern_bytes / max(1, kern_launches)
        traffic, traffic_round = load_pmc(kname) if kname else (None, None)
        # SURVEY 8(d)'s algorithmic bytes for the dominant kernel (the contract's `achieved`): the extend
        # reads a 28 B ray and writes a 16 B hit per segment, 44 B per world.hit call
        seg_per_launch = segs / max(1, kern_launches)
        alg = 44.0 * seg_per_launch
        achieved = alg / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "kernel": kname, "avg_launch_ms": round(avg_launch_s * 1e3, 4),
                "alg_bytes_per_launch": int(alg), "alg_model": "SURVEY 8(d): 44 B per segment (28 B ray in, 16 B hit out)",
                "segments_per_launch": int(seg_per_launch), "launches_per_step": kern_launches // args.steps,
                "kernel_share_of_step": round(kern_ms / args.steps / (dt / args.steps * 1e3), 4),
                "segments_per_sample": round(segs / max(1, samples), 4)}
        # the whole step against the same roofline: SURVEY 8(d)'s frame model over the pipelined step time
        fbytes = frame_model_bytes(all_segs, all_samples) / max(1, args.steps)
        roof["frame_model"] = "SURVEY 8(d): 212 B per segment + 124 B per sample, per step, over ms_per_step"
        roof["frame_bytes_per_step"] = int(fbytes)
        roof["achieved_frame"] = round(fbytes / (dt / args.steps) / 1e9, 2)
        roof["frac_frame"] = round(roof["achieved_frame"] / HBM_PEAK_GBS, 5)
        # the library's own f64 byte model of the same launches (rs_render_stats.kernel_bytes: the
        # 32-byte path records, hits, queue slots and radiance this kernel actually moves), secondary
        if avg_launch_s > 0:
            roof["achieved_lib"] = round(bytes_per_launch / avg_launch_s / 1e9, 2)
            roof["frac_lib"] = round(roof["achieved_lib"] / HBM_PEAK_GBS, 5)
            roof["lib_bytes_per_launch"] = int(bytes_per_launch)
        if traffic is not None:
            # PMC bytes per launch of this kernel from rocprofv3 --pmc passes of this same command
            # (tools/gpu.sh pmc -> profiles/pmc_summary.json)
            roof["traffic_profile"] = traffic_round
            roof["traffic_derivation"] = ("2 x FETCH_SIZE + WRITE_SIZE per launch: on gfx950 every L2 read request to "
                                          "the fabric (TCC_EA0_RDREQ) is 128 B and FETCH_SIZE counts 64 B of it, for "
                                          "coalesced 4-32 B/lane reads and 16 B gathers alike; WRITE_SIZE is exact for "
                                          "32 B/lane stores (calibrated on known byte counts: tools/micro/pmc_calib.hip, "
                                          "profiles/r4/calib); counts L2 misses served by the Infinity Cache as well")
            roof["traffic_over_alg"] = round(traffic / alg, 3) if alg else None
            roof["traffic_over_lib"] = round(traffic / bytes_per_launch, 3) if bytes_per_launch else None
        cpu = None
        if args.cpu_baseline and world == 1:
            log("timing CPU baseline (oracle restatement) ...")
            cpu = cpu_baseline(cam, scene_world, args.spp, args.depth, args.seed, args.cpu_row_step,
                               args.cpu_threads or host_cpus()[0] + 1)
        line = {
            "metric": "Msamples/s (whole node) + ms/frame, RTIOW-13.1 scene 800x500x64spp",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
            "frame_latency_ms": round(latency_ms, 4),
            "scaling": "weak" if args.split == "passes" else "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: RTIOW final scene regenerated from seed 7 (restated ChaCha12), per-sample RNG streams",
            "config": {"workload": f"rtow_13_1 balls_scene(seed 7)+light, {W}x{H}, {n_eff} spp, depth {args.depth}",
                       "width": W, "height": H, "spp": n_eff, "depth": args.depth, "split": args.split,
                       "lanes": LANES or "default", "frames_in_flight": FRAMES or "default",
                       "samples_per_frame": W * H * n_eff, "frames_per_step": world if args.split == "passes" else 1},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if share:
            line["row_share"] = share
        if cpu:
            line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
