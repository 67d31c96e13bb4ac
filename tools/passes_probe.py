"""Time rs_render_device_passes (K passes as one sample stream) against K pipelined rs_render_device frames on the
bench frame and on its N = 8 row share (rows 0::8), and check the streamed passes against the one-call frames.

usage: python tools/passes_probe.py [--k 30] [--reps 3] [--lib path/to/libraysnail_hip.so]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=30)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--height", type=int, default=500)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--lanes", default="1,2,3,4", help="wavefront lanes of the streamed passes")
    ap.add_argument("--row-steps", default="1,8", help="frames: rows 0::k of the frame (k = 8: one rank's share at N = 8)")
    args = ap.parse_args()
    args.lanes = [int(x) for x in args.lanes.split(",")]
    import numpy as np
    import torch
    from raysnail_amd import scenes
    torch.cuda.set_device(0)
    cam, world, _, _ = scenes.rtow_13_1(args.width, args.height)
    ds = world.device_scene()
    H, W = args.height, args.width
    s = torch.cuda.current_stream().cuda_stream
    bufs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(args.k)]
    photo = cam.take_photo().samples(args.spp).depth(args.depth).seed(1)
    K = args.k
    for label, rows in [(f"rows::{k}", (0, 0, k)) for k in map(int, args.row_steps.split(","))]:
        def singles():
            for k in range(K):
                ds.render_device(cam.desc, photo.rows(*rows).pass_index(k).settings(), bufs[k].data_ptr(), s,
                                 stats=False)

        def stream():
            ds.render_device_passes(cam.desc, photo.rows(*rows).pass_index(0).settings(),
                                    [bufs[k].data_ptr() for k in range(K)], s, stats=False)
        def stream_slots():
            # the passes in three calls of K / 3 (asynchronous: each call a frame slot of its own, the three streams
            # concurrent)
            n3 = K // 3
            for j in range(3):
                ds.render_device_passes(cam.desc, photo.rows(*rows).pass_index(j * n3).settings(),
                                        [bufs[j * n3 + k].data_ptr() for k in range(n3)], s, stats=False)
        res = {"frame": f"{W}x{H}x{args.spp} {label}", "K": K}

        def lanes(n, fn):
            def run():
                ds.set_lanes(n)
                fn()
            return run
        for name, fn in [("single_calls", lanes(0, singles))] + [(f"passes_stream_l{n}", lanes(n, stream))
                                                                  for n in args.lanes] + \
                [("passes_stream_3calls", lanes(1, stream_slots))]:
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) / K * 1e3)
            res[name + "_ms_per_frame"] = [round(t, 4) for t in ts]
            res[name + "_median"] = round(sorted(ts)[len(ts) // 2], 4)
        # the last three streamed passes against one-call frames of the same passes (the lattice rows)
        ds.set_lanes(args.lanes[-1])
        stream()
        torch.cuda.synchronize()
        got = {k: bufs[k].cpu().numpy().copy() for k in range(K - 3, K)}
        ok = True
        for k in range(K - 3, K):
            ref = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
            ds.render_device(cam.desc, photo.rows(*rows).pass_index(k).settings(), ref.data_ptr(), s)
            ok &= bool(np.array_equal(got[k][rows[0]::rows[2]], ref.cpu().numpy()[rows[0]::rows[2]]))
        res["bit_identical_last3"] = ok
        st = ds.render_device_passes(cam.desc, photo.rows(*rows).pass_index(0).settings(),
                                     [bufs[k].data_ptr() for k in range(K)], s)
        res["stream_launches"] = int(st.launches)
        res["stream_kernel_launches"] = int(st.kernel_launches)
        res["stream_samples"] = int(st.samples)
        res["stream_timed_ms_per_frame"] = round(st.ms / K, 4)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
