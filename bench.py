#!/usr/bin/env python3
"""bench.py — tracked frames/sec of the 1080p x 128-object TBD loop on MI355X.

Workload (BASELINE.json configs[2]): one synthetic 1920x1080 sequence of
`warmup + steps` frames with 128 moving textured objects per GPU, rendered
into HBM before timing (tbdk_synth_render).  A "step" is one frame through the
full loop of libtbdk (tbdk_tbd_run over the timed frames: per frame the same
work as tbdk_tbd_step, with the next frame's pyramid and tracker-independent
PyrLK enqueued before the host tracker step): 3-level pyramid + Scharr planes, GFTT in
the boxes of new / re-detect tracks, sparse PyrLK (win 21) over every track's
corners, per-track similarity fit (KLT box propagation), and the native
cv::tbd::Tracker step on the frame's ground-truth detections.

Multi-GPU: one process per GPU (torchrun), one independent sequence per GPU
(seed + rank), no data-path collective; value = frames of all ranks / max
wall time over ranks ("scaling": "weak").

Prints ONE JSON line on rank 0 (contract in the task description), including
"roofline" for the dominant kernel (lk_sparse, VALU-bound -> TFLOP/s against
the 157.3 TF f32 peak) and "cpu_baseline" (the CPU oracle restatement of the
same per-frame KLT work, timed on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "tracked frames/sec, 1080p×128-object TBD loop @ 1/2/4/8 MI355X"
PEAK_F32_TFLOPS = 157.3      # MI355X_MICROARCH.md: peak FP32 (vector == f32 MFMA)
PEAK_HBM_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E peak (spec)


def lk_flops(points_levels: float, iters: float, win: int) -> float:
    """per point per level 441*30 (I / dI bilinear + G) plus,
    per Newton iteration, 441*13 (J bilinear, diff, 2 FMA) for win 21."""
    area = win * win
    return points_levels * area * 30.0 + iters * area * 13.0


def pyr_bytes(w: int, h: int, nlevels: int) -> int:
    """B_pyr = sum_{L<n-1} (|L| + |L+1|) for the new frame."""
    sizes = []
    for _ in range(nlevels):
        sizes.append(w * h)
        w, h = (w + 1) // 2, (h + 1) // 2
    return sum(sizes[i] + sizes[i + 1] for i in range(nlevels - 1))


def max_over_ranks(value: float, world: int, device=None) -> float:
    """Max of a per-rank wall time over all ranks (the contract's job time).
    Collective only when world > 1; the tensor lives on `device` (cuda for
    RCCL, cpu for gloo)."""
    if world <= 1:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def replica_throughput(steps: int, world: int, max_elapsed: float) -> float:
    """Whole-job frames/s: every rank runs its own sequence of `steps` frames
    (replicas, weak scaling), all finished within the max-over-ranks time."""
    return steps * world / max_elapsed


def pmc_traffic(kernel_substr: str):
    """HBM bytes per launch of a kernel from the newest committed PMC summary
    (profiles/rNN_pmc.json: FETCH_SIZE x2 + WRITE_SIZE, separate --pmc passes,
    see tools/profile_round.sh).  None when no summary covers the kernel."""
    d = os.path.join(ROOT, "profiles")
    try:
        files = sorted(f for f in os.listdir(d) if f.endswith("_pmc.json"))
    except OSError:
        return None, None
    for f in reversed(files):
        k = json.load(open(os.path.join(d, f)))["kernels"]
        for name, v in k.items():
            if kernel_substr in name and v.get("fetch_bytes") is not None and v.get("write_bytes") is not None:
                return v["fetch_bytes"] + v["write_bytes"], f
    return None, None


def cpu_baseline(frames_host, gt, args, seconds: float):
    """The oracle (CPU restatement of the reference path) running the same
    per-frame KLT work: pyramid, GFTT in every box every `redetect` frames
    (single-threaded, as the reference's goodFeaturesToTrack), multithreaded
    LK over the tracked corners (the reference's parallel_for_ over points).
    The host tracker step (~1 ms, identical code on both sides) is excluded."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import _oracle as O

    threads = min(16, os.cpu_count() or 1)
    pts = None
    prev = None
    done = 0
    t0 = time.perf_counter()
    n = frames_host.shape[0]
    for f in range(n):
        img = frames_host[f]
        P = O.Pyramid(img, (args.win, args.win), args.max_level)
        if prev is not None and pts is not None and len(pts):
            nxt, st, _, _ = O.lk(prev, P, pts, (args.win, args.win), args.max_level, 30, 0.01, 0, 1e-4,
                                 O.ACCUM_SSE2, threads)
            pts = nxt[st == 1]
        if f % args.redetect == 0 or pts is None:
            rois = [tuple(int(v) for v in g[1:]) for g in gt[f] if g[0]]
            got = O.gftt_rois(img, rois, 256, 0.01, 3.0)
            pts = np.concatenate(got).astype(np.float32) if got else np.zeros((0, 2), np.float32)
        prev = P
        done += 1
        if time.perf_counter() - t0 > seconds and done >= 3:
            break
    el = time.perf_counter() - t0
    return {"value": done / el, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"first {done} frames of the rank-0 sequence, {args.width}x{args.height}x{args.objects} "
                      f"objects: oracle pyramid + GFTT(256/box, every {args.redetect} frames, 1 thread) + "
                      f"PyrLK win {args.win} SSE2-order ({threads} threads); tracker step excluded"}


FB_ITER_BYTES_PER_PX = 56  # fb_iter algorithmic bytes per pixel: flow 8 + R0 20 + R1 20 in, flow 8 out


def farneback_secondary(ctx, args, device, cpu: bool):
    """BASELINE configs[4]'s dense Farneback variant on a synthetic 4K pair
    sequence (3840x2160, 512 objects): frame pairs/s through tbdk_farneback
    (cv::cuda::FarnebackOpticalFlow defaults), the fb_iter kernel's HBM
    roofline, and the CPU oracle on one pair.  Reported, never `value`."""
    import torch
    from opencv_amd import farneback as F
    from opencv_amd import klt

    w, h, n = args.fb_width, args.fb_height, args.fb_pairs
    frames, _ = klt.synth_render(args.seed + 7, w, h, args.fb_objects, 0, n + 3, device=device, ctx=ctx)
    fb = F.FarnebackOpticalFlow.create(ctx=ctx)
    flow = torch.empty((h, w, 2), dtype=torch.float32, device=frames.device)
    for i in range(2):
        fb.calc(frames[i], frames[i + 1], flow)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        fb.calc(frames[i], frames[i + 1], flow)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ctx.timing_select(["fb_iter", "fb_pyr", "fb_polyexp", "fb_flow_init"])
    ctx.timing_enable(True)
    for i in range(n):
        fb.calc(frames[i], frames[i + 1], flow)
    torch.cuda.synchronize()
    kern = {}
    for name in ("fb_iter", "fb_pyr", "fb_polyexp", "fb_flow_init"):
        c, ms = ctx.timing_query(name)
        kern[name] = {"launches": c, "avg_us": (ms / c * 1000.0) if c else None, "ms_per_pair": ms / n}
    ctx.timing_enable(False)
    ctx.timing_select(None)
    levels = fb.levels(w, h)
    it_bytes = FB_ITER_BYTES_PER_PX * sum(a * b for a, b in levels) * fb.getNumIters() * n
    gbs = it_bytes / (kern["fb_iter"]["ms_per_pair"] * n * 1e-3) / 1e9 if kern["fb_iter"]["launches"] else 0.0
    # PMC bytes per fb_iter launch (the committed summary's mean over a pair's
    # launches, all levels) x launches per pair -> HBM bytes per pair
    per_launch, traffic_src = pmc_traffic("fb_iter_kernel<6, false>")
    launches_per_pair = kern["fb_iter"]["launches"] / n
    traffic = per_launch * launches_per_pair if per_launch is not None else None
    alg_pair = it_bytes / n
    out = {"value": round(n / wall, 2), "unit": "pairs/s", "ms_per_pair": round(1000 * wall / n, 3),
           "config": {"workload": f"Farneback {w}x{h} x {args.fb_objects} objects (BASELINE configs[4] dense "
                                  "variant, u8 pixels)", "params": "cv::cuda::FarnebackOpticalFlow defaults: "
                                  "5 levels, pyrScale 0.5, winSize 13, 10 iters, polyN 5, sigma 1.1, box blur",
                      "levels": [list(l) for l in levels], "pairs": n},
           "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                        "kernel": "fb_iter", "bytes_per_px": FB_ITER_BYTES_PER_PX,
                        "algorithmic_bytes_per_pair": alg_pair, "traffic_unit": "bytes per pair (all fb_iter launches)",
                        "note": "achieved = algorithmic bytes of every level's 10 launches / summed fb_iter time "
                                "(HIP events on the launch stream)"},
           "kernels": kern}
    if cpu:
        import importlib
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests"))
        O = importlib.import_module("_oracle")
        a_, b_ = frames[0].cpu().numpy(), frames[1].cpu().numpy()
        t1 = time.perf_counter()
        O.farneback(a_, b_)
        dt = time.perf_counter() - t1
        out["cpu_baseline"] = {"value": round(1.0 / dt, 4), "unit": "pairs/s", "cores": 1, "kind": "port",
                               "sample": f"one {w}x{h} pair through oracle/farneback_oracle.c (the reference's "
                                         "calcOpticalFlowFarneback restated, running-sum box blur), 1 thread"}
    del frames
    return out


def pyr_f16_bytes(w: int, h: int, nlevels: int) -> int:
    """Algorithmic HBM bytes of one fp16 pyramid build from a u8 frame: frame
    read (1 B/px) and level 0 written (2 B/px); per further level the previous
    level read and the level written (2 B/px each); per level its fp16 (Ix, Iy)
    plane written (4 B/px) from the level read (2 B/px)."""
    sizes = []
    for _ in range(nlevels):
        sizes.append(w * h)
        w, h = (w + 1) // 2, (h + 1) // 2
    b = sizes[0] * 3 + sum(2 * sizes[i - 1] + 2 * sizes[i] for i in range(1, nlevels))
    return b + sum(6 * s for s in sizes)


def lk_f16_secondary(ctx, args, device, cpu: bool):
    """BASELINE configs[4]'s fp16 pixel path: synthetic 4K pairs (3840x2160,
    512 objects x 256 points), per pair the next frame's fp16 pyramid (3 levels,
    Scharr planes; the previous pyramid is reused) and sparse PyrLK (win 21) of
    every point on the fp16 levels (tbdk_lk_sparse on TBDK_DEPTH_16F pyramids).
    Pairs/s, the LK VALU roofline and the pyramid's HBM roofline, and the fp16
    oracle on a bounded sample.  Reported, never `value`."""
    import numpy as np
    import torch
    from opencv_amd import klt

    w, h, n, per_box = args.fb_width, args.fb_height, args.f16_pairs, 256
    win, ml = (args.win, args.win), args.max_level
    frames, gt = klt.synth_render(args.seed + 13, w, h, args.fb_objects, 0, n + 1, device=device, ctx=ctx)
    rng = np.random.default_rng(args.seed)
    pts_h = np.concatenate([np.stack([rng.uniform(x, x + bw, per_box), rng.uniform(y, y + bh, per_box)], 1)
                            for v, x, y, bw, bh in gt[0].numpy() if v]).astype(np.float32)
    pts = torch.from_numpy(pts_h).to(frames.device)
    pyrs = [klt.Pyramid(ctx, w, h, ml, win, torch.float16) for _ in range(2)]
    lk = klt.SparsePyrLKOpticalFlow(win, ml, 30)

    def run(timing: bool):
        pyrs[0].build(frames[0])
        its = 0
        for i in range(n):
            pyrs[(i + 1) % 2].build(frames[i + 1])
            r = lk.calc(pyrs[i % 2], pyrs[(i + 1) % 2], pts, want_err=True, want_iters=timing)
            if timing:
                its += int(r.iters.sum().item())
        return its

    run(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(False)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ctx.timing_select(["pyr_build", "lk_sparse"])
    ctx.timing_enable(True)
    iters = run(True)
    torch.cuda.synchronize()
    kern = {}
    for name in ("pyr_build", "lk_sparse"):
        c, ms = ctx.timing_query(name)
        kern[name] = {"launches": c, "avg_us": (ms / c * 1000.0) if c else None}
    ctx.timing_enable(False)
    ctx.timing_select(None)
    nlev = pyrs[0].nlevels
    npts = len(pts_h)
    lkk, pk = kern["lk_sparse"], kern["pyr_build"]
    flops = lk_flops(npts * nlev, iters / n, args.win)  # per launch (one pair)
    tf = flops / (lkk["avg_us"] * 1e-6) / 1e12
    pb = pyr_f16_bytes(w, h, nlev)
    gbs = pb / (pk["avg_us"] * 1e-6) / 1e9
    out = {"value": round(n / wall, 2), "unit": "pairs/s", "points_per_s": round(n * npts / wall, 1),
           "ms_per_pair": round(1000 * wall / n, 3), "dtype": "f16 pixels, f32 arithmetic",
           "config": {"workload": f"sparse PyrLK {w}x{h}, {args.fb_objects} objects x {per_box} points "
                                  "(BASELINE configs[4] fp16 pixel path)", "points": npts, "levels": nlev,
                      "win": args.win, "pairs": n, "mean_iters_per_point": iters / n / npts},
           "roofline": {"bound": "mfma", "achieved": round(tf, 3), "peak": PEAK_F32_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(tf / PEAK_F32_TFLOPS, 4), "traffic": None, "kernel": "lk_sparse (lk_f16_kernel)",
                        "flops_per_launch": flops,
                        "note": "VALU-bound (fp32 FMA on fp16 taps, no MFMA); algorithmic flops per SURVEY.md §8(d)"},
           "roofline_pyramid": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                "frac": round(gbs / PEAK_HBM_GBS, 4), "bytes_per_launch": pb,
                                "kernel": "pyr_build (fp16 levels + fp16 Scharr planes)"},
           "kernels": kern}
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as O
        a_, b_ = frames[0].cpu().numpy(), frames[1].cpu().numpy()
        threads = min(16, os.cpu_count() or 1)
        sample = pts_h[:: max(1, npts // 8192)]
        t1 = time.perf_counter()
        R0, R1 = O.Pyramid16(a_, win, ml), O.Pyramid16(b_, win, ml)
        tp = (time.perf_counter() - t1) / 2
        t1 = time.perf_counter()
        O.lk16(R0, R1, sample, win, ml, nthreads=threads)
        tl = (time.perf_counter() - t1) * npts / len(sample)
        out["cpu_baseline"] = {"value": round(1.0 / (tp + tl), 4), "unit": "pairs/s", "cores": threads,
                               "kind": "port",
                               "sample": f"oracle/klt16_oracle.c: one fp16 pyramid (1 thread) + LK of {len(sample)} of "
                                         f"the {npts} points ({threads} threads), LK time scaled to all points"}
    del frames, pyrs
    return out


def hog_secondary(ctx, args, device, cpu: bool):
    """The sample's detection step in GPU mode (samples/gpu/tbd.cpp:384-443,
    596-606): cv::cuda::HOG 48x96 people detector, 15 levels, scale 1.05, hit
    threshold 0.45, win stride 8, group threshold 2, on BGRA frames: frames/s of
    detectMultiScale through tbdk_hog_detect_multiscale (device levels, host
    grouping, synchronous), per-kernel times, and the CPU oracle on one frame.
    Reported, never `value`."""
    import torch
    from opencv_amd import hog as H
    from opencv_amd import klt

    w, h, n = args.hog_width, args.hog_height, args.hog_frames
    gray, _ = klt.synth_render(args.seed + 11, w, h, args.objects, 0, n, device=device, ctx=ctx)
    frames = torch.stack([gray, gray.flip(2), gray.flip(1), torch.full_like(gray, 255)], 3).contiguous()
    hg = H.HOG.create((48, 96), ctx=ctx)
    hg.setSVMDetector(hg.getDefaultPeopleDetector())
    hg.setNumLevels(15)
    hg.setHitThreshold(0.45)
    found = [len(hg.detectMultiScale(frames[i])) for i in range(min(2, n))]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        hg.detectMultiScale(frames[i])
    wall = time.perf_counter() - t0
    names = ["hog_resize", "hog_grad", "hog_block", "hog_window"]
    ctx.timing_select(names)
    ctx.timing_enable(True)
    for i in range(n):
        hg.detectMultiScale(frames[i])
    kern = {}
    for name in names:
        c, ms = ctx.timing_query(name)
        kern[name] = {"launches": c, "avg_us": (ms / c * 1000.0) if c else None, "ms_per_frame": ms / n}
    ctx.timing_enable(False)
    ctx.timing_select(None)
    out = {"value": round(n / wall, 2), "unit": "frames/s", "ms_per_frame": round(1000 * wall / n, 3),
           "config": {"workload": f"HOG detectMultiScale {w}x{h} BGRA synthetic frames ({args.objects} objects)",
                      "params": "48x96 people detector, nlevels 15, scale 1.05, hit 0.45, win stride 8x8, "
                                "group threshold 2 (the sample's GPU-mode settings)",
                      "detections_first_frames": found, "frames": n},
           "kernels": kern,
           "note": "wall time includes the per-call detector upload, the hit download and host grouping"}
    if cpu:
        import importlib
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests"))
        O = importlib.import_module("_oracle")
        img = frames[0, ..., :3].cpu().numpy()
        t1 = time.perf_counter()
        O.hog_detect_multiscale(img, O.hog_params(win=(48, 96)), hg.svm, hit_threshold=0.45, nlevels=15)
        dt = time.perf_counter() - t1
        out["cpu_baseline"] = {"value": round(1.0 / dt, 4), "unit": "frames/s", "cores": 1, "kind": "port",
                               "sample": f"one {w}x{h} BGR frame through oracle/hog_oracle.c (the reference's "
                                         "HOGDescriptor::detectMultiScale restated), 1 thread"}
    del frames, gray
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=480)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--objects", type=int, default=128)
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--win", type=int, default=21)
    ap.add_argument("--max-level", type=int, default=2)
    ap.add_argument("--redetect", type=int, default=5)
    ap.add_argument("--bounds", choices=["reference", "frame"], default="reference",
                    help="reference: the tracker's hard-coded 1280x720 filter (tbd.cpp:218); frame: W x H")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--api", choices=["run", "ahead", "step"], default="run",
                    help="run: tbdk_tbd_run (native frame loop with look-ahead); ahead: per-frame "
                         "tbdk_tbd_step_ahead; step: per-frame tbdk_tbd_step (no look-ahead)")
    ap.add_argument("--lk-impl", type=int, default=0, help="PyrLK kernel (ctx option lk_impl; 0 auto)")
    ap.add_argument("--early-gftt", type=int, default=2, choices=[0, 1, 2],
                    help="ctx option tbd_early_gftt (A/B runs; 0 off, 1 new tracks, 2 + re-detection boxes)")
    ap.add_argument("--no-spec-lookahead", action="store_true", help="ctx option tbd_spec_lookahead = 0 (A/B runs)")
    ap.add_argument("--no-zero-copy", action="store_true", help="ctx option tbd_zero_copy = 0 (A/B runs)")
    ap.add_argument("--timing-every", type=int, default=5,
                    help="HIP events on every Nth launch of the timed kernels in the timed region")
    ap.add_argument("--kstats", default="lk_sparse",
                    help="kernels timed with HIP events in the timed region (comma list, 'all' or 'none'); "
                         "each timed launch adds two event records to the frame's host work.  The other "
                         "kernels are timed in a separate pass over the same frames (not `value`)")
    ap.add_argument("--no-step-api", action="store_true", help="skip the secondary per-frame tbdk_tbd_step pass")
    ap.add_argument("--no-farneback", action="store_true", help="skip the secondary dense Farneback measurement")
    ap.add_argument("--fb-width", type=int, default=3840)
    ap.add_argument("--fb-height", type=int, default=2160)
    ap.add_argument("--fb-objects", type=int, default=512)
    ap.add_argument("--fb-pairs", type=int, default=10)
    ap.add_argument("--no-f16", action="store_true", help="skip the secondary fp16 pixel path measurement")
    ap.add_argument("--f16-pairs", type=int, default=10)
    ap.add_argument("--no-hog", action="store_true", help="skip the secondary HOG detector measurement")
    ap.add_argument("--hog-width", type=int, default=1920)
    ap.add_argument("--hog-height", type=int, default=1080)
    ap.add_argument("--hog-frames", type=int, default=60)
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    from opencv_amd import klt, tbd

    ctx = klt.Context.get(dev)
    if args.lk_impl:
        ctx.set_option("lk_impl", args.lk_impl)
    ctx.set_option("tbd_early_gftt", args.early_gftt)
    ctx.set_option("tbd_spec_lookahead", 0 if args.no_spec_lookahead else 1)
    ctx.set_option("tbd_zero_copy", 0 if args.no_zero_copy else 1)
    nframes = args.warmup + args.steps
    frames, gt = klt.synth_render(args.seed + rank, args.width, args.height, args.objects, 0, nframes,
                                  device=dev, ctx=ctx)
    gtn = gt.numpy()
    dets = [tbd.detections_from_gt(gtn[f]) for f in range(nframes)]
    over = {}
    if args.bounds == "frame":
        over = dict(bounds_xmax=args.width, bounds_ymax=args.height)
    cfg = tbd.default_config(args.width, args.height, win=args.win, max_level=args.max_level,
                             redetect_every=args.redetect, **over)
    loop = tbd.TbdLoop(cfg, ctx=ctx)
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()

    for f in range(args.warmup):
        loop.step(frames[f], f, dets[f], stream)
    frame_list = [frames[f] for f in range(args.warmup, nframes)]
    packed = tbd.TbdLoop.pack_detections(dets[args.warmup:])  # host detections staged like the frames

    timed = ["pyr_build", "lk_sparse", "gftt", "tbd_fit"] if args.kstats == "all" else \
        [] if args.kstats == "none" else [k for k in args.kstats.split(",") if k]
    ctx.timing_select(timed or None)
    # events on every 5th timed launch: each timed launch costs two event records of
    # host work on the frame's critical path (~5 % of the frame when every launch is
    # timed); 5 is odd, so a frame's alternating launch kinds are sampled alike
    ctx.set_option("timing_every", args.timing_every)
    ctx.timing_enable(bool(timed))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if args.api == "run":
        ms = loop.run(frame_list, args.warmup, None, stream, packed=packed)
    else:
        ms = []
        for f in range(args.warmup, nframes):
            nxt = frames[f + 1] if args.api == "ahead" and f + 1 < nframes else None
            ms.append(loop.step(frames[f], f, dets[f], stream, next_frame=nxt))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    el = max_over_ranks(el, world, device="cuda")
    lk_pts = lk_it = klt_pts = ntr = redet = early = 0
    h_wait = h_trk = h_step = h_launch = 0.0
    for m in ms:
        lk_pts += m.lk_points
        lk_it += m.lk_iters
        klt_pts += m.klt_points
        ntr += m.ntracks
        redet += m.redetected
        early += m.early_gftt
        h_wait += m.host_wait_us
        h_trk += m.host_tracker_us
        h_step += m.host_step_us
        h_launch += m.host_launch_us

    kstats = {}
    for name in timed:
        c, ms = ctx.timing_query(name)
        kstats[name] = {"launches": ctx.timing_calls(name), "timed_launches": c,
                        "avg_us": (ms / c * 1000.0) if c else None, "total_ms_timed": ms}
    ctx.timing_enable(False)
    ctx.timing_select(None)
    ctx.set_option("timing_every", 1)
    nolaunch = {"launches": 0, "avg_us": None, "total_ms": 0.0}

    # secondary: the same frames through the per-frame tbdk_tbd_step API (no
    # look-ahead), a fresh loop, no timing events; reported, never `value`
    step_api = None
    if args.api != "step" and not args.no_step_api:
        loop2 = tbd.TbdLoop(cfg, ctx=ctx)
        for f in range(args.warmup):
            loop2.step(frames[f], f, dets[f], stream)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for f in range(args.warmup, nframes):
            loop2.step(frames[f], f, dets[f], stream)
        torch.cuda.synchronize()
        el2 = max_over_ranks(time.perf_counter() - t1, world, device="cuda")
        step_api = {"value": round(replica_throughput(args.steps, world, el2), 2), "unit": "frames/s",
                    "api": "tbdk_tbd_step per frame from Python"}
        del loop2

    # the kernels not timed in the timed region: a separate pass over the same
    # frames with events on them (a fresh loop; its wall time is not reported)
    rest = [k for k in ("pyr_build", "lk_sparse", "gftt", "tbd_fit") if k not in timed]
    kstats_aside = {}
    if rest:
        loop3 = tbd.TbdLoop(cfg, ctx=ctx)
        for f in range(args.warmup):
            loop3.step(frames[f], f, dets[f], stream)
        ctx.timing_select(rest)
        ctx.timing_enable(True)
        loop3.run(frame_list, args.warmup, None, stream, packed=packed)
        torch.cuda.synchronize()
        for name in rest:
            c, ms = ctx.timing_query(name)
            kstats_aside[name] = {"launches": c, "avg_us": (ms / c * 1000.0) if c else None, "total_ms": ms}
        ctx.timing_enable(False)
        ctx.timing_select(None)
        del loop3

    lk = kstats.get("lk_sparse", nolaunch)
    nlev = args.max_level + 1
    if lk["launches"]:
        flops_per_launch = lk_flops(lk_pts * nlev, lk_it, args.win) / lk["launches"]
        achieved = flops_per_launch / (lk["avg_us"] * 1e-6) / 1e12
    else:
        flops_per_launch, achieved = 0.0, 0.0
    # the auto choice is lk_multi_kernel (several points per wave) for the odd square windows it covers
    traffic, traffic_src = pmc_traffic(f"lk_multi_kernel<{args.win}, {args.win}>")
    if traffic is None:
        traffic, traffic_src = pmc_traffic(f"lk_strip_kernel<{args.win}, {args.win}>")
    roofline = {"bound": "mfma", "achieved": round(achieved, 3), "peak": PEAK_F32_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_F32_TFLOPS, 4), "traffic": traffic, "kernel": "lk_sparse",
                "traffic_source": traffic_src,
                "note": "PyrLK is VALU (int16 dot2 + fp32) bound, no MFMA use; peak = fp32 vector rate; "
                        "algorithmic flops per SURVEY.md §8(d) with the measured iteration count; "
                        f"launch duration = HIP events on every {args.timing_every}th launch of the timed region",
                "flops_per_launch": flops_per_launch,
                "mean_points_per_launch": lk_pts / max(1, lk["launches"]),
                "mean_iters_per_point": lk_it / max(1, lk_pts)}
    pb = pyr_bytes(args.width, args.height, nlev)
    pyr = kstats.get("pyr_build", kstats_aside.get("pyr_build", nolaunch))
    pyr_gbs = pb / (pyr["avg_us"] * 1e-6) / 1e9 if pyr["launches"] else 0.0
    roof_pyr = {"bound": "hbm", "achieved": round(pyr_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(pyr_gbs / PEAK_HBM_GBS, 4), "bytes_per_launch": pb, "kernel": "pyr_build"}
    # north_star's "HBM-read roofline on pyramid+PyrLK": SURVEY §8d bytes B_pyr + B_lk + N*21,
    # with B_lk at its upper bound (2 full pyramids), over the two stages' summed time
    w_, h_, lv_bytes = args.width, args.height, 0
    for _ in range(nlev):
        lv_bytes += w_ * h_
        w_, h_ = (w_ + 1) // 2, (h_ + 1) // 2
    b_lk = 2 * lv_bytes + 21 * (lk_pts / max(1, args.steps))
    t_pl = ((pyr["avg_us"] or 0.0) + (lk["avg_us"] or 0.0)) * 1e-6
    hbm_pl = (pb + b_lk) / t_pl / 1e9 if t_pl > 0 else 0.0
    roof_pl = {"bound": "hbm", "achieved": round(hbm_pl, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
               "frac": round(hbm_pl / PEAK_HBM_GBS, 4), "bytes_per_frame": pb + b_lk,
               "kernels": "pyr_build + lk_sparse",
               "note": "B_lk taken at its SURVEY §8d upper bound (2 full pyramids); PyrLK is compute-bound "
                       "(~360 flop/B vs ridge ~20), so this fraction is structurally small (DESIGN.md §3)"}


    out = {
        "metric": METRIC,
        "value": round(replica_throughput(args.steps, world, el), 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1000.0, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (deterministic in-repo generator, opencv_amd/csrc/synth_spec.h)",
        "config": {"workload": f"TBD loop {args.width}x{args.height} x {args.objects} objects "
                               f"(BASELINE configs[2]), {nframes}-frame sequence per GPU",
                   "levels": nlev, "win": args.win, "gftt": f"256/box, q 0.01, minDist 3, every {args.redetect}",
                   "tracker_bounds": args.bounds, "parallelism": f"replicas x{world} (one sequence per GPU)",
                   "api": {"run": "tbdk_tbd_run (native frame loop, look-ahead)",
                           "ahead": "tbdk_tbd_step_ahead per frame", "step": "tbdk_tbd_step per frame"}[args.api]},
        "step_api": step_api,
        "roofline": roofline,
        "roofline_pyramid": roof_pyr,
        "roofline_hbm_pyr_lk": roof_pl,
        "kernels": kstats,
        "kernels_aside": kstats_aside,
        "per_frame": {"lk_points": lk_pts / args.steps, "tracked_points": klt_pts / args.steps,
                      "tracks": ntr / args.steps, "gftt_rois": redet / args.steps,
                      "gftt_rois_early": early / args.steps,
                      "host_wait_us": h_wait / args.steps, "host_tracker_us": h_trk / args.steps,
                      "host_step_us": h_step / args.steps, "host_launch_us": h_launch / args.steps},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        nb = min(nframes, 40)
        out["cpu_baseline"] = cpu_baseline(frames[:nb].cpu().numpy(), gtn[:nb], args, args.cpu_baseline_seconds)
    else:
        out["cpu_baseline"] = None
    if rank == 0 and not args.no_farneback:
        del frames, frame_list
        out["farneback"] = farneback_secondary(ctx, args, dev, cpu=world == 1 and not args.no_cpu_baseline)
    if rank == 0 and not args.no_f16:
        out["lk_f16"] = lk_f16_secondary(ctx, args, dev, cpu=world == 1 and not args.no_cpu_baseline)
    if rank == 0 and not args.no_hog:
        out["hog"] = hog_secondary(ctx, args, dev, cpu=world == 1 and not args.no_cpu_baseline)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
