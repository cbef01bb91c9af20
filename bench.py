#!/usr/bin/env python3
"""bench.py — tracked frames/sec of the 1080p x 128-object TBD loop on MI355X.

Workload (BASELINE.json configs[2]): one synthetic 1920x1080 sequence of 500
frames (or warmup + steps, if more) with 128 moving textured objects per GPU,
rendered into HBM before timing (tbdk_synth_render).  A "step" is one frame
through the full loop of libtbdk: frames [0, warmup) go through tbdk_tbd_step
untimed, frames [warmup, warmup + steps) through tbdk_tbd_run (per frame the
same work as tbdk_tbd_step, with the next frame's pyramid and the
tracker-independent PyrLK enqueued before the host tracker step): 3-level
pyramid + Scharr planes, GFTT in the boxes of new / re-detect tracks, sparse
PyrLK (win 21) over every track's corners, per-track similarity fit (KLT box
propagation), and the native cv::tbd::Tracker step on the frame's
ground-truth detections.

Secondary objects (never `value`): the whole sequence in steady state, median
of 5 runs (`sequence`); the same frames uploaded from pinned host memory
(`with_h2d`); KITTI-shaped configs[3] (`kitti`); per-frame API (`step_api`);
dense Farneback and the fp16 pixel path (configs[4]); the HOG detector.

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


def pyr_build_bytes(w: int, h: int, nlevels: int, pad: int = 32, copy_l0: bool = True) -> int:
    """The bytes a levels-only build must move: the frame read once, every
    padded level written (reflect-101 frame included), and each level from 2 on
    reading its interior predecessor (level 1 is made from the frame itself).
    copy_l0 False: the TBD loop's build inside tbdk_tbd_run since round 6 (ctx
    option tbd_borrow_l0), where level 0 is the frame itself and no padded copy
    is written.  B_pyr above leaves out the padded level-0 copy as well."""
    sizes, padded = [], []
    for _ in range(nlevels):
        sizes.append(w * h)
        padded.append((w + 2 * pad) * (h + 2 * pad))
        w, h = (w + 1) // 2, (h + 1) // 2
    return sizes[0] + sum(padded[0 if copy_l0 else 1:]) + sum(sizes[1:nlevels - 1])


def max_over_ranks(value: float, world: int, device=None) -> float:
    """Max of a per-rank wall time over all ranks (the contract's job time).
    Collective only when world > 1; the tensor lives on `device` (cpu: the
    bench's group is gloo, see main())."""
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


def _pmc_summaries(suffix: str):
    d = os.path.join(ROOT, "profiles")
    try:
        return d, sorted(f for f in os.listdir(d) if f.endswith(suffix))
    except OSError:
        return d, []


def pmc_traffic(kernel_substr: str, suffix: str = "_pmc_loop.json"):
    """HBM bytes per launch of a kernel from the newest committed PMC summary
    (separate --pmc passes, tools/profile_round.sh): FETCH_SIZE + WRITE_SIZE as
    counted.  The loop's kernels read profiles/rNN_pmc_loop.json, whose passes
    run only the contract's legs (bench.py --no-secondary: the 1080p x 128 loop),
    so no other configuration's launches of the same kernel (the 4K pyramid leg,
    the bounds-at-frame leg) enter the means; the secondaries' kernels read
    rNN_pmc.json (suffix).  The guide's x2 applies to wide (16 B per lane)
    streaming reads; these kernels load 4 B per lane (or less), and the
    pyramid's counts match its known read / write sets without it (DESIGN.md
    §7).  None when no summary covers the kernel."""
    d, files = _pmc_summaries(suffix)
    for f in reversed(files):
        k = json.load(open(os.path.join(d, f)))["kernels"]
        for name, v in k.items():
            if kernel_substr in name and v.get("fetch_bytes") is not None and v.get("write_bytes") is not None:
                return v["fetch_size_kib"] * 1024 + v["write_bytes"], f
    return None, None


def ktrace_loop_avg_us(kernel: str):
    """Mean rocprofv3 kernel-trace duration (us) of `kernel` over the contract's
    loop only: the newest committed profiles/rNN_kernel_stats_loop.csv
    (tools/profile_round.sh: `rocprofv3 --kernel-trace --stats -- bench.py
    --no-secondary --no-cpu-baseline`, configs[2]'s launches only; the full
    rNN_kernel_stats.csv also averages the KITTI, bounds-at-frame, fp16 and dense
    legs' launches of the same kernel).  (avg_us, calls, source) or (None, None, None)."""
    import csv

    d, files = _pmc_summaries("_kernel_stats_loop.csv")
    for f in reversed(files):
        for row in csv.DictReader(open(os.path.join(d, f))):
            if row["Name"].startswith(kernel):
                return float(row["AverageNs"]) / 1000.0, int(row["Calls"]), f
    return None, None, None


def ktrace_grid_us(frags, pick: str = "max_grid"):
    """Kernel-trace durations (rocprofv3's GPU start / end: no launch cost) per
    kernel and grid from the newest committed profiles/rNN_ktrace_grid.json
    (tools/ktrace_by_grid.py over the profiled bench run): for each kernel name
    fragment the entry of the largest grid (pick "max_grid": the 4K leg's
    launches) or of the most dispatches (pick "most": the loop's, which since
    round 5 run beside the critical PyrLK, so their durations include that
    overlap); (sum of their mean durations in us, [(kernel, grid, dispatches,
    avg_us)], source) or (None, None, None)."""
    d, files = _pmc_summaries("_ktrace_grid.json")
    if not files:
        return None, None, None
    ents = json.load(open(os.path.join(d, files[-1])))["entries"]
    tot, used = 0.0, []
    for frag in frags:
        c = [e for e in ents if frag in e["kernel"]]
        if not c:
            return None, None, None
        if pick.startswith("dispatches:"):  # the entry of a leg with its own dispatch count
            c = [e for e in c if e["dispatches"] == int(pick.split(":")[1])]
            if not c:
                return None, None, None
        e = max(c, key=(lambda e: e["grid"]) if pick != "most" else (lambda e: e["dispatches"]))
        tot += e["avg_us"]
        used.append((e["kernel"], e["grid"], e["dispatches"], e["avg_us"]))
    return round(tot, 3), used, files[-1]


# ---- host cores and rank pinning --------------------------------------------------------------


def parse_cpulist(s: str) -> list:
    out = []
    for part in s.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def host_cores():
    """CPUs this process may use: its affinity mask, capped by a cgroup v2 CPU
    quota when one is set (the GPU box gives each GPU a share of a larger host)."""
    aff = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    n = len(aff) if quota is None else min(len(aff), quota)
    return n, {"affinity_cpus": len(aff), "cgroup_cpu_quota": quota}


def _gpu_bdfs_kfd(sysroot: str):
    """PCI addresses of the GPUs in HIP device order from the KFD topology
    (nodes with SIMDs, in node order, location_id = bus << 8 | dev << 3 | fn);
    None when a GPU node carries no location_id."""
    root = os.path.join(sysroot, "class/kfd/kfd/topology/nodes")
    out = []
    for n in sorted(os.listdir(root), key=int):
        props = {}
        for line in open(os.path.join(root, n, "properties")):
            kv = line.split()
            if len(kv) == 2:
                try:
                    props[kv[0]] = int(kv[1])
                except ValueError:
                    pass
        if props.get("simd_count", 0) > 0:
            if "location_id" not in props:
                return None
            dom, loc = props.get("domain", 0), props["location_id"]
            out.append(f"{dom:04x}:{(loc >> 8) & 0xFF:02x}:{(loc >> 3) & 0x1F:02x}.{loc & 7:x}")
    return out or None


def _gpu_bdfs_drm(sysroot: str):
    """Fallback: the AMD display-class PCI devices behind /sys/class/drm/card*,
    in PCI address order (the order KFD enumerates them on a node)."""
    root = os.path.join(sysroot, "class/drm")
    bdfs = set()
    for c in os.listdir(root):
        if not c.startswith("card") or "-" in c:
            continue
        dev = os.path.join(root, c, "device")
        try:
            if open(os.path.join(dev, "vendor")).read().strip() != "0x1002":
                continue
            if not open(os.path.join(dev, "class")).read().strip().startswith("0x03"):
                continue
            bdfs.add(os.path.basename(os.path.realpath(dev)))
        except OSError:
            continue
    return sorted(bdfs) or None


def gpu_numa_cpus(local_rank: int, sysroot: str = "/sys"):
    """(numa node, cpus, source) of the host CPUs local to the local_rank-th
    visible GPU, from sysfs only (no GPU call, so it can run before HIP starts):
    the GPU's PCI address from the KFD topology, else from the DRM cards; its
    CPUs from the PCI device's local_cpulist, else its NUMA node's cpulist.
    None when sysfs does not say."""
    bdfs, src = None, None
    for fn, name in ((_gpu_bdfs_kfd, "kfd"), (_gpu_bdfs_drm, "drm")):
        try:
            bdfs = fn(sysroot)
        except (OSError, ValueError):
            bdfs = None
        if bdfs:
            src = name
            break
    if not bdfs:
        return None
    try:
        vis = os.environ.get("ROCR_VISIBLE_DEVICES") or os.environ.get("HIP_VISIBLE_DEVICES")
        if vis:
            bdfs = [bdfs[int(i)] for i in vis.split(",")]
        bdf = bdfs[local_rank]
        dev = os.path.join(sysroot, "bus/pci/devices", bdf)
        node = -1
        try:
            node = int(open(os.path.join(dev, "numa_node")).read())
        except (OSError, ValueError):
            pass
        try:
            cpus = parse_cpulist(open(os.path.join(dev, "local_cpulist")).read())
            if cpus:
                return node, cpus, f"{src}:{bdf}:local_cpulist"
        except (OSError, ValueError):
            pass
        if node < 0:
            return None
        cpus = parse_cpulist(open(os.path.join(sysroot, f"devices/system/node/node{node}/cpulist")).read())
        return (node, cpus, f"{src}:{bdf}:numa_node") if cpus else None
    except (OSError, ValueError, IndexError):
        return None


def pin_rank(local_rank: int):
    """Pin this rank (before any GPU call, so the HIP runtime's threads inherit
    it) to the CPUs NUMA-local to its GPU: each rank's host loop and tracker then
    run next to their device and off the other ranks' cores.
    Returns what was done, for the JSON line."""
    got = gpu_numa_cpus(local_rank)
    if got is None:
        return {"pinned": False, "reason": "no NUMA / local_cpulist information for the GPU in sysfs"}
    node, cpus, src = got
    allowed = sorted(set(cpus) & os.sched_getaffinity(0))
    if not allowed:
        return {"pinned": False, "numa_node": node, "source": src,
                "reason": "GPU-local CPUs outside the affinity mask"}
    if set(allowed) == os.sched_getaffinity(0):
        return {"pinned": False, "numa_node": node, "source": src, "cpus": len(allowed),
                "reason": "the affinity mask is already GPU-local"}
    # every thread the process has so far (none is a HIP thread yet: pinning
    # precedes the first GPU call), so later threads inherit the mask
    _pin_all_threads(allowed)
    return {"pinned": True, "numa_node": node, "source": src, "cpus": len(allowed)}


def _pin_all_threads(cpus):
    for tid in os.listdir("/proc/self/task"):
        try:
            os.sched_setaffinity(int(tid), cpus)
        except OSError:
            pass
    os.sched_setaffinity(0, cpus)


def pin_rank_by_device(dev: int, sysroot: str = "/sys"):
    """Second chance when sysfs could not name the GPU before HIP started: its
    PCI address as the runtime reports it (torch device properties, after
    device init), then that PCI device's local_cpulist / NUMA node.  Every
    thread of the process is re-pinned (the runtime's included); no re-exec."""
    import torch

    try:
        pr = torch.cuda.get_device_properties(dev)
        bdf = f"{int(getattr(pr, 'pci_domain_id', 0)):04x}:{int(pr.pci_bus_id):02x}:{int(pr.pci_device_id):02x}.0"
    except (AttributeError, RuntimeError, TypeError, ValueError):
        return {"pinned": False, "reason": "no PCI address from the runtime"}
    d = os.path.join(sysroot, "bus/pci/devices", bdf)
    cpus, node = [], -1
    try:
        node = int(open(os.path.join(d, "numa_node")).read())
    except (OSError, ValueError):
        pass
    try:
        cpus = parse_cpulist(open(os.path.join(d, "local_cpulist")).read())
    except (OSError, ValueError):
        if node >= 0:
            try:
                cpus = parse_cpulist(open(os.path.join(sysroot, f"devices/system/node/node{node}/cpulist")).read())
            except (OSError, ValueError):
                pass
    if not cpus:
        return {"pinned": False, "pci": bdf, "reason": "no local_cpulist / NUMA node for the GPU's PCI device"}
    allowed = sorted(set(cpus) & os.sched_getaffinity(0))
    if not allowed:
        return {"pinned": False, "pci": bdf, "reason": "GPU-local CPUs outside the affinity mask"}
    if set(allowed) == os.sched_getaffinity(0):
        return {"pinned": False, "pci": bdf, "cpus": len(allowed), "reason": "the affinity mask is already GPU-local"}
    _pin_all_threads(allowed)
    return {"pinned": True, "pci": bdf, "numa_node": node, "source": "runtime PCI address", "cpus": len(allowed)}


# ---- CPU baseline -----------------------------------------------------------------------------


def native_oracle():
    """Build the oracle's sources -O3 -march=native for THIS host (the CPU
    baseline of SURVEY.md §8d; -ffp-contract=off keeps its results identical to
    the test build) and point tests/_oracle.py at it.  Must run before the first
    import of _oracle.  Returns the library path, or None (the shipped -O2 build
    is used)."""
    import subprocess
    import tempfile

    if "_oracle" in sys.modules:
        return os.environ.get("TBDK_ORACLE_LIB")
    out = os.path.join(tempfile.mkdtemp(prefix="tbdk_oracle_"), "liboracle_native.so")
    try:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native", f"NATIVE_OUT={out}"],
                       check=True, capture_output=True, timeout=300)
    except (OSError, subprocess.SubprocessError):
        return None
    os.environ["TBDK_ORACLE_LIB"] = out
    return out


class _NativeTracker:
    """tbd_oracle.Tracker's interface over libtbdk's host tracker (tbdk_tracker_*:
    host C++, the same code the GPU loop's tracker step runs), so the CPU
    baseline's tracker step costs what the reference's C++ tracker costs, not
    what the pure-Python checker costs."""

    def __init__(self, bounds):
        import numpy as np
        from opencv_amd import tbd
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import tbd_oracle as T

        self.np, self.tbd, self.T = np, tbd, T
        self.t = tbd.Tracker(bounds=bounds)
        self.tracks = []
        self.true_positives, self.false_negatives, self.false_positives, self.ground_truths = [], [], [], []

    def step(self, dets, frame_id, preds):
        d = self.np.zeros(len(dets), self.tbd.DET_DTYPE)
        for i, x in enumerate(dets):
            d[i] = (x.id, x.bbox.x, x.bbox.y, x.bbox.width, x.bbox.height, x.confidence)
        m = self.t.performTrackingStep(d, frame_id, preds)
        self.true_positives.append(m.tp)
        self.false_negatives.append(m.fn)
        self.false_positives.append(m.fp)
        self.ground_truths.append(m.gt)
        T = self.T
        self.tracks = [T.Track(id=r.id, bboxes=[T.Rect(r.x, r.y, r.width, r.height)], age=r.age,
                               totalVisibleCount=r.total_visible,
                               predPosition=T.Rect(r.pred_x, r.pred_y, r.pred_w, r.pred_h))
                       for r in self.t.getTracks()]


def cpu_baseline(frames_host, gt, args, seconds: float, threads: int, max_frames=None):
    """The CPU loop of the same workload on this host: oracle/tbd_loop_oracle.py
    (the reference's primitives composed as the GPU loop composes them: pyramid,
    GFTT(256/box, q 0.01, minDist 3) on new / re-detect / depleted tracks, PyrLK
    win 21 3 levels in the reference's SSE2 accumulation order, getRTMatrix fit,
    the tracker step) with `threads` threads: PyrLK over points (the
    reference's parallel_for_), the boxes' goodFeaturesToTrack calls concurrently
    (one ROI per call, as the reference's single-threaded GFTT), and the C++
    tracker.  Frame 0 (no tracking yet) runs untimed; frames 1.. are timed until
    `seconds` have passed (at least 3)."""
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import tbd_loop_oracle as L

    W, H = frames_host.shape[2], frames_host.shape[1]
    bounds = (0, W, 0, H) if args.bounds == "frame" else (0, 1280, 0, 720)
    pool = ThreadPoolExecutor(threads) if threads > 1 else None
    lp = L.KltTbdLoop(W, H, win=args.win, max_level=args.max_level, redetect_every=args.redetect,
                      accum=L.O.ACCUM_SSE2, nthreads=threads, tracker=_NativeTracker(bounds), gftt_pool=pool)
    lp.step(frames_host[0], 0, L.detections(gt[0], 0))
    n = frames_host.shape[0] if max_frames is None else min(max_frames, frames_host.shape[0])
    done = 0
    t0 = time.perf_counter()
    for f in range(1, n):
        lp.step(frames_host[f], f, L.detections(gt[f], f))
        done += 1
        if time.perf_counter() - t0 > seconds and done >= 3:
            break
    el = time.perf_counter() - t0
    if pool is not None:
        pool.shutdown()
    return done / el, done


def cpu_baseline_line(frames_host, gt, args, restore_affinity=None):
    """cpu_baseline object: every CPU this process may use (the rank's pinning
    undone for the measurement), plus a 1-thread figure on a shorter sample."""
    pinned = os.sched_getaffinity(0)
    if restore_affinity:
        os.sched_setaffinity(0, restore_affinity)
    try:
        lib = native_oracle()
        cores, info = host_cores()
        fps, n = cpu_baseline(frames_host, gt, args, args.cpu_baseline_seconds, cores)
        fps1, n1 = cpu_baseline(frames_host, gt, args, args.cpu_baseline_seconds_1t, 1)
    finally:
        os.sched_setaffinity(0, pinned)
    cal = None
    try:  # the restatement against the real reference on a shape-matched input
        c = json.load(open(os.path.join(ROOT, "profiles", "r05_cpu_calibration.json")))
        m = c["inputs"]["matched_iterations"]["results"]
        r1, r8 = m["lk_1080p_128x256_1t_ms"], m["lk_1080p_128x256_8t_ms"]
        cal = {"restatement_over_reference_lk_1t": r1["ratio"], "restatement_over_reference_lk_8t": r8["ratio"],
               "per_iteration_1t": r1["ratio_per_iteration"], "per_iteration_8t": r8["ratio_per_iteration"],
               "mean_iters_restatement": r1["mean_iters"], "mean_iters_reference": r1["reference_mean_iters"],
               "source": "profiles/r05_cpu_calibration.json (tests/calibrate_cpu.py vs BASELINE.md §2)",
               "note": "PyrLK per call, 1080p x 32k points on an input blurred to the reference figure's iteration "
                       "count (13.4 per point against its 8-12): the C restatement is this many times slower than "
                       "the reference's SSE2 build per call, and per Newton iteration at the reference's 12 and 8 "
                       "iterations per point"}
    except (OSError, KeyError, ValueError):
        pass
    # the restatement is slower than the reference's SSE2 build: the reference's own
    # CPU path on this host would reach about value x the per-iteration ratio (the larger of the two
    # reference iteration counts' ratios, multi-threaded: the figure most favourable to the reference)
    ref_eq = None
    if cal:
        r = max(cal["per_iteration_8t"])
        ref_eq = {"value": round(fps * r, 3), "unit": "frames/s", "ratio": r,
                  "range": [round(fps * min(cal["per_iteration_8t"]), 3), round(fps * r, 3)],
                  "note": "value x the restatement/reference time ratio per Newton iteration (8 threads, the "
                          "reference at 8 and 12 iterations per point); PyrLK is >= 95 % of the CPU loop"}
    return {"value": round(fps, 3), "unit": "frames/s", "cores": cores, "kind": "port", "calibration": cal,
            "value_reference_equivalent": ref_eq,
            "value_1_thread": round(fps1, 4), "frames_1_thread": n1, "host": info,
            "build": "oracle/ sources -O3 -march=native -ffp-contract=off, built on this host" if lib else
                     "oracle/liboracle.so as shipped (-O2; the native build failed)",
            "sample": f"frames 1..{n} of the rank-0 sequence ({args.width}x{args.height} x {args.objects} objects, "
                      f"frame 0 untimed) through oracle/tbd_loop_oracle.py: pyramid, GFTT(256/box, every "
                      f"{args.redetect} frames or < 32 points, the boxes' calls on {cores} threads), PyrLK win "
                      f"{args.win} {args.max_level + 1} levels in the reference's SSE2 accumulation order "
                      f"({cores} threads), getRTMatrix fit, and the C++ tracker step; the 1-thread figure over "
                      f"frames 1..{n1 + 1}"}


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
    per_launch, traffic_src = pmc_traffic("fb_iter_kernel<6, false>", "_pmc.json")
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
    """Algorithmic HBM bytes of one fp16 pyramid build from a u8 frame, the
    bytes that must move: the frame read once (1 B/px), every level written
    once (2 B/px) and every level above 0 read once for the next level and its
    own Scharr plane (2 B/px), every fp16 (Ix, Iy) plane written (4 B/px).
    (Rounds 1-3 counted level 0 and each level's Scharr source as separate
    reads, as the one-launch-per-plane build does: pyr_f16_bytes_per_plane.)"""
    sizes = []
    for _ in range(nlevels):
        sizes.append(w * h)
        w, h = (w + 1) // 2, (h + 1) // 2
    return sizes[0] + 2 * sum(sizes) + 2 * sum(sizes[1:]) + 4 * sum(sizes)


def pyr_f16_bytes_per_plane(w: int, h: int, nlevels: int) -> int:
    """the rounds 1-3 count: frame read and level 0 written (3 B/px), per
    further level the previous level read and the level written, per level its
    Scharr source read and plane written (6 B/px)"""
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
    ptr = pmc_pyr_traffic("f16", [("pyr_fp_jobs_kernel<false>", nlev)])  # counters of the role-split build
    gbs = pb / (pk["avg_us"] * 1e-6) / 1e9
    out = {"value": round(n / wall, 2), "unit": "pairs/s", "points_per_s": round(n * npts / wall, 1),
           "ms_per_pair": round(1000 * wall / n, 3), "dtype": "f16 pixels, f32 arithmetic",
           "config": {"workload": f"sparse PyrLK {w}x{h}, {args.fb_objects} objects x {per_box} points "
                                  "(BASELINE configs[4] fp16 pixel path)", "points": npts, "levels": nlev,
                      "win": args.win, "pairs": n, "mean_iters_per_point": iters / n / npts},
           "roofline": {"bound": "valu", "achieved": round(tf, 3), "peak": PEAK_F32_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(tf / PEAK_F32_TFLOPS, 4), "traffic": None, "kernel": "lk_sparse (lk_f16_kernel)",
                        "flops_per_launch": flops,
                        "note": "VALU-bound (fp32 FMA on fp16 taps, no MFMA); algorithmic flops per SURVEY.md §8(d)"},
           "roofline_pyramid": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                "frac": round(gbs / PEAK_HBM_GBS, 4), "bytes_per_launch": pb,
                                "bytes_per_launch_per_plane_count": pyr_f16_bytes_per_plane(w, h, nlev),
                                "traffic": ptr[0], "traffic_fetch_x2": ptr[1], "traffic_source": ptr[2],
                                "traffic_over_algorithmic": round(ptr[0] / pb, 3) if ptr[0] else None,
                                "avg_us": round(pk["avg_us"], 2),
                                "kernel": "pyr_build (fp16 levels + fp16 Scharr planes; klt_pyr_fp.hip, "
                                          f"{nlev} role-split launches)"},
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


def dense_lk_secondary(ctx, args, device, cpu: bool):
    """dense PyrLK, cv::cuda::DensePyrLKOpticalFlow's interface
    with its defaults (win 13, maxLevel 3, 30 iterations) on synthetic 1080p
    pairs, computed as the CPU calcOpticalFlowPyrLK at every pixel
    (tbdk_lk_dense: per pair the next frame's pyramid with Scharr planes, the
    case images of the previous one, the PyrLK of all 2.07 M pixels).
    Pairs/s and pixels/s, the per-point-setup path (ctx option lk_dense_case 0)
    beside it, and the oracle on a pixel sample.  Reported, never `value`."""
    import numpy as np
    import torch
    from opencv_amd import klt

    w, h, n = args.width, args.height, args.dense_pairs
    frames, _ = klt.synth_render(args.seed + 17, w, h, args.objects, 0, n + 1, device=device, ctx=ctx)
    win, ml = (13, 13), 3
    lk = klt.DensePyrLKOpticalFlow.create(win, ml, 30)
    pyrs = [klt.Pyramid(ctx, w, h, ml, win) for _ in range(2)]
    flow = torch.empty((h, w, 2), dtype=torch.float32, device=frames.device)

    def run():
        pyrs[0].build(frames[0])
        for i in range(n):
            pyrs[(i + 1) % 2].build(frames[i + 1])
            lk.calc(pyrs[i % 2], pyrs[(i + 1) % 2], flow)

    res = {}
    try:
        for mode in (1, 0):
            ctx.set_option("lk_dense_case", mode)
            run()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run()
            torch.cuda.synchronize()
            res[mode] = (time.perf_counter() - t0) / n
    finally:
        ctx.set_option("lk_dense_case", 1)
    out = {"value": round(1.0 / res[1], 2), "unit": "pairs/s", "mpix_per_s": round(w * h / res[1] / 1e6, 1),
           "ms_per_pair": round(1000 * res[1], 3), "dtype": "u8",
           "per_point_setup": {"value": round(1.0 / res[0], 2), "unit": "pairs/s",
                               "note": "ctx option lk_dense_case 0: the sparse kernel's per-point window setup over "
                                       "the pixel grid (round 4's dense path)"},
           "config": {"workload": f"dense PyrLK {w}x{h} synthetic pairs (cv::cuda::DensePyrLKOpticalFlow defaults)",
                      "win": 13, "max_level": ml, "iters": 30, "pairs": n,
                      "per_pair": "next pyramid (levels + Scharr planes) + case images + PyrLK of every pixel"}}
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as O
        a_, b_ = frames[0].cpu().numpy(), frames[1].cpu().numpy()
        threads = min(16, os.cpu_count() or 1)
        ys, xs = np.mgrid[0:h:16, 0:w:16]
        sample = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.float32)
        t1 = time.perf_counter()
        P0, P1 = O.Pyramid(a_, win, ml), O.Pyramid(b_, win, ml)
        tp = (time.perf_counter() - t1) / 2
        t1 = time.perf_counter()
        O.lk(P0, P1, sample, win=win, max_level=ml, accum=O.ACCUM_SSE2, nthreads=threads, want_err=False)
        tl = (time.perf_counter() - t1) * (w * h) / len(sample)
        out["cpu_baseline"] = {"value": round(1.0 / (tp + tl), 4), "unit": "pairs/s", "cores": threads,
                               "kind": "port",
                               "sample": f"oracle/klt_oracle.c: one pyramid (1 thread) + calcOpticalFlowPyrLK of "
                                         f"{len(sample)} grid pixels (every 16th row and column, {threads} threads, "
                                         "SSE2 order), LK time scaled to all pixels"}
    del frames, pyrs, flow
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


# ---- the contract ----------------------------------------------------------------------------


def rank_env():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(argv, n: int, script: str = None, poll_s: float = 0.2) -> int:
    """`bench.py --gpus N` without a launcher (WORLD_SIZE unset): start N rank
    processes of this same script, one per GPU (WORLD_SIZE = N, RANK =
    LOCAL_RANK = i, MASTER_ADDR 127.0.0.1 and a free MASTER_PORT), as
    torch.distributed.run would.  This process makes no GPU call and execs
    nothing: the ranks are children, rank 0's stdout (the one JSON line) is
    relayed, the others' stdout is dropped, stderr is inherited.  When a rank
    fails the others are ended (their exact PIDs) and its exit code returned,
    so a failure cannot leave the rest waiting in a barrier.  Returns the exit
    code (0 when every rank exited 0)."""
    import subprocess
    import threading

    script = script or os.path.abspath(__file__)
    port = _free_port()
    procs, lines = [], []
    for r in range(n):
        env = dict(os.environ, WORLD_SIZE=str(n), RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))

    def relay():
        for ln in procs[0].stdout:
            lines.append(ln)
            sys.stdout.write(ln)
            sys.stdout.flush()

    th = threading.Thread(target=relay, daemon=True)
    th.start()
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(poll_s)
    th.join(timeout=30)
    if rc == 0 and sum(1 for ln in lines if ln.lstrip().startswith("{")) != 1:
        print(f"bench.py: rank 0 printed {len(lines)} stdout lines, expected one JSON line", file=sys.stderr)
        rc = 1
    return rc


def check_world(gpus: int, world: int) -> None:
    """--gpus N must agree with the launcher's WORLD_SIZE (torchrun sets it):
    a mismatch would print a line whose n_gpus is not what was asked for."""
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world} (the launcher started {world} ranks); "
                         "run `bench.py --gpus N` alone (it starts N ranks itself) or under torchrun "
                         "with --nproc-per-node equal to --gpus")


def gather_seeds(seed: int, world: int):
    """Every rank's sequence seed on every rank (gloo; outside the timed region),
    for the line: the replicas ran seeds s..s+N-1."""
    if world <= 1:
        return [seed]
    import torch.distributed as dist

    out = [None] * world
    dist.all_gather_object(out, seed)
    return out


_T0 = time.perf_counter()


def hbm_copy_peak(dev, ctx=None, nbytes: int = 1 << 31, reps: int = 20) -> dict:
    """an HBM roofline also against a measured stream-copy peak.
    libtbdk's hand-written copy kernel (tbdk_hbm_copy: global_load_dwordx4 /
    global_store_dwordx4, four 16-byte loads in flight per lane) over a 2 GiB
    buffer (far beyond the L2s and the 256 MB Infinity Cache), read + write bytes
    / HIP-event time (events on the launch stream), best of `reps` copies after
    warm-up; the torch copy_ figure beside it."""
    import torch
    from opencv_amd import klt

    ctx = ctx or klt.Context.get(dev)
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    src.copy_(torch.arange(nbytes // 4, dtype=torch.int32, device=dev).view(torch.uint8))
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream()

    def best_of(fn):
        for _ in range(3):
            fn()
        best = None
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        return best

    t_torch = best_of(lambda: dst.copy_(src))
    dst.zero_()
    t_k = best_of(lambda: klt.hbm_copy(dst, src, ctx=ctx, stream=stream))
    ok = bool(torch.equal(dst, src))
    del src, dst
    gbs = 2 * nbytes / (t_k / 1000.0) / 1e9
    return {"value": round(gbs, 1), "unit": "GB/s", "bytes": 2 * nbytes, "copies": reps, "checked": ok,
            "frac_of_spec": round(gbs / PEAK_HBM_GBS, 4),
            "torch_copy_gbs": round(2 * nbytes / (t_torch / 1000.0) / 1e9, 1),
            "note": "tbdk_hbm_copy (hand-written 16 B/lane stream copy) of a 2 GiB buffer: read + write bytes / "
                    "fastest HIP-event time; torch_copy_gbs: torch copy_ of the same buffers"}


def add_copy_peak_fracs(obj, peak_gbs: float):
    """Every HBM-bound roofline object in the line gets its fraction of the
    measured copy peak beside the spec-peak fraction."""
    if isinstance(obj, dict):
        if obj.get("bound") == "hbm" and isinstance(obj.get("achieved"), (int, float)):
            obj["copy_peak"] = peak_gbs
            obj["frac_copy_peak"] = round(obj["achieved"] / peak_gbs, 4)
        for v in obj.values():
            add_copy_peak_fracs(v, peak_gbs)


def progress(msg: str, rank: int = 0):
    """one line per bench leg on stderr (rank 0): a long run under a profiler
    shows it is alive; stdout keeps the single JSON line"""
    if rank == 0:
        print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def init_rank_group(world: int, rank: int, local: int) -> None:
    """Select the rank's GPU and, at world > 1, join the job's process group.

    The replicas exchange nothing on the data path: the
    contract's barriers and the max-over-ranks time go over a gloo (host)
    group, so no RCCL communicator creates GPU streams.  HIP maps a process's
    streams onto its 4 hardware queues in creation order, and the TBD loop
    drops from ~4.8k to ~3k frames/s when more than four streams exist before
    its own."""
    import torch
    import torch.distributed as dist

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if os.environ.get("TBDK_BENCH_SHARE_GPU") == "1":
            # rehearsal of the N-rank path on a box with fewer GPUs than ranks:
            # ranks share the GPUs round-robin (the throughput is then not a
            # scaling figure; device_count() does not initialise the GPU)
            local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        torch.cuda.set_device(0)


def run_contract(args, world: int, rank: int, measure, sync, dist_device, cpu_leg=None):
    """The bench contract, independent of what a step is: the rank's own
    sequence (seed + rank), W untimed warm-up steps, then EXACTLY K steps
    bracketed by a barrier + device sync on both sides, the max time over ranks,
    value = steps of all ranks / that time (replicas, weak scaling), and the CPU
    baseline on rank 0 at N = 1 only.  Returns (line, per-step results)."""
    import torch.distributed as dist

    progress("rendering the sequence", rank)
    measure.prepare(args.seed + rank)
    seeds = gather_seeds(args.seed + rank, world)
    progress("warm-up", rank)
    measure.warmup(args.warmup)
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    per_step = measure.timed(args.steps)
    sync()
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    el = max_over_ranks(el, world, device=dist_device)
    line = {
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
        "rank_seeds": seeds,
    }
    progress(f"timed region: {line['value']} frames/s", rank)
    if cpu_leg is not None and rank == 0 and world == 1:
        progress("cpu baseline")
    line["cpu_baseline"] = cpu_leg() if (cpu_leg is not None and rank == 0 and world == 1) else None
    return line, per_step


class TbdMeasure:
    """BASELINE configs[2]: the rank's synthetic 1080p x 128-object sequence of
    max(sequence_frames, W + K) frames rendered into HBM; warm-up = frames
    [0, W) one tbdk_tbd_step at a time, the timed steps = frames [W, W + K)
    through tbdk_tbd_run (or the per-frame APIs, --api)."""

    def __init__(self, args, ctx, dev):
        self.args, self.ctx, self.dev = args, ctx, dev

    def prepare(self, seed: int):
        import torch
        from opencv_amd import klt, tbd

        a = self.args
        self.nseq = max(a.sequence_frames, a.warmup + a.steps)
        self.frames, gt = klt.synth_render(seed, a.width, a.height, a.objects, 0, self.nseq, device=self.dev,
                                           ctx=self.ctx)
        self.gtn = gt.numpy()
        self.dets = [tbd.detections_from_gt(self.gtn[f]) for f in range(self.nseq)]
        over = dict(bounds_xmax=a.width, bounds_ymax=a.height) if a.bounds == "frame" else {}
        self.cfg = tbd.default_config(a.width, a.height, win=a.win, max_level=a.max_level,
                                      redetect_every=a.redetect, **over)
        self.stream = torch.cuda.current_stream()
        self.loop = tbd.TbdLoop(self.cfg, ctx=self.ctx)
        torch.cuda.synchronize()

    def new_loop(self, warmup: int):
        from opencv_amd import tbd

        loop = tbd.TbdLoop(self.cfg, ctx=self.ctx)
        for f in range(warmup):
            loop.step(self.frames[f], f, self.dets[f], self.stream)
        return loop

    def warmup(self, w: int):
        from opencv_amd import tbd

        a, ctx = self.args, self.ctx
        for f in range(w):
            self.loop.step(self.frames[f], f, self.dets[f], self.stream)
        self.w = w
        self.frame_list = [self.frames[f] for f in range(w, w + a.steps)]
        self.packed = tbd.TbdLoop.pack_detections(self.dets[w:w + a.steps])  # staged like the frames
        self.timed_kernels = ["pyr_build", "lk_sparse", "gftt", "tbd_fit"] if a.kstats == "all" else \
            [] if a.kstats == "none" else [k for k in a.kstats.split(",") if k]
        ctx.timing_select(self.timed_kernels or None)
        # events on every Nth timed launch: each costs two event records of host
        # work on the frame's critical path (~5 % of the frame when every launch is timed)
        ctx.set_option("timing_every", a.timing_every)
        ctx.timing_enable(bool(self.timed_kernels))

    def timed(self, k: int):
        a, w = self.args, self.w
        if a.api == "run":
            return list(self.loop.run(self.frame_list, w, None, self.stream, packed=self.packed))
        out = []
        for f in range(w, w + k):
            nxt = self.frames[f + 1] if a.api == "ahead" and f + 1 < self.nseq else None
            out.append(self.loop.step(self.frames[f], f, self.dets[f], self.stream, next_frame=nxt))
        return out


def timed_on_all_ranks(fn, world):
    """Barrier + sync, fn(), sync, barrier; the max wall time over ranks."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    return max_over_ranks(el, world, device="cpu")


def sequence_repeats(m: TbdMeasure, world: int, runs: int, skip: int):
    """the whole sequence in steady state (frames [skip, nseq)
    after `skip` warm-up frames), a fresh loop per run, median of `runs` runs."""
    from opencv_amd import tbd

    frames = [m.frames[f] for f in range(skip, m.nseq)]
    packed = tbd.TbdLoop.pack_detections(m.dets[skip:m.nseq])
    fps = []
    for _ in range(runs):
        loop = m.new_loop(skip)
        el = timed_on_all_ranks(lambda: loop.run(frames, skip, None, m.stream, packed=packed), world)
        fps.append(replica_throughput(len(frames), world, el))
        del loop
    return {"frames": len(frames), "skip": skip, "runs_fps": [round(v, 1) for v in fps],
            "median_fps": round(sorted(fps)[len(fps) // 2], 2), "unit": "frames/s",
            "api": "tbdk_tbd_run", "note": "whole 500-frame sequence after 20 warm-up frames, fresh loop per run"}


def with_h2d(m: TbdMeasure, world: int, runs: int, skip: int):
    """§8d's with-H2D variant: the same frames from page-locked host memory
    through tbdk_tbd_run_host (each frame uploaded into a device ring two
    frames ahead, on its own stream).  Never `value`."""
    from opencv_amd import tbd

    host = m.frames.cpu().pin_memory()
    packed = tbd.TbdLoop.pack_detections(m.dets[skip:m.nseq])
    fps = []
    for _ in range(runs):
        loop = m.new_loop(skip)
        el = timed_on_all_ranks(lambda: loop.run_host(host[skip:], skip, None, m.stream, packed=packed), world)
        fps.append(replica_throughput(m.nseq - skip, world, el))
        del loop
    px = m.args.width * m.args.height
    med = sorted(fps)[len(fps) // 2]
    del host
    return {"frames": m.nseq - skip, "runs_fps": [round(v, 1) for v in fps], "median_fps": round(med, 2),
            "unit": "frames/s", "h2d_bytes_per_frame": px, "h2d_gbs": round(med / world * px / 1e9, 3),
            "api": "tbdk_tbd_run_host (pinned host frames, upload ring)"}


def bounds_frame_leg(m: TbdMeasure, world: int, runs: int, skip: int):
    """The KLT-propagated regime: the same sequence with the
    tracker's bounds filter at the frame (W x H) instead of the reference's
    hard-coded 1280 x 720 (tbd.cpp:218), so every object's track lives and is
    propagated by PyrLK and GFTT runs on re-detection frames and depleted sets
    only.  Frames [skip, nseq) through tbdk_tbd_run after `skip` warm-up frames,
    a fresh loop per run, median of `runs`.  Never `value` (configs[2] keeps
    the reference's filter)."""
    from opencv_amd import tbd

    a = m.args
    cfg = tbd.default_config(a.width, a.height, win=a.win, max_level=a.max_level, redetect_every=a.redetect,
                             bounds_xmax=a.width, bounds_ymax=a.height)
    frames = [m.frames[f] for f in range(skip, m.nseq)]
    packed = tbd.TbdLoop.pack_detections(m.dets[skip:m.nseq])
    fps, per = [], None
    for _ in range(runs):
        loop = tbd.TbdLoop(cfg, ctx=m.ctx)
        for f in range(skip):
            loop.step(m.frames[f], f, m.dets[f], m.stream)
        res = []
        el = timed_on_all_ranks(lambda: res.extend(loop.run(frames, skip, None, m.stream, packed=packed)), world)
        fps.append(replica_throughput(len(frames), world, el))
        per = res
        del loop
    nf = max(1, len(per))
    return {"median_fps": round(sorted(fps)[len(fps) // 2], 2), "runs_fps": [round(v, 1) for v in fps],
            "unit": "frames/s", "frames": len(frames),
            "per_frame": {"tracks": sum(x.ntracks for x in per) / nf, "lk_points": sum(x.lk_points for x in per) / nf,
                          "gftt_rois": sum(x.redetected for x in per) / nf,
                          "klt_predicted": sum(x.klt_predicted for x in per) / nf},
            "tracker_bounds": f"0..{a.width} x 0..{a.height} (the frame)",
            "note": "secondary: every track propagated by KLT (no 1280x720 filter churn); not BASELINE's config"}


def copy_rate_at(ctx, traffic_bytes: int, reps: int = 25) -> dict:
    """The hand-written stream copy (tbdk_hbm_copy) moving the same number of
    bytes as a small kernel (read + write = traffic_bytes), timed the same way
    (HIP events on the launch stream, best of `reps` after warm-up): what one
    launch of that size can reach on this chip, launch latency included (a
    11 MiB copy reaches ~3 TB/s, a 2 GiB one ~5.7 TB/s)."""
    import torch
    from opencv_amd import klt

    n = max(16, (traffic_bytes // 2) // 16 * 16)
    src = torch.ones(n, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    st = torch.cuda.current_stream()
    best = None
    for i in range(reps + 5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        klt.hbm_copy(dst, src, ctx=ctx, stream=st)
        e1.record(st)
        e1.synchronize()
        if i >= 5:
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
    del src, dst
    return {"bytes": 2 * n, "us": round(best * 1000, 2), "gbs": round(2 * n / (best / 1000) / 1e9, 1)}


def pmc_pyr_traffic(kind: str, kernels):
    """HBM counter bytes per build of a pyramid build from the newest committed
    profiles/rNN_pmc_pyr_<kind>.json (tools/pmc_pyr_fp.sh: FETCH_SIZE and
    WRITE_SIZE passes over the probe, per kernel and grid size): for each kernel
    name fragment, the entry of the largest grid (the 4K build), fetch + write;
    (raw, fetch doubled, source file) or (None, None, None)."""
    d = os.path.join(ROOT, "profiles")
    try:
        files = sorted(f for f in os.listdir(d) if f.endswith(f"_pmc_pyr_{kind}.json"))
    except OSError:
        return None, None, None
    if not files:
        return None, None, None
    summ = json.load(open(os.path.join(d, files[-1])))
    raw = dbl = 0.0
    for frag, n in kernels:
        ent = [(int(k.rsplit("grid=", 1)[1]), v) for k, v in summ.items()
               if frag in k and "grid=" in k and "fetch_mb" in v and "write_mb" in v]
        if len(ent) < n:
            return None, None, None
        for _, v in sorted(ent, key=lambda e: -e[0])[:n]:
            raw += (v["fetch_mb"] + v["write_mb"]) * 1e6
            dbl += (2 * v["fetch_mb"] + v["write_mb"]) * 1e6
    return round(raw), round(dbl), files[-1]


def pyramid_4k_leg(ctx, dev, builds: int = 200) -> dict:
    """roofline_pyramid_4k: the u8 levels-only pyramid build (the TBD loop's
    pyramid, 3 levels, win 21) of a 3840x2160 frame (BASELINE configs[4]'s size),
    where the build's bytes are large enough for the HBM roofline to be the
    bound: algorithmic bytes (pyr_build_bytes: frame read once, every padded
    level written, level 2 reading level 1) / the build's HIP-event time (both
    launches), mean over `builds` builds alternating two frames."""
    import torch
    from opencv_amd import klt

    W, H, ml = 3840, 2160, 2
    fr, _ = klt.synth_render(7, W, H, 64, 0, 2, ctx=ctx)
    P = klt.Pyramid(ctx, W, H, ml, (21, 21), derivs=False)
    for i in range(10):
        P.build(fr[i & 1])
    torch.cuda.synchronize()
    ctx.timing_select(["pyr_build"])
    ctx.timing_enable(True)
    for i in range(builds):
        P.build(fr[i & 1])
    torch.cuda.synchronize()
    c, ms = ctx.timing_query("pyr_build")
    ctx.timing_enable(False)
    ctx.timing_select(None)
    us = ms / c * 1000.0
    b = pyr_build_bytes(W, H, ml + 1)
    gbs = b / (us * 1e-6) / 1e9
    del fr, P
    cp = copy_rate_at(ctx, b)
    tr, tr2, src = pmc_pyr_traffic("u8", [("pyr_build_kernel", 1), ("pyr_down_padded_kernel", 1)])
    kt_us, kt_used, kt_src = ktrace_grid_us(("pyr_build_kernel", "pyr_down_padded_kernel"), "max_grid")
    # the borrowed build (tbdk_pyr_build_borrowed: level 0 is the frame, no padded
    # copy; the reference GPU class's pyramid): 180 timed + 10 warm-up builds, so
    # that its kernel-trace entries are told apart by their dispatch count
    PB = klt.Pyramid(ctx, W, H, ml, (21, 21), derivs=False)
    fr, _ = klt.synth_render(7, W, H, 64, 0, 2, ctx=ctx)
    for i in range(10):
        PB.build_borrowed(fr[i & 1])
    torch.cuda.synchronize()
    ctx.timing_select(["pyr_build"])
    ctx.timing_enable(True)
    for i in range(180):
        PB.build_borrowed(fr[i & 1])
    torch.cuda.synchronize()
    cb, msb = ctx.timing_query("pyr_build")
    ctx.timing_enable(False)
    ctx.timing_select(None)
    del fr, PB
    usb = msb / cb * 1000.0
    bb = pyr_build_bytes(W, H, ml + 1, copy_l0=False)
    gbsb = bb / (usb * 1e-6) / 1e9
    # (its level-2 launch has the padded build's grid: one kernel-trace entry for both)
    ktb_us, ktb_used, ktb_src = ktrace_grid_us(("pyr_build_kernel",), "dispatches:190")
    ktd_us, ktd_used, _ = ktrace_grid_us(("pyr_down_padded_kernel",), "max_grid")
    if ktb_us is not None and ktd_us is not None:
        ktb_us, ktb_used = round(ktb_us + ktd_us, 3), ktb_used + ktd_used
    else:
        ktb_us = ktb_used = ktb_src = None
    borrowed = {"achieved": round(gbsb, 1), "frac": round(gbsb / PEAK_HBM_GBS, 4), "bytes_per_launch": bb,
                "avg_us": round(usb, 2), "builds": cb, "kernel_trace_us": ktb_us, "kernel_trace_launches": ktb_used,
                "kernel_trace_source": ktb_src,
                "frac_kernel_trace": round(bb / (ktb_us * 1e-6) / 1e9 / PEAK_HBM_GBS, 4) if ktb_us else None,
                "kernel": "tbdk_pyr_build_borrowed (levels 1-2 from the frame; level 0 is the frame itself)",
                "note": "algorithmic bytes: the frame read once, levels 1.. written padded, level 2 reading level 1 "
                        "(no level-0 copy: cudaoptflow/src/pyrlk.cpp:144-145)"}
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4), "bytes_per_launch": b, "avg_us": round(us, 2), "builds": c,
            "borrowed_level0": borrowed,
            "traffic": tr, "traffic_fetch_x2": tr2, "traffic_source": src,
            "traffic_over_algorithmic": round(tr / b, 3) if tr else None,
            "size_matched_copy": cp, "frac_size_matched_copy": round(gbs / cp["gbs"], 4),
            "kernel_trace_us": kt_us, "kernel_trace_launches": kt_used, "kernel_trace_source": kt_src,
            "frac_kernel_trace": round(b / (kt_us * 1e-6) / 1e9 / PEAK_HBM_GBS, 4) if kt_us else None,
            "kernel": "pyr_build (levels only, u8, 3840x2160, 3 levels)",
            "note": "algorithmic bytes (frame read once, padded levels written, level 2 reading level 1) / the "
                    "build's HIP-event time (events on the launch stream around its launches)"}


def standalone_pyr(ctx, W: int, H: int, builds: int = 200) -> dict:
    """The loop's levels-only u8 build (3 levels, win 21) of a W x H frame on an
    otherwise idle GPU: HIP events around every build (mean over `builds`,
    alternating two frames), beside the uncontended kernel-trace durations of
    the same build from the committed rocprofv3 summary of
    tools/probe_pyr_build.py (profiles/rNN_pyr_probe_ktrace.json, per grid)."""
    import torch
    from opencv_amd import klt

    fr, _ = klt.synth_render(7, W, H, 64, 0, 2, ctx=ctx)
    P = klt.Pyramid(ctx, W, H, 2, (21, 21), derivs=False)
    for i in range(10):
        P.build(fr[i & 1])
    torch.cuda.synchronize()
    ctx.timing_select(["pyr_build"])
    ctx.timing_enable(True)
    for i in range(builds):
        P.build(fr[i & 1])
    torch.cuda.synchronize()
    c, ms = ctx.timing_query("pyr_build")
    ctx.timing_enable(False)
    ctx.timing_select(None)
    del fr, P
    out = {"avg_us": round(ms / c * 1000.0, 2), "builds": c, "kernel_trace_us": None, "kernel_trace_source": None}
    d, files = _pmc_summaries("_pyr_probe_ktrace.json")
    if files:
        ents = json.load(open(os.path.join(d, files[-1])))["entries"]
        sel = PYR_PROBE_GRIDS.get((W, H))
        if sel:
            us = [e["avg_us"] for e in ents for k, g in sel if k in e["kernel"] and e["grid"] == g]
            if len(us) == len(sel):
                out.update(kernel_trace_us=round(sum(us), 3), kernel_trace_source=files[-1],
                           kernel_trace_launches=[list(x) for x in sel])
    return out


# the levels-only build's launches (kernel, grid size) per frame size, as
# tools/ktrace_by_grid.py keys them (two-role launch with the copy role, level 2)
PYR_PROBE_GRIDS = {(1920, 1080): (("pyr_build_kernel", 297984), ("pyr_down_padded_kernel", 85504)),
                   (3840, 2160): (("pyr_build_kernel", 1110272), ("pyr_down_padded_kernel", 154624))}


def kitti_leg(args, ctx, dev, world: int, rank: int):
    """BASELINE configs[3]: KITTI-shaped 1242x375 sequences, one per GPU (seed
    s + rank, sequences s..s+7 at 8 GPUs), 128 objects, the full loop; frames of
    all ranks / max time.  Reported, never `value`."""
    import torch
    from opencv_amd import klt, tbd

    w, h, n, skip = 1242, 375, args.kitti_frames, 20
    frames, gt = klt.synth_render(args.seed + rank, w, h, args.objects, 0, n, device=dev, ctx=ctx)
    dets = [tbd.detections_from_gt(gt[f].numpy()) for f in range(n)]
    cfg = tbd.default_config(w, h, win=args.win, max_level=args.max_level, redetect_every=args.redetect)
    stream = torch.cuda.current_stream()
    fl = [frames[f] for f in range(skip, n)]
    packed = tbd.TbdLoop.pack_detections(dets[skip:])
    fps = []
    for _ in range(3):
        loop = tbd.TbdLoop(cfg, ctx=ctx)
        for f in range(skip):
            loop.step(frames[f], f, dets[f], stream)
        el = timed_on_all_ranks(lambda: loop.run(fl, skip, None, stream, packed=packed), world)
        fps.append(replica_throughput(len(fl), world, el))
        del loop
    del frames
    return {"value": round(sorted(fps)[1], 2), "unit": "frames/s", "runs_fps": [round(v, 1) for v in fps],
            "n_gpus": world, "config": {"workload": f"TBD loop {w}x{h} x {args.objects} objects (BASELINE configs[3]),"
                                                    f" one sequence per GPU (seeds s..s+{world - 1})",
                                        "frames_timed": len(fl), "tracker_bounds": "reference"}}


PYR_KERNELS = ("pyr_build_kernel", "pad_copy_kernel", "pyr_down_padded_kernel", "scharr_levels_kernel")


def pmc_bytes(kernel_substrs):
    """Sum over kernels of the committed loop-only PMC summary's per-launch
    bytes (profiles/rNN_pmc_loop.json, see pmc_traffic; raw FETCH_SIZE,
    FETCH_SIZE x2 as the guide's wide-read correction, WRITE_SIZE); None when
    no summary covers them."""
    d, files = _pmc_summaries("_pmc_loop.json")
    for f in reversed(files):
        k = json.load(open(os.path.join(d, f)))["kernels"]
        hit = [(n, v) for n, v in k.items() if any(s in n for s in kernel_substrs)
               and v.get("fetch_bytes") is not None and v.get("write_bytes") is not None]
        if hit:
            raw = sum(v["fetch_size_kib"] * 1024 for _, v in hit)
            return {"source": f, "kernels": [n.split("(")[0] for n, _ in hit], "fetch_raw": raw,
                    "fetch_x2": 2 * raw, "write": sum(v["write_bytes"] for _, v in hit)}
    return None


class RehearsalMeasure:
    """Stands in for TbdMeasure in `--rehearse` runs (no GPU): records its
    seed, sleeps `ms` per step."""

    def __init__(self, ms: float):
        self.ms, self.seed = ms, None

    def prepare(self, seed: int):
        self.seed = seed

    def warmup(self, w: int):
        time.sleep(self.ms * w / 1000.0)

    def timed(self, k: int):
        time.sleep(self.ms * k / 1000.0)
        return [None] * k


def rehearse(args, world: int, rank: int):
    """The contract (rank group, seeds, barriers, max-over-ranks time, one line
    on rank 0) with RehearsalMeasure instead of the GPU loop; rank r is
    (1 + r) times slower, so the job time is the last rank's."""
    import torch.distributed as dist

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    m = RehearsalMeasure(args.rehearse * (1 + rank))
    line, _ = run_contract(args, world, rank, m, lambda: None, "cpu", cpu_leg=None)
    line.update({"dtype": "u8", "data": "rehearsal (no GPU work: each step sleeps)",
                 "config": {"workload": "bench.py --rehearse", "parallelism": f"replicas x{world}"}})
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return line


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=480)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--sequence-frames", type=int, default=500,
                    help="frames rendered per GPU (configs[2]'s sequence); the timed steps are frames "
                         "[warmup, warmup + steps) of it")
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
    ap.add_argument("--cpu-baseline-seconds-1t", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pin", action="store_true", help="do not pin the rank to its GPU's NUMA-local CPUs")
    ap.add_argument("--api", choices=["run", "ahead", "step"], default="run",
                    help="run: tbdk_tbd_run (native frame loop with look-ahead); ahead: per-frame "
                         "tbdk_tbd_step_ahead; step: per-frame tbdk_tbd_step (no look-ahead)")
    ap.add_argument("--lk-impl", type=int, default=0, help="PyrLK kernel (ctx option lk_impl; 0 auto)")
    ap.add_argument("--early-gftt", type=int, default=2, choices=[0, 1, 2],
                    help="ctx option tbd_early_gftt (A/B runs; 0 off, 1 new tracks, 2 + re-detection boxes)")
    ap.add_argument("--no-spec-lookahead", action="store_true", help="ctx option tbd_spec_lookahead = 0 (A/B runs)")
    ap.add_argument("--no-zero-copy", action="store_true", help="ctx option tbd_zero_copy = 0 (A/B runs)")
    ap.add_argument("--ctx-option", action="append", default=[], metavar="NAME=VALUE",
                    help="extra tbdk_ctx_set_option before the legs (A/B runs), repeatable")
    ap.add_argument("--pyr-derivs", action="store_true",
                    help="ctx option tbd_pyr_derivs = 1: loop pyramids with Scharr planes (A/B runs)")
    ap.add_argument("--timing-every", type=int, default=10,
                    help="HIP events on a pseudo-random 1/N of the timed kernels' launches in the timed region "
                         "(N = 10: ~90 PyrLK launches sampled over 480 frames; the events' host work costs the "
                         "frame ~0.9 %% at 10, ~1.8 %% at 5)")
    ap.add_argument("--kstats", default="lk_sparse",
                    help="kernels timed with HIP events in the timed region (comma list, 'all' or 'none'); "
                         "each timed launch adds two event records to the frame's host work.  The other "
                         "kernels are timed in a separate pass over the same frames (not `value`)")
    ap.add_argument("--repeats", type=int, default=5, help="runs of the whole sequence (median reported)")
    ap.add_argument("--no-secondary", action="store_true", help="only the contract line (A/B runs)")
    ap.add_argument("--no-step-api", action="store_true", help="skip the secondary per-frame tbdk_tbd_step pass")
    ap.add_argument("--no-h2d", action="store_true", help="skip the with-H2D (tbdk_tbd_run_host) variant")
    ap.add_argument("--no-kitti", action="store_true", help="skip the KITTI-shaped configs[3] measurement")
    ap.add_argument("--no-bounds-frame", action="store_true",
                    help="skip the secondary leg with the tracker's bounds at the frame (every object propagated)")
    ap.add_argument("--no-pyr4k", action="store_true", help="skip the 4K u8 levels-only pyramid roofline leg")
    ap.add_argument("--kitti-frames", type=int, default=500)
    ap.add_argument("--no-farneback", action="store_true", help="skip the secondary dense Farneback measurement")
    ap.add_argument("--fb-width", type=int, default=3840)
    ap.add_argument("--fb-height", type=int, default=2160)
    ap.add_argument("--fb-objects", type=int, default=512)
    ap.add_argument("--fb-pairs", type=int, default=10)
    ap.add_argument("--no-f16", action="store_true", help="skip the secondary fp16 pixel path measurement")
    ap.add_argument("--f16-pairs", type=int, default=10)
    ap.add_argument("--no-copy-peak", action="store_true", help="skip the measured HBM stream-copy peak")
    ap.add_argument("--no-hog", action="store_true", help="skip the secondary HOG detector measurement")
    ap.add_argument("--no-dense", action="store_true", help="skip the secondary dense PyrLK measurement")
    ap.add_argument("--dense-pairs", type=int, default=5)
    ap.add_argument("--hog-width", type=int, default=1920)
    ap.add_argument("--hog-height", type=int, default=1080)
    ap.add_argument("--hog-frames", type=int, default=60)
    ap.add_argument("--rehearse", type=float, default=None, metavar="MS_PER_STEP",
                    help="rehearse the multi-rank contract with no GPU: every step of rank r sleeps "
                         "MS_PER_STEP x (1 + r) ms (tests/test_bench_dist.py); the line says data: rehearsal")
    args = ap.parse_args(argv)
    argv = list(sys.argv[1:] if argv is None else argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: this process starts the N ranks itself (before any GPU call)
        raise SystemExit(spawn_ranks(argv, args.gpus))
    world, rank, local = rank_env()
    check_world(args.gpus, world)
    if args.rehearse is not None:
        return rehearse(args, world, rank)
    if args.no_secondary:
        args.no_step_api = args.no_h2d = args.no_kitti = args.no_farneback = args.no_f16 = args.no_hog = True
        args.no_dense = True
        args.no_bounds_frame = args.no_pyr4k = True
        args.no_copy_peak = True
        args.repeats = 0

    full_affinity = os.sched_getaffinity(0)
    pin = {"pinned": False, "reason": "--no-pin"} if args.no_pin else pin_rank(local)  # before any GPU call

    import torch
    import torch.distributed as dist

    init_rank_group(world, rank, local)
    dev = torch.cuda.current_device()
    if not args.no_pin and not pin.get("pinned") and "already" not in pin.get("reason", ""):
        first = pin.get("reason")
        pin = pin_rank_by_device(dev)
        pin["sysfs_before_init"] = first

    from opencv_amd import klt, tbd

    ctx = klt.Context.get(dev)
    if args.lk_impl:
        ctx.set_option("lk_impl", args.lk_impl)
    ctx.set_option("tbd_early_gftt", args.early_gftt)
    ctx.set_option("tbd_spec_lookahead", 0 if args.no_spec_lookahead else 1)
    ctx.set_option("tbd_zero_copy", 0 if args.no_zero_copy else 1)
    ctx.set_option("tbd_pyr_derivs", 1 if args.pyr_derivs else 0)
    for kv in args.ctx_option:
        name, _, val = kv.partition("=")
        ctx.set_option(name, int(val))

    m = TbdMeasure(args, ctx, dev)
    # the CPU baseline (rank 0, N = 1) runs after every GPU leg: 20 s of all-core
    # host load between the timed region and the secondary GPU legs left those
    # legs measuring a cooled-down device (whole-sequence repeats ~9 % below
    # the timed region right after it)
    line, ms = run_contract(args, world, rank, m, torch.cuda.synchronize, "cpu", cpu_leg=None)
    nb = 60  # frames handed to the CPU baseline (it stops at its time budget)
    cpu_in = (m.frames[:nb].cpu().numpy(), m.gtn[:nb]) if (rank == 0 and world == 1 and
                                                          not args.no_cpu_baseline) else None
    stream, cfg, frames, dets = m.stream, m.cfg, m.frames, m.dets
    timed = m.timed_kernels
    lk_pts = lk_it = klt_pts = ntr = redet = early = 0
    h_wait = h_trk = h_step = h_launch = 0.0
    for x in ms:
        lk_pts += x.lk_points
        lk_it += x.lk_iters
        klt_pts += x.klt_points
        ntr += x.ntracks
        redet += x.redetected
        early += x.early_gftt
        h_wait += x.host_wait_us
        h_trk += x.host_tracker_us
        h_step += x.host_step_us
        h_launch += x.host_launch_us
    kstats = {}
    for name in timed:
        c, t_ms = ctx.timing_query(name)
        kstats[name] = {"launches": ctx.timing_calls(name), "timed_launches": c,
                        "avg_us": (t_ms / c * 1000.0) if c else None, "total_ms_timed": t_ms}
    ctx.timing_enable(False)
    ctx.timing_select(None)
    ctx.set_option("timing_every", 1)
    nolaunch = {"launches": 0, "avg_us": None, "total_ms": 0.0}
    w0, nframes = args.warmup, args.warmup + args.steps

    # the whole-sequence and with-H2D legs right after the timed region: the
    # per-frame step-API pass below leaves the device in a state that measured
    # the sequence ~7 % lower when it ran first
    if args.repeats > 0:
        progress("whole-sequence repeats", rank)
        line["sequence"] = sequence_repeats(m, world, args.repeats, 20)
    if not args.no_h2d:
        progress("with-H2D variant", rank)
        line["with_h2d"] = with_h2d(m, world, 3, 20)
    if not args.no_bounds_frame and args.bounds == "reference":
        progress("bounds-frame variant", rank)
        line["bounds_frame"] = bounds_frame_leg(m, world, 3, 20)

    # secondary: the same frames through the per-frame tbdk_tbd_step API (no
    # look-ahead), a fresh loop, no timing events; reported, never `value`
    step_api = None
    if args.api != "step" and not args.no_step_api:
        progress("step-API pass", rank)
        loop2 = m.new_loop(w0)
        el2 = timed_on_all_ranks(lambda: [loop2.step(frames[f], f, dets[f], stream) for f in range(w0, nframes)],
                                 world)
        step_api = {"value": round(replica_throughput(args.steps, world, el2), 2), "unit": "frames/s",
                    "api": "tbdk_tbd_step per frame from Python"}
        del loop2

    # the kernels not timed in the timed region: a separate pass over the same
    # frames with events on every launch (a fresh loop; its wall time is not reported)
    # lk_sparse is always in it: its every-launch average checks the sampled one
    rest = [k for k in ("pyr_build", "lk_sparse", "gftt", "tbd_fit") if k not in timed or k == "lk_sparse"]
    kstats_aside = {}
    if rest:
        progress("per-kernel event pass", rank)
        loop3 = m.new_loop(w0)
        ctx.timing_select(rest)
        ctx.timing_enable(True)
        loop3.run(m.frame_list, w0, None, stream, packed=m.packed)
        torch.cuda.synchronize()
        for name in rest:
            c, t_ms = ctx.timing_query(name)
            kstats_aside[name] = {"launches": c, "avg_us": (t_ms / c * 1000.0) if c else None, "total_ms": t_ms}
        ctx.timing_enable(False)
        ctx.timing_select(None)
        del loop3

    lk = kstats.get("lk_sparse", kstats_aside.get("lk_sparse", nolaunch))
    nlev = args.max_level + 1
    lk_every = kstats_aside.get("lk_sparse", {}).get("avg_us")
    # the line's achieved / frac: the every-launch average (the separate pass over the same frames:
    # every PyrLK launch of the loop, ~900 at 480 frames), not the timed region's sampled events
    # (a pseudo-random 1/N of its launches: 5 at the driver's --steps 20); sampled figures beside it
    lk_avg = lk_every if lk_every else lk["avg_us"]
    if lk["launches"] and lk_avg:
        flops_per_launch = lk_flops(lk_pts * nlev, lk_it, args.win) / lk["launches"]
        achieved = flops_per_launch / (lk_avg * 1e-6) / 1e12
    else:
        flops_per_launch, achieved = 0.0, 0.0
    # the auto choice is lk_multi_kernel (several points per wave) for the odd square windows it covers
    # the loop's FLY instance (lk_multi_kernel<W, W, true, false>: FLY, not the dense mode)
    traffic, traffic_src = pmc_traffic(f"lk_multi_kernel<{args.win}, {args.win}, true, false>")
    if traffic is None:  # summaries written before the dense mode's template argument existed
        traffic, traffic_src = pmc_traffic(f"lk_multi_kernel<{args.win}, {args.win}, true>")
    if traffic is None:
        traffic, traffic_src = pmc_traffic(f"lk_strip_kernel<{args.win}, {args.win}>")
    kt_loop = ktrace_loop_avg_us(f"void tbdk::lk_multi_kernel<{args.win}, {args.win}, true, false>")
    roofline = {"bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_F32_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_F32_TFLOPS, 4), "traffic": traffic, "kernel": "lk_sparse",
                "traffic_source": traffic_src,
                "note": "PyrLK is VALU (int16 dot2 + fp32) bound, no MFMA (no contraction on this path); peak = "
                        "fp32 vector rate; algorithmic flops per SURVEY.md §8(d) with the measured iteration "
                        "count per launch of the timed region; launch duration = avg_us_every_launch (HIP events "
                        "on every PyrLK launch of a separate pass over the same frames, on the launch stream); "
                        f"avg_us_sampled / frac_sampled: events on a pseudo-random 1/{args.timing_every} of the "
                        "timed region's own launches; traffic = raw FETCH_SIZE + WRITE_SIZE per launch "
                        "(committed PMC summary, no x2: the kernel's global loads are 4 B per lane, the guide's x2 "
                        "is for 16 B/lane streaming reads)",
                "access_width": "global_load_dword (4 B/lane, u8 rows as unaligned dwords); stores 8 B/lane",
                "avg_us": round(lk_avg, 3) if lk_avg else None,
                "duration_source": "every launch (separate pass)" if lk_every else "sampled launches",
                "avg_us_sampled": lk["avg_us"],
                "timed_launches_sampled": lk.get("timed_launches", lk["launches"]),
                "frac_sampled": (round(flops_per_launch / (lk["avg_us"] * 1e-6) / 1e12 / PEAK_F32_TFLOPS, 4)
                                 if lk["avg_us"] else None),
                "avg_us_every_launch": lk_every,
                "avg_us_kernel_trace_loop": kt_loop[0], "kernel_trace_loop_calls": kt_loop[1],
                "kernel_trace_loop_source": kt_loop[2],
                "frac_kernel_trace_loop": (round(flops_per_launch / (kt_loop[0] * 1e-6) / 1e12 / PEAK_F32_TFLOPS, 4)
                                           if kt_loop[0] else None),
                "frac_every_launch": (round(flops_per_launch / (lk_every * 1e-6) / 1e12 / PEAK_F32_TFLOPS, 4)
                                      if lk_every else None),
                "flops_per_launch": flops_per_launch,
                "mean_points_per_launch": lk_pts / max(1, lk["launches"]),
                "mean_iters_per_point": lk_it / max(1, lk_pts)}
    pb = pyr_bytes(args.width, args.height, nlev)
    borrow = "tbd_borrow_l0=1" in [kv.replace(" ", "") for kv in args.ctx_option] and not args.pyr_derivs
    pbb = pyr_build_bytes(args.width, args.height, nlev, copy_l0=not borrow)
    pyr = kstats.get("pyr_build", kstats_aside.get("pyr_build", nolaunch))
    pyr_gbs = pbb / (pyr["avg_us"] * 1e-6) / 1e9 if pyr["launches"] else 0.0
    cnt = pmc_bytes(PYR_KERNELS)
    cp_pyr = copy_rate_at(ctx, pbb) if not args.no_copy_peak else None
    kt_us, kt_used, kt_src = ktrace_grid_us(("pyr_build_kernel", "pyr_down_padded_kernel"), "most")
    # the same build uncontended (the loop's runs beside the critical PyrLK since round 5)
    sa_pyr = standalone_pyr(ctx, args.width, args.height) if not args.no_pyr4k else None
    roof_pyr = {"bound": "hbm", "achieved": round(pyr_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(pyr_gbs / PEAK_HBM_GBS, 4), "bytes_per_launch": pbb, "b_pyr_survey": pb,
                "size_matched_copy": cp_pyr,
                "frac_size_matched_copy": round(pyr_gbs / cp_pyr["gbs"], 4) if cp_pyr else None,
                "kernel_trace_us": kt_us, "kernel_trace_launches": kt_used, "kernel_trace_source": kt_src,
                "frac_kernel_trace": round(pbb / (kt_us * 1e-6) / 1e9 / PEAK_HBM_GBS, 4) if kt_us else None,
                "kernel": "pyr_build",
                "traffic": (cnt["fetch_raw"] + cnt["write"]) if cnt else None,
                "traffic_fetch_x2": (cnt["fetch_x2"] + cnt["write"]) if cnt else None,
                "traffic_over_algorithmic": round((cnt["fetch_raw"] + cnt["write"]) / pbb, 3) if cnt else None,
                "traffic_kernels": cnt["kernels"] if cnt else None, "traffic_source": cnt["source"] if cnt else None,
                "level0": "the frame itself (tbd_borrow_l0: no padded copy)" if borrow else "padded copy",
                "standalone": sa_pyr,
                "frac_standalone": round(pyr_build_bytes(args.width, args.height, nlev) / (sa_pyr["avg_us"] * 1e-6)
                                         / 1e9 / PEAK_HBM_GBS, 4) if sa_pyr else None,
                "note": "achieved = the loop's build's algorithmic bytes (frame read once, every padded level "
                        "written -- from level 1 on when level 0 is the frame itself --, levels >= 2 reading their "
                        "predecessor; bytes_per_launch) / the build's HIP-event time (its launches); b_pyr_survey = "
                        "SURVEY §8d's B_pyr (no level-0 copy); traffic = FETCH_SIZE + WRITE_SIZE per build from the "
                        "committed PMC summary (4-byte loads: no x2)"}
    # north_star's "HBM-read roofline on pyramid+PyrLK": SURVEY §8d bytes B_pyr + B_lk + N*21,
    # with B_lk at its upper bound (2 full pyramids), over the two stages' summed time
    w_, h_, lv_bytes = args.width, args.height, 0
    for _ in range(nlev):
        lv_bytes += w_ * h_
        w_, h_ = (w_ + 1) // 2, (h_ + 1) // 2
    b_lk = 2 * lv_bytes + 21 * (lk_pts / max(1, args.steps))
    t_pl = ((pyr["avg_us"] or 0.0) + (lk["avg_us"] or 0.0)) * 1e-6
    hbm_pl = (pbb + b_lk) / t_pl / 1e9 if t_pl > 0 else 0.0
    roof_pl = {"bound": "hbm", "achieved": round(hbm_pl, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
               "frac": round(hbm_pl / PEAK_HBM_GBS, 4), "bytes_per_frame": pbb + b_lk,
               "kernels": "pyr_build + lk_sparse",
               "note": "B_lk taken at its SURVEY §8d upper bound (2 full pyramids); PyrLK is compute-bound "
                       "(~360 flop/B vs ridge ~20), so this fraction is structurally small (DESIGN.md §3)"}

    line.update({
        "dtype": "u8",
        "data": "synthetic (deterministic in-repo generator, opencv_amd/csrc/synth_spec.h)",
        "config": {"workload": f"TBD loop {args.width}x{args.height} x {args.objects} objects "
                               f"(BASELINE configs[2]), frames [{w0}, {nframes}) of a {m.nseq}-frame sequence "
                               "per GPU",
                   "levels": nlev, "win": args.win, "gftt": f"256/box, q 0.01, minDist 3, every {args.redetect}",
                   "tracker_bounds": args.bounds, "parallelism": f"replicas x{world} (one sequence per GPU)",
                   "api": {"run": "tbdk_tbd_run (native frame loop, look-ahead)",
                           "ahead": "tbdk_tbd_step_ahead per frame", "step": "tbdk_tbd_step per frame"}[args.api]},
        "host_pinning": pin,
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
    })
    del m.frames, frames, m.loop
    if not args.no_kitti:
        progress("KITTI configs[3] leg", rank)
        line["kitti"] = kitti_leg(args, ctx, dev, world, rank)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # before any leg imports _oracle: every CPU baseline of the line runs the
        # -O3 -march=native build (native_oracle() is a no-op once _oracle is loaded)
        native_oracle()
    if rank == 0 and not args.no_pyr4k:
        progress("4K pyramid roofline")
        line["roofline_pyramid_4k"] = pyramid_4k_leg(ctx, dev)
    if rank == 0 and not args.no_farneback:
        progress("Farneback secondary")
        line["farneback"] = farneback_secondary(ctx, args, dev, cpu=world == 1 and not args.no_cpu_baseline)
    if rank == 0 and not args.no_f16:
        progress("fp16 PyrLK secondary")
        line["lk_f16"] = lk_f16_secondary(ctx, args, dev, cpu=world == 1 and not args.no_cpu_baseline)
    if rank == 0 and not args.no_dense:
        progress("dense PyrLK secondary")
        line["dense_lk"] = dense_lk_secondary(ctx, args, dev, cpu=world == 1 and not args.no_cpu_baseline)
    if rank == 0 and not args.no_hog:
        progress("HOG secondary")
        line["hog"] = hog_secondary(ctx, args, dev, cpu=world == 1 and not args.no_cpu_baseline)
    if rank == 0 and not args.no_copy_peak:
        progress("HBM copy peak")
        line["hbm_copy_peak"] = hbm_copy_peak(dev, ctx)
        add_copy_peak_fracs(line, line["hbm_copy_peak"]["value"])
    if cpu_in is not None:
        progress("cpu baseline")
        line["cpu_baseline"] = cpu_baseline_line(cpu_in[0], cpu_in[1], args, restore_affinity=full_affinity)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
