"""Per-wave timeline of the lk_multi launches (probe build with -DTBDK_LK_TRACE:
opencv_amd/lib/libtbdk_trace.so, selected by TBDK_LIB).  Each wave records its
start / end (s_memrealtime, 10 ns), HW_ID / XCC_ID, its Newton steps, J reloads
and the max iterations of its points.

  loop        the TBD loop of bench.py's configs[2] (1080p x 128), frames
              [20, 20 + F) traced, every PyrLK launch of the frame
  standalone  GFTT corners (256 per box) of frame 0's boxes tracked into frame 1
              in several point orders (natural, by iterations descending /
              ascending, shuffled) -- how order and grouping move the tail

Prints a per-launch summary and writes the raw records to gpurun_out/."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from opencv_amd import klt, tbd

CAP = 1 << 19  # records
TICK_US = 0.01


def arm(lib, buf):
    buf.zero_()
    torch.cuda.synchronize()
    assert lib.tbdk_probe_lk_trace(C.c_void_p(buf.data_ptr()), C.c_uint(16 * CAP)) == 0


def records(lib, buf):
    n = C.c_uint()
    assert lib.tbdk_probe_lk_trace_count(C.byref(n)) == 0
    n = min(n.value, CAP)
    r = buf[: 16 * n].view(-1, 16).cpu().numpy().view(np.uint64)
    return r[r[:, 0] != 0]  # waves with no valid point exit before recording


def split_launches(r):
    """records -> list of launches (key, n, records sorted by start): same key
    and n, starts within 400 us of the previous wave of that group"""
    out = []
    order = np.argsort(r[:, 0], kind="stable")
    r = r[order]
    groups = {}
    for row in r:
        key = (int(row[4]), int(row[3] >> 32))
        g = groups.get(key)
        if g is None or row[0] - g[-1][-1][0] > 40000:
            groups.setdefault(key, []).append([row])
        else:
            g[-1].append(row)
    for key, ls in groups.items():
        for l in ls:
            out.append((key, np.array(l)))
    out.sort(key=lambda t: t[1][0, 0])
    return out


def summarize(rec, label=""):
    t0 = rec[:, 0].min()
    st = (rec[:, 0] - t0) * TICK_US
    en = (rec[:, 1] - t0) * TICK_US
    dur = en - st
    span = en.max()
    steps = (rec[:, 5] & 0xFFFF).astype(np.int64)
    rel = ((rec[:, 5] >> 16) & 0xFFFF).astype(np.int64)
    mit = ((rec[:, 5] >> 32) & 0xFFFF).astype(np.int64)
    ends = np.sort(en)
    q = lambda f: ends[min(len(ends) - 1, int(f * len(ends)))]
    simd = (rec[:, 2] & 0xFFFFFFFF).astype(np.int64)
    xcc = (rec[:, 2] >> 32).astype(np.int64) & 0xF
    cu = (simd >> 8) & 0xF
    sh = (simd >> 12) & 1
    se = (simd >> 13) & 0x7
    sid = (simd >> 4) & 3
    uniq = len(set(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist(), sid.tolist())))
    occ = dur.sum() / span / 1024.0
    # resident waves over time (1 us bins)
    nb = int(span) + 1
    o = np.zeros(nb + 1)
    for a, b in zip(st, en):
        o[int(a)] += 1
        o[int(b)] -= 1
    o = np.cumsum(o)[:nb]
    last = np.argsort(en)[-5:][::-1]
    ph = rec[:, 6:14].copy().view(np.uint32).astype(np.float64) * TICK_US  # (waves, 16) phase stamps
    phs = []
    for L in (2, 1, 0):
        a0, a1, a2, a3 = ph[:, 4 * L], ph[:, 4 * L + 1], ph[:, 4 * L + 2], ph[:, 4 * L + 3]
        ok = a3 > 0
        if ok.sum():
            phs.append(f"L{L}: setup {np.mean(a1[ok] - a0[ok]):.2f} jload {np.mean(a2[ok] - a1[ok]):.2f} "
                       f"newton {np.mean(a3[ok] - a2[ok]):.2f}")
    e = ph[:, 12]
    ok = e > 0
    if ok.sum():
        phs.append(f"err {np.mean(e[ok] - ph[ok, 3]):.2f}")
    s = (f"{label} waves {len(rec)} span {span:.1f} us; ends p50 {q(.5):.1f} p90 {q(.9):.1f} p99 {q(.99):.1f}; "
         f"starts max {st.max():.1f}; dur p50 {np.median(dur):.1f} p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f}; "
         f"waves/SIMD mean {occ:.2f} (SIMDs used {uniq}); resident peak {o.max():.0f}; "
         f"steps mean {steps.mean():.1f} max {steps.max()}; reloads mean {rel.mean():.2f}; maxit mean {mit.mean():.1f}\n")
    s += "   phases (mean us): " + "; ".join(phs) + "\n"
    s += "   occupancy by 10%% of span: " + " ".join(
        f"{o[int(i * nb / 10):int((i + 1) * nb / 10)].mean() / 1024:.2f}" for i in range(10)) + "\n"
    s += "   last waves (start, dur, steps, reloads, maxit): " + "; ".join(
        f"({st[i]:.1f}, {dur[i]:.1f}, {steps[i]}, {rel[i]}, {mit[i]})" for i in last)
    return s


def run_loop(lib, buf, frames_traced):
    ctx = klt.Context.get(0)
    W, H, NOBJ = 1920, 1080, 128
    nseq = 20 + frames_traced
    frames, gt = klt.synth_render(20261015, W, H, NOBJ, 0, nseq, ctx=ctx)
    gtn = gt.numpy()
    dets = [tbd.detections_from_gt(gtn[f]) for f in range(nseq)]
    cfg = tbd.default_config(W, H, win=21, max_level=2, redetect_every=5)
    loop = tbd.TbdLoop(cfg, ctx=ctx)
    s = torch.cuda.current_stream()
    for f in range(20):
        loop.step(frames[f], f, dets[f], s)
    torch.cuda.synchronize()
    arm(lib, buf)
    list(loop.run([frames[f] for f in range(20, nseq)], 20, dets[20:nseq], s))
    torch.cuda.synchronize()
    return records(lib, buf)


def run_standalone(lib, buf):
    ctx = klt.Context.get(0)
    W, H, NOBJ = 1920, 1080, 128
    frames, gt = klt.synth_render(20261015, W, H, NOBJ, 0, 2, ctx=ctx)
    rois = []
    for v, x, y, w, h in gt[0].numpy().tolist():
        x0, y0 = max(0, x), max(0, y)
        x1, y1 = min(W, x + w), min(H, y + h)
        if v and x1 - x0 >= 8 and y1 - y0 >= 8:
            rois.append((x0, y0, x1 - x0, y1 - y0))
    det = klt.GoodFeaturesToTrackDetector(256, 0.01, 3.0)
    c, n = det.detect_rois(frames[0], rois)
    c, n = c.cpu().numpy(), n.cpu().numpy()
    pts = np.concatenate([c[i, :n[i]] for i in range(len(rois))]).astype(np.float32)
    P0 = klt.Pyramid(ctx, W, H, 2, derivs=False).build(frames[0])
    P1 = klt.Pyramid(ctx, W, H, 2, derivs=False).build(frames[1])
    lk = klt.SparsePyrLKOpticalFlow((21, 21), 2, 30)
    d = torch.from_numpy(pts).cuda()
    r = lk.calc(P0, P1, d, want_iters=True)
    torch.cuda.synchronize()
    it = r.iters.cpu().numpy()
    print(f"standalone: {len(pts)} GFTT points in {len(rois)} boxes; iters mean {it.mean():.2f} p99 "
          f"{np.percentile(it, 99):.0f} max {it.max()}", flush=True)
    rng = np.random.default_rng(1)
    orders = {"natural": np.arange(len(pts)), "iters_desc": np.argsort(-it, kind="stable"),
              "iters_asc": np.argsort(it, kind="stable"), "shuffled": rng.permutation(len(pts))}
    out = {}
    for name, o in orders.items():
        dd = torch.from_numpy(pts[o]).cuda()
        for _ in range(3):
            lk.calc(P0, P1, dd)
        torch.cuda.synchronize()
        ctx.timing_select(["lk_sparse"])
        ctx.timing_enable(True)
        for _ in range(10):
            lk.calc(P0, P1, dd)
        torch.cuda.synchronize()
        cnt, ms = ctx.timing_query("lk_sparse")
        ctx.timing_enable(False)
        arm(lib, buf)
        lk.calc(P0, P1, dd)
        torch.cuda.synchronize()
        rec = records(lib, buf)
        out[name] = rec
        print(summarize(rec, f"[{name}] event avg {ms / cnt * 1000:.1f} us;"), flush=True)
    return out


def main():
    lib = C.CDLL(os.environ["TBDK_LIB"])
    buf = torch.zeros(16 * CAP, dtype=torch.int64, device="cuda")
    mode = sys.argv[1] if len(sys.argv) > 1 else "loop"
    os.makedirs("gpurun_out", exist_ok=True)
    if mode == "standalone":
        out = run_standalone(lib, buf)
        np.savez_compressed("gpurun_out/lk_trace_standalone.npz", **out)
        return
    rec = run_loop(lib, buf, int(sys.argv[2]) if len(sys.argv) > 2 else 20)
    np.savez_compressed("gpurun_out/lk_trace_loop.npz", rec=rec)
    ls = split_launches(rec)
    print(f"loop: {len(rec)} wave records, {len(ls)} launches", flush=True)
    for key, l in ls:
        print(summarize(l, f"[key {key[0] & 0xFFFFF:x} n {key[1]}]"), flush=True)


if __name__ == "__main__":
    main()
