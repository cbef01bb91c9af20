"""The GPU loop against the oracle pipeline in the exact order and in the
reference's SSE2 accumulation order over a whole sequence, for configurations
beside the one tests/test_gpu_tbd_e2e.py asserts (same procedure: GPU-rendered
frames handed to two CPU oracle workers, tests/_loop_worker.py; the oracle runs
here only as the checker).  Writes gpurun_out/loop_divergence_<W>x<H>_<seed>.json.

  python tests/loop_divergence_gpu.py W H OBJECTS FRAMES SEED
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import _loop_compare as LC  # noqa: E402
import tbd_loop_oracle as L  # noqa: E402
from test_gpu_tbd_e2e import METRIC_KEYS, _gpu_rows, _host_cores  # noqa: E402


def main(argv):
    from opencv_amd import klt, tbd

    W, H, N, F, seed = (int(v) for v in argv[1:6])
    ctx = klt.Context.get(0)
    frames, gt = klt.synth_render(seed, W, H, N, 0, F, ctx=ctx)
    ogt = L.O.synth_gt(seed, W, H, N, 0, F)
    assert np.array_equal(gt.numpy(), ogt)
    with tempfile.TemporaryDirectory() as tmp:
        host = frames.cpu().numpy()
        for f0 in (0, F // 2, F - 1):
            assert np.array_equal(host[f0], L.O.synth(seed, W, H, N, f0, 1)[0][0]), f"frame {f0}"
        fpath = os.path.join(tmp, "frames.npy")
        np.save(fpath, host)
        del host
        cores = _host_cores()
        ta = max(1, cores * 5 // 8)
        tb = max(1, cores - ta)
        worker = os.path.join(ROOT, "tests", "_loop_worker.py")
        env = dict(os.environ, HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
        outs = {k: os.path.join(tmp, f"{k}.json") for k in ("exact", "sse2")}
        procs = [subprocess.Popen([sys.executable, worker, str(W), str(H), str(N), str(F), str(seed), k,
                                   "1" if k == "exact" else "0", str(th), outs[k], fpath], env=env)
                 for k, th in (("exact", ta), ("sse2", tb))]
        cfg = tbd.default_config(W, H)
        loop = tbd.TbdLoop(cfg, ctx=ctx)
        dets = [tbd.detections_from_gt(ogt[f]) for f in range(F)]
        gm, grows, gpreds = [], [], []
        for f in range(F):
            m = loop.step(frames[f], f, dets[f], next_frame=frames[f + 1] if f + 1 < F else None)
            gm.append({k: getattr(m, k) for k in METRIC_KEYS})
            grows.append(_gpu_rows(loop.tracks()))
            gpreds.append(loop.predictions())
        torch.cuda.synchronize()
        t0 = time.time()
        for p in procs:
            p.wait(timeout=max(1.0, 900 - (time.time() - t0)))
            assert p.returncode == 0, "oracle worker failed"
        ex, ss = (json.load(open(outs[k])) for k in ("exact", "sse2"))
    exact_frames = 0
    pred_dev = 0.0
    for f in range(F):
        op = {int(k): v for k, v in ex["preds"][f].items()}
        same = gm[f] == ex["metrics"][f] and grows[f] == [tuple(r) for r in ex["rows"][f]] and \
            gpreds[f].keys() == op.keys()
        if same:
            for k, (cx, cy) in gpreds[f].items():
                pred_dev = max(pred_dev, abs(cx - op[k][0]), abs(cy - op[k][1]))
        exact_frames += same
    ls = LC.LoopStats()
    for f in range(F):
        ls.add(f, gm[f], ss["metrics"][f], grows[f], ss["rows"][f])
    report = {"config": {"width": W, "height": H, "objects": N, "frames": F, "seed": seed,
                         "oracle_threads": [ta, tb]},
              "gpu_vs_exact_loop": {"frames_equal": exact_frames, "frames": F, "max_pred_dev_px": pred_dev},
              "gpu_vs_sse2_loop": ls.summary(), "per_call_exact_vs_sse2": ex["shadow"],
              "redetected_total": sum(m["redetected"] for m in gm),
              "klt_predicted_total": sum(m["klt_predicted"] for m in gm)}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    path = os.path.join(ROOT, "gpurun_out", f"loop_divergence_{W}x{H}_{seed}.json")
    with open(path, "w") as fh:
        json.dump(report, fh, indent=1)
    print(json.dumps(report))


if __name__ == "__main__":
    main(sys.argv)
