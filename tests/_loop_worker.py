"""CPU-only worker (TEST INFRASTRUCTURE ONLY): runs the oracle TBD loop
(oracle/tbd_loop_oracle.py) over a synthetic sequence in one PyrLK
accumulation order and writes every frame's metrics, track rows and KLT
predictions as JSON, so tests/test_gpu_tbd_e2e.py can run the exact-order and
the SSE2-order pipelines in two processes beside the GPU loop.  Never touches
the GPU (no torch import).

  python tests/_loop_worker.py W H N F SEED {exact|sse2} SHADOW THREADS OUT.json [FRAMES.npy]

FRAMES.npy (optional): the sequence's frames (F, H, W) u8, memory-mapped, in
place of rendering them with the oracle's generator (the caller checks they
are the generator's frames).
"""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

import numpy as np  # noqa: E402

import tbd_loop_oracle as L  # noqa: E402
import _loop_compare as LC  # noqa: E402


def run(W, H, N, F, seed, accum, shadow, threads, frames_path=None):
    if frames_path:
        frames = np.load(frames_path, mmap_mode="r")
        assert frames.shape == (F, H, W) and frames.dtype == np.uint8
        gt = L.O.synth_gt(seed, W, H, N, 0, F)
    else:
        frames, gt = L.O.synth(seed, W, H, N, 0, F)
    pool = ThreadPoolExecutor(threads) if threads > 1 else None
    lp = L.KltTbdLoop(W, H, accum=L.O.ACCUM_EXACT if accum == "exact" else L.O.ACCUM_SSE2,
                      shadow_accum=L.O.ACCUM_SSE2 if shadow else None, nthreads=threads, gftt_pool=pool)
    cs = LC.CallStats()
    out = {"metrics": [], "rows": [], "preds": []}
    for f in range(F):
        m = lp.step(np.ascontiguousarray(frames[f]) if frames_path else frames[f], f, L.detections(gt[f], f))
        cs.add(lp.shadow)
        out["metrics"].append(m)
        out["rows"].append([list(r) for r in lp.track_rows()])
        out["preds"].append({str(k): [float(v[0]), float(v[1])] for k, v in lp.preds.items()})
    if pool is not None:
        pool.shutdown()
    out["shadow"] = cs.summary() if shadow else None
    return out


def main(argv):
    W, H, N, F, seed = (int(v) for v in argv[:5])
    accum, shadow, threads, path = argv[5], bool(int(argv[6])), int(argv[7]), argv[8]
    out = run(W, H, N, F, seed, accum, shadow, threads, argv[9] if len(argv) > 9 else None)
    tmp = path + ".tmp"
    with open(tmp, "w") as fh:
        json.dump(out, fh)
    os.replace(tmp, path)


if __name__ == "__main__":
    main(sys.argv[1:])
