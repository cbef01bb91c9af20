"""The sample's tracking driver (samples/gpu/tbd.cpp: parseBboxFile,
parseDetections, the history-age draw, setTracks from the output buffers,
writeTrackingOutputToFile) in libtbdk (tbd_app.cpp) against the pure-Python
restatement oracle/tbd_app_oracle.py: output files byte-identical, metrics
equal.  Host only (no GPU).

Parity pinning: the glibc rand() restatement is checked against this host's
libc; the file formats and the metric arithmetic have no reference-produced
fixture (the sample's outputs are not in the reference tree), so beyond that
the two restatements are checked against each other — parity unpinned
against reference outputs."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import tbd_app_oracle as A  # noqa: E402
import tbd_oracle as T  # noqa: E402
from opencv_amd import _lib, tbd  # noqa: E402

# TBDK_APP: another build of the CLI (tests/test_host_sanitizers.py runs a sanitized one)
APP = os.environ.get("TBDK_APP") or os.path.join(ROOT, "opencv_amd", "bin", "tbdk_tbd_app")


def write_gt_file(path, seed, nobj=24, nframes=60, start=0, w=1280, h=720, poses=False, history=None,
                  world=False, crlf=False, extra_frames=0, drop_frames=()):
    """Ground-truth bbox file in the sample's format frame|id|x1|x2|y1|y2[|wx|wy[|wz]]:
    moving boxes (some leave the window, some cross), per-frame dropouts."""
    rng = np.random.default_rng(seed)
    pos = rng.uniform([0, 0], [w - 100, h - 100], size=(nobj, 2))
    vel = rng.uniform(-9, 9, size=(nobj, 2))
    size = rng.uniform(30, 140, size=(nobj, 2))
    ids = rng.permutation(1000)[:nobj]
    lines = []
    if history is not None:
        lines.append("history|" + ",".join(str(a) for a in history))
    nl = "\r\n" if crlf else "\n"
    for f in range(nframes + extra_frames):
        fn = start + f
        if f in drop_frames:
            continue
        if poses:
            lines.append(f"{fn}|-1|{rng.uniform(-5, 5):.3f}|{rng.uniform(-5, 5):.3f}|{rng.uniform(0, 360):.2f}")
        for k in range(nobj):
            if rng.random() < 0.08:   # missed in this frame
                continue
            x1, y1 = pos[k] + vel[k] * f + rng.normal(0, 1.5, 2)
            x2, y2 = x1 + size[k][0] + rng.normal(0, 2), y1 + size[k][1] + rng.normal(0, 2)
            row = f"{fn}|{ids[k]}|{x1:.2f}|{x2:.2f}|{y1:.2f}|{y2:.2f}"
            if world:
                row += f"|{rng.uniform(-50, 50):.3f}|{rng.uniform(-50, 50):.3f}"
                if k % 2:
                    row += f"|{rng.uniform(0, 3):.3f}"
            lines.append(row)
    with open(path, "w", newline="") as fh:
        fh.write(nl.join(lines) + nl)


def write_det_file(path, seed, nframes=40, w=1280, h=720):
    """External-detection file frame|x1|x2|y1|y2 (no ids), with false positives."""
    rng = np.random.default_rng(seed)
    lines = ["# comment line without separators"]
    for f in range(nframes):
        for _ in range(rng.integers(0, 12)):
            x1, y1 = rng.uniform(0, w - 80), rng.uniform(0, h - 80)
            lines.append(f"{f}|{x1:.1f}|{x1 + rng.uniform(20, 80):.1f}|{y1:.1f}|{y1 + rng.uniform(20, 80):.1f}")
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")


# ---- glibc rand() ----

@pytest.mark.parametrize("seed", [1, 0, 42, 2**31 + 5, 2**32 - 1])
def test_rand_matches_libc(seed):
    libc = ctypes.CDLL(None)
    libc.srand(ctypes.c_uint(seed))
    ref = [libc.rand() for _ in range(3000)]
    r = tbd.CRand(seed)
    assert [r.rand() for _ in range(3000)] == ref
    o = A.CRand(seed)
    assert [o.rand() for _ in range(3000)] == ref


@pytest.mark.parametrize("arg", ["1", "7,3", "5,3,2", "0.2,0.2,0.6", "1,1,1,1,1,1,1", " 2,  3"])
def test_history_distribution_and_draw(arg):
    nat = tbd.parse_history_distribution(arg)
    ora = A.parse_history_distribution(arg)
    assert np.array_equal(np.float32(nat), np.float32(ora))
    r, o = tbd.CRand(7), A.CRand(7)
    assert [r.history_age(nat) for _ in range(2000)] == [A.draw_history_age(o, ora) for _ in range(2000)]


def test_history_distribution_bad():
    with pytest.raises(_lib.TbdkError):
        tbd.parse_history_distribution("a,b")
    with pytest.raises(A.ParseError):
        A.parse_history_distribution("a,b")


# ---- parseBboxFile / parseDetections ----

def _seq_both(path, nframes, cls=0):
    seq = tbd.Sequence()
    seq.parseBboxFile(path, nframes, cls)
    poses, hist = [], []
    table = A.parse_bbox_file(path, nframes, poses, hist)
    return seq, table, poses, hist


@pytest.mark.parametrize("kw", [dict(), dict(start=7), dict(poses=True, world=True), dict(crlf=True),
                                dict(history=[1, 2, 1, 3]), dict(extra_frames=15), dict(drop_frames=(0, 3, 4, 30)),
                                dict(start=5, drop_frames=(0,))])
def test_parse_bbox_file(tmp_path, kw):
    p = str(tmp_path / "gt.txt")
    write_gt_file(p, 11, nframes=40, **kw)
    seq, table, poses, hist = _seq_both(p, 40)
    nf, npose, nh = seq.info()
    assert nf == len(table) and npose == len(poses) and nh == len(hist)
    assert seq.history() == hist
    for i, pz in enumerate(poses):
        assert seq.cameraPose(i) == pz
    nt, no = tbd.Trajectories(), {}
    for f in range(40):
        d = seq.detections(f, trajectories=nt)
        o = A.parse_detections(table, f, no)
        assert [tuple(x) for x in d[["id", "x", "y", "width", "height"]].tolist()] == \
            [(x.id, x.bbox.x, x.bbox.y, x.bbox.width, x.bbox.height) for x in o]
    assert len(nt) == len(no)


def test_parse_detection_file(tmp_path):
    p = str(tmp_path / "det.txt")
    write_det_file(p, 3)
    seq, table, _, _ = _seq_both(p, 40)
    for f in range(40):
        d = seq.detections(f)
        o = A.parse_detections(table, f, None)
        assert len(d) == len(o) and all(d["id"] == -2)
        assert [tuple(x) for x in d[["x", "y", "width", "height"]].tolist()] == \
            [(x.bbox.x, x.bbox.y, x.bbox.width, x.bbox.height) for x in o]


@pytest.mark.parametrize("text", ["x|1|2|3|4|5\n", "1|2|3|4|5|\n", "3|7|1|2|abc|4\n"])
def test_parse_errors(tmp_path, text):
    p = str(tmp_path / "bad.txt")
    open(p, "w").write(text)
    seq = tbd.Sequence()
    with pytest.raises(_lib.TbdkError):
        seq.parseBboxFile(p, 10)
    with pytest.raises(A.ParseError):
        A.parse_bbox_file(p, 10, [], [])


def test_missing_and_empty_files(tmp_path):
    for p in [str(tmp_path / "absent.txt"), str(tmp_path / "empty.txt")]:
        if "empty" in p:
            open(p, "w").close()
        seq, table, _, _ = _seq_both(p, 25)
        assert seq.info()[0] == len(table) == 0


# ---- the driver end to end: output files byte-identical ----

def _run_both(tmp_path, ped=None, veh=None, tag="a", **kw):
    outs = [str(tmp_path / f"ped_{tag}.txt"), str(tmp_path / f"veh_{tag}.txt")]
    r = tbd.run_app(pedestrian_bbox_filename=ped, vehicle_bbox_filename=veh,
                    pedestrian_tracking_filepath=outs[0] if ped else None,
                    vehicle_tracking_filepath=outs[1] if veh else None,
                    history_distribution=kw.get("history_distribution"),
                    num_tracking_iters=kw.get("num_iters", 1), num_tracking_frames=kw.get("num_frames", 60),
                    seed=kw.get("seed", 1))
    res, log = A.app_run(ped, veh, num_frames=kw.get("num_frames", 60), num_iters=kw.get("num_iters", 1),
                         history_distribution=kw.get("history_distribution"), seed=kw.get("seed", 1))
    for c, f in enumerate([ped, veh]):
        if not f:
            continue
        want = "".join(it[c][0] for it in res)
        got = open(outs[c]).read()
        assert got == want, f"class {c}: native output differs from the oracle"
        m = res[-1][c][1]
        s = r["scenario"][c]
        for k in ("mt", "pt", "ml", "idsw", "fm", "frames"):
            assert s[k] == m[k], k
        for k in ("mota", "amota", "motp"):
            assert (np.isnan(s[k]) and np.isnan(m[k])) or s[k] == m[k], k
    return r, res


@pytest.mark.parametrize("hist", [None, "7,3", "5,3,2", "1,1,1,1"])
def test_app_matches_oracle(tmp_path, hist):
    ped = str(tmp_path / "ped.txt")
    write_gt_file(ped, 21, nobj=30, nframes=60, poses=True)
    r, res = _run_both(tmp_path, ped=ped, history_distribution=hist, num_frames=60)
    m = res[0][0][1]
    assert m["frames"] == 60 and m["mt"] + m["pt"] + m["ml"] > 20


def test_app_two_classes_iterations_provided_history(tmp_path):
    ped, veh = str(tmp_path / "ped.txt"), str(tmp_path / "veh.txt")
    rng = np.random.default_rng(5)
    write_gt_file(ped, 31, nobj=20, nframes=50, start=3, history=list(rng.integers(1, 4, 50)))
    write_gt_file(veh, 32, nobj=12, nframes=50, start=3, world=True)
    _run_both(tmp_path, ped=ped, veh=veh, history_distribution="2,1,1", num_frames=50, num_iters=2)


def test_app_detection_file_and_id_switches(tmp_path):
    det = str(tmp_path / "det.txt")
    write_det_file(det, 9, nframes=40)
    _run_both(tmp_path, ped=det, num_frames=40, tag="d")
    # crossing objects with dropouts: ID switches and fragmentations occur
    ped = str(tmp_path / "cross.txt")
    with open(ped, "w") as fh:
        for f in range(40):
            for k in range(16):
                if (f + k) % 7 == 0:
                    continue
                x = 100 + k * 60 + (f * 12 if k % 2 else -f * 12)
                y = 200 + (k % 4) * 30
                fh.write(f"{f}|{k}|{x}|{x + 50}|{y}|{y + 50}\n")
    r, res = _run_both(tmp_path, ped=ped, num_frames=40, tag="x")
    m = res[0][0][1]
    assert m["idsw"] > 0 and m["fm"] > 0


def test_app_cli(tmp_path):
    ped = str(tmp_path / "ped.txt")
    write_gt_file(ped, 41, nobj=16, nframes=30)
    out = str(tmp_path / "cli_out.txt")
    p = subprocess.run([APP, "--pedestrian_bbox_filename", ped, "--write_tracking", "true",
                        "--pedestrian_tracking_filepath", out, "--num_tracking_frames", "30",
                        "--history_distribution", "6,4", "--scale", "1.05"], capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr
    res, log = A.app_run(ped, None, num_frames=30, history_distribution="6,4")
    assert open(out).read() == res[0][0][0]
    switches = [ln for ln in p.stdout.splitlines() if ln.startswith("[frame")]
    assert switches == log


# ---- Tracker API pieces: setTracks from the output buffer, colours from rand() ----

def test_tracker_buffers_and_colours(tmp_path):
    ped = str(tmp_path / "ped.txt")
    write_gt_file(ped, 51, nobj=20, nframes=30)
    seq = tbd.Sequence()
    seq.parseBboxFile(ped, 30)
    nt = tbd.Tracker()
    rng = tbd.CRand(1)
    nt.setRand(rng)
    buf = tbd.TrackBuffer(3)
    table = A.parse_bbox_file(ped, 30, [], [])
    ot = T.Tracker()
    ot.rng = A.CRand(1)
    obuf = [[], [], []]
    ntraj, otraj = tbd.Trajectories(), {}
    for f in range(30):
        d = seq.detections(f, trajectories=ntraj)
        od = A.parse_detections(table, f, otraj)
        age = 1 + (f * 7) % 3
        if f >= age:
            nt.setTracks(buf, (f - age) % 3)
            ot.set_tracks(obuf[(f - age) % 3])
        else:
            nt.setTracks(None)
            ot.set_tracks([])
        nt.performTrackingStep(d, f, trajectories=ntraj)
        ot.step(od, f, traj=otraj)
        nt.storeTracks(buf, f % 3)
        obuf[f % 3] = [__import__("copy").deepcopy(t) for t in ot.tracks]
        got = [(t.id, t.x, t.y, t.width, t.height, t.age) for t in nt.getTracks()]
        want = [(t.id, t.bboxes[-1].x, t.bboxes[-1].y, t.bboxes[-1].width, t.bboxes[-1].height, t.age)
                for t in ot.tracks]
        assert got == want, f"frame {f}"
    # same number of rand() draws consumed (3 per created track)
    assert rng.rand() == ot.rng.rand()
    out = str(tmp_path / "o.txt")
    m = tbd.write_tracking_output(nt, [1] * 30, ntraj, 30, out)
    txt, om = A.write_tracking_output(ot, [1] * 30, otraj, 30)
    assert open(out).read() == txt and m["mt"] == om["mt"]


def test_empty_scenario_nan_formatting(tmp_path):
    """No frames stepped: MOTA = 1 - 0/0 prints as the host's printf does."""
    nt = tbd.Tracker()
    out = str(tmp_path / "e.txt")
    tbd.write_tracking_output(nt, [], tbd.Trajectories(), 0, out)
    txt, _ = A.write_tracking_output(T.Tracker(), [], {}, 0)
    assert open(out).read() == txt
