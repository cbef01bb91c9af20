"""tbd_app_oracle.py — pure-Python restatement of the tracking driver of the
reference sample samples/gpu/tbd.cpp (TEST INFRASTRUCTURE ONLY: tests/ use it
as the checker of libtbdk's tbd_app.cpp; the product never imports it).

  glibc rand()/srand()                 stdlib/random_r.c (TYPE_3), the sample's
                                       unseeded rand() (tbd.cpp:71-73, samples/gpu/tbd.cpp:660)
  Trajectory                           modules/trackingbydetection/include/opencv2/tbd.hpp:46-80,
                                       src/tbd.cpp:119-171
  parse_history_distribution           samples/gpu/tbd.cpp:258-291
  parse_bbox_file                      samples/gpu/tbd.cpp:1163-1295
  parse_detections                     samples/gpu/tbd.cpp:1297-1340
  draw_history_age                     samples/gpu/tbd.cpp:656-671
  write_tracking_output                samples/gpu/tbd.cpp:946-1120
  app_run                              samples/gpu/tbd.cpp:479-706, 823-841

C semantics restated: std::stoi/stoul/stod/stof are prefix parses of the field
(decimal forms only here: hex floats, inf/nan spellings and strtod's underflow
ERANGE are not modelled), float32 arithmetic for the history draw (numpy),
std::map default-inserting lookups, iostream double output = printf %g, and
the x86 sign of 0/0 (printed "-nan").
"""
from __future__ import annotations

import math
import re
import sys
import os

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import tbd_oracle as T  # noqa: E402

RAND_MAX = 2147483647


class CRand:
    """glibc random_r TYPE_3: r[i] = r[i-3] + r[i-31] (mod 2^32), output >> 1."""

    def __init__(self, seed: int = 1):
        self.srand(seed)

    def srand(self, seed: int):
        seed &= 0xFFFFFFFF
        if seed == 0:
            seed = 1
        word = seed - (1 << 32) if seed >= (1 << 31) else seed
        st = [word]
        for _ in range(1, 31):
            hi = int(word / 127773)          # C truncating division
            lo = word - hi * 127773
            word = 16807 * lo - 2836 * hi
            if word < 0:
                word += 2147483647
            st.append(word)
        self.st = [v & 0xFFFFFFFF for v in st]
        self.f, self.b = 3, 0
        for _ in range(310):
            self.rand()

    def rand(self) -> int:
        val = (self.st[self.f] + self.st[self.b]) & 0xFFFFFFFF
        self.st[self.f] = val
        self.f += 1
        if self.f >= 31:
            self.f = 0
            self.b += 1
        else:
            self.b += 1
            if self.b >= 31:
                self.b = 0
        return val >> 1


class Trajectory:
    def __init__(self, id_: int = -1):
        self.id = id_
        self.presentFrames: list[int] = []
        self.positionPerFrame: dict[int, T.Rect] = {}
        self.isTrackedPerFrame: dict[int, bool] = {}
        self.trackIdPerFrame: dict[int, int] = {}
        self.predPosPerFrame: dict[int, T.Rect] = {}
        self.trackPosPerFrame: dict[int, T.Rect] = {}
        self.bboxOverlapPerFrame: dict[int, float] = {}

    # tbd.cpp:141-146
    def add_position(self, frame: int, bbox: T.Rect):
        self.presentFrames.append(frame)
        self.positionPerFrame[frame] = bbox

    # tbd.cpp:148-171
    def add_tracking_info(self, frame: int, track):
        if track is not None:
            self.isTrackedPerFrame[frame] = True
            self.trackIdPerFrame[frame] = track.id
            bbox = track.bboxes[-1]
            gt = self.positionPerFrame.setdefault(frame, T.Rect(0, 0, 0, 0))
            self.trackPosPerFrame[frame] = bbox
            self.predPosPerFrame[frame] = track.predPosition
            self.bboxOverlapPerFrame[frame] = T.compute_bounding_box_overlap(bbox, gt)
        else:
            self.isTrackedPerFrame[frame] = False


# ---- std::sto* as prefix parses ----
_INT = re.compile(r"[ \t\n\v\f\r]*([+-]?\d+)")
_FLT = re.compile(r"[ \t\n\v\f\r]*([+-]?(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?)")


class ParseError(ValueError):
    pass


def stoi(s: str) -> int:
    m = _INT.match(s)
    if not m:
        raise ParseError("stoi")
    v = int(m.group(1))
    if not -2**31 <= v < 2**31:
        raise ParseError("stoi")
    return v


def stoul(s: str) -> int:
    m = _INT.match(s)
    if not m:
        raise ParseError("stoul")
    v = int(m.group(1))
    if abs(v) >= 2**64:
        raise ParseError("stoul")
    return v % 2**64


def stod(s: str) -> float:
    m = _FLT.match(s)
    if not m:
        raise ParseError("stod")
    v = float(m.group(1))
    if math.isinf(v):
        raise ParseError("stod")
    return v


def stof(s: str) -> np.float32:
    m = _FLT.match(s)
    if not m:
        raise ParseError("stof")
    v = np.float32(float(m.group(1)))   # strtof rounds the decimal once; exact for short decimals
    if np.isinf(v):
        raise ParseError("stof")
    return v


def substr(s: str, pos: int, n: int | None = None) -> str:
    if pos > len(s):
        raise ParseError("substr")
    return s[pos:] if n is None else s[pos:pos + n]


# ---- parseHistoryDistribution (samples/gpu/tbd.cpp:258-291) ----
def parse_history_distribution(arg: str) -> list:
    dist = []
    prev = 0
    while True:
        pos = arg.find(",", prev)
        dist.append(stof(substr(arg, prev, pos if pos >= 0 else None)))
        prev = pos + 1
        if pos < 0:
            break
    total = np.float32(0)
    for v in dist:
        total = np.float32(total + v)
    return [np.float32(v / total) for v in dist]


# ---- the history draw (samples/gpu/tbd.cpp:656-671) ----
def draw_history_age(rng: CRand, dist) -> int:
    cum = np.float32(0)
    r = np.float32(np.float32(rng.rand()) / np.float32(RAND_MAX))
    for i, v in enumerate(dist):
        cum = np.float32(cum + v)
        if r < cum:
            return i + 1
    return len(dist)


# ---- parseBboxFile (samples/gpu/tbd.cpp:1163-1295) ----
def parse_bbox_file(path: str, num_frames: int, poses: list, history: list) -> list:
    """Returns per_frame_bboxes (list of frames of rows [objId, v1, ...]);
    appends to the shared poses / history lists as the reference does."""
    parse_poses = len(poses) == 0
    per_frame, cur = [], []
    prev_frame = start_frame = -1
    try:
        data = open(path, "rb").read().decode("latin-1")
    except OSError:
        data = ""
    lines = data.split("\n")
    if lines and lines[-1] == "":
        lines.pop()
    for line in lines:
        pos = line.find("|")
        if pos < 0:
            continue
        if not history and "history" in line:
            prev = pos + 1
            while True:
                pos = line.find(",", prev)
                v = stoul(substr(line, prev, pos if pos >= 0 else None))
                history.append(v & 0xFFFFFFFF)  # int val = stoul(..); vector<unsigned>::push_back(val)
                prev = pos + 1
                if pos < 0:
                    break
            continue
        prev = pos + 1
        frame_num = stoi(line[:pos])
        is_gt = line.count("|") > 4
        if start_frame == -1:
            start_frame = frame_num if is_gt else 0
            prev_frame = start_frame
        for _ in range(prev_frame, frame_num):
            per_frame.append(cur)
            cur = []
        if not is_gt:
            obj = -2
        else:
            pos = line.find("|", prev)
            obj = stoi(substr(line, prev, pos if pos >= 0 else None))
            prev = pos + 1
        if parse_poses and obj == -1:
            pose = []
            while True:
                pos = line.find("|", prev)
                pose.append(stod(substr(line, prev, pos if pos >= 0 else None)))
                prev = pos + 1
                if pos < 0:
                    break
            poses.append(pose)
        elif obj != -1:
            info = [float(obj)]
            while True:
                pos = line.find("|", prev)
                info.append(stod(substr(line, prev, pos if pos >= 0 else None)))
                prev = pos + 1
                if pos < 0:
                    break
            cur.append(info)
        prev_frame = frame_num
    # for (int i = prev_frame; i < start_frame + num_frames; i++): unsigned compare
    end = (start_frame + num_frames) % 2**32
    i = prev_frame
    while i % 2**32 < end:
        per_frame.append(cur)
        cur = []
        i += 1
    return per_frame


def _d2i(v: float) -> int:
    if not (-2147483649.0 < v < 2147483648.0):
        return -2**31
    return int(v)


# ---- parseDetections (samples/gpu/tbd.cpp:1297-1340) ----
def parse_detections(per_frame: list, frame: int, traj: dict | None) -> list:
    if not per_frame or frame >= len(per_frame):
        return []
    out = []
    for b in per_frame[frame]:
        b = list(b) + [0.0] * max(0, 5 - len(b))
        oid = _d2i(b[0])
        r = T.Rect(_d2i(b[1]), _d2i(b[3]), _d2i(b[2] - b[1]), _d2i(b[4] - b[3]))
        out.append(T.Detection(oid, frame, r, 1.0))
        if oid >= 0 and traj is not None:
            if oid not in traj:
                traj[oid] = Trajectory(oid)
            traj[oid].add_position(frame, r)
    return out


def c_g(v: float) -> str:
    """ostream << double: printf("%g"); NaN sign as glibc prints it."""
    if math.isnan(v):
        return "-nan" if math.copysign(1.0, v) < 0 else "nan"
    return "%g" % v


def c_divd(a: float, b: float) -> float:
    """double division on x86: 0/0 is the default NaN (sign bit set)."""
    if b == 0:
        if a == 0 or math.isnan(a):
            return -math.nan if not math.isnan(a) else a
        return math.copysign(math.inf, a) * math.copysign(1.0, b)
    return a / b


def _sub_from_one(x: float) -> float:
    """1 - x; a NaN operand is returned (x86 subsd propagates it with its sign)."""
    return x if math.isnan(x) else 1 - x


# ---- App::writeTrackingOutputToFile (samples/gpu/tbd.cpp:946-1120) ----
def write_tracking_output(tk: T.Tracker, history_ages: list, traj: dict, frame_count: int, log: list | None = None):
    out = ["history|" + ",".join(str(a) for a in history_ages) + "\n"]
    nsw = max([frame_count, len(tk.true_positives)] +
              [f + 1 for t in traj.values() for f in t.presentFrames if f >= 0])
    idsw = [0] * nsw
    frag = {}
    mt = pt = ml = 0
    for key in sorted(traj):
        tr = traj[key]
        frag[tr.id] = 0
        is_new, prev_tracked, prev_id, ntracked = True, False, -1, 0
        for pfid, fnum in enumerate(tr.presentFrames):
            tracked = tr.isTrackedPerFrame.setdefault(fnum, False)
            if tracked:
                tid = tr.trackIdPerFrame.setdefault(fnum, 0)
                if is_new:
                    prev_id = tid
                elif tid != prev_id:
                    if log is not None:
                        log.append(f"[frame {fnum}] target {tr.id} switched from track {prev_id} to track {tid}")
                    if fnum >= 0:
                        idsw[fnum] += 1
                    prev_id = tid
                ntracked += 1
            if not is_new and not prev_tracked and tracked:
                frag[tr.id] += 1
            prev_tracked = tracked
            is_new = pfid == 0
        ratio = c_divd(float(ntracked), float(len(tr.presentFrames)))
        if ratio >= 0.8:
            mt += 1
        elif ratio > 0.2:
            pt += 1
        else:
            ml += 1
    for key in sorted(traj):
        tr = traj[key]
        cells = []
        for fnum in tr.presentFrames:
            tracked = tr.isTrackedPerFrame.setdefault(fnum, False)
            tid = tr.trackIdPerFrame.setdefault(fnum, 0)
            cells.append(f"{fnum},{int(tracked)},{tid}")
        out.append(f"object|{tr.id}|" + ";".join(cells) + f"|FM,{frag[tr.id]}\n")
    total = 0.0
    nf = len(tk.true_positives)
    for f in range(nf):
        out.append(f"frame|{f}|TP,{tk.true_positives[f]};FN,{tk.false_negatives[f]};FP,{tk.false_positives[f]};"
                   f"GT,{tk.ground_truths[f]};c,{tk.num_matches[f]};IDSW,{idsw[f]};sum_di,{c_g(tk.bbox_overlap[f])}\n")
        total += tk.bbox_overlap[f]
    mota_n = amota_n = mota_d = motp_d = 0.0
    for f in range(nf):
        mota_n += tk.false_negatives[f] + tk.false_positives[f] + idsw[f]
        amota_n += tk.false_negatives[f] + tk.false_positives[f]
        mota_d += tk.ground_truths[f]
        motp_d += tk.num_matches[f]
    mota = _sub_from_one(c_divd(mota_n, mota_d))
    amota = _sub_from_one(c_divd(amota_n, mota_d))
    motp = c_divd(total, motp_d)
    out.append(f"scenario|MT,{mt};PT,{pt};ML,{ml};MOTA,{c_g(mota)};A-MOTA,{c_g(amota)};MOTP,{c_g(motp)}\n")
    metrics = dict(mt=mt, pt=pt, ml=ml, idsw=sum(idsw[:nf]), fm=sum(frag.values()), frames=nf,
                   mota=mota, amota=amota, motp=motp)
    return "".join(out), metrics


# ---- App::run, tracking section (samples/gpu/tbd.cpp:479-706, 823-841) ----
def app_run(ped_file=None, veh_file=None, num_frames=100, num_iters=1, history_distribution=None,
            seed=1, write=True, tracker_kwargs=None):
    """Returns (per iteration: [pedestrian output text, vehicle output text]), log lines."""
    dist = parse_history_distribution(history_distribution) if history_distribution else [np.float32(1.0)]
    poses, history = [], []
    files = [ped_file, veh_file]
    tables = [parse_bbox_file(f, num_frames, poses, history) if f else [] for f in files]
    use_provided = len(history) > 0
    rng = CRand(seed)
    H = len(dist)
    results, log = [], []
    for _ in range(num_iters):
        traj = [{}, {}]
        buf = [[[] for _ in range(H)], [[] for _ in range(H)]]
        ages = []
        trackers = [T.Tracker(**(tracker_kwargs or {})), T.Tracker(**(tracker_kwargs or {}))]
        for tk in trackers:
            tk.rng = rng
        frame_id = 0
        while frame_id < num_frames:
            dets = [parse_detections(tables[c], frame_id, traj[c]) for c in range(2)]
            if frame_id == 0:
                for c in range(2):
                    buf[c] = [[] for _ in range(H)]
                    trackers[c].reset()
            age = history[frame_id] if use_provided else draw_history_age(rng, dist)
            ages.append(age)
            for c in range(2):
                prior = buf[c][(frame_id - age) % H] if frame_id >= age else []
                trackers[c].set_tracks(prior)
            for c in range(2):
                if files[c]:
                    trackers[c].step(dets[c], frame_id, traj=traj[c])
            for c in range(2):
                buf[c][frame_id % H] = [__import__("copy").deepcopy(t) for t in trackers[c].tracks]
            frame_id += 1
        texts = []
        for c in range(2):
            txt, m = write_tracking_output(trackers[c], ages, traj[c], frame_id, log if write else None)
            texts.append((txt, m))
        results.append(texts)
    return results, log
