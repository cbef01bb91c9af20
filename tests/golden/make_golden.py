"""Regenerates tests/golden/*.json.

These fixtures pin the in-repo synthetic sequence (opencv_amd/csrc/synth_spec.h)
so that any change to the generator is caught.  They are produced by the CPU
oracle (oracle/), NOT by the reference — the reference cannot be built here
(DESIGN.md §Oracle).

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import _oracle as O  # noqa: E402

out = {}
fr, gt = O.synth(20261015, 640, 480, 32, 0, 3)
out["640x480x32"] = [hashlib.sha256(fr[f].tobytes()).hexdigest() for f in range(3)]
out["640x480x32_gt"] = hashlib.sha256(gt.tobytes()).hexdigest()
fr, gt = O.synth(20261015, 1920, 1080, 128, 0, 2)
out["1920x1080x128"] = [hashlib.sha256(fr[f].tobytes()).hexdigest() for f in range(2)]
out["1920x1080x128_gt"] = hashlib.sha256(gt.tobytes()).hexdigest()
with open(os.path.join(HERE, "synth_hashes.json"), "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
