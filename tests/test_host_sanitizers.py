"""the host restatement's C++ (the cv::tbd::Tracker restatement
tbd_tracker.cpp, the sample driver / file formats tbd_app.cpp and the CLI)
under AddressSanitizer + UndefinedBehaviorSanitizer.  `make host-asan` builds
them host-only (no HIP kernels) into build/asan/; the tracker and sample-driver
test modules then run in a child process against that library (TBDK_LIB,
TBDK_HOST_ONLY) and CLI (TBDK_APP), with the sanitizer runtimes preloaded
(Python itself is not instrumented).  Any ASan report or UBSan runtime error
fails the run (halt_on_error; -fno-sanitize-recover)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    assert os.path.isabs(p) and os.path.exists(p), f"{name} not found"
    return p


def test_tracker_and_driver_under_asan_ubsan():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "opencv_amd", "csrc"), "host-asan"])
    lib = os.path.join(ROOT, "build", "asan", "libtbdk_host.so")
    app = os.path.join(ROOT, "build", "asan", "tbdk_tbd_app")
    env = dict(os.environ)
    env.update(LD_PRELOAD=f"{_runtime('libasan.so')}:{_runtime('libubsan.so')}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",  # CPython's own allocations are not ours to judge
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TBDK_LIB=lib, TBDK_HOST_ONLY="1", TBDK_APP=app)
    code = ("import sys, pytest; from opencv_amd import _lib; "
            f"assert _lib.load()._name == {lib!r}; "
            "sys.exit(pytest.main(['-q', '-x', '-p', 'no:cacheprovider', 'tests/test_tracker_oracle.py', "
            "'tests/test_tbd_app.py']))")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert " passed" in out and " failed" not in out


def test_flat_map_matches_unordered_map_under_asan_ubsan(tmp_path):
    """The TBD loop's lookup tables (opencv_amd/csrc/flat_map.hpp: track id ->
    slot, track id -> corner count, early box -> row) against std::unordered_map
    over random insert / set / erase / find / clear sequences, host-built with
    AddressSanitizer + UndefinedBehaviorSanitizer."""
    exe = str(tmp_path / "flat_map_check")
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=undefined", "-I", os.path.join(ROOT, "opencv_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "flat_map_check.cpp"), "-o", exe])
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "flat_map ok" in p.stdout, p.stdout + p.stderr


def test_tracker_first_round_solver_matches_dense_under_asan_ubsan(tmp_path):
    """The tracker's first assignment round solved on the cost entries' value
    kinds (tbd_tracker.cpp, the default) against the same tracker solving every
    round on the dense matrix (Tracker::setDenseSolver), frame by frame over 64
    scenarios (ties, duplicates, dropouts, clutter, zero-size boxes, padding
    values below 1, at 1 and outside (0, 1e7)); at least one frame must reach
    the dense rounds after the first.  Host-built with ASan + UBSan."""
    exe = str(tmp_path / "tracker_solver_check")
    csrc = os.path.join(ROOT, "opencv_amd", "csrc")
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=undefined", "-I", csrc,
                           os.path.join(ROOT, "tests", "cpp", "tracker_solver_check.cpp"),
                           os.path.join(csrc, "tbd_tracker.cpp"), "-o", exe])
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "tracker solver ok" in p.stdout, p.stdout + p.stderr
