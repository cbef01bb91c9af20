"""The multi-GPU contract of bench.py, rehearsed on CPU with gloo at world
size 2 (replicas only: no data-path collective; the job time is the max over
ranks and the value counts every rank's frames)."""
import os
import socket
import sys

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dist.barrier()
    elapsed = [1.5, 2.0][rank]  # rank 1 is the straggler
    el = bench.max_over_ranks(elapsed, world, device="cpu")
    q.put((rank, el, bench.replica_throughput(480, world, el)))
    dist.barrier()
    dist.destroy_process_group()


def test_replica_timing_world_size_2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [2.0, 2.0]           # both ranks see the max time
    assert all(abs(r[2] - 480 * 2 / 2.0) < 1e-12 for r in res)  # frames of all ranks / max time


def _group_worker(rank, world, port, q, share=False):
    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if share:  # the one-GPU rehearsal switch: ranks wrap onto the devices there are
        os.environ["TBDK_BENCH_SHARE_GPU"] = "1"
        torch.cuda.device_count = lambda: 1
    dev = []
    torch.cuda.set_device = lambda d: dev.append(d)  # no GPU here; record the selection
    bench.init_rank_group(world, rank, rank)
    backend = dist.get_backend()
    el = bench.max_over_ranks([1.0, 4.0][rank], world, device="cpu")
    q.put((rank, backend, dev, el))
    dist.barrier()
    dist.destroy_process_group()


def test_rank_group_is_host_only_world_size_2():
    """bench.init_rank_group at world size 2: each rank selects its own GPU and
    the job's group is gloo, so no RCCL communicator (and none of its GPU
    streams) exists before the TBD loop's own streams — HIP's creation-order
    queue mapping cannot push the loop onto a shared hardware queue
    (DESIGN.md §8)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_group_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == ["gloo", "gloo"]
    assert [r[2] for r in res] == [[0], [1]]
    assert [r[3] for r in res] == [4.0, 4.0]


def test_rank_group_shared_gpu_rehearsal():
    """TBDK_BENCH_SHARE_GPU=1 (rehearsing the N-rank bench on a box with fewer
    GPUs than ranks): rank i selects GPU i mod device_count; the group is the
    same gloo group.  Without the switch each rank keeps its own GPU (above)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_group_worker, args=(r, 2, port, q, True)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == ["gloo", "gloo"]
    assert [r[2] for r in res] == [[0], [0]]


def test_bench_creates_no_rccl_group():
    """No code path of bench.py creates an RCCL (nccl) process group."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'init_process_group("nccl"' not in src and "init_process_group('nccl'" not in src


def test_single_rank_needs_no_collective():
    sys.path.insert(0, ROOT)
    import bench

    assert bench.max_over_ranks(3.0, 1) == 3.0
    assert bench.replica_throughput(100, 1, 0.5) == 200.0


class _FakeMeasure:
    """Stands in for bench.TbdMeasure: records the seed, sleeps per step."""

    def __init__(self, per_step):
        self.per_step, self.seed, self.warm = per_step, None, None

    def prepare(self, seed):
        self.seed = seed

    def warmup(self, w):
        self.warm = w

    def timed(self, k):
        import time

        time.sleep(self.per_step * k)
        return list(range(k))


def _contract_worker(rank, world, port, q):
    import argparse

    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    args = argparse.Namespace(seed=100, warmup=3, steps=10)
    calls = []
    m = _FakeMeasure([0.01, 0.03][rank])  # rank 1 is the straggler
    line, per = bench.run_contract(args, world, rank, m, lambda: None, "cpu", cpu_leg=lambda: calls.append(1) or 1)
    q.put((rank, m.seed, m.warm, len(per), line["value"], line["ms_per_step"], line["cpu_baseline"], len(calls)))
    dist.barrier()
    dist.destroy_process_group()


def test_run_contract_rank_plumbing_world_size_2():
    """bench.run_contract under gloo, world size 2, GPU legs stubbed: each rank
    runs its own sequence (seed + rank), the job time is the slower rank's, the
    value counts both ranks' steps, and no CPU baseline runs at N > 1."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_contract_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [100, 101] and all(r[2] == 3 and r[3] == 10 for r in res)
    assert res[0][4] == res[1][4] and res[0][5] == res[1][5]  # one job time on every rank
    el = res[0][5] * 10 / 1000.0
    assert el >= 0.3 and abs(res[0][4] - 2 * 10 / el) < 1e-6 * res[0][4] + 0.02  # slowest rank's 0.3 s
    assert all(r[6] is None and r[7] == 0 for r in res)


def test_run_contract_single_rank_runs_cpu_baseline():
    import argparse

    sys.path.insert(0, ROOT)
    import bench

    calls = []
    args = argparse.Namespace(seed=7, warmup=1, steps=4)
    line, per = bench.run_contract(args, 1, 0, _FakeMeasure(0.001), lambda: None, "cpu",
                                   cpu_leg=lambda: calls.append(1) or {"value": 1.0})
    assert calls == [1] and line["cpu_baseline"] == {"value": 1.0}
    assert line["n_gpus"] == 1 and line["steps"] == 4 and len(per) == 4
    assert abs(line["value"] - 4 / (line["ms_per_step"] * 4 / 1000.0)) < 0.05 * line["value"]


def test_host_topology_helpers():
    sys.path.insert(0, ROOT)
    import bench

    assert bench.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    n, info = bench.host_cores()
    assert 1 <= n <= info["affinity_cpus"]
    r = bench.pin_rank(0)  # no KFD topology here: nothing pinned, nothing changed
    assert isinstance(r, dict) and "pinned" in r


def test_copy_peak_fractions_on_hbm_rooflines_only():
    """hbm_copy_peak's value lands beside every HBM roofline (nested ones too),
    never on a VALU one."""
    sys.path.insert(0, ROOT)
    import bench

    line = {"roofline": {"bound": "valu", "achieved": 20.0},
            "roofline_pyramid": {"bound": "hbm", "achieved": 400.0},
            "farneback": {"roofline": {"bound": "hbm", "achieved": 2000.0}}}
    bench.add_copy_peak_fracs(line, 5000.0)
    assert "frac_copy_peak" not in line["roofline"]
    assert line["roofline_pyramid"]["frac_copy_peak"] == 0.08
    assert line["farneback"]["roofline"]["frac_copy_peak"] == 0.4
    assert line["farneback"]["roofline"]["copy_peak"] == 5000.0


def _fake_sysfs(root, kfd_location=True):
    """Two GPUs on PCI 0000:c1:00.0 (NUMA node 1, CPUs 16-31) and
    0000:05:00.0 (node 0, CPUs 0-15 by local_cpulist) plus a CPU KFD node; KFD
    lists them in the order c1, 05 (not PCI order)."""
    import pathlib

    r = pathlib.Path(root)
    gpus = [("0000:c1:00.0", 0xC100, 1, None), ("0000:05:00.0", 0x0500, 0, "0-15")]
    kfd = r / "class/kfd/kfd/topology/nodes"
    (kfd / "0").mkdir(parents=True)
    (kfd / "0/properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    for i, (bdf, loc, node, local) in enumerate(gpus, 1):
        (kfd / str(i)).mkdir()
        (kfd / f"{i}/properties").write_text(
            f"simd_count 1024\ndomain 0\n" + (f"location_id {loc}\n" if kfd_location else "") + "gfx_target_version 90500\n")
        d = r / "bus/pci/devices" / bdf
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{node}\n")
        (d / "vendor").write_text("0x1002\n")
        (d / "class").write_text("0x038000\n")
        if local:
            (d / "local_cpulist").write_text(local + "\n")
        card = r / f"class/drm/card{i - 1}"
        card.mkdir(parents=True)
        (card / "device").symlink_to(d)
        (r / f"class/drm/card{i - 1}-DP-1").mkdir()
    nd = r / "devices/system/node"
    (nd / "node0").mkdir(parents=True)
    (nd / "node0/cpulist").write_text("0-15,64-79\n")
    (nd / "node1").mkdir()
    (nd / "node1/cpulist").write_text("16-31\n")


def test_gpu_numa_cpus_fake_sysfs(tmp_path, monkeypatch):
    """bench.gpu_numa_cpus over a fake sysfs tree: the KFD order with
    location_id; without it the DRM cards in PCI order; the PCI device's
    local_cpulist before its NUMA node's cpulist; ROCR_VISIBLE_DEVICES
    remapping; nothing when sysfs has neither"""
    sys.path.insert(0, ROOT)
    import bench

    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    a = tmp_path / "a"
    _fake_sysfs(a)
    assert bench.gpu_numa_cpus(0, str(a)) == (1, list(range(16, 32)), "kfd:0000:c1:00.0:numa_node")
    assert bench.gpu_numa_cpus(1, str(a)) == (0, list(range(16)), "kfd:0000:05:00.0:local_cpulist")
    assert bench.gpu_numa_cpus(2, str(a)) is None
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1")
    assert bench.gpu_numa_cpus(0, str(a))[2] == "kfd:0000:05:00.0:local_cpulist"
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    b = tmp_path / "b"
    _fake_sysfs(b, kfd_location=False)
    assert bench.gpu_numa_cpus(0, str(b)) == (0, list(range(16)), "drm:0000:05:00.0:local_cpulist")
    assert bench.gpu_numa_cpus(1, str(b)) == (1, list(range(16, 32)), "drm:0000:c1:00.0:numa_node")
    assert bench.gpu_numa_cpus(0, str(tmp_path / "empty")) is None


def test_pin_by_runtime_pci_address_fake_sysfs(tmp_path, monkeypatch):
    """bench.pin_rank_by_device: the runtime's PCI address (faked) -> the fake
    sysfs tree's local_cpulist; the affinity change itself is stubbed"""
    import types

    import torch

    sys.path.insert(0, ROOT)
    import bench

    _fake_sysfs(tmp_path)
    props = types.SimpleNamespace(pci_domain_id=0, pci_bus_id=0x05, pci_device_id=0)
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda d: props)
    pinned = []
    monkeypatch.setattr(bench, "_pin_all_threads", lambda cpus: pinned.append(cpus))
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(64)))
    r = bench.pin_rank_by_device(0, str(tmp_path))
    assert r["pinned"] and r["pci"] == "0000:05:00.0" and pinned == [list(range(16))]
    props.pci_bus_id = 0xC1  # no local_cpulist: its NUMA node's cpulist
    r = bench.pin_rank_by_device(0, str(tmp_path))
    assert r["pinned"] and r["numa_node"] == 1 and pinned[-1] == list(range(16, 32))
    props.pci_bus_id = 0x99
    assert not bench.pin_rank_by_device(0, str(tmp_path))["pinned"]


def test_loop_traffic_fields_from_committed_loop_summary():
    """the loop's traffic fields come from the newest
    committed loop-only PMC summary (profiles/rNN_pmc_loop.json: only
    configs[2]'s launches counted) and reproduce from it: the levels-only
    1080p build's counter bytes are within 10 % of its algorithmic bytes
    (round 4's name-keyed means, with the 4K legs mixed in, gave 1.68x), and
    PyrLK's per-launch bytes stay below two full pyramids (SURVEY §8d's
    B_lk bound).  The kernel-trace helper finds the loop's and the 4K build's
    grids in the committed per-grid summary."""
    import bench

    p = bench.pmc_bytes(["pyr_build_kernel", "pyr_down_padded_kernel"])
    assert p is not None and p["source"].endswith("_pmc_loop.json")
    alg = bench.pyr_build_bytes(1920, 1080, 3)
    # the summary's build: with the padded level-0 copy (rounds 4-5, early round 6) or with the
    # frame itself as level 0 (tbd_borrow_l0, round 6)
    ratios = [(p["fetch_raw"] + p["write"]) / a for a in (alg, bench.pyr_build_bytes(1920, 1080, 3, copy_l0=False))]
    assert any(0.85 < r < 1.1 for r in ratios), ratios
    lk, src = bench.pmc_traffic("lk_multi_kernel<21, 21, true, false>")  # the name bench.main looks up
    assert src is not None and src.endswith("_pmc_loop.json")
    assert 0 < lk < 2 * alg
    us, used, gsrc = bench.ktrace_grid_us(["pyr_build_kernel", "pyr_down_padded_kernel"], pick="max_grid")
    assert us is not None and gsrc.endswith("_ktrace_grid.json") and len(used) == 2
    us1, used1, _ = bench.ktrace_grid_us(["pyr_build_kernel", "pyr_down_padded_kernel"], pick="most")
    # the loop's 1080p grids (fewer threads than the 4K leg's); since round 5 the loop
    # builds its look-ahead pyramid beside the critical PyrLK, so their durations
    # include that overlap and are not compared with the 4K leg's
    assert us1 is not None and us1 > 0 and all(u[1] < g[1] for u, g in zip(used1, used))


def _json_lines(out):
    import json

    return [json.loads(ln) for ln in out.splitlines() if ln.lstrip().startswith("{")]


def test_main_gpus_2_starts_two_ranks(monkeypatch, capsys):
    """`bench.py --gpus 2` with no launcher starts two rank
    processes itself (gloo group, no GPU in --rehearse mode) and relays rank
    0's single line: n_gpus 2, seeds s and s+1, value = the steps of both
    ranks / the slower rank's time."""
    import pytest

    sys.path.insert(0, ROOT)
    import bench

    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "2", "--steps", "10", "--warmup", "2", "--seed", "500", "--rehearse", "10"])
    assert e.value.code == 0
    lines = _json_lines(capsys.readouterr().out)
    assert len(lines) == 1
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["rank_seeds"] == [500, 501] and ln["steps"] == 10
    el = ln["ms_per_step"] * 10 / 1000.0
    assert el >= 0.2  # rank 1 sleeps 2 x 10 ms per step
    assert abs(ln["value"] - 2 * 10 / el) < 0.01 * ln["value"]
    assert ln["data"].startswith("rehearsal")


def test_gpus_world_size_mismatch_fails(monkeypatch):
    import pytest

    sys.path.insert(0, ROOT)
    import bench

    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "1", "--rehearse", "1"])
    assert e.value.code and "WORLD_SIZE=2" in str(e.value.code)
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "4", "--rehearse", "1"])
    assert e.value.code and "--gpus 4" in str(e.value.code)


def test_spawn_ranks_ends_the_job_when_a_rank_fails(tmp_path):
    """A rank that fails ends the job with its exit code; the rank still
    running (here: sleeping, as one waiting in a barrier would) is ended."""
    import time

    sys.path.insert(0, ROOT)
    import bench

    s = tmp_path / "r.py"
    s.write_text("import os, sys, time\n"
                 "if os.environ['RANK'] == '1':\n    sys.exit(3)\n"
                 "time.sleep(600)\n")
    t0 = time.time()
    assert bench.spawn_ranks([], 2, script=str(s)) == 3
    assert time.time() - t0 < 60


def test_torchrun_gpus_2_matches_launcher(tmp_path):
    """The driver's N > 1 form: torch.distributed.run --nproc-per-node 2 ...
    bench.py --gpus 2 (WORLD_SIZE from the launcher, no self-spawn)."""
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "1",
                        "--rehearse", "5"], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1 and lines[0]["n_gpus"] == 2 and len(lines[0]["rank_seeds"]) == 2
