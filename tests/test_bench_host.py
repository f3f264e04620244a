"""bench.py's host description (CPU): the cgroup CPU quota beside the
affinity mask, so a cpu_baseline measured on many threads says how many CPUs'
worth of time it actually had."""
import os


def test_cgroup_cpu_quota(tmp_path):
    import bench

    (tmp_path / "cpu.max").write_text("1600000 100000\n")
    assert bench.cgroup_cpu_quota(str(tmp_path)) == 16.0
    (tmp_path / "cpu.max").write_text("max 100000\n")
    assert bench.cgroup_cpu_quota(str(tmp_path)) is None
    v1 = tmp_path / "v1"
    (v1 / "cpu").mkdir(parents=True)
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("800000\n")
    (v1 / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert bench.cgroup_cpu_quota(str(v1)) == 8.0
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("-1\n")
    assert bench.cgroup_cpu_quota(str(v1)) is None
    assert bench.cgroup_cpu_quota(str(tmp_path / "missing")) is None


def test_cpu_info_keys():
    import bench

    info = bench.cpu_info()
    assert set(info) >= {"nproc", "affinity", "cpu_model", "cgroup_cpu_quota"}
    assert info["affinity"] == len(os.sched_getaffinity(0))


def test_rank_guard():
    """--gpus N means N ranks: without a launcher the
    bench starts N children through torch.distributed.run on 127.0.0.1 (and
    exits with their code); a launcher world that differs from --gpus is
    refused; a matching world, or N = 1, runs in this process"""
    import argparse

    import bench

    seen = []

    def spawn(cmd):
        seen.append(cmd)
        return 7

    a = argparse.Namespace(gpus=4)
    assert bench.rank_guard(a, ["--gpus", "4", "--steps", "3"], {}, spawn) == 7
    cmd = seen[0]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == [os.path.abspath(bench.__file__), "--gpus", "4", "--steps", "3"][-4:]
    assert bench.rank_guard(a, [], {"WORLD_SIZE": "4"}, spawn) is None
    assert bench.rank_guard(a, [], {"WORLD_SIZE": "1"}, spawn) == 2
    assert bench.rank_guard(argparse.Namespace(gpus=1), [], {}, spawn) is None
    assert bench.rank_guard(argparse.Namespace(gpus=1), [], {"WORLD_SIZE": "2"}, spawn) == 2
    assert len(seen) == 1


def test_rank_guard_spawns_ranks(tmp_path):
    """end to end on the CPU: `bench.py --gpus 2` with no launcher starts two
    ranks whose own guard passes (WORLD_SIZE = 2); they stop at the GPU
    check (this container has no GPU) with the guard's message, not with a
    world-1 line"""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=str(tmp_path),
                       env={**os.environ, "HIP_VISIBLE_DEVICES": ""})
    assert r.returncode != 0
    assert "starting 2 ranks" in r.stderr
    assert "2 RCCL ranks need 2 GPUs" in r.stderr
    assert '"metric"' not in r.stdout
