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
