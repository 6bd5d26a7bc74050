"""bench.py's host-side pieces that need no GPU: the cpu_baseline object of
the JSON line (the C restatement of the reference's make.go split-and-align,
timed at the job's CPU share and at n = 10) and its labels."""
import numpy as np

import bench
from oracle import oracle as o


def test_cpu_baseline_object():
    blob = o.synth_uniform_c(1, 0, 32 << 20)
    cb = bench.cpu_baseline(blob, threads=2)
    assert cb["kind"] == "port" and cb["unit"] == "GiB/s" and cb["cores"] == 2
    for k in ("value", "n10_gibs", "single_thread_gibs", "ids_sha512_256_gibs"):
        assert cb[k] > 0, k
    assert "n=10" in cb["sample"] and "2 threads" in cb["sample"]


def test_cpu_share_reads_omp_num_threads(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    assert bench.cpu_share() == 16
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert 1 <= bench.cpu_share() <= 16


def test_data_labels_name_the_generator_seeds(monkeypatch):
    monkeypatch.setattr("sys.argv", ["bench.py"])
    a = bench.parse()
    # the default per-GPU shape is BASELINE config 5's shard at every N
    assert (a.gib, a.seed, a.workload, a.config) == (32.0, 3, "uniform", "config 5 shard")
    assert (a.steps, a.warmup) == (20, 5)
    assert "seed 3" in bench.DATA_LABEL["uniform"].format(seed=a.seed)
    monkeypatch.setattr("sys.argv", ["bench.py", "--workload", "dedup"])
    a = bench.parse()
    assert "seed 2" in bench.DATA_LABEL["dedup"].format(seed=a.seed)
    assert (a.gib, a.config) == (16.0, "config 3")
    monkeypatch.setattr("sys.argv", ["bench.py", "--workload", "zeros"])
    assert bench.parse().config == "config 4"
    monkeypatch.setattr("sys.argv", ["bench.py", "--config5"])
    a = bench.parse()
    assert (a.gib, a.seed, a.workload) == (32.0, 3, "uniform")  # BASELINE config 5's shards
    monkeypatch.setattr("sys.argv", ["bench.py", "--config2"])
    a = bench.parse()
    assert (a.gib, a.seed, a.workload, a.config) == (1.0, 1, "uniform", "config 2")
    monkeypatch.setattr("sys.argv", ["bench.py", "--gib", "0.25"])
    a = bench.parse()
    assert (a.gib, a.seed, a.config) == (0.25, 3, None)


def test_traffic_lookup_by_launch_size(tmp_path, monkeypatch):
    """roofline.traffic is the PMC figure of launches of the same size only."""
    import json
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "traffic_uniform_64.json").write_text(
        json.dumps({"bytes": 64, "hbm_bytes_per_launch": 65.0}))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.load_traffic("uniform", 64) == 65.0
    assert bench.load_traffic("uniform", 128) is None


def test_cpu_leg_matches_the_sequential_chain():
    """What the baseline times is the reference's result: split-and-align ==
    the sequential Next loop (make_test.go:16-80)."""
    blob = o.synth_uniform_c(2, 0, 8 << 20)
    assert np.array_equal(o.chunk_parallel(blob, bench.MIN, bench.AVG, bench.MAX, 4),
                          o.chunk_stream(blob, bench.MIN, bench.AVG, bench.MAX))


def test_refuses_a_gpu_count_other_than_the_world_size():
    """A line for N GPUs must come from N ranks: `--gpus 2` without
    torch.distributed.run (WORLD_SIZE unset) stops before anything runs."""
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-cpu"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0 and "WORLD_SIZE 1" in r.stderr, r.stderr[-2000:]
    assert not r.stdout.strip()
