"""bench.py's multi-rank harness on CPU (gloo, world_size 2): the barrier +
max-over-ranks timing, the whole-job value and rank-0-only output, with a fake
engine standing in for the GPU (the -m gpu tests and the driver's runs cover the
real engine).  SURVEY.md §8e: shards are independent, no data-path collective."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


class FakeEngine:
    """Answers like GpuEngine; CRCs come from the oracle (test infrastructure only)."""

    def __init__(self, device, batches, lanes, wgs):
        import oracle
        self.batches = batches
        self.lib = oracle.OracleLib()
        self.steps = 0

    def step(self, i):
        self.steps += 1

    def probe(self, i):
        pass

    def sync(self):
        pass

    def kernel_ms(self, fn, steps):
        return 0.02, 0.022

    def region_ms(self, fn, steps):
        return 0.019

    def outputs(self, j):
        b = self.batches[j]
        return self.lib.batch(b.payload, b.off, b.lens, threads=2)


def fake_cpu(batch, budget, threads=0):
    one = {"gibps": 0.5, "threads": 1, "packets": batch.n, "reps": 1, "runs": 5, "spread": [0.5, 0.5]}
    return {"1thread": one, "all": dict(one, gibps=2.0, threads=2),
            "host": {"affinity_cores": 2, "cgroup_cpu_quota": None, "cgroup_file": None}, "speedup": 4.0}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, ws, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(ws),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import io
    import contextlib
    import bench
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main(["--config", "small", "--rotate", "2", "--steps", "6", "--warmup", "1", "--gpus", str(ws)],
                   engine_factory=FakeEngine, cpu_factory=fake_cpu)
    q.put((rank, buf.getvalue()))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("ws", [2, 4])
def test_multi_rank_gloo_harness(ws):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, ws, port, q)) for r in range(ws)]
    for p in ps:
        p.start()
    outs = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert all(outs[r].strip() == "" for r in range(1, ws))   # only rank 0 prints
    lines = [l for l in outs[0].splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == ws and d["steps"] == 6 and d["scaling"] == "weak"
    assert d["unit"] == "GiB/s" and d["higher_is_better"] is True and d["dtype"] == "u8"
    # whole-job value: every rank's bytes over the max-over-ranks span
    per_rank = 6 * 2048 * 1200
    assert d["value"] == pytest.approx(ws * per_rank / (d["ms_per_step"] * 6e-3) / 2**30, rel=0.02)
    assert d["roofline"]["bound"] == "hbm" and d["roofline"]["peak"] == 8000.0
    assert d["cpu_baseline"] is None                   # (timed at N = 1 only, on rank 0)
    assert d["config"]["workgroups_per_cu"] == ("default (2)" if d["config"]["steps_per_launch"] > 1 else "default (1)") and d["config"]["kernel_path"] == 0


@pytest.mark.timeout(300)
def test_gpus_n_without_a_launcher_spawns_n_ranks(monkeypatch, capfd):
    """`bench.py --gpus 2` with no torch.distributed.run around it starts the two
    ranks itself: one line, n_gpus 2, every rank gated -- never a
    one-rank line for --gpus N."""
    import bench
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    rc = bench.main(["--config", "small", "--rotate", "2", "--steps", "6", "--warmup", "1", "--gpus", "2"],
                    engine_factory=FakeEngine, cpu_factory=fake_cpu)
    assert rc == 0
    out = capfd.readouterr().out
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "2 independent shards (no collective)"
    assert d["cpu_baseline"] is None


def test_cpu_line_states_quota_and_speedup():
    """The cpu_baseline object names its thread count, the measured speed-up over one
    thread, the affinity mask and the cgroup quota."""
    import bench
    cpu = {"1thread": {"gibps": 0.5, "threads": 1, "packets": 10, "reps": 1, "runs": 5, "spread": [0.4, 0.6]},
           "all": {"gibps": 7.0, "threads": 16, "packets": 100, "reps": 2, "runs": 5, "spread": [6.5, 7.2]},
           "host": {"affinity_cores": 256, "cgroup_cpu_quota": 16.0, "cgroup_file": "/sys/fs/cgroup/cpu.max"},
           "speedup": 14.0}
    d = bench.cpu_line(cpu)
    assert d["cores"] == 16 and d["speedup_vs_1thread"] == 14.0 and d["cgroup_cpu_quota"] == 16.0
    assert "median of 5" in d["sample"] and "quota 16.0" in d["sample"]
    th, info = bench.baseline_threads()
    q = info["cgroup_cpu_quota"]
    assert th == (min(info["affinity_cores"], int(np.ceil(q))) if q else info["affinity_cores"])


def test_traffic_files_match_their_entry_and_build(tmp_path, monkeypatch):
    """profiles/traffic_<cfg>.json belongs to the plain / list entry and
    traffic_<cfg>_binned.json to the binned one; bench.py hands each line its own, and
    only when the record's library_sha256 is the build the run loaded (VERDICT r5 #2:
    a stale pass of an older build is not this run's traffic)."""
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "traffic_cfg2.json").write_text(json.dumps({"hbm_bytes_per_batch": 86e6, "library_sha256": "aa"}))
    (prof / "traffic_cfg3_binned.json").write_text(json.dumps({"hbm_bytes_per_batch": 1.0, "binned": True,
                                                                "library_sha256": "aa"}))
    (prof / "traffic_cfg3.json").write_text(json.dumps({"hbm_bytes_per_batch": 1.0, "binned": True,
                                                         "library_sha256": "aa"}))   # (mislabelled)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.load_traffic("cfg2", False, "aa")["hbm_bytes_per_batch"] == 86e6
    assert bench.load_traffic("cfg2", False, "bb") is None             # another build
    assert bench.load_traffic("cfg2", False, None) is None             # library not found
    assert bench.load_traffic("cfg3", True, "aa")["binned"] is True
    assert bench.load_traffic("cfg3", False, "aa") is None             # tag disagrees with the name
    assert bench.load_traffic("cfg4", False, "aa") is None             # no record


def test_committed_traffic_records_name_their_build():
    """Every committed traffic record names the library build it was measured with."""
    import glob
    for f in glob.glob(os.path.join(ROOT, "profiles", "traffic_*.json")):
        d = json.load(open(f))
        assert len(d.get("library_sha256") or "") == 64, f


def test_one_rank_line_carries_the_cpu_baseline(monkeypatch):
    """At N = 1 rank 0 times the CPU baseline and the line carries it (cores, kind)."""
    import io
    import contextlib
    import bench
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main(["--config", "small", "--rotate", "2", "--steps", "4", "--warmup", "1"],
                   engine_factory=FakeEngine, cpu_factory=fake_cpu)
    d = json.loads([l for l in buf.getvalue().splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 1
    assert d["cpu_baseline"]["cores"] == 2 and d["cpu_baseline"]["kind"] == "port"


def test_cpu_baseline_uses_the_affinity_cores():
    """The CPU baseline runs on the cores of the process's affinity mask, capped by
    the cgroup CPU quota when there is one, and says how many; median of 5 runs."""
    import bench
    assert bench.host_cores() == len(os.sched_getaffinity(0))
    from enethip import workloads
    b = workloads.fixed(512, 1200, seed=1, name="t")
    r = bench.cpu_baseline(b, 0.05)
    th, _ = bench.baseline_threads()
    assert r["all"]["threads"] == th and r["1thread"]["threads"] == 1
    assert r["all"]["runs"] == 5 and r["speedup"] > 0


def test_cfg4_shards_partition_the_million_packets():
    """bench.py --config cfg4 (SURVEY §8e, strong scaling): rank r of k checksums
    the contiguous packet range [r N/k, (r+1) N/k) of the 1 M x 1200 B workload --
    the shards cover every packet once, each shard's bytes are that range of the
    one splitmix64 payload stream, and a shard under 320 MiB is kept resident in
    enough copies to stay out of the 256 MiB Infinity Cache."""
    import bench
    from enethip import workloads
    n, L = 1 << 20, 1200
    for k in (4, 8):
        total = 0
        for r in (0, k - 1):
            bs = bench.make_batches("cfg4", 5, r, k)
            b = bs[0]
            lo = n * r // k
            assert b.n == n * (r + 1) // k - lo and (b.lens == L).all()
            assert len(bs) * b.payload_bytes >= bench.CFG4_RESIDENT and all(x is b for x in bs)
            ref = workloads.splitmix64(workloads.SEED_PAYLOAD, 4, start=lo * L // 8).view(np.uint8)
            assert (b.payload[:32] == ref).all()
            total += b.n
        assert total == 2 * (n // k)


def test_kernel_name_follows_the_entry_and_knobs():
    """The dominant kernel each bench form names (rocprof's spelling of
    crc32_vring_kernel<LG, TR, NT, ABL, BIN, WK, ROT, VF, DYN>): product list form,
    binned records (one workgroup per CU) and the compact records instance (two),
    the records ablations, the dynamic-rounds twins."""
    import argparse
    import bench

    def name(local_tiles=False, **kw):
        a = dict(path=0, lanes=0, binned=False, ablate=0, wgs=0)
        a.update(kw)
        return bench.kernel_name(argparse.Namespace(**a), local_tiles=local_tiles)

    assert name() == "crc32_vring_kernel<3, 0, 0, 0, 0, 0, 0, 0, 0>"
    assert name(binned=True) == "crc32_vring_kernel<2, 0, 0, 0, 1, 0, 0, 0, 0>"
    assert name(binned=True, wgs=2) == "crc32_vring_kernel<2, 0, 0, 0, 2, 0, 0, 0, 0>"
    assert name(binned=True, ablate=38912) == "crc32_vring_kernel<2, 0, 0, 19, 1, 0, 0, 0, 0>"
    assert name(binned=True, ablate=524288) == "crc32_vring_kernel<2, 0, 0, 0, 1, 0, 0, 0, 1>"
    assert name(binned=True, ablate=8388608) == "crc32_vring_kernel<2, 0, 0, 0, 1, 0, 0, 0, 0>"
    assert name(ablate=524288) == "crc32_vring_kernel<3, 0, 0, 0, 0, 0, 0, 0, 1>"
    assert name(ablate=8388608) == "crc32_vring_kernel<3, 0, 0, 0, 0, 0, 0, 0, 2>"
    # the one-launch local-tile records instance (batches of one tile per workgroup)
    assert name(binned=True, local_tiles=True) == "crc32_vring_kernel<2, 0, 0, 0, 3, 0, 0, 0, 0>"
    assert name(binned=True, local_tiles=True, wgs=2) == "crc32_vring_kernel<2, 0, 0, 0, 3, 0, 0, 0, 0>"
    assert name(binned=True, local_tiles=True, lanes=8) == "crc32_vring_kernel<3, 0, 0, 0, 3, 0, 0, 0, 0>"
    assert name(binned=True, local_tiles=True, path=17) == "crc32_vring_kernel<2, 0, 0, 0, 1, 0, 0, 0, 0>"
    assert name(binned=True, local_tiles=True, ablate=38912) == "crc32_vring_kernel<2, 0, 0, 19, 1, 0, 0, 0, 0>"


def test_shard_option_measures_one_cfg4_shard(monkeypatch):
    """`bench.py --config cfg4 --shard R/N`: rank R's contiguous shard
    of an N-GPU cfg4 run, measured alone on one device, so the driver's N-GPU curve
    has a per-GPU point to be read against; invalid with --gpus N or another config."""
    import io
    import contextlib
    import bench
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main(["--config", "cfg4", "--shard", "7/8", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"],
                   engine_factory=FakeEngine, cpu_factory=fake_cpu)
    d = json.loads([l for l in buf.getvalue().splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 1 and d["scaling"] == "strong"
    assert d["config"]["packets_per_gpu"] == (1 << 20) // 8
    assert "shard 7 of 8" in d["config"]["workload"] and d["config"]["parallelism"].startswith("shard 7/8 alone")
    for bad in (["--config", "cfg2", "--shard", "0/2"], ["--config", "cfg4", "--shard", "2/2"],
                ["--config", "cfg4", "--shard", "0/2", "--gpus", "2"]):
        with pytest.raises(SystemExit):
            bench.main(bad + ["--steps", "2", "--warmup", "1", "--no-cpu-baseline"], engine_factory=FakeEngine,
                       cpu_factory=fake_cpu)
