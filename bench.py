#!/usr/bin/env python3
"""bench.py -- device-resident batched CRC32 (ENet checksum path) on MI355X.

Metric (BASELINE.json): device-resident batched CRC32 GiB/s on 64 K x 1200 B
packets (cfg2) + fraction of the HBM-read roofline.  One STEP = one launch of
enet_hip_crc32_batch_device over one 75 MiB batch already resident in HBM.
Steps rotate over ROTATE distinct batches (> 256 MiB in total) so the Infinity
Cache cannot serve them.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

N > 1: every rank processes its own cfg2-sized partition (independent packet
shards, no collective on the data path: SURVEY.md §8e) -> "scaling": "weak".
value = sum of payload bytes over all ranks / max over ranks of the timed span.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "enet-csharp_amd"))

HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec, 8.0 TB/s (MI355X_MICROARCH.md)
GIB = float(1 << 30)
METRIC = "device-resident batched CRC32 GiB/s (64K×1200B) + % HBM-read peak"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rotate", type=int, default=5, help="distinct resident batches cycled through")
    ap.add_argument("--lanes", type=int, default=0, help="lanes per packet (0 = library default)")
    ap.add_argument("--wgs", type=int, default=0,
                    help="workgroups per CU (enet_hip_set_tuning; 0 = the library default: "
                         "2 for a multi-batch vring launch, 1 for a single batch)")
    ap.add_argument("--streams", type=int, default=6,
                    help="HIP streams the captured steps rotate over: batches are independent, so a "
                         "launch's prologue overlaps the previous launch's tail (1 = serial)")
    ap.add_argument("--config", default="cfg2", choices=["cfg2", "cfg3", "cfg4", "small"],
                    help="cfg2 = the metric's workload; cfg3 = mixed lengths; cfg4 = 1 M x 1200 B split into one "
                         "contiguous shard per rank (strong scaling); small = harness tests only")
    ap.add_argument("--list", type=int, default=5,
                    help="consecutive steps (batches) checksummed per launch through "
                         "enet_hip_crc32_batch_list_device (<= --rotate, so the batches of one launch "
                         "are distinct); 0 = one enet_hip_crc32_batch_device call per step.  A step is "
                         "always one pass over one batch")
    ap.add_argument("--path", type=int, default=0,
                    help="kernel path (enet_hip_set_kernel_path; 0 = the library default -- tuning sweeps only; "
                         "a path the product library does not build runs on libenethip_diag.so)")
    ap.add_argument("--ablate", type=int, default=0,
                    help="diagnostics library: enet_hip_diag_ablation value, set after the oracle gate "
                         "(WRONG CRCs by design: a measurement of the kernel's parts, never a result)")
    ap.add_argument("--binned", action="store_true",
                    help="length-binned entry (enet_hip_crc32_batch_device_binned): for mixed lengths (cfg3)")
    ap.add_argument("--launch", default="graph", choices=["graph", "direct"],
                    help="graph = the timed steps replayed from one captured HIP graph; direct = the same "
                         "launches enqueued one by one inside the timed region")
    ap.add_argument("--shard", default=None, metavar="R/N",
                    help="cfg4 only, no launcher: measure rank R's shard of an N-GPU cfg4 run on this one device "
                         "(the per-GPU point the driver's N-GPU scaling line should show)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="wall budget per CPU-baseline leg")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0 = every core this process may run on, sched_getaffinity)")
    ap.add_argument("--sustain-ms", type=float, default=30.0,
                    help="length of the serial sustained-rate region reported beside the value (0 = skip)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ distributed plumbing

def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return ws, rank, local


def dist_init(ws: int):
    if ws <= 1:
        return None
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # gloo: only the barrier and the max-over-ranks timing cross ranks (no data-path collective)
    dist.init_process_group(backend="gloo")
    return dist


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, x: float) -> float:
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, x: float) -> float:
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def timed_region(dist, sync, steps: int, step_fn):
    """barrier + sync | K steps | sync + barrier; returns this rank's seconds."""
    sync()
    barrier(dist)
    t0 = time.perf_counter()
    for i in range(steps):
        step_fn(i)
    sync()
    t1 = time.perf_counter()
    barrier(dist)
    return t1 - t0


# ------------------------------------------------------------------ the GPU engine

class GpuEngine:
    """Resident batches + launches through the C-ABI on torch's current stream."""

    def __init__(self, device: int, batches, lanes: int, wgs: int, diag: bool = False):
        import torch
        import enethip
        if not torch.cuda.is_available():
            raise SystemExit("bench.py: no GPU visible -- the HIP path has no CPU fallback")
        # one rank per GPU; more ranks than GPUs (the 2-rank test on a 1-GPU box) share them
        device %= torch.cuda.device_count()
        torch.cuda.set_device(device)
        self.torch = torch
        self.ctx = enethip.Context(device, lanes, wgs, diag=diag)
        self.num_cus = torch.cuda.get_device_properties(device).multi_processor_count
        self.stream = torch.cuda.Stream()          # dedicated stream: handle != 0
        self.h = self.stream.cuda_stream
        self.streams = [self.stream]
        self.bufs = []
        for b in batches:
            self.bufs.append(dict(
                payload=torch.from_numpy(b.payload).cuda(),
                off=torch.from_numpy(b.off.view(np.int64)).cuda(),
                lens=torch.from_numpy(b.lens.view(np.int32)).cuda(),
                out=torch.zeros(b.n, dtype=torch.int32, device="cuda"),
                n=b.n, nbytes=b.payload_bytes))
        self.sink = torch.zeros(4, dtype=torch.int32, device="cuda")
        self.graph = None
        self.binned = False
        self.list = 0                              # batches per launch (batch-list entry), 0 = off
        self.ws = {}                               # binned: one workspace per stream
        torch.cuda.synchronize()

    def set_streams(self, n: int):
        self.streams = [self.stream] + [self.torch.cuda.Stream() for _ in range(max(1, n) - 1)]

    def set_binned(self, on: bool):
        self.binned = on
        if on:
            nb = self.ctx.binned_workspace_size(max(b["n"] for b in self.bufs))
            for s in self.streams:
                self.ws[s.cuda_stream] = self.torch.zeros(nb, dtype=self.torch.uint8, device="cuda")

    def set_list(self, n: int):
        self.list = min(n, len(self.bufs))    # the batches of one launch are distinct

    def launch_plan(self, steps: int) -> list:
        """(first step, step count) of each launch covering steps 0 .. steps-1: one
        step per launch, or --list consecutive steps per batch-list launch."""
        per = self.list or 1
        return [(i, min(per, steps - i)) for i in range(0, steps, per)]

    def launch(self, first: int, count: int, stream=None):
        """Checksum steps first .. first+count-1 (step i = resident batch i % rotate)."""
        h = self.h if stream is None else stream.cuda_stream
        if self.list:
            bs = [self.bufs[(first + t) % len(self.bufs)] for t in range(count)]
            self.ctx.crc32_batch_list_device([(x["payload"], x["off"], x["lens"], x["n"], x["out"]) for x in bs], h)
        else:
            for t in range(count):
                self.step(first + t, stream)

    def step(self, i: int, stream=None):
        b = self.bufs[i % len(self.bufs)]
        h = self.h if stream is None else stream.cuda_stream
        if self.binned:
            w = self.ws[h]
            self.ctx.crc32_batch_device_binned(b["payload"], b["off"], b["lens"], b["n"], b["out"], w, w.numel(), h)
        else:
            self.ctx.crc32_batch_device(b["payload"], b["off"], b["lens"], b["n"], b["out"], h)

    def probe(self, i: int):
        b = self.bufs[i % len(self.bufs)]
        self.ctx.read_probe_device(b["payload"], (b["payload"].numel() // 16) * 16, self.sink, self.h)

    def sync(self):
        self.torch.cuda.synchronize()

    def capture(self, steps: int):
        """Capture the launches of `steps` steps (rotating batches) into one HIP graph:
        the timed region then replays it with one host call, so host launch overhead
        (Python + ctypes) cannot starve the GPU.  Each graph node is one ordinary
        launch; launch k goes to stream k % len(streams) (independent batches:
        consecutive launches may overlap at their boundary, every launch still
        checksums all of its batches)."""
        torch = self.torch
        self.sync()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=self.stream):
            for s in self.streams[1:]:
                s.wait_stream(self.stream)
            for k, (first, count) in enumerate(self.launch_plan(steps)):
                self.launch(first, count, self.streams[k % len(self.streams)])
            for s in self.streams[1:]:
                self.stream.wait_stream(s)
        self.sync()
        self.graph = g

    def replay(self, _i: int = 0):
        self.graph.replay()

    def direct(self, steps: int):
        """The captured launches, enqueued directly (same streams, same fork/join)."""
        for s in self.streams[1:]:
            s.wait_stream(self.stream)
        for k, (first, count) in enumerate(self.launch_plan(steps)):
            self.launch(first, count, self.streams[k % len(self.streams)])
        for s in self.streams[1:]:
            self.stream.wait_stream(s)

    def kernel_ms(self, fn, steps: int) -> tuple[float, float]:
        """HIP events on the launch stream: (mean per-launch kernel ms, span ms per
        step).  A spin kernel heads the queue so every event/launch pair is enqueued
        before the GPU reaches it: the events then bracket the kernels only."""
        torch = self.torch
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * steps)]
        self.sync()
        with torch.cuda.stream(self.stream):
            torch.cuda._sleep(int(2e8))          # ~0.1 s of spin on the GPU
            for i in range(steps):
                ev[2 * i].record(self.stream)
                fn(i)
                ev[2 * i + 1].record(self.stream)
        self.sync()
        per = [ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(steps)]
        span = ev[0].elapsed_time(ev[-1]) / steps
        return float(np.median(per)), float(span)

    def region_ms(self, fn, steps: int) -> float:
        """Average launch duration over a serial timed region: two HIP events on the
        launch stream around `steps` back-to-back launches (no events in between, so
        no per-event boundary cost; the inter-launch gaps are included, which makes
        this an upper bound on the kernel's own duration).  A spin kernel heads the
        queue so host launch overhead cannot leave the GPU idle between launches."""
        torch = self.torch
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        self.sync()
        with torch.cuda.stream(self.stream):
            torch.cuda._sleep(int(2e8))
            e0.record(self.stream)
            for i in range(steps):
                fn(i)
            e1.record(self.stream)
        self.sync()
        return float(e0.elapsed_time(e1)) / steps

    def outputs(self, j: int) -> np.ndarray:
        return self.bufs[j]["out"].cpu().numpy().view(np.uint32)


# ------------------------------------------------------------------ CPU baseline

def host_cores() -> int:
    """The cores this process may run on (its affinity mask: taskset limits included),
    not the machine's count.  A cgroup CPU quota is not visible here: see
    cgroup_cpu_quota()."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cgroup_cpu_quota():
    """(CPUs the cgroup's CPU quota allows = quota / period, the file it came from), or
    (None, file) when unlimited or unreadable.  cgroup v2 cpu.max of this process's own
    group (then the root's), else v1 cfs_quota_us / cfs_period_us.  The affinity mask
    can list far more cores than the quota lets the process use at once (a 16-CPU
    share of a 256-thread host), and a thread count above the quota only time-slices."""
    cands = []
    try:
        for line in open("/proc/self/cgroup"):
            parts = line.strip().split(":", 2)
            if len(parts) == 3 and parts[0] == "0":
                cands.append(f"/sys/fs/cgroup{parts[2]}/cpu.max")
    except OSError:
        pass
    cands.append("/sys/fs/cgroup/cpu.max")
    for p in cands:
        try:
            q, per = open(p).read().split()[:2]
        except (OSError, ValueError):
            continue
        return (None if q == "max" else float(q) / float(per)), p
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return (None if q <= 0 else q / per), "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"
    except (OSError, ValueError):
        return None, None


def baseline_threads(requested: int = 0) -> tuple[int, dict]:
    """Threads for the all-cores CPU leg: the affinity mask's cores, capped by the
    cgroup quota (rounded up), unless `requested` says otherwise; plus what was read."""
    aff = host_cores()
    quota, src = cgroup_cpu_quota()
    th = requested or (min(aff, max(1, int(np.ceil(quota)))) if quota else aff)
    return th, {"affinity_cores": aff, "cgroup_cpu_quota": None if quota is None else round(quota, 2),
                "cgroup_file": src}


def cpu_baseline(batch, budget_s: float, threads: int = 0, runs: int = 5):
    """The oracle's C restatement of packet.cs:142-160 (kind "port": the C# reference
    cannot run here), timed on this host on a bounded sample of the same batch, as
    SURVEY §8d asks: one thread, and all the cores the process may use (static
    contiguous packet partition, one pthread per core); the median of `runs` timed
    runs each.  A run is one call over a sample sized to budget_s / runs seconds, so
    every thread gets one contiguous multi-MB range (thread start is noise)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    lib = oracle.OracleLib()
    threads, info = baseline_threads(threads)
    res = {"host": info}
    for label, th in (("1thread", 1), ("all", threads)):
        # calibration: the first packets of the batch, then a sample sized to one run
        n = batch.n
        k = min(n, 4096 * th)
        t0 = time.perf_counter()
        out = lib.batch(batch.payload, batch.off[:k], batch.lens[:k], threads=th)
        dt = max(time.perf_counter() - t0, 1e-6)
        rate = float(batch.lens[:k].astype(np.uint64).sum()) / dt
        per_run = budget_s / max(1, runs)
        sample_n = int(min(n, max(k, rate * per_run / max(1.0, float(batch.lens.mean())))))
        nb = float(batch.lens[:sample_n].astype(np.uint64).sum())
        reps = max(1, int(rate * per_run / max(1.0, nb)))       # (the whole batch is shorter than a run)
        rates = []
        for _ in range(max(1, runs)):
            t0 = time.perf_counter()
            for _ in range(reps):
                out = lib.batch(batch.payload, batch.off[:sample_n], batch.lens[:sample_n], threads=th)
            rates.append(nb * reps / (time.perf_counter() - t0) / GIB)
        res[label] = dict(gibps=float(np.median(rates)), threads=th, packets=sample_n, reps=reps, runs=len(rates),
                          spread=[round(min(rates), 3), round(max(rates), 3)])
        del out
    res["speedup"] = res["all"]["gibps"] / max(res["1thread"]["gibps"], 1e-9)
    return res


# ------------------------------------------------------------------ main

# cfg4: a shard must stay out of the Infinity Cache (256 MiB) across steps, so a
# rank whose shard is smaller keeps this many bytes of copies of it resident
CFG4_RESIDENT = 320 << 20


def make_batches(cfg: str, rotate: int, rank: int, world: int = 1):
    from enethip import workloads
    if cfg == "cfg4":                                  # shard `rank` of `world`, contiguous packets
        b = workloads.cfg4(rank, world)
        copies = max(1, -(-CFG4_RESIDENT // max(1, b.payload_bytes)))
        return [b] * copies                            # the same bytes in `copies` distinct device buffers
    out = []
    for j in range(rotate):
        seed = workloads.SEED_PAYLOAD + 7919 * (rank * rotate + j)
        if cfg == "cfg2":
            out.append(workloads.fixed(65536, 1200, seed=seed, name="cfg2"))
        elif cfg == "small":
            out.append(workloads.fixed(2048, 1200, seed=seed, name="small"))
        elif cfg.startswith("fixed:"):                 # tools only: fixed:<packets>[:<bytes>]
            parts = cfg.split(":")
            out.append(workloads.fixed(int(parts[1]), int(parts[2]) if len(parts) > 2 else 1200, seed=seed,
                                       name=cfg))
        else:
            out.append(workloads.mixed(262144, 64, 1400, seed=seed, name="cfg3"))
    return out


PRODUCT_PATHS = (0, 13, 17)                # built in libenethip.so (the rest: libenethip_diag.so)
PRODUCT_LANES = (0, 4, 8)                  # lanes per packet libenethip.so takes (the rest: diagnostics)


def kernel_name(args, list_launch: bool = False, local_tiles: bool = False) -> str:
    """The dominant kernel of the measured entry point (as rocprofv3 names it:
    crc32_vring_kernel<LG, TR, NT, ABL, BIN, WK, ROT, VF, DYN>; DYN = 1 / 2, the chip-wide
    / pair rounds, when the diagnostics ablation 524288 / 8388608 selects them).
    local_tiles: the binned batch fits one tile per workgroup, so the default path runs
    the one-launch local-tile records instance (BIN = 3)."""
    path = getattr(args, "path", 0)
    if list_launch and path == 13 and args.lanes in (0, 4, 8) and not args.binned:
        # batch lists: the lean kernel's list instance, 8 lanes per packet unless set
        return f"crc32_lean_list_kernel<{3 if args.lanes in (0, 8) else 2}, 16, 2>"
    lanes = args.lanes or (4 if args.binned else 8)   # the library's defaults (auto_lanes / binned)
    lg = {4: 2, 8: 3}.get(lanes)
    if path and path not in (17, 18, 21):
        return f"kernel path {path}"
    dyn = 2 if (args.ablate & 8388608) else 1 if (args.ablate & 524288) else 0   # (pair / chip-wide rounds)
    if args.binned and local_tiles and path == 0 and args.ablate == 0 and lg is not None:
        return f"crc32_vring_kernel<{lg}, 0, 0, 0, 3, 0, 0, 0, 0>"
    if args.binned:
        dyn = 0 if dyn == 2 else dyn                          # (no pair rounds for the records instance)
        abl = (args.ablate >> 11) & 255
        abl = abl if abl in (2, 19, 64, 83) and lg == 2 else 0   # (the records instance's ablations, 4 lanes)
        dyn = 0 if abl else dyn
        bin_ = 2 if getattr(args, "wgs", 0) >= 2 else 1          # (two workgroups per CU: the compact instance)
        return (f"crc32_vring_kernel<{lg}, 0, 0, {abl}, {bin_}, 0, 0, 0, {dyn}>" if path in (0, 17)
                else f"crc32_lean_kernel<0, {lg}, 16, 2, 128>")
    if lg is None:
        return "crc32_stream_kernel / crc32_direct_kernel"
    nt, rot = (1 if path == 18 else 0), (1 if path == 21 else 0)
    dyn = dyn if not (nt or rot or (args.ablate & ~(524288 | 8388608))) else 0
    return f"crc32_vring_kernel<{lg}, 0, {nt}, 0, 0, 0, {rot}, 0, {dyn}>"


def load_traffic(cfg: str, binned: bool = False, lib_sha256: str | None = None):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/), or None
    when there is none for this entry: profiles/traffic_<cfg>.json is the plain /
    batch-list entry's, traffic_<cfg>_binned.json the length-binned entry's, and each
    file's "binned" tag must agree with its name.  The pass records the sha256 of the
    library it ran (tools/traffic.py): a record of any other build -- an older pass, a
    rebuilt library, the diagnostics library -- is not this run's traffic, so None
    (VERDICT r5 #2)."""
    p = os.path.join(ROOT, "profiles", f"traffic_{cfg}{'_binned' if binned else ''}.json")
    try:
        doc = json.load(open(p))
    except (OSError, ValueError):
        return None
    if bool(doc.get("binned", False)) != bool(binned):
        return None
    if lib_sha256 is None or doc.get("library_sha256") != lib_sha256:
        return None
    return doc


def cpu_line(cpu: dict) -> dict:
    """The bench line's cpu_baseline object from cpu_baseline()'s result."""
    a, one, host = cpu["all"], cpu["1thread"], cpu["host"]
    quota = host.get("cgroup_cpu_quota")
    return {
        "value": round(a["gibps"], 3),
        "unit": "GiB/s",
        "cores": a["threads"],
        "kind": "port",
        "sample": (f"oracle C restatement of packet.cs:142-160 (byte-serial loop, one ENetBuffer per packet), "
                   f"first {a['packets']} packets of the cfg batch x {a['reps']} per run, median of {a['runs']} "
                   f"runs (spread {a['spread'][0]}-{a['spread'][1]} GiB/s) on {a['threads']} threads; "
                   f"1 thread: {one['gibps']:.3f} GiB/s (median of {one['runs']}); measured speed-up "
                   f"{cpu['speedup']:.1f}x over 1 thread; host: {host['affinity_cores']} cores in the affinity "
                   f"mask, cgroup CPU quota {quota if quota is not None else 'none'}"
                   f"{' (' + host['cgroup_file'] + ')' if host.get('cgroup_file') else ''}"),
        "speedup_vs_1thread": round(cpu["speedup"], 2),
        "one_thread": round(one["gibps"], 3),
        "cgroup_cpu_quota": quota,
        "affinity_cores": host["affinity_cores"],
    }


def _rank_main(rank: int, n: int, port: int, argv, engine_factory, cpu_factory):
    """One self-launched rank (spawn start method: a fresh interpreter that has not
    touched the GPU)."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.exit(main(argv, engine_factory, cpu_factory))


def spawn_ranks(n: int, argv, engine_factory=None, cpu_factory=None) -> int:
    """`bench.py --gpus N` with no launcher around it: start N rank processes (one per
    GPU, as torch.distributed.run would: RANK / LOCAL_RANK / WORLD_SIZE, rendezvous on
    127.0.0.1) and return the worst exit code.  This process never initialises the GPU,
    and the ranks are children (no exec).  Rank 0 prints the one line."""
    import socket
    import multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_rank_main, args=(r, n, port, argv, engine_factory, cpu_factory)) for r in range(n)]
    for p in ps:
        p.start()
    for p in ps:
        p.join()
    codes = [p.exitcode for p in ps]
    bad = [c for c in codes if c != 0]
    if bad:
        print(f"bench.py: self-launched ranks exited with {codes}", file=sys.stderr)
        return 1
    return 0


def main(argv=None, engine_factory=None, cpu_factory=None):
    args = parse(argv)
    ws, rank, local = dist_env()
    if args.shard and args.gpus > 1:
        raise SystemExit("bench.py: --shard R/N measures one shard on one device (no --gpus N)")
    if ws <= 1 and args.gpus > 1:
        # no launcher: measure N GPUs by starting the N ranks here (never print a
        # one-rank line for --gpus N)
        return spawn_ranks(args.gpus, argv if argv is not None else sys.argv[1:], engine_factory, cpu_factory)
    if ws > 1 and args.gpus != ws:
        print(f"bench.py: --gpus {args.gpus} under a launcher of {ws} ranks: measuring {ws}", file=sys.stderr)
        args.gpus = ws
    shard = None
    if args.shard:
        r_, n_ = (int(x) for x in args.shard.split("/"))
        if args.config != "cfg4" or ws != 1 or not 0 <= r_ < n_:
            raise SystemExit("bench.py: --shard R/N needs --config cfg4, one process and 0 <= R < N")
        shard = (r_, n_)
    dist = dist_init(ws)
    batches = make_batches(args.config, args.rotate, *(shard if shard else (rank, ws)))
    diag = args.path not in PRODUCT_PATHS or args.lanes not in PRODUCT_LANES or args.ablate != 0
    eng = (engine_factory or GpuEngine)(local, batches, args.lanes, args.wgs, *((diag,) if diag else ()))
    if hasattr(eng, "set_streams"):
        eng.set_streams(args.streams)
    if args.path:
        eng.ctx.set_kernel_path(args.path)
    if args.binned:
        eng.set_binned(True)
    if args.list > 1 and not args.binned and hasattr(eng, "set_list"):   # (binned: one batch per launch)
        eng.set_list(args.list)
    plan = eng.launch_plan(args.steps) if hasattr(eng, "launch_plan") else [(i, 1) for i in range(args.steps)]
    per_launch_steps = plan[0][1]             # steps (batches) one launch checksums

    # correctness gate (untimed): first resident batch vs the oracle
    eng.step(0)
    eng.sync()
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    exp = oracle.OracleLib().batch(batches[0].payload, batches[0].off, batches[0].lens, threads=8)
    if not (eng.outputs(0) == exp).all():
        raise SystemExit("bench.py: GPU CRCs differ from the oracle -- refusing to report a number")

    if args.ablate:                       # (diagnostics: from here on the CRCs are wrong by design)
        eng.ctx.diag_ablation(args.ablate)
    for first, count in (eng.launch_plan(args.warmup) if hasattr(eng, "launch_plan") else
                         [(i, 1) for i in range(args.warmup)]):
        eng.launch(first, count) if hasattr(eng, "launch") else eng.step(first)
    if hasattr(eng, "capture"):
        eng.capture(args.steps)
        for bf in eng.bufs:               # one untimed replay (graph upload / warm), checked:
            bf["out"].zero_()             # every rotating batch's CRCs from the graph vs the oracle
        eng.replay()
        eng.sync()
        lib = oracle.OracleLib()
        for j in range(0 if args.ablate else min(args.steps, len(batches))):
            ref = lib.batch(batches[j].payload, batches[j].off, batches[j].lens, threads=8)
            if not (eng.outputs(j) == ref).all():
                raise SystemExit(f"bench.py: graph replay CRCs of batch {j} differ from the oracle")
        eng.replay()                      # untimed again: the GPU idled through the oracle check
        eng.sync()
        if args.launch == "direct":
            secs = timed_region(dist, eng.sync, 1, lambda _i: eng.direct(args.steps))
        else:
            secs = timed_region(dist, eng.sync, 1, eng.replay)
    else:
        secs = timed_region(dist, eng.sync, args.steps, eng.step)    # (engines without a graph)
    secs_max = max_over_ranks(dist, secs)
    bytes_rank = float(sum(batches[i % len(batches)].payload_bytes for i in range(args.steps)))
    bytes_all = sum_over_ranks(dist, bytes_rank)
    value = bytes_all / secs_max / GIB

    # per-launch kernel duration via HIP events on the launch stream (for the roofline)
    # (a) serial timed region, events at its two ends only -> roofline.achieved;
    # (b) each launch bracketed by its own event pair (median), reported beside it
    nk = min(len(plan), 100)
    lfn = (lambda k: eng.launch(*plan[k])) if hasattr(eng, "launch") else eng.step
    r_ms = eng.region_ms(lfn, nk)
    k_ms, span_ms = eng.kernel_ms(lfn, nk)
    p_ms = eng.region_ms(eng.probe, nk)
    # sustained: the same serial launches over a region of --sustain-ms (the burst
    # value above is a short replay; a box's clocks settle over several ms of load)
    sus = None
    if args.sustain_ms > 0 and hasattr(eng, "launch"):
        nsus = max(nk, int(args.sustain_ms / max(r_ms, 1e-3)))
        s_ms = eng.region_ms(lambda k: eng.launch(*plan[k % len(plan)]), nsus)
        sus = {"GiBps": round(float(batches[0].payload_bytes) * sum(plan[k % len(plan)][1] for k in range(nsus)) /
                              (s_ms * nsus * 1e-3) / GIB, 1),
               "launches": nsus, "ms": round(s_ms * nsus, 2)}
    per_launch = float(batches[0].payload_bytes) * sum(c for _, c in plan[:nk]) / nk
    probe_bytes = float((batches[0].payload.nbytes // 16) * 16)
    achieved = per_launch / (r_ms * 1e-3) / 1e9
    probe = probe_bytes / (p_ms * 1e-3) / 1e9

    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:    # (the CPU baseline: rank 0 at N = 1 only)
        cpu = (cpu_factory or cpu_baseline)(batches[0], args.cpu_seconds, args.cpu_threads)

    # the binned entry's one-launch form: the batch fits one tile of <= 1024 packets per
    # workgroup (crc32_kernels.hip enet_hip_crc32_batch_device_binned)
    wgs_eff = min(args.wgs, 2) if args.wgs >= 1 else 2       # (the local tiles' default: two per CU)
    local_tiles = (args.binned and args.path == 0 and args.ablate == 0 and
                   batches[0].n <= 1024 * getattr(eng, "num_cus", 0) * wgs_eff)
    if rank == 0:
        import enethip
        traffic = load_traffic(args.config, args.binned, enethip.library_sha256(diag))
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(secs_max / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "strong" if args.config == "cfg4" else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 payload, device-resident)",
            "config": {
                "workload": {"cfg2": "cfg2: 65536 packets x 1200 B packed",
                             "cfg3": "cfg3: 262144 packets x U[64,1400] B packed",
                             "cfg4": (f"cfg4: 1048576 packets x 1200 B, shard {shard[0]} of {shard[1]} (contiguous "
                                      f"packets) measured alone on one device" if shard else
                                      f"cfg4: 1048576 packets x 1200 B, shard {rank} of {ws} (contiguous packets)"),
                             "small": "small: 2048 packets x 1200 B (harness tests)"}[args.config] +
                            f", {len(batches)} rotating resident batches per GPU",
                "packets_per_gpu": batches[0].n,
                "payload_bytes_per_step": int(batches[0].payload_bytes),
                "steps_per_launch": per_launch_steps,
                "parallelism": (f"shard {shard[0]}/{shard[1]} alone (the per-GPU point of {shard[1]} independent "
                                f"shards)" if shard else f"{ws} independent shards (no collective)"),
                "lanes_per_packet": args.lanes or "default",
                "streams": args.streams,
                "entry": ("enet_hip_crc32_batch_device_binned" if args.binned else
                          "enet_hip_crc32_batch_list_device" if per_launch_steps > 1 else
                          "enet_hip_crc32_batch_device"),
                "workgroups_per_cu": args.wgs or f"default ({2 if per_launch_steps > 1 or local_tiles else 1})",
                "launch": args.launch,
                "kernel_path": args.path,
                **({"ablation": args.ablate, "note": "ABLATION: wrong CRCs by design"} if args.ablate else {}),
            },
            "hbm_read_frac": round(value * GIB / 1e9 / (HBM_PEAK_GBPS * ws), 4),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": (None if not (traffic or {}).get("hbm_bytes_per_batch") else
                            round(traffic["hbm_bytes_per_batch"] * per_launch / float(batches[0].payload_bytes))),
                "traffic_source": (None if not traffic else
                                   f"profiles/traffic_{args.config}{'_binned' if args.binned else ''}.json "
                                   f"(FETCH_SIZE pass of library sha256 {traffic['library_sha256'][:12]}, "
                                   f"the build this run loaded)"),
                "kernel": kernel_name(args, per_launch_steps > 1, local_tiles),
                "kernel_ms": round(r_ms, 5),
                "kernel_ms_timing": f"HIP events around {nk} serial launches on the launch stream",
                "kernel_ms_bracketed_median": round(k_ms, 5),
                "read_probe_GBps": round(probe, 1),
            },
            "sustained": sus,
            "cpu_baseline": None if cpu is None else cpu_line(cpu),
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
