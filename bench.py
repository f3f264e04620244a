#!/usr/bin/env python3
"""bench.py — encode+decode GB/s of the MI355X Huffman byte codec.

BASELINE.json metric: "encode+decode GB/s on 1 GiB bytes at 1/2/4/8 MI355X;
% HBM roofline". One step = one pass of the hot path over the rank's bytes,
inputs resident in HBM when the timed region starts:

    hist256 (pass 1) -> [N>1: ONE RCCL all-gather of a 258 x int64 row
    (weights + 8 tail bytes) inside the library, huff_mgpu_compress] ->
    host HuffTree -> chunk bits + scan -> pack (pass 2) -> block-parallel decode

--scaling weak (default): every rank holds --bytes-per-gpu (1 GiB), its slice
of one global synthetic stream generated on device by offset; value = bytes
of all ranks / max over ranks of the step time.
--scaling strong: --total-bytes (1 GiB) split N ways (SURVEY §8d's 1/2/4/8
curve); a 512 MiB buffer is rewritten between timed steps so no rank's shard
sits in the 256 MiB Infinity Cache; each step is bracketed by barriers and
its time summed.

At N=1 the headline is configs[1] (1 GiB uniform); a side result carries
configs[2] (1 GiB Zipf(1.2), the general pack/decode kernels) with its own
kernels, roofline and cpu_baseline (--side none skips it).

Run: python bench.py [--gpus N --steps K --warmup W --workload uniform|zipf|text]
     N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "huff-encoding_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import huff_coding as H  # noqa: E402
from huff_coding import device as D  # noqa: E402
from huff_coding import mgpu  # noqa: E402

METRIC = "encode+decode GB/s on 1 GiB bytes at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
SEEDS = {"uniform": 0x5EED0001, "zipf": 0x5EED0002, "text": 0x5EED0005}
CONFIG_OF = {"uniform": "BASELINE configs[1]", "zipf": "BASELINE configs[2]",
             "text": "stand-in for configs[4] enwik8"}


def human(n: int) -> str:
    for unit, s in (("GiB", 30), ("MiB", 20), ("KiB", 10)):
        if n >= 1 << s and n % (1 << s) == 0:
            return f"{n >> s} {unit}"
    return f"{n} B"


def enwik8_path():
    """$ENWIK8: the real text when the box has it"""
    p = os.environ.get("ENWIK8")
    return p if p and os.path.isfile(p) else None


def cgroup_cpu_quota(root: str = "/sys/fs/cgroup"):
    """CPUs' worth of time the cgroup grants (cgroup v2 cpu.max "<quota>
    <period>", else v1 cfs_quota_us / cfs_period_us); None when unlimited or
    unknown. A mask of many threads may still get only this many CPUs."""
    try:
        with open(os.path.join(root, "cpu.max")) as f:
            q, per = f.read().split()[:2]
            return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:  # cgroup v1
        with open(os.path.join(root, "cpu", "cpu.cfs_quota_us")) as f, \
                open(os.path.join(root, "cpu", "cpu.cfs_period_us")) as g:
            q, per = int(f.read()), int(g.read())
            return round(q / per, 2) if q > 0 else None
    except (OSError, ValueError):
        return None


def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = cgroup_cpu_quota()
    return {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cpu_model": model,
            "cgroup_cpu_quota": quota}


def cpu_baseline(workload: str, target_s: float):
    """The oracle's restatement of the reference CPU path (12-thread rationed
    histogram, host tree, bit-serial encode, bit-walk decode), timed on a
    bounded sample of the same workload on this host."""
    import oracle as O

    gen = {"uniform": O.gen_uniform, "zipf": O.gen_zipf, "text": O.gen_text}[workload]

    def run(nbytes):
        data = gen(SEEDS[workload], nbytes)
        t0 = O.now()
        w = O.weights_threaded(data, 12)
        tree = O.Tree.from_weights(w)
        comp, pad = O.compress_with_tree(data, tree)
        t1 = O.now()
        back = O.decompress(comp, pad, tree)
        t2 = O.now()
        assert back == data.tobytes()
        return t1 - t0, t2 - t1

    e, d = run(1 << 20)
    scale = max(1.0, target_s / max(e + d, 1e-6))
    n = int(min(256 << 20, (1 << 20) * scale)) & ~0xFFFF
    e, d = run(n)
    # "cpu-fast" (SURVEY §8d): table-driven encode/decode on ALL the host
    # threads in this process's affinity mask (the honest upper CPU
    # reference), and on 16 (the box's nominal CPU share) beside it; a 1 GiB
    # sample of the same stream (256 MiB when the mask has <= 16 threads);
    # second of two runs (the first faults the pages in)
    aff = max(1, len(os.sched_getaffinity(0)))

    def fast(threads, nbytes):
        data = gen(SEEDS[workload], nbytes)
        for _ in range(2):
            _, back, fe, fd = O.fast_roundtrip(data, threads)
        assert np.array_equal(back, data)
        return {"value": round(nbytes / (fe + fd) / 1e9, 4), "unit": "GB/s", "cores": threads,
                "encode_GBps": round(nbytes / fe / 1e9, 4), "decode_GBps": round(nbytes / fd / 1e9, 4),
                "sample": f"{nbytes} B; table-driven histogram+tree+encode and 12-bit-table decode "
                          f"(oracle fast_roundtrip), {threads} threads"}

    f_all = fast(aff, max(n, (1 << 30) if aff > 16 else (256 << 20)))
    f_16 = fast(min(16, aff), max(n, 256 << 20)) if aff > 16 else None
    return {"value": round(n / (e + d) / 1e9, 6), "unit": "GB/s", "cores": 12, "kind": "port",
            "host": cpu_info(),
            "sample": f"{n} B of the same {workload} stream; encode {n / e / 1e9:.4f} GB/s (12-thread "
                      f"histogram + 1-thread bit-serial encode), decode {n / d / 1e9:.4f} GB/s (1-thread "
                      f"tree walk); oracle/huff_oracle.c restatement of huff_coding (Rust not buildable here)",
            "fast": f_all, "fast_16_threads": f_16}


PHASE_KERNELS = {  # bench phase -> device kernels (names as in tools/summarize_prof.py)
    "hist": ["k_hist1x2", "k_rows_sum"],
    "chunk_bits": ["k_chunk_bits"],
    "scan": ["k_scan_tiles", "k_scan_fix"],
}


# the index-free decode pipeline of the general path: its
# kernels' HBM bytes per launch from profiles/traffic_<kind>_indexfree.json
# (tools/make_traffic.py over a kbench --phase indexless PMC run)
INDEXFREE_KERNELS = ["k_spec_lds", "k_fix_list", "k_fix_chain", "k_scan_tiles", "k_scan_fix_small", "k_mark_lite",
                     "k_decode_fixed_skip"]


def traffic_name(kind, fixed8):
    """the PMC summary's workload name: the general kernels on all-8-bit
    uniform bytes (the `general` record, HUFF_DISABLE_FIXED8=1) have their own
    (profiles/traffic_uniform_general*.json, tools/gpu_r6_traffic.sh)"""
    return f"{kind}_general" if kind == "uniform" and not fixed8 else kind


def indexfree_traffic(kind, fixed8):
    """HBM bytes of one index-free decode of the 1 GiB job: the byte map's
    for all-8-bit codes, else the sum over the pipeline's kernels"""
    if fixed8:
        return dominant_traffic(kind, "decode", True, None)
    path = os.path.join(ROOT, "profiles", f"traffic_{traffic_name(kind, fixed8)}_indexfree.json")
    if not os.path.exists(path):
        return None, None
    t = json.load(open(path))
    if not all(k in t for k in INDEXFREE_KERNELS):
        return None, None
    return int(sum(t[k]["hbm_bytes"] for k in INDEXFREE_KERNELS)), os.path.relpath(path, ROOT)


def dominant_traffic(kind, phase, fixed8, dec_kernel):
    """HBM bytes per launch of the dominant phase from the committed PMC
    summary of this workload (profiles/traffic_<kind>.json, written by
    tools/make_traffic.py from a rocprofv3 --pmc run of the same kernels)."""
    path = os.path.join(ROOT, "profiles", f"traffic_{traffic_name(kind, fixed8)}.json")
    if not os.path.exists(path):
        return None, None
    t = json.load(open(path))
    names = PHASE_KERNELS.get(phase)
    if phase == "pack":
        names = ["k_bytemap"] if fixed8 else ["k_pack"]
    elif phase == "decode":
        names = ["k_bytemap"] if fixed8 else [dec_kernel or "k_decode_fixed"]
    if not names or not all(n in t for n in names):
        return None, None
    return int(sum(t[n]["hbm_bytes"] for n in names)), os.path.relpath(path, ROOT)


class Setup:
    def __init__(self, args, world, rank, local):
        self.args, self.world, self.rank, self.local = args, world, rank, local
        self.ctx = H.Context(local)
        self.stream = torch.cuda.current_stream()
        self.ctx.set_stream(self.stream.cuda_stream)
        self.nccl = args.dist_backend == "nccl"
        self.dev = torch.device("cuda", local) if self.nccl else None
        self.comm, self.comm_note = None, None
        if world > 1 and self.nccl:
            self.comm, self.comm_note = self.native_comm()
        self.dx = mgpu.DeviceExchange(self.dev) if world > 1 and self.nccl and self.comm is None else None
        self._flush = None
        self.ceil = None
        self.rccl_world = self.observed_world()

    def flush_buffer(self):
        """512 MiB rewritten before each strong-scaling step: no shard stays
        in the 256 MiB Infinity Cache"""
        if self._flush is None:
            self._flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
        return self._flush

    def observed_world(self):
        """the world size RCCL itself reports (ncclCommCount through
        huff_comm_world) on the communicator the step uses, checked equal on
        every rank; at N = 1 the step runs no collective (said so); with gloo
        (rehearsal) torch's group size, labelled so"""
        if self.world == 1:
            return {"world": 1, "source": "single rank: the step runs no collective"}
        if not self.nccl:
            return {"world": dist.get_world_size(), "source": "torch.distributed gloo group (no RCCL: rehearsal)"}
        if self.comm is None:
            return {"world": None, "source": "no library communicator (torch RCCL all_gather)"}
        # every rank reaches the all_reduce below, also one whose readout
        # failed (a sentinel), so no rank blocks in it
        note = None
        try:
            w, r = self.comm.observed_world()
        except Exception as e:
            w, r, note = -1, -1, f"huff_comm_world failed on rank {self.rank}: {e}"
        t = torch.tensor([w, -w, int(r != self.rank)], device=self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        lo, hi, bad = -int(t[1].item()), int(t[0].item()), int(t[2].item())
        if note or lo != hi or bad or lo < 1:
            return {"world": None, "source": note or f"ranks disagree: RCCL world {lo}..{hi}, rank mismatch {bad}"}
        return {"world": w, "source": "ncclCommCount / ncclCommUserRank via huff_comm_world"}

    def native_comm(self):
        """the library's own RCCL communicator (huff_comm) on every rank, or
        none on any (then torch's RCCL group carries the one all-gather; the
        JSON says which ran). Ranks agree before and after the collective init."""
        uid, note = None, None
        if self.rank == 0:
            try:
                uid = mgpu.NativeComm.unique_id()
            except Exception as e:
                note = f"huff_comm_unique_id failed: {e}"
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        comm = None
        if obj[0] is not None:
            try:
                comm = mgpu.NativeComm(self.ctx, self.world, self.rank, obj[0])
            except Exception as e:
                note = f"huff_comm_init failed on rank {self.rank}: {e}"
        ok = torch.tensor([1 if comm is not None else 0], device=self.dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            if comm is not None:
                comm.close()
            return None, (note or "huff_comm unavailable on another rank") + "; torch RCCL all_gather used"
        return comm, None

    def barrier(self):
        if self.world > 1:
            dist.barrier()

    def max_over_ranks(self, v: float) -> float:
        if self.world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=self.dev or "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())


def make_input(s: Setup, kind: str, n: int):
    x = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    src = "synthetic (counter-based generator on device; see DESIGN.md)"
    ew = enwik8_path() if kind == "text" else None
    if ew:  # configs[4]: the real enwik8, tiled to the shard (each rank at its global offset)
        raw = np.fromfile(ew, dtype=np.uint8)
        start = (s.rank * n) % raw.size
        reps = (start + n + raw.size - 1) // raw.size
        host = np.tile(raw, reps)[start:start + n]
        x[:n].copy_(torch.from_numpy(host))
        src = f"enwik8 from $ENWIK8 ({raw.size} B) tiled to {n} B per rank"
    else:
        D.generate(s.ctx, kind, SEEDS[kind], x.data_ptr(), n, offset=s.rank * n,
                   cdf=D.zipf_cdf(1.2) if kind == "zipf" else None)
    return x, src


def run_workload(s: Setup, kind: str, n: int, with_cpu: bool, strong: bool = False):
    """one bench record: `strong` times each step alone after an Infinity
    Cache flush (SURVEY §8d's strong-scaling curve), else back to back"""
    args, world, rank = s.args, s.world, s.rank
    flush = s.flush_buffer() if strong else None
    ctx = s.ctx
    x, data_src = make_input(s, kind, n)
    job = H.EncodeJob(ctx, x.data_ptr(), n)
    dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    state = {"out": torch.empty(n + 128, dtype=torch.uint8, device="cuda"), "cap": n + 128}

    def encode():
        """N=1: compress() in one native call (pass 1, tree, pass 2);
        N>1: huff_mgpu_compress (pass 1, RCCL all-gather, tree, bit base, pass 2)"""
        if world == 1:
            return job.compress(state["out"].data_ptr(), state["cap"])
        if s.comm is not None:
            tree, _, bits, _ = s.comm.compress(job, state["out"].data_ptr(), state["cap"])
            return tree, bits
        if s.dx is not None:
            hists, tails = s.dx(job)
        else:
            hists, tails = mgpu.exchange(job.hist(), x[n - 8:n], device=s.dev)
        tree, _, bits = job.pack_shards(hists, rank, tails, state["out"].data_ptr(), state["cap"])
        return tree, bits

    def encode_grow():
        try:
            return encode()
        except H.HuffError as e:  # compressed shard larger than the buffer: grow once, redo
            if getattr(e, "bits_needed", None) is None:
                raise
            state["cap"] = (e.bit_base % 8 + e.bits_needed + 7) // 8 + 128
            state["out"] = torch.empty(state["cap"], dtype=torch.uint8, device="cuda")
            return encode()

    # Weak steps are software-pipelined: at N=1 the next step's pass 1 is queued
    # between this step's pack and its decode (huff_enc_hist_launch), so the
    # host tree build overlaps the decode instead of idling the GPU (~27 us a
    # step, profiles/r06/pipeline). Every step still runs pass 1, tree, pass 2
    # and decode over the whole batch.
    # N>1 over the library's communicator the same: the next step's exchange
    # (pass 1, row, all-gather, rows to the host) is queued ahead of the decode
    # (huff_mgpu_exchange_launch), every rank at the same point.
    pipe = (world == 1 or s.comm is not None) and flush is None and not args.no_pipeline

    def step(more=False):
        tree, bits = encode_grow()
        if pipe and more:
            if world == 1:
                job.hist_launch()
            else:
                s.comm.exchange_launch(job)
        job.decode(tree, state["out"].data_ptr(), dec.data_ptr())
        return bits, tree

    for i in range(args.warmup):
        step(i + 1 < args.warmup)
    torch.cuda.synchronize()
    if not args.no_verify:
        assert torch.equal(dec[:n], x[:n]), "decode(encode(x)) != x"

    # timed region: K steps (weak: back to back; strong: each step alone,
    # after a 512 MiB rewrite that evicts the Infinity Cache). The library's
    # HIP-event kernel timing runs on every --time-every'th step of it (each
    # event-carrying dispatch leaves ~5 us of idle behind it: profiles/r06/timing)
    every = max(1, args.time_every)
    ctx.reset_timing()
    bits, tree = 0, None
    if flush is None:
        s.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            ctx.set_timing(i % every == 0)
            bits, tree = step(i + 1 < args.steps)
        torch.cuda.synchronize()
        s.barrier()
        elapsed = time.perf_counter() - t0
    else:
        elapsed = 0.0
        for i in range(args.steps):
            flush.fill_(i & 0xFF)  # torch's stream: outside the library's kernel timing
            s.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.set_timing(i % every == 0)
            bits, tree = step()
            torch.cuda.synchronize()
            s.barrier()
            elapsed += time.perf_counter() - t0
    elapsed = s.max_over_ranks(elapsed)
    kstats = {k: ctx.kernel_time(k) for k in ("hist", "chunk_bits", "scan", "pack", "decode")}
    ctx.set_timing(False)

    # end-to-end encode and decode apart (same K, same buffers)
    s.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tree, bits = encode_grow()
    torch.cuda.synchronize()
    t_enc = s.max_over_ranks(time.perf_counter() - t0)
    s.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        job.decode(tree, state["out"].data_ptr(), dec.data_ptr())
    torch.cuda.synchronize()
    t_dec = s.max_over_ranks(time.perf_counter() - t0)

    # index-free decode (huff_dev_decompress, comp.rs:487-519): the same
    # stream as the reference holds it, without the restart index
    comp_bytes = (bits + 7) // 8
    pad = (8 - bits % 8) % 8
    got = D.decompress_dev(ctx, tree, state["out"].data_ptr(), comp_bytes, pad, dec.data_ptr(), n + 64)
    torch.cuda.synchronize()
    assert got == n and (args.no_verify or torch.equal(dec[:n], x[:n])), "index-free decode != x"
    s.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        D.decompress_dev(ctx, tree, state["out"].data_ptr(), comp_bytes, pad, dec.data_ptr(), n + 64)
    torch.cuda.synchronize()
    t_idx = s.max_over_ranks(time.perf_counter() - t0)

    _, ln = tree.code_table()  # letters present in the input are exactly those with a code
    present = np.asarray(ln) > 0
    fixed8 = bool((ln[present] == 8).all()) and os.environ.get("HUFF_DISABLE_FIXED8", "0") in ("", "0")
    maxlen = int(ln[present].max())  # the decode kernel the runtime picks (runtime.cpp, huff_enc::decode)
    dec_kernel = "k_decode" if maxlen > 32 else "k_decode_fixed"
    ms_per_step = elapsed * 1e3 / args.steps
    value = world * n / (elapsed / args.steps) / 1e9
    nchunks = (n + 65535) // 65536
    algo = {  # algorithmic bytes per launch
        "hist": n,
        "chunk_bits": nchunks * (1024 + 8),
        "scan": nchunks * 16,
        "pack": n + comp_bytes,
        "decode": comp_bytes + n,
    }
    kernels = {}
    for k, b in algo.items():
        ms, cnt = kstats[k]
        if cnt:
            avg = ms / cnt
            kernels[k] = {"avg_ms": round(avg, 5), "launches": cnt, "algo_bytes": b,
                          "GBps": round(b / (avg * 1e-3) / 1e9, 1)}
    dom = max(kernels, key=lambda k: kernels[k]["avg_ms"])
    ach = kernels[dom]["GBps"]
    # the committed PMC summaries are per launch of a 1 GiB job: other sizes get none
    traffic, traffic_src = (dominant_traffic(kind, dom, fixed8, dec_kernel) if n == 1 << 30 else (None, None))
    enc_ms = sum(kernels[k]["avg_ms"] for k in ("hist", "chunk_bits", "scan", "pack") if k in kernels)
    if s.ceil is None:  # measured HBM ceilings of this GPU, same run (huff_dev_calibrate)
        s.ceil = D.calibrate(ctx, x.data_ptr(), dec.data_ptr(), n & ~15, 5)
    read_ceil, copy_ceil = s.ceil
    # the index-free decode against the roofline: C + N algorithmic bytes over
    # its wall time per call (the host read of the letter count included), and
    # the pipeline's PMC bytes when a summary exists for this workload at 1 GiB
    idx_ach = (comp_bytes + n) / (t_idx / args.steps) / 1e9
    idx_traffic, idx_src = indexfree_traffic(kind, fixed8) if n == 1 << 30 else (None, None)
    indexfree_roofline = {"algo_bytes": comp_bytes + n, "achieved": round(idx_ach, 1), "unit": "GB/s",
                          "frac": round(idx_ach / HBM_PEAK_GBPS, 4), "traffic": idx_traffic,
                          "traffic_x_algo": round(idx_traffic / (comp_bytes + n), 3) if idx_traffic else None,
                          "traffic_source": idx_src}
    collective = None
    if world > 1:
        how = ("huff_mgpu_compress (library RCCL communicator)" if s.comm is not None
               else "torch.distributed " + ("RCCL" if s.nccl else "gloo (rehearsal)"))
        collective = f"all_gather int64[258] (weights + tail bytes) per rank via {how}"
    r = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": data_src,
        "config": {"workload": f"{human(n * world)} {kind} bytes"
                               + (f" ({human(n)} per GPU)" if world > 1 else "")
                               + f" ({CONFIG_OF[kind]}), encode+decode, bit-exact",
                   "bytes_per_gpu": n, "global_bytes": n * world,
                   "compressed_bytes_per_gpu": comp_bytes, "bits_per_byte": round(bits / n, 4),
                   "kernel_path": "fixed8 byte map (all codes 8 bits)" if fixed8 else "general bit pack/decode",
                   "parallelism": f"shard{world}", "collective": collective,
                   "rccl_world": s.rccl_world},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": traffic, "traffic_source": traffic_src,
                     "ceilings_measured": {"read_GBps": round(read_ceil, 1), "copy_GBps": round(copy_ceil, 1),
                                           "how": "huff_dev_calibrate: 16-B nontemporal stream, best of 5"},
                     "frac_of_copy_ceiling": round(ach / copy_ceil, 4)},
        "kernels": kernels,
        "kernel_timing_every": every,  # kernels[*].launches: the sampled steps
        "pipelined": pipe,
        "e2e": {"encode_GBps": round(world * n / (t_enc / args.steps) / 1e9, 1),
                "decode_GBps": round(world * n / (t_dec / args.steps) / 1e9, 1),
                "encode_ms": round(t_enc * 1e3 / args.steps, 4), "decode_ms": round(t_dec * 1e3 / args.steps, 4),
                "indexfree_decode_GBps": round(world * n / (t_idx / args.steps) / 1e9, 1),
                "indexfree_decode_ms": round(t_idx * 1e3 / args.steps, 4),
                "indexfree_roofline": indexfree_roofline,
                "note": "encode = pass 1 + host tree + pass 2 (+ the collective at N>1); decode = restart-index "
                        "decode; indexfree = huff_dev_decompress of the bare stream (spec/fix/scan/mark/decode, "
                        "one host read of the symbol count)"},
        "kernel_enc_GBps": round(n / (enc_ms * 1e-3) / 1e9, 1),
        "host_gap_ms": round(ms_per_step - sum(k["avg_ms"] for k in kernels.values()), 4),
        "kernel_dec_GBps": kernels.get("decode", {}).get("GBps"),
    }
    if s.comm_note:
        r["config"]["collective_note"] = s.comm_note
    if with_cpu:
        r["cpu_baseline"] = cpu_baseline(kind, args.cpu_seconds)
    del x, dec, state, job
    torch.cuda.empty_cache()
    return r


def file_path_bench(s: Setup, kind: str, n: int, steps: int):
    """the .hff file path (huff_file_compress /
    huff_file_decompress = read_compress_write / read_decompress_write,
    huff/src/comp.rs:32-280) on an n-byte file in the page cache: wall time
    of each call, file reads, PCIe copies and file writes included. The CLI's
    default -b 2G (one block) round-trips; -b 256Mi exercises the pipelined
    multi-block compress, whose output is the reference's bug-compatible
    stitching (decodable only when every block's padding is 0 or 4, SURVEY
    App. C.3), so its round trip is reported, not asserted."""
    import shutil
    import tempfile

    x, _ = make_input(s, kind, n)
    host = x[:n].cpu().numpy()
    del x
    torch.cuda.empty_cache()
    d = tempfile.mkdtemp(prefix="huffbench")
    try:
        p = os.path.join(d, "in")
        host.tofile(p)
        res = {"file_bytes": n, "workload": f"{human(n)} {kind} file", "steps": steps,
               "how": "wall time of one library call, file in the page cache, best of the timed steps"}
        # the host's own page-cache rates on the same file (numpy, one thread)
        t0 = time.perf_counter()
        np.fromfile(p, np.uint8)
        t1 = time.perf_counter()
        host.tofile(p + ".copy")
        t2 = time.perf_counter()
        os.remove(p + ".copy")
        res["host_io"] = {"read_GBps": round(n / (t1 - t0) / 1e9, 3), "write_GBps": round(n / (t2 - t1) / 1e9, 3),
                          "how": "np.fromfile / ndarray.tofile of the same 1 GiB, one thread"}
        for bs, name in ((2_000_000_000, "b2G"), (256 << 20, "b256Mi")):
            tc, td = [], []
            for i in range(steps + 1):
                for f in (p + ".hff", p + ".out"):  # new files, as the CLI writes (not a truncation)
                    if os.path.exists(f):
                        os.remove(f)
                t0 = time.perf_counter()
                H.read_compress_write(p, p + ".hff", bs, s.ctx)
                t1 = time.perf_counter()
                try:
                    H.read_decompress_write(p + ".hff", p + ".out", bs, s.ctx)
                except H.HuffError as e:  # the stitched multi-block stream may not decode (as in the reference)
                    if name == "b2G":
                        raise
                    res[name + "_decompress_error"] = str(e)
                t2 = time.perf_counter()
                if i:
                    tc.append(t1 - t0)
                    td.append(t2 - t1)
            same = os.path.getsize(p + ".out") == n and np.array_equal(np.fromfile(p + ".out", np.uint8), host)
            if name == "b2G":
                assert same, "file round trip != input"
            res[name] = {"compress_GBps": round(n / min(tc) / 1e9, 3), "decompress_GBps": round(n / min(td) / 1e9, 3),
                         "compress_ms": round(min(tc) * 1e3, 2), "decompress_ms": round(min(td) * 1e3, 2),
                         "hff_bytes": os.path.getsize(p + ".hff"), "roundtrip_equal": bool(same)}
            if name != "b2G":
                res[name]["note"] = ("several blocks: the reference CLI's stitched stream does not round-trip "
                                     "(DESIGN.md §6, bug-compatible; tests/test_gpu_parity.py file-path windows "
                                     "pin the bytes against the oracle)")
        return res
    finally:
        shutil.rmtree(d, ignore_errors=True)


def free_port() -> int:
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def rank_guard(args, argv=None, environ=None, spawn=None):
    """--gpus N means N ranks. Without a launcher (no WORLD_SIZE) and N > 1,
    start N rank processes as children (torch.distributed.run on 127.0.0.1)
    and return the exit code to exit with; a launcher whose world differs
    from --gpus is an error (a wasted lease otherwise). Returns None when
    this process is one of the N ranks. Runs before anything touches the GPU
    (no device query, no exec: the ranks are children)."""
    import subprocess
    environ = os.environ if environ is None else environ
    argv = sys.argv[1:] if argv is None else argv
    ws = environ.get("WORLD_SIZE")
    if ws is None:
        if args.gpus <= 1:
            return None
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
        print(f"bench.py: --gpus {args.gpus} without a launcher: starting {args.gpus} ranks", file=sys.stderr,
              flush=True)
        return (spawn or subprocess.call)(cmd)
    if int(ws) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={ws} ranks; refusing to "
              f"report a {ws}-rank line as {args.gpus}", file=sys.stderr, flush=True)
        return 2
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="uniform", choices=sorted(SEEDS))
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="the main line's mode; the other mode is reported under 'scaling_other'")
    ap.add_argument("--bytes-per-gpu", type=int, default=1 << 30, help="weak scaling: bytes per rank")
    ap.add_argument("--total-bytes", type=int, default=1 << 30, help="strong scaling: bytes over all ranks")
    ap.add_argument("--side", default="zipf", choices=["zipf", "text", "none"],
                    help="N=1: a second workload reported under 'side' (configs[2] by default)")
    ap.add_argument("--no-general", action="store_true",
                    help="N=1: skip the 'general' record (the headline workload through the general "
                         "scan + bit-pack kernels, HUFF_DISABLE_FIXED8=1)")
    ap.add_argument("--no-other-scaling", action="store_true", help="skip the 'scaling_other' record")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--file-path", default="zipf", choices=["zipf", "text", "uniform", "none"],
                    help="N=1: time the .hff file path on a 1 GiB file of this workload")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="N=1: run each step's pass 1 after the previous decode (no overlap of the tree build)")
    ap.add_argument("--time-every", type=int, default=4,
                    help="kernel durations (HIP events) sampled on every Nth timed step")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N>1 path with several ranks on one GPU")
    args = ap.parse_args()
    rc = rank_guard(args)
    if rc is not None:
        sys.exit(rc)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    ndev = torch.cuda.device_count()
    if world > 1 and args.dist_backend == "nccl" and ndev < world:
        print(f"bench.py: {world} RCCL ranks need {world} GPUs, this node shows {ndev}", file=sys.stderr, flush=True)
        sys.exit(2)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, ndev)
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    s = Setup(args, world, rank, local)
    n_weak = args.bytes_per_gpu
    n_strong = (args.total_bytes // world) & ~0xFFFF
    strong = args.scaling == "strong"
    with_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline
    result = run_workload(s, args.workload, n_strong if strong else n_weak, with_cpu, strong)
    if not args.no_other_scaling:
        # the 1/2/4/8 curve of the metric is strong scaling of 1 GiB
        # (1 GiB / N per rank, caches flushed); the weak line (1 GiB per rank)
        # beside it, whichever is the main line
        o = run_workload(s, args.workload, n_weak if strong else n_strong, False, not strong)
        result["scaling_other"] = {k: o[k] for k in ("scaling", "value", "unit", "ms_per_step", "n_gpus", "steps",
                                                     "kernels", "roofline", "e2e")}
        result["scaling_other"]["bytes_per_gpu"] = o["config"]["bytes_per_gpu"]
        result["scaling_other"]["global_bytes"] = o["config"]["global_bytes"]
    if world == 1 and not args.no_general:
        # the north-star kernels (per-byte lookup + exclusive scan + bit-pack
        # and the bit decoder) on the headline workload: the byte map off
        prev = os.environ.get("HUFF_DISABLE_FIXED8")
        os.environ["HUFF_DISABLE_FIXED8"] = "1"
        try:
            g = run_workload(s, args.workload, n_strong if strong else n_weak, False, strong)
        finally:
            if prev is None:
                del os.environ["HUFF_DISABLE_FIXED8"]
            else:
                os.environ["HUFF_DISABLE_FIXED8"] = prev
        result["general"] = {k: g[k] for k in ("value", "unit", "ms_per_step", "kernels", "roofline", "e2e",
                                               "host_gap_ms")}
        result["general"]["kernel_path"] = g["config"]["kernel_path"]
        result["general"]["note"] = "the headline workload with HUFF_DISABLE_FIXED8=1 (general kernels)"
    if world == 1 and args.side != "none" and args.side != args.workload:
        result["side"] = {args.side: run_workload(s, args.side, n_weak, with_cpu)}
    if world == 1 and args.file_path != "none":
        result["file_path"] = file_path_bench(s, args.file_path, n_weak, 2)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if s.comm is not None:
        s.comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
