#!/usr/bin/env python3
"""bench.py -- Namazu decision engine on MI355X.

Headline workload (BASELINE.json configs[1]): replayable-policy seed sweep,
2^20 seeds x 4096-event ZooKeeper-style packet trace, maxInterval 100 ms, on
each GPU (weak scaling: every rank sweeps 2^20 seeds per step). Step i sweeps a
fresh range of decimal seeds, (i * N + rank) * 2^20 .., so no seed is swept
twice; steps are pipelined over 3 plans / HIP streams so one step's
latency-bound kernels overlap the neighbouring steps. One step =
  seed prefix hashing (seed strings generated on the device) + bucketing +
  the K1 sweep (stats for every seed) + that batch's top-64;
after the last step, inside the timing: the device merge of the steps' top-64
lists (+ RCCL all_gather and the host merge when N > 1).
Inputs are resident in HBM before the timed region; the per-trace plan
(correction tables) is built once, outside it. Defaults are the driver's
settings (--steps 20 --warmup 5).

Metric: schedule decisions/s (seeds x events / s), whole job.
Also reported (same JSON line): the roofline of the dominant kernel
(k_replayable_sweep_oq, HIP events on its launch stream), a CPU baseline
(the oracle's C restatement on the host cores, bounded sample) and
secondary lines for the random-policy sweep (configs[3]) and the banded
edit-distance all-pairs search (configs[2]), each on a per-GPU share.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU, RCCL).
"""
import argparse
import ctypes
import gc
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PEAK_CLOCK_GHZ = 2.4  # MI355X peak engine clock
PEAK_VALU_TOPS = 256 * 4 * 32 * PEAK_CLOCK_GHZ * 1e9 / 1e12  # 78.6 T int32 lane-ops/s (2 cyc/wave64 instr/SIMD)
PEAK_HBM_GBS = 8000.0
MAX_INTERVAL_NS = 100_000_000
# VALU lane-instructions per unit (decision / trace pair) of each dominant kernel, measured by rocprofv3
# (SQ_INSTS_VALU x 64 / units per launch) on this bench's own workloads: profiles/valu_per_unit.json,
# written by tools/valu_per_unit.py from the latest profile summary. The ED kernels' counts depend on
# the cut-off and so hold for these synthetic workloads only. HBM traffic = 2 x FETCH_SIZE + WRITE_SIZE
# (MI355X_MICROARCH.md: gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads).
VALU_TABLE = os.path.join(HERE, "profiles", "valu_per_unit.json")


# the K1 kernel a replayable plan runs (nmz_replayable_plan_kernel): wavelet-tree statistics by default,
# order-query statistics with NMZ_REPLAY_WT=0 (or when the trees do not fit), the per-decision sweep with
# NMZ_REPLAY_OQ=0 on top
K1_KERNELS = {2: "k_replayable_sweep_wt", 1: "k_replayable_sweep_oq", 0: "k_replayable_sweep_fast"}
K1_ALGORITHM = {
    "k_replayable_sweep_wt": "wavelet-tree statistics: per (seed, hint-length class) three bucket-indexed searches "
                             "and two wavelet-tree descents over the rank permutation of the C-sorted segment "
                             "(DESIGN.md section 4); units = seed x event decisions covered",
    "k_replayable_sweep_oq": "order-query statistics: per (seed, hint-length class) binary searches over "
                             "C-mod-m-sorted blocks (DESIGN.md section 4); units = seed x event decisions covered",
}


def k1_kernel(L, plan):
    if os.environ.get("NMZ_REPLAY_OQ") == "0":
        return "k_replayable_sweep_fast"
    return K1_KERNELS[L.nmz_replayable_plan_kernel(plan)]


def valu_entry(kernel):
    try:
        return json.load(open(VALU_TABLE))[kernel]
    except (OSError, KeyError, ValueError):
        return None


_FPS = None


def isa_state(e):
    """Whether the kernels a valu_per_unit.json entry profiled are the kernels the shipped library runs:
    (fresh, {kernel: [profiled fingerprint, current fingerprint]}) from tools/kernel_isa.py."""
    global _FPS
    sys.path.insert(0, os.path.join(HERE, "tools"))
    import kernel_isa
    if _FPS is None:
        _FPS = kernel_isa.kernel_fingerprints(os.path.join(HERE, "namazu_amd", "libnmz_gpu.so"))
    prof = e.get("isa") or {}
    detail = {k: [v, kernel_isa.lookup(_FPS, k)] for k, v in prof.items()}
    fresh = bool(detail) and all(a is not None and a == b for a, b in detail.values())
    return fresh, detail


def issue_ceiling(kernel, isa, lane_instr, kernel_ms):
    """This launch's VALU issue time at the measured issue cost of the kernel's instruction forms
    (tools/issue_ceiling.py -> profiles/issue_ceiling.json: mean cycles per wave-instruction of the hot loop)
    over the measured kernel time, at the clock the chip held in the kernel's profile; None when the entry is
    missing or priced other machine code."""
    try:
        e = json.load(open(os.path.join(HERE, "profiles", "issue_ceiling.json")))["kernels"][kernel]
    except (OSError, KeyError, ValueError):
        return None
    if not e.get("isa") or any(isa.get(k, [None, None])[1] != h for k, h in e["isa"].items()):
        return None
    cyc = lane_instr / 64.0 * e["hot_loop"]["mean_cost"] / 1024.0
    return cyc / (e["clock_ghz"] * 1e9) / (kernel_ms * 1e-3)


def roofline_valu(kernel, units, kernel_ms):
    """VALU issue roofline of `kernel`: measured lane-instructions per unit x units / kernel time. The entry's
    lane-instructions per unit hold only for the machine code that was profiled: when the shipped kernel's
    fingerprint differs (or the entry has none) the roofline is marked stale and carries no frac."""
    e = valu_entry(kernel)
    if e is None:
        return {"bound": "valu", "kernel": kernel, "kernel_ms": kernel_ms, "stale": True, "achieved": None,
                "frac": None, "peak": PEAK_VALU_TOPS, "unit": "Tops/s", "traffic": None,
                "why": "no profiles/valu_per_unit.json entry for this kernel yet"}
    fresh, isa = isa_state(e)
    achieved = e["ops_per_unit"] * units / (kernel_ms * 1e-3) / 1e12
    traffic = e.get("hbm_bytes_per_launch")
    if traffic is not None and units != e["units_per_launch"]:
        traffic = traffic * units / e["units_per_launch"]
    if not fresh:
        return {"bound": "valu", "kernel": kernel, "kernel_ms": kernel_ms, "stale": True, "achieved": None,
                "frac": None, "peak": PEAK_VALU_TOPS, "unit": "Tops/s", "traffic": None,
                "frac_if_profile_held": achieved / PEAK_VALU_TOPS, "ops_source": e["source"], "isa": isa,
                "why": "the profiled kernel's machine code differs from the shipped library's (tools/kernel_isa.py)"}
    ceil = issue_ceiling(kernel, isa, e["ops_per_unit"] * units, kernel_ms)
    return {"bound": "valu", "achieved": achieved, "peak": PEAK_VALU_TOPS, "unit": "Tops/s", "stale": False,
            "frac_of_issue_ceiling": ceil,
            "frac": achieved / PEAK_VALU_TOPS, "traffic": traffic, "isa": isa, "traffic_unit": "bytes/launch (2 x FETCH_SIZE + WRITE_SIZE)",
            "kernel": kernel, "kernel_ms": kernel_ms, "ops_per_unit": e["ops_per_unit"], "units_per_launch": units,
            "ops_source": e["source"],
            # the same lane-ops against the issue ceiling at the engine clock the chip held during this
            # kernel's profile (GRBM_GUI_ACTIVE / duration), not the 2.4 GHz peak clock
            "clock_ghz": e.get("clock_ghz"),
            "frac_at_clock": (achieved / (PEAK_VALU_TOPS * e["clock_ghz"] / PEAK_CLOCK_GHZ)
                              if e.get("clock_ghz") else None)}


# The driver parses the LAST stdout line and keeps only the tail of stdout: the final line is a compact headline
# (configs[1]: value, roofline, cpu_baseline, a short per-leg summary) capped at HEADLINE_MAX_BYTES; every
# secondary leg goes out as its own earlier line ({"secondary_leg": ...}) and the full record to a file.
HEADLINE_MAX_BYTES = 4096
NMZ_TIMING_SPANS = 2  # nmz_timing_enable mode: in-kernel spans only (include/nmz_gpu.h)
HEADLINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                 "vs_baseline", "dtype", "data", "config")
ROOFLINE_KEYS = ("bound", "kernel", "achieved", "peak", "unit", "frac", "declared_model_frac",
                 "declared_model_ops_per_unit", "traffic", "kernel_ms", "kernel_ms_source",
                 "ops_per_unit", "units_per_launch", "unit_kind", "frac_of_issue_ceiling", "frac_at_clock",
                 "clock_ghz", "kernel_ms_span", "kernel_ms_serial_span", "kernel_ms_events", "stale", "ops_source")
CPU_KEYS = ("value", "unit", "cores", "kind", "sample", "parity_with_gpu", "seconds")


def _round(v):
    if isinstance(v, float):
        return float(f"{v:.5g}")
    if isinstance(v, dict):
        return {k: _round(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_round(x) for x in v]
    return v


def leg_summary(leg):
    """One secondary leg as {leg, value, unit, ms_per_step, kernel, frac} for the headline's secondary_summary."""
    cfg = leg.get("config") or {}
    rf = leg.get("roofline") or {}
    out = {"leg": leg.get("leg") or cfg.get("workload", leg.get("metric", "?"))[:40], "value": leg.get("value"),
           "unit": leg.get("unit")}
    for k in ("ms_per_step", "kernel_ms"):
        if leg.get(k) is not None:
            out[k] = leg[k]
    if rf:
        out["kernel"] = rf.get("kernel")
        out["frac"] = rf.get("frac")
    if "lines" in leg:  # the K1 cliffs leg: one figure per line
        out["value"] = [x.get("value") for x in leg["lines"]]
    if "gpu_batch" in leg:  # configs[0]
        out["value"], out["ms"] = leg["gpu_batch"]["value"], leg["gpu_batch"]["ms"]
    return _round(out)


def headline_record(line):
    """The compact final stdout line: the headline fields, a trimmed roofline and cpu_baseline, the end-to-end
    figures and a per-leg summary of the secondary legs, below HEADLINE_MAX_BYTES (optional parts are dropped,
    last first, if it would not fit)."""
    rec = {k: line[k] for k in HEADLINE_KEYS if k in line}
    if line.get("roofline"):
        rec["roofline"] = {k: line["roofline"][k] for k in ROOFLINE_KEYS if k in line["roofline"]}
    if line.get("cpu_baseline"):
        rec["cpu_baseline"] = {k: line["cpu_baseline"][k] for k in CPU_KEYS if k in line["cpu_baseline"]}
    e2e = line.get("end_to_end")
    if e2e:
        rec["end_to_end"] = {k: e2e[k] for k in ("value", "mode", "ms_per_trace", "traces", "plan_ms",
                                                 "agrees_with_one_at_a_time") if k in e2e}
        nb = e2e.get("native_batch")
        if nb:
            rec["end_to_end"]["native_batch"] = {k: nb[k] for k in ("value", "ms_per_trace",
                                                                    "agrees_with_one_at_a_time") if k in nb}
    optional = []
    if line.get("secondary"):
        rec["secondary_summary"] = [leg_summary(s) for s in line["secondary"]]
        optional.append("secondary_summary")
    if line.get("full_record"):
        rec["full_record"] = line["full_record"]
    rec = _round(rec)
    optional += ["end_to_end", "data"]
    text = json.dumps(rec, separators=(",", ":"))
    while len(text) >= HEADLINE_MAX_BYTES and optional:
        rec.pop(optional.pop(0), None)
        text = json.dumps(rec, separators=(",", ":"))
    return text


def cpu_threads():
    """Host threads for the CPU baselines: the cores this process may run on (on the GPU box the CPU share
    set by OMP_NUM_THREADS, since nproc there counts the whole machine)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def zk_hints(n_events, seed=0x5EED):
    """ZooKeeper-style replay hints: decimal signed int64 (pynmz zookeeper.py:113 format)."""
    from namazu_amd.synth import splitmix64 as sm
    return [str(int(x)) for x in sm(seed, n_events).view(np.int64)]


def decimal_csr(lo, n):
    from namazu_amd.explorepolicy import to_csr
    return to_csr([str(i) for i in range(lo, lo + n)])


def host_ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if "NMZ_BENCH_DEVICE" in os.environ:
            self.local_rank = int(os.environ["NMZ_BENCH_DEVICE"])
        self.pg = None

    def init(self, torch):
        if self.world > 1:
            import torch.distributed as dist
            # NMZ_BENCH_BACKEND=gloo + NMZ_BENCH_DEVICE=0 rehearse the N > 1 path with several ranks on one
            # GPU (RCCL refuses two ranks per device); the driver's runs use the defaults (RCCL, rank i on GPU i)
            backend = os.environ.get("NMZ_BENCH_BACKEND", "nccl")
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local_rank))
            else:
                dist.init_process_group(backend)
            self.pg = dist

    def barrier(self):
        if self.pg:
            self.pg.barrier()

    def max(self, torch, v):
        if not self.pg:
            return v
        t = torch.tensor([v], dtype=torch.float64, device="cuda")
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())


_HIP = []


def _hip():
    """The HIP runtime torch loaded (hipMemcpyAsync for the bench's own copies on the library's streams)."""
    if not _HIP:
        h = ctypes.CDLL("libamdhip64.so")
        h.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                     ctypes.c_void_p]
        h.hipMemcpyAsync.restype = ctypes.c_int
        _HIP.append(h)
    return _HIP[0]


def hip_check(rc):
    if rc != 0:
        raise RuntimeError(f"HIP error {rc}")


def merge_topk(entries, k):
    from namazu_amd.dist import merge_topk as _merge
    return _merge([entries], k)


def bench_replayable(args, torch, D, ctx, L, stream):
    from namazu_amd import _lib
    from namazu_amd.explorepolicy import to_csr
    S, E = args.seeds, args.events
    hints = zk_hints(E)
    hoff, hb = to_csr(hints)
    # The job: K = args.steps batches of S fresh seeds per rank. Timed step i sweeps the decimal seeds
    # (i * world + rank) * S .. + S - 1 (generated on the device: nmz_replayable_sweep_decimal_topk_dev, no seed
    # CSR), so no step re-sweeps another's seeds; its top-64 goes to slot i of a [K][64] list buffer. After the last
    # step one device merge (nmz_topk_merge_dev) gives the rank's top-64 of the whole job, (N > 1) one RCCL
    # all_gather brings every rank's list, and the host merges them: all inside the timed region.
    # Consecutive steps are pipelined over NP plans and HIP streams (NMZ_BENCH_PIPELINE, default 3): the
    # latency-bound kernels around one step's sweep (seed prefix, bucketing, top-k) and the tail of its persistent
    # sweep grid overlap the neighbouring steps. Every step does all of its work on its own batch.
    # Each pipeline slot is its own context (nmz_open) and runs on that context's stream (nmz_ctx_stream): streams
    # that share one of the process's hardware queues (GPU_MAX_HW_QUEUES, 4) dispatch in order, so a sweep waiting
    # for the CUs another slot's sweep holds would stall the kernels queued behind it on the other slot -- measured
    # 83 us per step with torch pool streams vs 59 with the contexts' own streams (tools/step_ab.py, 200 steps)
    NP = max(1, int(os.environ.get("NMZ_BENCH_PIPELINE", "3")))
    K_TOP = 64
    csr0 = decimal_csr(D.rank * S, S)  # timed step 0's seeds: the CPU baseline's sample and the end-to-end seeds
    ctxs = [ctx] + [_lib.Context(D.local_rank) for _ in range(NP - 1)]
    plans = []
    t0 = time.time()
    for sp in range(NP):
        plan = ctypes.c_void_p()
        _lib.check(L.nmz_replayable_plan_create(ctxs[sp].handle, host_ptr(hoff), host_ptr(hb), E, MAX_INTERVAL_NS, S,
                                                ctypes.byref(plan)))
        plans.append(plan)
    plan_ms = (time.time() - t0) * 1e3 / NP
    k1 = k1_kernel(L, plans[0])
    dev = torch.device("cuda", D.local_rank)
    streams = [torch.cuda.ExternalStream(c.stream(), device=dev) for c in ctxs]
    d_stats = [torch.empty(S * 32, dtype=torch.uint8, device=dev) for _ in range(NP)]
    n_lists = max(args.steps, 1)
    d_lists = torch.empty(n_lists * K_TOP * 24, dtype=torch.uint8, device=dev)
    d_scratch = torch.empty_like(d_lists)
    d_job = torch.empty(K_TOP * 24, dtype=torch.uint8, device=dev)
    # N > 1: every rank's job list lands in one [N][64] buffer (views of it as all_gather's outputs) and the device
    # merges them (nmz_topk_merge_dev), so the host only copies the final 64 entries (pinned, asynchronous)
    d_gath = torch.empty(max(D.world, 1) * K_TOP * 24, dtype=torch.uint8, device=dev)
    gathered = list(d_gath.view(D.world, K_TOP * 24).unbind(0)) if D.world > 1 else None
    d_final = torch.empty_like(d_job)
    h_final = torch.empty(K_TOP * 24, dtype=torch.uint8).pin_memory()
    h_view = h_final.numpy()  # (a view made before the timing: reading the answer is a numpy copy)
    done_ev = torch.cuda.Event(enable_timing=True)
    start_ev = torch.cuda.Event(enable_timing=True)  # the GPU's own span of the timed region (vs the host clock)
    # the host merge of the job (one list per rank) is the check outside the timing; NMZ_BENCH_HOST_MERGE=1 times
    # it instead of the device merge (A/B)
    host_merge = os.environ.get("NMZ_BENCH_HOST_MERGE") == "1"
    # how the last step's stream learns that the other slots are done before the job merge: "event" (stream waits:
    # barrier packets on the last stream's queue) or "host" (the host waits for those streams, which end first, then
    # enqueues the merge: measured slower, 0.075-0.077 vs 0.070-0.071 ms per step -- the host's wake-up costs more)
    host_join = os.environ.get("NMZ_BENCH_JOIN", "event") == "host"
    spin = os.environ.get("NMZ_BENCH_SPIN", "1") == "1"
    # the timed K1 launches record their own execution spans (in-kernel wall clock, no HIP event records between
    # a stream's launches: each record is a marker the queue stalls on, ~6 us at the step's ends);
    # NMZ_BENCH_TIMED_EVENTS=1 brackets them with HIP events as well (A/B of their cost)
    timed_events = os.environ.get("NMZ_BENCH_TIMED_EVENTS", "0") == "1"
    # seed ranges outside the job's for the untimed launches (warm-up, kernel timing)
    spare_lo = (args.steps + 1) * D.world * S + D.rank * S

    torch.cuda.synchronize()  # the buffers above (allocated on torch's stream) before the contexts' streams use them

    def sweep(sp, lo, out_list):
        _lib.check(L.nmz_replayable_sweep_decimal_topk_dev(plans[sp], lo, S, K_TOP,
                                                           ctypes.c_void_p(d_stats[sp].data_ptr()),
                                                           ctypes.c_void_p(out_list),
                                                           ctypes.c_void_p(streams[sp].cuda_stream)))

    def step(i):
        sweep(i % NP, (i * D.world + D.rank) * S, d_lists.data_ptr() + (i % n_lists) * K_TOP * 24)

    def join(last=0):  # stream `last` waits for the other slots' work
        for sp in range(NP):
            if sp != last:
                streams[last].wait_stream(streams[sp])

    for j in range(max(args.warmup, NP)):
        sweep(j % NP, spare_lo, d_lists.data_ptr() + (j % n_lists) * K_TOP * 24)
    join()
    # the job merge's kernels and the host merge, once outside the timing (first launches load their code)
    _lib.check(L.nmz_topk_merge_dev(ctx.handle, ctypes.c_void_p(d_lists.data_ptr()), n_lists, K_TOP,
                                    ctypes.c_void_p(d_scratch.data_ptr()), ctypes.c_void_p(d_job.data_ptr()),
                                    ctypes.c_void_p(streams[0].cuda_stream)))
    merge_topk(d_job.cpu().numpy().tobytes(), K_TOP)
    torch.cuda.synchronize()
    # the roofline's kernel time: K1 launched back to back on ONE stream (no other stream's kernels beside it, the
    # way rocprofv3 --kernel-trace times a dispatch), HIP events around each K1 launch plus its in-kernel span;
    # enough launches that the engine clock has ramped (a handful after an idle sync run slow)
    tot, cnt = ctypes.c_double(), ctypes.c_uint64()
    for _ in range(20):
        sweep(0, spare_lo, d_job.data_ptr())
    _lib.check(L.nmz_timing_enable(ctx.handle, 1))
    L.nmz_timing_read(ctx.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1)
    L.nmz_timing_read_span(ctx.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1)
    for _ in range(50):
        sweep(0, spare_lo, d_job.data_ptr())
    torch.cuda.synchronize()
    _lib.check(L.nmz_timing_read(ctx.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1))
    kern_ms = tot.value / max(cnt.value, 1)
    _lib.check(L.nmz_timing_read_span(ctx.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1))
    kern_ms_serial_span = tot.value / cnt.value if cnt.value else None
    _lib.check(L.nmz_timing_enable(ctx.handle, 0))
    # the timed region: exactly args.steps pipelined steps + the job's merge; K1's launches record their spans
    # (timing is per context: every slot's context records its own launches)
    for c in ctxs:
        _lib.check(L.nmz_timing_enable(c.handle, 1 if timed_events else NMZ_TIMING_SPANS))
        L.nmz_timing_read(c.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1)
        L.nmz_timing_read_span(c.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1)
    # the job's merges run on the stream of the last step (in order behind its top-k; the other slots' streams
    # finished earlier, so waiting for them costs no cross-queue round trip at the end)
    last = (args.steps - 1) % NP if args.steps else 0
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    start_ev.record(streams[0])
    for i in range(args.steps):
        step(i)
    enq = time.perf_counter() - t0  # the host's enqueue time of the steps (host-bound pipeline when ~ el)
    marks = {}
    if host_join:
        # the other slots' last steps end while the last step's sweep still runs: the host waits for them and
        # then enqueues the merge behind the last step, in order on its stream (no cross-queue barrier packet)
        for sp in range(NP):
            if sp != last:
                streams[sp].synchronize()
    else:
        join(last)
    marks["joined"] = time.perf_counter() - t0
    with torch.cuda.stream(streams[last]):
        sl = ctypes.c_void_p(streams[last].cuda_stream)
        _lib.check(L.nmz_topk_merge_dev(ctx.handle, ctypes.c_void_p(d_lists.data_ptr()), args.steps, K_TOP,
                                        ctypes.c_void_p(d_scratch.data_ptr()), ctypes.c_void_p(d_job.data_ptr()),
                                        sl))
        if host_merge:
            if D.pg:
                D.pg.all_gather(gathered, d_job)
            parts = [g.cpu().numpy() for g in gathered] if D.pg else [d_job.cpu().numpy()]
            merged = merge_topk(b"".join(x.tobytes() for x in parts), K_TOP)
        else:
            fin = d_job
            if D.pg:
                D.pg.all_gather(gathered, d_job)
                _lib.check(L.nmz_topk_merge_dev(ctx.handle, ctypes.c_void_p(d_gath.data_ptr()), D.world, K_TOP,
                                                ctypes.c_void_p(d_scratch.data_ptr()),
                                                ctypes.c_void_p(d_final.data_ptr()), sl))
                fin = d_final
            # the 1.5 KB answer to pinned host memory on the last slot's stream (a plain hipMemcpyAsync: torch's
            # pinned allocator would record the library context's stream on the buffer)
            hip_check(_hip().hipMemcpyAsync(ctypes.c_void_p(h_final.data_ptr()), ctypes.c_void_p(fin.data_ptr()),
                                            ctypes.c_size_t(K_TOP * 24), 2, sl))
            done_ev.record()
    marks["copy_enqueued"] = time.perf_counter() - t0
    if not host_merge:
        if spin:  # the host polls for the answer
            while not done_ev.query():
                pass
        else:
            done_ev.synchronize()
        marks["answer_seen"] = time.perf_counter() - t0
        # the 1,536 bytes through ctypes (a copy of the pinned buffer through a numpy view measured 30-50 us here
        # against 12-21; NMZ_BENCH_READ=view, A/B)
        if os.environ.get("NMZ_BENCH_READ") == "view":
            merged = h_view.view(_lib.TOPK_DTYPE).copy()
        else:
            merged = np.frombuffer(ctypes.string_at(h_final.data_ptr(), K_TOP * 24), dtype=_lib.TOPK_DTYPE)
    marks["answer_read"] = time.perf_counter() - t0
    if os.environ.get("NMZ_BENCH_STREAM_SYNC") == "1":  # A/B: each slot's stream first
        for st_ in streams:
            st_.synchronize()
        marks["streams_synced"] = time.perf_counter() - t0
    torch.cuda.synchronize()
    marks["synchronized"] = time.perf_counter() - t0
    D.barrier()
    el = time.perf_counter() - t0
    marks = {k: round(v * 1e6, 1) for k, v in marks.items()}
    kern_ms_timed = None
    ev_tot = ev_cnt = sp_tot = sp_cnt = 0
    for c in ctxs:
        if timed_events:
            _lib.check(L.nmz_timing_read(c.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1))
            ev_tot, ev_cnt = ev_tot + tot.value, ev_cnt + cnt.value
        # the timed launches' execution spans as the kernel records them (first workgroup start to last workgroup
        # end): a pipelined launch's HIP events would also time its wait for the CUs another stream's K1 holds
        _lib.check(L.nmz_timing_read_span(c.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1))
        sp_tot, sp_cnt = sp_tot + tot.value, sp_cnt + cnt.value
        _lib.check(L.nmz_timing_enable(c.handle, 0))
    if timed_events:
        kern_ms_timed = ev_tot / max(ev_cnt, 1)
    kern_ms_span = sp_tot / sp_cnt if sp_cnt else None
    gpu_ms = start_ev.elapsed_time(done_ev) if not host_merge else None
    el_max = D.max(torch, el)
    # the job's answer, checked outside the timing: every step's list is the exact top-64 of its own range, so the
    # job's top-64 is the merge of those lists; timed step 0's stats (seeds "0".."S-1" on rank 0) for the CPU
    # baseline's parity check
    # (N > 1: the rank's own list is that merge, and the job's list the host merge of the gathered rank lists)
    lists = np.frombuffer(d_lists.cpu().numpy().tobytes(), dtype=_lib.TOPK_DTYPE)
    own = np.frombuffer(d_job.cpu().numpy().tobytes(), dtype=_lib.TOPK_DTYPE)
    want = merge_topk(b"".join(lists[i * K_TOP:(i + 1) * K_TOP].tobytes() for i in range(args.steps)), K_TOP)
    job_ok = bool(np.array_equal(want, own))
    if D.world == 1:
        job_ok = job_ok and bool(np.array_equal(want, merged))
    elif not host_merge:
        job_ok = job_ok and bool(np.array_equal(merge_topk(d_gath.cpu().numpy().tobytes(), K_TOP), merged))
    sweep(0, D.rank * S, d_job.data_ptr())
    torch.cuda.synchronize()
    stats = np.frombuffer(d_stats[0].cpu().numpy().tobytes(), dtype=_lib.SCHED_STATS_DTYPE)
    seed_lo = [D.rank * S]
    d_soff = [torch.from_numpy(csr0[0].view(np.int32)).to(dev)]
    d_sb = [torch.from_numpy(csr0[1]).to(dev)]
    for plan in plans:
        L.nmz_replayable_plan_destroy(plan)
    torch.cuda.synchronize()
    for c in ctxs[1:]:
        c.close()
    # configs[1] as stated, end to end: a new trace's plan (tables built and sorted from host hints) + one
    # 2^20-seed sweep with top-k + the copy of the top-k to the host, per trace
    e2e, e2e_plan, e2e_heads = [], [], []
    e2e_hints = [to_csr(zk_hints(E, seed=0x5EED + 1 + i)) for i in range(args.e2e_traces)]
    d_tk = torch.empty(K_TOP * 24, dtype=torch.uint8, device=dev)
    for i, (ho, hbb) in enumerate(e2e_hints):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        plan = ctypes.c_void_p()
        _lib.check(L.nmz_replayable_plan_create(ctx.handle, host_ptr(ho), host_ptr(hbb), E, MAX_INTERVAL_NS, S,
                                                ctypes.byref(plan)))
        e2e_plan.append(time.perf_counter() - t0)
        _lib.check(L.nmz_replayable_sweep_topk_dev(plan, ctypes.c_void_p(d_soff[0].data_ptr()),
                                                   ctypes.c_void_p(d_sb[0].data_ptr()), S, seed_lo[0], K_TOP,
                                                   ctypes.c_void_p(d_stats[0].data_ptr()),
                                                   ctypes.c_void_p(d_tk.data_ptr()), stream))
        tk0 = d_tk.cpu().numpy()
        e2e.append(time.perf_counter() - t0)
        e2e_heads.append(int(np.frombuffer(tk0.tobytes(), dtype=_lib.TOPK_DTYPE)["seed"][0]))
        L.nmz_replayable_plan_destroy(plan)
    # the same per-trace work as a stream of traces, the way a sweep tool over many recorded traces runs it: trace
    # i + 2's plan build is enqueued (nmz_replayable_plan_create_async, on two contexts' streams) while trace i
    # sweeps (two sweep streams, alternating); trace i's top-64 reaches pinned host memory by an asynchronous copy
    # and is read (and its plan destroyed) after trace i + 1's sweep is enqueued. Every trace gets its own plan,
    # sweep and top-k on the host, from one host thread
    e2e_pipe = None
    if args.e2e_traces >= 2:
        ctx2 = _lib.Context(D.local_rank)
        ctxs = [ctx, ctx2]
        tks = [torch.empty(K_TOP * 24, dtype=torch.uint8, device=dev) for _ in range(2)]
        tkh = [torch.empty(K_TOP * 24, dtype=torch.uint8).pin_memory() for _ in range(2)]
        evs = [torch.cuda.Event() for _ in range(2)]
        sts = [d_stats[0], torch.empty(S * 32, dtype=torch.uint8, device=dev)]
        T = len(e2e_hints)

        def make(i):
            ho, hbb = e2e_hints[i]
            p = ctypes.c_void_p()
            _lib.check(L.nmz_replayable_plan_create_async(ctxs[i % 2].handle, host_ptr(ho), host_ptr(hbb), E,
                                                          MAX_INTERVAL_NS, S, ctypes.byref(p)))
            return p

        # consecutive traces sweep on two streams: trace i's top-k selection overlaps trace i + 1's sweep
        sws = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]

        seedset = [None]  # one prepared seed set (prefix hashes bucketed once) for every trace of the stream

        def sweep(i, p):
            with torch.cuda.stream(sws[i % 2]):
                _lib.check(L.nmz_replayable_sweep_seeds_topk_dev(p, seedset[0], seed_lo[0], K_TOP,
                                                                 ctypes.c_void_p(sts[i % 2].data_ptr()),
                                                                 ctypes.c_void_p(tks[i % 2].data_ptr()),
                                                                 ctypes.c_void_p(sws[i % 2].cuda_stream)))
                tkh[i % 2].copy_(tks[i % 2], non_blocking=True)  # on the same stream, after the sweep
                evs[i % 2].record()

        def finish(i, p, heads):
            evs[i % 2].synchronize()
            heads.append(int(np.frombuffer(tkh[i % 2].numpy().tobytes(), dtype=_lib.TOPK_DTYPE)["seed"][0]))
            L.nmz_replayable_plan_destroy(p)

        # plan builds enqueued this many traces ahead (a producer thread measured slower: 0.23 ms/trace)
        AHEAD = int(os.environ.get("NMZ_BENCH_AHEAD", "2"))

        def run(n):
            heads, iter_s = [], []
            ss = ctypes.c_void_p()
            _lib.check(L.nmz_replayable_seeds_create(ctx.handle, ctypes.c_void_p(d_soff[0].data_ptr()),
                                                     ctypes.c_void_p(d_sb[0].data_ptr()), S, 0, ctypes.byref(ss)))
            seedset[0] = ss
            plans = {j: make(j) for j in range(min(AHEAD, n))}
            for i in range(n):
                ti = time.perf_counter()
                if i + AHEAD < n:
                    plans[i + AHEAD] = make(i + AHEAD)
                sweep(i, plans[i])
                if i >= 1:
                    finish(i - 1, plans.pop(i - 1), heads)
                iter_s.append(time.perf_counter() - ti)
            finish(n - 1, plans.pop(n - 1), heads)
            L.nmz_replayable_seeds_destroy(ss)
            return heads, iter_s

        run(min(T, 6))  # each context's pooled buffers and pinned staging for its live plans
        torch.cuda.synchronize()
        gc.collect()  # a full collection inside the timed traces costs ~50 ms (the bench holds many objects)
        gc.disable()
        t0 = time.perf_counter()
        heads, iter_s = run(T)
        t1 = time.perf_counter()
        gc.enable()
        e2e_pipe = dict(traces=T, ms_per_trace=(t1 - t0) * 1e3 / T, top1=heads[:4],
                        agrees=heads == e2e_heads, iter_ms_median=float(np.median(iter_s)) * 1e3,
                        iter_ms_max=float(np.max(iter_s)) * 1e3, iter_max_at=int(np.argmax(iter_s)))
        ctx2.close()
    # the same stream of traces through the native batch entry point (nmz_replayable_sweep_traces: the pipeline
    # above inside the library, one call for all traces; a Go caller's form)
    e2e_native = None
    if args.e2e_traces >= 2:
        T = len(e2e_hints)
        offs = (ctypes.c_void_p * T)(*[ctypes.c_void_p(ho.ctypes.data) for ho, _ in e2e_hints])
        byts = (ctypes.c_void_p * T)(*[ctypes.c_void_p(hbb.ctypes.data) for _, hbb in e2e_hints])
        nev = np.full(T, E, np.uint32)
        out = np.zeros(T * K_TOP, _lib.TOPK_DTYPE)

        def batch():
            _lib.check(L.nmz_replayable_sweep_traces(ctx.handle, T, offs, byts, host_ptr(nev), MAX_INTERVAL_NS,
                                                     seed_lo[0], S, K_TOP, host_ptr(out)))

        batch()  # first call: the helper context, streams and pooled buffers
        torch.cuda.synchronize()
        ms = []
        for _ in range(3):
            gc.collect()
            gc.disable()
            t0 = time.perf_counter()
            batch()
            ms.append((time.perf_counter() - t0) * 1e3 / T)
            gc.enable()
        heads = [int(x) for x in out["seed"][::K_TOP]]
        e2e_native = dict(traces=T, ms_per_trace=float(np.median(ms)), ms_per_trace_runs=ms, top1=heads[:4],
                          agrees=heads == e2e_heads)
    return dict(S=S, E=E, hints=(hoff, hb), seeds=csr0, elapsed=el_max,
                kern_ms=kern_ms, kern_ms_events=kern_ms_timed, kern_ms_serial_span=kern_ms_serial_span,
                kern_ms_span=kern_ms_span, enqueue_ms=enq * 1e3, gpu_ms=gpu_ms, host_marks_us=marks, plan_ms=plan_ms, stats=stats, topk=merged, pipeline=NP, job_ok=job_ok,
                e2e_s=e2e, e2e_plan_s=e2e_plan, e2e_pipe=e2e_pipe, e2e_native=e2e_native, k1_kernel=k1)


def cpu_baseline_replayable(r, args):
    from oracle import oracle as O
    n = min(args.cpu_seeds, r["S"])
    soff, sb = r["seeds"]
    hoff, hb = r["hints"]
    threads = cpu_threads()
    t0 = time.perf_counter()
    st, _ = O.replayable_sweep(soff[: n + 1].copy(), sb, hoff, hb, MAX_INTERVAL_NS, nthreads=threads)
    dt = time.perf_counter() - t0
    parity = bool(np.array_equal(st, r["stats"][:n]))
    n1 = max(n // 16, 1)  # single core, a sixteenth of the sample
    t0 = time.perf_counter()
    O.replayable_sweep(soff[: n1 + 1].copy(), sb, hoff, hb, MAX_INTERVAL_NS, nthreads=1)
    dt1 = time.perf_counter() - t0
    return dict(value=n * r["E"] / dt, unit="decisions/s", cores=threads, kind="port",
                sample=f"first {n} of {r['S']} seeds x {r['E']} events (oracle/nmz_oracle.c, OpenMP)",
                parity_with_gpu=parity, seconds=round(dt, 3), cpu_model=cpu_model(),
                single_core=dict(value=n1 * r["E"] / dt1, sample=f"first {n1} seeds", seconds=round(dt1, 3)))


def config3_trace(E=10_000):
    """configs[3] / configs[0] trace: 16 entities entity-(i%16) (explorepolicytester.go:36), entity-0..3
    prioritized, every event a deferred PacketEvent (faultable); event hashes SplitMix64(0x5EED1)."""
    from namazu_amd import _lib
    from namazu_amd.synth import splitmix64 as sm
    ent = np.arange(E) % 16
    evhash = sm(0x5EED1, E)
    evclass = np.where(ent < 4, _lib.NMZ_EV_PRIORITIZED, 0).astype(np.uint8) | np.uint8(_lib.NMZ_EV_FAULTABLE)
    return evhash, evclass


def bench_random_fault_sweep(args, torch, D, ctx, L, stream):
    """configs[3]: 10^7 schedules (seeds 0..10^7-1) over the 16-entity 10k-event trace, p = 0.1, split over the
    ranks by shard_range (strong scaling: the job is fixed). One step = each rank's sweep of its share + its
    device top-64 + (N > 1) RCCL all_gather of the ranks' top-64 lists + the deterministic merge."""
    from namazu_amd import _lib
    from namazu_amd import dist as nd
    S_total, E, K = args.random_total, 10_000, 64
    evhash, evclass = config3_trace(E)
    params = _lib.resolve_random_params(30_000_000, 100_000_000, 0.1)
    dev = torch.device("cuda", D.local_rank)
    sh = nd.RandomShardSweep(ctx, torch, dev, evhash, evclass, params, 0, S_total, D.world, D.rank, k=K)
    gathered = [torch.empty_like(sh.d_topk) for _ in range(D.world)] if D.world > 1 else None

    def step():
        sh.step(stream)
        if D.pg:
            D.pg.all_gather(gathered, sh.d_topk)

    step()
    torch.cuda.synchronize()
    tot, cnt = ctypes.c_double(), ctypes.c_uint64()
    _lib.check(L.nmz_timing_enable(ctx.handle, 1))
    L.nmz_timing_read(ctx.handle, b"random_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1)
    steps = args.random_steps
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    D.barrier()
    el = D.max(torch, time.perf_counter() - t0)
    _lib.check(L.nmz_timing_read(ctx.handle, b"random_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1))
    _lib.check(L.nmz_timing_enable(ctx.handle, 0))
    parts = [g.cpu().numpy() for g in gathered] if gathered else [sh.d_topk.cpu().numpy()]
    merged = nd.merge_topk(parts, K)
    kern_ms = tot.value / max(cnt.value, 1)
    out = dict(metric="random-policy fault-sweep decisions/s", value=S_total * E * steps / el, unit="decisions/s",
               n_gpus=D.world, steps=steps, ms_per_step=el / steps * 1e3, scaling="strong",
               config={"workload": "configs[3] random fault sweep", "schedules": S_total, "events": E,
                       "entities": 16, "prioritized": 4, "fault_probability": 0.1, "topk": K,
                       "parallelism": f"seed-range x{D.world}" + (" + RCCL all_gather top-k" if D.world > 1 else "")},
               kernel_ms=kern_ms,
               roofline=roofline_valu("k_random_sweep", sh.n * E, kern_ms),
               topk_head=[[int(x["seed"]), int(x["n_fault"]), int(x["sum_delay_ns"])] for x in merged[:4]])
    if D.rank == 0 and args.cpu_baseline and D.world == 1:
        from oracle import oracle as O
        p = O.random_params(30_000_000, 100_000_000, 0.1)
        n = args.cpu_random_seeds
        threads = cpu_threads()
        t0 = time.perf_counter()
        st, _, _ = O.random_sweep(0, n, evhash, evclass, p, nthreads=threads)
        dt = time.perf_counter() - t0
        n1 = max(n // 16, 1)
        t0 = time.perf_counter()
        O.random_sweep(0, n1, evhash, evclass, p, nthreads=1)
        dt1 = time.perf_counter() - t0
        # the winners' stats and the first seeds' stats vs the oracle
        ok = bool(np.array_equal(st, sh.stats()[:n]))
        for e in merged[:2]:
            ost, _, _ = O.random_sweep(int(e["seed"]), 1, evhash, evclass, p)
            ok = ok and int(ost["n_fault"][0]) == int(e["n_fault"]) and \
                int(ost["sum_delay_ns"][0]) == int(e["sum_delay_ns"]) % (1 << 64)
        out["cpu_baseline"] = dict(value=n * E / dt, unit="decisions/s", cores=threads, kind="port",
                                   sample=f"first {n} seeds x {E} events (oracle/nmz_oracle.c, full Go Seed per "
                                          f"decision)", seconds=round(dt, 3), parity_with_gpu=ok,
                                   cpu_model=cpu_model(),
                                   single_core=dict(value=n1 * E / dt1, sample=f"first {n1} seeds",
                                                    seconds=round(dt1, 3)))
    sh.close()
    return out


def bench_replayable_cliffs(args, torch, D, ctx, L, stream):
    """K1 outside configs[1]'s comfort zone (the reference accepts any Duration, replayablepolicy.go:66-72):
    maxInterval 2 s and 3 s (residues >= 2^31: the 32-bit sums overflow and are corrected) at configs[1]'s shape,
    and a 10,000-event trace whose order-query row image exceeds LDS (class segments split into passes). One
    2^20-seed sweep + top-64 per step on one stream (no pipelining), decisions/s and the sweep's kernel time."""
    from namazu_amd import _lib
    S = args.seeds
    csr = decimal_csr(0, S)
    dev = torch.device("cuda", D.local_rank)
    d_soff = torch.from_numpy(csr[0].view(np.int32)).to(dev)
    d_sb = torch.from_numpy(csr[1]).to(dev)
    d_stats = torch.empty(S * 32, dtype=torch.uint8, device=dev)
    d_tk = torch.empty(64 * 24, dtype=torch.uint8, device=dev)
    out = []
    for E, m in ((4096, 2_000_000_000), (4096, 3_000_000_000), (10_000, MAX_INTERVAL_NS)):
        hoff, hb = __import__("namazu_amd.explorepolicy", fromlist=["to_csr"]).to_csr(zk_hints(E))
        plan = ctypes.c_void_p()
        _lib.check(L.nmz_replayable_plan_create(ctx.handle, host_ptr(hoff), host_ptr(hb), E, m, S, ctypes.byref(plan)))

        def step():
            _lib.check(L.nmz_replayable_sweep_topk_dev(plan, ctypes.c_void_p(d_soff.data_ptr()),
                                                       ctypes.c_void_p(d_sb.data_ptr()), S, 0, 64,
                                                       ctypes.c_void_p(d_stats.data_ptr()),
                                                       ctypes.c_void_p(d_tk.data_ptr()), stream))
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        tot, cnt = ctypes.c_double(), ctypes.c_uint64()
        _lib.check(L.nmz_timing_enable(ctx.handle, 1))
        L.nmz_timing_read(ctx.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1)
        steps = 10
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        _lib.check(L.nmz_timing_read(ctx.handle, b"replayable_sweep", ctypes.byref(tot), ctypes.byref(cnt), 1))
        _lib.check(L.nmz_timing_enable(ctx.handle, 0))
        stats = np.frombuffer(d_stats.cpu().numpy().tobytes(), dtype=_lib.SCHED_STATS_DTYPE)
        parity = None
        if D.rank == 0 and args.cpu_baseline:
            from oracle import oracle as O
            n = 2048
            st, _ = O.replayable_sweep(csr[0][: n + 1].copy(), csr[1], hoff, hb, m, nthreads=cpu_threads())
            parity = bool(np.array_equal(st, stats[:n]))
        L.nmz_replayable_plan_destroy(plan)
        out.append(dict(events=E, max_interval_ns=m, value=S * E * steps / el, unit="decisions/s",
                        ms_per_step=el / steps * 1e3, kernel_ms=tot.value / max(cnt.value, 1),
                        parity_with_oracle_first_2048_seeds=parity))
    return dict(metric="replayable seed sweep outside configs[1]: long intervals and long traces",
                config={"workload": "K1 cliffs: maxInterval 2 s / 3 s at 2^20 x 4,096; 2^20 seeds x 10,000 events",
                        "seeds": S}, lines=out)


def bench_visualize(args, torch, D, ctx, L, stream):
    """`nmz tools visualize` over a 100k-run store (2,048 events, 16 entities; runs repeat earlier runs exactly or
    re-interleaved across entities): the unique-trace curve in the reference's default partial-order mode and
    in exact mode, one nmz_unique_traces_dev call each (signatures + radix-sort classes) on device-resident
    traces. The reference compares every new run with every unique one so far (O(n^2) equality tests,
    visualize.go:126-172); its CPU restatement runs on a sample."""
    from namazu_amd import _lib
    from namazu_amd import synth
    N, Lx = args.vis_traces, 2048
    t0 = time.time()
    ts, ent, n_bases = synth.po_store(N, Lx)
    synth_s = time.time() - t0
    dev = torch.device("cuda", D.local_rank)
    d_off = torch.from_numpy(ts.off.view(np.int64)).to(dev)
    d_sym = torch.from_numpy(ts.sym.view(np.int64)).to(dev)
    d_ent = torch.from_numpy(ent.view(np.int32)).to(dev)
    d_sig = torch.empty(2 * N, dtype=torch.int64, device=dev)
    d_first = torch.empty(N, dtype=torch.int32, device=dev)

    def run(po):
        _lib.check(L.nmz_unique_traces_dev(ctx.handle, ctypes.c_void_p(d_off.data_ptr()),
                                           ctypes.c_void_p(d_sym.data_ptr()),
                                           ctypes.c_void_p(d_ent.data_ptr()) if po else None, N, 16,
                                           ctypes.c_void_p(d_sig.data_ptr()), ctypes.c_void_p(d_first.data_ptr()),
                                           stream))

    out = dict(metric="visualize unique-trace curve, traces/s", unit="traces/s",
               config={"workload": "nmz tools visualize (gnuplot) over a stored-run set", "traces": N, "events": Lx,
                       "entities": 16, "distinct_runs_by_construction": n_bases}, synth_s=round(synth_s, 2))
    for po in (True, False):
        run(po)
        torch.cuda.synchronize()
        tot, cnt = ctypes.c_double(), ctypes.c_uint64()
        _lib.check(L.nmz_timing_enable(ctx.handle, 1))
        L.nmz_timing_read(ctx.handle, b"trace_sig", ctypes.byref(tot), ctypes.byref(cnt), 1)
        steps = 3
        t0 = time.perf_counter()
        for _ in range(steps):
            run(po)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps
        _lib.check(L.nmz_timing_read(ctx.handle, b"trace_sig", ctypes.byref(tot), ctypes.byref(cnt), 1))
        _lib.check(L.nmz_timing_enable(ctx.handle, 0))
        first = d_first.cpu().numpy().view(np.uint32)
        uniq = int((first == np.arange(N)).sum())
        sig_ms = tot.value / max(cnt.value, 1)
        algo_bytes = ts.sym.nbytes + (ent.nbytes if po else 0) + 16 * N  # symbols (+ entity ids) read, sig written
        key = "k_trace_sig:" + ("po" if po else "exact")
        prof = valu_entry(key) or {}
        traffic_fresh = bool(prof) and isa_state(prof)[0]
        achieved = algo_bytes / (sig_ms * 1e-3) / 1e9
        out["po" if po else "exact"] = dict(
            value=N / el, ms=el * 1e3, unique=uniq, sig_kernel_ms=sig_ms,
            roofline={"bound": "hbm", "kernel": "k_trace_sig", "achieved": achieved, "peak": PEAK_HBM_GBS,
                      "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS, "algorithmic_bytes": algo_bytes,
                      "traffic": prof.get("hbm_bytes_per_launch") if traffic_fresh else None,
                      "traffic_stale": not traffic_fresh,
                      "traffic_unit": "bytes/launch (2 x FETCH_SIZE + WRITE_SIZE)",
                      "ops_per_unit": prof.get("ops_per_unit"), "ops_unit": "VALU lane-instr per trace"})
    out["value"] = out["po"]["value"]
    out["roofline"] = out["po"]["roofline"]
    out["po"]["unique_matches_construction"] = out["po"]["unique"] == n_bases
    if D.rank == 0 and args.cpu_baseline:
        from oracle import oracle as O
        n = args.vis_cpu_traces
        raw = [list(zip(ent[i * Lx:(i + 1) * Lx].tolist(), ts.sym[i * Lx:(i + 1) * Lx].tolist())) for i in range(n)]
        t0 = time.perf_counter()
        curve = O.unique_curve_po(raw)
        dt = time.perf_counter() - t0
        from namazu_amd.historystorage import TraceSet
        sub_ts = TraceSet([ts.sym[i * Lx:(i + 1) * Lx] for i in range(n)])
        fe = np.zeros(n, np.uint32)
        ent_sub = np.ascontiguousarray(ent[:n * Lx])
        _lib.check(L.nmz_unique_traces(ctx.handle, _lib.ptr(sub_ts.off), _lib.ptr(sub_ts.sym), _lib.ptr(ent_sub), n,
                                       _lib.ptr(fe)))
        gpu_curve = np.cumsum(fe == np.arange(n)).tolist()
        out["cpu_baseline"] = dict(value=n / dt, unit="traces/s", cores=1, kind="port",
                                   sample=f"first {n} runs, oracle.unique_curve_po (the reference's loops, O(n^2) "
                                          f"in runs: the rate falls as the store grows)",
                                   seconds=round(dt, 3), parity_with_gpu=gpu_curve == curve)
    return out


def bench_config0(args, torch, D, ctx, L):
    """configs[0]: the random policy over one 10k-event trace under one seed, the reference's own CPU case.
    Reported: the CPU restatement on one core (the reference decides on one goroutine per event, seeding Go's
    rand per event: impl.go:39), the GPU decision of the whole trace in one nmz_random_decide call, and the
    online path's per-event decision latency through QueueEvent (enqueue -> decided): events sent back to back
    (the decision thread batches them) and one at a time (each waits for its own launch)."""
    from namazu_amd.config import Config
    from namazu_amd.explorepolicy import Random
    from namazu_amd.signal import Event
    from oracle import oracle as O
    E = 10_000
    evhash, evclass = config3_trace(E)
    p = Random()
    p.LoadConfig(Config({"explorePolicy": "random", "explorePolicyParam": {
        "minInterval": "30ms", "maxInterval": "100ms", "faultActionProbability": 0.1, "seed": 1,
        "prioritizedEntities": [f"entity-{i}" for i in range(4)]}}))
    pr = O.random_params(30_000_000, 100_000_000, 0.1)
    t0 = time.perf_counter()
    st, dl, fl = O.random_sweep(1, 1, evhash, evclass, pr, n_dump=1, nthreads=1)
    cpu_s = time.perf_counter() - t0

    class _Ev:  # the trace's events as the kernel sees them (hash + class), for decide_events
        def __init__(self, i):
            self.i = i
    p.event_inputs = lambda evs: (evhash[[e.i for e in evs]], evclass[[e.i for e in evs]])
    evs = [_Ev(i) for i in range(E)]
    p.decide_events(evs[:16])  # warm the launch path
    times = []
    for _ in range(5):
        t0 = time.perf_counter()
        d, f = p.decide_events(evs)
        times.append(time.perf_counter() - t0)
    parity = bool(np.array_equal(d, dl[0]) and np.array_equal(f, fl[0].astype(bool)))
    # online: QueueEvent with real events under configs[0]'s parameters (30-100 ms delays): each event is decided
    # inside QueueEvent (the library's host decision path) and released by the native time-bounded queue at
    # enqueue + delay; latency = enqueue -> decided, delivered-delay error = release - (enqueue + decided delay)
    q = Random()
    q.LoadConfig(Config({"explorePolicy": "random", "explorePolicyParam": {
        "minInterval": "30ms", "maxInterval": "100ms", "faultActionProbability": 0.1, "seed": 1,
        "prioritizedEntities": [f"entity-{i}" for i in range(4)]}}))
    events = [Event.packet(f"entity-{i % 16}", f"entity-{i % 16}", f"entity-{(i + 1) % 16}", {"n": i})
              for i in range(2000)]

    def run(evs, one_at_a_time):
        q.online.latencies_ns.clear()
        q.online.delivery_err_ns.clear()
        for ev in evs:
            q.QueueEvent(ev)
            if one_at_a_time:
                q.online.wait_decided(10)
        q.online.wait_delivered(30)
        for _ in evs:
            q.ActionChan().get(timeout=10)
        lat = np.array(q.online.latencies_ns, np.float64) / 1e3
        err = np.array(q.online.delivery_err_ns, np.float64) / 1e3
        return dict(events=len(lat), p50=float(np.percentile(lat, 50)), p99=float(np.percentile(lat, 99)),
                    delivered_delay_error_us=dict(p50=float(np.percentile(err, 50)),
                                                  p99=float(np.percentile(err, 99)), max=float(err.max())))
    run(events[:50], False)  # warm-up
    burst = run(events, False)
    single = run(events[:300], True)
    # the fixed-duration lane (BasicTBQueue's one goroutine for min == max, util/queue/impl.go:77-89): the random
    # policy with maxInterval unset (= minInterval = 1 ms), a 200-event burst through QueueEvent: released in order
    # at ~1, 2, ..., 200 ms, each at (the previous release or its enqueue) + 1 ms
    f = Random()
    f.LoadConfig(Config({"explorePolicy": "random", "explorePolicyParam": {"minInterval": "1ms", "seed": 1}}))
    ch = f.ActionChan()
    t0 = ch.L.nmz_monotonic_ns()
    for ev in events[:200]:
        f.QueueEvent(ev)
    rel = []
    for _ in range(200):
        ch.get(timeout=10)
        rel.append(ch.last_release_ns - t0)
    rel = np.array(rel, np.float64)
    late = np.array(list(ch.delivery_err_ns)[-200:], np.float64) / 1e3
    fixed_lane = dict(events=200, duration_ms=1.0, last_release_ms=float(rel[-1] / 1e6),
                      min_gap_ms=float(np.diff(rel).min() / 1e6),
                      release_after_rule_us=dict(p50=float(np.percentile(late, 50)), p99=float(np.percentile(late, 99)),
                                                 max=float(late.max())),
                      what="random policy, maxInterval = minInterval = 1 ms: one FIFO lane, item k released at "
                           "max(its enqueue, release k-1) + 1 ms (impl.go:77-89); the burst ends at ~200 ms")
    ch.close()
    return dict(metric="configs[0] random policy, one seed over one 10k-event trace", unit="decisions/s",
                cpu_1core=dict(value=E / cpu_s, seconds=round(cpu_s, 4), kind="port",
                               note="oracle/nmz_oracle.c: full Go rand.Seed per decision, as the reference reseeds "
                                    "per event (util/queue/impl.go:39)"),
                gpu_batch=dict(value=E / min(times), ms=min(times) * 1e3,
                               note="nmz_random_decide, the whole trace in one call (host arrays in and out)"),
                parity_with_gpu=parity,
                fixed_duration_lane=fixed_lane,
                queue_event_latency_us=dict(mode=q.online.mode, burst=burst, one_at_a_time=single,
                                            what="enqueue -> decided inside QueueEvent (nmz_random_decide_host: the "
                                                 "kernels' closed forms on the host); delivered-delay error = "
                                                 "native release time - (enqueue + decided delay)"))


def bench_ed_secondary(args, torch, D, ctx, L, stream, spec):
    """All-pairs banded edit-distance k-NN (configs[2] and configs[4]).
    Total work is fixed (strong scaling): rank r runs shard r of N(N-1)/2 pairs; the partial k-NN key
    lists are all_gathered over RCCL and merged on the device (nmz_knn_merge_dev) inside the step."""
    from namazu_amd import _lib
    from namazu_amd import synth
    N, k, ED_LEN, ED_BAND = spec["traces"], spec["k"], spec["events"], spec["band"]
    t0 = time.time()
    ts = getattr(synth, spec["generator"])(N, ED_LEN, **spec.get("gen_kwargs", {}))
    synth_s = time.time() - t0
    plan = ctypes.c_void_p()
    dev = torch.device("cuda", D.local_rank)
    D.barrier()
    t0 = time.time()
    # the store's event hashes reach every device as 1/N shares over its own PCIe link plus one RCCL all_gather
    # over xGMI (not the whole store through every link), then the plan is built from device memory
    total = int(ts.off[-1])
    share = -(-total // D.world)
    lo, hi = min(D.rank * share, total), min((D.rank + 1) * share, total)
    mine = torch.zeros(max(share, 1), dtype=torch.int64, device=dev)
    if hi > lo:
        mine[:hi - lo] = torch.from_numpy(np.ascontiguousarray(ts.sym[lo:hi]).view(np.int64)).to(dev)
    if D.pg:
        full = torch.empty(max(share, 1) * D.world, dtype=torch.int64, device=dev)
        D.pg.all_gather_into_tensor(full, mine)
    else:
        full = mine
    torch.cuda.synchronize()
    upload_ms = (time.time() - t0) * 1e3
    _lib.check(L.nmz_ed_plan_create_dev(ctx.handle, host_ptr(ts.off), ctypes.c_void_p(full.data_ptr()), N, ED_BAND,
                                        ctypes.byref(plan)))
    del full, mine
    plan_ms = (time.time() - t0) * 1e3
    kind = {3: "k_ed_wide", 2: "k_ed_bv", 1: "k_ed_tile", 0: "k_ed_generic"}[L.nmz_ed_plan_is_fast(plan)]
    if D.pg:  # every rank must hold the same plan (kernel, store, options), or the shards would not partition
        from namazu_amd import dist as nd
        nd.check_ed_plans(D.pg, L, plan, device=dev)
    d_knn = torch.empty(N * k, dtype=torch.int64, device=dev)
    d_parts = torch.empty(D.world * N * k, dtype=torch.int64, device=dev) if D.world > 1 else None
    d_out = torch.empty(N * k, dtype=torch.int64, device=dev) if D.world > 1 else d_knn

    def step():
        _lib.check(L.nmz_ed_allpairs_knn_shard_dev(plan, k, D.rank, D.world, ctypes.c_void_p(d_knn.data_ptr()),
                                                   stream))
        if D.pg:
            D.pg.all_gather_into_tensor(d_parts, d_knn)
            _lib.check(L.nmz_knn_merge_dev(ctx.handle, ctypes.c_void_p(d_parts.data_ptr()), D.world, N, k,
                                           ctypes.c_void_p(d_out.data_ptr()), stream))
            _lib.check(L.nmz_ed_knn_fill_dev(plan, k, ctypes.c_void_p(d_out.data_ptr()), stream))

    step()
    torch.cuda.synchronize()
    tname = kind[2:].encode()
    _lib.check(L.nmz_timing_enable(ctx.handle, 1))
    tot, cnt = ctypes.c_double(), ctypes.c_uint64()
    L.nmz_timing_read(ctx.handle, tname, ctypes.byref(tot), ctypes.byref(cnt), 1)
    # the two-phase bit-parallel search's kernels (csrc/ed.hip ed_bv_two_phase): filter passes and DP work items
    phase_t = {n: (ctypes.c_double(), ctypes.c_uint64()) for n in (b"ed_qg_filter", b"ed_bv_dp")}
    for n, (a, b) in phase_t.items():
        L.nmz_timing_read(ctx.handle, n, ctypes.byref(a), ctypes.byref(b), 1)
    steps = spec["steps"]
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    D.barrier()
    el = D.max(torch, time.perf_counter() - t0)
    _lib.check(L.nmz_timing_read(ctx.handle, tname, ctypes.byref(tot), ctypes.byref(cnt), 1))
    for n, (a, b) in phase_t.items():
        _lib.check(L.nmz_timing_read(ctx.handle, n, ctypes.byref(a), ctypes.byref(b), 1))
    phase_ms = {n.decode(): a.value / steps for n, (a, b) in phase_t.items() if b.value}  # per search
    _lib.check(L.nmz_timing_enable(ctx.handle, 0))
    counters = np.zeros(_lib.NMZ_ED_NCOUNTERS, np.uint64)
    _lib.check(L.nmz_ed_plan_counters(plan, _lib.ptr(counters), stream))
    single = None
    if kind in ("k_ed_bv", "k_ed_wide") and D.rank == 0:
        # single queries against the resident store (SearchSimilar): stored traces as queries, one call
        # (k_ed_bv_query for band <= 64, k_ed_wide_query above)
        from namazu_amd.historystorage import TraceSet
        NQ = 8 if kind == "k_ed_bv" else 4
        qset = TraceSet([ts.trace(i) for i in range(NQ)])
        kq = k + 1  # a stored trace queried finds itself too
        qi = np.zeros(NQ * kq, np.uint32)
        qd = np.zeros(NQ * kq, np.uint32)
        reps = []
        for _ in range(3):
            t0 = time.perf_counter()
            _lib.check(L.nmz_ed_plan_query_knn(plan, _lib.ptr(qset.off), _lib.ptr(qset.sym), NQ, kq, _lib.ptr(qi),
                                               _lib.ptr(qd)))
            reps.append(time.perf_counter() - t0)
        # the all-pairs k-NN lists of the same traces (self excluded) must agree with the single-query answers
        agree = None
        if D.world == 1:
            keys8 = d_out.cpu().numpy().view(np.uint64).reshape(N, k)[:NQ]
            agree = True
            for i in range(NQ):
                keep = qi.reshape(NQ, kq)[i] != i
                ids_i, ds_i = qi.reshape(NQ, kq)[i][keep][:k], qd.reshape(NQ, kq)[i][keep][:k]
                agree &= bool(np.array_equal((keys8[i] >> np.uint64(32)).astype(np.uint32), ds_i) and
                              np.array_equal((keys8[i] & np.uint64(0xFFFFFFFF)).astype(np.uint32), ids_i))
        single = dict(queries=NQ, ms_per_query=min(reps) * 1e3 / NQ, pairs_per_s=NQ * N / min(reps),
                      agrees_with_allpairs=agree, kernel=kind + "_query",
                      what=f"nmz_ed_plan_query_knn: {NQ} stored traces as queries vs the resident store, host arrays "
                           "in and out; agrees_with_allpairs compares each answer (self excluded) with the "
                           "all-pairs k-NN list")
    L.nmz_ed_plan_destroy(plan)
    pairs = N * (N - 1) // 2
    cells_per_pair = ED_LEN * (2 * ED_BAND + 1) - ED_BAND * (ED_BAND + 1)
    kern_ms = tot.value / max(cnt.value, 1)
    out = dict(metric="trace-pair edit distances/s (banded, all-pairs k-NN)", value=pairs * steps / el,
               unit="pairs/s", n_gpus=D.world, steps=steps, ms_per_step=el / steps * 1e3, scaling="strong",
               config={"workload": spec["workload"], "traces": N, "events": ED_LEN, "generator": spec["generator"],
                       "distinct_symbols": int(len(np.unique(ts.sym))),
                       "band": ED_BAND, "k": k, "parallelism": f"pair-tile shards x{D.world}" +
                       (" + RCCL all_gather k-NN merge" if D.world > 1 else "")},
               kernel=kind, kernel_ms=kern_ms, plan_ms=plan_ms, synth_s=round(synth_s, 2),
               plan_upload_ms=upload_ms,
               end_to_end_ms=plan_ms + el / steps * 1e3,
               end_to_end_note="plan (1/N upload of the store per device + RCCL all_gather + device plan build) + one "
                               "search step; the plan is built once per store, the headline value re-searches it",
               roofline=roofline_valu(spec.get("valu_key", kind), (pairs + D.world - 1) // D.world, kern_ms),
               nominal_band_cells_per_s=pairs * cells_per_pair * steps / el)
    if single:
        out["single_query"] = single
    if phase_ms:
        # two-phase search: the roofline belongs to the dominant kernel -- the DP over the pairs the filter kept
        # (unit: DP pair, counted by the kernel) or, when nearly every pair is settled by the filter, the filter
        # passes (unit: pair; both passes per search)
        dp_ms, f_ms = phase_ms.get("ed_bv_dp", 0.0), phase_ms.get("ed_qg_filter", 0.0)
        gen = spec.get("valu_key", kind).split(":")[-1]
        out["phases_ms"] = {"filter_count_plus_write": f_ms, "dp": dp_ms, "rest": kern_ms - f_ms - dp_ms}
        if dp_ms >= f_ms and counters[0]:
            out["roofline"] = roofline_valu(f"k_ed_bv_dp:{gen}", int(counters[0]), dp_ms)
        else:
            out["roofline"] = roofline_valu(f"k_ed_qg_filter:{gen}", (pairs + D.world - 1) // D.world, f_ms)
    if counters[3]:  # k_ed_bv work counters of the last step (this rank's shard)
        c = [int(x) for x in counters]
        shard_pairs = (pairs + D.world - 1) // D.world
        out["search"] = dict(
            shard_pairs=shard_pairs, dp_pairs=c[0], qgram_settled_pairs=c[5],
            length_band_settled_pairs=shard_pairs - c[0] - c[5], in_band_pairs=c[1],
            in_band_frac_of_shard_pairs=c[1] / shard_pairs, dp_frac_of_shard_pairs=c[0] / shard_pairs,
            mean_cutoff_column=32 * c[2] / c[3], full_columns=ED_LEN,
            executed_cells_per_s=c[2] * 32 * 2 * (2 * ED_BAND + 1) * D.world / (el / steps),
            live_cells_per_s=c[4] * 32 * (2 * ED_BAND + 1) * D.world / (el / steps),
            note="cells = band cells (2w+1 per column); executed = every candidate x 32-column block a lane stepped "
                 "(2 query columns each), live = the query columns still running in those blocks; q-gram settled = "
                 "pairs whose bigram profiles are > 4w apart, so ED > w is proven without a DP (result w + 1, exact)")
    keys = d_out.cpu().numpy().view(np.uint64).reshape(N, k)
    if D.rank == 0 and args.cpu_baseline and D.world == 1:
        from oracle import oracle as O
        threads = min(16, os.cpu_count() or 1)
        q = 0
        cand = np.array([c for c in range(N) if c != q], np.uint32)
        pairs_s = np.stack([np.full(len(cand), q, np.uint32), cand], 1)
        t0 = time.perf_counter()
        dist = O.ed_pairs(ts.off, ts.sym, pairs_s, ED_BAND, nthreads=threads)
        dt = time.perf_counter() - t0
        order = np.lexsort((cand, dist))[:k]
        ok = (keys[q] >> np.uint64(32)).astype(np.uint32).tolist() == dist[order].tolist() and \
            (keys[q] & np.uint64(0xFFFFFFFF)).astype(np.uint32).tolist() == cand[order].tolist()
        out["cpu_baseline"] = dict(value=len(cand) / dt, unit="pairs/s", cores=threads, kind="port",
                                   sample=f"trace 0 vs all {len(cand)} others (oracle/nmz_oracle.c full-band DP, "
                                          f"no cut-off)", seconds=round(dt, 3), parity_with_gpu=bool(ok))
    return out


def headline_line(args, torch, D, ctx, L, stream):
    """configs[1], the headline (see the module docstring)."""
    r = bench_replayable(args, torch, D, ctx, L, stream)
    decisions = D.world * r["S"] * r["E"] * args.steps
    value = decisions / r["elapsed"]
    dec_launch = r["S"] * r["E"]
    line = {
        "metric": "schedule decisions/sec + trace-pair edit distances/sec at 1/2/4/8 MI355X",
        "value": value,
        "unit": "decisions/s",
        "n_gpus": D.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["elapsed"] / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (ZooKeeper-style hints: signed decimal SplitMix64, seed 0x5EED; decimal seeds)",
        "config": {"workload": "configs[1] replayable seed sweep", "seeds_per_gpu": r["S"], "events": r["E"],
                   "max_interval_ns": MAX_INTERVAL_NS, "topk": 64, "pipeline_streams": r["pipeline"],
                   "seeds": "a fresh range of 2^20 decimal seeds per step and rank (seeds (i*N + rank)*2^20 ..)",
                   "unit_kind": "stats-equivalent decision: a (seed, event) decision whose effect on the seed's "
                                "statistics (sum, max, argmax, top-64) the sweep covers, bit-exact vs the "
                                "per-decision oracle; K1 derives them from searches, not event by event",
                   "parallelism": f"seed-range x{D.world}" + (" + RCCL all_gather top-k" if D.world > 1 else "")},
        "roofline": roofline_valu(r["k1_kernel"], dec_launch, r["kern_ms"]),
        # a new trace's plan (tables + segment sorts + allocations), median over the end-to-end traces;
        # plan_ms_first_three includes the process's first launches (module load) when the bench starts
        "plan_ms": float(np.median(r["e2e_plan_s"])) * 1e3,
        "plan_ms_first_three": r["plan_ms"],
        "topk_head": [int(x) for x in r["topk"]["seed"][:4]],
        "job_topk_equals_merge_of_step_lists": r["job_ok"],
        # host time to enqueue the K steps (the timed region's first part): close to ms_per_step * K means the
        # host's launches, not the GPU, set the step
        "enqueue_ms": r["enqueue_ms"],
        # the GPU's clock over the same region (HIP event before step 0 on the first slot's stream -> the event after
        # the answer's copy): the rest of ms_per_step * K is the host's (first launch, wake-up after the last event)
        "gpu_ms": r["gpu_ms"],
        "host_marks_us": r["host_marks_us"],  # host clock from the region's start at each step of its end
        "steady_state":"value: one trace's resident plan (built once, before the timed region) sweeps a fresh seed "
                        "range every step, and the job's top-64 is merged on the device (+ RCCL all_gather for N > "
                        "1) inside the timing; end_to_end below builds a new trace's plan inside the timing",
    }
    one = {"value": dec_launch / float(np.median(r["e2e_s"])), "unit": "decisions/s",
           "ms_median": float(np.median(r["e2e_s"])) * 1e3, "traces": len(r["e2e_s"]),
           "plan_ms": float(np.median(r["e2e_plan_s"])) * 1e3,
           "what": "per trace, one at a time: nmz_replayable_plan_create from host hints (table, sorts and wavelet "
                   "trees: one plan kernel) + one 2^20-seed sweep with top-64 + top-64 copy to the host"}
    p, nat = r.get("e2e_pipe"), r.get("e2e_native")
    if p:
        # a stream of traces (how a sweep tool over many recorded traces runs): the throughput figure; the same
        # stream through the native batch entry point and the one-at-a-time latency inside
        line["end_to_end"] = {
            "value": dec_launch / (p["ms_per_trace"] * 1e-3), "unit": "decisions/s", "mode": "stream",
            "ms_per_trace": p["ms_per_trace"], "traces": p["traces"], "plan_ms": one["plan_ms"],
            "top1_head": p["top1"], "agrees_with_one_at_a_time": p["agrees"],
            "iter_ms_median": p["iter_ms_median"], "iter_ms_max": p["iter_ms_max"],
            "what": "every trace gets its own plan (nmz_replayable_plan_create_async from host hints, inside the "
                    "timing), one 2^20-seed sweep with top-64 and the top-64 on the host; the seeds' prefix hashes "
                    "are prepared once for the stream (nmz_replayable_seeds_create, inside the timing); one host "
                    "thread enqueues trace i+2's plan build (two contexts) while trace i sweeps (two streams); whole "
                    "elapsed time / traces. plan_ms: one plan built alone (one_at_a_time)",
            "one_at_a_time": one}
        if nat:
            line["end_to_end"]["native_batch"] = {
                "value": dec_launch / (nat["ms_per_trace"] * 1e-3), "ms_per_trace": nat["ms_per_trace"],
                "ms_per_trace_runs": nat["ms_per_trace_runs"], "agrees_with_one_at_a_time": nat["agrees"],
                "what": "the same stream in one nmz_replayable_sweep_traces call (the pipeline inside the library), "
                        "median of 3 calls"}
    else:
        line["end_to_end"] = dict(one, mode="one_at_a_time")
    if line["roofline"]:
        rf = line["roofline"]
        if r["k1_kernel"] in K1_ALGORITHM:
            # the kernel derives each seed's statistics (sum, max, argmax) from searches, not one decision
            # at a time: a unit is a decision whose effect on the statistics is covered, bit-exact vs the oracle
            rf["unit_kind"] = "stats-equivalent decision"
            # its lane-instructions per decision are the per-seed searches spread over the 4,096 decisions they
            # settle. The per-decision kernel's own ceiling (issue peak / its measured lane-instructions per
            # decision) is the rate an ideal event-by-event sweep could reach on this chip.
            rf["algorithm"] = K1_ALGORITHM[r["k1_kernel"]]
            pd = valu_entry("k_replayable_sweep_fast")
            if pd and isa_state(pd)[0]:
                ceil = PEAK_VALU_TOPS * 1e12 / pd["ops_per_unit"]
                rf["per_decision_ceiling"] = ceil
                rf["vs_per_decision_ceiling"] = line["value"] / ceil
        rf["kernel_ms_source"] = ("HIP events around K1, 50 launches back to back on one stream (as rocprofv3 "
                                  "times a dispatch)")
        # the timed region's own K1 launches: HIP events (include waits for CUs held by the other streams' kernels)
        # and the union of their in-kernel spans; the serial launches' in-kernel span
        rf["kernel_ms_events"] = r["kern_ms_events"]
        rf["kernel_ms_span"] = r["kern_ms_span"]
        rf["kernel_ms_serial_span"] = r["kern_ms_serial_span"]
        # the same lane-ops over the whole pipelined step (every kernel of the step on the clock)
        if not rf.get("stale"):
            rf["frac_of_step"] = (rf["ops_per_unit"] * dec_launch / (line["ms_per_step"] * 1e-3) / 1e12 /
                                  PEAK_VALU_TOPS)
    # survey 8(d) declared model for the reference's byte-serial algorithm: 6*len(hint)+18 ops per decision
    hoff = r["hints"][0]
    mean_len = float(np.mean(np.diff(hoff.astype(np.int64))))
    if line["roofline"]:
        rf = line["roofline"]
        rf["declared_model_ops_per_unit"] = 6 * mean_len + 18
        # the same decisions priced at SURVEY 8(d)'s per-decision model (the reference's byte-serial FNV over
        # seed || hint, then the modulo) over the measured K1 time: far above 1, because K1 does not decide event by
        # event (unit_kind); frac (measured lane-instructions) is the kernel's own utilisation
        if rf.get("kernel_ms"):
            rf["declared_model_frac"] = (rf["declared_model_ops_per_unit"] * dec_launch / (rf["kernel_ms"] * 1e-3) /
                                         1e12 / PEAK_VALU_TOPS)
    if D.rank == 0 and D.world == 1 and args.cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_replayable(r, args)
    return line


def bench_group(args, torch):
    """--group: every leg through one device group (nmz_open_group over devices 0..N-1 in this one process:
    a context + worker thread per device, one RCCL communicator; csrc/group.hip), as a Go host binding the C ABI
    would drive N GPUs. configs[1]: per step N x 2^20 decimal seeds (generated on the devices) x 4,096 hints with
    the merged top-64 on the host; configs[3]: 10^7 schedules split over the shards, merged top-64; configs[2]
    (clustered): the all-pairs k-NN, lists merged over RCCL and returned to the host. Every call is synchronous
    (host results), so this measures the C ABI's own multi-GPU path, not the pipelined torchrun path."""
    from namazu_amd import _lib
    from namazu_amd import group as G
    from namazu_amd import synth
    from namazu_amd.explorepolicy import to_csr
    n_dev = args.gpus
    n_shards = args.group_shards or n_dev
    g = G.Group(tuple(range(n_dev)), n_shards=n_shards)
    S, E = args.seeds, args.events
    hoff, hb = to_csr(zk_hints(E))
    t0 = time.perf_counter()
    rp = G.ReplayableGroupPlan(g, hoff, hb, MAX_INTERVAL_NS, max_seeds_per_shard=(S * n_dev + n_shards - 1) // n_shards)
    plan_ms = (time.perf_counter() - t0) * 1e3
    total = S * n_dev
    for i in range(args.warmup):
        rp.sweep_decimal(i * total, total, k=64, stats=False)
    t0 = time.perf_counter()
    for i in range(args.steps):
        _, tk = rp.sweep_decimal((args.warmup + i) * total, total, k=64, stats=False)
    el = time.perf_counter() - t0
    rp.close()
    line = {"metric": "schedule decisions/sec + trace-pair edit distances/sec at 1/2/4/8 MI355X",
            "value": total * E * args.steps / el, "unit": "decisions/s", "n_gpus": n_dev, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (ZooKeeper-style hints: signed decimal SplitMix64, seed 0x5EED; decimal seeds)",
            "config": {"workload": "configs[1] replayable seed sweep through a device group (C ABI)",
                       "seeds_per_gpu": S, "events": E, "max_interval_ns": MAX_INTERVAL_NS, "topk": 64,
                       "shards": n_shards,
                       "parallelism": f"nmz_open_group x{n_dev} (one process, RCCL all_gather top-k)"},
            "plan_ms": plan_ms, "topk_head": [int(x) for x in tk["seed"][:4]],
            "what": "per step: nmz_replayable_group_sweep_decimal -- every shard's sweep + device top-64, the "
                    "per-rank merge, RCCL all_gather, the final merge and the copy to the host"}
    sec = []
    if "random" in args.legs:
        evhash, evclass = config3_trace(10_000)
        params = _lib.resolve_random_params(30_000_000, 100_000_000, 0.1)
        n = args.random_total
        rg = G.RandomGroupPlan(g, evhash, evclass, params, max_seeds_per_shard=(n + n_shards - 1) // n_shards)
        rg.sweep(0, n, k=64, stats=False)
        t0 = time.perf_counter()
        for _ in range(args.random_steps):
            _, tk = rg.sweep(0, n, k=64, stats=False)
        el = time.perf_counter() - t0
        rg.close()
        sec.append(dict(metric="random-policy fault-sweep decisions/s", value=n * 10_000 * args.random_steps / el,
                        unit="decisions/s", n_gpus=n_dev, steps=args.random_steps,
                        ms_per_step=el / args.random_steps * 1e3, scaling="strong",
                        config={"workload": "configs[3] random fault sweep through a device group (C ABI)",
                                "schedules": n, "events": 10_000, "shards": n_shards},
                        topk_head=[[int(x["seed"]), int(x["n_fault"]), int(x["sum_delay_ns"])] for x in tk[:4]]))
    if "ed_clustered" in args.legs:
        N = args.ed_traces
        ts = synth.clustered_traces(N, 2048, family=1024)
        t0 = time.perf_counter()
        ep = G.EdGroupPlan(g, ts, 32)
        eplan_ms = (time.perf_counter() - t0) * 1e3
        eplan_parts = ep.timing()  # per local device: 1/N share upload, RCCL all_gather, device plan build
        ep.knn(8)
        t0 = time.perf_counter()
        for _ in range(args.ed_steps):
            ids, ds = ep.knn(8)
        el = time.perf_counter() - t0
        ep.close()
        pairs = N * (N - 1) // 2
        sec.append(dict(metric="trace-pair edit distances/s (banded, all-pairs k-NN)", value=pairs * args.ed_steps / el,
                        unit="pairs/s", n_gpus=n_dev, steps=args.ed_steps, ms_per_step=el / args.ed_steps * 1e3,
                        scaling="strong", plan_ms=eplan_ms, plan_upload_ms=eplan_parts["upload_ms"],
                        plan_gather_ms=eplan_parts["gather_ms"], plan_build_ms=eplan_parts["build_ms"],
                        plan_note="the store reaches each device as a 1/N share + one RCCL all_gather, then the plan "
                                  "is built from device memory (nmz_ed_group_plan_create); times per local device",
                        config={"workload": "configs[2] clustered all-pairs search through a device group (C ABI)",
                                "traces": N, "events": 2048, "band": 32, "k": 8, "shards": n_shards},
                        what="per step: nmz_ed_group_allpairs_knn -- shards, per-rank merge, RCCL all_gather, merge, "
                             "fill, ids and distances to the host"))
    line["secondary"] = sec
    g.close()
    return line


def write_final(out_fd, line, path):
    """The full record (every leg, every field) to `path`, then the compact headline as the last stdout line."""
    if path:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            with open(path, "w") as f:
                json.dump(line, f, indent=1)
            line = dict(line, full_record=os.path.relpath(os.path.abspath(path), HERE))
        except OSError as e:
            print(f"bench: could not write {path}: {e}", file=sys.stderr)
    os.write(out_fd, (headline_record(line) + "\n").encode())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # the driver's settings (python bench.py --steps 20 --warmup 5): a run with no flags measures what it measures
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--seeds", type=int, default=1 << 20)
    ap.add_argument("--events", type=int, default=4096)
    ap.add_argument("--cpu-seeds", type=int, default=1 << 18)
    ap.add_argument("--random-total", type=int, default=10_000_000)
    ap.add_argument("--random-steps", type=int, default=3)
    ap.add_argument("--cpu-random-seeds", type=int, default=256)
    ap.add_argument("--e2e-traces", type=int, default=64)
    ap.add_argument("--ed-traces", type=int, default=100_000)
    ap.add_argument("--ed-steps", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", dest="cpu_baseline", action="store_false")
    ap.add_argument("--no-secondary", dest="secondary", action="store_false")
    ap.add_argument("--full-record", default=os.path.join("gpurun_out", "bench_full.json"),
                    help="file for the full JSON record (every leg); '' to skip. stdout's last line is the compact "
                         "headline")
    ap.add_argument("--vis-traces", type=int, default=100_000)
    ap.add_argument("--vis-cpu-traces", type=int, default=1000)
    ap.add_argument("--group", action="store_true",
                    help="run the legs through one nmz_open_group over devices 0..N-1 in this process (C ABI "
                         "multi-GPU path) instead of one process per GPU")
    ap.add_argument("--group-shards", type=int, default=0, help="shards of the --group run (0: one per device)")
    ap.add_argument("--legs", default="replayable,random,ed_clustered,ed_survey,ed_alphabet,ed_wide,replayable_cliffs,"
                                      "visualize,config0",
                    help="comma list of legs to run (profiling runs one leg at a time); the headline line "
                         "needs 'replayable'")
    args = ap.parse_args()
    args.legs = set(args.legs.split(","))
    # The JSON lines are the only output on stdout (one per secondary leg, then the compact headline last):
    # whatever the libraries write to fd 1 during the run
    # (gloo's connection messages, HIP/RCCL diagnostics) goes to stderr instead.
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)

    import torch
    if args.group:
        line = bench_group(args, torch)
        write_final(out_fd, line, args.full_record)
        return
    D = Dist()
    torch.cuda.set_device(D.local_rank)
    D.init(torch)
    from namazu_amd import _lib
    L = _lib.load()
    ctx = _lib.Context(D.local_rank)
    # a real stream for the library calls and torch's own work (copies, RCCL collectives): the default stream's
    # handle is NULL, which the C ABI reads as "the context's own stream" (a non-blocking stream that torch's
    # default stream does not wait for)
    torch.cuda.set_stream(torch.cuda.Stream(torch.device("cuda", D.local_rank)))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert stream.value, "the bench's stream must not be the NULL stream"

    line = {}
    if "replayable" in args.legs:
        line = headline_line(args, torch, D, ctx, L, stream)
    if args.secondary:
        ed3 = dict(workload="configs[2] historystorage all-pairs search, clustered (families of 1,024 "
                            "near-duplicate runs)", traces=args.ed_traces, events=2048, band=32, k=8,
                   generator="clustered_traces", gen_kwargs=dict(family=1024), steps=args.ed_steps,
                   valu_key="k_ed_bv:clustered")
        ed3s = dict(workload="configs[2] historystorage all-pairs search, survey generator (independent "
                             "mutations: every pair beyond the band)", traces=args.ed_traces, events=2048, band=32,
                    k=8, generator="synth_traces", steps=args.ed_steps, valu_key="k_ed_bv:survey")
        ed3a = dict(workload="configs[2] historystorage all-pairs search, clustered, store-wide alphabet of "
                             "thousands of events (each family of 1,024 runs records its own 40 event maps out of "
                             "20,000): compact bit-parallel tables", traces=args.ed_traces, events=2048, band=32, k=8,
                    generator="clustered_traces",
                    gen_kwargs=dict(family=1024, n_symbols=40, alphabet_total=20_000), steps=args.ed_steps,
                    valu_key="k_ed_bv:alphabet")
        ed5 = dict(workload="configs[4] long-trace stress, wide band", traces=256, events=65536, band=4096, k=8,
                   generator="etcd_traces", steps=args.ed_steps, valu_key="k_ed_wide")
        sec = []

        def add(name, leg):  # each leg on its own stdout line as it finishes (never the last line)
            leg = dict(leg, leg=name)
            sec.append(leg)
            if D.rank == 0:
                os.write(out_fd, (json.dumps({"secondary_leg": leg}) + "\n").encode())
        if "random" in args.legs:
            add("random", bench_random_fault_sweep(args, torch, D, ctx, L, stream))
        for leg, spec in (("ed_clustered", ed3), ("ed_survey", ed3s), ("ed_alphabet", ed3a), ("ed_wide", ed5)):
            if leg in args.legs:
                add(leg, bench_ed_secondary(args, torch, D, ctx, L, stream, spec))
        if "replayable_cliffs" in args.legs and D.rank == 0:
            add("replayable_cliffs", bench_replayable_cliffs(args, torch, D, ctx, L, stream))
        if "visualize" in args.legs and D.rank == 0:
            add("visualize", bench_visualize(args, torch, D, ctx, L, stream))
        if "config0" in args.legs and D.rank == 0 and D.world == 1 and args.cpu_baseline:
            add("config0", bench_config0(args, torch, D, ctx, L))
        line["secondary"] = sec
    if D.rank == 0:
        write_final(out_fd, line, args.full_record)
    ctx.close()
    if D.pg:
        D.pg.destroy_process_group()


if __name__ == "__main__":
    main()
