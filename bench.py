#!/usr/bin/env python3
"""Benchmark of the MI355X batched workflow-history replay engine.

Metric (BASELINE.json): history events replayed/s and workflows rebuilt/s per node,
as a fraction of the HBM roofline.  Workload (configs[1]): 1M activity-heavy
workflows x 203 events, synthetic, NDC builder, on each GPU
(weak scaling: N GPUs replay N x 1M workflows, sharded by historyShardID =
Fingerprint32(workflowID) % 16384 and assigned shard->GPU greedily).

One "step" = one replay of the whole device-resident batch: the replay kernels of the
batch's slice classes (C2: k_replay_fast; C3-C5: k_replay_cls and its k_replay_reg retry
passes, the PAR slices, the general kernel for what fits no other) + k_tables + k_finalize.
Inputs are uploaded before the timed region; host SoA packing and H2D time are
reported separately.  The CPU baseline is the CPU restatement (oracle/) run with one
task per workflow on the host's cores over a bounded sample.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--wfs M] [--config C]
       (N>1: torchrun --nproc-per-node N bench.py --gpus N ...)
Other lines: --long-stride 125000 (configs[3]: histories at the 204,800-event count limit
mixed in), --tasks (with the stateBuilder task lists), --carry (replay onto a loaded
state), --ndc-forks (configs[4]'s conflict-resolution rounds).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from cadence_amd import abi  # noqa: E402

NUM_SHARDS = 16384
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

from cadence_amd.synth import DeviceBatch, RESULT_DTYPE, ROW_BYTES  # noqa: E402


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def workflow_weights(config: int, total_wfs: int, seed: int, long_stride: int = 0) -> np.ndarray:
    """Planned event count of every workflow of the population (synth.cpp plan_one),
    drawn without generating the histories: the shard->GPU assignment's weights."""
    L = abi.lib()
    p = abi.CdrSynthParams(config=config, n_wfs=0, seed=seed, long_stride=long_stride)
    w = np.zeros(total_wfs, np.uint32)
    rc = L.cdr_synth_weights(C.byref(p), total_wfs, w.ctypes.data)
    if rc:
        raise RuntimeError(f"cdr_synth_weights rc={rc}")
    return w


BIG_HISTORY = 100_000  # shards holding a >=100k-event history are spread first


def assign_shards(total_wfs: int, world: int, rank: int, lengths=None):
    """workflow ids "wf-<i>" -> historyShardID (Fingerprint32 % 16384, common/util.go:249-252)
    -> GPU: greedy largest-first (LPT) on the shards' event counts, shards that hold a
    >=100k-event history dealt first.  Returns (my workflow indices,
    per-GPU event load)."""
    L = abi.lib()
    shard = np.empty(total_wfs, np.int32)
    L.cdr_synth_shards(total_wfs, NUM_SHARDS, shard.ctypes.data)
    lengths = np.ones(total_wfs) if lengths is None else np.asarray(lengths, np.float64)
    w = np.bincount(shard, weights=lengths, minlength=NUM_SHARDS)
    big = np.bincount(shard, weights=(lengths >= BIG_HISTORY).astype(np.float64), minlength=NUM_SHARDS) > 0
    owner = np.zeros(NUM_SHARDS, np.int32)
    load = np.zeros(world)
    for s in np.lexsort((-w, ~big)):  # big-history shards first, then by events, descending
        g = int(np.argmin(load))
        owner[s] = g
        load[g] += w[s]
    mine = np.nonzero(owner[shard] == rank)[0].astype(np.uint32)
    return mine, load


def _np_dtype(ty, names):
    fmt = {C.c_uint32: "<u4", C.c_int32: "<i4", C.c_uint64: "<u8", C.c_int64: "<i8"}
    types = dict(ty._fields_)
    return np.dtype({"names": list(names), "formats": [fmt[types[n]] for n in names],
                     "offsets": [getattr(ty, n).offset for n in names], "itemsize": C.sizeof(ty)})


def refresh_measure(torch, L, ctx, db, stream, steps):
    """refreshTasks (refresh.hip, cdr_refresh_tasks_async) over the rebuilt states of the
    timed replay: K launches timed with HIP events on the launch stream, after the
    headline's timed region (it is not part of `value`).  Task slices per entry: the
    refresher's bound (3 + pending activity / child / cancel / signal capacities transfer
    tasks, 6 timer tasks)."""
    n = db.info.n_entries
    # a byte copy viewed through the partial dtype: the table offsets between the named
    # fields must survive (a structured copy would not keep the gaps)
    raw = np.frombuffer(db.h_caps, np.uint8).copy()
    caps = raw.view(_np_dtype(abi.CdrWfCaps, (
        "act_cap", "child_cap", "cancel_cap", "signal_cap", "xfer_off", "ttask_off", "xfer_cap", "ttask_cap")))
    xcap = 3 + caps["act_cap"].astype(np.uint64) + caps["child_cap"] + caps["cancel_cap"] + caps["signal_cap"]
    caps["xfer_cap"] = xcap.astype(np.uint32)
    caps["ttask_cap"] = 6
    caps["xfer_off"] = np.concatenate([[0], np.cumsum(xcap)[:-1]]).astype(np.uint64)
    caps["ttask_off"] = np.arange(n, dtype=np.uint64) * 6
    dev = torch.device("cuda", torch.cuda.current_device())
    caps_t = torch.from_numpy(raw).to(dev)
    dbr = abi.CdrDevBatch.from_buffer_copy(db.db)
    dbr.caps = caps_t.data_ptr()
    xt = torch.zeros(int(xcap.sum()) * C.sizeof(abi.CdrTask), dtype=torch.uint8, device=dev)
    tt = torch.zeros(n * 6 * C.sizeof(abi.CdrTask), dtype=torch.uint8, device=dev)
    nt = torch.zeros(2 * n, dtype=torch.int32, device=dev)
    out = abi.CdrOut.from_buffer_copy(db.out)
    out.transfer, out.timer_tasks, out.n_tasks = xt.data_ptr(), tt.data_ptr(), nt.data_ptr()
    now = int(db.meta.now_ns)

    def launch():
        rc = L.cdr_refresh_tasks_async(ctx, C.byref(dbr), C.byref(out), now, abi.REFRESH_ADVANCED_VISIBILITY,
                                       C.c_void_p(stream))
        if rc:
            raise RuntimeError(f"cdr_refresh_tasks_async rc={rc}")

    launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    counts = nt.view(-1, 2).sum(dim=0).tolist()
    res = np.frombuffer(db.results(), dtype=RESULT_DTYPE)
    ok = res["code"] == 0
    rows = sum(int(res[f][ok].sum()) * b for f, b in ROW_BYTES.items() if f in (
        "n_activity", "n_timer", "n_child", "n_cancel", "n_signal"))
    # per entry: lane_wf, result, caps, desc, ExecutionInfo, the start event's columns and
    # attribute words, the closing event's type/version, n_tasks; + pending rows + tasks
    per_entry = 4 + C.sizeof(abi.CdrWfResult) + C.sizeof(abi.CdrWfCaps) + C.sizeof(abi.CdrWfDesc) + 256 + 44 + 12 + 8
    alg = n * per_entry + rows + (counts[0] + counts[1]) * C.sizeof(abi.CdrTask)
    return {"kernel": "k_refresh", "kernel_ms": ms, "entries": n, "ok_entries": int(ok.sum()),
            "transfer_tasks": int(counts[0]), "timer_tasks": int(counts[1]),
            "entries_per_s": n / (ms / 1e3), "algorithmic_bytes_per_launch": alg,
            "achieved_gbs": alg / (ms / 1e3) / 1e9, "frac": alg / (ms / 1e3) / 1e9 / PEAK_HBM_GBS}


def encode_measure(torch, L, ctx, db, stream, steps):
    """SQL row blobs (encode.hip, cdr_encode_rows_async) of the pending TimerInfo and
    RequestCancelInfo rows of the replayed states: K launches per table timed with HIP
    events on the launch stream, outside the headline's timed region.  Algorithmic
    bytes per row: the record read (40 B) + the blob slot written (48 / 80 B)."""
    res = np.frombuffer(db.results(), dtype=RESULT_DTYPE)
    ok = res["code"] == 0
    out = {}
    for name, tid, size, stride, cnt, tot in (("timer", 1, 45, 48, "n_timer", db.info.totals.timer),
                                              ("cancel", 3, 66, 80, "n_cancel", db.info.totals.cancel)):
        rows = int(res[cnt][ok].sum())
        if rows == 0:  # (C1/C2 hold no such rows: an empty launch would report 0 of the roofline)
            out[name] = {"kernel": "k_encode_rows", "rows": 0, "note": "no rows of this table in the workload: not launched"}
            continue
        blobs = torch.empty(max(16, tot * stride), dtype=torch.uint8, device="cuda")

        def launch():
            rc = L.cdr_encode_rows_async(ctx, tid, C.byref(db.db), C.byref(db.out),
                                         C.c_void_p(blobs.data_ptr()), C.c_void_p(stream))
            if rc:
                raise RuntimeError(f"cdr_encode_rows_async rc={rc}")
        launch()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            launch()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / steps
        alg = rows * (40 + stride)
        out[name] = {"kernel": "k_encode_rows", "kernel_ms": ms, "rows": rows, "rows_per_s": rows / (ms / 1e3),
                     "algorithmic_bytes_per_launch": alg, "achieved_gbs": alg / (ms / 1e3) / 1e9,
                     "frac": alg / (ms / 1e3) / 1e9 / PEAK_HBM_GBS}
        del blobs
    return out


def stream_peak_gbs(torch, nbytes=4 << 30, reps=10):
    """Read + write bandwidth of libcdr's float4 copy kernel (cdr_stream_copy_async, the
    MI355X guide's ~6.3 TB/s recipe), timed with HIP events on the stream it runs on: the
    achievable ceiling beside the 8 TB/s spec peak."""
    L = abi.lib()
    a = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    st = torch.cuda.current_stream()
    run = lambda: L.cdr_stream_copy_async(C.c_void_p(b.data_ptr()), C.c_void_p(a.data_ptr()),
                                          C.c_uint64(nbytes), C.c_void_p(st.cuda_stream))
    if run():
        raise RuntimeError("cdr_stream_copy_async failed")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        run()
    e1.record(st)
    torch.cuda.synchronize()
    dt = e0.elapsed_time(e1) / 1e3 / reps
    del a, b
    return 2 * nbytes / dt / 1e9


def host_cores() -> tuple:
    """(cores this process may run on, how that was found): the CPU affinity mask,
    bounded by the cgroup's CPU quota (cgroup v2 cpu.max, v1 cfs_quota_us / period) when
    one is set; CDR_CPU_THREADS overrides."""
    if os.environ.get("CDR_CPU_THREADS"):
        return max(1, int(os.environ["CDR_CPU_THREADS"])), "CDR_CPU_THREADS"
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    how = f"sched_getaffinity={n}"
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None:
        how += f", cgroup quota {quota:g} CPUs"
        n = max(1, min(n, int(quota)))
    else:
        how += ", no cgroup quota"
    return n, how


def cpu_baseline(config, n_wfs, seed, min_seconds=10.0):
    """CPU restatement (oracle/) on the box's host cores, one task per workflow (the
    analogue of the reference's goroutine-per-workflow), over a bounded sample."""
    import oracle
    from cadence_amd import engine
    b = engine.synth_batch(config, n_wfs, seed)
    pl = engine.plan(b)
    n_ev = len(b.events)
    threads, cores_how = host_cores()
    res = {}
    for th in (threads, 1):
        reps, t0 = 0, time.perf_counter()
        while True:
            oracle.replay(b, pl, threads=th)
            reps += 1
            el = time.perf_counter() - t0
            if el >= (min_seconds if th == threads else min_seconds / 4) or reps >= 200:
                break
        res[th] = n_ev * reps / el
    # refreshTasks on the same sample (oracle/refresh_ref.cpp, one thread), beside k_refresh
    out = oracle.replay(b, pl, threads=threads)
    out.alloc_tasks(pl)
    bs, cs = b.cstruct(), out.cstruct()
    reps, t0 = 0, time.perf_counter()
    while True:
        oracle.lib().cdro_refresh_tasks(C.byref(bs), pl.caps, C.byref(cs), bs.now_ns, 1)
        reps += 1
        if time.perf_counter() - t0 >= min_seconds / 4 or reps >= 1000:
            break
    refresh_eps = b.n_wfs * reps / (time.perf_counter() - t0)
    return {"value": res[threads], "unit": "events/s", "cores": threads, "cores_source": cores_how, "kind": "port",
            "refresh_entries_per_s_1thread": refresh_eps,
            "sample": f"config {config}: {n_wfs} workflows x {n_ev // max(1, n_wfs)} events, replayed "
                      f"{'repeatedly'} for >= {min_seconds:.0f} s; single-thread {res[1]:.4g} events/s; "
                      f"the Go stateBuilder cannot run here (no Go toolchain)",
            "single_thread_events_per_s": res[1], "workflows_per_s": res[threads] / (n_ev / max(1, n_wfs))}


def init_dist(torch):
    """One process per GPU (torch.distributed.run's env): (dist or None, world, rank, local
    rank, the device the counters reduce on).  RCCL (backend "nccl") between the GPUs of the
    node; CDR_BENCH_BACKEND=gloo rehearses the multi-rank path on a box with fewer GPUs than
    ranks (ranks share a device, the counters reduce on the host; the timings then mean
    nothing)."""
    world, rank, local = dist_env()
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("CDR_BENCH_BACKEND", "nccl")
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()) if backend == "gloo" else local)
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return dist, world, rank, local, "cpu" if backend == "gloo" else "cuda"
    torch.cuda.set_device(0)
    return None, 1, 0, 0, "cuda"


def finish_dist(dist):
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def reduce_step(dist, torch, stats, elapsed: float):
    """The multi-GPU step's only collective: the sum over ranks of the
    int64 counters [events, entries, OK entries, cdr_checksum_async digest sum] (the
    digest sum wraps mod 2^64, so the all-reduced value is the single-process sum) and
    the max over ranks of the timed region.  `stats` is a 4-element int64 tensor on the
    collective's device (cuda for RCCL, cpu for the gloo tests)."""
    t_el = torch.tensor([elapsed], dtype=torch.float64, device=stats.device)
    if dist:
        dist.all_reduce(stats)
        dist.all_reduce(t_el, op=dist.ReduceOp.MAX)
    return [int(x) for x in stats.tolist()], float(t_el.item())


def lib_sha1() -> str:
    import hashlib
    return hashlib.sha1(open(abi.LIB_PATH, "rb").read()).hexdigest()


def load_traffic(workload):
    """PMC HBM bytes per launch (tools/pmc.sh + tools/traffic.py) for this workload, used
    only when they were collected on this very build of libcdr.so (same SHA-1); else
    (None, reason)."""
    try:
        d = json.load(open(os.path.join(HERE, "profiles", f"traffic_{workload}.json")))
    except (OSError, ValueError):
        return None, "no PMC summary for this workload"
    if d.get("workload") != workload:
        return None, "no PMC summary for this workload"
    if d.get("lib_sha1") != lib_sha1():
        return None, "stale: PMC summary from another build of libcdr.so"
    return d, None


def parity_check(db, ctx, stream, config, mine, seed, long_stride=0):
    """Full-size parity: every entry's output digest on the GPU (k_digest) against the
    CPU restatement's (oracle/, restated hash in digest_ref.cpp) over the same
    population, entry by entry.  Runs after the timed region."""
    import oracle
    t0 = time.perf_counter()
    got, got_sum = db.digests(ctx, stream)
    threads = host_cores()[0]
    want, want_sum, hist = oracle.synth_digests(config, mine, seed, threads=threads, long_stride=long_stride)
    bad = np.nonzero(got != want)[0] if len(got) == len(want) else np.arange(max(len(got), len(want)))
    return {"checked": True, "entries": int(len(want)), "mismatched_entries": int(len(bad)),
            "first_mismatches": bad[:8].tolist(), "gpu_checksum": got_sum, "oracle_checksum": want_sum,
            "oracle_status": hist, "cpu_threads": threads, "seconds": time.perf_counter() - t0,
            "method": "per-entry digest of the persisted projection (cdr_entry_digests_async vs "
                      "oracle/digest_ref.cpp), CopyToPersistence mutableStateBuilder.go:257-270"}


def compare_task_lists(got, nt, caps_g, ref, caps_r, ne):
    """Entries (of the first ne) whose transfer / timer task lists differ, byte for byte:
    got = {"xfer", "ttask"} device buffers as bytes, nt = their [n_xfer, n_timer] per entry,
    caps_g / caps_r the two plans' task offsets, ref the oracle's Outputs(tasks=True).
    Returns (mismatched entries, the oracle's task count)."""
    sz = C.sizeof(abi.CdrTask)
    want = {k: bytes(ref.tasks[k]) for k in ("xfer", "ttask")}
    bad, n_tasks = [], 0
    for w in range(ne):
        for k, kind, off_g, off_r in ((0, "xfer", caps_g[w].xfer_off, caps_r[w].xfer_off),
                                      (1, "ttask", caps_g[w].ttask_off, caps_r[w].ttask_off)):
            n_r = int(ref.tasks["n"][2 * w + k])
            n_tasks += n_r
            g = got[kind][int(off_g) * sz:(int(off_g) + int(nt[w, k])) * sz]
            r = want[kind][int(off_r) * sz:(int(off_r) + n_r) * sz]
            if g != r:
                bad.append(w)
                break
    return bad, n_tasks


def task_parity(db, config, mine, seed, long_stride=0, sample=20000):
    """The --tasks line's task lists (cdr_out.transfer / timer_tasks) against the oracle's
    (oracle.replay(tasks=True), stateBuilder.go:613-804) for the entries of the first
    `sample` workflows of this rank's population, entry by entry and byte for byte (the
    per-entry state digests of parity_check do not cover the task lists).  Runs after the
    timed region."""
    import oracle
    from cadence_amd import engine
    t0 = time.perf_counter()
    m = min(len(mine), sample)
    sb = engine.synth_batch(config, m, seed, index_map=np.asarray(mine[:m], np.uint32), long_stride=long_stride)
    pl = engine.plan(sb)
    ref = oracle.replay(sb, pl, threads=host_cores()[0], tasks=True)
    ne = sb.n_wfs  # the DeviceBatch's first ne entries are these workflows' (natural order)
    sz = C.sizeof(abi.CdrTask)
    nt = db.out_t["n_tasks"][: 8 * ne].view(db.torch.int32).cpu().numpy().reshape(-1, 2)
    caps = db.h_caps
    hi_x = int(caps[ne - 1].xfer_off) + int(nt[ne - 1, 0]) if ne else 0
    hi_t = int(caps[ne - 1].ttask_off) + int(nt[ne - 1, 1]) if ne else 0
    got = {"xfer": db.out_t["transfer"][: hi_x * sz].cpu().numpy().tobytes(),
           "ttask": db.out_t["timer_tasks"][: hi_t * sz].cpu().numpy().tobytes()}
    bad, n_tasks = compare_task_lists(got, nt, caps, ref, pl.caps, ne)
    return {"checked": True, "sample_workflows": m, "entries": ne, "tasks": n_tasks,
            "mismatched_entries": len(bad), "first_mismatches": bad[:8], "seconds": time.perf_counter() - t0,
            "method": "byte-for-byte task lists (transfer + timer) of the first sample workflows' entries, GPU vs "
                      "oracle.replay(tasks=True)"}


def host_path_measure(config, seed, n_sample, ctx_dev, long_stride=0):
    """What a caller holding DECODED histories (cdr_event records, the Go side's
    []*HistoryEvent after thriftrw decode) sees through the drop-in boundary: the same
    population's first n_sample workflows as a host batch, (a) the host planner + packer
    stages alone (cdr_plan_caps, cdr_plan_slices_ex, cdr_pack_slices on the host's cores,
    into a page-locked slab), and (b) the whole cdr_replay_batch call (plan + pack + H2D +
    replay + D2H of every record), warm (the context's staging and workspace already
    sized).  The headline's timed step excludes all of this (device-resident input)."""
    from cadence_amd import engine
    L = abi.lib()
    b = engine.synth_batch(config, n_sample, seed, long_stride=long_stride)
    n_ev = len(b.events)
    threads = host_cores()[0]
    import torch
    res = {}
    for rep in range(2):  # the second pass is the warm one
        t0 = time.perf_counter()
        pl = engine.plan(b)
        t1 = time.perf_counter()
        ns, rows, nw = C.c_uint32(), C.c_uint64(), C.c_uint32()
        mode = abi.PLAN_WAVE | abi.PLAN_PAR
        L.cdr_plan_slices_ex(b.wfs, pl.caps, b.n_wfs, mode, None, None, None, None, C.byref(ns), C.byref(rows),
                             C.byref(nw))
        lane = np.zeros(ns.value * 64, np.int32)
        slen = np.zeros(ns.value, np.uint32)
        row0 = np.zeros(ns.value, np.uint64)
        fl = np.zeros(ns.value, np.uint32)
        L.cdr_plan_slices_ex(b.wfs, pl.caps, b.n_wfs, mode, lane.ctypes.data, slen.ctypes.data, row0.ctypes.data,
                             fl.ctypes.data, C.byref(ns), C.byref(rows), C.byref(nw))
        t2 = time.perf_counter()
        bs = b.cstruct()
        aw = L.cdr_plan_arena_words(C.byref(bs))
        if rep == 0:
            slab_t = torch.empty(int(rows.value) * 64 * abi.EL_BYTES, dtype=torch.uint8, pin_memory=True)
            arena_t = torch.empty(max(1, aw) * 8, dtype=torch.uint8, pin_memory=True)
        s = abi.CdrSlices(n_slices=ns.value, n_rows=rows.value, arena_words=aw)
        s.slice_row0, s.slice_len, s.lane_wf = row0.ctypes.data, slen.ctypes.data, lane.ctypes.data
        s.slab, s.arena, s.slice_flags = slab_t.data_ptr(), arena_t.data_ptr(), fl.ctypes.data
        t3 = time.perf_counter()
        if L.cdr_pack_slices(C.byref(bs), C.byref(s), threads):
            raise RuntimeError("cdr_pack_slices failed")
        t4 = time.perf_counter()
        dev = slab_t.to("cuda", non_blocking=True)
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        del dev
        res = {"plan_caps_s": t1 - t0, "plan_slices_s": t2 - t1, "pack_s": t4 - t3, "h2d_s": t5 - t4,
               "h2d_gbs": slab_t.numel() / max(t5 - t4, 1e-9) / 1e9}
    host_s = res["plan_caps_s"] + res["plan_slices_s"] + res["pack_s"]
    res.update({"events": n_ev, "workflows": n_sample, "threads": threads,
                "host_planner_packer_events_per_s": n_ev / host_s,
                "host_planner_packer_h2d_events_per_s": n_ev / (host_s + res["h2d_s"])})
    # the whole drop-in call, warm
    eng = engine.Engine(torch.cuda.current_device())
    try:
        eng.replay(b)
        t0 = time.perf_counter()
        eng.replay(b)
        res["replay_batch_s"] = time.perf_counter() - t0
    finally:
        eng.close()
    res["replay_batch_events_per_s"] = n_ev / res["replay_batch_s"]
    res["method"] = ("cdr_plan_caps + cdr_plan_slices_ex + cdr_pack_slices (host threads) into a pinned slab + its H2D; "
                     "and one warm cdr_replay_batch call (plan + pack + H2D + replay + D2H) on the same sample")
    return res


def canonical_event_bytes(batch) -> np.ndarray:
    """SURVEY 8(d) canonical input bytes of every entry of a host batch: sum over its events
    of 48 B core + A[type]."""
    from cadence_amd.synth import A_TYPE
    words = C.sizeof(abi.CdrEvent) // 4
    n = batch.n_wfs
    if not len(batch.events):
        return np.zeros(n, np.int64)
    ty = np.frombuffer(batch.events, dtype=np.uint32).reshape(-1, words)[:, abi.CdrEvent.type.offset // 4]
    cum = np.concatenate([[0], np.cumsum(48 + A_TYPE[np.minimum(ty, 255)])])
    wf = np.frombuffer(batch.wfs, dtype=np.uint8).reshape(n, C.sizeof(abi.CdrWfDesc))

    def col(name):
        o = getattr(abi.CdrWfDesc, name).offset
        return wf[:, o:o + 8].copy().view(np.uint64).ravel().astype(np.int64)
    off, ln = col("ev_off"), col("ev_len")
    return cum[off + ln] - cum[off]


def carry_cpu_baseline(cfg, n_sample, seed, min_seconds=10.0):
    """The carry line's CPU leg: oracle.replay of the second halves onto the first halves'
    loaded states (the restated mutableStateBuilder.Load + applyEvents, mutableStateBuilder.go:
    272-295, stateBuilder.go:112-611) on the box's host cores, over a sample split the way the
    GPU line splits its population (engine.split_half); events counted as the GPU line counts
    them (the suffixes')."""
    import oracle
    from cadence_amd import engine
    b = engine.synth_batch(cfg, n_sample, seed)
    cut = engine.split_half(b)
    pre, _ = engine.cut_batches(b, cut)
    th, how = host_cores()
    pre_out = oracle.replay(pre, engine.plan(pre), threads=th)
    suf = engine.suffix_batch(b, cut, pre, pre_out)
    spl = engine.plan(suf)
    n_ev = int(sum(int(suf.wfs[w].ev_len) for w in range(suf.n_wfs)))
    res = {}
    for t in (th, 1):
        reps, t0 = 0, time.perf_counter()
        while True:
            oracle.replay(suf, spl, threads=t)
            reps += 1
            el = time.perf_counter() - t0
            if el >= (min_seconds if t == th else min_seconds / 4) or reps >= 200:
                break
        res[t] = n_ev * reps / el
    return {"value": res[th], "unit": "events/s", "cores": th, "cores_source": how, "kind": "port",
            "single_thread_events_per_s": res[1],
            "sample": f"config {cfg}: {n_sample} workflows split at the call nearest their middle; the "
                      f"second halves ({n_ev} events) replayed onto the first halves' oracle states, "
                      f"repeatedly for >= {min_seconds:.0f} s"}


def ndc_cpu_baseline(n_sample, seed, min_seconds=10.0):
    """configs[4]'s CPU leg: oracle.ndc_replicate (the restated stateRebuilder /
    conflict-resolution rounds, nDCConflictResolver.go:117-184, nDCStateRebuilder.go:92-160)
    on the box's host cores over a sample of the same forked population; events counted as
    the GPU line counts them (base + every rebuilt branch + every applied task)."""
    import oracle
    from cadence_amd import ndc
    base, rebuild, forks = ndc.synth_forked(5, n_sample, seed)
    threads, how = host_cores()
    reps, t0 = 0, time.perf_counter()
    while True:
        _, _, _, decs, rounds = oracle.ndc_replicate(base, rebuild, forks, threads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= min_seconds or reps >= 50:
            break
    ev = ndc_counts(base, rebuild, forks, rounds, decs)[0]
    return {"value": ev * reps / el, "unit": "events/s", "cores": threads, "cores_source": how, "kind": "port",
            "sample": f"forked config 5: {n_sample} workflows (base + 2 fork rounds), oracle.ndc_replicate repeated "
                      f"for >= {min_seconds:.0f} s; the Go stateRebuilder cannot run here (no Go toolchain)",
            "workflows_per_s": n_sample * reps / el}


def ndc_counts(base, rebuild, forks, rounds, decs):
    """What one replication run of a (shard of the) forked population replays: (events,
    base events, events per round, decision counts per round, SURVEY 8(d) canonical event
    bytes).  A round replays the rebuilt branch of every workflow whose rebuild ran and
    succeeded and the task's events of every workflow whose apply ran and succeeded (a SKIP /
    BACKFILL decision, a failed branch step or rebuild leaves the apply record CDR_NOT_RUN or
    failed: none of its events is counted).  `rounds` / `decs` as DeviceReplicator.run (or
    oracle.ndc_replicate) return them."""
    n = base.n_wfs

    def codes(out):
        return np.frombuffer(out.result, dtype=np.int32).reshape(-1, C.sizeof(abi.CdrWfResult) // 4)[:n, 0]
    ev_base = int(sum(base.wfs[w].ev_len for w in range(n)))
    lens_rb = np.array([rebuild.wfs[w].ev_len for w in range(n)], np.int64)
    cb_rb = canonical_event_bytes(rebuild)
    ev_bytes = int(canonical_event_bytes(base).sum())
    ev_rounds, acts = [], {}
    for k, (fb, _, _) in enumerate(forks):
        rb_out, ap_out = rounds[k]
        ok_ap, ok_rb = codes(ap_out) == abi.OK, codes(rb_out) == abi.OK
        lens_fb = np.array([fb.wfs[w].ev_len for w in range(n)], np.int64)
        ev_rounds.append(int(lens_fb[ok_ap].sum() + lens_rb[ok_rb].sum()))
        ev_bytes += int(canonical_event_bytes(fb)[ok_ap].sum() + cb_rb[ok_rb].sum())
        acts[f"round{k}"] = {abi.NDC_ACTIONS[a]: int(c) for a, c in
                             zip(*np.unique([decs[k][w].action for w in range(n)], return_counts=True))}
    return ev_base + sum(ev_rounds), ev_base, ev_rounds, acts, ev_bytes


def ndc_forks_line(args):
    """configs[4]'s conflict-resolution path at scale: the forked config-5 population
    (cadence_amd.ndc.synth_forked: a base branch and two fork rounds per workflow,
    nDC_integration_test.go:224-308) replicated device-resident (cdr_ndc_replicate_async,
    nDCHistoryReplicator.go:330-398 -> nDCConflictResolver.go:117-184 -> nDCStateRebuilder.go:
    92-160).  A step = the base branch replayed into the state buffer + both rounds (branch,
    rebuild replay + refreshTasks + verify, apply onto the rebuilt state in memory or the loaded
    one, VersionHistories sync).  value = events replayed per second (base + rebuilt + applied
    events) over all ranks; parity: the final state, the VersionHistories and each round's
    decisions against oracle.ndc_replicate, entry by entry, on every rank.
    N > 1 (torch.distributed.run): each rank replicates the workflows of its historyShardIDs
    (Fingerprint32(workflowID) % 16384, greedy on events, as the headline line) — no
    data-path collective; one all-reduce of [events, workflows, OK states, state digest sum],
    the max of the timed region and the parity counts closes the run."""
    import torch
    from cadence_amd import engine, ndc
    dist, world, rank, local, coll_dev = init_dist(torch)
    eng = engine.Engine(torch.cuda.current_device())
    total = args.wfs * world
    mine, load = assign_shards(total, world, rank, workflow_weights(5, total, args.seed))
    n = len(mine)
    t0 = time.perf_counter()
    import threading
    beat = threading.Event()

    def heartbeat():  # long host phases at 1M workflows: a progress line every minute
        while not beat.wait(60):
            log(f"[rank {rank}] NDC forks: {time.perf_counter() - t0:.0f}s")
    threading.Thread(target=heartbeat, daemon=True).start()
    base, rebuild, forks = ndc.synth_forked(5, n, args.seed, index_map=mine)
    log(f"[rank {rank}] NDC forks: synthesized {n} of {total} forked workflows ({time.perf_counter() - t0:.0f}s)")
    rep = ndc.DeviceReplicator(eng, base, rebuild, forks)
    setup_s = time.perf_counter() - t0
    log(f"[rank {rank}] NDC forks: {n} workflows, host synth + plan + upload {setup_s:.1f}s")
    state, vhs, pool, decs, rounds = rep.run()  # warm-up (and the decisions the events count from)
    events, ev_base, ev_rounds, acts, ev_bytes = ndc_counts(base, rebuild, forks, rounds, decs)

    def step():
        rep.reset()
        rep.base_replay()
        for k in range(len(rep.rounds)):
            rep.round(k)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.steps):
        step()
    e1.record()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    dev_ms = e0.elapsed_time(e1) / args.steps
    # the final states' per-entry digests (k_digest over the state buffer) and their sum: the
    # product checksum the ranks reduce
    stream = torch.cuda.current_stream().cuda_stream
    per = torch.zeros(max(1, n), dtype=torch.int64, device="cuda")
    dsum = torch.zeros(1, dtype=torch.int64, device="cuda")
    rc = abi.lib().cdr_entry_digests_async(eng.ctx, C.byref(rep.base_db), C.byref(rep.state), C.c_void_p(per.data_ptr()),
                                           C.c_void_p(dsum.data_ptr()), C.c_void_p(stream))
    if rc:
        raise RuntimeError(f"cdr_entry_digests_async rc={rc}")
    torch.cuda.synchronize()
    ok = int((np.frombuffer(state.result, dtype=np.int32).reshape(-1, C.sizeof(abi.CdrWfResult) // 4)[:n, 0]
              == abi.OK).sum())
    stats = torch.tensor([events, n, ok, int(dsum.item())], dtype=torch.int64, device=coll_dev)
    (tot_events, tot_wfs, tot_ok, checksum), elapsed = reduce_step(dist, torch, stats, elapsed)
    parity = None
    if not args.no_parity:
        import oracle
        t1 = time.perf_counter()
        g_state, g_vhs, g_pool, g_decs, _ = rep.run()
        r_state, r_vhs, r_pool, r_decs, _ = oracle.ndc_replicate(base, rebuild, forks, threads=host_cores()[0])
        bad = engine.compare(base, g_state, r_state, limit=10 ** 9)
        bad_dec = sum(1 for k in range(len(forks)) for w in range(n)
                      if bytes(g_decs[k][w]) != bytes(r_decs[k][w]))
        vb = sum(1 for w in range(n) if ndc.branch_items(g_vhs, g_pool, w, g_vhs[w].current) !=
                 ndc.branch_items(r_vhs, r_pool, w, r_vhs[w].current) or g_vhs[w].n_branches != r_vhs[w].n_branches)
        bad_st = len({b.split(':')[0] for b in bad})
        flag = torch.tensor([bad_st, bad_dec, vb, n], dtype=torch.int64, device=coll_dev)
        if dist:
            dist.all_reduce(flag)
        bad_st, bad_dec, vb, n_all = [int(x) for x in flag.tolist()]
        parity = {"checked": True, "entries": n_all, "mismatched_entries": bad_st,
                  "mismatched_decisions": bad_dec, "mismatched_version_histories": vb,
                  "first_mismatches": bad[:4], "seconds": time.perf_counter() - t1, "ranks": world,
                  "method": "engine.compare of the final persisted state + each round's decisions + the current "
                            "branch's VersionHistory, GPU vs oracle.ndc_replicate, on every rank (counts summed)"}
        log(f"[rank {rank}] NDC parity (all ranks): {bad_st} states, {bad_dec} decisions, {vb} VHs differ "
            f"({parity['seconds']:.1f}s)")
    if rank != 0:
        beat.set()
        rep.close()
        finish_dist(dist)
        return
    ms = elapsed / args.steps * 1e3
    # algorithmic bytes per step, this rank's: every replayed event's 48 B +
    # A[type] (the base branch, each round's rebuilt branch and applied task, counted as
    # `events` is) + the per-workflow records each replay writes (264 B), base + 2 rounds x
    # (rebuild + apply); the roofline is one GPU's, on its own bytes and device time
    alg = ev_bytes + n * 264 * (1 + 2 * len(forks))
    workload = f"C5-forked-{args.wfs}wf-ndc-replicate"
    traffic, tnote = load_traffic(workload)
    line = {
        "metric": "history events replayed/sec + workflows rebuilt/sec (node), % of HBM roofline",
        "value": tot_events * args.steps / elapsed, "unit": "events/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms, "device_ms_per_step_rank0": dev_ms, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic forked config 5 (cadence_amd.ndc.synth_forked)",
        "config": {"workload": workload, "workflows_per_gpu": args.wfs, "rounds": len(forks),
                   "events_per_step": tot_events, "events_rank0": events, "events_base_rank0": ev_base,
                   "events_rounds_rank0": ev_rounds, "decisions_rank0": acts,
                   "sharding": f"Fingerprint32(workflowID) % {NUM_SHARDS} -> greedy shard->GPU",
                   "parallelism": f"shard{world}"},
        "workflows_per_s": tot_wfs * args.steps / elapsed,
        "roofline": {"bound": "hbm", "achieved": alg / (dev_ms / 1e3) / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": alg / (dev_ms / 1e3) / 1e9 / PEAK_HBM_GBS,
                     "traffic": traffic["bytes_per_launch"] if traffic else None,
                     "traffic_note": tnote or (traffic.get("source") + "; per step: every k_* kernel of the "
                                               "step (the VersionHistories reset copy excluded)"),
                     "algorithmic_bytes_per_step": alg,
                     "bytes_breakdown": {"events": ev_bytes, "records": alg - ev_bytes},
                     "kernel": "k_ndc_branch + k_replay* + k_refresh + k_ndc_verify/apply (one step)"},
        "host": {"setup_s": setup_s},
        "checksum": checksum & 0xFFFFFFFFFFFFFFFF, "ok_workflows": tot_ok,
        "cpu_baseline": None if (args.no_cpu_baseline or world > 1) else ndc_cpu_baseline(min(n, 20000), args.seed),
        "parity": parity, "parity_checked": parity is not None and parity["mismatched_entries"] == 0
        and parity["mismatched_decisions"] == 0 and parity["mismatched_version_histories"] == 0,
        "shard_load_events": load.tolist(),
    }
    beat.set()
    print(json.dumps(line), flush=True)
    rep.close()
    finish_dist(dist)


def carry_line(args):
    """Carry-in replay at full size (the north star's drop-in for every
    applyEvents caller, not just rebuild): every history of the config's population is cut at
    the call boundary nearest after its middle; the first half replays into a state buffer
    (k_replay_cls, untimed), then a step = the second half replayed onto those LOADED states
    (cdr_dev_batch.carry: mutableStateBuilder.Load mutableStateBuilder.go:272-295, then
    applyEvents, nDCHistoryReplicator.go:330-398) through the register-table kernels'
    carry-in instantiations.  value = suffix events per second.  Parity, entry by entry: the
    GPU's carried replay against the oracle's carried replay of the oracle's own prefix
    states, and against the oracle's WHOLE-history replay (split equals whole).
    N > 1 (torch.distributed.run): each rank takes the workflows of its historyShardIDs
    (Fingerprint32(workflowID) % 16384, greedy on events); one all-reduce of [events,
    workflows, OK entries, digest sum], the max of the timed region and the parity counts."""
    import torch
    from cadence_amd import engine, ndc
    dist, world, rank, local, coll_dev = init_dist(torch)
    eng = engine.Engine(torch.cuda.current_device())
    L = abi.lib()
    cfg = args.config
    seed = args.seed if args.seed != 0x5EED0002 else 0x5EED0000 + cfg
    total = args.wfs * world
    mine, load = assign_shards(total, world, rank, workflow_weights(cfg, total, seed))
    t0 = time.perf_counter()
    b = engine.synth_batch(cfg, len(mine), seed, index_map=mine)
    n_wf, n = len(mine), b.n_wfs  # entries: a continue-as-new run is an entry of its own (never split)
    cut = engine.split_half(b)
    pre, suf = engine.cut_batches(b, cut)
    log(f"[rank {rank}] carry: {n} C{cfg} entries of {n_wf} workflows, {int((cut > 0).sum())} split "
        f"({time.perf_counter() - t0:.0f}s)")
    dev = ndc._Dev()
    stream = torch.cuda.current_stream().cuda_stream
    # the first halves: replayed once into the state buffer the steps load from
    pre_pl = engine.plan(pre)
    pre_db = ndc.upload_batch(dev, pre, pre_pl.caps, cls=True)
    pre_out = ndc.alloc_out(dev, n, pre_pl.totals)
    rc = L.cdr_replay_sliced_async(eng.ctx, C.byref(pre_db), C.byref(pre_out), C.c_void_p(stream))
    if rc:
        raise RuntimeError(f"prefix replay rc={rc}")
    torch.cuda.synchronize()
    # planning reads the loaded states (a host copy: row counts and keys)
    pre_host = ndc.download_out(dev, pre_out, n, pre_pl)
    pre_res = pre_host.result
    codes = np.frombuffer(pre_res, dtype=np.int32).reshape(n, -1)[:, 0]
    src = np.where((cut > 0) & (codes == abi.OK), np.arange(n), -1).astype(np.int32)
    # an entry whose prefix failed replays WHOLE on a fresh builder (engine.suffix_batch's rule)
    for w in np.nonzero((cut > 0) & (codes != abi.OK))[0]:
        suf.wfs[w] = b.wfs[w]
    suf.carry = engine.Carry(src=src, state=pre_host)
    spl = engine.plan(suf)
    caps, tot = spl.caps, spl.totals
    suf.carry = None
    suf_db = ndc.upload_batch(dev, suf, caps)
    dc = abi.CdrCarry()  # the device copy: the loaded states in HBM
    dc.src, dc.caps, dc.n_src, dc.totals, dc.state = dev.up(src), pre_db.caps, n, pre_pl.totals, pre_out
    suf_db.carry = dev.up(dc)
    suf_out = ndc.alloc_out(dev, n, tot, tasks=args.tasks)
    setup_s = time.perf_counter() - t0
    flags = np.frombuffer(caps, dtype=np.uint32).reshape(n, -1)[:, abi.CdrWfCaps.flags.offset // 4]
    route = {k: int(((flags & m) != 0)[src >= 0].sum()) for k, m in
             (("reg0", abi.CAP_REG0), ("reg", abi.CAP_REG), ("reg2", abi.CAP_REG2))}
    log(f"[rank {rank}] carry: setup {setup_s:.1f}s, carried entries by variant {route}")

    def step():
        rc = L.cdr_replay_sliced_async(eng.ctx, C.byref(suf_db), C.byref(suf_out), C.c_void_p(stream))
        if rc:
            raise RuntimeError(f"carry replay rc={rc}")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    L.cdr_timing_begin(eng.ctx, args.steps)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t1
    ms = elapsed / args.steps * 1e3
    kms = (C.c_float * args.steps)()
    nk = C.c_uint32(args.steps)
    L.cdr_timing_read(eng.ctx, kms, C.byref(nk))
    kern_ms = float(np.mean(kms[:nk.value])) if nk.value else ms
    # events and algorithmic bytes of a step: the suffix events (48 B + A[type] each), the
    # loaded records read (ExecutionInfo + rows, the per-row bytes of SURVEY 8(d)) and the
    # records written
    from cadence_amd.synth import A_TYPE
    words = C.sizeof(abi.CdrEvent) // 4
    ev = np.frombuffer(b.events, dtype=np.uint32).reshape(-1, words)
    wfa = np.frombuffer(suf.wfs, dtype=np.uint8).reshape(n, -1)
    o_off, o_len = abi.CdrWfDesc.ev_off.offset, abi.CdrWfDesc.ev_len.offset
    s_off = wfa[:, o_off:o_off + 8].copy().view(np.int64).ravel()
    s_len = wfa[:, o_len:o_len + 8].copy().view(np.int64).ravel()
    mask = np.zeros(len(ev) + 1, np.int64)
    np.add.at(mask, s_off, 1)
    np.add.at(mask, s_off + s_len, -1)
    in_suf = np.cumsum(mask)[:len(ev)] > 0
    types = ev[in_suf, abi.CdrEvent.type.offset // 4]
    events = int(in_suf.sum())
    ev_bytes = int((48 + A_TYPE[np.minimum(types, 41)]).sum())
    out_res = (abi.CdrWfResult * n)()
    dev.down(out_res, suf_out.result)
    row_b = {"n_activity": 128, "n_timer": 32, "n_child": 48, "n_cancel": 24, "n_signal": 40}
    res_np = np.frombuffer(out_res, dtype=np.uint32).reshape(n, -1)
    pre_np = np.frombuffer(pre_res, dtype=np.uint32).reshape(n, -1)

    def rows(rn, sel):
        tot_ = 0
        for f, bb in row_b.items():
            tot_ += int(rn[sel, getattr(abi.CdrWfResult, f).offset // 4].astype(np.int64).sum()) * bb
        return tot_ + 16 * int(rn[sel, abi.CdrWfResult.n_vh.offset // 4].astype(np.int64).sum())
    carried = src >= 0
    loaded_b = int(carried.sum()) * 256 + rows(pre_np, carried)
    out_b = n * 264 + rows(res_np, np.ones(n, bool))
    alg = ev_bytes + loaded_b + out_b  # SURVEY 8(d) canonical bytes: no task bytes (a17 prices none)
    out_codes = res_np[:, 0].view(np.int32)
    n_xfer = n_ttask = 0
    if args.tasks:
        nt_h = (C.c_int32 * (2 * n))()
        dev.down(nt_h, suf_out.n_tasks)
        nt = np.frombuffer(nt_h, np.int32).reshape(n, 2).astype(np.int64)
        n_xfer, n_ttask = int(nt[:, 0].sum()), int(nt[:, 1].sum())
    # per-entry digests of the carried replay (k_digest) and their sum: the product checksum
    per = torch.zeros(max(1, n), dtype=torch.int64, device="cuda")
    tsum = torch.zeros(1, dtype=torch.int64, device="cuda")
    rc = L.cdr_entry_digests_async(eng.ctx, C.byref(suf_db), C.byref(suf_out), C.c_void_p(per.data_ptr()),
                                   C.c_void_p(tsum.data_ptr()), C.c_void_p(stream))
    if rc:
        raise RuntimeError(f"cdr_entry_digests_async rc={rc}")
    torch.cuda.synchronize()
    stats = torch.tensor([events, n_wf, int((out_codes == abi.OK).sum()), int(tsum.item())], dtype=torch.int64,
                         device=coll_dev)
    (tot_events, tot_wfs, tot_ok, checksum), elapsed = reduce_step(dist, torch, stats, elapsed)
    parity = None
    if not args.no_parity:
        import oracle
        t1 = time.perf_counter()
        got = per[:n].cpu().numpy().view(np.uint64).copy()
        th = host_cores()[0]
        ref_pre = oracle.replay(pre, pre_pl, threads=th)
        sb = engine.Batch(events=b.events, wfs=suf.wfs, kvs=b.kvs, rps=b.rps, cluster=b.cluster, now_ns=b.now_ns,
                          uuid_seed=b.uuid_seed, empty_uuid=b.empty_uuid, carry=engine.Carry(src=src, state=ref_pre))
        rpl = engine.plan(sb)
        ref = oracle.replay(sb, rpl, threads=th, tasks=args.tasks)
        want, _ = oracle.entry_digests(sb, rpl, ref, th)
        whole, _, _ = oracle.synth_digests(cfg, mine, seed, threads=th)
        bad = np.nonzero(got != want)[0]
        bad_whole = np.nonzero(got != whole)[0]
        parity = {"checked": True, "entries": n, "mismatched_entries": int(len(bad)),
                  "first_mismatches": bad[:8].tolist(), "split_vs_whole_mismatched_entries": int(len(bad_whole)),
                  "seconds": time.perf_counter() - t1,
                  "method": "per-entry digest (cdr_entry_digests_async vs oracle/digest_ref.cpp) of the carried "
                            "replay against the oracle's carried replay of its own prefix states, and against the "
                            "oracle's whole-history replay"}
        if args.tasks:  # every entry's task lists, byte for byte (stateBuilder.go:606-608 of the carried call)
            sz = C.sizeof(abi.CdrTask)
            xb = (C.c_uint8 * (max(1, tot.xfer) * sz))()
            tb = (C.c_uint8 * (max(1, tot.ttask) * sz))()
            dev.down(xb, suf_out.transfer)
            dev.down(tb, suf_out.timer_tasks)
            tbad, tn = compare_task_lists({"xfer": bytes(xb), "ttask": bytes(tb)}, nt, caps, ref, rpl.caps, n)
            parity["tasks"] = {"entries": n, "tasks": tn, "mismatched_entries": len(tbad), "first_mismatches": tbad[:8]}
            parity["seconds"] = time.perf_counter() - t1
        log(f"[rank {rank}] carry parity: {len(bad)} of {n} entries differ from the oracle's carried replay, "
            f"{len(bad_whole)} from the whole-history replay"
            + (f", {parity['tasks']['mismatched_entries']} task lists" if args.tasks else "")
            + f" ({parity['seconds']:.1f}s)")
        flag = torch.tensor([parity["mismatched_entries"], parity["split_vs_whole_mismatched_entries"],
                             parity["tasks"]["mismatched_entries"] if args.tasks else 0, n], dtype=torch.int64,
                            device=coll_dev)
        if dist:
            dist.all_reduce(flag)
        (parity["mismatched_entries_all_ranks"], parity["split_vs_whole_mismatched_entries_all_ranks"],
         parity["task_mismatched_entries_all_ranks"], parity["entries_all_ranks"]) = [int(x) for x in flag.tolist()]
    if rank != 0:
        dev.close()
        finish_dist(dist)
        return
    achieved = alg / (kern_ms / 1e3) / 1e9
    workload = f"C{cfg}-{args.wfs}wf-carry-half" + ("-tasks" if args.tasks else "")
    traffic, tnote = load_traffic(workload)
    line = {
        "metric": "history events replayed/sec + workflows rebuilt/sec (node), % of HBM roofline",
        "value": tot_events * args.steps / elapsed, "unit": "events/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": f"synthetic config {cfg}, each history's second half applied onto its first half's loaded state",
        "config": {"workload": workload, "workflows_per_gpu": args.wfs, "entries_rank0": n,
                   "carried_entries_rank0": int(carried.sum()), "events_per_step": tot_events,
                   "events_rank0": events, "routing_rank0": route,
                   "sharding": f"Fingerprint32(workflowID) % {NUM_SHARDS} -> greedy shard->GPU",
                   "status": {abi.STATUS.get(int(v), str(int(v))): int(c) for v, c in
                              zip(*np.unique(out_codes, return_counts=True))},
                   "parallelism": f"shard{world}"},
        "workflows_per_s": tot_wfs * args.steps / elapsed,
        "cpu_baseline": None if (args.no_cpu_baseline or world > 1) else carry_cpu_baseline(cfg, 20000, seed),
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS,
                     "traffic": traffic["bytes_per_launch"] if traffic else None, "traffic_note": tnote or traffic.get("source"),
                     "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": alg,
                     "bytes_breakdown": {"events": ev_bytes, "loaded_state": loaded_b, "written": out_b}},
        "tasks": {"transfer": n_xfer, "timer": n_ttask, "bytes": (n_xfer + n_ttask) * C.sizeof(abi.CdrTask),
                  "note": "task rows written (cdr_task), not in the canonical bytes"} if args.tasks else None,
        "host": {"setup_s": setup_s},
        "checksum": checksum & 0xFFFFFFFFFFFFFFFF, "ok_entries": tot_ok,
        "parity": parity, "parity_checked": parity is not None and parity["mismatched_entries_all_ranks"] == 0
        and parity["task_mismatched_entries_all_ranks"] == 0,
        "shard_load_events": load.tolist(),
    }
    print(json.dumps(line), flush=True)
    dev.close()
    finish_dist(dist)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--wfs", type=int, default=1_000_000, help="workflows per GPU")
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--seed", type=int, default=0x5EED0002)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stream-peak", action="store_true")
    ap.add_argument("--no-fast-path", action="store_true", help="replay every slice with the general kernel")
    ap.add_argument("--no-wave", action="store_true", help="no wave slices: divergent histories in lane slices")
    ap.add_argument("--wave-all", action="store_true", help="every divergent history on a wave slice")
    ap.add_argument("--no-refresh", action="store_true", help="skip the refreshTasks / row-encoder side measurements")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the drop-in host path measurement (decoded histories -> cdr_replay_batch)")
    ap.add_argument("--host-path-wfs", type=int, default=200000,
                    help="workflows of the host-path sample (the population's first ones)")
    ap.add_argument("--no-parity", action="store_true", help="skip the full-size GPU == oracle digest check")
    ap.add_argument("--no-par", action="store_true",
                    help="long register-table histories on wave slices instead of CDR_SLICE_PAR slices")
    ap.add_argument("--no-cls", action="store_true",
                    help="register-table slices on k_replay_reg alone (no class-sorted blocks, k_replay_cls off)")
    ap.add_argument("--cls-in-step", action="store_true",
                    help="class-sorted blocks built on the device (k_cls_count / k_cls_fill) INSIDE every timed step, "
                         "instead of emitted by the host packer")
    ap.add_argument("--ndc-forks", action="store_true",
                    help="configs[4]'s conflict-resolution line: the forked config-5 population replicated on "
                         "the device (base branch + 2 fork rounds per step); --wfs workflows")
    ap.add_argument("--long-stride", type=int, default=0,
                    help="configs[3] load balance: every workflow at index long_stride/2 mod long_stride is generated "
                         "at the history count limit (204,800 events); 125000 mixes 8 into 1M")
    ap.add_argument("--tasks", action="store_true",
                    help="also emit the stateBuilder's transfer / timer task lists (cdr_out.transfer / timer_tasks; "
                         "k_replay_fast<TASKS> for C1/C2, the register-table kernels' TASKS instantiations "
                         "(k_replay_reg<..., TASKS>) for the register-table / PAR slices of C3-C5, the general "
                         "kernel for the rest)")
    ap.add_argument("--carry", action="store_true",
                    help="carry-in line: each history's second half replayed onto its first half's loaded state "
                         "(--config, --wfs)")
    args = ap.parse_args()
    import torch  # before libcdr.so: torch's HIP runtime must be the process's one (tests/conftest.py)
    L = abi.lib()
    if L.cdr_build_flags():  # a profiling / tuning variant never reaches a reported line
        raise SystemExit(f"libcdr.so is a variant build (cdr_build_flags = {L.cdr_build_flags():#x}); rebuild it")
    if args.ndc_forks:
        return ndc_forks_line(args)
    if args.carry:
        return carry_line(args)

    import torch
    dist, world, rank, local, coll_dev = init_dist(torch)
    ctx = L.cdr_create(torch.cuda.current_device(), None)
    if not ctx:
        raise SystemExit("cdr_create failed (no GPU?) — the engine has no CPU fallback")
    if args.no_fast_path:
        L.cdr_set_fast_path(ctx, 0)

    total = args.wfs * world
    mine, load = assign_shards(total, world, rank, workflow_weights(args.config, total, args.seed, args.long_stride))
    log(f"[rank {rank}] {len(mine)} of {total} workflows (shard->GPU greedy over {NUM_SHARDS} shards)")
    # the register-table slices' class-sorted blocks: emitted by the host packer beside the
    # slab (default; host packing time cls_pack_s), built on the device in every step
    # (--cls-in-step), or none (--no-cls)
    # (with task lists: no wave / PAR slices, cdr_replay_sliced_async's contract for task
    # emission; the class kernels' TASKS instantiations stage the register-table slices' tasks
    # and k_tasks_merge orders them)
    cls_src = None if args.no_cls else "device" if args.cls_in_step else "host"
    db = DeviceBatch(torch, args.config, mine, args.seed,
                     plan_mode=0 if args.no_wave else abi.PLAN_WAVE
                     | (abi.PLAN_WAVE_ALL if args.wave_all else 0) | (0 if args.no_par else abi.PLAN_PAR)
                     # task batches: the PAR histories one per slice (their slices replay on k_replay_reg<TASKS>)
                     | (abi.PLAN_PAR_SOLO if args.tasks and not args.no_par else 0),
                     ctx_for_cls=ctx, cls=cls_src, long_stride=args.long_stride, tasks=args.tasks)
    if args.no_cls:
        L.cdr_set_cls_path(ctx, abi.CLS_OFF)
    log(f"[rank {rank}] {db.n_fast} of {db.info.n_slices} slices on the fast-path kernel, {db.n_wave} wave slices")
    if args.tasks and db.n_wave:
        raise SystemExit("--tasks: the plan has wave slices (no task emission there); use --no-wave")
    log(f"[rank {rank}] packed {db.n_events:,} events in {db.pack_s:.2f}s (host SoA) + {db.cls_pack_s:.2f}s "
        f"(class blocks, {db.cls_where}), H2D {db.h2d_s:.2f}s "
        f"({db.in_bytes / 1e9:.2f} GB in, {db.out_bytes / 1e9:.2f} GB out buffers)")
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        if db.cls_where == "device" and args.cls_in_step:  # the class sort inside the step
            rows_t, row0_t, _ = db.cls_dev
            rc = L.cdr_cls_plan_async(ctx, C.byref(db.db), C.c_void_p(rows_t.data_ptr()),
                                      C.c_void_p(row0_t.data_ptr()), C.c_void_p(stream))
            rc = rc or L.cdr_cls_pack_async(ctx, C.byref(db.db), C.c_void_p(stream))
            if rc:
                raise RuntimeError(f"class block build rc={rc}")
        rc = L.cdr_replay_sliced_async(ctx, C.byref(db.db), C.byref(db.out), C.c_void_p(stream))
        if rc:
            raise RuntimeError(f"cdr_replay_sliced_async rc={rc}")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    L.cdr_timing_begin(ctx, args.steps)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ms = (C.c_float * args.steps)()
    n = C.c_uint32(args.steps)
    L.cdr_timing_read(ctx, ms, C.byref(n))
    kern_ms = float(np.mean(np.frombuffer(ms, np.float32)[: n.value]))

    # verification + the only collective: RCCL allreduce of counters and checksums
    res = db.results()
    alg_bytes, n_ok, ev_b, wf_b, row_b = db.algorithmic_bytes(res)
    n_xfer, n_ttask = db.task_counts()
    # the task rows written (cdr_task): listed apart, not in `achieved` / `frac` — SURVEY §8(d)
    # prices no task bytes (a17: counts only); `frac_with_task_bytes` counts them as written
    task_b = (n_xfer + n_ttask) * C.sizeof(abi.CdrTask)
    csum = torch.zeros(1, dtype=torch.int64, device="cuda")
    L.cdr_checksum_async(ctx, C.byref(db.db), C.byref(db.out), C.c_void_p(csum.data_ptr()), C.c_void_p(stream))
    stats = torch.tensor([db.n_events, db.info.n_entries, n_ok, 0], dtype=torch.int64, device="cuda")
    stats[3] = csum[0]
    stats = stats.to(coll_dev)
    (tot_events, tot_wfs, tot_ok, checksum), elapsed = reduce_step(dist, torch, stats, elapsed)
    if tot_ok != tot_wfs:
        log(f"WARNING: {tot_wfs - tot_ok} workflows did not replay OK")

    parity = None if args.no_parity else parity_check(db, ctx, stream, args.config, mine, args.seed, args.long_stride)
    if parity:
        log(f"[rank {rank}] parity: {parity['mismatched_entries']} of {parity['entries']} entries differ from the "
            f"oracle ({parity['seconds']:.1f}s)")
        flag = torch.tensor([parity["mismatched_entries"], parity["entries"]], dtype=torch.int64, device=coll_dev)
        if dist:
            dist.all_reduce(flag)
        parity["mismatched_entries_all_ranks"], parity["entries_all_ranks"] = [int(x) for x in flag.tolist()]
        if args.tasks:
            parity["tasks"] = task_parity(db, args.config, mine, args.seed, args.long_stride)
            log(f"[rank {rank}] task parity: {parity['tasks']['mismatched_entries']} of {parity['tasks']['entries']} "
                f"entries' task lists differ ({parity['tasks']['tasks']} tasks, {parity['tasks']['seconds']:.1f}s)")
    encode = None if args.no_refresh else encode_measure(torch, L, ctx, db, stream, max(1, args.steps))
    refresh = None if args.no_refresh else refresh_measure(torch, L, ctx, db, stream, max(1, args.steps))
    if rank != 0:
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return
    ms_per_step = elapsed / args.steps * 1e3
    ev_per_s = tot_events * args.steps / elapsed
    wf_per_s = tot_wfs * args.steps / elapsed
    # the bytes priced: on the fast kernel's workloads the bytes its packed input needs (the
    # delta bits skip implied event_id / version columns, so SURVEY §8(d)'s canonical price —
    # reported beside — overstates them and can exceed the peak); elsewhere the canonical price
    fast_enc = args.config in (1, 2) and not args.no_fast_path and db.n_fast == db.info.n_slices
    priced = db.encoded_bytes(res) if fast_enc else alg_bytes
    achieved = priced / (kern_ms / 1e3) / 1e9
    workload = (f"C{args.config}-{args.wfs}wf-sliced" + (f"-long{args.long_stride}" if args.long_stride else "")
                + ("-tasks" if args.tasks else ""))
    traffic, traffic_note = load_traffic(workload)
    bld = db.builders()
    names = {abi.BUILDER_LOCAL: "local", abi.BUILDER_2DC: "2DC", abi.BUILDER_NDC: "NDC"}
    builders = {names[int(k)]: int(c) for k, c in zip(*np.unique(bld, return_counts=True))}
    peak_meas = None if args.no_stream_peak else stream_peak_gbs(torch)
    traffic_gbs = traffic["bytes_per_launch"] / (kern_ms / 1e3) / 1e9 if traffic else None
    cpu = None if (args.no_cpu_baseline or args.gpus > 1) else cpu_baseline(args.config, 20000, args.seed)
    host_path = None if (args.no_host_path or world > 1) else \
        host_path_measure(args.config, args.seed, args.host_path_wfs, ctx, args.long_stride)
    line = {
        "metric": "history events replayed/sec + workflows rebuilt/sec (node), % of HBM roofline",
        "value": ev_per_s, "unit": "events/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "int64", "data": "synthetic (deterministic generator, SURVEY §8(d) shapes)",
        "config": {"workload": workload, "workflows_per_gpu": args.wfs, "events_per_gpu": db.n_events,
                   "events_per_workflow": round(db.n_events / max(1, len(mine)), 2),
                   "builder": next(iter(builders)) if len(builders) == 1 else "mixed", "builders": builders,
                   "sharding": f"Fingerprint32(workflowID) % {NUM_SHARDS} -> greedy shard->GPU",
                   "parallelism": f"shard{world}"},
        "workflows_per_s": wf_per_s,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS,
                     "achieved_basis": ("encoded input: bytes the packed events need (delta bits applied) + outputs"
                                        if fast_enc else "canonical SURVEY §8(d) bytes"),
                     "traffic": traffic["bytes_per_launch"] if traffic else None,
                     "traffic_note": traffic_note or traffic.get("source"),
                     # HBM bytes actually moved per launch (PMC of this build) / the live kernel time:
                     # the roofline position
                     "traffic_gbs": traffic_gbs,
                     "traffic_frac": traffic_gbs / PEAK_HBM_GBS if traffic else None,
                     "position": "traffic_frac (HBM bytes moved per launch, PMC of this build, / kernel time / 8 TB/s)",
                     "canonical_bytes_per_launch": alg_bytes,
                     "canonical_frac": alg_bytes / (kern_ms / 1e3) / 1e9 / PEAK_HBM_GBS,
                     "encoded_bytes_per_launch": priced if fast_enc else None,
                     "kernel": ("k_replay_fast" if args.config in (1, 2) and not args.no_fast_path else "k_replay*")
                     + ("<TASKS>" if args.tasks else ""),
                     "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": priced,
                     "bytes_breakdown": {"events": ev_b, "per_workflow": wf_b, "pending_rows": row_b,
                                         "tasks_not_priced": task_b},
                     "frac_with_task_bytes": ((alg_bytes + task_b) / (kern_ms / 1e3) / 1e9 / PEAK_HBM_GBS
                                              if args.tasks else None),
                     "stream_copy_peak_gbs": peak_meas,
                     "traffic_frac_of_stream_copy": (traffic_gbs / peak_meas if traffic and peak_meas else None)},
        "cpu_baseline": cpu,
        "refresh": refresh,
        "encode": encode,
        "host": {"soa_pack_s": db.pack_s, "h2d_s": db.h2d_s,
                 "h2d_gbs": db.in_bytes / max(db.h2d_s, 1e-9) / 1e9,
                 # class-sorted blocks of the register-table slices: where they came from, the
                 # host packer's time for them (part of the SoA packing), a device build
                 # outside the step (0 unless cls_where == "device" without --cls-in-step)
                 "cls_where": db.cls_where, "cls_in_step": bool(args.cls_in_step and db.cls_where == "device"),
                 "cls_pack_s": db.cls_pack_s, "cls_rows": db.cls_rows,
                 "cls_build_s": 0.0 if args.cls_in_step else db.cls_s,
                 # one batch end to end on this rank: host packing (slab + class blocks) + H2D +
                 # one replay step
                 "per_batch_s": db.pack_s + db.cls_pack_s + db.h2d_s + ms_per_step / 1e3,
                 "per_batch_events_per_s": db.n_events / (db.pack_s + db.cls_pack_s + db.h2d_s + ms_per_step / 1e3)},
        "tasks": {"transfer": n_xfer, "timer": n_ttask, "bytes": task_b} if args.tasks else None,
        "host_path": host_path,
        "checksum": checksum & 0xFFFFFFFFFFFFFFFF, "ok_workflows": tot_ok,
        "parity_checked": bool(parity) and parity["mismatched_entries_all_ranks"] == 0
        and (not parity.get("tasks") or parity["tasks"]["mismatched_entries"] == 0),
        "parity": parity,
        "shard_load_events": load.tolist(),
    }
    print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    L.cdr_destroy(ctx)


if __name__ == "__main__":
    main()
