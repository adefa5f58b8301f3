#!/usr/bin/env python3
"""Benchmark of the MI355X batched workflow-history replay engine.

Metric (BASELINE.json): history events replayed/s and workflows rebuilt/s per node,
as a fraction of the HBM roofline.  Workload (configs[1]): 1M activity-heavy
workflows x 203 events, synthetic, NDC builder, on each GPU
(weak scaling: N GPUs replay N x 1M workflows, sharded by historyShardID =
Fingerprint32(workflowID) % 16384 and assigned shard->GPU greedily).

One "step" = one replay of the whole device-resident batch (k_replay + k_finalize).
Inputs are uploaded before the timed region; host SoA packing and H2D time are
reported separately.  The CPU baseline is the CPU restatement (oracle/) run with one
task per workflow on the host's cores over a bounded sample.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--wfs M] [--config C]
       (N>1: torchrun --nproc-per-node N bench.py --gpus N ...)
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

# SURVEY §8(d) canonical algorithmic bytes
A_TYPE = np.zeros(256, np.int64)
for _name, _b in (("WorkflowExecutionStarted", 96), ("ActivityTaskScheduled", 48), ("DecisionTaskScheduled", 12),
                  ("DecisionTaskCompleted", 12), ("TimerStarted", 8), ("StartChildWorkflowExecutionInitiated", 16),
                  ("SignalExternalWorkflowExecutionInitiated", 12), ("DecisionTaskStarted", 4),
                  ("ActivityTaskStarted", 4), ("DecisionTaskTimedOut", 4), ("ChildWorkflowExecutionStarted", 4),
                  ("WorkflowExecutionContinuedAsNew", 4), ("UpsertWorkflowSearchAttributes", 8)):
    A_TYPE[abi.EV[_name]] = _b
ROW_BYTES = {"n_activity": 128, "n_timer": 32, "n_child": 48, "n_cancel": 24, "n_signal": 40}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def assign_shards(total_wfs: int, world: int, rank: int, lengths=None):
    """workflow ids "wf-<i>" -> historyShardID -> GPU (greedy largest-first on events)."""
    L = abi.lib()
    shard = np.empty(total_wfs, np.int32)
    L.cdr_synth_shards(total_wfs, NUM_SHARDS, shard.ctypes.data)
    w = np.bincount(shard, weights=lengths, minlength=NUM_SHARDS) if lengths is not None else \
        np.bincount(shard, minlength=NUM_SHARDS).astype(np.float64)
    owner = np.zeros(NUM_SHARDS, np.int32)
    load = np.zeros(world)
    for s in np.argsort(-w, kind="stable"):
        g = int(np.argmin(load))
        owner[s] = g
        load[g] += w[s]
    mine = np.nonzero(owner[shard] == rank)[0].astype(np.uint32)
    return mine, load


class DeviceBatch:
    """Synthetic batch generated straight into the sliced layout, uploaded to HBM."""

    def __init__(self, torch, config, index_map, seed, target_len=0, plan_mode=abi.PLAN_WAVE):
        L = abi.lib()
        self.torch = torch
        self.index_map = index_map
        p = abi.CdrSynthParams(config=config, n_wfs=len(index_map), seed=seed, target_len=target_len, max_len=0,
                               error_rate=0.0, builder=-1, rebuild=0, index_map=index_map.ctypes.data,
                               plan_mode=plan_mode)
        self.params = p
        t0 = time.perf_counter()
        info = abi.CdrSynthPlanInfo()
        assert L.cdr_synth_sliced_plan(C.byref(p), C.byref(info)) == 0
        self.info = info
        self.h_slab = np.empty(info.n_rows * 64 * abi.EL_BYTES, np.uint8)
        self.h_lane = np.empty(info.n_slices * 64, np.int32)
        self.h_slen = np.empty(info.n_slices, np.uint32)
        self.h_row0 = np.empty(info.n_slices, np.uint64)
        self.h_sc_off = np.zeros(info.n_slices, np.uint64)
        self.h_sc_act = np.zeros(info.n_slices, np.uint32)
        self.h_sc_tim = np.zeros(info.n_slices, np.uint32)
        self.h_sflags = np.zeros(info.n_slices, np.uint32)
        self.h_arena = np.empty(max(1, info.arena_words), np.uint64)
        self.h_wfs = (abi.CdrWfDesc * info.n_entries)()
        self.h_caps = (abi.CdrWfCaps * info.n_entries)()
        self.h_kvs = np.zeros(max(1, info.n_kvs) * 2, np.uint32)
        self.h_rps = (abi.CdrResetPoint * max(1, info.n_rps))()
        s = abi.CdrSlices(n_slices=info.n_slices, n_rows=info.n_rows, arena_words=info.arena_words)
        s.slice_row0, s.slice_len, s.lane_wf = self.h_row0.ctypes.data, self.h_slen.ctypes.data, \
            self.h_lane.ctypes.data
        s.slab = self.h_slab.ctypes.data
        s.arena = self.h_arena.ctypes.data
        s.slice_scratch_off, s.slice_act_slots, s.slice_tim_slots = (
            self.h_sc_off.ctypes.data, self.h_sc_act.ctypes.data, self.h_sc_tim.ctypes.data)
        s.slice_flags = self.h_sflags.ctypes.data
        meta = abi.CdrBatch()
        threads = min(32, os.cpu_count() or 8)
        rc = L.cdr_synth_sliced_fill(C.byref(p), C.byref(s), self.h_wfs, self.h_caps, self.h_kvs.ctypes.data,
                                     self.h_rps, C.byref(meta), threads)
        assert rc == 0, rc
        self.meta = meta
        self.pack_s = time.perf_counter() - t0
        # ---- upload (H2D timed separately)
        dev = torch.device("cuda", torch.cuda.current_device())
        t0 = time.perf_counter()
        self.keep = []

        def up(a):
            t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to(dev)
            self.keep.append(t)
            return t.data_ptr()

        def up_ct(a):
            return up(np.frombuffer(a, np.uint8))

        db = abi.CdrDevBatch()
        db.ev.n_slices, db.ev.n_rows, db.ev.arena_words = info.n_slices, info.n_rows, info.arena_words
        db.ev.slice_row0, db.ev.slice_len, db.ev.lane_wf = up(self.h_row0), up(self.h_slen), up(self.h_lane)
        db.ev.slab = up(self.h_slab)
        db.ev.arena = up(self.h_arena)
        db.ev.slice_scratch_off = up(self.h_sc_off)
        db.ev.slice_act_slots = up(self.h_sc_act)
        db.ev.slice_tim_slots = up(self.h_sc_tim)
        db.ev.slice_flags = up(self.h_sflags)
        L.cdr_plan_scratch(self.h_caps, self.h_lane.ctypes.data, info.n_slices, None, None, None, None,
                           C.byref(sc_words := C.c_uint64()), None)
        self.scratch_t = torch.zeros(max(8, sc_words.value * 8), dtype=torch.uint8, device=dev)
        db.scratch = self.scratch_t.data_ptr()
        db.wfs, db.caps = up_ct(self.h_wfs), up_ct(self.h_caps)
        db.kvs, db.rps = up(self.h_kvs), up_ct(self.h_rps)
        db.n_wfs = info.n_entries
        db.max_act_slots = int(self.h_sc_act.max()) if len(self.h_sc_act) else 0
        db.max_tim_slots = int(self.h_sc_tim.max()) if len(self.h_sc_tim) else 0
        self.n_fast = int(((self.h_sflags & abi.SLICE_FAST) != 0).sum())
        self.n_wave = int(((self.h_sflags & abi.SLICE_WAVE) != 0).sum())
        db.n_fast_slices = self.n_fast
        db.n_wave_slices = self.n_wave
        db.empty_uuid = meta.empty_uuid
        db.cluster = meta.cluster
        db.now_ns = meta.now_ns
        db.uuid_seed = meta.uuid_seed
        self.db = db
        tot = info.totals
        out = abi.CdrOut()
        sizes = {"result": info.n_entries * C.sizeof(abi.CdrWfResult),
                 "exec": info.n_entries * C.sizeof(abi.CdrExecInfo),
                 "repl": info.n_entries * C.sizeof(abi.CdrReplState),
                 "vh": tot.vh * C.sizeof(abi.CdrVHItem), "act": tot.act * C.sizeof(abi.CdrActivityInfo),
                 "timer": tot.timer * C.sizeof(abi.CdrTimerInfo), "child": tot.child * C.sizeof(abi.CdrChildInfo),
                 "cancel": tot.cancel * C.sizeof(abi.CdrCancelInfo),
                 "signal": tot.signal * C.sizeof(abi.CdrSignalInfo),
                 "rp": tot.rp * C.sizeof(abi.CdrResetPoint), "sa": tot.sa * C.sizeof(abi.CdrKV)}
        self.out_bytes = sum(sizes.values())
        self.out_t = {}
        for k, nb in sizes.items():
            t = torch.zeros(max(8, nb), dtype=torch.uint8, device=dev)
            self.out_t[k] = t
            setattr(out, k, t.data_ptr())
        self.out = out
        torch.cuda.synchronize()
        self.h2d_s = time.perf_counter() - t0
        self.in_bytes = self.h_slab.nbytes + self.h_arena.nbytes
        types = abi.slab_columns(self.h_slab, self.h_row0, self.h_slen, ("type_flags",))["type_flags"] & 0xFF
        self.type_counts = np.bincount(types, minlength=256)
        self.n_events = int(self.type_counts[:abi.EV["UpsertWorkflowSearchAttributes"] + 1].sum())

    def results(self):
        n = self.info.n_entries
        raw = self.out_t["result"][: n * C.sizeof(abi.CdrWfResult)].cpu().numpy().copy()
        return (abi.CdrWfResult * n).from_buffer(raw)

    def algorithmic_bytes(self, res):
        ev_bytes = int((self.type_counts[:42] * (48 + A_TYPE[:42])).sum())
        n_ok, vh, rows, repl = 0, 0, 0, 0
        arr = np.frombuffer(res, dtype=np.dtype([("code", "<i4"), ("flags", "<u4"), ("fid", "<i8"), ("fix", "<i8"),
                                                   ("n_activity", "<u4"), ("n_timer", "<u4"), ("n_child", "<u4"),
                                                   ("n_cancel", "<u4"), ("n_signal", "<u4"), ("n_vh", "<u4"),
                                                   ("n_rp", "<u4"), ("n_sa", "<u4")]))
        builders = np.frombuffer(self.h_wfs, dtype=np.uint8).reshape(len(self.h_wfs), -1)
        ok = arr["code"] == 0
        n_ok = int(ok.sum())
        vh = int(arr["n_vh"][ok].sum())
        for f, b in ROW_BYTES.items():
            rows += int(arr[f][ok].sum()) * b
        # builder field offset in cdr_wf_desc
        boff = abi.CdrWfDesc.builder.offset
        bld = builders[:, boff:boff + 4].copy().view(np.uint32)[:, 0]
        repl = int(((bld == abi.BUILDER_2DC) & ok).sum()) * 32
        wf_bytes = len(arr) * (256 + 8) + 16 * vh + repl
        return ev_bytes + wf_bytes + rows, n_ok, ev_bytes, wf_bytes, rows


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
    res = np.frombuffer(db.results(), dtype=np.dtype([("code", "<i4"), ("flags", "<u4"), ("fid", "<i8"),
                                                      ("fix", "<i8"), ("n_activity", "<u4"), ("n_timer", "<u4"),
                                                      ("n_child", "<u4"), ("n_cancel", "<u4"), ("n_signal", "<u4"),
                                                      ("n_vh", "<u4"), ("n_rp", "<u4"), ("n_sa", "<u4")]))
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
    res = np.frombuffer(db.results(), dtype=np.dtype([("code", "<i4"), ("flags", "<u4"), ("fid", "<i8"),
                                                      ("fix", "<i8"), ("n_activity", "<u4"), ("n_timer", "<u4"),
                                                      ("n_child", "<u4"), ("n_cancel", "<u4"), ("n_signal", "<u4"),
                                                      ("n_vh", "<u4"), ("n_rp", "<u4"), ("n_sa", "<u4")]))
    ok = res["code"] == 0
    out = {}
    for name, tid, size, stride, cnt, tot in (("timer", 1, 45, 48, "n_timer", db.info.totals.timer),
                                              ("cancel", 3, 66, 80, "n_cancel", db.info.totals.cancel)):
        rows = int(res[cnt][ok].sum())
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


def stream_peak_gbs(torch, nbytes=4 << 30, reps=5):
    a = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        b.copy_(a)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    del a, b
    return 2 * nbytes / dt / 1e9


def cpu_baseline(config, n_wfs, seed, min_seconds=10.0):
    """CPU restatement (oracle/) on the box's host cores, one task per workflow (the
    analogue of the reference's goroutine-per-workflow), over a bounded sample."""
    import oracle
    from cadence_amd import engine
    b = engine.synth_batch(config, n_wfs, seed)
    pl = engine.plan(b)
    n_ev = len(b.events)
    threads = max(1, min(os.cpu_count() or 1, int(os.environ.get("CDR_CPU_THREADS", "16"))))
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
    return {"value": res[threads], "unit": "events/s", "cores": threads, "kind": "port",
            "refresh_entries_per_s_1thread": refresh_eps,
            "sample": f"config {config}: {n_wfs} workflows x {n_ev // max(1, n_wfs)} events, replayed "
                      f"{'repeatedly'} for >= {min_seconds:.0f} s; single-thread {res[1]:.4g} events/s; "
                      f"the Go stateBuilder cannot run here (no Go toolchain)",
            "single_thread_events_per_s": res[1], "workflows_per_s": res[threads] / (n_ev / max(1, n_wfs))}


def load_traffic(workload):
    p = os.path.join(HERE, "profiles", "traffic_latest.json")
    try:
        d = json.load(open(p))
        if d.get("workload") == workload:
            return d
    except Exception:
        pass
    return None


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
    args = ap.parse_args()

    import torch
    world, rank, local = dist_env()
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist = None
        torch.cuda.set_device(0)
    L = abi.lib()
    ctx = L.cdr_create(torch.cuda.current_device())
    if not ctx:
        raise SystemExit("cdr_create failed (no GPU?) — the engine has no CPU fallback")
    if args.no_fast_path:
        L.cdr_set_fast_path(ctx, 0)

    total = args.wfs * world
    mine, _ = assign_shards(total, world, rank)
    log(f"[rank {rank}] {len(mine)} of {total} workflows (shard->GPU greedy over {NUM_SHARDS} shards)")
    db = DeviceBatch(torch, args.config, mine, args.seed, plan_mode=0 if args.no_wave else abi.PLAN_WAVE | (abi.PLAN_WAVE_ALL if args.wave_all else 0))
    log(f"[rank {rank}] {db.n_fast} of {db.info.n_slices} slices on the fast-path kernel, {db.n_wave} wave slices")
    log(f"[rank {rank}] packed {db.n_events:,} events in {db.pack_s:.2f}s (host SoA), H2D {db.h2d_s:.2f}s "
        f"({db.in_bytes / 1e9:.2f} GB in, {db.out_bytes / 1e9:.2f} GB out buffers)")
    stream = torch.cuda.current_stream().cuda_stream

    def step():
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
    csum = torch.zeros(1, dtype=torch.int64, device="cuda")
    L.cdr_checksum_async(ctx, C.byref(db.db), C.byref(db.out), C.c_void_p(csum.data_ptr()), C.c_void_p(stream))
    stats = torch.tensor([db.n_events, db.info.n_entries, n_ok, 0], dtype=torch.int64, device="cuda")
    stats[3] = csum[0]
    t_el = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if dist:
        dist.all_reduce(stats)
        dist.all_reduce(t_el, op=dist.ReduceOp.MAX)
    torch.cuda.synchronize()
    elapsed = float(t_el.item())
    tot_events, tot_wfs, tot_ok, checksum = [int(x) for x in stats.tolist()]
    if tot_ok != tot_wfs:
        log(f"WARNING: {tot_wfs - tot_ok} workflows did not replay OK")

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
    achieved = alg_bytes / (kern_ms / 1e3) / 1e9
    workload = f"C{args.config}-{args.wfs}wf-sliced"
    traffic = load_traffic(workload)
    peak_meas = None if args.no_stream_peak else stream_peak_gbs(torch)
    cpu = None if (args.no_cpu_baseline or args.gpus > 1) else cpu_baseline(args.config, 20000, args.seed)
    line = {
        "metric": "history events replayed/sec + workflows rebuilt/sec (node), % of HBM roofline",
        "value": ev_per_s, "unit": "events/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "int64", "data": "synthetic (deterministic generator, SURVEY §8(d) shapes)",
        "config": {"workload": workload, "workflows_per_gpu": args.wfs, "events_per_gpu": db.n_events,
                   "events_per_workflow": round(db.n_events / max(1, len(mine)), 2), "builder": "NDC",
                   "sharding": f"Fingerprint32(workflowID) % {NUM_SHARDS} -> greedy shard->GPU",
                   "parallelism": f"shard{world}"},
        "workflows_per_s": wf_per_s,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS,
                     "traffic": traffic["bytes_per_launch"] if traffic else None,
                     # HBM bytes actually moved per launch (PMC) / the live kernel time
                     "traffic_gbs": traffic["bytes_per_launch"] / (kern_ms / 1e3) / 1e9 if traffic else None,
                     "kernel": "k_replay_fast" if args.config in (1, 2) and not args.no_fast_path else "k_replay*",
                     "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": alg_bytes,
                     "bytes_breakdown": {"events": ev_b, "per_workflow": wf_b, "pending_rows": row_b},
                     "stream_copy_peak_gbs": peak_meas},
        "cpu_baseline": cpu,
        "refresh": refresh,
        "encode": encode,
        "host": {"soa_pack_s": db.pack_s, "h2d_s": db.h2d_s,
                 "h2d_gbs": db.in_bytes / max(db.h2d_s, 1e-9) / 1e9},
        "checksum": checksum & 0xFFFFFFFFFFFFFFFF, "ok_workflows": tot_ok,
    }
    print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    L.cdr_destroy(ctx)


if __name__ == "__main__":
    main()
