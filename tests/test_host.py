"""CPU-only checks of the C-ABI library: it loads, exports every symbol the headers
declare, its struct layouts match the Python mirrors, and the host-side planner and
packer are correct (no GPU compute is called here)."""
import ctypes as C
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from cadence_amd import abi, engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in ("cdr.h", "synth.h"):
        src = open(os.path.join(ROOT, "include", "cdr", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"CDR_HD [^(]*\(", "", src)  # header-inline helpers are not exports
        names |= set(re.findall(r"\b(cdr_[a-z0-9_]+)\s*\(", src))
    return names


def test_library_exports_every_declared_symbol():
    L = abi.lib()
    declared = _declared()
    assert len(declared) >= 15
    missing = [n for n in sorted(declared) if not hasattr(L, n)]
    assert not missing, missing
    assert set(abi.EXPORTS) >= declared - {"cdr_struct_size"}


def test_in_tree_library_is_the_product_build():
    """No profiling or tuning variant (cdr_build_flags) in the library the tests, smoke()
    and bench.py load."""
    assert abi.lib().cdr_build_flags() == 0


def test_struct_layouts_match_mirrors():
    abi.check_layouts()


def test_plan_slices_sorted_and_padded():
    b = engine.synth_batch(0, 300, seed=3)
    L = abi.lib()
    ns, rows = C.c_uint32(), C.c_uint64()
    assert L.cdr_plan_slices(b.wfs, b.n_wfs, None, None, None, C.byref(ns), C.byref(rows)) == 0
    lane = (C.c_int32 * (ns.value * 64))()
    slen = (C.c_uint32 * ns.value)()
    row0 = (C.c_uint64 * ns.value)()
    assert L.cdr_plan_slices(b.wfs, b.n_wfs, lane, slen, row0, C.byref(ns), C.byref(rows)) == 0
    lane = np.frombuffer(lane, np.int32)
    assert sorted(lane[lane >= 0].tolist()) == list(range(b.n_wfs))
    lens = np.array([b.wfs[w].ev_len if w >= 0 else 0 for w in lane]).reshape(-1, 64)
    assert (lens.max(1) == np.frombuffer(slen, np.uint32)).all()
    assert (np.diff(lens.max(1)) <= 0).all()  # longest slices first
    assert np.frombuffer(row0, np.uint64)[-1] + slen[ns.value - 1] == rows.value


def test_pack_round_trip():
    """Every event lands in its (slice, row, lane) cell with the operands the kernel
    reads; padding cells are PAD."""
    b = engine.synth_batch(0, 150, seed=11, error_rate=0.2)
    L = abi.lib()
    ns, rows = C.c_uint32(), C.c_uint64()
    L.cdr_plan_slices(b.wfs, b.n_wfs, None, None, None, C.byref(ns), C.byref(rows))
    n = rows.value * 64
    lane = np.zeros(ns.value * 64, np.int32)
    slen = np.zeros(ns.value, np.uint32)
    row0 = np.zeros(ns.value, np.uint64)
    L.cdr_plan_slices(b.wfs, b.n_wfs, lane.ctypes.data, slen.ctypes.data, row0.ctypes.data, C.byref(ns),
                      C.byref(rows))
    slab = np.zeros(n * abi.EL_BYTES, np.uint8)
    aw = L.cdr_plan_arena_words(C.byref(b.cstruct()))
    arena = np.zeros(max(1, aw), np.uint64)
    s = abi.CdrSlices(n_slices=ns.value, n_rows=rows.value, arena_words=aw)
    s.slice_row0, s.slice_len, s.lane_wf = row0.ctypes.data, slen.ctypes.data, lane.ctypes.data
    s.slab = slab.ctypes.data
    s.arena = arena.ctypes.data
    assert L.cdr_pack_slices(C.byref(b.cstruct()), C.byref(s), 2) == 0
    cols = abi.slab_columns(slab, row0, slen)
    assert all(len(v) == n for v in cols.values())
    for i, w in enumerate(lane):
        sl, l = divmod(i, 64)
        if w < 0:
            continue
        d = b.wfs[w]
        for k in range(slen[sl]):
            j = (int(row0[sl]) + k) * 64 + l
            if k >= d.ev_len:
                assert cols["type_flags"][j] == 0xFF
                continue
            e = b.events[d.ev_off + k]
            assert cols["type_flags"][j] & 0xFF == e.type
            assert bool(cols["type_flags"][j] & abi.SEF_BATCH_FIRST) == bool(e.flags & 1 or k == 0)
            p = b.events[d.ev_off + k - 1] if k > 0 else None
            assert bool(cols["type_flags"][j] & abi.SEF_ID_NEXT) == (p is not None and e.event_id == p.event_id + 1)
            assert bool(cols["type_flags"][j] & abi.SEF_VER_SAME) == (p is not None and e.version == p.version)
            need = (int(cols["type_flags"][j]) >> 16) & 0x1F  # CDR_SEF_NEED_{TS,KEY,AUX,H,N}
            if e.type == abi.EV["ActivityTaskScheduled"]:
                assert need == 0x1F
            elif e.type == abi.EV["ActivityTaskCompleted"]:
                assert need == 0x02
            assert (cols["event_id"][j], cols["version"][j], cols["timestamp"][j], cols["task_id"][j]) == (
                e.event_id, e.version, e.timestamp, e.task_id)
            if e.type == abi.EV["ActivityTaskScheduled"]:
                a = e.a.at_sched
                off = int(cols["aux"][j]) & 0xFFFFFFFF
                rec = abi.AttrATSched.from_buffer_copy(arena[off:off + C.sizeof(abi.AttrATSched) // 8].tobytes())
                assert bytes(rec) == bytes(a)
                assert int(cols["key"][j]) & 0xFFFFFFFF == a.activity_id
                assert (int(cols["key"][j]) >> 32) & 0xFFFFFFFF == a.stc_s & 0xFFFFFFFF
                assert (int(cols["aux"][j]) >> 32) & 0xFFFFFFFF == a.hb_s & 0xFFFFFFFF
                assert cols["h"][j] == a.s2c_s & 0xFFFFFFFF and cols["n"][j] == a.s2s_s
            elif e.type == abi.EV["ActivityTaskStarted"]:
                assert cols["key"][j] == e.a.at.scheduled_event_id and cols["h"][j] == e.a.at.request_id
            elif e.type == abi.EV["TimerStarted"]:
                assert cols["key"][j] == e.a.timer.timer_id and cols["aux"][j] == e.a.timer.start_to_fire_s


def test_plan_caps_bound_oracle_outputs():
    import oracle
    b = engine.synth_batch(4, 200, seed=5)
    pl = engine.plan(b)
    out = oracle.replay(b, pl)
    for w in range(b.n_wfs):
        r, c = out.result[w], pl.caps[w]
        if r.code == abi.OK:
            assert r.n_activity <= c.act_cap and r.n_timer <= c.timer_cap and r.n_vh <= c.vh_cap


def test_plan_rejects_inconsistent_new_run():
    b = engine.synth_batch(4, 20, seed=9)
    for w in range(b.n_wfs):
        if b.wfs[w].newrun >= 0:
            b.wfs[b.wfs[w].newrun].run_id += 1
            break
    with pytest.raises(RuntimeError):
        engine.plan(b)


def test_fingerprint32_shard_mapping():
    """farmhash Fingerprint32 % numShards (common/util.go:249-252).  No reference
    test pins concrete hash values (parity unpinned); check determinism, range and
    spread instead."""
    L = abi.lib()
    ids = [f"workflow-{i}".encode() for i in range(20000)]
    shards = [L.cdr_workflow_id_to_shard(s, len(s), 16384) for s in ids]
    assert all(0 <= x < 16384 for x in shards)
    assert shards == [L.cdr_workflow_id_to_shard(s, len(s), 16384) for s in ids]
    counts = np.bincount([L.cdr_workflow_id_to_shard(s, len(s), 8) for s in ids], minlength=8)
    assert counts.min() > 2000  # roughly uniform
    for n in range(0, 40):  # every length branch of Hash32
        s = bytes(range(65, 65 + n))
        assert L.cdr_fingerprint32(s, n) == L.cdr_fingerprint32(s, n)


def test_engine_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        engine.Engine(0)


def test_fast_path_eligibility():
    """The planner routes sequential-activity histories (C1/C2 shapes, NDC or local
    builder) to the fast-path kernel and everything else to the general one."""
    for cfg, builder, expect_all in ((1, -1, True), (2, -1, True), (2, abi.BUILDER_LOCAL, True),
                                     (2, abi.BUILDER_2DC, False), (3, -1, False), (4, -1, False)):
        b = engine.synth_batch(cfg, 256, seed=7, builder=builder)
        nf, ns = engine.fast_slices(b)
        assert (nf == ns) if expect_all else (nf < ns), (cfg, builder, nf, ns)
    pl = engine.plan(engine.synth_batch(2, 64, seed=1))
    assert all(pl.caps[w].flags & abi.CAP_FAST for w in range(64))


def test_wave_slices_plan_and_pack():
    """CDR_PLAN_WAVE: divergent entries get one wave slice each (after the lane
    slices), their events packed 64 to a row (event k in row k/64, lane k%64)."""
    b = engine.synth_batch(3, 150, seed=11)
    pl = engine.plan(b)
    L = abi.lib()
    ns, rows, nw = C.c_uint32(), C.c_uint64(), C.c_uint32()
    mode = abi.PLAN_WAVE | abi.PLAN_WAVE_ALL  # also the lane-friendly (CAP_LANE) entries
    L.cdr_plan_slices_ex(b.wfs, pl.caps, b.n_wfs, mode, None, None, None, None, C.byref(ns),
                         C.byref(rows), C.byref(nw))
    lane = np.zeros(ns.value * 64, np.int32)
    slen = np.zeros(ns.value, np.uint32)
    row0 = np.zeros(ns.value, np.uint64)
    flags = np.zeros(ns.value, np.uint32)
    L.cdr_plan_slices_ex(b.wfs, pl.caps, b.n_wfs, mode, lane.ctypes.data, slen.ctypes.data,
                         row0.ctypes.data, flags.ctypes.data, C.byref(ns), C.byref(rows), C.byref(nw))
    waves = np.nonzero(flags & abi.SLICE_WAVE)[0]
    assert len(waves) == nw.value > 0
    wave_wfs = {int(lane[s * 64]) for s in waves}
    assert all((pl.caps[w].flags & abi.CAP_WAVE) for w in wave_wfs)
    assert all((lane[s * 64 + 1:(s + 1) * 64] == -1).all() for s in waves)
    # every entry exactly once
    placed = sorted(int(x) for x in lane if x >= 0)
    assert placed == list(range(b.n_wfs))
    # scratch planning keeps the wave flag and gives wave slices no slots
    words, nf = C.c_uint64(), C.c_uint32()
    act = np.zeros(ns.value, np.uint32)
    L.cdr_plan_scratch(pl.caps, lane.ctypes.data, ns.value, None, act.ctypes.data, None, flags.ctypes.data,
                       C.byref(words), C.byref(nf))
    assert (flags[waves] == abi.SLICE_WAVE).all() and (act[waves] == 0).all()
    # pack and read back one wave workflow
    aw = L.cdr_plan_arena_words(C.byref(b.cstruct()))
    slab = np.zeros(int(rows.value) * 64 * abi.EL_BYTES, np.uint8)
    arena = np.zeros(max(1, aw), np.uint64)
    s_ = abi.CdrSlices(n_slices=ns.value, n_rows=rows.value, arena_words=aw)
    s_.slice_row0, s_.slice_len, s_.lane_wf = row0.ctypes.data, slen.ctypes.data, lane.ctypes.data
    s_.slab, s_.arena, s_.slice_flags = slab.ctypes.data, arena.ctypes.data, flags.ctypes.data
    assert L.cdr_pack_slices(C.byref(b.cstruct()), C.byref(s_), 2) == 0
    cols = abi.slab_columns(slab)
    s = int(waves[len(waves) // 2])
    w = int(lane[s * 64])
    d = b.wfs[w]
    n = int(d.ev_len)
    assert slen[s] == (n + 63) // 64
    r0 = int(row0[s])
    got = cols["event_id"][r0 * 64:(r0 + int(slen[s])) * 64][:n]
    want = [b.events[d.ev_off + k].event_id for k in range(n)]
    assert got.tolist() == want
    tf = cols["type_flags"][r0 * 64:(r0 + int(slen[s])) * 64]
    assert [int(x) & 0xFF for x in tf[:n]] == [b.events[d.ev_off + k].type for k in range(n)]
    assert all((int(x) & 0xFF) == 0xFF for x in tf[n:])


def test_register_table_entries_stay_in_lane_slices():
    """The register-table caps (CDR_CAP_REG / REG2) keep a divergent history in a lane
    slice under CDR_PLAN_WAVE (other CDR_CAP_WAVE entries get wave slices: the general lane
    kernel is only the fallback for what fits neither); PLAN_WAVE_ALL sends them to waves."""
    b = engine.synth_batch(3, 300, seed=12)
    pl = engine.plan(b)
    lane_ok = [w for w in range(b.n_wfs) if pl.caps[w].flags & abi.CAP_LANE]
    assert lane_ok and all(pl.caps[w].flags & abi.CAP_WAVE for w in lane_ok)
    for w in lane_ok:
        c = pl.caps[w]
        assert c.act_live <= 6 and c.timer_live <= 10 and b.wfs[w].ev_len <= 512
    n_all = engine.slice_kinds(b, pl, abi.PLAN_WAVE | abi.PLAN_WAVE_ALL)[1]
    n_def = engine.slice_kinds(b, pl, abi.PLAN_WAVE)[1]
    keep = [w for w in range(b.n_wfs) if (pl.caps[w].flags & abi.CAP_WAVE) and
            (pl.caps[w].flags & (abi.CAP_REG | abi.CAP_REG2))]
    assert keep and n_def == n_all - len(keep)
    # the small-table corner carries CDR_CAP_REG too
    assert all(pl.caps[w].flags & abi.CAP_REG for w in range(b.n_wfs) if pl.caps[w].flags & abi.CAP_REG0)


def test_long_histories_get_wave_slices():
    """CDR_PLAN_WAVE's long-history rule (cdr.h CDR_PLAN_NO_LONG): a register-table history
    longer than T = max(CDR_LONG_MIN, CDR_LONG_FACTOR x lane events per resident slot) — T /
    CDR_LONG_REG2_DIV for CDR_CAP_REG2 — gets a wave slice of its own; CDR_PLAN_NO_LONG
    keeps it in a lane slice."""
    b = engine.synth_batch(4, 3000, seed=13)
    pl = engine.plan(b)
    regcap = abi.CAP_REG | abi.CAP_REG2
    flags = [pl.caps[w].flags for w in range(b.n_wfs)]
    lens = [int(b.wfs[w].ev_len) for w in range(b.n_wfs)]
    lane_ev = sum(n for f, n in zip(flags, lens) if not (f & abi.CAP_WAVE) or (f & regcap))
    thr = max(1024, 2 * (lane_ev // (64 * 2048)))
    thr2 = max(512, thr // 2)
    divergent = sum(1 for f in flags if (f & abi.CAP_WAVE) and not (f & regcap))
    long_ = sum(1 for f, n in zip(flags, lens) if (f & abi.CAP_WAVE) and (f & regcap) and
                n > (thr if f & abi.CAP_REG else thr2))
    assert long_ > 0
    assert engine.slice_kinds(b, pl, abi.PLAN_WAVE)[1] == divergent + long_
    assert engine.slice_kinds(b, pl, abi.PLAN_WAVE | abi.PLAN_NO_LONG)[1] == divergent


def _plan(b, pl, mode):
    L = abi.lib()
    ns, rows, nw = C.c_uint32(), C.c_uint64(), C.c_uint32()
    L.cdr_plan_slices_ex(b.wfs, pl.caps, b.n_wfs, mode, None, None, None, None, C.byref(ns), C.byref(rows),
                         C.byref(nw))
    lane = np.zeros(ns.value * 64, np.int32)
    slen = np.zeros(ns.value, np.uint32)
    row0 = np.zeros(ns.value, np.uint64)
    flags = np.zeros(ns.value, np.uint32)
    L.cdr_plan_slices_ex(b.wfs, pl.caps, b.n_wfs, mode, lane.ctypes.data, slen.ctypes.data, row0.ctypes.data,
                         flags.ctypes.data, C.byref(ns), C.byref(rows), C.byref(nw))
    return lane.reshape(-1, 64), slen, row0, flags


def test_par_slices_plan():
    """CDR_PLAN_PAR: the long register-table histories the long-history rule would give wave
    slices become the FIRST slices, CDR_PAR_LANES (16) to a slice, flagged CDR_SLICE_PAR, and
    balanced: longest-first into the lightest slice, so the summed lengths of any two slices
    differ by at most one history's length; the scratch planner keeps the flag (register-table lanes); the class
    ranges leave them out (they are launched as slices 0 .. n_par - 1)."""
    b = engine.synth_batch(4, 3000, seed=13)
    pl = engine.plan(b)
    L = abi.lib()
    lw, _, _, fw = _plan(b, pl, abi.PLAN_WAVE)
    lp, slen, row0, fp = _plan(b, pl, abi.PLAN_WAVE | abi.PLAN_PAR)
    n_long = int(((fw & abi.SLICE_WAVE) != 0).sum()) - int(((fp & abi.SLICE_WAVE) != 0).sum())
    par = np.nonzero(fp & abi.SLICE_PAR)[0]
    assert n_long > 0 and len(par) == (n_long + 15) // 16
    assert (par == np.arange(len(par))).all()  # the first slices
    ws = [int(x) for s in par for x in lp[s] if x >= 0]
    assert len(ws) == n_long and all((lp[s][16:] == -1).all() for s in par)
    lens = [int(b.wfs[w].ev_len) for w in ws]
    for s in par:  # lanes filled from 0
        k = int((lp[s] >= 0).sum())
        assert (lp[s][:k] >= 0).all()
    sums = [sum(int(b.wfs[w].ev_len) for w in lp[s] if w >= 0) for s in par]
    if len(par) > 1:
        assert max(sums) - min(sums) <= max(lens)
    assert all(pl.caps[w].flags & (abi.CAP_REG | abi.CAP_REG2) for w in ws)
    assert all(int(slen[s]) == max(int(b.wfs[w].ev_len) for w in lp[s] if w >= 0) for s in par)
    assert sorted(int(x) for x in lp.ravel() if x >= 0) == list(range(b.n_wfs))  # every entry once
    words, nf = C.c_uint64(), C.c_uint32()
    L.cdr_plan_scratch(pl.caps, lp.ctypes.data, len(fp), None, None, None, fp.ctypes.data, C.byref(words),
                       C.byref(nf))
    assert (fp[par] == abi.SLICE_PAR).all()
    lo, hi = (C.c_uint32 * 6)(), (C.c_uint32 * 6)()
    L.cdr_plan_class_ranges(fp.ctypes.data, len(fp), lo, hi)
    assert min(lo[c] for c in range(6) if hi[c]) >= len(par)


def test_par_solo_plan():
    """CDR_PLAN_PAR_SOLO (task batches): the same long register-table histories as CDR_PLAN_PAR,
    each alone in lane 0 of its own PAR slice (the first slices, longest first), the 512 longest
    at most; every entry still planned once."""
    b = engine.synth_batch(4, 3000, seed=13)
    pl = engine.plan(b)
    lp, slen, _, fp = _plan(b, pl, abi.PLAN_WAVE | abi.PLAN_PAR)
    ls, slen1, _, fs = _plan(b, pl, abi.PLAN_WAVE | abi.PLAN_PAR | abi.PLAN_PAR_SOLO)
    par, par1 = np.nonzero(fp & abi.SLICE_PAR)[0], np.nonzero(fs & abi.SLICE_PAR)[0]
    ws = sorted(int(x) for s in par for x in lp[s] if x >= 0)
    assert (par1 == np.arange(len(par1))).all() and len(par1) == min(len(ws), 512)
    assert all(ls[s][0] >= 0 and (ls[s][1:] == -1).all() for s in par1)
    ws1 = [int(ls[s][0]) for s in par1]
    assert len(ws) > 0 and (sorted(ws1) == ws if len(ws) <= 512 else len(ws1) == 512)
    lens = [int(b.wfs[w].ev_len) for w in ws1]
    assert lens == sorted(lens, reverse=True)
    assert all(int(slen1[s]) == int(b.wfs[int(ls[s][0])].ev_len) for s in par1)
    assert sorted(int(x) for x in ls.ravel() if x >= 0) == list(range(b.n_wfs))


def test_par_slices_capped():
    """At most CDR_PAR_MAX_SLICES PAR slices (env CDR_PAR_MAX here, read once per process, so
    in a child process): the longest histories keep them, the rest return to the register-table
    lane slices, and every entry is still planned once."""
    code = r"""
import numpy as np
from cadence_amd import abi, engine
import importlib.util, sys
spec = importlib.util.spec_from_file_location("th", "tests/test_host.py")
th = importlib.util.module_from_spec(spec); spec.loader.exec_module(th)
b = engine.synth_batch(4, 3000, seed=13)
pl = engine.plan(b)
lp, _, _, fp = th._plan(b, pl, abi.PLAN_WAVE | abi.PLAN_PAR)
par = np.nonzero(fp & abi.SLICE_PAR)[0]
assert len(par) == 2, len(par)
ws = [int(x) for s in par for x in lp[s] if x >= 0]
rest = [int(x) for s in range(len(par), len(fp)) for x in lp[s]
        if x >= 0 and pl.caps[x].flags & (abi.CAP_REG | abi.CAP_REG2)]
assert len(ws) == 32 and min(b.wfs[w].ev_len for w in ws) >= max(b.wfs[w].ev_len for w in rest)
assert sorted(int(x) for x in lp.ravel() if x >= 0) == list(range(b.n_wfs))
print("ok")
"""
    env = dict(os.environ, CDR_PAR_MAX="2")
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-2000:]


def test_register_lanes_ordered_by_entity_counts():
    """Within a length class, register-table lanes follow their entity counts (scheduled
    activities, then started timers, then initiated externals, descending), so that the
    class-sorted blocks' aligned regions carry little padding."""
    b = engine.synth_batch(3, 2000, seed=17)
    pl = engine.plan(b)
    lp, _, _, _ = _plan(b, pl, abi.PLAN_WAVE)
    order = [int(x) for x in lp.ravel() if x >= 0]
    reg = [w for w in order if (pl.caps[w].flags & (abi.CAP_REG | abi.CAP_REG2 | abi.CAP_REG0)) and
           not (pl.caps[w].flags & abi.CAP_FAST)]
    lcl = lambda w: int(np.log2(float(b.wfs[w].ev_len) + 1.0) * 16.0)  # noqa: E731
    cnt = _entity_counts(b)
    key = lambda w: tuple(cnt[w])  # noqa: E731
    pairs = 0
    for a, c in zip(reg, reg[1:]):
        grp = lambda w: (pl.caps[w].flags & abi.CAP_REG0, pl.caps[w].flags & abi.CAP_REG)  # noqa: E731
        if grp(a) == grp(c) and lcl(a) == lcl(c):
            assert key(a) >= key(c), (a, c, key(a), key(c))
            pairs += 1
    assert pairs > 100


def _entity_counts(b):
    """Per entry: (scheduled activities, started user timers, initiated children + request-
    cancels + signals) — the lane planner's ordering counts, from the events."""
    import ctypes as C
    words = C.sizeof(abi.CdrEvent) // 4
    ty = np.frombuffer(b.events, dtype=np.uint32).reshape(-1, words)[:, abi.CdrEvent.type.offset // 4]
    wf = np.ctypeslib.as_array(b.wfs)
    out = np.zeros((b.n_wfs, 3), np.int64)
    E = abi.EV
    for j, types in enumerate(([E["ActivityTaskScheduled"]], [E["TimerStarted"]],
                               [E["StartChildWorkflowExecutionInitiated"],
                                E["RequestCancelExternalWorkflowExecutionInitiated"],
                                E["SignalExternalWorkflowExecutionInitiated"]])):
        hit = np.isin(ty, types).astype(np.int64)
        cum = np.concatenate([[0], np.cumsum(hit)])
        off, ln = wf["ev_off"].astype(np.int64), wf["ev_len"].astype(np.int64)
        out[:, j] = cum[off + ln] - cum[off]
    return out


def _order_key(cnt):
    sat = lambda v, bits: np.minimum(v, (1 << bits) - 1)  # noqa: E731
    return (sat(cnt[:, 0], 10) << 22) | (sat(cnt[:, 1], 11) << 11) | sat(cnt[:, 2], 11)


@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_caps_pending_tables_live_bound(cfg):
    """cdr_wf_caps: order_key packs the entity counts; the five pending tables' capacities
    are peak live sets — at most the counts, at least the rows the oracle persists."""
    import oracle
    b = engine.synth_batch(cfg, 1500, seed=29 + cfg, error_rate=0.0)
    pl = engine.plan(b)
    caps = np.ctypeslib.as_array(pl.caps)
    cnt = _entity_counts(b)
    assert np.array_equal(caps["order_key"].astype(np.int64), _order_key(cnt))
    assert (caps["act_cap"] <= cnt[:, 0]).all() and (caps["timer_cap"] <= cnt[:, 1]).all()
    assert (caps["act_cap"] == caps["act_live"]).all()
    out = oracle.replay(b, pl)
    res = np.ctypeslib.as_array(out.result)
    for f, c in (("n_activity", "act_cap"), ("n_timer", "timer_cap"), ("n_child", "child_cap"),
                 ("n_cancel", "cancel_cap"), ("n_signal", "signal_cap")):
        assert (res[f][:b.n_wfs] <= caps[c]).all(), f
    assert int(caps["act_cap"].sum()) < int(cnt[:, 0].sum()) or cnt[:, 0].sum() == 0


def test_lane_order_restated():
    """Lane slices without wave/PAR routing (plan mode 0): entries in kernel-group order
    (fast, 3-, 6-, 12-activity register tables, general), within a group by length class
    (16 per octave, descending), then — register-table groups — scheduled activities, started
    timers and initiated externals, then working-slot footprint and length (all descending),
    stable; each group starts a fresh slice (host.cpp cdr_plan_slices_ex)."""
    import math
    for cfg in (2, 3, 4, 5):
        b = engine.synth_batch(cfg, 3000, seed=17 + cfg)
        pl = engine.plan(b)
        lane, slen, _, _ = _plan(b, pl, 0)
        caps = np.ctypeslib.as_array(pl.caps)
        lens = np.ctypeslib.as_array(b.wfs)["ev_len"].astype(np.int64)

        def group(w):
            f = int(caps["flags"][w])
            return (0 if f & abi.CAP_FAST else 1 if f & abi.CAP_REG0 else 2 if f & abi.CAP_REG else
                    3 if f & abi.CAP_REG2 else 4)

        okey = _order_key(_entity_counts(b))

        def key(w):
            g = group(w)
            counts = 1 <= g <= 3
            slots = int(caps["act_live"][w]) * 12 + int(caps["timer_live"][w]) * 4  # CDR_ACT/TIM_PLANES
            return (g, -int(math.log2(lens[w] + 1.0) * 16.0), -int(okey[w]) if counts else 0, -slots, -int(lens[w]))
        order = sorted(range(b.n_wfs), key=key)  # Python's sort is stable
        expect = []
        for i, w in enumerate(order):
            if i and group(w) != group(order[i - 1]):
                expect += [-1] * (-len(expect) % 64)
            expect.append(w)
        expect += [-1] * (-len(expect) % 64)
        assert lane.ravel().tolist() == expect, cfg
        exp_len = [max([int(lens[w]) for w in expect[s:s + 64] if w >= 0], default=0)
                   for s in range(0, len(expect), 64)]
        assert slen.tolist() == exp_len


def test_bench_traffic_only_for_its_build(tmp_path, monkeypatch):
    """bench.load_traffic uses a PMC summary only when it was collected on this very build of
    libcdr.so (same SHA-1); another build's summary is reported stale, a missing one absent."""
    import json
    import bench
    (tmp_path / "profiles").mkdir()
    monkeypatch.setattr(bench, "HERE", str(tmp_path))
    monkeypatch.setattr(bench, "lib_sha1", lambda: "a" * 40)
    t, note = bench.load_traffic("C9-1wf-sliced")
    assert t is None and "no PMC summary" in note
    rec = {"workload": "C9-1wf-sliced", "lib_sha1": "b" * 40, "bytes_per_launch": 1.0e9}
    (tmp_path / "profiles" / "traffic_C9-1wf-sliced.json").write_text(json.dumps(rec))
    t, note = bench.load_traffic("C9-1wf-sliced")
    assert t is None and "stale" in note
    rec["lib_sha1"] = "a" * 40
    (tmp_path / "profiles" / "traffic_C9-1wf-sliced.json").write_text(json.dumps(rec))
    t, note = bench.load_traffic("C9-1wf-sliced")
    assert t["bytes_per_launch"] == 1.0e9 and not note
