"""On-device history decode (cdr/ingest.h, csrc/ingest.hip).

CPU (no GPU): the decode restatement (oracle/thrift_decode.py) pinned to the reference's
golden thriftrw bytes (common/codec/version0Thriftrw_test.go:42-64) and the codec's two
error cases (:87-104); the synthetic encoder (csrc/thrift_enc.cpp) round-trips every
config through the restatement (decode(encode(batch)) == batch up to a renaming of
handles); malformed blobs report the codec / protocol errors.

GPU: the device decode == the restatement record for record (events, search-attribute
pairs, reset points, string table, statuses) on every config and on corrupted input;
at 100k workflows the decode round-trips the synthetic population; replaying the
decoded batch gives the same outputs as replaying the original (strings compared)."""
import ctypes as C
import struct

import numpy as np
import pytest

from cadence_amd import abi, engine, ingest
from oracle import thrift_decode as TD

# version0Thriftrw_test.go:42-64: HistoryEvent{Version 1234, EventId 130, Timestamp
# 112345132134, EventType RequestCancelExternalWorkflowExecutionInitiated,
# RequestCancelExternal...Attributes{Domain, WorkflowExecution{WorkflowId, RunId},
# ChildWorkflowOnly true, Control}} with the codec preamble
GOLDEN = bytes([
    89, 10, 0, 10, 0, 0, 0, 0, 0, 0, 0, 130, 10, 0, 20, 0, 0, 0, 26, 40, 74, 172, 102,
    8, 0, 30, 0, 0, 0, 23, 10, 0, 35, 0, 0, 0, 0, 0, 0, 4, 210, 12, 1, 44, 11, 0, 20,
    0, 0, 0, 25, 115, 111, 109, 101, 32, 114, 97, 110, 100, 111, 109, 32, 116, 97, 114,
    103, 101, 116, 32, 100, 111, 109, 97, 105, 110, 12, 0, 30, 11, 0, 10, 0, 0, 0, 30,
    115, 111, 109, 101, 32, 114, 97, 110, 100, 111, 109, 32, 116, 97, 114, 103, 101,
    116, 32, 119, 111, 114, 107, 102, 108, 111, 119, 32, 73, 68, 11, 0, 20, 0, 0, 0, 25,
    115, 111, 109, 101, 32, 114, 97, 110, 100, 111, 109, 32, 116, 97, 114, 103, 101, 116,
    32, 114, 117, 110, 32, 73, 68, 0, 11, 0, 40, 0, 0, 0, 19, 115, 111, 109, 101, 32, 114,
    97, 110, 100, 111, 109, 32, 99, 111, 110, 116, 114, 111, 108, 2, 0, 50, 1, 0, 0,
])


def golden_history():
    """The golden HistoryEvent as the one event of a History node: list<HistoryEvent>
    embeds each struct's encoding verbatim (protocol.Binary)."""
    return bytes([0x59, 15, 0, 10, 12]) + struct.pack(">i", 1) + GOLDEN[1:] + b"\x00"


def one_blob(blob: bytes, seeds=(b"", b"emptyUuid"), domain_map=()):
    return ingest.Encoded(np.frombuffer(blob or b"\0", np.uint8).copy(), np.array([0, len(blob)], np.uint64),
                          np.array([0, 1], np.uint32), list(seeds), {}, list(domain_map))


def oracle_decode(enc: ingest.Encoded):
    return TD.decode_blobs(enc.blob_bytes.tobytes(), enc.blob_off, enc.entry_blob0, enc.seeds, enc.domain_map, abi)


def check_golden_event(e, strings):
    S = lambda h: strings[h]  # noqa: E731
    assert (e.event_id, e.version, e.timestamp, e.type) == (130, 1234, 112345132134,
                                                            abi.EV["RequestCancelExternalWorkflowExecutionInitiated"])
    x = e.a.ext
    assert S(x.domain) == b"some random target domain"
    assert (S(x.workflow_id), S(x.run_id)) == (b"some random target workflow ID", b"some random target run ID")
    assert S(x.control) == b"some random control"
    assert x.flags & abi.XF_CHILD_ONLY
    assert x.flags & abi.XF_DOMAIN_MISSING  # no domain map given: the cache lookup fails


def test_golden_bytes_oracle():
    ev, kvs, rps, ev_off, st, est, strings = oracle_decode(one_blob(golden_history()))
    assert st == [0] and est == [0] and len(ev) == 1 and ev_off == [0, 1]
    check_golden_event(ev[0], strings)
    assert ev[0].flags == abi.EVF_BATCH_FIRST


def test_golden_domain_resolution_oracle():
    seeds = [b"", b"emptyUuid", b"some random target domain", b"target-domain-id"]
    ev, *_ , strings = oracle_decode(one_blob(golden_history(), seeds, [(2, 3)]))
    x = ev[0].a.ext
    assert (x.domain, x.target_domain_id, x.flags & abi.XF_DOMAIN_MISSING) == (2, 3, 0)


def test_codec_errors_oracle():
    """version0Thriftrw_test.go:87-104: an empty blob is MissingBinaryEncodingVersion, a
    wrong first byte InvalidBinaryEncodingVersion; truncation and a negative length are
    protocol errors; a History with no events cannot be applied."""
    cases = {b"": TD.DEC_MISSING_VERSION, bytes([0x58]) + golden_history()[1:]: TD.DEC_INVALID_VERSION,
             golden_history()[:-9]: TD.DEC_TRUNCATED, bytes([0x59, 0]): TD.DEC_NO_EVENTS,
             bytes([0x59, 15, 0, 10, 12, 0xFF, 0xFF, 0xFF, 0xFF, 0]): TD.DEC_BAD_SIZE,
             bytes([0x59, 9, 0, 10, 0]): TD.DEC_BAD_TYPE}
    for blob, want in cases.items():
        ev, kvs, rps, ev_off, st, est, strings = oracle_decode(one_blob(blob))
        assert st == [want] and est == [want] and len(ev) == 0, (blob[:12], st)


# ------------------------------------------------------------ synthetic round trips
HANDLE_FIELDS = {  # union member -> handle fields (the rest compared by value)
    "started": ("workflow_type", "task_list", "cron_schedule", "parent_domain_id", "parent_workflow_id",
                "parent_run_id", "continued_run_id", "nonretriable", "memo"),
    "dt_sched": ("task_list",), "dt": ("request_id", "binary_checksum"),
    "at_sched": ("activity_id", "task_list", "nonretriable", "domain", "target_domain_id"),
    "at": ("request_id", "activity_id"),
    "timer": ("timer_id",), "ext": ("domain", "workflow_id", "run_id", "workflow_type", "signal_name", "input",
                                    "control", "target_domain_id"),
    "ref": ("run_id",), "can": ("new_execution_run_id",), "upsert": (),
}
SKIP_FIELDS = {"started": ("search_attr_off", "reset_points_off"), "upsert": ("search_attr_off",)}
# the union fields each event type's attribute struct carries on the wire (shared.thrift);
# others (set by the synthetic generator, unused by the replay) cannot round-trip
WIRE_FIELDS = {
    "DecisionTaskStarted": ("scheduled_event_id", "request_id"),
    "DecisionTaskCompleted": ("scheduled_event_id", "started_event_id", "binary_checksum"),
    "DecisionTaskTimedOut": ("scheduled_event_id", "started_event_id", "timeout_type"),
    "DecisionTaskFailed": ("scheduled_event_id", "started_event_id"),
    "ActivityTaskStarted": ("scheduled_event_id", "request_id", "attempt"),
    "ActivityTaskCompleted": ("scheduled_event_id", "started_event_id"),
    "ActivityTaskFailed": ("scheduled_event_id", "started_event_id"),
    "ActivityTaskCanceled": ("scheduled_event_id", "started_event_id"),
    "ActivityTaskTimedOut": ("scheduled_event_id", "started_event_id", "timeout_type"),
    "ActivityTaskCancelRequested": ("activity_id",), "RequestCancelActivityTaskFailed": ("activity_id",),
    "TimerStarted": ("timer_id", "start_to_fire_s"), "TimerFired": ("timer_id", "started_event_id"),
    "TimerCanceled": ("timer_id", "started_event_id"), "CancelTimerFailed": ("timer_id",),
    "StartChildWorkflowExecutionInitiated": ("domain", "workflow_id", "workflow_type", "input", "control",
                                             "parent_close_policy", "flags", "target_domain_id"),
    "SignalExternalWorkflowExecutionInitiated": ("domain", "workflow_id", "run_id", "signal_name", "input",
                                                 "control", "flags", "target_domain_id"),
    "RequestCancelExternalWorkflowExecutionInitiated": ("domain", "workflow_id", "run_id", "control", "flags",
                                                        "target_domain_id"),
    "StartChildWorkflowExecutionFailed": ("initiated_event_id",),
}


def member(t):
    """The cdr_event union member of event type t (schema.h)."""
    n = abi.EVENT_TYPES[t] if t < len(abi.EVENT_TYPES) else ""
    if n == "WorkflowExecutionStarted":
        return "started"
    if n == "DecisionTaskScheduled":
        return "dt_sched"
    if n in ("DecisionTaskStarted", "DecisionTaskCompleted", "DecisionTaskTimedOut", "DecisionTaskFailed"):
        return "dt"
    if n == "ActivityTaskScheduled":
        return "at_sched"
    if n.startswith("ActivityTask") or n == "RequestCancelActivityTaskFailed":
        return "at"
    if n in ("TimerStarted", "TimerFired", "TimerCanceled", "CancelTimerFailed"):
        return "timer"
    if n in ("StartChildWorkflowExecutionInitiated", "SignalExternalWorkflowExecutionInitiated",
             "RequestCancelExternalWorkflowExecutionInitiated"):
        return "ext"
    if n == "WorkflowExecutionContinuedAsNew":
        return "can"
    if n == "UpsertWorkflowSearchAttributes":
        return "upsert"
    if n.startswith("ChildWorkflowExecution") or n in (
            "StartChildWorkflowExecutionFailed", "RequestCancelExternalWorkflowExecutionFailed",
            "ExternalWorkflowExecutionCancelRequested", "SignalExternalWorkflowExecutionFailed",
            "ExternalWorkflowExecutionSignaled"):
        return "ref"
    return None


class Renaming:
    """orig handle -> decoded handle, checked to be a function (and injective)."""

    def __init__(self):
        self.f, self.g = {0: 0}, {0: 0}

    def same(self, a, b, what):
        if self.f.setdefault(a, b) != b or self.g.setdefault(b, a) != a:
            raise AssertionError(f"{what}: handle {a} -> {b}, but earlier {self.f[a]} / {self.g[b]}")


def round_trip_equal(src: engine.Batch, dec, limit=10**9):
    """decode(encode(src)) == src up to a consistent renaming of handles."""
    events, kvs, rps, ev_off = dec[0], dec[1], dec[2], dec[3]
    R = Renaming()
    n_ev = 0
    for w in range(src.n_wfs):
        d = src.wfs[w]
        assert ev_off[w + 1] - ev_off[w] == d.ev_len, w
        for k in range(d.ev_len):
            a, b = src.events[d.ev_off + k], events[int(ev_off[w]) + k]
            n_ev += 1
            assert (a.event_id, a.version, a.timestamp, a.task_id, a.type) == (
                b.event_id, b.version, b.timestamp, b.task_id, b.type), (w, k)
            assert bool(a.flags & abi.EVF_BATCH_FIRST) == bool(b.flags & abi.EVF_BATCH_FIRST) or k == 0
            m = member(a.type)
            if m is None:
                continue
            xa, xb = getattr(a.a, m), getattr(b.a, m)
            hf = HANDLE_FIELDS[m]
            wire = WIRE_FIELDS.get(abi.EVENT_TYPES[a.type])
            for f, _ in type(xa)._fields_:
                if f.startswith("_") or f in SKIP_FIELDS.get(m, ()) or (wire is not None and f not in wire):
                    continue
                va, vb = getattr(xa, f), getattr(xb, f)
                if m == "started" and f == "parent_domain_id" and xa.flags & abi.SF_PARENT_DOMAIN_MISSING:
                    continue  # the cache lookup failed: no ID
                if m == "ext" and f == "target_domain_id" and xa.flags & abi.XF_DOMAIN_MISSING:
                    continue
                if m == "at_sched" and f == "target_domain_id" and xa.flags & abi.AF_DOMAIN_MISSING:
                    continue
                if f in hf:
                    R.same(va, vb, f"{m}.{f}")
                else:
                    assert va == vb, (w, k, m, f, va, vb)
            if m in ("started", "upsert"):
                n = xa.search_attr_len
                for q in range(n):
                    ka, kb = src.kvs[xa.search_attr_off + q], kvs[xb.search_attr_off + q]
                    kb = kb if isinstance(kb, tuple) else (kb.key, kb.value)
                    R.same(ka.key, kb[0], "kv.key")
                    R.same(ka.value, kb[1], "kv.value")
            if m == "started" and xa.flags & abi.SF_HAS_RESET_POINTS:
                for q in range(xa.reset_points_len):
                    pa, pb = src.rps[xa.reset_points_off + q], rps[xb.reset_points_off + q]
                    assert pa.flags == pb.flags
                    for f in ("first_decision_completed_id", "created_time_nano", "expiring_time_nano"):
                        assert getattr(pa, f) == getattr(pb, f)
                    R.same(pa.binary_checksum, pb.binary_checksum, "rp.checksum")
                    R.same(pa.run_id, pb.run_id, "rp.run_id")
        if n_ev > limit:
            break
    round_trip_equal.renaming = R
    return n_ev


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5])
def test_encode_decode_round_trip_oracle(cfg):
    b = engine.synth_batch(cfg, 30, seed=0xD0 + cfg)
    enc = ingest.encode_batch(b)
    dec = oracle_decode(enc)
    assert set(dec[4]) == {0}
    assert round_trip_equal(b, dec) == len(b.events)


def test_fixture_histories_round_trip_oracle():
    """The reference's own JSON history (archival_workflow_history_v1) and the
    hand-crafted NDC branches, through the encoder and the restated decoder."""
    from cadence_amd.history import from_cadence_json
    import json
    import os
    here = os.path.join(os.path.dirname(__file__), "golden")
    doc = json.load(open(os.path.join(here, "archival_workflow_history_v1.input.json")))
    events = doc if isinstance(doc, list) else doc.get("events", doc)
    b = from_cadence_json(events, batching="each")
    dec = oracle_decode(ingest.encode_batch(b))
    assert round_trip_equal(b, dec) == len(b.events)
    S = dec[6]
    e0 = dec[0][0]
    assert S[e0.a.started.task_list] == b.strings[b.events[0].a.started.task_list].encode()


def _cross_domain_activities(missing=False):
    """Activities with no, an empty, a known and an unknown target domain
    (ActivityTaskScheduledEventAttributes.domain, shared.thrift:615)."""
    from cadence_amd.history import HistoryBuilder
    from tests import test_refresh as TR
    hb = HistoryBuilder()
    if missing:
        hb.domains_missing.add("gone-dom")
    w = hb.workflow(workflow_id="wf", run_id="run", request_id="req", retention_days=2)
    w.calls = TR._cross_domain_calls() + [[TR._act(8, "gone", "gone-dom")]]
    return hb.build(now_ns=TR.NOW)


@pytest.mark.parametrize("missing", [False, True])
def test_activity_domain_round_trip_oracle(missing):
    """Field 25 (domain) of ActivityTaskScheduled is encoded, decoded and resolved through
    the caller's domain map like the external events' domains: the decoded record carries
    the name and the cache's ID, or the domain-missing flag."""
    b = _cross_domain_activities(missing)
    enc = ingest.encode_batch(b)
    dec = oracle_decode(enc)
    assert round_trip_equal(b, dec) == len(b.events)
    S = dec[6]
    at = [e.a.at_sched for e in dec[0] if e.type == abi.EV["ActivityTaskScheduled"]]
    assert [S[x.domain] for x in at] == [b"", b"", b"remote-dom", b"gone-dom"]
    assert [bool(x.flags & abi.AF_DOMAIN_MISSING) for x in at] == [False, False, False, missing]
    assert S[at[2].target_domain_id] == b"id-of-remote-dom"


# ------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("missing", [False, True])
def test_activity_domain_decode_gpu(engine_gpu, missing):
    enc = ingest.encode_batch(_cross_domain_activities(missing))
    assert_same_decode(ingest.decode(engine_gpu, enc), oracle_decode(enc))


def decoded_tuple(d: ingest.Decoded):
    return (d.events, d.kvs, d.rps, d.ev_off, d.blob_status, d.entry_status, d.strings)


def _by_string(e, strings):
    """An event's header and union with handle fields as strings."""
    m = member(e.type)
    d = {"hdr": bytes(e)[:40]}
    if m:
        x = getattr(e.a, m)
        for f, _ in type(x)._fields_:
            v = getattr(x, f)
            d[f] = strings[v] if f in HANDLE_FIELDS[m] and v < len(strings) else v
    return d


def assert_same_decode(gpu: ingest.Decoded, ref, by_string=False):
    """Record-for-record equality; `by_string`: handle fields compared as the strings
    they name (malformed input: a field repeated inside a struct interns every
    occurrence on the device, while a record keeps the last, so the numbering may count
    strings no record names)."""
    ev, kvs, rps, ev_off, st, est, strings = ref
    assert list(gpu.blob_status) == list(st) and list(gpu.entry_status) == list(est)
    assert list(gpu.ev_off) == list(ev_off)
    assert len(gpu.events) == len(ev)
    if by_string:
        bad = [i for i in range(len(ev)) if _by_string(gpu.events[i], gpu.strings) != _by_string(ev[i], strings)]
        assert not bad, (len(bad), bad[:5], _by_string(gpu.events[bad[0]], gpu.strings), _by_string(ev[bad[0]], strings))
        assert [(gpu.strings[k.key], gpu.strings[k.value]) for k in gpu.kvs] == [(strings[a], strings[b])
                                                                               for a, b in kvs]
        return
    bad = [i for i in range(len(ev)) if bytes(gpu.events[i]) != bytes(ev[i])]
    if bad:
        i = bad[0]
        ga, ra = bytes(gpu.events[i]), bytes(ev[i])
        diff = [j for j in range(len(ga)) if ga[j] != ra[j]]
        ns = [h for h in range(min(len(gpu.strings), len(strings))) if gpu.strings[h] != strings[h]]
        raise AssertionError(f"{len(bad)} events differ; first {i} type {ev[i].type} bytes {diff[:16]} "
                             f"gpu {ga[diff[0] & ~3:(diff[0] & ~3) + 8].hex()} ref {ra[diff[0] & ~3:(diff[0] & ~3) + 8].hex()}; "
                             f"strings {len(gpu.strings)} vs {len(strings)}, first differing handle "
                             f"{ns[:3]} {[gpu.strings[h] for h in ns[:3]]} {[strings[h] for h in ns[:3]]}")
    assert [(k.key, k.value) for k in gpu.kvs] == list(kvs)
    assert [bytes(p) for p in gpu.rps] == [bytes(p) for p in rps]
    assert gpu.strings == strings


@pytest.mark.gpu
def test_golden_bytes_gpu(engine_gpu):
    d = ingest.decode(engine_gpu, one_blob(golden_history()))
    check_golden_event(d.events[0], d.strings)
    assert_same_decode(d, oracle_decode(one_blob(golden_history())))


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5])
def test_decode_matches_oracle_gpu(engine_gpu, cfg):
    b = engine.synth_batch(cfg, 60, seed=0xD0 + cfg)
    enc = ingest.encode_batch(b)
    assert_same_decode(ingest.decode(engine_gpu, enc), oracle_decode(enc))


@pytest.mark.gpu
def test_decode_errors_match_oracle_gpu(engine_gpu):
    """Corrupted blobs among good ones: every status as the restatement, the good blobs'
    records unaffected."""
    b = engine.synth_batch(3, 40, seed=9)
    enc = ingest.encode_batch(b)
    raw = bytearray(enc.blob_bytes.tobytes())
    rng = np.random.default_rng(4)
    nb = len(enc.blob_off) - 1
    for bi in rng.choice(nb, size=min(nb, 25), replace=False):
        lo, hi = int(enc.blob_off[bi]), int(enc.blob_off[bi + 1])
        kind = rng.integers(4)
        if kind == 0:
            raw[lo] = 0x58  # wrong preamble
        elif kind == 1 and hi - lo > 12:  # a byte in the middle (any wire effect)
            p = int(rng.integers(lo + 1, hi))
            raw[p] = int(rng.integers(256))
        elif kind == 2:  # negative list count
            raw[lo + 5:lo + 9] = b"\xff\xff\xff\xff"
        else:  # a length past the end
            raw[hi - 1] = 0x7F
    enc.blob_bytes = np.frombuffer(bytes(raw), np.uint8).copy()
    ref = oracle_decode(enc)
    assert len(set(ref[4])) > 1
    assert_same_decode(ingest.decode(engine_gpu, enc), ref, by_string=True)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [2, 3, 5])
def test_decoded_batch_replays_like_the_original_gpu(engine_gpu, cfg):
    """Replay(decode(encode(b))) on the GPU == the oracle's replay(b): every persisted
    field equal, handle fields through the decode's renaming (events) and the seeds
    (cdr_wf_desc strings)."""
    import oracle
    b = engine.synth_batch(cfg, 200, seed=0xE0 + cfg)
    enc = ingest.encode_batch(b)
    d = ingest.decode(engine_gpu, enc)
    assert round_trip_equal(b, decoded_tuple(d)) == len(b.events)
    ren = dict(round_trip_equal.renaming.f)
    ren.update(enc.seed_of)
    ren[b.empty_uuid] = 1
    db = ingest.to_batch(b, enc, d)
    got = engine_gpu.replay(db)
    ref = oracle.replay(b)
    n_ok = 0
    for w in range(b.n_wfs):
        ga, gb = engine.export_state(_raw(db), got, w), engine.export_state(_raw(b), ref, w)
        assert ga["result"] == gb["result"], w
        if gb["result"]["status"] != "OK":
            continue
        n_ok += 1
        rb = _renamed(gb, ren)
        for t in ("sa", "timer"):  # rows keyed by a handle come in handle order: compare as sets
            ga[t] = sorted(ga[t], key=repr)
            rb[t] = sorted(rb[t], key=repr)
        if ga != rb:
            diffs = {k: [(f, ga[k][f] if isinstance(ga[k], dict) else ga[k], rb[k][f] if isinstance(rb[k], dict)
                          else rb[k]) for f in (ga[k] if isinstance(ga[k], dict) else [0])
                         if (ga[k][f] if isinstance(ga[k], dict) else ga[k]) != (rb[k][f] if isinstance(rb[k], dict)
                                                                               else rb[k])]
                     for k in ga if ga[k] != rb.get(k)}
            raise AssertionError(f"wf {w}: {diffs}")
    assert n_ok > 0


def _raw(b):
    import dataclasses
    return dataclasses.replace(b, strings=[])


def _renamed(state, ren):
    def conv(k, v):
        if isinstance(v, dict):
            return {kk: conv(kk, x) for kk, x in v.items()}
        if isinstance(v, list):
            return [conv(k, x) for x in v]
        if k in engine._HANDLE_FIELDS and isinstance(v, int):
            return ren.get(v, ("unmapped", v))
        return v
    return conv(None, state)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5])
def test_device_plan_pack_replay_gpu(engine_gpu, cfg):
    """Decode -> device caps / host plan / device pack -> replay, all on the GPU from the
    blobs: equal to the host path (cdr_plan_caps + cdr_pack_slices + replay) on the same
    decoded batch, record for record, and the device capacities equal the host planner's."""
    import oracle
    b = engine.synth_batch(cfg, 300, seed=0xF0 + cfg)
    enc = ingest.encode_batch(b)
    d = ingest.decode(engine_gpu, enc)
    db = ingest.to_batch(b, enc, d)
    got = ingest.replay_on_device(engine_gpu, b, enc, d)
    host_pl = engine.plan(db)
    assert bytes(got.plan.caps) == bytes(host_pl.caps)
    assert bytes(got.plan.totals) == bytes(host_pl.totals)
    ref = oracle.replay(db)
    bad = engine.compare(db, got, ref)
    assert not bad, "\n".join(bad)
    assert engine.status_histogram(got) == engine.status_histogram(ref)


@pytest.mark.gpu
def test_fullsize_round_trip_gpu(engine_gpu):
    """100k workflows of config 3 (~20M events, ~2 GB of blobs): every event's
    id / version / timestamp / task id / type / batch flag equal to the original
    (numpy over the whole arrays), the attribute unions of a 20k-event sample equal up to
    the handle renaming."""
    import time
    b = engine.synth_batch(3, 100_000, seed=0x5EED0003)
    enc = ingest.encode_batch(b, threads=16)
    t0 = time.perf_counter()
    d = ingest.decode(engine_gpu, enc)
    print(f"decode {len(b.events):,} events / {len(enc.blob_off) - 1:,} blobs / {enc.blob_bytes.nbytes / 1e9:.2f} GB"
          f" in {time.perf_counter() - t0:.2f}s (incl. H2D / D2H)")
    assert d.n_bad_blobs == 0
    n = len(b.events)
    assert len(d.events) == n
    starts = np.array([b.wfs[w].ev_off for w in range(b.n_wfs)], np.uint64)
    assert np.array_equal(starts, d.ev_off[:-1]), "entries are contiguous in order in both"
    ea = np.frombuffer(b.events, np.uint8).reshape(n, -1)
    eb = np.frombuffer(d.events, np.uint8).reshape(n, -1)
    assert np.array_equal(ea[:, :36], eb[:, :36])  # event_id, version, timestamp, task_id, type
    fa = ea[:, 36:40].copy().view(np.uint32)[:, 0] & abi.EVF_BATCH_FIRST
    fb = eb[:, 36:40].copy().view(np.uint32)[:, 0] & abi.EVF_BATCH_FIRST
    assert np.array_equal(fa, fb)
    # unions: a sample of whole entries through the renaming check
    rng = np.random.default_rng(1)
    ws = np.sort(rng.choice(b.n_wfs, size=100, replace=False))
    sub_w = (abi.CdrWfDesc * len(ws))(*[b.wfs[int(w)] for w in ws])
    sub_off = np.array([d.ev_off[int(w)] for w in ws] + [0], np.uint64)
    import dataclasses
    src = dataclasses.replace(b, wfs=sub_w)
    ev_off = [int(d.ev_off[int(w)]) for w in ws]
    ev_off = [(ev_off[i], ev_off[i] + sub_w[i].ev_len) for i in range(len(ws))]
    flat_off = [0]
    for w in range(len(ws)):
        flat_off.append(flat_off[-1] + sub_w[w].ev_len)
    evs = [d.events[k] for lo, hi in ev_off for k in range(lo, hi)]
    for w in range(len(ws)):
        sub_w[w].ev_off = b.wfs[int(ws[w])].ev_off
    n_checked = round_trip_equal(src, (evs, d.kvs, d.rps, flat_off))
    assert n_checked == sum(sub_w[w].ev_len for w in range(len(ws)))
    del sub_off
