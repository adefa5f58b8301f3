"""The Cassandra persisted form: each row's CQL bound values, as the
Cassandra persistence's statements bind them (cassandraPersistenceUtil.go updateExecution
:625-890, updateActivityInfos :1264-1337, updateTimerInfos :1384-1422,
updateChildExecutionInfos :1444-1503, updateRequestCancelInfos :1530-1568,
updateSignalInfos :1590-1631; templates cassandraPersistence.go:114-306,439-520; column
types schema/cassandra/cadence/schema.cql:23-228).

CPU: the restatement (oracle/cql_values.py) decodes under the statements' column types with
every byte consumed, and its fixed points (the empty run / domain IDs, emptyInitiatedID,
event_store_version, timestamps in milliseconds, the zero time, nil blobs) are checked by
hand.  gocql is not vendored in the reference and no reference test holds CQL bytes, so
the layout is pinned by the templates and the schema, not by a reference vector.
GPU (-m gpu): encode_var.hip's CQL form (cdr_encode_cql_async) == the restatement byte for
byte, status for status, for every row of every OK entry of the synthetic configs.
"""
import struct

import numpy as np
import pytest

from cadence_amd import abi, engine
from oracle import cql_values as cq
from oracle import thrift_binary as tb

from .test_encode_var import _S, list_body, memo_body, persist_for, string_table, uuid_of


def test_uuid_parse_is_gocqls():
    u = uuid_of(3)
    assert cq.parse_uuid(u.encode()) == bytes.fromhex(u.replace("-", ""))
    assert cq.parse_uuid(u.replace("-", "").upper().encode()) == bytes.fromhex(u.replace("-", ""))
    assert cq.parse_uuid(b"ab-cd" + b"0" * 28) == bytes.fromhex("abcd" + "0" * 28)  # '-' after an even count
    for bad in (b"", b"a-bcd" + b"0" * 28, b"0" * 31, b"0" * 33, b"g" * 32):
        with pytest.raises(cq.BadUUID):
            cq.parse_uuid(bad)
    assert cq.parse_uuid(cq.EMPTY_RUN_ID) == bytes.fromhex("30000000" "0000" "f000" "f000" "000000000000")


def test_value_encodings():
    assert cq.val(None) == b"\xff\xff\xff\xff" and cq.val(b"") == b"\x00\x00\x00\x00"
    assert cq.timestamp(1_600_000_000_123_999_999) == struct.pack(">iq", 8, 1_600_000_000_123)
    assert cq.timestamp(-1) == struct.pack(">iq", 8, -1)  # floor, as Unix()*1e3 + Nanosecond()/1e6
    assert cq.timestamp(0, zero=True) == b"\x00\x00\x00\x00"
    assert cq.list_text(list_body(5)) == cq.val(struct.pack(">i", 2) + b"".join(
        struct.pack(">i", len(e)) + e for e in (b"err5_0", b"err5_1")))


def test_rows_decode_under_the_schema():
    strs = string_table(64, memo=[9], lists=[12])
    S = _S(strs)
    a = abi.CdrActivityInfo(version=3, schedule_id=5, scheduled_event_batch_id=4, scheduled_time=77_000_000,
                            started_id=-23, expiration_time=99_000_000, cancel_request_id=-23, activity_id=7,
                            task_list=11, nonretriable=12, s2s=1, s2c=2, stc=3, hb=4, flags=0x2, backoff_coefficient=2.5)
    v = cq.decode(cq.activity(a, S), cq.ACTIVITY_TYPES)
    assert v[0] == v[2] == struct.pack(">q", 5) and v[4] is None and v[7] is None and v[11] is None
    assert v[5] == struct.pack(">q", 77) and v[8] == b"" and v[18] == b""  # not started: the zero time
    assert v[9] == strs[7] and v[23] == b"\x01" and v[25] == struct.pack(">d", 2.5)
    assert v[29] == list_body(12)[1:] and v[32] is None and v[33] == b""
    t = abi.CdrTimerInfo(version=1, timer_id=13, started_id=6, expiry_time=5_000_000_123, task_id=1)
    v = cq.decode(cq.timer(t, S), cq.TIMER_TYPES)
    assert v[0] == v[2] == strs[13] and v[4] == struct.pack(">q", 5000)
    c = abi.CdrChildInfo(version=1, initiated_id=9, initiated_event_batch_id=8, started_id=-23, create_request_lo=1,
                         create_request_hi=2, started_workflow_id=3, started_run_id=0, domain_name=7, workflow_type=11,
                         parent_close_policy=2)
    v = cq.decode(cq.child(c, S), cq.CHILD_TYPES)
    assert v[7] == cq.parse_uuid(cq.EMPTY_RUN_ID) and v[9] == bytes.fromhex("0" * 15 + "2" + "0" * 15 + "1")
    c.started_run_id = 4  # not a UUID
    with pytest.raises(cq.BadUUID):
        cq.child(c, S)
    r = abi.CdrCancelInfo(version=1, initiated_event_batch_id=2, initiated_id=3, cancel_request_lo=4,
                          cancel_request_hi=5)
    assert cq.decode(cq.cancel(r, S), cq.CANCEL_TYPES)[4] == tb.uuid_text(4, 5).encode()
    g = abi.CdrSignalInfo(version=1, initiated_event_batch_id=2, initiated_id=3, signal_request_lo=4,
                          signal_request_hi=5, signal_name=7, input=3, control=0)
    v = cq.decode(cq.signal(g, S), cq.SIGNAL_TYPES)
    assert v[6] == strs[3] and v[7] is None


@pytest.mark.parametrize("builder", [abi.BUILDER_LOCAL, abi.BUILDER_2DC, abi.BUILDER_NDC])
def test_execution_values_decode(builder):
    strs = string_table(64, memo=[9], lists=[12])
    S = _S(strs)
    x = abi.CdrExecInfo(domain_id=1, workflow_id=7, run_id=5, create_request_id=13, task_list=11, workflow_type=3,
                        memo=9, nonretriable=12, branch_tree_id=17, branch_id_lo=1, branch_id_hi=2,
                        flags=0x001 | 0x002 | 0x010 | 0x020 | 0x040 | (0x100 if builder == abi.BUILDER_NDC else 0x008),
                        signal_count=4, attempt=2, next_event_id=42)
    repl = abi.CdrReplState(current_version=7, start_version=5, last_write_version=7, last_write_event_id=40,
                            lri_mask=0b101)
    repl.lri_version[0], repl.lri_last_event_id[0], repl.lri_version[2], repl.lri_last_event_id[2] = 1, 2, 3, 4
    rp = abi.CdrResetPoint(binary_checksum=21, run_id=1, first_decision_completed_id=4, created_time_nano=5, flags=0x7F)
    vals = cq.execution(x, builder, S, persist_for(3), repl=repl, vh_items=[(3, 1), (9, 4)], rps=[(rp, S)],
                        sa=[(13, 15)], cluster_names=[23, 25, 27])
    v = cq.decode(vals, cq.EXEC_TYPES + cq.EXEC_TAIL[builder])
    assert v[3] == cq.parse_uuid(cq.EMPTY_DOMAIN_ID) and v[4] == b"" and v[6] == struct.pack(">q", -7)
    assert v[8] is None and v[42][:1] == b"\x59" and v[43] == b"thriftrw" and v[52] == struct.pack(">i", -1)
    assert (v[53] is None) == (builder == abi.BUILDER_NDC)
    assert v[56] == struct.pack(">i", 1) + cq.val(strs[13]) + cq.val(strs[15])
    assert v[57] == tb._memo_fields(memo_body(9))[2:]
    assert v[-1 if builder != abi.BUILDER_NDC else -3] == struct.pack(">q", 42)  # next_event_id
    if builder == abi.BUILDER_2DC:
        lri = v[62]
        assert struct.unpack(">i", lri[:4])[0] == 2 and cq.val(strs[23]) in lri and cq.val(strs[27]) in lri
    if builder == abi.BUILDER_NDC:
        assert v[-1] == b"thriftrw" and v[-2][:1] == b"\x59"


# ---------------------------------------------------------------- GPU
UUID_FIELDS = {"exec": ("domain_id", "run_id", "create_request_id", "parent_domain_id", "parent_run_id"),
               "child": ("started_run_id",)}


def _table(b, out):
    """A string table over every handle the outputs name, UUID texts where a uuid column
    reads the handle (a few left as non-UUIDs to exercise the status), Memo / list bodies
    where those are read."""
    from .test_encode_var import HANDLE_FIELDS
    hmax, memo, lists, uuids = 64, set(), set(), set()
    for w in range(b.n_wfs):
        if out.result[w].code != abi.OK:
            continue
        x = out.exec[w]
        hmax = max([hmax] + [getattr(x, f) for f in HANDLE_FIELDS["exec"]])
        uuids |= {getattr(x, f) for f in UUID_FIELDS["exec"] if getattr(x, f)}
        if x.memo:
            memo.add(x.memo)
        if x.nonretriable:
            lists.add(x.nonretriable)
        for t in ("act", "timer", "child", "signal", "rp", "sa"):
            for r in out.rows(w, t):
                hs = HANDLE_FIELDS.get(t, ("timer_id",))
                hmax = max([hmax] + [getattr(r, f) for f in hs])
                if t == "act" and r.nonretriable:
                    lists.add(r.nonretriable)
                if t == "child" and r.started_run_id:
                    uuids.add(r.started_run_id)
    strs = string_table(hmax + 1, memo, lists - memo)
    for h in sorted(uuids - memo - lists):
        if h % 17 != 3:
            strs[h] = uuid_of(h).encode()
    return strs


def _expect(fn):
    try:
        return fn(), 0
    except cq.BadUUID:
        return None, 1


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_gpu_cql_values(engine_gpu, cfg):
    b = engine.synth_batch(cfg, 300, seed=0x5EED0700 + cfg)
    out = engine_gpu.replay(b)
    strs = _table(b, out)
    S = _S(strs)
    makers = {"act": cq.activity, "timer": cq.timer, "child": cq.child, "cancel": cq.cancel, "signal": cq.signal}
    types = {"act": cq.ACTIVITY_TYPES, "timer": cq.TIMER_TYPES, "child": cq.CHILD_TYPES, "cancel": cq.CANCEL_TYPES,
             "signal": cq.SIGNAL_TYPES}
    for table, mk in makers.items():
        got, codes = engine_gpu.encode_blobs(b, out, table, strs, form="cql")
        n = 0
        for w in range(b.n_wfs):
            if out.result[w].code != abi.OK:
                continue
            base = getattr(out.plan.caps[w], table + "_off")
            for j, row in enumerate(out.rows(w, table)):
                want, code = _expect(lambda: mk(row, S))
                r = base + j
                assert codes[r] == code, (table, w, j, codes[r], code)
                if code == 0:
                    assert got[r] == want, (table, w, j)
                    cq.decode(got[r], types[table])
                n += 1
        if cfg in (3, 4, 5):
            assert n > 0, table
    persist = (abi.CdrExecPersist * b.n_wfs)(*[persist_for(w) for w in range(b.n_wfs)])
    names = [(4 * i + 1) for i in range(b.cluster.n_clusters)]
    got, codes = engine_gpu.encode_blobs(b, out, "exec", strs, persist, names, form="cql")
    n_ok = 0
    for w in range(b.n_wfs):
        if out.result[w].code != abi.OK:
            continue
        bld = b.wfs[w].builder
        want, code = _expect(lambda: cq.execution(
            out.exec[w], bld, S, persist[w], repl=out.repl[w],
            vh_items=[(v.event_id, v.version) for v in out.rows(w, "vh")],
            rps=[(p, S) for p in out.rows(w, "rp")], sa=[(kv.key, kv.value) for kv in out.rows(w, "sa")],
            cluster_names=names))
        assert codes[w] == code, (w, codes[w], code)
        if code == 0:
            assert got[w] == want, w
            cq.decode(got[w], cq.EXEC_TYPES + cq.EXEC_TAIL[bld])
            n_ok += 1
    assert n_ok > 0
