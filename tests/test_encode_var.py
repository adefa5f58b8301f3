"""Variable-size persisted-format row blobs: the SQL persistence's
thriftrw blobs of ActivityInfo, ChildExecutionInfo, SignalInfo and the execution row's
WorkflowExecutionInfo (sqlblobs.thrift:73-193; workflowStateMaps.go:48-83,371-385,632-639;
sqlExecutionManagerUtil.go:1197-1308).

CPU: the oracle's blobs (oracle/thrift_binary.py; its binary-protocol writer is pinned
by the reference's golden HistoryEvent in tests/test_encode.py) parse back under the
IDL's field IDs and types, restated below, with every byte consumed and field IDs
ascending (thriftrw writes fields in IDL order), and the nested blobs (branch token,
reset points, version histories) parse the same way.  The reference has no sqlblobs
golden bytes, so parity of the row layouts is pinned by the IDL and the row writers'
field lists, not by a reference vector.  GPU (-m gpu): encode_var.hip's blobs and
per-row statuses == the oracle's for every row of every OK entry of the synthetic
configs, with a synthetic string table that mixes UUID texts, non-UUID strings, Memo
struct bodies and list bodies (so the MustParseUUID failure path is exercised too).
"""
import hashlib
import struct

import numpy as np
import pytest

from cadence_amd import abi, engine
from oracle import thrift_binary as tb

# sqlblobs.thrift field types (id -> thrift type) of the structs the encoder writes
ACTIVITY = {10: 10, 12: 10, 14: 11, 16: 11, 18: 10, 20: 10, 22: 11, 24: 11, 26: 10, 28: 11, 30: 11, 32: 8,
            34: 8, 36: 8, 38: 8, 40: 2, 42: 10, 44: 8, 46: 8, 48: 11, 50: 11, 52: 2, 54: 8, 56: 8, 58: 8, 60: 10,
            62: 4, 64: 15, 66: 11, 68: 11, 70: 11}                               # :136-168
CHILD = {10: 10, 12: 10, 14: 10, 16: 11, 18: 11, 20: 11, 22: 11, 24: 11, 26: 11, 28: 11, 30: 11, 32: 11,
         35: 8}                                                                  # :170-184
SIGNAL = {10: 10, 11: 10, 12: 11, 14: 11, 16: 11, 18: 11}                        # :186-193
EXEC = {10: 11, 12: 11, 14: 11, 16: 10, 18: 10, 20: 11, 22: 11, 24: 11, 26: 11, 28: 8, 30: 8, 32: 11, 34: 8,
        36: 8, 38: 10, 40: 10, 44: 10, 46: 13, 48: 10, 50: 10, 52: 10, 54: 10, 56: 10, 58: 10, 60: 10, 62: 10,
        64: 8, 66: 10, 68: 10, 69: 10, 70: 2, 71: 10, 72: 11, 74: 11, 76: 11, 78: 11, 80: 10, 82: 10, 84: 8,
        86: 8, 88: 8, 90: 8, 92: 4, 94: 10, 96: 15, 98: 2, 100: 11, 102: 8, 104: 11, 106: 10, 108: 10, 110: 11,
        112: 11, 114: 11, 115: 11, 116: 11, 118: 13, 120: 13, 122: 11, 124: 11}  # :73-134
# shared.thrift nested structs
RESET_POINTS = {10: 15}                                                          # :521-523
RESET_POINT_INFO = {10: 11, 20: 11, 30: 10, 40: 10, 50: 10, 60: 2}               # :525-532
HISTORY_BRANCH = {10: 11, 20: 11, 30: 15}                                        # :1541-1545
VERSION_HISTORIES = {10: 8, 20: 15}                                              # :1560-1563
VERSION_HISTORY = {10: 11, 20: 15}                                               # :1554-1557
VERSION_HISTORY_ITEM = {10: 10, 20: 10}                                          # :1548-1551
FIXED = {2: 1, 3: 1, 4: 8, 6: 2, 8: 4, 10: 8}


class Reader:
    def __init__(self, b: bytes):
        self.b, self.p = b, 0

    def take(self, n):
        assert self.p + n <= len(self.b), "truncated"
        v = self.b[self.p:self.p + n]
        self.p += n
        return v

    def i32(self):
        return struct.unpack(">i", self.take(4))[0]

    def value(self, t):
        if t in FIXED:
            return self.take(FIXED[t])
        if t == 11:
            return self.take(self.i32())
        if t == 15:
            et, n = self.take(1)[0], self.i32()
            return [self.value(et) for _ in range(n)]
        if t == 13:
            kt, vt, n = self.take(1)[0], self.take(1)[0], self.i32()
            return [(self.value(kt), self.value(vt)) for _ in range(n)]
        if t == 12:
            return self.struct(None)
        raise AssertionError(f"type {t}")

    def struct(self, schema):
        out, last = {}, -1
        while True:
            t = self.take(1)[0]
            if t == 0:
                return out
            fid = struct.unpack(">h", self.take(2))[0]
            assert fid > last, f"field {fid} after {last}"
            last = fid
            if schema is not None:
                assert schema.get(fid) == t, f"field {fid}: type {t}, IDL {schema.get(fid)}"
            out[fid] = self.value(t)


def parse(blob: bytes, schema) -> dict:
    r = Reader(blob)
    d = r.struct(schema)
    assert r.p == len(blob), "trailing bytes"
    return d


def parse_nested(blob: bytes, schema) -> dict:
    assert blob[:1] == b"\x59", "codec preamble"
    return parse(blob[1:], schema)


def uuid_of(h: int) -> str:
    x = hashlib.sha256(f"u{h}".encode()).hexdigest()[:32]
    return f"{x[:8]}-{x[8:12]}-{x[12:16]}-{x[16:20]}-{x[20:]}"


def memo_body(h: int) -> bytes:
    ents = b"".join(struct.pack(">i", 2) + f"k{i}".encode() + struct.pack(">i", 3 + i) + bytes(range(3 + i))
                    for i in range(h % 3))
    return tb.field(tb.T_MAP, 10, struct.pack(">bbi", tb.T_STRING, tb.T_STRING, h % 3) + ents) + b"\x00"


def list_body(h: int) -> bytes:
    elems = [f"err{h}_{i}".encode() for i in range(h % 3)]
    return struct.pack(">bi", tb.T_STRING, len(elems)) + b"".join(struct.pack(">i", len(e)) + e for e in elems)


def string_table(n: int, memo=(), lists=()) -> list:
    """Synthetic handle table: UUID texts (36- and 32-char), other strings, Memo struct
    bodies and list<string> bodies for the handles used that way."""
    memo, lists = set(memo), set(lists)
    out = []
    for h in range(n):
        if h == 0:
            s = b""
        elif h in memo:
            s = memo_body(h)
        elif h in lists:
            s = list_body(h)
        elif h % 4 == 1:
            s = uuid_of(h).encode()
        elif h % 4 == 2:
            s = uuid_of(h).replace("-", "").upper().encode()
        elif h % 4 == 3:
            s = bytes((h * 7 + i) & 0xFF for i in range(h % 29))
        else:
            s = b"x" * (h % 7) + str(h).encode()
        out.append(s)
    return out


def persist_for(w: int) -> abi.CdrExecPersist:
    return abi.CdrExecPersist(start_version=w % 5 - 1, current_version=w % 7, start_time=1_600_000_000_000_000_000 + w,
                              last_updated_time=abi.ZERO_TIME_NANOS if w % 3 == 0 else 1_700_000_000_000_000_000 + w,
                              history_size=1000 + w, sticky_s2s_timeout=w % 11, execution_context=(w * 5) % 40,
                              sticky_task_list=(w * 3) % 50, client_library_version=w % 13,
                              client_feature_version=0, client_impl=(w * 7) % 17)


# ---------------------------------------------------------------- CPU
def test_bad_uuid():
    with pytest.raises(tb.BadUUID):
        tb.parse_uuid(b"id-of-domain")
    with pytest.raises(tb.BadUUID):
        tb.parse_uuid(b"0123456789abcdef0123456789abcdeg")
    assert tb.parse_uuid(uuid_of(3).encode()) == bytes.fromhex(uuid_of(3).replace("-", ""))
    assert tb.must_parse_uuid(b"") is None


def _S(strings):
    return lambda h: strings[h]


def test_row_blobs_parse_under_the_idl():
    strs = string_table(64, memo=[9], lists=[12])
    S = _S(strs)
    a = abi.CdrActivityInfo(version=3, schedule_id=5, scheduled_event_batch_id=4, scheduled_time=77, started_id=-23,
                            expiration_time=99, cancel_request_id=-23, activity_id=7, request_id=0, task_list=11,
                            nonretriable=12, s2s=1, s2c=2, stc=3, hb=4, flags=0x2, backoff_coefficient=2.5)
    d = parse(tb.activity_info_blob(a, S), ACTIVITY)
    assert 14 not in d and 22 not in d and 70 not in d  # nil events / failure details
    assert d[26] == struct.pack(">q", abi.ZERO_TIME_NANOS)  # not started: Go's zero time
    assert d[28] == strs[7] and d[64] == [f"err12_{i}".encode() for i in range(0)] and d[62] == struct.pack(">d", 2.5)
    c = abi.CdrChildInfo(version=1, initiated_id=9, initiated_event_batch_id=8, started_id=12, create_request_lo=1,
                         create_request_hi=2, started_workflow_id=3, started_run_id=5, domain_name=7, workflow_type=11,
                         parent_close_policy=2)
    d = parse(tb.child_info_blob(c, S), CHILD)
    assert d[22] == bytes.fromhex(uuid_of(5).replace("-", "")) and 16 not in d and 24 not in d
    assert d[28] == b"00000000-0000-0002-0000-000000000001"
    c.started_run_id = 0
    assert 22 not in parse(tb.child_info_blob(c, S), CHILD)
    c.started_run_id = 4  # not a UUID: MustParseUUID panics
    with pytest.raises(tb.BadUUID):
        tb.child_info_blob(c, S)
    g = abi.CdrSignalInfo(version=1, initiated_event_batch_id=2, initiated_id=3, signal_request_lo=4,
                          signal_request_hi=5, signal_name=7, input=3, control=0)
    d = parse(tb.signal_info_blob(g, S), SIGNAL)
    assert d[16] == strs[3] and 18 not in d


@pytest.mark.parametrize("builder", [abi.BUILDER_LOCAL, abi.BUILDER_2DC, abi.BUILDER_NDC])
def test_exec_blob_parses_under_the_idl(builder):
    strs = string_table(64, memo=[9], lists=[12])
    S = _S(strs)
    x = abi.CdrExecInfo(parent_domain_id=5, parent_workflow_id=7, parent_run_id=0, initiated_id=3, task_list=11,
                        workflow_type=13, memo=9, nonretriable=12, branch_tree_id=17, branch_id_lo=1, branch_id_hi=2,
                        flags=0x001 | 0x002 | 0x010 | 0x020 | 0x040 | (0x100 if builder == abi.BUILDER_NDC else 0x008),
                        signal_count=4, attempt=2)
    repl = abi.CdrReplState(last_write_event_id=40, lri_mask=0b101)
    repl.lri_version[0], repl.lri_last_event_id[0], repl.lri_version[2], repl.lri_last_event_id[2] = 1, 2, 3, 4
    rp = abi.CdrResetPoint(binary_checksum=21, run_id=1, first_decision_completed_id=4, created_time_nano=5, flags=0x7F)
    blob = tb.exec_info_blob(x, builder, S, persist_for(3), repl=repl, vh_items=[(3, 1), (9, 4)], rps=[(rp, S)],
                             sa=[(13, 15)], cluster_names=[23, 25, 27])
    d = parse(blob, EXEC)
    assert d[10] == bytes.fromhex(uuid_of(5).replace("-", "")) and 14 not in d  # parent run "" -> nil
    assert d[70] == b"\x01" and d[76] == b"" and 102 not in d and 20 not in d
    assert (44 in d) == (builder == abi.BUILDER_2DC) and (122 in d) == (builder == abi.BUILDER_NDC)
    assert (104 in d) == (builder != abi.BUILDER_NDC)
    token = tb.history_branch(strs[17], b"00000000-0000-0002-0000-000000000001")
    hb = parse_nested(token, HISTORY_BRANCH)
    assert hb[10] == strs[17] and hb[30] == []
    if builder == abi.BUILDER_2DC:
        assert [k for k, _ in d[46]] == [strs[23], strs[27]]
    if builder == abi.BUILDER_NDC:
        vhs = parse_nested(d[122], VERSION_HISTORIES)
        assert vhs[10] == b"\x00\x00\x00\x00" and len(vhs[20]) == 1
        assert vhs[20][0][10] == token and len(vhs[20][0][20]) == 2
    rps = parse_nested(d[115], RESET_POINTS)
    assert len(rps[10]) == 1 and set(rps[10][0]) == set(RESET_POINT_INFO)
    assert d[116] == b"thriftrw" and d[118] == [(strs[13], strs[15])]
    assert [k for k, _ in d[120]] == [b"k0", b"k1", b"k2"][:9 % 3]
    # a nil ResetPoints still serializes (SerializeResetPoints of &ResetPoints{})
    x.flags &= ~0x040
    assert parse(tb.exec_info_blob(x, builder, S, persist_for(3), repl=repl, cluster_names=[23, 25, 27]),
                 EXEC)[115] == b"\x59\x00"


# ---------------------------------------------------------------- GPU
HANDLE_FIELDS = {
    "exec": ("domain_id", "workflow_id", "run_id", "create_request_id", "parent_domain_id", "parent_workflow_id",
             "parent_run_id", "task_list", "workflow_type", "cron_schedule", "memo", "nonretriable",
             "branch_tree_id", "decision_request_id"),
    "act": ("activity_id", "request_id", "task_list", "nonretriable"),
    "child": ("started_workflow_id", "started_run_id", "domain_name", "workflow_type"),
    "signal": ("signal_name", "input", "control"),
    "rp": ("binary_checksum", "run_id"),
    "sa": ("key", "value"),
}


def _table(b, out):
    """The string table covering every handle the outputs name (and the persistence
    context's), with Memo / list bodies where the handle is used that way."""
    hmax, memo, lists = 64, set(), set()
    for w in range(b.n_wfs):
        if out.result[w].code != abi.OK:
            continue
        x = out.exec[w]
        hmax = max([hmax] + [getattr(x, f) for f in HANDLE_FIELDS["exec"]])
        if x.memo:
            memo.add(x.memo)
        if x.nonretriable:
            lists.add(x.nonretriable)
        for t in ("act", "child", "signal", "rp", "sa"):
            for r in out.rows(w, t):
                hmax = max([hmax] + [getattr(r, f) for f in HANDLE_FIELDS[t]])
                if t == "act" and r.nonretriable:
                    lists.add(r.nonretriable)
    return string_table(hmax + 1, memo, lists - memo)


def _expect(fn):
    try:
        return fn(), 0
    except tb.BadUUID:
        return None, 1


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_gpu_variable_row_blobs(engine_gpu, cfg):
    b = engine.synth_batch(cfg, 300, seed=0x5EED0600 + cfg)
    out = engine_gpu.replay(b)
    strs = _table(b, out)
    S = _S(strs)
    makers = {"act": tb.activity_info_blob, "child": tb.child_info_blob, "signal": tb.signal_info_blob}
    for table, mk in makers.items():
        got, codes = engine_gpu.encode_blobs(b, out, table, strs)
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
                n += 1
        assert set(got) == set(codes) and len(got) == n
        if cfg in (3, 4, 5):
            assert n > 0, table
    # the execution row
    persist = (abi.CdrExecPersist * b.n_wfs)(*[persist_for(w) for w in range(b.n_wfs)])
    names = [(4 * i + 1) for i in range(b.cluster.n_clusters)]
    got, codes = engine_gpu.encode_blobs(b, out, "exec", strs, persist, names)
    n_ok = 0
    for w in range(b.n_wfs):
        if out.result[w].code != abi.OK:
            assert w not in got
            continue
        bld = b.wfs[w].builder
        want, code = _expect(lambda: tb.exec_info_blob(
            out.exec[w], bld, S, persist[w], repl=out.repl[w],
            vh_items=[(v.event_id, v.version) for v in out.rows(w, "vh")],
            rps=[(p, S) for p in out.rows(w, "rp")], sa=[(kv.key, kv.value) for kv in out.rows(w, "sa")],
            cluster_names=names))
        assert codes[w] == code, (w, codes[w], code)
        if code == 0:
            assert got[w] == want, w
            parse(got[w], EXEC)
            n_ok += 1
    assert n_ok > 0
