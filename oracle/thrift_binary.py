"""TEST INFRASTRUCTURE ONLY: thriftrw binary-protocol writer (restated) and the SQL
persistence's row blobs, the parity checker for cadence_amd/csrc/encode.hip.

Protocol (go.uber.org/thriftrw protocol.Binary, used by common/persistence/sql/blob.go:61-73
and common/codec/version0Thriftrw.go:45-84): a struct is its set fields in IDL order,
each a type byte, a big-endian i16 field ID and the value, then a 0 stop byte; i64 / i32
/ i16 are big-endian, bool one byte, string / binary a big-endian i32 length + bytes,
struct nested as above.  Pinned byte-exact by the golden HistoryEvent of
common/codec/version0Thriftrw_test.go:42-64 (tests/test_encode.py).
"""
from __future__ import annotations

import struct

T_BOOL, T_I32, T_I64, T_STRING, T_STRUCT = 2, 8, 10, 11, 12


def field(ttype: int, fid: int, payload: bytes) -> bytes:
    return struct.pack(">bh", ttype, fid) + payload


def i64(fid: int, v: int) -> bytes:
    return field(T_I64, fid, struct.pack(">q", v))


def i32(fid: int, v: int) -> bytes:
    return field(T_I32, fid, struct.pack(">i", v))


def boolean(fid: int, v: bool) -> bytes:
    return field(T_BOOL, fid, b"\x01" if v else b"\x00")


def string(fid: int, v: bytes | str) -> bytes:
    b = v.encode() if isinstance(v, str) else v
    return field(T_STRING, fid, struct.pack(">i", len(b)) + b)


def struct_(fields: list[bytes]) -> bytes:
    return b"".join(fields) + b"\x00"


def sub(fid: int, fields: list[bytes]) -> bytes:
    return field(T_STRUCT, fid, struct_(fields))


def uuid_text(lo: int, hi: int) -> str:
    """RFC 4122 text form of the 128-bit (hi, lo) pair (cdr.h cdr_encode_rows_async)."""
    h = f"{hi & (2**64 - 1):016x}{lo & (2**64 - 1):016x}"
    return f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:]}"


def timer_info_blob(t) -> bytes:
    """timerInfoToBlob(&sqlblobs.TimerInfo{Version, StartedID, ExpiryTimeNanos, TaskID})
    (workflowStateMaps.go:242-247; sqlblobs.thrift:201-206)."""
    return struct_([i64(10, t.version), i64(12, t.started_id), i64(14, t.expiry_time), i64(16, t.task_id)])


def request_cancel_info_blob(c) -> bytes:
    """requestCancelInfoToBlob(&sqlblobs.RequestCancelInfo{Version, InitiatedEventBatchID,
    CancelRequestID}) (workflowStateMaps.go:507-511; sqlblobs.thrift:195-199)."""
    return struct_([i64(10, c.version), i64(11, c.initiated_event_batch_id),
                    string(12, uuid_text(c.cancel_request_lo, c.cancel_request_hi))])


# ---------------------------------------------------------------- variable-size rows
# The row writers' structs whose size depends on the data: string / binary
# fields come from a handle table (handle 0 = "" / nil).  Conventions of the table the
# encoder reads (include/cdr/cdr.h cdr_encode_blobs_async): a plain string or binary field
# is its bytes; a NonRetriableErrors handle is the wire body of the list<string> (element
# type, i32 count, elements — what cdr_ingest_decode interns); a Memo handle is the wire
# body of the Memo struct (its fields and stop byte).
T_DOUBLE, T_I16, T_MAP, T_LIST = 4, 6, 13, 15
ZERO_TIME_NANOS = -6795364578871345152  # time.Time{}.UnixNano() (int64 wrap of year-1 seconds x 1e9)
ENCODING_THRIFTRW = b"thriftrw"  # common/constants.go:62
PREAMBLE = b"\x59"  # common/codec/version0Thriftrw.go:45-64 (preambleVersion0)


class BadUUID(ValueError):
    """sqldb.MustParseUUID would panic (common/persistence/sql/storage/sqldb/uuid.go:39-45)."""


def double(fid: int, v: float) -> bytes:
    return field(T_DOUBLE, fid, struct.pack(">d", v))


def raw_field(ttype: int, fid: int, body: bytes) -> bytes:
    return field(ttype, fid, body)


def parse_uuid(s: bytes) -> bytes:
    """google/uuid.Parse of the canonical 36-char and the bare 32-hex forms -> 16 bytes."""
    t = s.decode("latin-1")
    if len(t) == 36:
        if t[8] != "-" or t[13] != "-" or t[18] != "-" or t[23] != "-":
            raise BadUUID(t)
        t = t.replace("-", "", 4)
    if len(t) != 32 or any(c not in "0123456789abcdefABCDEF" for c in t):
        raise BadUUID(s)
    return bytes.fromhex(t)


def must_parse_uuid(s: bytes) -> bytes | None:
    return None if s == b"" else parse_uuid(s)


def activity_info_blob(a, S) -> bytes:
    """activityInfoToBlob(&sqlblobs.ActivityInfo{...}) as updateActivityInfos builds it on a
    replayed row (workflowStateMaps.go:48-83; sqlblobs.thrift:136-168): ScheduledEvent /
    StartedEvent are nil on replay (ReplicateActivityTaskScheduledEvent,
    mutableStateBuilder.go:1982-2028, sets neither), so their binary fields are absent and
    their encodings are ""; StartedIdentity, LastFailureReason, LastWorkerIdentity are "".
    S(handle) -> bytes."""
    retry = bool(a.flags & 0x2)
    started = a.started_time if a.flags & 0x4 else ZERO_TIME_NANOS
    f = [i64(10, a.version), i64(12, a.scheduled_event_batch_id), string(16, b""), i64(18, a.scheduled_time),
         i64(20, a.started_id), string(24, b""), i64(26, started), string(28, S(a.activity_id)),
         string(30, S(a.request_id)), i32(32, a.s2s), i32(34, a.s2c), i32(36, a.stc), i32(38, a.hb),
         boolean(40, bool(a.flags & 0x1)), i64(42, a.cancel_request_id), i32(44, a.timer_task_status),
         i32(46, a.attempt), string(48, S(a.task_list)), string(50, b""), boolean(52, retry),
         i32(54, a.initial_interval), i32(56, a.maximum_interval), i32(58, a.maximum_attempts),
         i64(60, a.expiration_time), double(62, a.backoff_coefficient)]
    if a.nonretriable:
        f.append(raw_field(T_LIST, 64, S(a.nonretriable)))
    f += [string(66, b""), string(68, b"")]
    return struct_(f)


def child_info_blob(c, S) -> bytes:
    """childExecutionInfoToBlob (workflowStateMaps.go:371-385; sqlblobs.thrift:170-184):
    InitiatedEvent / StartedEvent nil on replay (mutableStateBuilder.go:3256-3325), their
    encodings ""; StartedRunID is MustParseUUID(StartedRunID) (nil while not started);
    CreateRequestID the row's UUID in RFC 4122 text form."""
    run = must_parse_uuid(S(c.started_run_id))
    f = [i64(10, c.version), i64(12, c.initiated_event_batch_id), i64(14, c.started_id), string(18, b""),
         string(20, S(c.started_workflow_id))]
    if run is not None:
        f.append(string(22, run))
    f += [string(26, b""), string(28, uuid_text(c.create_request_lo, c.create_request_hi)),
          string(30, S(c.domain_name)), string(32, S(c.workflow_type)), i32(35, c.parent_close_policy)]
    return struct_(f)


def signal_info_blob(g, S) -> bytes:
    """signalInfoToBlob (workflowStateMaps.go:632-639; sqlblobs.thrift:186-193): Input /
    Control are the initiating event's binaries (nil -> absent)."""
    f = [i64(10, g.version), i64(11, g.initiated_event_batch_id),
         string(12, uuid_text(g.signal_request_lo, g.signal_request_hi)), string(14, S(g.signal_name))]
    if g.input:
        f.append(string(16, S(g.input)))
    if g.control:
        f.append(string(18, S(g.control)))
    return struct_(f)


def _list(fid: int, etype: int, elems: list[bytes]) -> bytes:
    return field(T_LIST, fid, struct.pack(">bi", etype, len(elems)) + b"".join(elems))


def history_branch(tree_id: bytes, branch_id: bytes) -> bytes:
    """NewHistoryBranchToken's token (dataInterfaces.go:2428-2440): the thriftrw encoding
    (preamble 0x59) of HistoryBranch{TreeID, BranchID, Ancestors: []} (shared.thrift:1541-1545)."""
    return PREAMBLE + struct_([string(10, tree_id), string(20, branch_id), _list(30, T_STRUCT, [])])


def reset_points_blob(rps) -> bytes:
    """SerializeResetPoints (serializer.go:120-125, thriftrw): ResetPoints{Points} with the
    ResetPointInfo optional fields present as their flags say (shared.thrift:521-532);
    rps None -> &ResetPoints{} (Points nil)."""
    if rps is None:
        return PREAMBLE + struct_([])
    pts = []
    for p, S in rps:
        f = []
        if p.flags & 0x01:
            f.append(string(10, S(p.binary_checksum)))
        if p.flags & 0x02:
            f.append(string(20, S(p.run_id)))
        if p.flags & 0x04:
            f.append(i64(30, p.first_decision_completed_id))
        if p.flags & 0x08:
            f.append(i64(40, p.created_time_nano))
        if p.flags & 0x10:
            f.append(i64(50, p.expiring_time_nano))
        if p.flags & 0x20:
            f.append(boolean(60, bool(p.flags & 0x40)))
        pts.append(struct_(f))
    return PREAMBLE + struct_([_list(10, T_STRUCT, pts)])


def version_histories_blob(token: bytes, items) -> bytes:
    """SerializeVersionHistories (serializer.go:161-166) of the single current branch:
    VersionHistories{CurrentVersionHistoryIndex: 0, Histories: [{BranchToken, Items}]}
    (versionHistory.go:135-149,411-423; shared.thrift:1548-1563)."""
    its = [struct_([i64(10, e), i64(20, v)]) for e, v in items]
    h = struct_([string(10, token), _list(20, T_STRUCT, its)])
    return PREAMBLE + struct_([i32(10, 0), _list(20, T_STRUCT, [h])])


def _memo_fields(body: bytes) -> bytes | None:
    """The map body of Memo field 10 inside a Memo struct body (None if absent)."""
    p = 0
    while True:
        t = body[p]
        if t == 0:
            return None
        fid = struct.unpack(">h", body[p + 1:p + 3])[0]
        p += 3
        if t == T_MAP and fid == 10:
            q = p + 6
            n = struct.unpack(">i", body[p + 2:p + 6])[0]
            for _ in range(2 * n):
                q += 4 + struct.unpack(">i", body[q:q + 4])[0]
            return body[p:q]
        if t in (T_STRING,):
            p += 4 + struct.unpack(">i", body[p:p + 4])[0]
        else:
            raise ValueError(f"unexpected Memo field type {t}")


def exec_info_blob(x, builder, S, persist, repl=None, vh_items=(), rps=None, sa=None, cluster_names=()) -> bytes:
    """workflowExecutionInfoToBlob of buildExecutionRow (sqlExecutionManagerUtil.go:1197-1308;
    sqlblobs.thrift:73-134) for a replayed ExecutionInfo `x` (cdr_exec_info), the entry's
    builder (1 = 2DC: LastWriteEventID + LastReplicationInfo; 2 = NDC: VersionHistories),
    the persistence-side fields in `persist` (cdr_exec_persist), reset points
    [(row, S)], search attributes [(key, value)] and, for 2DC, `repl` (cdr_repl_state)
    with `cluster_names[i]` the map key of cluster i (maps in key-index order: Go's map
    iteration order is random, so the reference has no fixed byte order for them)."""
    f = []
    parent = S(x.parent_domain_id) != b""
    if parent:
        f.append(string(10, parse_uuid(S(x.parent_domain_id))))
        f.append(string(12, S(x.parent_workflow_id)))
        run = must_parse_uuid(S(x.parent_run_id))
        if run is not None:
            f.append(string(14, run))
        f.append(i64(16, x.initiated_id))
    f.append(i64(18, x.completion_event_batch_id))
    f += [string(24, S(x.task_list)), string(26, S(x.workflow_type)), i32(28, x.workflow_timeout),
          i32(30, x.decision_timeout_value)]
    if persist.execution_context:
        f.append(string(32, S(persist.execution_context)))
    f += [i32(34, x.state), i32(36, x.close_status), i64(38, persist.start_version),
          i64(40, persist.current_version)]
    if builder == 1:
        f.append(i64(44, repl.last_write_event_id))
        ents = []
        for i in range(len(cluster_names)):
            if repl.lri_mask >> i & 1:
                ents.append(struct.pack(">i", len(S(cluster_names[i]))) + S(cluster_names[i]) +
                            struct_([i64(10, repl.lri_version[i]), i64(12, repl.lri_last_event_id[i])]))
        f.append(field(T_MAP, 46, struct.pack(">bbi", T_STRING, T_STRUCT, len(ents)) + b"".join(ents)))
    f += [i64(48, x.last_event_task_id), i64(50, x.last_first_event_id), i64(52, x.last_processed_event),
          i64(54, persist.start_time), i64(56, persist.last_updated_time), i64(58, x.decision_version),
          i64(60, x.decision_schedule_id), i64(62, x.decision_started_id), i32(64, x.decision_timeout),
          i64(66, x.decision_attempt), i64(68, x.decision_started_ts), i64(69, x.decision_scheduled_ts)]
    cancel = bool(x.flags & 0x001)
    if cancel:
        f.append(boolean(70, True))
    f += [i64(71, x.decision_original_scheduled_ts), string(72, S(x.create_request_id)),
          string(74, S(x.decision_request_id))]
    if cancel:
        f.append(string(76, b""))
    f += [string(78, S(persist.sticky_task_list)), i64(80, persist.sticky_s2s_timeout), i64(82, x.attempt),
          i32(84, x.initial_interval), i32(86, x.maximum_interval), i32(88, x.maximum_attempts),
          i32(90, x.expiration_seconds), double(92, x.backoff_coefficient),
          i64(94, x.expiration_time if x.flags & 0x004 else ZERO_TIME_NANOS)]
    if x.nonretriable:
        f.append(raw_field(T_LIST, 96, S(x.nonretriable)))
    f.append(boolean(98, bool(x.flags & 0x002)))
    f.append(string(100, S(x.cron_schedule)))
    token = history_branch(S(x.branch_tree_id), uuid_text(x.branch_id_lo, x.branch_id_hi).encode())
    if x.flags & 0x008:
        f.append(string(104, token))
    f += [i64(106, x.signal_count), i64(108, persist.history_size), string(110, S(persist.client_library_version)),
          string(112, S(persist.client_feature_version)), string(114, S(persist.client_impl))]
    f.append(string(115, reset_points_blob(rps if x.flags & 0x040 else None)))
    f.append(string(116, ENCODING_THRIFTRW))
    if x.flags & 0x020:
        ents = [struct.pack(">i", len(S(k))) + S(k) + struct.pack(">i", len(S(v))) + S(v) for k, v in sa or []]
        f.append(field(T_MAP, 118, struct.pack(">bbi", T_STRING, T_STRING, len(ents)) + b"".join(ents)))
    if x.flags & 0x010:
        body = _memo_fields(S(x.memo)) if x.memo else None
        if body is not None:
            f.append(field(T_MAP, 120, body))
    if builder == 2:
        vtok = token if x.flags & 0x100 else b""
        f.append(string(122, version_histories_blob(vtok, vh_items)))
        f.append(string(124, ENCODING_THRIFTRW))
    return struct_(f)
