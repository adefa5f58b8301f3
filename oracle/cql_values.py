"""TEST INFRASTRUCTURE ONLY: the Cassandra persistence's row values, restated — the parity
checker for cadence_amd/csrc/encode_var.hip's CQL form (cdr_encode_cql_async).

What it restates (paths relative to the reference root):
  the statements   common/persistence/cassandra/cassandraPersistence.go:114-306 (UDT
                   templates), :439-520 (templateUpdateWorkflowExecution*Query,
                   templateUpdate{Activity,Timer,ChildExecution,RequestCancel,Signal}InfoQuery)
  their values     common/persistence/cassandra/cassandraPersistenceUtil.go updateExecution
                   :625-890, updateActivityInfos :1264-1337, updateTimerInfos :1384-1422,
                   updateChildExecutionInfos :1444-1503, updateRequestCancelInfos :1530-1568,
                   updateSignalInfos :1590-1631
  column types     schema/cassandra/cadence/schema.cql:23-228
  the encoding     github.com/gocql/gocql v0.0.0-20171220143535-56a164ee9f31 (go.mod:22) — a
                   third-party dependency not vendored in the reference: its marshalling of
                   bound values (marshal.go) and the CQL v4 native protocol's [bytes] value
                   (int32 length, -1 = null) restated from the published protocol spec and
                   the library's documented behaviour.  No reference test holds CQL bytes:
                   parity of this layout is UNPINNED by reference vectors; it is pinned by
                   the templates' field lists and the schema's column types, which the test
                   decodes the values against.
A row's values are the SET part of its statement (map key + UDT fields, or the execution
row's UDT + replication_state / version_histories + next_event_id); WHERE / IF values are
the caller's.
"""
from __future__ import annotations

import struct

from . import thrift_binary as tb

EMPTY_DOMAIN_ID = b"10000000-0000-f000-f000-000000000000"  # cassandraPersistence.go:46
EMPTY_RUN_ID = b"30000000-0000-f000-f000-000000000000"     # :48
EMPTY_INITIATED_ID = -7                                      # :69
EVENT_STORE_VERSION = -1                                     # cassandraPersistenceUtil.go:35
ZERO_TIME_NANOS = tb.ZERO_TIME_NANOS


class BadUUID(ValueError):
    pass


def val(b: bytes | None) -> bytes:
    """A CQL [bytes] value: int32 length + bytes; None is null (length -1)."""
    return struct.pack(">i", -1) if b is None else struct.pack(">i", len(b)) + b


def bigint(v: int) -> bytes:
    return val(struct.pack(">q", v))


def cint(v: int) -> bytes:
    return val(struct.pack(">i", v))


def boolean(v: bool) -> bytes:
    return val(b"\x01" if v else b"\x00")


def double(v: float) -> bytes:
    return val(struct.pack(">d", v))


def timestamp(ns: int, zero: bool = False) -> bytes:
    """marshalTimestamp of a time.Time: the zero time -> []byte{}; else
    UTC().Unix()*1e3 + Nanosecond()/1e6, i.e. floor(ns / 1e6) milliseconds."""
    return val(b"") if zero else bigint(ns // 1_000_000)


def text(b: bytes) -> bytes:
    return val(b)


def blob_or_null(b: bytes | None) -> bytes:
    return val(b)


def parse_uuid(s: bytes) -> bytes:
    """gocql ParseUUID: '-' skipped where an even number of hex digits has been read,
    exactly 32 hex digits."""
    out, j = bytearray(16), 0
    for c in s:
        if c == ord("-") and j % 2 == 0:
            continue
        ch = chr(c)
        if j >= 32 or ch not in "0123456789abcdefABCDEF":
            raise BadUUID(s)
        out[j // 2] |= int(ch, 16) << (0 if j % 2 else 4)
        j += 1
    if j != 32:
        raise BadUUID(s)
    return bytes(out)


def uuid(s: bytes) -> bytes:
    return val(parse_uuid(s))


def uuid_val(lo: int, hi: int) -> bytes:
    return uuid(tb.uuid_text(lo, hi).encode())


def list_text(body: bytes | None) -> bytes:
    """list<text> of a handle holding the thrift list<string> wire body (type byte, i32
    count, i32-length elements): nil -> null; CQL body = count + [bytes] elements."""
    return val(None if body is None else body[1:])


def activity(a, S) -> bytes:
    tset = bool(a.flags & 0x4)  # CDR_AI_STARTED_TIME_SET
    nr = S(a.nonretriable) if a.nonretriable else None
    return b"".join([
        bigint(a.schedule_id),                       # activity_map[ ? ]
        bigint(a.version), bigint(a.schedule_id), bigint(a.scheduled_event_batch_id),
        val(None),                                    # scheduled_event (nil on replay)
        timestamp(a.scheduled_time), bigint(a.started_id), val(None), timestamp(a.started_time, not tset),
        text(S(a.activity_id)), text(S(a.request_id)), val(None),  # details
        cint(a.s2s), cint(a.s2c), cint(a.stc), cint(a.hb), boolean(bool(a.flags & 0x1)),  # CDR_AI_CANCEL_REQUESTED
        bigint(a.cancel_request_id), timestamp(a.last_heartbeat_time, not tset), cint(a.timer_task_status),
        cint(a.attempt), text(S(a.task_list)), text(b""), boolean(bool(a.flags & 0x2)),  # CDR_AI_HAS_RETRY
        cint(a.initial_interval), double(a.backoff_coefficient), cint(a.maximum_interval),
        timestamp(a.expiration_time), cint(a.maximum_attempts), list_text(nr),
        text(b""), text(b""), val(None), text(b"")])


def timer(t, S) -> bytes:
    return b"".join([text(S(t.timer_id)), bigint(t.version), text(S(t.timer_id)), bigint(t.started_id),
                     timestamp(t.expiry_time), bigint(t.task_id)])


def child(c, S) -> bytes:
    run = S(c.started_run_id)
    return b"".join([
        bigint(c.initiated_id), bigint(c.version), bigint(c.initiated_id), bigint(c.initiated_event_batch_id),
        val(None), bigint(c.started_id), text(S(c.started_workflow_id)), uuid(run if run else EMPTY_RUN_ID),
        val(None), uuid_val(c.create_request_lo, c.create_request_hi), text(b""), text(S(c.domain_name)),
        text(S(c.workflow_type)), cint(c.parent_close_policy)])


def cancel(c, S) -> bytes:
    return b"".join([bigint(c.initiated_id), bigint(c.version), bigint(c.initiated_id),
                     bigint(c.initiated_event_batch_id),
                     text(tb.uuid_text(c.cancel_request_lo, c.cancel_request_hi).encode())])


def signal(g, S) -> bytes:
    return b"".join([bigint(g.initiated_id), bigint(g.version), bigint(g.initiated_id),
                     bigint(g.initiated_event_batch_id), uuid_val(g.signal_request_lo, g.signal_request_hi),
                     text(S(g.signal_name)), blob_or_null(S(g.input) if g.input else None),
                     blob_or_null(S(g.control) if g.control else None)])


def _map(entries) -> bytes:
    return val(struct.pack(">i", len(entries)) + b"".join(entries))


def execution(x, builder, S, persist, repl=None, vh_items=(), rps=None, sa=None, cluster_names=()) -> bytes:
    """updateExecution's SET values (cassandraPersistenceUtil.go:625-890) for a replayed
    ExecutionInfo `x`, the entry's builder (0 local, 1 2DC, 2 NDC) and the persistence-side
    fields in `persist` (cdr_exec_persist); reset points [(row, S)], search attributes
    [(key, value)], 2DC `repl` with cluster_names[i] the LastReplicationInfo key of cluster i."""
    f = [uuid(S(x.domain_id)), text(S(x.workflow_id)), uuid(S(x.run_id))]
    if S(x.parent_domain_id) != b"":
        f += [uuid(S(x.parent_domain_id)), text(S(x.parent_workflow_id)), uuid(S(x.parent_run_id)),
              bigint(x.initiated_id)]
    else:
        f += [uuid(EMPTY_DOMAIN_ID), text(b""), uuid(EMPTY_RUN_ID), bigint(EMPTY_INITIATED_ID)]
    f += [bigint(x.completion_event_batch_id), val(None), text(b""), text(S(x.task_list)), text(S(x.workflow_type)),
          cint(x.workflow_timeout), cint(x.decision_timeout_value),
          blob_or_null(S(persist.execution_context) if persist.execution_context else None),
          cint(x.state), cint(x.close_status), bigint(x.last_first_event_id), bigint(x.last_event_task_id),
          bigint(x.next_event_id), bigint(x.last_processed_event),
          timestamp(persist.start_time, persist.start_time == ZERO_TIME_NANOS),
          timestamp(persist.last_updated_time, persist.last_updated_time == ZERO_TIME_NANOS),
          uuid(S(x.create_request_id)), cint(x.signal_count), bigint(persist.history_size),
          bigint(x.decision_version), bigint(x.decision_schedule_id), bigint(x.decision_started_id),
          text(S(x.decision_request_id)), cint(x.decision_timeout), bigint(x.decision_attempt),
          bigint(x.decision_started_ts), bigint(x.decision_scheduled_ts), bigint(x.decision_original_scheduled_ts),
          boolean(bool(x.flags & 0x001)), text(b""), text(S(persist.sticky_task_list)),
          cint(persist.sticky_s2s_timeout), text(S(persist.client_library_version)),
          text(S(persist.client_feature_version)), text(S(persist.client_impl)),
          val(tb.reset_points_blob(rps if x.flags & 0x040 else None)), text(tb.ENCODING_THRIFTRW),
          cint(x.attempt), boolean(bool(x.flags & 0x002)), cint(x.initial_interval), double(x.backoff_coefficient),
          cint(x.maximum_interval), timestamp(x.expiration_time, not x.flags & 0x004), cint(x.maximum_attempts),
          list_text(S(x.nonretriable) if x.nonretriable else None), cint(EVENT_STORE_VERSION)]
    token = tb.history_branch(S(x.branch_tree_id), tb.uuid_text(x.branch_id_lo, x.branch_id_hi).encode())
    f.append(val(token if x.flags & 0x008 else None))
    f += [text(S(x.cron_schedule)), cint(x.expiration_seconds)]
    if x.flags & 0x020:
        f.append(_map([val(S(k)) + val(S(v)) for k, v in sa or []]))
    else:
        f.append(val(None))
    memo = tb._memo_fields(S(x.memo)) if (x.flags & 0x010) and x.memo else None
    f.append(val(None) if memo is None else val(memo[2:]))
    if builder == 1:
        f += [bigint(repl.current_version), bigint(repl.start_version), bigint(repl.last_write_version),
              bigint(repl.last_write_event_id)]
        ents = [val(S(cluster_names[i])) + val(struct.pack(">iq", 8, repl.lri_version[i]) +
                                               struct.pack(">iq", 8, repl.lri_last_event_id[i]))
                for i in range(len(cluster_names)) if repl.lri_mask >> i & 1]
        f += [_map(ents), bigint(x.next_event_id)]
    elif builder == 2:
        vtok = token if x.flags & 0x100 else b""
        f += [bigint(x.next_event_id), val(tb.version_histories_blob(vtok, vh_items)), text(tb.ENCODING_THRIFTRW)]
    else:
        f.append(bigint(x.next_event_id))
    return b"".join(f)


# ---- the statements' value types (schema.cql), for decoding values back
ACTIVITY_TYPES = ["bigint", "bigint", "bigint", "bigint", "blob", "timestamp", "bigint", "blob", "timestamp", "text",
                  "text", "blob", "int", "int", "int", "int", "boolean", "bigint", "timestamp", "int", "int", "text",
                  "text", "boolean", "int", "double", "int", "timestamp", "int", "list<text>", "text", "text", "blob",
                  "text"]
TIMER_TYPES = ["text", "bigint", "text", "bigint", "timestamp", "bigint"]
CHILD_TYPES = ["bigint", "bigint", "bigint", "bigint", "blob", "bigint", "text", "uuid", "blob", "uuid", "text", "text",
               "text", "int"]
CANCEL_TYPES = ["bigint", "bigint", "bigint", "bigint", "text"]
SIGNAL_TYPES = ["bigint", "bigint", "bigint", "bigint", "uuid", "text", "blob", "blob"]
EXEC_TYPES = ["uuid", "text", "uuid", "uuid", "text", "uuid", "bigint", "bigint", "blob", "text", "text", "text", "int",
              "int", "blob", "int", "int", "bigint", "bigint", "bigint", "bigint", "timestamp", "timestamp", "uuid",
              "int", "bigint", "bigint", "bigint", "bigint", "text", "int", "bigint", "bigint", "bigint", "bigint",
              "boolean", "text", "text", "int", "text", "text", "text", "blob", "text", "int", "boolean", "int",
              "double", "int", "timestamp", "int", "list<text>", "int", "blob", "text", "int", "map<text,blob>",
              "map<text,blob>"]
EXEC_TAIL = {0: ["bigint"], 1: ["bigint", "bigint", "bigint", "bigint", "map<text,replication_info>", "bigint"],
             2: ["bigint", "blob", "text"]}
FIXED = {"bigint": 8, "int": 4, "boolean": 1, "double": 8, "uuid": 16, "timestamp": 8}


def decode(values: bytes, types: list) -> list:
    """Split a row's values by the statement's types, checking each value's size and
    every byte consumed; returns the raw values (None = null)."""
    out, p = [], 0

    def take(n):
        nonlocal p
        assert p + n <= len(values), "truncated"
        b = values[p:p + n]
        p += n
        return b
    for t in types:
        n = struct.unpack(">i", take(4))[0]
        if n < 0:
            out.append(None)
            continue
        b = take(n)
        if t == "timestamp":
            assert n in (0, 8), (t, n)
        elif t in FIXED:
            assert n == FIXED[t], (t, n)
        elif t.startswith("list<") or t.startswith("map<"):
            q, cnt = 4, struct.unpack(">i", b[:4])[0]
            for _ in range(cnt * (2 if t.startswith("map<") else 1)):
                q += 4 + struct.unpack(">i", b[q:q + 4])[0]
            assert q == len(b), (t, "collection body")
        out.append(b)
    assert p == len(values), "trailing bytes"
    return out
