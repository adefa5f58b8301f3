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
