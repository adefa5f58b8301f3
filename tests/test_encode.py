"""Persisted-format row encoders: the SQL persistence's thriftrw
binary-protocol blobs of pending TimerInfo / RequestCancelInfo rows.

CPU: the restated binary-protocol writer (oracle/thrift_binary.py) reproduces the
reference's golden HistoryEvent bytes (common/codec/version0Thriftrw_test.go:42-64)
byte for byte, which pins the protocol; the row blobs follow the field lists of
workflowStateMaps.go:242-247 and :507-511.  GPU (-m gpu): encode.hip's blobs == the
oracle's for every row of every OK entry on the synthetic configs.
"""
import pytest

from cadence_amd import abi, engine
from oracle import thrift_binary as tb

# common/codec/version0Thriftrw_test.go:55-64 (preamble byte 89 = version 0, then the
# binary-protocol HistoryEvent)
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


def test_writer_matches_reference_golden_history_event():
    """HistoryEvent{EventId 130, Timestamp, EventType 23 (RequestCancelExternal...
    Initiated), Version 1234, attributes (field 300){Domain, WorkflowExecution{WorkflowId,
    RunId}, Control, ChildWorkflowOnly}} in IDL field order (shared.thrift)."""
    ev = tb.struct_([
        tb.i64(10, 130), tb.i64(20, 112345132134), tb.i32(30, 23), tb.i64(35, 1234),
        tb.sub(300, [tb.string(20, "some random target domain"),
                     tb.sub(30, [tb.string(10, "some random target workflow ID"),
                                 tb.string(20, "some random target run ID")]),
                     tb.string(40, b"some random control"), tb.boolean(50, True)]),
    ])
    assert bytes([89]) + ev == GOLDEN


def test_row_blob_sizes_and_uuid_text():
    t = abi.CdrTimerInfo(version=3, started_id=7, expiry_time=-5, task_id=1)
    b = tb.timer_info_blob(t)
    assert len(b) == 45 and b[:3] == bytes([10, 0, 10]) and b[-1] == 0
    assert b[-9:-1] == (1).to_bytes(8, "big")
    c = abi.CdrCancelInfo(version=1, initiated_event_batch_id=2, cancel_request_lo=0x0123456789ABCDEF,
                          cancel_request_hi=0xFEDCBA9876543210)
    b = tb.request_cancel_info_blob(c)
    assert len(b) == 66
    assert b[22:29] == bytes([11, 0, 12, 0, 0, 0, 36])
    assert b[29:65].decode() == "fedcba98-7654-3210-0123-456789abcdef"


def _expected(batch, out, table):
    enc, size = {"timer": (tb.timer_info_blob, 45), "cancel": (tb.request_cancel_info_blob, 66)}[table]
    off = {"timer": "timer_off", "cancel": "cancel_off"}[table]
    want = {}
    for w in range(batch.n_wfs):
        if out.result[w].code != abi.OK:
            continue
        base = getattr(out.plan.caps[w], off)
        for j, row in enumerate(out.rows(w, table)):
            want[base + j] = enc(row)
    return want, size


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [0, 3, 4, 5])
def test_gpu_row_blobs(engine_gpu, cfg):
    b = engine.synth_batch(cfg, 300, seed=0x5EED0500 + cfg, error_rate=0.1 if cfg in (0, 3) else 0.0)
    out = engine_gpu.replay(b)
    for table in ("timer", "cancel"):
        want, size = _expected(b, out, table)
        got = engine_gpu.encode_rows(b, out, table)
        assert want, table
        assert set(got) == set(want), table
        bad = [r for r, blob in want.items() if got[r] != blob]
        assert not bad, f"{table}: {len(bad)} rows differ, first {bad[0]}"
