"""The CPU restatement (oracle/) checked against the reference's own known-answer
tests, restated case by case.  No GPU needed."""
import ctypes as C

import pytest

import oracle
from cadence_amd import abi
from cadence_amd.history import HistoryBuilder

NS = 1_000_000_000


def run(hb, **kw):
    b = hb.build(**kw)
    return b, oracle.replay(b)


# ---- 1. nDCStateRebuilder_test.go:239-347 TestRebuild ---------------------------
def test_ndc_state_rebuilder_rebuild():
    hb = HistoryBuilder()
    w = hb.workflow(workflow_id="other random workflow ID", run_id="target-run-id", request_id="req",
                    domain_id="target-domain-id", builder=abi.BUILDER_NDC, failover_version=1234,
                    expected_next_event_id=3)
    w.calls = [
        [{"eventId": 1, "version": 12, "eventType": "WorkflowExecutionStarted",
          "workflowExecutionStartedEventAttributes": {
              "workflowType": {"name": "some random workflow type"},
              "taskList": {"name": "some random workflow type"},
              "executionStartToCloseTimeoutSeconds": 123, "taskStartToCloseTimeoutSeconds": 233}}],
        [{"eventId": 2, "version": 12, "eventType": "WorkflowExecutionSignaled"}],
    ]
    b, out = run(hb)
    r, x = out.result[0], out.exec[0]
    assert r.code == abi.OK
    S = b.strings
    assert S[x.domain_id] == "target-domain-id"
    assert S[x.workflow_id] == "other random workflow ID"
    assert S[x.run_id] == "target-run-id"
    vh = out.rows(0, "vh")
    assert [(i.event_id, i.version) for i in vh] == [(2, 12)]
    assert x.next_event_id == 3 and x.signal_count == 1
    # NextEventID != baseNextEventID -> error (nDCStateRebuilder.go:139-143)
    w.expected_next_event_id = 4
    _, out2 = run(hb)
    assert out2.result[0].code == 12


# ---- 2. conflictResolver_test.go:162-300 TestReset (2DC, only event 1 applied) ---
def test_conflict_resolver_reset():
    hb = HistoryBuilder()
    w = hb.workflow(workflow_id="wid", run_id="rid", request_id="createRequestID", domain_id="domainID",
                    builder=abi.BUILDER_2DC, failover_version=abi.EMPTY_VERSION)
    # event1 has no EventType: GetEventType() of nil is WorkflowExecutionStarted (0)
    w.calls = [[{"eventId": 1, "version": 12, "eventType": 0,
                 "workflowExecutionStartedEventAttributes": {
                     "workflowType": {"name": "some random workflow type"},
                     "taskList": {"name": "some random workflow type"},
                     "executionStartToCloseTimeoutSeconds": 123, "taskStartToCloseTimeoutSeconds": 233}}]]
    cluster = abi.CdrClusterMeta()
    cluster.failover_version_increment = 10
    cluster.current_cluster = 0  # "active"; version 12 -> cluster 1 ("standby"), as mocked at :302
    cluster.n_clusters = 2
    cluster.initial_version[0] = 1
    cluster.initial_version[1] = 2
    b, out = run(hb, cluster=cluster)
    r, x, rs = out.result[0], out.exec[0], out.repl[0]
    S = b.strings
    assert r.code == abi.OK
    assert S[x.task_list] == S[x.workflow_type] == "some random workflow type"
    assert (x.workflow_timeout, x.decision_timeout_value) == (123, 233)
    assert (x.state, x.close_status) == (abi.STATE_CREATED, abi.CLOSE_NONE)
    assert (x.last_first_event_id, x.next_event_id, x.last_processed_event) == (1, 2, -23)
    assert (x.decision_version, x.decision_schedule_id, x.decision_started_id) == (-24, -23, -23)
    assert S[x.decision_request_id] == "emptyUuid"
    assert (x.decision_timeout, x.decision_attempt, x.decision_started_ts) == (0, 0, 0)
    assert x.initiated_id == -23
    assert S[x.create_request_id] == "createRequestID"
    assert (S[x.parent_domain_id], S[x.parent_workflow_id], S[x.parent_run_id]) == ("", "", "")
    assert rs.present == 1
    assert (rs.current_version, rs.start_version, rs.last_write_version, rs.last_write_event_id) == (12, 12, 12, 1)
    assert rs.lri_mask == 0b10 and (rs.lri_version[1], rs.lri_last_event_id[1]) == (12, 1)


# ---- 3. versionHistory_test.go:156-292 AddOrUpdateItem --------------------------
def _vh(items, eid, ver, cap=16):
    arr = (abi.CdrVHItem * cap)(*[abi.CdrVHItem(e, v) for e, v in items])
    n = C.c_uint32(len(items))
    rc = oracle.lib().cdro_vh_add_or_update(arr, C.byref(n), cap, eid, ver)
    return rc, [(arr[i].event_id, arr[i].version) for i in range(n.value)]


def test_vh_add_or_update_version_increase():  # :156-180
    assert _vh([(3, 0), (6, 4)], 8, 5) == (0, [(3, 0), (6, 4), (8, 5)])


def test_vh_add_or_update_event_id_increase():  # :182-204
    assert _vh([(3, 0), (6, 4)], 8, 4) == (0, [(3, 0), (8, 4)])


def test_vh_add_or_update_failed_lower_version():  # :206-216
    assert _vh([(3, 0), (6, 4)], 8, 3)[0] == 5


def test_vh_add_or_update_failed_event_id_not_increasing():  # :218-231
    assert _vh([(3, 0), (6, 4)], 5, 4)[0] == 6
    assert _vh([(3, 0), (6, 4)], 6, 4)[0] == 6


def test_vh_add_or_update_failed_version_not_increasing():  # :233-249
    # the reference's three items, each an error; the version check comes first
    # (versionHistory.go:213-218), so each is the lower-version one
    for event_id in (6, 2, 7):
        assert _vh([(3, 0), (6, 4)], event_id, 3)[0] == 5, event_id


def test_vh_item_panics():  # NewVersionHistoryItem versionHistory.go:31-42
    assert _vh([], -1, 1)[0] == 34
    assert _vh([], 1, -2)[0] == 34
    assert _vh([], 1, abi.EMPTY_VERSION)[0] == 0


# ---- 4. workflowExecutionInfo.go:45-147 state / close-status transitions ---------
def _expected_transition(cur, cur_close, st, cs):
    # written from the Go switch, case by case
    S, Cl = abi, abi
    if cur == S.STATE_VOID:
        return True
    if cur == S.STATE_CREATED:
        if st in (S.STATE_CREATED, S.STATE_RUNNING, S.STATE_ZOMBIE):
            return cs == Cl.CLOSE_NONE
        if st == S.STATE_COMPLETED:
            return cs in (Cl.CLOSE_TERMINATED, Cl.CLOSE_TIMED_OUT)
        return False
    if cur == S.STATE_RUNNING:
        if st == S.STATE_CREATED:
            return False
        if st in (S.STATE_RUNNING, S.STATE_ZOMBIE):
            return cs == Cl.CLOSE_NONE
        if st == S.STATE_COMPLETED:
            return cs != Cl.CLOSE_NONE
        return False
    if cur == S.STATE_COMPLETED:
        return st == S.STATE_COMPLETED and cs == cur_close
    if cur == S.STATE_ZOMBIE:
        if st in (S.STATE_CREATED, S.STATE_RUNNING):
            return cs == Cl.CLOSE_NONE
        if st in (S.STATE_COMPLETED, S.STATE_ZOMBIE):
            return cs != Cl.CLOSE_NONE
        return False
    return False


def test_state_transition_table_exhaustive():
    L = oracle.lib()
    for cur in range(5):
        for cur_close in range(7):
            for st in range(5):
                for cs in range(7):
                    assert L.cdro_state_transition(cur, cur_close, st, cs) == int(
                        _expected_transition(cur, cur_close, st, cs)), (cur, cur_close, st, cs)


# ---- 5. timerBuilder_test.go:85-215 timer picks, restated as replayed histories --
def _head(hb, wid="w"):
    w = hb.workflow(workflow_id=wid, run_id="r-" + wid, request_id="q", builder=abi.BUILDER_NDC,
                    failover_version=1)
    t0 = 1_500_000_000 * NS
    w.calls = [[{"eventId": 1, "version": 1, "timestamp": t0, "eventType": "WorkflowExecutionStarted",
                 "workflowExecutionStartedEventAttributes": {"taskList": {"name": "tl"},
                                                             "taskStartToCloseTimeoutSeconds": 10}},
                {"eventId": 2, "version": 1, "timestamp": t0 + 1, "eventType": "DecisionTaskScheduled",
                 "decisionTaskScheduledEventAttributes": {"startToCloseTimeoutSeconds": 10}}],
               [{"eventId": 3, "version": 1, "timestamp": t0 + 2, "eventType": "DecisionTaskStarted",
                 "decisionTaskStartedEventAttributes": {"scheduledEventId": 2, "requestId": "r1"}}]]
    return w, t0


def test_timer_builder_single_user_timer():  # :85-112
    hb = HistoryBuilder()
    w, t0 = _head(hb)
    w.calls.append([
        {"eventId": 4, "version": 1, "timestamp": t0 + 3, "eventType": "DecisionTaskCompleted",
         "decisionTaskCompletedEventAttributes": {"scheduledEventId": 2, "startedEventId": 3}},
        {"eventId": 5, "version": 1, "timestamp": t0 + 4, "eventType": "TimerStarted",
         "timerStartedEventAttributes": {"timerId": "tid1", "startToFireTimeoutSeconds": 1}}])
    b, out = run(hb)
    (t,) = out.rows(0, "timer")
    assert b.strings[t.timer_id] == "tid1" and t.started_id == 5 and t.task_id == 1
    assert t.expiry_time == t0 + 4 + NS


def test_timer_builder_multiple_user_timers():  # :114-170
    hb = HistoryBuilder()
    w, t0 = _head(hb)
    w.calls.append([
        {"eventId": 4, "version": 1, "timestamp": t0 + 3, "eventType": "DecisionTaskCompleted",
         "decisionTaskCompletedEventAttributes": {"scheduledEventId": 2, "startedEventId": 3}},
        {"eventId": 5, "version": 1, "timestamp": t0 + 4, "eventType": "TimerStarted",
         "timerStartedEventAttributes": {"timerId": "tid-after", "startToFireTimeoutSeconds": 15}},
        {"eventId": 6, "version": 1, "timestamp": t0 + 5, "eventType": "TimerStarted",
         "timerStartedEventAttributes": {"timerId": "tid-before", "startToFireTimeoutSeconds": 1}}])
    b, out = run(hb)
    got = {b.strings[t.timer_id]: t.task_id for t in out.rows(0, "timer")}
    # both were the head when started: tid-after at event 5, tid-before at event 6
    assert got == {"tid-after": 1, "tid-before": 1}
    # a later-expiring timer started second never becomes the head
    hb = HistoryBuilder()
    w, t0 = _head(hb)
    w.calls.append([
        {"eventId": 4, "version": 1, "timestamp": t0 + 3, "eventType": "DecisionTaskCompleted",
         "decisionTaskCompletedEventAttributes": {"scheduledEventId": 2, "startedEventId": 3}},
        {"eventId": 5, "version": 1, "timestamp": t0 + 4, "eventType": "TimerStarted",
         "timerStartedEventAttributes": {"timerId": "tid-before", "startToFireTimeoutSeconds": 1}},
        {"eventId": 6, "version": 1, "timestamp": t0 + 5, "eventType": "TimerStarted",
         "timerStartedEventAttributes": {"timerId": "tid-after", "startToFireTimeoutSeconds": 15}}])
    b, out = run(hb)
    got = {b.strings[t.timer_id]: t.task_id for t in out.rows(0, "timer")}
    assert got == {"tid-before": 1, "tid-after": 0}


def test_timer_builder_activity_timer():  # :190-215 ScheduleToStart first, Heartbeat after start
    hb = HistoryBuilder()
    w, t0 = _head(hb)
    w.calls.append([
        {"eventId": 4, "version": 1, "timestamp": t0 + 3, "eventType": "DecisionTaskCompleted",
         "decisionTaskCompletedEventAttributes": {"scheduledEventId": 2, "startedEventId": 3}},
        {"eventId": 5, "version": 1, "timestamp": t0 + 4, "eventType": "ActivityTaskScheduled",
         "activityTaskScheduledEventAttributes": {
             "activityId": "test-id", "scheduleToStartTimeoutSeconds": 2, "startToCloseTimeoutSeconds": 2,
             "heartbeatTimeoutSeconds": 1, "scheduleToCloseTimeoutSeconds": 3, "taskList": {"name": "task-list"}}}])
    b, out = run(hb)
    (a,) = out.rows(0, "act")
    assert a.timer_task_status == abi.TTS_SCHEDULE_TO_START
    w.calls.append([{"eventId": 6, "version": 1, "timestamp": t0 + 5, "eventType": "ActivityTaskStarted",
                     "activityTaskStartedEventAttributes": {"scheduledEventId": 5, "requestId": "x"}}])
    b, out = run(hb)
    (a,) = out.rows(0, "act")
    assert a.timer_task_status == abi.TTS_SCHEDULE_TO_START | abi.TTS_HEARTBEAT
    assert a.started_id == 6 and a.started_time == t0 + 5 and a.last_heartbeat_time == t0 + 5


# ---- 6. mutableStateBuilder_test.go:82-257,478-491 ------------------------------
def test_transient_decision_after_failure():
    """Started, DTScheduled, DTStarted, DTFailed replayed on a 2DC builder: FailDecision
    increments the attempt and a transient decision is scheduled at the call's
    NextEventID with now (mutableStateDecisionTaskManager.go:169-198,635-656)."""
    hb = HistoryBuilder()
    w = hb.workflow(workflow_id="some random workflow ID", run_id="rid", request_id="q", builder=abi.BUILDER_2DC,
                    failover_version=12)
    t = 1_600_000_000 * NS
    w.calls = [[
        {"eventId": 1, "version": 12, "timestamp": t, "eventType": "WorkflowExecutionStarted",
         "workflowExecutionStartedEventAttributes": {"workflowType": {"name": "some random workflow type"},
                                                     "taskList": {"name": "some random tasklist"},
                                                     "executionStartToCloseTimeoutSeconds": 222,
                                                     "taskStartToCloseTimeoutSeconds": 11}},
        {"eventId": 2, "version": 12, "timestamp": t, "eventType": "DecisionTaskScheduled",
         "decisionTaskScheduledEventAttributes": {"startToCloseTimeoutSeconds": 11, "attempt": 0}},
        {"eventId": 3, "version": 12, "timestamp": t, "eventType": "DecisionTaskStarted",
         "decisionTaskStartedEventAttributes": {"scheduledEventId": 2, "requestId": "req-3"}},
        {"eventId": 4, "version": 12, "timestamp": t, "eventType": "DecisionTaskFailed",
         "decisionTaskFailedEventAttributes": {"scheduledEventId": 2, "startedEventId": 3}}]]
    cluster = abi.CdrClusterMeta(failover_version_increment=10, current_cluster=0, n_clusters=2)
    cluster.initial_version[0], cluster.initial_version[1] = 2, 1
    b, out = run(hb, cluster=cluster, now_ns=123456789)
    x = out.exec[0]
    assert out.result[0].code == abi.OK
    assert x.state == abi.STATE_RUNNING
    assert (x.decision_attempt, x.decision_schedule_id, x.decision_started_id) == (1, 1, -23)
    assert (x.decision_version, x.decision_timeout, x.decision_scheduled_ts) == (12, 11, 123456789)
    assert x.decision_original_scheduled_ts == 0
    # a replicated DecisionTaskStarted resets the attempt to 0 (:224)
    w.calls.append([
        {"eventId": 5, "version": 12, "timestamp": t, "eventType": "DecisionTaskScheduled",
         "decisionTaskScheduledEventAttributes": {"startToCloseTimeoutSeconds": 11, "attempt": 123}},
        {"eventId": 6, "version": 12, "timestamp": t + 1, "eventType": "DecisionTaskStarted",
         "decisionTaskStartedEventAttributes": {"scheduledEventId": 5, "requestId": "req-6"}}])
    b, out = run(hb, cluster=cluster)
    x = out.exec[0]
    assert (x.decision_attempt, x.decision_schedule_id, x.decision_started_id) == (0, 5, 6)


def test_merge_map_of_byte_array():  # :478-491 via UpsertWorkflowSearchAttributes
    hb = HistoryBuilder()
    w, t0 = _head(hb)
    w.calls.append([
        {"eventId": 4, "version": 1, "timestamp": t0 + 3, "eventType": "DecisionTaskCompleted",
         "decisionTaskCompletedEventAttributes": {"scheduledEventId": 2, "startedEventId": 3}},
        {"eventId": 5, "version": 1, "eventType": "UpsertWorkflowSearchAttributes",
         "upsertWorkflowSearchAttributesEventAttributes": {"searchAttributes": {"indexedFields": {}}}}])
    b, out = run(hb)
    assert out.exec[0].flags & abi.XI_HAS_SEARCH_ATTR and out.result[0].n_search_attr == 0
    w.calls[-1].append({"eventId": 6, "version": 1, "eventType": "UpsertWorkflowSearchAttributes",
                        "upsertWorkflowSearchAttributesEventAttributes": {
                            "searchAttributes": {"indexedFields": {"key": "val"}}}})
    w.calls[-1].append({"eventId": 7, "version": 1, "eventType": "UpsertWorkflowSearchAttributes",
                        "upsertWorkflowSearchAttributesEventAttributes": {
                            "searchAttributes": {"indexedFields": {"number": "1", "key": "val2"}}}})
    b, out = run(hb)
    got = {b.strings[kv.key]: b.strings[kv.value] for kv in out.rows(0, "sa")}
    assert got == {"key": "val2", "number": "1"}


# ---- 7. stateBuilder_test.go dispatch checks (state side) -----------------------
def test_unknown_event_type_is_bad_request():  # stateBuilder.go:597-599
    hb = HistoryBuilder()
    w, t0 = _head(hb)
    w.calls.append([{"eventId": 4, "version": 1, "eventType": 99}])
    _, out = run(hb)
    assert (out.result[0].code, out.result[0].fail_event_id) == (3, 4)


def test_empty_history_is_internal_failure():  # stateBuilder.go:121-123
    hb = HistoryBuilder()
    w = hb.workflow(workflow_id="w", run_id="r", request_id="q")
    w.calls = []
    _, out = run(hb)
    assert out.result[0].code == 1


def test_batch_id_is_first_event_of_call():  # stateBuilder.go:260, :1814 of the test
    hb = HistoryBuilder()
    w, t0 = _head(hb)
    w.calls.append([
        {"eventId": 4, "version": 1, "timestamp": t0 + 3, "eventType": "DecisionTaskCompleted",
         "decisionTaskCompletedEventAttributes": {"scheduledEventId": 2, "startedEventId": 3}},
        {"eventId": 5, "version": 1, "timestamp": t0 + 4, "eventType": "ActivityTaskScheduled",
         "activityTaskScheduledEventAttributes": {"activityId": "a", "scheduleToCloseTimeoutSeconds": 9}}])
    _, out = run(hb)
    (a,) = out.rows(0, "act")
    assert a.scheduled_event_batch_id == 4
    assert out.exec[0].last_first_event_id == 4 and out.exec[0].next_event_id == 6


def test_activity_started_missing_is_panic():  # mutableStateBuilder.go:2089-2091
    hb = HistoryBuilder()
    w, t0 = _head(hb)
    w.calls.append([{"eventId": 4, "version": 1, "eventType": "ActivityTaskStarted",
                     "activityTaskStartedEventAttributes": {"scheduledEventId": 77}}])
    _, out = run(hb)
    assert out.result[0].code == 32


def test_continue_as_new_without_new_run_history():  # stateBuilder.go:538-540
    hb = HistoryBuilder()
    w, t0 = _head(hb)
    w.calls.append([
        {"eventId": 4, "version": 1, "eventType": "DecisionTaskCompleted",
         "decisionTaskCompletedEventAttributes": {"scheduledEventId": 2, "startedEventId": 3}},
        {"eventId": 5, "version": 1, "eventType": "WorkflowExecutionContinuedAsNew",
         "workflowExecutionContinuedAsNewEventAttributes": {"newExecutionRunId": "nr"}}])
    _, out = run(hb)
    assert (out.result[0].code, out.result[0].fail_event_id) == (2, 5)
