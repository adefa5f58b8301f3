"""Decoded-history construction: HistoryEvent-like dicts -> the ABI's cdr_event batch.

This is the host-side packing step the reference performs implicitly by holding
``[]*shared.HistoryEvent`` (thrift-decoded, .gen/go/shared/shared.go:19567-19615):
events keep their ids, versions, timestamps and task ids; strings are interned to
u32 handles (0 = "", 1 = "emptyUuid"); attribute fields the replay path reads are
copied into the per-type attribute records of include/cdr/schema.h.

Two front ends:
  * ``HistoryBuilder`` — programmatic (used to restate the reference's KATs);
  * ``from_cadence_json`` — the JSON form of shared.HistoryEvent the reference's
    fixtures use (e.g. service/worker/archiver/testdata/*.json).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

from . import abi
from .engine import Batch, default_cluster


class Interner:
    def __init__(self):
        self.strings = ["", "emptyUuid"]
        self.index = {"": 0, "emptyUuid": 1}

    def __call__(self, s) -> int:
        if s is None:
            return 0
        if isinstance(s, bytes):
            s = "b64:" + s.hex()
        h = self.index.get(s)
        if h is None:
            h = len(self.strings)
            self.strings.append(s)
            self.index[s] = h
        return h


@dataclass
class Workflow:
    workflow_id: str
    run_id: str
    request_id: str
    domain_id: str = "domain-id"
    builder: int = abi.BUILDER_NDC
    failover_version: int = 0
    retention_days: int = 1
    expected_next_event_id: int = 0
    calls: list = field(default_factory=list)  # list of lists of event dicts
    new_run_history: list | None = None        # events of the continue-as-new run
    new_run_call: int = 0
    new_run_ndc: bool = True
    new_run_request_id: str = "new-run-request-id"


class HistoryBuilder:
    def __init__(self):
        self.intern = Interner()
        self.workflows: list[Workflow] = []
        self.domains_missing: set = set()
        self.domain_ids: dict = {}

    def workflow(self, **kw) -> Workflow:
        w = Workflow(**kw)
        self.workflows.append(w)
        return w

    # ---- event conversion (attribute names follow shared.thrift)
    def _event(self, e: dict, batch_first: bool, kvs: list, rps: list) -> abi.CdrEvent:
        I = self.intern
        out = abi.CdrEvent()
        out.event_id = int(e["eventId"])
        out.version = int(e.get("version", 0))  # GetVersion() of a nil pointer is 0
        out.timestamp = int(e.get("timestamp", 0))
        out.task_id = int(e.get("taskId", 0))
        et = e.get("eventType", "WorkflowExecutionStarted")
        out.type = abi.EV[et] if isinstance(et, str) else int(et)
        out.flags = abi.EVF_BATCH_FIRST if batch_first else 0
        a = out.a

        def attrs(key):
            return e.get(key) or {}

        name = abi.EVENT_TYPES[out.type] if out.type < len(abi.EVENT_TYPES) else None
        if name == "WorkflowExecutionStarted":
            x = attrs("workflowExecutionStartedEventAttributes")
            s = a.started
            s.workflow_type = I((x.get("workflowType") or {}).get("name", ""))
            s.task_list = I((x.get("taskList") or {}).get("name", ""))
            s.exec_timeout_s = int(x.get("executionStartToCloseTimeoutSeconds", 0))
            s.task_timeout_s = int(x.get("taskStartToCloseTimeoutSeconds", 0))
            s.cron_schedule = I(x.get("cronSchedule", ""))
            s.attempt = int(x.get("attempt", 0))
            s.first_decision_backoff_s = int(x.get("firstDecisionTaskBackoffSeconds", 0))
            init = x.get("initiator")  # ContinueAsNewInitiator: Decider 0, RetryPolicy 1, CronSchedule 2
            cron_init = init in ("CronSchedule", "CRON_SCHEDULE", 2)
            s.expiration_ts = int(x.get("expirationTimestamp", 0))
            f = 0
            if x.get("parentWorkflowDomain") is not None:
                f |= abi.SF_HAS_PARENT_DOMAIN
                dom = x["parentWorkflowDomain"]
                if dom in self.domains_missing:
                    f |= abi.SF_PARENT_DOMAIN_MISSING
                s.parent_domain_id = I(self.domain_ids.get(dom, "id-of-" + dom))
            if x.get("parentWorkflowExecution") is not None:
                f |= abi.SF_HAS_PARENT_EXEC
                s.parent_workflow_id = I(x["parentWorkflowExecution"].get("workflowId", ""))
                s.parent_run_id = I(x["parentWorkflowExecution"].get("runId", ""))
            if x.get("parentInitiatedEventId") is not None:
                f |= abi.SF_HAS_PARENT_INITIATED
                s.parent_initiated_id = int(x["parentInitiatedEventId"])
            if cron_init:
                f |= abi.SF_CRON_INITIATOR
            if init is not None:
                f |= abi.SF_HAS_INITIATOR
                if init in ("RetryPolicy", "RETRY_POLICY", 1):
                    f |= abi.SF_RETRY_INITIATOR
                elif init in ("Decider", "DECIDER", 0):
                    f |= abi.SF_DECIDER_INITIATOR
            rp = x.get("retryPolicy")
            if rp is not None:
                f |= abi.SF_HAS_RETRY
                s.backoff_coefficient = float(rp.get("backoffCoefficient", 0))
                s.retry_initial_s = int(rp.get("initialIntervalInSeconds", 0))
                s.retry_max_interval_s = int(rp.get("maximumIntervalInSeconds", 0))
                s.retry_max_attempts = int(rp.get("maximumAttempts", 0))
                s.retry_expiration_s = int(rp.get("expirationIntervalInSeconds", 0))
                s.nonretriable = I("\x1f".join(rp.get("nonRetriableErrorReasons") or []))
            if x.get("memo") is not None:
                f |= abi.SF_HAS_MEMO
                s.memo = I(repr(sorted((x["memo"].get("fields") or {}).items())))
            if x.get("searchAttributes") is not None:
                f |= abi.SF_HAS_SEARCH_ATTR
                fields = x["searchAttributes"].get("indexedFields") or {}
                s.search_attr_off = len(kvs)
                s.search_attr_len = len(fields)
                for k, v in fields.items():
                    kvs.append((I(k), I(v)))
            prp = x.get("prevAutoResetPoints")
            if prp is not None and prp.get("points") is not None:
                f |= abi.SF_HAS_RESET_POINTS
                s.reset_points_off = len(rps)
                s.reset_points_len = len(prp["points"])
                for p in prp["points"]:
                    r = abi.CdrResetPoint()
                    pf = 0
                    if "binaryChecksum" in p:
                        pf |= abi.RP_HAS_CHECKSUM
                        r.binary_checksum = I(p["binaryChecksum"])
                    if "runId" in p:
                        pf |= abi.RP_HAS_RUN_ID
                        r.run_id = I(p["runId"])
                    if "firstDecisionCompletedId" in p:
                        pf |= abi.RP_HAS_FIRST_DC_ID
                        r.first_decision_completed_id = int(p["firstDecisionCompletedId"])
                    if "createdTimeNano" in p:
                        pf |= abi.RP_HAS_CREATED
                        r.created_time_nano = int(p["createdTimeNano"])
                    if "expiringTimeNano" in p:
                        pf |= abi.RP_HAS_EXPIRING
                        r.expiring_time_nano = int(p["expiringTimeNano"])
                    if "resettable" in p:
                        pf |= abi.RP_HAS_RESETTABLE | (abi.RP_RESETTABLE if p["resettable"] else 0)
                    r.flags = pf
                    rps.append(r)
            s.continued_run_id = I(x.get("continuedExecutionRunId", ""))
            s.flags = f
        elif name == "DecisionTaskScheduled":
            x = attrs("decisionTaskScheduledEventAttributes")
            a.dt_sched.attempt = int(x.get("attempt", 0))
            a.dt_sched.start_to_close_s = int(x.get("startToCloseTimeoutSeconds", 0))
            a.dt_sched.task_list = I((x.get("taskList") or {}).get("name", ""))
        elif name in ("DecisionTaskStarted", "DecisionTaskCompleted", "DecisionTaskTimedOut", "DecisionTaskFailed"):
            x = attrs(name[0].lower() + name[1:] + "EventAttributes")
            a.dt.scheduled_event_id = int(x.get("scheduledEventId", 0))
            a.dt.started_event_id = int(x.get("startedEventId", 0))
            a.dt.request_id = I(x.get("requestId", ""))
            a.dt.binary_checksum = I(x.get("binaryChecksum", ""))
            to = x.get("timeoutType", 0)
            a.dt.timeout_type = {"START_TO_CLOSE": 0, "SCHEDULE_TO_START": 1, "SCHEDULE_TO_CLOSE": 2,
                                 "HEARTBEAT": 3}.get(to, to) if isinstance(to, str) else int(to)
        elif name == "ActivityTaskScheduled":
            x = attrs("activityTaskScheduledEventAttributes")
            s = a.at_sched
            s.activity_id = I(x.get("activityId", ""))
            s.task_list = I((x.get("taskList") or {}).get("name", ""))
            s.s2s_s = int(x.get("scheduleToStartTimeoutSeconds", 0))
            s.s2c_s = int(x.get("scheduleToCloseTimeoutSeconds", 0))
            s.stc_s = int(x.get("startToCloseTimeoutSeconds", 0))
            s.hb_s = int(x.get("heartbeatTimeoutSeconds", 0))
            dom = x.get("domain", "")  # the activity's target domain (refreshTasks, getTargetDomainID)
            s.domain = I(dom)
            if dom:
                s.target_domain_id = I(self.domain_ids.get(dom, "id-of-" + dom))
                s.flags |= abi.AF_DOMAIN_MISSING if dom in self.domains_missing else 0
            rp = x.get("retryPolicy")
            if rp is not None:
                s.flags |= abi.AF_HAS_RETRY
                s.backoff_coefficient = float(rp.get("backoffCoefficient", 0))
                s.retry_initial_s = int(rp.get("initialIntervalInSeconds", 0))
                s.retry_max_interval_s = int(rp.get("maximumIntervalInSeconds", 0))
                s.retry_max_attempts = int(rp.get("maximumAttempts", 0))
                s.retry_expiration_s = int(rp.get("expirationIntervalInSeconds", 0))
                s.nonretriable = I("\x1f".join(rp.get("nonRetriableErrorReasons") or []))
        elif name in ("ActivityTaskStarted", "ActivityTaskCompleted", "ActivityTaskFailed", "ActivityTaskTimedOut",
                      "ActivityTaskCanceled", "ActivityTaskCancelRequested", "RequestCancelActivityTaskFailed"):
            x = attrs(name[0].lower() + name[1:] + "EventAttributes")
            a.at.scheduled_event_id = int(x.get("scheduledEventId", 0))
            a.at.started_event_id = int(x.get("startedEventId", 0))
            a.at.request_id = I(x.get("requestId", ""))
            a.at.activity_id = I(x.get("activityId", ""))
        elif name in ("TimerStarted", "TimerFired", "TimerCanceled", "CancelTimerFailed"):
            x = attrs(name[0].lower() + name[1:] + "EventAttributes")
            a.timer.timer_id = I(x.get("timerId", ""))
            a.timer.start_to_fire_s = int(x.get("startToFireTimeoutSeconds", 0))
            a.timer.started_event_id = int(x.get("startedEventId", 0))
        elif name in ("StartChildWorkflowExecutionInitiated", "SignalExternalWorkflowExecutionInitiated",
                      "RequestCancelExternalWorkflowExecutionInitiated"):
            x = attrs(name[0].lower() + name[1:] + "EventAttributes")
            ex = a.ext
            ex.domain = I(x.get("domain", ""))
            ex.flags = abi.XF_DOMAIN_MISSING if x.get("domain", "") in self.domains_missing else 0
            ex.flags |= abi.XF_CHILD_ONLY if x.get("childWorkflowOnly") else 0
            dom = x.get("domain", "")
            ex.target_domain_id = I(self.domain_ids.get(dom, "id-of-" + dom))  # the domain cache's ID
            we = x.get("workflowExecution") or {}
            ex.workflow_id = I(x.get("workflowId", we.get("workflowId", "")))
            ex.run_id = I(we.get("runId", ""))
            ex.workflow_type = I((x.get("workflowType") or {}).get("name", ""))
            ex.signal_name = I(x.get("signalName", ""))
            ex.input = I(x.get("input"))
            ex.control = I(x.get("control"))
            pcp = x.get("parentClosePolicy", 0)
            ex.parent_close_policy = {"ABANDON": 0, "REQUEST_CANCEL": 1, "TERMINATE": 2}.get(pcp, pcp) \
                if isinstance(pcp, str) else int(pcp)
        elif name in ("StartChildWorkflowExecutionFailed", "ChildWorkflowExecutionStarted",
                      "ChildWorkflowExecutionCompleted", "ChildWorkflowExecutionFailed",
                      "ChildWorkflowExecutionCanceled", "ChildWorkflowExecutionTimedOut",
                      "ChildWorkflowExecutionTerminated", "SignalExternalWorkflowExecutionFailed",
                      "ExternalWorkflowExecutionSignaled", "RequestCancelExternalWorkflowExecutionFailed",
                      "ExternalWorkflowExecutionCancelRequested"):
            x = attrs(name[0].lower() + name[1:] + "EventAttributes")
            a.ref.initiated_event_id = int(x.get("initiatedEventId", 0))
            a.ref.run_id = I((x.get("workflowExecution") or {}).get("runId", ""))
        elif name == "WorkflowExecutionContinuedAsNew":
            x = attrs("workflowExecutionContinuedAsNewEventAttributes")
            a.can.new_execution_run_id = I(x.get("newExecutionRunId", ""))
        elif name == "UpsertWorkflowSearchAttributes":
            x = attrs("upsertWorkflowSearchAttributesEventAttributes")
            fields = (x.get("searchAttributes") or {}).get("indexedFields") or {}
            a.upsert.search_attr_off = len(kvs)
            a.upsert.search_attr_len = len(fields)
            for k, v in fields.items():
                kvs.append((I(k), I(v)))
        return out

    def build(self, now_ns: int = 1_700_000_000_000_000_000, uuid_seed: int = 1,
              cluster: abi.CdrClusterMeta | None = None) -> Batch:
        I = self.intern
        events, descs, kvs, rps = [], [], [], []
        for wi, w in enumerate(self.workflows):
            d = abi.CdrWfDesc()
            d.wf_key = 0x1000 + wi
            d.ev_off = len(events)
            for c in w.calls:
                for j, e in enumerate(c):
                    events.append(self._event(e, j == 0, kvs, rps))
            d.ev_len = len(events) - d.ev_off
            d.domain_id = I(w.domain_id)
            d.workflow_id = I(w.workflow_id)
            d.run_id = I(w.run_id)
            d.request_id = I(w.request_id)
            d.builder = w.builder
            d.retention_days = w.retention_days
            d.failover_version = w.failover_version
            d.expected_next_event_id = w.expected_next_event_id
            d.parent = -1
            d.newrun = -1
            descs.append(d)
            if w.new_run_history is not None:
                n = abi.CdrWfDesc()
                n.wf_key = 0x100000 + wi
                n.ev_off = len(events)
                for j, e in enumerate(w.new_run_history):
                    events.append(self._event(e, j == 0, kvs, rps))
                n.ev_len = len(events) - n.ev_off
                can = [e for c in w.calls[w.new_run_call:w.new_run_call + 1] for e in c
                       if e.get("eventType") == "WorkflowExecutionContinuedAsNew"]
                nr_run = (can[0].get("workflowExecutionContinuedAsNewEventAttributes") or {}).get(
                    "newExecutionRunId", "") if can else ""
                n.domain_id = d.domain_id
                n.workflow_id = d.workflow_id
                n.run_id = I(nr_run)
                n.request_id = I(w.new_run_request_id)
                n.builder = abi.BUILDER_NDC if w.new_run_ndc else abi.BUILDER_2DC
                n.retention_days = w.retention_days
                n.failover_version = w.failover_version
                n.parent = len(descs) - 1
                n.newrun = -1
                d.newrun = len(descs)
                d.newrun_call = w.new_run_call
                d.newrun_ndc = 1 if w.new_run_ndc else 0
                descs.append(n)
        ev = (abi.CdrEvent * len(events))(*events)
        wf = (abi.CdrWfDesc * len(descs))(*descs)
        kv = (abi.CdrKV * len(kvs))(*[abi.CdrKV(k, v) for k, v in kvs])
        rp = (abi.CdrResetPoint * len(rps))(*rps)
        return Batch(events=ev, wfs=wf, kvs=kv, rps=rp, cluster=cluster or default_cluster(), now_ns=now_ns,
                     uuid_seed=uuid_seed, empty_uuid=1, strings=list(I.strings))


def from_cadence_json(events: list, *, workflow_id="wid", run_id="rid", request_id="req",
                      builder=abi.BUILDER_NDC, failover_version=0, batching="single", **kw) -> Batch:
    """One workflow from a JSON list of shared.HistoryEvent.  JSON fixtures carry no
    batch boundaries: ``batching="single"`` replays them as one applyEvents call (as
    conflictResolver.reset replays pages, conflictResolver.go:94-133), ``"each"`` as
    one call per event."""
    hb = HistoryBuilder()
    w = hb.workflow(workflow_id=workflow_id, run_id=run_id, request_id=request_id, builder=builder,
                    failover_version=failover_version, **kw)
    w.calls = [list(events)] if batching == "single" else [[e] for e in events]
    return hb.build()
