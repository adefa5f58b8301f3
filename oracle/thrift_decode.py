"""TEST INFRASTRUCTURE ONLY: CPU restatement of the on-device history decode
(cadence_amd/csrc/ingest.hip, cdr/ingest.h) — the parity checker for it.

Restates go.uber.org/thriftrw protocol.Binary decoding (the wire rules of
common/codec/version0Thriftrw.go:62-84 Decode: preamble 0x59, then a binary-protocol
struct) of shared.History{10: list<HistoryEvent>} into the replay's record form
(schema.h cdr_event / cdr_kv / cdr_reset_point), field by field from the IDL
(idl/github.com/uber/cadence/shared.thrift:868-920 and the attribute structs), with the
string-table convention of cdr/ingest.h: seeds keep their handles, every other distinct
string gets n_seeds + its rank by cdr_str_hash, the empty string is 0, Memo and
non-empty nonRetriableErrorReasons are interned by their value bytes.  Pure Python,
recursive, written independently of the device parser; pinned to the golden bytes of
common/codec/version0Thriftrw_test.go:42-64 (tests/test_ingest.py).
"""
from __future__ import annotations

import ctypes as C
import struct

M64 = (1 << 64) - 1
T_STOP, T_BOOL, T_BYTE, T_DOUBLE, T_I16, T_I32, T_I64, T_STRING, T_STRUCT, T_MAP, T_SET, T_LIST = (
    0, 2, 3, 4, 6, 8, 10, 11, 12, 13, 14, 15)
FIXED = {T_BOOL: 1, T_BYTE: 1, T_I16: 2, T_I32: 4, T_I64: 8, T_DOUBLE: 8}
DEC_OK, DEC_MISSING_VERSION, DEC_INVALID_VERSION, DEC_TRUNCATED, DEC_DEPTH, DEC_NO_EVENTS, DEC_BAD_SIZE, \
    DEC_BAD_TYPE = range(8)
MAX_DEPTH = 16


class DecodeError(Exception):
    def __init__(self, code):
        super().__init__(code)
        self.code = code


def mix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def str_hash(b: bytes) -> int:
    """cdr_str_hash (cdr/ingest.h)."""
    h = 0xCBF29CE484222325
    for c in b:
        h = ((h ^ c) * 0x100000001B3) & M64
    h = mix64(h ^ ((len(b) * 0x9E3779B97F4A7C15) & M64))
    return h or 1


# ------------------------------------------------------------------ wire values
class Reader:
    def __init__(self, data: bytes, pos: int, end: int):
        self.d, self.p, self.end = data, pos, end

    def take(self, n):
        if self.end - self.p < n:
            raise DecodeError(DEC_TRUNCATED)
        v = self.d[self.p:self.p + n]
        self.p += n
        return v

    def u8(self):
        return self.take(1)[0]

    def i16(self):
        return struct.unpack(">h", self.take(2))[0]

    def i32(self):
        return struct.unpack(">i", self.take(4))[0]

    def i64(self):
        return struct.unpack(">q", self.take(8))[0]

    def size(self):
        n = self.i32()
        if n < 0:
            raise DecodeError(DEC_BAD_SIZE)
        return n

    def value(self, t, depth=0):
        """A generic wire value: ints / bytes / ("struct", {id: (type, value, (start, end))}) /
        ("list", elem type, [values]) / ("map", kt, vt, [(k, v)])."""
        if t in FIXED:
            raw = self.take(FIXED[t])
            if t == T_DOUBLE:
                return struct.unpack(">d", raw)[0]
            return int.from_bytes(raw, "big", signed=True) if t != T_BOOL else raw[0]
        if t == T_STRING:
            return bytes(self.take(self.size()))
        if t in (T_STRUCT, T_LIST, T_SET, T_MAP):
            if depth >= MAX_DEPTH:
                raise DecodeError(DEC_DEPTH)
            if t == T_STRUCT:
                fields = []
                while True:
                    ft = self.u8()
                    if ft == T_STOP:
                        return ("struct", fields)
                    fid = self.i16()
                    start = self.p
                    v = self.value(ft, depth + 1)
                    fields.append((fid, ft, v, (start, self.p)))
            if t in (T_LIST, T_SET):
                et = self.u8()
                n = self.size()
                return ("list", et, [self.value(et, depth + 1) for _ in range(n)])
            kt, vt = self.u8(), self.u8()
            n = self.size()
            return ("map", kt, vt, [(self.value(kt, depth + 1), self.value(vt, depth + 1)) for _ in range(n)])
        raise DecodeError(DEC_BAD_TYPE)


def fget(st, fid, ftype):
    """The value of field `fid` when it has wire type `ftype` (the last one wins, as a
    thriftrw FromWire loop assigns each occurrence in turn); None otherwise."""
    out = None
    for i, t, v, span in st[1]:
        if i == fid and t == ftype:
            out = (v, span)
    return out


# ------------------------------------------------------------------ the record form
class Interner:
    """Strings of one decode (seeds first)."""

    def __init__(self, seeds: list[bytes]):
        self.seed_index = {}
        for i, s in enumerate(seeds):
            if i and s and str_hash(s) not in self.seed_index:
                self.seed_index[str_hash(s)] = i
        self.n_seeds = len(seeds)
        self.new = {}  # hash -> bytes

    def add(self, b: bytes):
        if b:
            h = str_hash(b)
            if h not in self.seed_index and h not in self.new:
                self.new[h] = b

    def finish(self):
        self.rank = {h: self.n_seeds + r for r, h in enumerate(sorted(self.new))}

    def handle(self, b: bytes) -> int:
        if not b:
            return 0
        h = str_hash(b)
        return self.seed_index[h] if h in self.seed_index else self.rank[h]


def _name(v):  # WorkflowType / TaskList{10: name}
    return v if v is None else (fget(v[0], 10, T_STRING) or (b"", None))[0]


def decode_blobs(data: bytes, blob_off, entry_blob0, seeds: list[bytes], domain_map: list[tuple[int, int]],
                 abi):
    """Decode every blob; returns (events [CdrEvent], kvs [CdrKV], rps [CdrResetPoint],
    ev_off [n_entries + 1], blob_status, entry_status, strings [bytes per handle])."""
    n_blobs = len(blob_off) - 1
    parsed, status = [], []
    for b in range(n_blobs):
        r = Reader(data, int(blob_off[b]), int(blob_off[b + 1]))
        try:
            if r.end <= r.p:
                raise DecodeError(DEC_MISSING_VERSION)
            if r.u8() != 0x59:
                raise DecodeError(DEC_INVALID_VERSION)
            hist = r.value(T_STRUCT)
            evs = []
            lst = fget(hist, 10, T_LIST)
            if lst is not None and lst[0][1] == T_STRUCT:
                evs = lst[0][2]
            if not evs:
                raise DecodeError(DEC_NO_EVENTS)
            parsed.append(evs)
            status.append(DEC_OK)
        except DecodeError as e:
            parsed.append([])
            status.append(e.code)
    it = Interner(seeds)
    dom = {name: ident for name, ident in domain_map}

    # every kept string, in a first walk (the same accessors as the fill below)
    def strings_of(events):
        for ev in events:
            for s in _event(ev, None, None, data, it, dom, abi, collect=True):
                it.add(s)
    for b, evs in enumerate(parsed):
        strings_of(evs)
    it.finish()
    events, kvs, rps, ev_count = [], [], [], []
    for evs in parsed:
        for i, ev in enumerate(evs):
            e = _event(ev, kvs, rps, data, it, dom, abi)
            e.flags = abi.EVF_BATCH_FIRST if i == 0 else 0
            events.append(e)
        ev_count.append(len(evs))
    base = [0]
    for c in ev_count:
        base.append(base[-1] + c)
    ev_off = [base[entry_blob0[w]] for w in range(len(entry_blob0))]
    entry_status = []
    for w in range(len(entry_blob0) - 1):
        st = DEC_OK
        for b in range(entry_blob0[w], entry_blob0[w + 1]):
            if st == DEC_OK:
                st = status[b]
        entry_status.append(st)
    strings = list(seeds) + [it.new[h] for h in sorted(it.new)]
    return events, kvs, rps, ev_off, status, entry_status, strings


def _event(ev, kvs, rps, data, it, dom, abi, collect=False):
    """One HistoryEvent struct -> CdrEvent (or, with collect, the strings it keeps)."""
    out = []

    def S(b):  # a kept string
        if collect:
            out.append(b)
            return 0
        return it.handle(b)
    e = abi.CdrEvent()
    for fid, ft, v, span in ev[1]:
        if fid == 10 and ft == T_I64:
            e.event_id = v
        elif fid == 20 and ft == T_I64:
            e.timestamp = v
        elif fid == 30 and ft == T_I32:
            e.type = v & 0xFFFFFFFF
        elif fid == 35 and ft == T_I64:
            e.version = v
        elif fid == 36 and ft == T_I64:
            e.task_id = v
        elif ft == T_STRUCT and 40 <= fid <= 450 and fid % 10 == 0:
            _attrs(fid, v, e, S, kvs, rps, data, dom, collect)
    return out if collect else e


def _domain(dom, handle):
    ident = dom.get(handle)
    return (0, True) if ident is None else (ident, False)


def _retry(st, a, S, data):
    for fid, ft, v, span in st[1]:
        if fid == 10 and ft == T_I32:
            a.retry_initial_s = v
        elif fid == 20 and ft == T_DOUBLE:
            a.backoff_coefficient = v
        elif fid == 30 and ft == T_I32:
            a.retry_max_interval_s = v
        elif fid == 40 and ft == T_I32:
            a.retry_max_attempts = v
        elif fid == 60 and ft == T_I32:
            a.retry_expiration_s = v
        elif fid == 50 and ft == T_LIST:
            a.nonretriable = S(bytes(data[span[0]:span[1]])) if v[2] else 0
    return a


def _search_attrs(st, S, kvs, collect):
    off = len(kvs) if kvs is not None else 0
    n = 0
    m = fget(st, 10, T_MAP)
    if m is not None and m[0][1] == T_STRING and m[0][2] == T_STRING:
        for k, v in m[0][3]:
            kk, vv = S(k), S(v)
            if not collect:
                kvs.append((kk, vv))
            n += 1
    return off, n


def _attrs(fid, st, e, S, kvs, rps, data, dom, collect):
    from cadence_amd import abi
    a = e.a
    g = lambda f, t: fget(st, f, t)  # noqa: E731
    val = lambda f, t, d=0: (g(f, t) or (d, None))[0]  # noqa: E731
    if fid == 40:
        s = a.started
        s.workflow_type = S(_name(g(10, T_STRUCT)) or b"")
        flags = 0
        if g(12, T_STRING) is not None:
            flags |= abi.SF_HAS_PARENT_DOMAIN
            ident, miss = _domain(dom, S(g(12, T_STRING)[0]))
            s.parent_domain_id = ident
            flags |= abi.SF_PARENT_DOMAIN_MISSING if miss else 0
        pe = g(14, T_STRUCT)
        if pe is not None:
            flags |= abi.SF_HAS_PARENT_EXEC
            s.parent_workflow_id = S((fget(pe[0], 10, T_STRING) or (b"",))[0])
            s.parent_run_id = S((fget(pe[0], 20, T_STRING) or (b"",))[0])
        if g(16, T_I64) is not None:
            flags |= abi.SF_HAS_PARENT_INITIATED
            s.parent_initiated_id = g(16, T_I64)[0]
        s.task_list = S(_name(g(20, T_STRUCT)) or b"")
        s.exec_timeout_s = val(40, T_I32)
        s.task_timeout_s = val(50, T_I32)
        s.continued_run_id = S(val(54, T_STRING, b""))
        if g(55, T_I32) is not None:
            iv = g(55, T_I32)[0]
            flags |= abi.SF_HAS_INITIATOR | (abi.SF_CRON_INITIATOR if iv == 2 else 0) | (
                abi.SF_RETRY_INITIATOR if iv == 1 else 0) | (abi.SF_DECIDER_INITIATOR if iv == 0 else 0)
        rp = g(70, T_STRUCT)
        if rp is not None:
            flags |= abi.SF_HAS_RETRY
            _retry(rp[0], s, S, data)
        s.attempt = val(80, T_I32)
        s.expiration_ts = val(90, T_I64)
        s.cron_schedule = S(val(100, T_STRING, b""))
        s.first_decision_backoff_s = val(110, T_I32)
        memo = g(120, T_STRUCT)
        if memo is not None:
            flags |= abi.SF_HAS_MEMO
            s.memo = S(bytes(data[memo[1][0]:memo[1][1]]))
        sa = g(121, T_STRUCT)
        if sa is not None:
            flags |= abi.SF_HAS_SEARCH_ATTR
            s.search_attr_off, s.search_attr_len = _search_attrs(sa[0], S, kvs, collect)
        prp = g(130, T_STRUCT)
        if prp is not None:
            pts = fget(prp[0], 10, T_LIST)
            if pts is not None and pts[0][1] == T_STRUCT:
                flags |= abi.SF_HAS_RESET_POINTS
                s.reset_points_off = len(rps) if rps is not None else 0
                s.reset_points_len = len(pts[0][2])
                for pt in pts[0][2]:
                    p = abi.CdrResetPoint()
                    pf = 0
                    if fget(pt, 10, T_STRING) is not None:
                        pf |= abi.RP_HAS_CHECKSUM
                        p.binary_checksum = S(fget(pt, 10, T_STRING)[0])
                    if fget(pt, 20, T_STRING) is not None:
                        pf |= abi.RP_HAS_RUN_ID
                        p.run_id = S(fget(pt, 20, T_STRING)[0])
                    if fget(pt, 30, T_I64) is not None:
                        pf |= abi.RP_HAS_FIRST_DC_ID
                        p.first_decision_completed_id = fget(pt, 30, T_I64)[0]
                    if fget(pt, 40, T_I64) is not None:
                        pf |= abi.RP_HAS_CREATED
                        p.created_time_nano = fget(pt, 40, T_I64)[0]
                    if fget(pt, 50, T_I64) is not None:
                        pf |= abi.RP_HAS_EXPIRING
                        p.expiring_time_nano = fget(pt, 50, T_I64)[0]
                    if fget(pt, 60, T_BOOL) is not None:
                        pf |= abi.RP_HAS_RESETTABLE | (abi.RP_RESETTABLE if fget(pt, 60, T_BOOL)[0] else 0)
                    p.flags = pf
                    if not collect:
                        rps.append(p)
        s.flags = flags
        return
    if fid == 80:
        d = a.dt_sched
        d.task_list = S(_name(g(10, T_STRUCT)) or b"")
        d.start_to_close_s = val(20, T_I32)
        d.attempt = val(30, T_I64)
        return
    if fid == 130:
        x = a.at_sched
        x.activity_id = S(val(10, T_STRING, b""))
        x.domain = S(val(25, T_STRING, b""))
        if x.domain:  # ActivityTaskScheduledEventAttributes.domain (shared.thrift:615) -> getTargetDomainID
            x.target_domain_id, miss = _domain(dom, x.domain)
            x.flags |= abi.AF_DOMAIN_MISSING if miss else 0
        x.task_list = S(_name(g(30, T_STRUCT)) or b"")
        x.s2c_s, x.s2s_s, x.stc_s, x.hb_s = val(45, T_I32), val(50, T_I32), val(55, T_I32), val(60, T_I32)
        rp = g(110, T_STRUCT)
        if rp is not None:
            x.flags |= abi.AF_HAS_RETRY
            _retry(rp[0], x, S, data)
        return
    if fid in (180, 190, 230, 240):
        t = a.timer
        t.timer_id = S(val(10, T_STRING, b""))
        if fid == 180:
            t.start_to_fire_s = val(20, T_I64)
        elif fid != 240:
            t.started_event_id = val(20, T_I64)
        return
    if fid in (300, 340, 420):
        x = a.ext
        child, sig = fid == 340, fid == 420
        dom_name = S(val(10 if child else 20, T_STRING, b""))
        if not child:
            we = g(30, T_STRUCT)
            if we is not None:
                x.workflow_id = S((fget(we[0], 10, T_STRING) or (b"",))[0])
                x.run_id = S((fget(we[0], 20, T_STRING) or (b"",))[0])
        else:
            x.workflow_id = S(val(20, T_STRING, b""))
            x.workflow_type = S(_name(g(30, T_STRUCT)) or b"")
            x.parent_close_policy = val(81, T_I32)
        if sig:
            x.signal_name = S(val(40, T_STRING, b""))
        f_in = 50 if (child or sig) else None
        if f_in:
            x.input = S(val(f_in, T_STRING, b""))
        x.control = S(val(90 if child else (60 if sig else 40), T_STRING, b""))
        fl = 0
        if not child and val(70 if sig else 50, T_BOOL):
            fl |= abi.XF_CHILD_ONLY
        x.domain = dom_name
        ident, miss = _domain(dom, dom_name)
        x.target_domain_id = ident
        x.flags = fl | (abi.XF_DOMAIN_MISSING if miss else 0)
        return
    if fid == 330:
        a.can.new_execution_run_id = S(val(10, T_STRING, b""))
        return
    if fid == 450:
        sa = g(20, T_STRUCT)
        if sa is not None:
            a.upsert.search_attr_off, a.upsert.search_attr_len = _search_attrs(sa[0], S, kvs, collect)
        return
    ids = {90: (10, 0, 30, 0, 0, 0, 0), 100: (20, 30, 0, 0, 0, 0, 50), 110: (10, 20, 0, 0, 30, 0, 0),
           120: (10, 20, 0, 0, 0, 0, 0), 140: (10, 0, 30, 0, 0, 40, 0), 150: (20, 30, 0, 0, 0, 0, 0),
           160: (30, 40, 0, 0, 0, 0, 0), 170: (10, 20, 0, 0, 30, 0, 0), 200: (0, 0, 0, 10, 0, 0, 0),
           210: (0, 0, 0, 10, 0, 0, 0), 220: (30, 40, 0, 0, 0, 0, 0)}
    if fid in ids:
        sch, stt, req, aid, to, att, cks = ids[fid]
        act = fid >= 140
        x = a.at if act else a.dt
        if sch:
            x.scheduled_event_id = val(sch, T_I64)
        if stt:
            x.started_event_id = val(stt, T_I64)
        if req:
            x.request_id = S(val(req, T_STRING, b""))
        if aid:
            a.at.activity_id = S(val(aid, T_STRING, b""))
        if to:
            x.timeout_type = val(to, T_I32)
        if att:
            a.at.attempt = val(att, T_I32)
        if cks:
            a.dt.binary_checksum = S(val(cks, T_STRING, b""))
        return
    refs = {310: (50, 40), 320: (10, 30), 350: (60, 0), 360: (20, 30), 370: (50, 30), 380: (60, 40), 390: (50, 30),
            400: (50, 30), 410: (40, 20), 430: (50, 40), 440: (10, 30)}
    if fid in refs:
        init, we = refs[fid]
        a.ref.initiated_event_id = val(init, T_I64)
        if we:
            w = g(we, T_STRUCT)
            if w is not None:
                fget(w[0], 10, T_STRING) and S(fget(w[0], 10, T_STRING)[0])
                a.ref.run_id = S((fget(w[0], 20, T_STRING) or (b"",))[0])
        return

