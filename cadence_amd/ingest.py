"""Host side of the on-device history decode (cdr/ingest.h, csrc/ingest.hip).

``encode_batch`` writes a decoded batch as persisted history blobs (the synthetic-input
encoder, csrc/thrift_enc.cpp) and builds the string seeds and domain map the decoder
needs; ``decode`` runs cdr_ingest_decode on the device (through the HIP runtime libcdr
itself uses) and returns host copies of its outputs.  ``to_batch`` turns a decode into
an ``engine.Batch`` that replays like any other.
"""
from __future__ import annotations

import ctypes as C
import dataclasses

import numpy as np

from . import abi, engine


def stand_in(h: int, strings=None) -> bytes:
    """The encoder's string for handle h (csrc/thrift_enc.cpp)."""
    if strings is not None and h < len(strings):
        s = strings[h]
        return s.encode() if isinstance(s, str) else bytes(s)
    return b"h%08x" % h


def _table(strings):
    bs = [s.encode() if isinstance(s, str) else bytes(s) for s in strings]
    off = np.zeros(len(bs) + 1, np.uint64)
    off[1:] = np.cumsum([len(b) for b in bs]) if bs else []
    return np.frombuffer(b"".join(bs) or b"\0", np.uint8).copy(), off


@dataclasses.dataclass
class Encoded:
    blob_bytes: np.ndarray   # uint8
    blob_off: np.ndarray     # uint64 [n_blobs + 1]
    entry_blob0: np.ndarray  # uint32 [n_entries + 1]
    seeds: list              # bytes per seed handle
    seed_of: dict            # original handle -> seed handle (wf_desc strings, domains)
    domain_map: list         # (name seed handle, ID seed handle)


def encode_batch(batch: engine.Batch, threads: int = 8) -> Encoded:
    """Blobs of every entry of `batch` plus the seeds a caller would hold: "" and
    "emptyUuid", the cdr_wf_desc strings, and the domain names -> IDs the events use
    (the domain cache)."""
    L = abi.lib()
    strings = batch.strings if batch.strings else None
    if strings is not None:
        sb, so = _table(strings)
        n_str = len(strings)
    else:
        sb, so, n_str = np.zeros(1, np.uint8), np.zeros(1, np.uint64), 0
    nbytes, nblobs = C.c_uint64(), C.c_uint32()
    b = batch.cstruct()
    rc = L.cdr_synth_encode_history(C.byref(b), sb.ctypes.data, so.ctypes.data, n_str, None, None, None,
                                    C.byref(nbytes), C.byref(nblobs), threads)
    assert rc == 0, rc
    blob_bytes = np.zeros(max(1, nbytes.value), np.uint8)
    blob_off = np.zeros(nblobs.value + 1, np.uint64)
    entry_blob0 = np.zeros(batch.n_wfs + 1, np.uint32)
    rc = L.cdr_synth_encode_history(C.byref(b), sb.ctypes.data, so.ctypes.data, n_str, blob_bytes.ctypes.data,
                                    blob_off.ctypes.data, entry_blob0.ctypes.data, C.byref(nbytes),
                                    C.byref(nblobs), threads)
    assert rc == 0, rc
    # seeds: what a caller holds before reading history
    seeds, index, seed_of = [b"", b"emptyUuid"], {b"": 0, b"emptyUuid": 1}, {0: 0, batch.empty_uuid: 1}

    def seed(s: bytes) -> int:
        if s not in index:
            index[s] = len(seeds)
            seeds.append(s)
        return index[s]
    for w in range(batch.n_wfs):
        d = batch.wfs[w]
        for h in (d.domain_id, d.workflow_id, d.run_id, d.request_id):
            if h and h != batch.empty_uuid:
                seed_of[h] = seed(stand_in(h, strings))
    dmap = {}
    ev = np.frombuffer(batch.events, dtype=np.uint8).reshape(len(batch.events), -1)
    types = ev[:, 32:36].copy().view(np.uint32)[:, 0] if len(batch.events) else np.zeros(0, np.uint32)
    ext_t = {abi.EV["StartChildWorkflowExecutionInitiated"], abi.EV["SignalExternalWorkflowExecutionInitiated"],
             abi.EV["RequestCancelExternalWorkflowExecutionInitiated"]}
    at_t = abi.EV["ActivityTaskScheduled"]
    for k in np.nonzero(np.isin(types, list(ext_t) + [abi.EV["WorkflowExecutionStarted"], at_t]))[0]:
        e = batch.events[int(k)]
        if e.type == at_t:  # an activity's target domain (refreshTasks, getTargetDomainID)
            x = e.a.at_sched
            if x.domain and not (x.flags & abi.AF_DOMAIN_MISSING):
                dmap[stand_in(x.domain, strings)] = stand_in(x.target_domain_id, strings)
        elif e.type == abi.EV["WorkflowExecutionStarted"]:
            s = e.a.started
            if (s.flags & abi.SF_HAS_PARENT_DOMAIN) and not (s.flags & abi.SF_PARENT_DOMAIN_MISSING):
                ident = stand_in(s.parent_domain_id, strings)
                dmap[b"dn:" + ident] = ident
        elif not (e.a.ext.flags & abi.XF_DOMAIN_MISSING) and e.a.ext.domain:
            dmap[stand_in(e.a.ext.domain, strings)] = stand_in(e.a.ext.target_domain_id, strings)
    domain_map = [(seed(n), seed(i)) for n, i in sorted(dmap.items())]
    return Encoded(blob_bytes, blob_off, entry_blob0, seeds, seed_of, domain_map)


@dataclasses.dataclass
class Decoded:
    events: C.Array
    kvs: C.Array
    rps: C.Array
    ev_off: np.ndarray
    blob_status: np.ndarray
    entry_status: np.ndarray
    strings: list
    n_bad_blobs: int
    raw: object = None  # the cdr_ingest_out (device pointers, valid until the context's next ingest)


def decode(eng: engine.Engine, enc: Encoded) -> Decoded:
    """cdr_ingest_decode on the device; host copies of every output."""
    hip = engine._hip()
    L = abi.lib()
    ptrs = []

    def up(a: np.ndarray):
        a = np.ascontiguousarray(a)
        p = C.c_void_p()
        assert hip.hipMalloc(C.byref(p), C.c_size_t(max(8, a.nbytes))) == 0
        ptrs.append(p)
        if a.nbytes:
            assert hip.hipMemcpy(p, a.ctypes.data, C.c_size_t(a.nbytes), 1) == 0
        return p.value

    def down(ptr, dtype, n):
        out = np.zeros(max(1, n), dtype)
        if n:
            assert hip.hipMemcpy(out.ctypes.data, C.c_void_p(ptr), C.c_size_t(out.nbytes), 2) == 0
        return out[:n]
    try:
        sb, so = _table(enc.seeds)
        dm = np.array(enc.domain_map, np.uint32).reshape(-1) if enc.domain_map else np.zeros(2, np.uint32)
        inp = abi.CdrIngestIn()
        inp.blob_bytes, inp.blob_off, inp.entry_blob0 = up(enc.blob_bytes), up(enc.blob_off), up(enc.entry_blob0)
        inp.seed_bytes, inp.seed_off, inp.domain_map = up(sb), up(so), up(dm)
        inp.n_blobs, inp.n_entries = len(enc.blob_off) - 1, len(enc.entry_blob0) - 1
        inp.n_seeds, inp.n_domains = len(enc.seeds), len(enc.domain_map)
        out = abi.CdrIngestOut()
        rc = L.cdr_ingest_decode(eng.ctx, C.byref(inp), C.byref(out), None)
        if rc:
            raise RuntimeError(f"cdr_ingest_decode rc={rc}")
        ne = inp.n_entries
        ev = down(out.events, np.uint8, out.n_events * C.sizeof(abi.CdrEvent))
        kv = down(out.kvs, np.uint8, out.n_kvs * C.sizeof(abi.CdrKV))
        rp = down(out.rps, np.uint8, out.n_rps * C.sizeof(abi.CdrResetPoint))
        events = (abi.CdrEvent * max(1, out.n_events)).from_buffer_copy(ev.tobytes() or bytes(C.sizeof(abi.CdrEvent)))
        kvs = (abi.CdrKV * max(1, out.n_kvs)).from_buffer_copy(kv.tobytes() or bytes(8))
        rps = (abi.CdrResetPoint * max(1, out.n_rps)).from_buffer_copy(rp.tobytes() or bytes(C.sizeof(abi.CdrResetPoint)))
        ev_off = down(out.ev_off, np.uint64, ne + 1)
        bst = down(out.blob_status, np.int32, inp.n_blobs)
        est = down(out.entry_status, np.int32, ne)
        ref = down(out.str_ref, np.uint64, out.n_strings)
        ln = down(out.str_len, np.uint32, out.n_strings)
        raw = enc.blob_bytes.tobytes()
        sraw = sb.tobytes()
        strings = []
        for h in range(out.n_strings):
            r, n = int(ref[h]), int(ln[h])
            if r >> 63:
                r &= (1 << 63) - 1
                strings.append(sraw[r:r + n])
            else:
                strings.append(raw[r:r + n])
        events = events if out.n_events else (abi.CdrEvent * 0)()
        kvs = kvs if out.n_kvs else (abi.CdrKV * 0)()
        rps = rps if out.n_rps else (abi.CdrResetPoint * 0)()
        return Decoded(events, kvs, rps, ev_off, bst, est, strings, out.n_bad_blobs, out)
    finally:
        for p in ptrs:
            hip.hipFree(p)


def to_batch(src: engine.Batch, enc: Encoded, dec: Decoded) -> engine.Batch:
    """The decoded events as a replayable batch: `src`'s entries (their cdr_wf_desc
    strings re-pointed at the seed handles), the decoded events / kvs / reset points,
    the decode's string table."""
    wfs = (abi.CdrWfDesc * src.n_wfs)()
    C.memmove(wfs, src.wfs, C.sizeof(wfs))
    for w in range(src.n_wfs):
        d = wfs[w]
        d.ev_off = int(dec.ev_off[w])
        d.ev_len = int(dec.ev_off[w + 1] - dec.ev_off[w])
        for f in ("domain_id", "workflow_id", "run_id", "request_id"):
            setattr(d, f, enc.seed_of.get(getattr(d, f), 0))
    strings = [s.decode("latin-1") for s in dec.strings]
    return engine.Batch(events=dec.events, wfs=wfs, kvs=dec.kvs, rps=dec.rps, cluster=src.cluster,
                        now_ns=src.now_ns, uuid_seed=src.uuid_seed, empty_uuid=1, strings=strings)


def replay_on_device(eng: engine.Engine, src: engine.Batch, enc: Encoded, dec: Decoded,
                     plan_mode: int = abi.PLAN_WAVE) -> engine.Outputs:
    """cdr_ingest_plan (device caps + host slice plan + device pack) on the decode still
    resident in the context, then cdr_replay_sliced_async; host copies of the outputs
    (an engine.Outputs whose plan is the device-computed capacities)."""
    hip = engine._hip()
    L = abi.lib()
    meta = to_batch(src, enc, dec)
    mb = meta.cstruct()
    n = src.n_wfs
    caps = (abi.CdrWfCaps * max(1, n))()
    tot = abi.CdrTotals()
    db = abi.CdrDevBatch()
    rc = L.cdr_ingest_plan(eng.ctx, C.byref(dec.raw), C.byref(mb), plan_mode, C.byref(db), caps, C.byref(tot), None)
    if rc:
        raise RuntimeError(f"cdr_ingest_plan rc={rc}")
    pl = engine.Plan(caps, tot)
    out = engine.Outputs(meta, pl)
    ptrs = []

    def dz(nbytes):
        p = C.c_void_p()
        assert hip.hipMalloc(C.byref(p), C.c_size_t(max(8, nbytes))) == 0
        ptrs.append(p)
        hip.hipMemset(p, 0, C.c_size_t(max(8, nbytes)))
        return p.value
    try:
        dev = abi.CdrOut()
        host = out.cstruct()
        sizes = {"result": C.sizeof(out.result), "exec": C.sizeof(out.exec), "repl": C.sizeof(out.repl),
                 "last_decision": C.sizeof(out.last_decision)}
        for t in engine.TABLES:
            sizes[t] = C.sizeof(out.tables[t])
        for k, nb in sizes.items():
            setattr(dev, k, dz(nb))
        rc = L.cdr_replay_sliced_async(eng.ctx, C.byref(db), C.byref(dev), None)
        if rc:
            raise RuntimeError(f"cdr_replay_sliced_async rc={rc}")
        for k, nb in sizes.items():
            assert hip.hipMemcpy(C.c_void_p(getattr(host, k)), C.c_void_p(getattr(dev, k)), C.c_size_t(nb), 2) == 0
        return out
    finally:
        for p in ptrs:
            hip.hipFree(p)
