// thrift_enc.cpp — synthetic persisted histories: a decoded batch (cdr_event records)
// written back as the reference stores it, one thriftrw blob per applyEvents call
// (preambleVersion0 + shared.History{10: list<HistoryEvent>}; common/codec/
// version0Thriftrw.go:45-60 Encode, serializer.go:198-213), so that the on-device
// decoder (ingest.hip) has realistic input at any scale.  Handles become strings
// through the caller's table (handle h < n_str) or the stand-in "h%08x".
//
// Fields follow the IDL (idl/github.com/uber/cadence/shared.thrift); for every value
// the record form keeps, the encoder writes the wire field the decoder reads, in
// ascending field-id order as thriftrw does, and omits optional strings whose handle
// is 0.  Structure-valued handles are written as: Memo{fields: {"m": s(h)}},
// nonRetriableErrorReasons [s(h)], a parent domain named "dn:" + s(parent domain ID).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "cdr/cdr.h"
#include "cdr/synth.h"

namespace {

enum : uint8_t { T_BOOL = 2, T_DOUBLE = 4, T_I32 = 8, T_I64 = 10, T_STRING = 11, T_STRUCT = 12, T_MAP = 13, T_LIST = 15 };

struct W {
  std::string* o;
  const cdr_batch* b;
  const uint8_t* sb;
  const uint64_t* so;
  uint32_t ns;

  void u8(uint32_t v) { o->push_back((char)(uint8_t)v); }
  void be16(uint32_t v) {
    u8(v >> 8);
    u8(v);
  }
  void be32(uint32_t v) {
    for (int s = 24; s >= 0; s -= 8) u8(v >> s);
  }
  void be64(uint64_t v) {
    for (int s = 56; s >= 0; s -= 8) u8((uint32_t)(v >> s));
  }
  void hdr(uint8_t t, uint32_t id) {
    u8(t);
    be16(id);
  }
  void stop() { u8(0); }
  void i64(uint32_t id, int64_t v) {
    hdr(T_I64, id);
    be64((uint64_t)v);
  }
  void i32(uint32_t id, int32_t v) {
    hdr(T_I32, id);
    be32((uint32_t)v);
  }
  void boolean(uint32_t id, bool v) {
    hdr(T_BOOL, id);
    u8(v ? 1 : 0);
  }
  void dbl(uint32_t id, double v) {
    uint64_t u;
    std::memcpy(&u, &v, 8);
    hdr(T_DOUBLE, id);
    be64(u);
  }
  std::string s(uint32_t h) const {
    if (h < ns) return std::string((const char*)sb + so[h], (size_t)(so[h + 1] - so[h]));
    char buf[16];
    std::snprintf(buf, sizeof buf, "h%08x", h);
    return buf;
  }
  void bytes(const std::string& v) {
    be32((uint32_t)v.size());
    o->append(v);
  }
  void str(uint32_t id, uint32_t h) {  // optional string: omitted when its handle is 0
    if (!h) return;
    hdr(T_STRING, id);
    bytes(s(h));
  }
  void str_v(uint32_t id, const std::string& v) {
    hdr(T_STRING, id);
    bytes(v);
  }
  void named(uint32_t id, uint32_t h) {  // WorkflowType / TaskList{10: name}
    if (!h) return;
    hdr(T_STRUCT, id);
    str(10, h);
    stop();
  }
  void execution(uint32_t id, uint32_t wid, uint32_t rid) {
    if (!wid && !rid) return;
    hdr(T_STRUCT, id);
    str(10, wid);
    str(20, rid);
    stop();
  }
  void kv_map(uint32_t id, uint32_t off, uint32_t len) {  // SearchAttributes{10: map<string, binary>}
    hdr(T_STRUCT, id);
    hdr(T_MAP, 10);
    u8(T_STRING);
    u8(T_STRING);
    be32(len);
    for (uint32_t q = 0; q < len; q++) {
      const cdr_kv kv = b->kvs[off + q];
      bytes(kv.key ? s(kv.key) : std::string());
      bytes(kv.value ? s(kv.value) : std::string());
    }
    stop();
  }
  template <class A>
  void retry(uint32_t id, const A& a) {
    hdr(T_STRUCT, id);
    i32(10, a.retry_initial_s);
    dbl(20, a.backoff_coefficient);
    i32(30, a.retry_max_interval_s);
    i32(40, a.retry_max_attempts);
    if (a.nonretriable) {
      hdr(T_LIST, 50);
      u8(T_STRING);
      be32(1);
      bytes(s(a.nonretriable));
    }
    i32(60, a.retry_expiration_s);
    stop();
  }

  void started(const cdr_attr_wf_started& a) {
    hdr(T_STRUCT, 40);
    named(10, a.workflow_type);
    if (a.flags & CDR_SF_HAS_PARENT_DOMAIN) str_v(12, "dn:" + s(a.parent_domain_id));
    if (a.flags & CDR_SF_HAS_PARENT_EXEC) {
      hdr(T_STRUCT, 14);
      str(10, a.parent_workflow_id);
      str(20, a.parent_run_id);
      stop();
    }
    if (a.flags & CDR_SF_HAS_PARENT_INITIATED) i64(16, a.parent_initiated_id);
    named(20, a.task_list);
    i32(40, a.exec_timeout_s);
    i32(50, a.task_timeout_s);
    str(54, a.continued_run_id);
    if (a.flags & CDR_SF_HAS_INITIATOR)
      i32(55, (a.flags & CDR_SF_CRON_INITIATOR) ? 2 : (a.flags & CDR_SF_RETRY_INITIATOR) ? 1 : 0);
    if (a.flags & CDR_SF_HAS_RETRY) retry(70, a);
    i32(80, a.attempt);
    if (a.expiration_ts) i64(90, a.expiration_ts);
    str(100, a.cron_schedule);
    i32(110, a.first_decision_backoff_s);
    if (a.flags & CDR_SF_HAS_MEMO) {
      hdr(T_STRUCT, 120);
      hdr(T_MAP, 10);
      u8(T_STRING);
      u8(T_STRING);
      be32(1);
      bytes("m");
      bytes(s(a.memo));
      stop();
    }
    if (a.flags & CDR_SF_HAS_SEARCH_ATTR) kv_map(121, a.search_attr_off, a.search_attr_len);
    if (a.flags & CDR_SF_HAS_RESET_POINTS) {
      hdr(T_STRUCT, 130);
      hdr(T_LIST, 10);
      u8(T_STRUCT);
      be32(a.reset_points_len);
      for (uint32_t q = 0; q < a.reset_points_len; q++) {
        const cdr_reset_point& p = b->rps[a.reset_points_off + q];
        if (p.flags & CDR_RP_HAS_CHECKSUM) str_v(10, p.binary_checksum ? s(p.binary_checksum) : std::string());
        if (p.flags & CDR_RP_HAS_RUN_ID) str_v(20, p.run_id ? s(p.run_id) : std::string());
        if (p.flags & CDR_RP_HAS_FIRST_DC_ID) i64(30, p.first_decision_completed_id);
        if (p.flags & CDR_RP_HAS_CREATED) i64(40, p.created_time_nano);
        if (p.flags & CDR_RP_HAS_EXPIRING) i64(50, p.expiring_time_nano);
        if (p.flags & CDR_RP_HAS_RESETTABLE) boolean(60, (p.flags & CDR_RP_RESETTABLE) != 0);
        stop();
      }
      stop();
    }
    stop();
  }

  // decision / activity attribute structs: field ids of the kept values
  void dt_at(uint32_t attr, const cdr_event& e, uint32_t sched, uint32_t started, uint32_t req, uint32_t aid,
             uint32_t to, uint32_t att, uint32_t cks) {
    const bool act = attr >= 140;
    hdr(T_STRUCT, attr);
    struct F {
      uint32_t id;
      int kind;
    } f[7] = {{sched, 0}, {started, 1}, {req, 2}, {aid, 3}, {to, 4}, {att, 5}, {cks, 6}};
    // ascending field ids
    for (int i = 0; i < 7; i++)
      for (int j = i + 1; j < 7; j++)
        if (f[j].id < f[i].id) std::swap(f[i], f[j]);
    for (const F& x : f) {
      if (!x.id) continue;
      switch (x.kind) {
        case 0: i64(x.id, act ? e.a.at.scheduled_event_id : e.a.dt.scheduled_event_id); break;
        case 1: i64(x.id, act ? e.a.at.started_event_id : e.a.dt.started_event_id); break;
        case 2: str(x.id, act ? e.a.at.request_id : e.a.dt.request_id); break;
        case 3: str(x.id, e.a.at.activity_id); break;
        case 4: i32(x.id, act ? e.a.at.timeout_type : e.a.dt.timeout_type); break;
        case 5: i32(x.id, e.a.at.attempt); break;
        case 6: str(x.id, e.a.dt.binary_checksum); break;
      }
    }
    stop();
  }
  void ref(uint32_t attr, const cdr_event& e, uint32_t init, uint32_t we) {
    hdr(T_STRUCT, attr);
    if (we && we < init) execution(we, 0, e.a.ref.run_id);
    i64(init, e.a.ref.initiated_event_id);
    if (we && we > init) execution(we, 0, e.a.ref.run_id);
    stop();
  }

  void event(const cdr_event& e) {
    i64(10, e.event_id);
    i64(20, e.timestamp);
    i32(30, (int32_t)e.type);
    i64(35, e.version);
    i64(36, e.task_id);
    switch (e.type) {
      case CDR_EV_WF_STARTED: started(e.a.started); break;
      case CDR_EV_DT_SCHEDULED:
        hdr(T_STRUCT, 80);
        named(10, e.a.dt_sched.task_list);
        i32(20, e.a.dt_sched.start_to_close_s);
        i64(30, e.a.dt_sched.attempt);
        stop();
        break;
      case CDR_EV_DT_STARTED: dt_at(90, e, 10, 0, 30, 0, 0, 0, 0); break;
      case CDR_EV_DT_COMPLETED: dt_at(100, e, 20, 30, 0, 0, 0, 0, 50); break;
      case CDR_EV_DT_TIMED_OUT: dt_at(110, e, 10, 20, 0, 0, 30, 0, 0); break;
      case CDR_EV_DT_FAILED: dt_at(120, e, 10, 20, 0, 0, 0, 0, 0); break;
      case CDR_EV_AT_SCHEDULED: {
        const cdr_attr_at_scheduled& a = e.a.at_sched;
        hdr(T_STRUCT, 130);
        str(10, a.activity_id);
        str(25, a.domain);
        named(30, a.task_list);
        i32(45, a.s2c_s);
        i32(50, a.s2s_s);
        i32(55, a.stc_s);
        i32(60, a.hb_s);
        if (a.flags & CDR_AF_HAS_RETRY) retry(110, a);
        stop();
        break;
      }
      case CDR_EV_AT_STARTED: dt_at(140, e, 10, 0, 30, 0, 0, 40, 0); break;
      case CDR_EV_AT_COMPLETED: dt_at(150, e, 20, 30, 0, 0, 0, 0, 0); break;
      case CDR_EV_AT_FAILED: dt_at(160, e, 30, 40, 0, 0, 0, 0, 0); break;
      case CDR_EV_AT_TIMED_OUT: dt_at(170, e, 10, 20, 0, 0, 30, 0, 0); break;
      case CDR_EV_AT_CANCEL_REQUESTED: dt_at(200, e, 0, 0, 0, 10, 0, 0, 0); break;
      case CDR_EV_AT_REQ_CANCEL_FAILED: dt_at(210, e, 0, 0, 0, 10, 0, 0, 0); break;
      case CDR_EV_AT_CANCELED: dt_at(220, e, 30, 40, 0, 0, 0, 0, 0); break;
      case CDR_EV_TIMER_STARTED:
        hdr(T_STRUCT, 180);
        str(10, e.a.timer.timer_id);
        i64(20, e.a.timer.start_to_fire_s);
        stop();
        break;
      case CDR_EV_TIMER_FIRED:
      case CDR_EV_TIMER_CANCELED:
        hdr(T_STRUCT, e.type == CDR_EV_TIMER_FIRED ? 190 : 230);
        str(10, e.a.timer.timer_id);
        i64(20, e.a.timer.started_event_id);
        stop();
        break;
      case CDR_EV_CANCEL_TIMER_FAILED:
        hdr(T_STRUCT, 240);
        str(10, e.a.timer.timer_id);
        stop();
        break;
      case CDR_EV_CHILD_INITIATED: {
        const cdr_attr_external& x = e.a.ext;
        hdr(T_STRUCT, 340);
        str(10, x.domain);
        str(20, x.workflow_id);
        named(30, x.workflow_type);
        str(50, x.input);
        i32(81, x.parent_close_policy);
        str(90, x.control);
        stop();
        break;
      }
      case CDR_EV_SE_INITIATED: {
        const cdr_attr_external& x = e.a.ext;
        hdr(T_STRUCT, 420);
        str(20, x.domain);
        execution(30, x.workflow_id, x.run_id);
        str(40, x.signal_name);
        str(50, x.input);
        str(60, x.control);
        boolean(70, (x.flags & CDR_XF_CHILD_ONLY) != 0);
        stop();
        break;
      }
      case CDR_EV_RCE_INITIATED: {
        const cdr_attr_external& x = e.a.ext;
        hdr(T_STRUCT, 300);
        str(20, x.domain);
        execution(30, x.workflow_id, x.run_id);
        str(40, x.control);
        boolean(50, (x.flags & CDR_XF_CHILD_ONLY) != 0);
        stop();
        break;
      }
      case CDR_EV_RCE_FAILED: ref(310, e, 50, 40); break;
      case CDR_EV_EXT_CANCEL_REQUESTED: ref(320, e, 10, 30); break;
      case CDR_EV_CHILD_START_FAILED: ref(350, e, 60, 0); break;
      case CDR_EV_CHILD_STARTED: ref(360, e, 20, 30); break;
      case CDR_EV_CHILD_COMPLETED: ref(370, e, 50, 30); break;
      case CDR_EV_CHILD_FAILED: ref(380, e, 60, 40); break;
      case CDR_EV_CHILD_CANCELED: ref(390, e, 50, 30); break;
      case CDR_EV_CHILD_TIMED_OUT: ref(400, e, 50, 30); break;
      case CDR_EV_CHILD_TERMINATED: ref(410, e, 40, 20); break;
      case CDR_EV_SE_FAILED: ref(430, e, 50, 40); break;
      case CDR_EV_EXT_SIGNALED: ref(440, e, 10, 30); break;
      case CDR_EV_WF_CONTINUED_AS_NEW:
        hdr(T_STRUCT, 330);
        str(10, e.a.can.new_execution_run_id);
        stop();
        break;
      case CDR_EV_UPSERT_SA:
        hdr(T_STRUCT, 450);
        kv_map(20, e.a.upsert.search_attr_off, e.a.upsert.search_attr_len);
        stop();
        break;
      default:
        break;  // attributes the replay does not read: none written
    }
    stop();
  }

  // blobs of entry w: one per call
  void entry(uint32_t w, std::vector<uint64_t>* blob_ends) {
    const cdr_wf_desc& d = b->wfs[w];
    const cdr_event* ev = b->events + d.ev_off;
    uint64_t k = 0;
    while (k < d.ev_len) {
      uint64_t e = k + 1;
      while (e < d.ev_len && !(ev[e].flags & CDR_EVF_BATCH_FIRST)) e++;
      u8(CDR_THRIFT_PREAMBLE_V0_ENC);
      hdr(T_LIST, 10);
      u8(T_STRUCT);
      be32((uint32_t)(e - k));
      for (uint64_t i = k; i < e; i++) event(ev[i]);
      stop();
      blob_ends->push_back(o->size());
      k = e;
    }
  }
  static constexpr uint32_t CDR_THRIFT_PREAMBLE_V0_ENC = 0x59u;
};

}  // namespace

extern "C" int cdr_synth_encode_history(const cdr_batch* b, const uint8_t* str_bytes, const uint64_t* str_off,
                                        uint32_t n_str, uint8_t* blob_bytes, uint64_t* blob_off,
                                        uint32_t* entry_blob0, uint64_t* n_bytes, uint32_t* n_blobs, int threads) {
  if (!b || !n_bytes || !n_blobs || (n_str && (!str_bytes || !str_off))) return CDR_API_EINVAL;
  const uint32_t n = b->n_wfs;
  unsigned hw = std::thread::hardware_concurrency();
  const uint32_t nt = (uint32_t)std::max(1, std::min<int>(threads > 0 ? threads : (int)(hw ? hw : 4), 64));
  // each thread encodes a contiguous range of entries into its own buffer
  std::vector<std::string> buf(nt);
  std::vector<std::vector<uint64_t>> ends(nt);
  std::vector<std::vector<uint32_t>> eblobs(nt);
  std::vector<std::thread> pool;
  for (uint32_t t = 0; t < nt; t++)
    pool.emplace_back([&, t] {
      const uint32_t w0 = (uint32_t)((uint64_t)n * t / nt), w1 = (uint32_t)((uint64_t)n * (t + 1) / nt);
      W x{&buf[t], b, str_bytes, str_off, n_str};
      for (uint32_t w = w0; w < w1; w++) {
        eblobs[t].push_back((uint32_t)ends[t].size());
        x.entry(w, &ends[t]);
      }
    });
  for (auto& th : pool) th.join();
  uint64_t tot = 0, nb = 0;
  for (uint32_t t = 0; t < nt; t++) {
    tot += buf[t].size();
    nb += ends[t].size();
  }
  if (nb >= (1ull << 32)) return CDR_API_EINVAL;
  *n_bytes = tot;
  *n_blobs = (uint32_t)nb;
  if (!blob_bytes) return CDR_API_OK;
  if (!blob_off || !entry_blob0) return CDR_API_EINVAL;
  uint64_t pos = 0, bi = 0;
  uint32_t w = 0;
  for (uint32_t t = 0; t < nt; t++) {
    std::memcpy(blob_bytes + pos, buf[t].data(), buf[t].size());
    for (uint32_t q : eblobs[t]) entry_blob0[w++] = (uint32_t)(bi + q);
    uint64_t prev = 0;
    for (uint64_t e : ends[t]) {
      blob_off[bi++] = pos + prev;
      prev = e;
    }
    pos += buf[t].size();
  }
  blob_off[bi] = pos;
  entry_blob0[w] = (uint32_t)bi;
  return CDR_API_OK;
}
