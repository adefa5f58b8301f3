// encode_var.hip — the variable-size persisted-format row blobs: the SQL
// persistence's thriftrw binary-protocol blobs of ActivityInfo, ChildExecutionInfo and
// SignalInfo rows (common/persistence/sql/workflowStateMaps.go:48-83,371-385,632-639) and
// of the execution row (buildExecutionRow, sqlExecutionManagerUtil.go:1197-1308), IDL
// sqlblobs.thrift:73-193.  Their sizes depend on the strings they carry, so encoding is
// a size pass, an exclusive scan of the row sizes (hipcub) and a write pass that emits
// each row at its offset.
//
// One thread per entry writes its rows one after another (the rows of an entry are a
// handful; entries are read coalesced across the wavefront).  A row's bytes are emitted
// in protocol order through `Out`: aligned 4-byte words wholly inside the row are
// assembled in a register and stored once, the (at most 3 + 3) bytes at the row's ends,
// whose words a neighbouring row shares, are stored bytewise.  HBM-bound byte work.
//
// Protocol: go.uber.org/thriftrw protocol.Binary (blob.go:61-73), restated and pinned in
// oracle/thrift_binary.py; nested blobs (reset points, version histories, branch token)
// carry the codec's 0x59 preamble (common/codec/version0Thriftrw.go:45-64).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>

#include "cdr/cdr.h"
#include "ctx.h"

namespace {

constexpr uint32_t T_BOOL = 2, T_DOUBLE = 4, T_I32 = 8, T_I64 = 10, T_STRING = 11, T_STRUCT = 12, T_MAP = 13,
                   T_LIST = 15;
constexpr int64_t ZERO_TIME_NANOS = -6795364578871345152ll;  // time.Time{}.UnixNano()

struct Strs {
  const uint8_t* b;
  const uint64_t* off;
  uint32_t n;
  __device__ bool ok(uint32_t h) const { return h < n; }
  __device__ uint64_t len(uint32_t h) const { return h < n ? off[h + 1] - off[h] : 0; }
  __device__ const uint8_t* at(uint32_t h) const { return h < n ? b + off[h] : b; }
};

__device__ __forceinline__ uint32_t rd_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// the byte sink: counting (base == nullptr) or writing row bytes [start, end)
struct Out {
  uint8_t* base;
  uint64_t start, end, pos;
  uint32_t acc;
  int32_t err;
  __device__ void b(uint32_t v) {
    if (base) {
      const uint64_t a = pos, w = a & ~3ull;
      if (w >= start && w + 4 <= end) {
        acc |= (v & 0xFFu) << (8 * (uint32_t)(a & 3));
        if ((a & 3) == 3) {
          *(uint32_t*)(base + w) = acc;
          acc = 0;
        }
      } else if (a < end) {
        base[a] = (uint8_t)v;
      }
    }
    pos++;
  }
  __device__ void be16(uint32_t v) { b(v >> 8), b(v); }
  __device__ void be32(uint32_t v) { b(v >> 24), b(v >> 16), b(v >> 8), b(v); }
  __device__ void be64(uint64_t v) { be32((uint32_t)(v >> 32)), be32((uint32_t)v); }
  __device__ void fld(uint32_t t, uint32_t id) { b(t), be16(id); }
  __device__ void i64f(uint32_t id, int64_t v) { fld(T_I64, id), be64((uint64_t)v); }
  __device__ void i32f(uint32_t id, int32_t v) { fld(T_I32, id), be32((uint32_t)v); }
  __device__ void boolf(uint32_t id, bool v) { fld(T_BOOL, id), b(v ? 1u : 0u); }
  __device__ void dblf(uint32_t id, double v) { fld(T_DOUBLE, id), be64((uint64_t)__double_as_longlong(v)); }
  __device__ void raw(const uint8_t* p, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) b(p[i]);
  }
  __device__ void lit(const char* s, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) b((uint8_t)s[i]);
  }
  // a string / binary field holding handle h's bytes
  __device__ void strf(const Strs& S, uint32_t id, uint32_t h) {
    if (!S.ok(h)) err = err ? err : CDR_BLOB_E_HANDLE;
    const uint64_t n = S.len(h);
    fld(T_STRING, id), be32((uint32_t)n);
    if (n) raw(S.at(h), n);
  }
  __device__ void emptyf(uint32_t id) { fld(T_STRING, id), be32(0); }
  // RFC 4122 text of (hi, lo): 8-4-4-4-12 lowercase hex (oracle/thrift_binary.py uuid_text)
  __device__ void uuid_text(uint64_t lo, uint64_t hi) {
    for (uint32_t k = 0; k < 32; k++) {
      if (k == 8 || k == 12 || k == 16 || k == 20) b('-');
      const uint64_t w = k < 16 ? hi : lo;
      const uint32_t nib = (uint32_t)(w >> (4 * (15 - (k & 15)))) & 0xFu;
      b(nib < 10 ? '0' + nib : 'a' + nib - 10);
    }
  }
  __device__ void uuidf(uint32_t id, uint64_t lo, uint64_t hi) { fld(T_STRING, id), be32(36), uuid_text(lo, hi); }
};

// google/uuid.Parse of the canonical 36-char and bare 32-hex forms (sqldb.MustParseUUID,
// common/persistence/sql/storage/sqldb/uuid.go:39-45): false where Go would panic
__device__ bool parse_uuid(const Strs& S, uint32_t h, uint8_t* u) {
  const uint64_t n = S.len(h);
  if (!S.ok(h) || (n != 36 && n != 32)) return false;
  const uint8_t* s = S.at(h);
  if (n == 36 && (s[8] != '-' || s[13] != '-' || s[18] != '-' || s[23] != '-')) return false;
  uint32_t k = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (n == 36 && (i == 8 || i == 13 || i == 18 || i == 23)) continue;
    const uint32_t c = s[i];
    const int v = c >= '0' && c <= '9' ? (int)(c - '0') : c >= 'a' && c <= 'f' ? (int)(c - 'a' + 10)
                  : c >= 'A' && c <= 'F' ? (int)(c - 'A' + 10) : -1;
    if (v < 0) return false;
    if (k & 1) u[k >> 1] |= (uint8_t)v;
    else u[k >> 1] = (uint8_t)(v << 4);
    k++;
  }
  return k == 32;
}
// a binary field of MustParseUUID(string of h): absent for "", CDR_BLOB_E_UUID where Go panics
__device__ void uuid_bin_f(Out& o, const Strs& S, uint32_t id, uint32_t h) {
  if (S.len(h) == 0 && S.ok(h)) return;
  uint8_t u[16];
  if (!parse_uuid(S, h, u)) {
    o.err = o.err ? o.err : CDR_BLOB_E_UUID;
    return;
  }
  o.fld(T_STRING, id), o.be32(16);
  for (int i = 0; i < 16; i++) o.b(u[i]);
}

// ---------------------------------------------------------------- pending-table rows
// ActivityInfo (workflowStateMaps.go:48-83): ScheduledEvent / StartedEvent nil on replay
// (mutableStateBuilder.go:1982-2028,2083-2098), so fields 14 / 22 are absent and their
// encodings ""; StartedIdentity, LastFailureReason, LastWorkerIdentity ""; LastFailureDetails nil
__device__ void activity_row(Out& o, const Strs& S, const cdr_activity_info& a) {
  const bool retry = (a.flags & CDR_AI_HAS_RETRY) != 0;
  o.i64f(10, a.version);
  o.i64f(12, a.scheduled_event_batch_id);
  o.emptyf(16);
  o.i64f(18, a.scheduled_time);
  o.i64f(20, a.started_id);
  o.emptyf(24);
  o.i64f(26, (a.flags & CDR_AI_STARTED_TIME_SET) ? a.started_time : ZERO_TIME_NANOS);
  o.strf(S, 28, a.activity_id);
  o.strf(S, 30, a.request_id);
  o.i32f(32, a.s2s);
  o.i32f(34, a.s2c);
  o.i32f(36, a.stc);
  o.i32f(38, a.hb);
  o.boolf(40, (a.flags & CDR_AI_CANCEL_REQUESTED) != 0);
  o.i64f(42, a.cancel_request_id);
  o.i32f(44, a.timer_task_status);
  o.i32f(46, a.attempt);
  o.strf(S, 48, a.task_list);
  o.emptyf(50);
  o.boolf(52, retry);
  o.i32f(54, a.initial_interval);
  o.i32f(56, a.maximum_interval);
  o.i32f(58, a.maximum_attempts);
  o.i64f(60, a.expiration_time);
  o.dblf(62, a.backoff_coefficient);
  if (a.nonretriable) {  // the handle holds the list<string> wire body
    if (!S.ok(a.nonretriable)) o.err = o.err ? o.err : CDR_BLOB_E_HANDLE;
    o.fld(T_LIST, 64);
    o.raw(S.at(a.nonretriable), S.len(a.nonretriable));
  }
  o.emptyf(66);
  o.emptyf(68);
  o.b(0);
}

// ChildExecutionInfo (workflowStateMaps.go:371-385)
__device__ void child_row(Out& o, const Strs& S, const cdr_child_info& c) {
  o.i64f(10, c.version);
  o.i64f(12, c.initiated_event_batch_id);
  o.i64f(14, c.started_id);
  o.emptyf(18);
  o.strf(S, 20, c.started_workflow_id);
  uuid_bin_f(o, S, 22, c.started_run_id);
  o.emptyf(26);
  o.uuidf(28, c.create_request_lo, c.create_request_hi);
  o.strf(S, 30, c.domain_name);
  o.strf(S, 32, c.workflow_type);
  o.i32f(35, c.parent_close_policy);
  o.b(0);
}

// SignalInfo (workflowStateMaps.go:632-639): Input / Control nil -> absent
__device__ void signal_row(Out& o, const Strs& S, const cdr_signal_info& g) {
  o.i64f(10, g.version);
  o.i64f(11, g.initiated_event_batch_id);
  o.uuidf(12, g.signal_request_lo, g.signal_request_hi);
  o.strf(S, 14, g.signal_name);
  if (g.input) o.strf(S, 16, g.input);
  if (g.control) o.strf(S, 18, g.control);
  o.b(0);
}

// ---------------------------------------------------------------- the execution row
// NewHistoryBranchToken's token (dataInterfaces.go:2428-2440): 0x59 + HistoryBranch{TreeID,
// BranchID, Ancestors: []}
__device__ void branch_token(Out& o, const Strs& S, const cdr_exec_info& x) {
  o.b(0x59);
  o.strf(S, 10, x.branch_tree_id);
  o.uuidf(20, x.branch_id_lo, x.branch_id_hi);
  o.fld(T_LIST, 30), o.b(T_STRUCT), o.be32(0);
  o.b(0);
}
// SerializeResetPoints (serializer.go:120-125): 0x59 + ResetPoints{Points} (nil -> {})
__device__ void reset_points(Out& o, const Strs& S, const cdr_reset_point* rp, uint32_t n, bool present) {
  o.b(0x59);
  if (present) {
    o.fld(T_LIST, 10), o.b(T_STRUCT), o.be32(n);
    for (uint32_t q = 0; q < n; q++) {
      const cdr_reset_point p = rp[q];
      if (p.flags & CDR_RP_HAS_CHECKSUM) o.strf(S, 10, p.binary_checksum);
      if (p.flags & CDR_RP_HAS_RUN_ID) o.strf(S, 20, p.run_id);
      if (p.flags & CDR_RP_HAS_FIRST_DC_ID) o.i64f(30, p.first_decision_completed_id);
      if (p.flags & CDR_RP_HAS_CREATED) o.i64f(40, p.created_time_nano);
      if (p.flags & CDR_RP_HAS_EXPIRING) o.i64f(50, p.expiring_time_nano);
      if (p.flags & CDR_RP_HAS_RESETTABLE) o.boolf(60, (p.flags & CDR_RP_RESETTABLE) != 0);
      o.b(0);
    }
  }
  o.b(0);
}
// SerializeVersionHistories (serializer.go:161-166) of the current branch:
// 0x59 + VersionHistories{0, [VersionHistory{BranchToken, Items}]} (versionHistory.go:135-149,411-423)
__device__ void version_histories(Out& o, const Strs& S, const cdr_exec_info& x, const cdr_vh_item* vh, uint32_t n,
                                  uint64_t token_len) {
  o.b(0x59);
  o.i32f(10, 0);
  o.fld(T_LIST, 20), o.b(T_STRUCT), o.be32(1);
  o.fld(T_STRING, 10), o.be32((uint32_t)token_len);
  if (token_len) branch_token(o, S, x);
  o.fld(T_LIST, 20), o.b(T_STRUCT), o.be32(n);
  for (uint32_t q = 0; q < n; q++) {
    const cdr_vh_item it = vh[q];
    o.i64f(10, it.event_id);
    o.i64f(20, it.version);
    o.b(0);
  }
  o.b(0);
  o.b(0);
}
// byte range [m0, m1) of Memo field 10 (map<string, binary>) inside the Memo struct body
// handle h holds; false when absent (err set when the body is not a Memo struct)
__device__ bool memo_fields(const Strs& S, uint32_t h, uint64_t& m0, uint64_t& m1, int32_t& err) {
  const uint64_t n = S.len(h);
  const uint8_t* s = S.ok(h) ? S.at(h) : nullptr;
  uint64_t p = 0;
  while (s && p < n) {
    const uint32_t t = s[p];
    if (t == 0) return false;
    if (p + 3 > n) break;
    const uint32_t id = ((uint32_t)s[p + 1] << 8) | s[p + 2];
    p += 3;
    if (t == T_MAP && id == 10) {
      if (p + 6 > n) break;
      const uint32_t cnt = rd_be32(s + p + 2);
      uint64_t q = p + 6;
      for (uint64_t e = 0; e < 2ull * cnt && q + 4 <= n; e++) q += 4 + rd_be32(s + q);
      if (q > n) break;
      m0 = p, m1 = q;
      return true;
    }
    if (t != T_STRING || p + 4 > n) break;
    p += 4 + rd_be32(s + p);
  }
  err = err ? err : CDR_BLOB_E_MEMO;
  return false;
}

// buildExecutionRow (sqlExecutionManagerUtil.go:1197-1308) of a replayed ExecutionInfo
__device__ void exec_row(Out& o, const Strs& S, const cdr_exec_info& x, const cdr_exec_persist& ps, uint32_t builder,
                         const cdr_repl_state* rs, const cdr_vh_item* vh, uint32_t n_vh, const cdr_reset_point* rp,
                         uint32_t n_rp, const cdr_kv* sa, uint32_t n_sa, const uint32_t* cluster_names,
                         uint32_t n_clusters) {
  if (!S.ok(x.parent_domain_id)) o.err = o.err ? o.err : CDR_BLOB_E_HANDLE;
  if (S.len(x.parent_domain_id) != 0) {  // ParentDomainID != ""
    uint8_t u[16];
    if (!parse_uuid(S, x.parent_domain_id, u)) {
      o.err = o.err ? o.err : CDR_BLOB_E_UUID;
    } else {
      o.fld(T_STRING, 10), o.be32(16);
      for (int i = 0; i < 16; i++) o.b(u[i]);
    }
    o.strf(S, 12, x.parent_workflow_id);
    uuid_bin_f(o, S, 14, x.parent_run_id);
    o.i64f(16, x.initiated_id);
  }
  o.i64f(18, x.completion_event_batch_id);
  o.strf(S, 24, x.task_list);
  o.strf(S, 26, x.workflow_type);
  o.i32f(28, x.workflow_timeout);
  o.i32f(30, x.decision_timeout_value);
  if (ps.execution_context) o.strf(S, 32, ps.execution_context);
  o.i32f(34, x.state);
  o.i32f(36, x.close_status);
  o.i64f(38, ps.start_version);
  o.i64f(40, ps.current_version);
  if (builder == CDR_BUILDER_2DC) {  // replicationState != nil
    o.i64f(44, rs->last_write_event_id);
    uint32_t cnt = 0;
    for (uint32_t i = 0; i < n_clusters && i < CDR_MAX_CLUSTERS; i++) cnt += (rs->lri_mask >> i) & 1u;
    o.fld(T_MAP, 46), o.b(T_STRING), o.b(T_STRUCT), o.be32(cnt);
    for (uint32_t i = 0; i < n_clusters && i < CDR_MAX_CLUSTERS; i++) {
      if (!((rs->lri_mask >> i) & 1u)) continue;
      const uint32_t h = cluster_names[i];
      if (!S.ok(h)) o.err = o.err ? o.err : CDR_BLOB_E_HANDLE;
      o.be32((uint32_t)S.len(h));
      if (S.len(h)) o.raw(S.at(h), S.len(h));
      o.i64f(10, rs->lri_version[i]);
      o.i64f(12, rs->lri_last_event_id[i]);
      o.b(0);
    }
  }
  o.i64f(48, x.last_event_task_id);
  o.i64f(50, x.last_first_event_id);
  o.i64f(52, x.last_processed_event);
  o.i64f(54, ps.start_time);
  o.i64f(56, ps.last_updated_time);
  o.i64f(58, x.decision_version);
  o.i64f(60, x.decision_schedule_id);
  o.i64f(62, x.decision_started_id);
  o.i32f(64, x.decision_timeout);
  o.i64f(66, x.decision_attempt);
  o.i64f(68, x.decision_started_ts);
  o.i64f(69, x.decision_scheduled_ts);
  const bool cancel = (x.flags & CDR_XI_CANCEL_REQUESTED) != 0;
  if (cancel) o.boolf(70, true);
  o.i64f(71, x.decision_original_scheduled_ts);
  o.strf(S, 72, x.create_request_id);
  o.strf(S, 74, x.decision_request_id);
  if (cancel) o.emptyf(76);  // CancelRequestID: replay never sets it (mutableStateBuilder.go:2504-2510)
  o.strf(S, 78, ps.sticky_task_list);
  o.i64f(80, ps.sticky_s2s_timeout);
  o.i64f(82, (int64_t)x.attempt);
  o.i32f(84, x.initial_interval);
  o.i32f(86, x.maximum_interval);
  o.i32f(88, x.maximum_attempts);
  o.i32f(90, x.expiration_seconds);
  o.dblf(92, x.backoff_coefficient);
  o.i64f(94, (x.flags & CDR_XI_HAS_EXPIRATION) ? x.expiration_time : ZERO_TIME_NANOS);
  if (x.nonretriable) {
    if (!S.ok(x.nonretriable)) o.err = o.err ? o.err : CDR_BLOB_E_HANDLE;
    o.fld(T_LIST, 96);
    o.raw(S.at(x.nonretriable), S.len(x.nonretriable));
  }
  o.boolf(98, (x.flags & CDR_XI_HAS_RETRY) != 0);
  o.strf(S, 100, x.cron_schedule);
  Out cnt{nullptr, 0, 0, 0, 0, 0};
  branch_token(cnt, S, x);
  const uint64_t token_len = cnt.pos;
  if (x.flags & CDR_XI_HAS_BRANCH) {  // ExecutionInfo.BranchToken (non-NDC builders)
    o.fld(T_STRING, 104), o.be32((uint32_t)token_len);
    branch_token(o, S, x);
  }
  o.i64f(106, (int64_t)x.signal_count);
  o.i64f(108, ps.history_size);
  o.strf(S, 110, ps.client_library_version);
  o.strf(S, 112, ps.client_feature_version);
  o.strf(S, 114, ps.client_impl);
  const bool has_rp = (x.flags & CDR_XI_HAS_RESET_POINTS) != 0;
  cnt.pos = 0;
  reset_points(cnt, S, rp, n_rp, has_rp);
  o.fld(T_STRING, 115), o.be32((uint32_t)cnt.pos);
  reset_points(o, S, rp, n_rp, has_rp);
  o.fld(T_STRING, 116), o.be32(8), o.lit("thriftrw", 8);
  if (x.flags & CDR_XI_HAS_SEARCH_ATTR) {
    o.fld(T_MAP, 118), o.b(T_STRING), o.b(T_STRING), o.be32(n_sa);
    for (uint32_t q = 0; q < n_sa; q++) {
      const cdr_kv kv = sa[q];
      if (!S.ok(kv.key) || !S.ok(kv.value)) o.err = o.err ? o.err : CDR_BLOB_E_HANDLE;
      o.be32((uint32_t)S.len(kv.key)), o.raw(S.at(kv.key), S.len(kv.key));
      o.be32((uint32_t)S.len(kv.value)), o.raw(S.at(kv.value), S.len(kv.value));
    }
  }
  uint64_t m0 = 0, m1 = 0;
  if ((x.flags & CDR_XI_HAS_MEMO) && x.memo && memo_fields(S, x.memo, m0, m1, o.err)) {
    o.fld(T_MAP, 120);
    o.raw(S.at(x.memo) + m0, m1 - m0);
  }
  if (builder == CDR_BUILDER_NDC) {  // versionHistories != nil
    const uint64_t tl = (x.flags & CDR_XI_VH_BRANCH) ? token_len : 0;
    cnt.pos = 0;
    version_histories(cnt, S, x, vh, n_vh, tl);
    o.fld(T_STRING, 122), o.be32((uint32_t)cnt.pos);
    version_histories(o, S, x, vh, n_vh, tl);
    o.fld(T_STRING, 124), o.be32(8), o.lit("thriftrw", 8);
  }
  o.b(0);
}

// ================================================================ the Cassandra form
// The bound values of the CQL statements the Cassandra persistence writes a row with
// (common/persistence/cassandra/cassandraPersistenceUtil.go, templates in
// cassandraPersistence.go:114-306,439-...): each a CQL native-protocol [bytes] value —
// big-endian int32 length (-1 = null), then the value as gocql
// (github.com/gocql/gocql v0.0.0-20171220143535-56a164ee9f31, go.mod:22; not vendored in
// the reference, its marshalling restated from the CQL v4 protocol and gocql's marshal.go)
// encodes it for the column's CQL type.
struct Cql {
  Out& o;
  const Strs& S;
  __device__ void i64(int64_t v) { o.be32(8), o.be64((uint64_t)v); }
  __device__ void i32(int32_t v) { o.be32(4), o.be32((uint32_t)v); }
  __device__ void boo(bool v) { o.be32(1), o.b(v ? 1u : 0u); }
  __device__ void dbl(double v) { o.be32(8), o.be64((uint64_t)__double_as_longlong(v)); }
  __device__ void null() { o.be32(0xFFFFFFFFu); }
  __device__ void empty() { o.be32(0); }  // "" text; the zero time.Time (marshalTimestamp: []byte{})
  // timestamp: milliseconds since the epoch, UTC().Unix()*1e3 + Nanosecond()/1e6 = floor(ns / 1e6)
  __device__ void ts(int64_t ns, bool zero) {
    if (zero) return empty();
    const int64_t q = ns / 1000000, r = ns % 1000000;
    i64(r < 0 ? q - 1 : q);
  }
  __device__ void text(uint32_t h) {
    if (!S.ok(h)) o.err = o.err ? o.err : CDR_BLOB_E_HANDLE;
    const uint64_t n = S.len(h);
    o.be32((uint32_t)n);
    if (n) o.raw(S.at(h), n);
  }
  __device__ void blob_or_null(uint32_t h) {  // a []byte field: handle 0 is Go's nil
    if (h == 0) return null();
    text(h);
  }
  __device__ void lit(const char* s, uint32_t n) { o.be32(n), o.lit(s, n); }
  // uuid from a Go string: gocql ParseUUID (a '-' where an even number of hex digits has
  // been read is skipped; exactly 32 hex digits) — CDR_BLOB_E_UUID where it fails
  __device__ void uuid_str(uint32_t h) {
    uint8_t u[16] = {};
    const uint64_t n = S.len(h);
    const uint8_t* s = S.at(h);
    uint32_t j = 0;
    bool ok = S.ok(h);
    for (uint64_t i = 0; ok && i < n; i++) {
      const uint32_t c = s[i];
      if (c == '-' && (j & 1) == 0) continue;
      const int v = c >= '0' && c <= '9' ? (int)(c - '0') : c >= 'a' && c <= 'f' ? (int)(c - 'a' + 10)
                    : c >= 'A' && c <= 'F' ? (int)(c - 'A' + 10) : -1;
      if (v < 0 || j >= 32) {
        ok = false;
        break;
      }
      u[j >> 1] |= (uint8_t)(v << ((j & 1) ? 0 : 4));
      j++;
    }
    if (!ok || j != 32) o.err = o.err ? o.err : CDR_BLOB_E_UUID;
    o.be32(16);
    for (int i = 0; i < 16; i++) o.b(u[i]);
  }
  __device__ void uuid_val(uint64_t lo, uint64_t hi) { o.be32(16), o.be64(hi), o.be64(lo); }  // ParseUUID(uuid_text)
  __device__ void uuid_const(uint32_t first_nibble) {  // emptyDomainID / emptyRunID "x0000000-0000-f000-f000-000000000000"
    o.be32(16), o.be32(first_nibble << 28), o.be32(0x0000F000u), o.be32(0xF0000000u), o.be32(0);
  }
  // list<text> from a handle holding the thrift list<string> wire body (element type,
  // i32 count, elements as i32 length + bytes): the CQL body is the same minus the type byte
  __device__ void list_text(uint32_t h) {
    if (h == 0) return null();
    if (!S.ok(h) || S.len(h) < 5) {
      o.err = o.err ? o.err : CDR_BLOB_E_HANDLE;
      return null();
    }
    o.be32((uint32_t)(S.len(h) - 1));
    o.raw(S.at(h) + 1, S.len(h) - 1);
  }
};

__device__ void activity_cql(Out& o, const Strs& S, const cdr_activity_info& a) {  // updateActivityInfos :1264-1337
  Cql q{o, S};
  const bool tset = (a.flags & CDR_AI_STARTED_TIME_SET) != 0;
  q.i64(a.schedule_id);  // activity_map[ ? ]
  q.i64(a.version);
  q.i64(a.schedule_id);
  q.i64(a.scheduled_event_batch_id);
  q.null();  // scheduled_event: nil on replay (FromDataBlob(nil) = nil, "")
  q.ts(a.scheduled_time, false);
  q.i64(a.started_id);
  q.null();  // started_event
  q.ts(a.started_time, !tset);
  q.text(a.activity_id);
  q.text(a.request_id);
  q.null();  // details
  q.i32(a.s2s);
  q.i32(a.s2c);
  q.i32(a.stc);
  q.i32(a.hb);
  q.boo((a.flags & CDR_AI_CANCEL_REQUESTED) != 0);
  q.i64(a.cancel_request_id);
  q.ts(a.last_heartbeat_time, !tset);
  q.i32(a.timer_task_status);
  q.i32(a.attempt);
  q.text(a.task_list);
  q.empty();  // started_identity ""
  q.boo((a.flags & CDR_AI_HAS_RETRY) != 0);
  q.i32(a.initial_interval);
  q.dbl(a.backoff_coefficient);
  q.i32(a.maximum_interval);
  q.ts(a.expiration_time, false);
  q.i32(a.maximum_attempts);
  q.list_text(a.nonretriable);
  q.empty();  // last_failure_reason ""
  q.empty();  // last_worker_identity ""
  q.null();   // last_failure_details nil
  q.empty();  // event_data_encoding "" (no scheduled event)
}
__device__ void timer_cql(Out& o, const Strs& S, const cdr_timer_info& t) {  // updateTimerInfos :1384-1422
  Cql q{o, S};
  q.text(t.timer_id);  // timer_map[ ? ]
  q.i64(t.version);
  q.text(t.timer_id);
  q.i64(t.started_id);
  q.ts(t.expiry_time, false);
  q.i64(t.task_id);
}
__device__ void child_cql(Out& o, const Strs& S, const cdr_child_info& c) {  // updateChildExecutionInfos :1444-1503
  Cql q{o, S};
  q.i64(c.initiated_id);  // child_executions_map[ ? ]
  q.i64(c.version);
  q.i64(c.initiated_id);
  q.i64(c.initiated_event_batch_id);
  q.null();  // initiated_event: nil on replay
  q.i64(c.started_id);
  q.text(c.started_workflow_id);
  if (S.len(c.started_run_id) == 0 && S.ok(c.started_run_id))
    q.uuid_const(3);  // emptyRunID
  else
    q.uuid_str(c.started_run_id);
  q.null();  // started_event
  q.uuid_val(c.create_request_lo, c.create_request_hi);
  q.empty();  // event_data_encoding ""
  q.text(c.domain_name);
  q.text(c.workflow_type);
  q.i32(c.parent_close_policy);
}
__device__ void cancel_cql(Out& o, const Strs& S, const cdr_cancel_info& c) {  // updateRequestCancelInfos :1530-1568
  Cql q{o, S};
  q.i64(c.initiated_id);  // request_cancel_map[ ? ]
  q.i64(c.version);
  q.i64(c.initiated_id);
  q.i64(c.initiated_event_batch_id);
  o.be32(36), o.uuid_text(c.cancel_request_lo, c.cancel_request_hi);  // cancel_request_id text
}
__device__ void signal_cql(Out& o, const Strs& S, const cdr_signal_info& g) {  // updateSignalInfos :1590-1631
  Cql q{o, S};
  q.i64(g.initiated_id);  // signal_map[ ? ]
  q.i64(g.version);
  q.i64(g.initiated_id);
  q.i64(g.initiated_event_batch_id);
  q.uuid_val(g.signal_request_lo, g.signal_request_hi);
  q.text(g.signal_name);
  q.blob_or_null(g.input);
  q.blob_or_null(g.control);
}

// updateExecution (:625-890): the workflow_execution UDT, then replication_state (2DC:
// templateUpdateWorkflowExecutionWithReplicationQuery) or next_event_id, version_histories,
// version_histories_encoding (NDC), or next_event_id alone (local)
__device__ void exec_cql(Out& o, const Strs& S, const cdr_exec_info& x, const cdr_exec_persist& ps, uint32_t builder,
                         const cdr_repl_state* rs, const cdr_vh_item* vh, uint32_t n_vh, const cdr_reset_point* rp,
                         uint32_t n_rp, const cdr_kv* sa, uint32_t n_sa, const uint32_t* cluster_names,
                         uint32_t n_clusters) {
  Cql q{o, S};
  q.uuid_str(x.domain_id);
  q.text(x.workflow_id);
  q.uuid_str(x.run_id);
  if (!S.ok(x.parent_domain_id)) o.err = o.err ? o.err : CDR_BLOB_E_HANDLE;
  if (S.len(x.parent_domain_id) != 0) {
    q.uuid_str(x.parent_domain_id);
    q.text(x.parent_workflow_id);
    q.uuid_str(x.parent_run_id);
    q.i64(x.initiated_id);
  } else {
    q.uuid_const(1);  // emptyDomainID
    q.empty();
    q.uuid_const(3);  // emptyRunID
    q.i64(-7);        // emptyInitiatedID
  }
  q.i64(x.completion_event_batch_id);
  q.null();   // completion_event: not in the replay projection
  q.empty();  // its encoding ""
  q.text(x.task_list);
  q.text(x.workflow_type);
  q.i32(x.workflow_timeout);
  q.i32(x.decision_timeout_value);
  q.blob_or_null(ps.execution_context);
  q.i32(x.state);
  q.i32(x.close_status);
  q.i64(x.last_first_event_id);
  q.i64(x.last_event_task_id);
  q.i64(x.next_event_id);
  q.i64(x.last_processed_event);
  q.ts(ps.start_time, ps.start_time == ZERO_TIME_NANOS);
  q.ts(ps.last_updated_time, ps.last_updated_time == ZERO_TIME_NANOS);
  q.uuid_str(x.create_request_id);
  q.i32((int32_t)x.signal_count);
  q.i64(ps.history_size);
  q.i64(x.decision_version);
  q.i64(x.decision_schedule_id);
  q.i64(x.decision_started_id);
  q.text(x.decision_request_id);
  q.i32(x.decision_timeout);
  q.i64(x.decision_attempt);
  q.i64(x.decision_started_ts);
  q.i64(x.decision_scheduled_ts);
  q.i64(x.decision_original_scheduled_ts);
  q.boo((x.flags & CDR_XI_CANCEL_REQUESTED) != 0);
  q.empty();  // cancel_request_id: replay never sets it
  q.text(ps.sticky_task_list);
  q.i32((int32_t)ps.sticky_s2s_timeout);
  q.text(ps.client_library_version);
  q.text(ps.client_feature_version);
  q.text(ps.client_impl);
  const bool has_rp = (x.flags & CDR_XI_HAS_RESET_POINTS) != 0;
  Out cnt{nullptr, 0, 0, 0, 0, 0};
  reset_points(cnt, S, rp, n_rp, has_rp);
  o.be32((uint32_t)cnt.pos);
  reset_points(o, S, rp, n_rp, has_rp);
  q.lit("thriftrw", 8);
  q.i32((int32_t)x.attempt);
  q.boo((x.flags & CDR_XI_HAS_RETRY) != 0);
  q.i32(x.initial_interval);
  q.dbl(x.backoff_coefficient);
  q.i32(x.maximum_interval);
  q.ts(x.expiration_time, !(x.flags & CDR_XI_HAS_EXPIRATION));
  q.i32(x.maximum_attempts);
  q.list_text(x.nonretriable);
  q.i32(-1);  // defaultEventStoreVersionValue
  cnt.pos = 0;
  branch_token(cnt, S, x);
  const uint64_t token_len = cnt.pos;
  if (x.flags & CDR_XI_HAS_BRANCH) {
    o.be32((uint32_t)token_len);
    branch_token(o, S, x);
  } else {
    q.null();
  }
  q.text(x.cron_schedule);
  q.i32(x.expiration_seconds);
  if (x.flags & CDR_XI_HAS_SEARCH_ATTR) {  // map<text, blob>
    uint64_t n = 4;
    for (uint32_t i = 0; i < n_sa; i++) n += 8 + S.len(sa[i].key) + S.len(sa[i].value);
    o.be32((uint32_t)n), o.be32(n_sa);
    for (uint32_t i = 0; i < n_sa; i++) {
      const cdr_kv kv = sa[i];
      if (!S.ok(kv.key) || !S.ok(kv.value)) o.err = o.err ? o.err : CDR_BLOB_E_HANDLE;
      o.be32((uint32_t)S.len(kv.key)), o.raw(S.at(kv.key), S.len(kv.key));
      o.be32((uint32_t)S.len(kv.value)), o.raw(S.at(kv.value), S.len(kv.value));
    }
  } else {
    q.null();
  }
  uint64_t m0 = 0, m1 = 0;  // memo: the thrift map body minus its key / value type bytes
  if ((x.flags & CDR_XI_HAS_MEMO) && x.memo && memo_fields(S, x.memo, m0, m1, o.err)) {
    o.be32((uint32_t)(m1 - m0 - 2));
    o.raw(S.at(x.memo) + m0 + 2, m1 - m0 - 2);
  } else {
    q.null();
  }
  if (builder == CDR_BUILDER_2DC) {  // replication_state
    q.i64(rs->current_version);
    q.i64(rs->start_version);
    q.i64(rs->last_write_version);
    q.i64(rs->last_write_event_id);
    uint32_t cnt_c = 0;
    uint64_t n = 4;
    for (uint32_t i = 0; i < n_clusters && i < CDR_MAX_CLUSTERS; i++)
      if ((rs->lri_mask >> i) & 1u) cnt_c++, n += 4 + S.len(cluster_names[i]) + 4 + 24;
    o.be32((uint32_t)n), o.be32(cnt_c);
    for (uint32_t i = 0; i < n_clusters && i < CDR_MAX_CLUSTERS; i++) {
      if (!((rs->lri_mask >> i) & 1u)) continue;
      q.text(cluster_names[i]);
      o.be32(24);  // frozen<replication_info>{version, last_event_id}
      q.i64(rs->lri_version[i]);
      q.i64(rs->lri_last_event_id[i]);
    }
    q.i64(x.next_event_id);
  } else if (builder == CDR_BUILDER_NDC) {
    q.i64(x.next_event_id);
    const uint64_t tl = (x.flags & CDR_XI_VH_BRANCH) ? token_len : 0;
    cnt.pos = 0;
    version_histories(cnt, S, x, vh, n_vh, tl);
    o.be32((uint32_t)cnt.pos);
    version_histories(o, S, x, vh, n_vh, tl);
    q.lit("thriftrw", 8);
  } else {
    q.i64(x.next_event_id);
  }
}

struct BlobArgs {
  int table;
  int cql;  // 1: the Cassandra form (cdr_encode_cql_async)
  Strs S;
  const cdr_exec_persist* persist;
  const uint32_t* cluster_names;
  uint64_t* sizes;      // size pass: row sizes (n_rows + 1, last 0)
  const uint64_t* off;  // write pass: exclusive scan of the sizes
  uint8_t* blobs;
  int32_t* status;
};

__device__ void emit_row(const BlobArgs& A, const cdr_dev_batch& B, const cdr_out& O, uint32_t w, uint64_t row,
                         Out& o) {
  const cdr_wf_result& r = O.result[w];
  const cdr_wf_caps& c = B.caps[w];
  if (A.cql) {
    switch (A.table) {
      case 0: activity_cql(o, A.S, O.act[row]); break;
      case 1: timer_cql(o, A.S, O.timer[row]); break;
      case 2: child_cql(o, A.S, O.child[row]); break;
      case 3: cancel_cql(o, A.S, O.cancel[row]); break;
      case 4: signal_cql(o, A.S, O.signal[row]); break;
      default:
        exec_cql(o, A.S, O.exec[w], A.persist[w], B.wfs[w].builder, O.repl + w, O.vh + c.vh_off, r.n_vh,
                 O.rp + c.rp_off, r.n_reset_points, O.sa + c.sa_off, r.n_search_attr, A.cluster_names,
                 B.cluster.n_clusters);
    }
    return;
  }
  switch (A.table) {
    case 0: activity_row(o, A.S, O.act[row]); break;
    case 2: child_row(o, A.S, O.child[row]); break;
    case 4: signal_row(o, A.S, O.signal[row]); break;
    default:
      exec_row(o, A.S, O.exec[w], A.persist[w], B.wfs[w].builder, O.repl + w, O.vh + c.vh_off,
               r.n_vh, O.rp + c.rp_off, r.n_reset_points, O.sa + c.sa_off, r.n_search_attr, A.cluster_names,
               B.cluster.n_clusters);
  }
}

template <bool WRITE>
__global__ __launch_bounds__(256) void k_blobs(BlobArgs A, cdr_dev_batch B, cdr_out O) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= B.n_wfs) return;
  const cdr_wf_result& r = O.result[w];
  const cdr_wf_caps& c = B.caps[w];
  const bool ok = r.code == CDR_OK;
  uint64_t off0 = w;
  uint32_t cap = 1, n = ok ? 1u : 0u;
  if (A.table == 0) off0 = c.act_off, cap = c.act_cap, n = ok ? r.n_activity : 0u;
  if (A.table == 1) off0 = c.timer_off, cap = c.timer_cap, n = ok ? r.n_timer : 0u;
  if (A.table == 2) off0 = c.child_off, cap = c.child_cap, n = ok ? r.n_child : 0u;
  if (A.table == 3) off0 = c.cancel_off, cap = c.cancel_cap, n = ok ? r.n_cancel : 0u;
  if (A.table == 4) off0 = c.signal_off, cap = c.signal_cap, n = ok ? r.n_signal : 0u;
  for (uint32_t j = 0; j < cap; j++) {
    const uint64_t row = off0 + j;
    if (!WRITE) {
      Out o{nullptr, 0, 0, 0, 0, 0};
      if (j < n) emit_row(A, B, O, w, row, o);
      A.sizes[row] = o.pos;
      if (A.status) A.status[row] = j < n ? o.err : 0;
    } else if (j < n) {
      const uint64_t a = A.off[row], e = A.off[row + 1];
      Out o{A.blobs, a, e, a, 0, 0};
      emit_row(A, B, O, w, row, o);
    }
  }
}

}  // namespace

#define HIPCHK(x)                                                                                     \
  do {                                                                                                \
    hipError_t _e = (x);                                                                              \
    if (_e != hipSuccess) {                                                                           \
      fprintf(stderr, "cdr: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(_e), __FILE__, __LINE__); \
      return CDR_API_EDEVICE;                                                                         \
    }                                                                                                 \
  } while (0)

static int encode_var(int cql, cdr_ctx* ctx, int table, const cdr_dev_batch* in, const cdr_out* out,
                      const cdr_strtab* strs, const cdr_exec_persist* persist, const uint32_t* cluster_names,
                      uint64_t n_rows, uint64_t* row_off, uint8_t* blobs, int32_t* row_status, void* stream);

extern "C" int cdr_encode_blobs_async(cdr_ctx* ctx, int table, const cdr_dev_batch* in, const cdr_out* out,
                                      const cdr_strtab* strs, const cdr_exec_persist* persist,
                                      const uint32_t* cluster_names, uint64_t n_rows, uint64_t* row_off,
                                      uint8_t* blobs, int32_t* row_status, void* stream) {
  if (table != 0 && table != 2 && table != 4 && table != 5) return CDR_API_EINVAL;
  return encode_var(0, ctx, table, in, out, strs, persist, cluster_names, n_rows, row_off, blobs, row_status, stream);
}

extern "C" int cdr_encode_cql_async(cdr_ctx* ctx, int table, const cdr_dev_batch* in, const cdr_out* out,
                                    const cdr_strtab* strs, const cdr_exec_persist* persist,
                                    const uint32_t* cluster_names, uint64_t n_rows, uint64_t* row_off,
                                    uint8_t* values, int32_t* row_status, void* stream) {
  if (table < 0 || table > 5) return CDR_API_EINVAL;
  return encode_var(1, ctx, table, in, out, strs, persist, cluster_names, n_rows, row_off, values, row_status, stream);
}

static int encode_var(int cql, cdr_ctx* ctx, int table, const cdr_dev_batch* in, const cdr_out* out,
                      const cdr_strtab* strs, const cdr_exec_persist* persist, const uint32_t* cluster_names,
                      uint64_t n_rows, uint64_t* row_off, uint8_t* blobs, int32_t* row_status, void* stream) {
  if (!ctx || !in || !out || !strs || !row_off || !out->result) return CDR_API_EINVAL;
  if ((table == 0 && !out->act) || (table == 1 && !out->timer) || (table == 2 && !out->child) ||
      (table == 3 && !out->cancel) || (table == 4 && !out->signal))
    return CDR_API_EINVAL;
  if (table == 5 && (!out->exec || !out->repl || !persist || !out->vh || !out->rp || !out->sa || n_rows < in->n_wfs ||
                     (in->cluster.n_clusters > 0 && !cluster_names)))
    return CDR_API_EINVAL;
  if (strs->n == 0 || !strs->bytes || !strs->off) return CDR_API_EINVAL;
  HIPCHK(hipSetDevice(cdr_ctx_device(ctx)));
  hipStream_t st = (hipStream_t)stream;
  BlobArgs A{table, cql, Strs{strs->bytes, strs->off, strs->n}, persist, cluster_names, nullptr, row_off, blobs,
             row_status};
  const dim3 grid((in->n_wfs + 255) / 256), blk(256);
  if (!blobs) {  // size pass + exclusive scan into row_off[0 .. n_rows]
    uint64_t* sizes = (uint64_t*)cdr_ws_get(ctx, WS_ENC_SIZES, (n_rows + 1) * sizeof(uint64_t));
    if (!sizes) return CDR_API_ENOMEM;
    HIPCHK(hipMemsetAsync(sizes, 0, (n_rows + 1) * sizeof(uint64_t), st));
    A.sizes = sizes;
    if (in->n_wfs) hipLaunchKernelGGL(k_blobs<false>, grid, blk, 0, st, A, *in, *out);
    HIPCHK(hipGetLastError());
    size_t tmp = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, sizes, row_off, n_rows + 1, st));
    void* t = cdr_ws_get(ctx, WS_ENC_TMP, tmp ? tmp : 8);
    if (!t) return CDR_API_ENOMEM;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(t, tmp, sizes, row_off, n_rows + 1, st));
    return CDR_API_OK;
  }
  if (in->n_wfs) hipLaunchKernelGGL(k_blobs<true>, grid, blk, 0, st, A, *in, *out);
  HIPCHK(hipGetLastError());
  return CDR_API_OK;
}
