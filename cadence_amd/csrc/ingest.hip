// ingest.hip — on-device decode of thriftrw history blobs into the replay's input
// records (cdr/ingest.h).
//
// One lane per blob (one history node = one applyEvents batch).  A thrift binary
// value is only addressable after the one before it is parsed, so a blob is a
// sequential walk; the parallelism is across blobs (a 1M-workflow population has tens
// of millions of them).  Three passes read the bytes:
//   1. k_blob_count   events, search-attribute pairs, reset points and string fields
//                     per blob, and the decode status;
//   2. k_blob_intern  every string into a device open-addressing table keyed by its
//                     64-bit hash (atomicCAS on the key; seeds first, with their handles);
//                     then the new strings are sorted by hash (hipcub radix sort) and
//                     get handles n_seeds + rank;
//   3. k_blob_fill    the cdr_event / cdr_kv / cdr_reset_point records at the offsets an
//                     exclusive scan of pass 1's counts gives, handles looked up.
// The parser is one template (the pass is its parameter), so the three walks agree on
// every byte.  Wire format: go.uber.org/thriftrw protocol.Binary — a struct is fields
// (type byte, big-endian i16 id, value) ending in a 0 byte; i16/i32/i64/double
// big-endian; string/binary an i32 length and the bytes; list/set an element type, an
// i32 count and the elements; map key type, value type, i32 count, pairs.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <vector>

#include "cdr/cdr.h"
#include "cdr/ingest.h"
#include "ctx.h"
#include "internal.h"

#define HIPCHK(x)                                                                                     \
  do {                                                                                                \
    hipError_t _e = (x);                                                                              \
    if (_e != hipSuccess) {                                                                           \
      fprintf(stderr, "cdr: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(_e), __FILE__, __LINE__); \
      return CDR_API_EDEVICE;                                                                         \
    }                                                                                                 \
  } while (0)

namespace {

enum : uint32_t {
  T_STOP = 0, T_BOOL = 2, T_BYTE = 3, T_DOUBLE = 4, T_I16 = 6, T_I32 = 8, T_I64 = 10, T_STRING = 11,
  T_STRUCT = 12, T_MAP = 13, T_SET = 14, T_LIST = 15
};
constexpr uint32_t UNASSIGNED = 0xFFFFFFFFu;
constexpr uint64_t SEED_REF = 1ull << 63;

// ---------------------------------------------------------------- string table
struct STab {
  unsigned long long* key;  // 0 = empty slot
  uint32_t* val;            // handle (UNASSIGNED until ranked)
  uint64_t* ref;            // blob-byte offset of the first occurrence (| SEED_REF: seed byte offset)
  uint32_t* len;
  uint64_t mask;
  uint32_t* overflow;
};
__device__ __forceinline__ uint64_t slot0(uint64_t h, uint64_t mask) { return cdr_mix64(h) & mask; }

__device__ void tab_insert(const STab& T, uint64_t h, uint64_t ref, uint32_t len, uint32_t handle) {
  uint64_t i = slot0(h, T.mask);
  for (uint64_t probe = 0; probe <= T.mask; probe++, i = (i + 1) & T.mask) {
    // most string fields repeat a string already in the table (task lists, types, ids):
    // a plain load finds those without an atomic on a slot every lane of the chip hits
    const unsigned long long seen = __hip_atomic_load(&T.key[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (seen == (unsigned long long)h) return;
    if (seen != 0ull) continue;
    const unsigned long long k = atomicCAS(&T.key[i], 0ull, (unsigned long long)h);
    if (k == 0ull) {  // this lane owns the slot
      T.ref[i] = ref;
      T.len[i] = len;
      T.val[i] = handle;
      return;
    }
    if (k == h) return;
  }
  atomicOr(T.overflow, 1u);  // sized at twice the string fields: never taken
}

__device__ uint32_t tab_lookup(const STab& T, uint64_t h) {
  uint64_t i = slot0(h, T.mask);
  for (uint64_t probe = 0; probe <= T.mask; probe++, i = (i + 1) & T.mask) {
    const uint64_t k = T.key[i];
    if (k == h) return T.val[i];
    if (k == 0) break;
  }
  return 0;  // not interned (cannot happen after pass 2)
}

// ---------------------------------------------------------------- reader
// Each wavefront first copies its 64 consecutive blobs — one contiguous byte range — into
// LDS with 16-byte loads (64 lanes x 16 B per instruction, coalesced), so the parse reads
// bytes from LDS; a wave whose range exceeds its share of LDS (CDR_INGEST_STAGE) reads
// through a 16-byte aligned window held in registers (one global_load_dwordx4 per 16
// bytes instead of a load per byte), as does any byte outside the staged range; the last
// 16 bytes of the buffer, which an aligned window could overrun, are read byte by byte.
#ifndef CDR_INGEST_STAGE
#define CDR_INGEST_STAGE 12288 /* bytes of blob data staged in LDS per wavefront */
#endif
#define LDS3 __attribute__((address_space(3)))
extern __shared__ uint4 ing_lds[];
struct Rd {
  const uint8_t* b;  // blob_bytes
  uint64_t pos, end;
  uint64_t total;    // bytes in blob_bytes
  uint64_t wb;       // window address (16-aligned), ~0 = empty
  uint64_t w0, w1;
  const LDS3 uint8_t* sb;  // the wave's staged bytes: addresses [s_lo, s_lo + s_n)
  uint64_t s_lo, s_n;
  int32_t err;
  __device__ __forceinline__ void init(const uint8_t* base, uint64_t p, uint64_t e, uint64_t t) {
    b = base;
    pos = p;
    end = e;
    total = t;
    wb = ~0ull;
    sb = nullptr;
    s_lo = s_n = 0;
    err = CDR_DEC_OK;
  }
  __device__ __forceinline__ uint32_t at(uint64_t p) {
    // the window is aligned in the address space (the buffer itself need not be)
    const uint64_t addr = (uint64_t)(uintptr_t)(b + p), a = addr & ~15ull;
    if (addr - s_lo < s_n) return sb[addr - s_lo];
    if (a != wb) {
      const uint64_t lo = (uint64_t)(uintptr_t)b;
      if (a < lo || a + 16 > lo + total) return b[p];
      const uint4 v = *reinterpret_cast<const uint4*>((uintptr_t)a);
      w0 = (uint64_t)v.x | ((uint64_t)v.y << 32);
      w1 = (uint64_t)v.z | ((uint64_t)v.w << 32);
      wb = a;
    }
    const uint32_t o = (uint32_t)(addr - a);
    return (uint32_t)(((o < 8) ? (w0 >> (8 * o)) : (w1 >> (8 * (o - 8)))) & 0xFFu);
  }
  __device__ __forceinline__ bool ok() const { return err == CDR_DEC_OK; }
  __device__ __forceinline__ bool need(uint64_t n) {
    if (err) return false;
    if (end - pos < n) {
      err = CDR_DEC_TRUNCATED;
      pos = end;
      return false;
    }
    return true;
  }
  __device__ __forceinline__ uint32_t u8() {
    if (!need(1)) return 0;
    return at(pos++);
  }
  __device__ __forceinline__ uint32_t be16() {
    if (!need(2)) return 0;
    const uint32_t v = (at(pos) << 8) | at(pos + 1);
    pos += 2;
    return v;
  }
  __device__ __forceinline__ uint32_t be32() {
    if (!need(4)) return 0;
    const uint32_t v = (at(pos) << 24) | (at(pos + 1) << 16) | (at(pos + 2) << 8) | at(pos + 3);
    pos += 4;
    return v;
  }
  __device__ __forceinline__ uint64_t be64() {
    const uint64_t hi = be32();
    return (hi << 32) | be32();
  }
  __device__ __forceinline__ int32_t size() {  // a length / count: negative is a decode error
    const int32_t n = (int32_t)be32();
    if (n < 0 && !err) err = CDR_DEC_BAD_SIZE;
    return n < 0 ? 0 : n;
  }
  // cdr_str_hash of bytes [p, p + n), through the window
  __device__ uint64_t hash(uint64_t p, uint64_t n) {
    uint64_t h = 0xCBF29CE484222325ull;
    for (uint64_t i = 0; i < n; i++) h = (h ^ at(p + i)) * 0x100000001B3ull;
    h = cdr_mix64(h ^ (n * 0x9E3779B97F4A7C15ull));
    return h ? h : 1u;
  }
};

__device__ __forceinline__ uint32_t fixed_size(uint32_t t) {
  switch (t) {
    case T_BOOL: case T_BYTE: return 1;
    case T_I16: return 2;
    case T_I32: return 4;
    case T_I64: case T_DOUBLE: return 8;
    default: return 0;
  }
}

// skip one value of wire type t (iterative: an explicit stack of open containers)
__device__ __forceinline__ void skip_body(Rd& r, uint32_t t) {
  struct Fr {
    uint32_t kind, t1, t2;
    uint32_t n;  // remaining elements (maps: 2 per pair)
  };
  Fr st[CDR_THRIFT_MAX_DEPTH];
  int d = 0;
  uint32_t cur = t;
  for (;;) {
    if (!r.ok()) return;
    // ---- one value of type cur
    if (const uint32_t fs = fixed_size(cur)) {
      if (r.need(fs)) r.pos += fs;
    } else if (cur == T_STRING) {
      const uint32_t n = (uint32_t)r.size();
      if (r.need(n)) r.pos += n;
    } else if (cur == T_STRUCT || cur == T_LIST || cur == T_SET || cur == T_MAP) {
      if (d == CDR_THRIFT_MAX_DEPTH) {
        r.err = CDR_DEC_DEPTH;
        return;
      }
      Fr f{cur, 0, 0, 0};
      if (cur == T_LIST || cur == T_SET) {
        f.t1 = r.u8();
        f.n = (uint32_t)r.size();
      } else if (cur == T_MAP) {
        f.t1 = r.u8();
        f.t2 = r.u8();
        f.n = 2u * (uint32_t)r.size();
      }
      st[d++] = f;
    } else {
      r.err = CDR_DEC_BAD_TYPE;
      return;
    }
    // ---- the next value, from the innermost open container
    bool have = false;
    while (d > 0 && !have && r.ok()) {
      Fr& f = st[d - 1];
      if (f.kind == T_STRUCT) {
        const uint32_t ft = r.u8();
        if (ft == T_STOP) {
          d--;
          continue;
        }
        r.be16();
        cur = ft;
        have = true;
      } else if (f.n == 0) {
        d--;
      } else {
        cur = (f.kind == T_MAP && (f.n & 1u)) ? f.t2 : f.t1;
        f.n--;
        have = true;
      }
    }
    if (!have) return;
  }
}

// a container skipped out of line: the reader's fields go by value and the new position /
// error come back in registers, so a call site does not force the caller's reader (or any
// other parser state) into scratch memory; the walker's own stack lives in the callee's frame
struct SkipRes {
  uint64_t pos;
  int32_t err;
};
__device__ __attribute__((noinline)) SkipRes skip_v(const uint8_t* b, uint64_t pos, uint64_t end, uint64_t total,
                                                    const LDS3 uint8_t* sb, uint64_t s_lo, uint64_t s_n, uint32_t t) {
  Rd r;
  r.init(b, pos, end, total);
  r.sb = sb;
  r.s_lo = s_lo;
  r.s_n = s_n;
  skip_body(r, t);
  return SkipRes{r.pos, r.err};
}
__device__ __forceinline__ void skip(Rd& r, uint32_t t) {
  if (r.err) return;
  const SkipRes x = skip_v(r.b, r.pos, r.end, r.total, r.sb, r.s_lo, r.s_n, t);
  r.pos = x.pos;
  r.err = x.err;
}

// skip one value: a fixed-size or string value inline; a container through skip() (a call:
// its explicit stack lives in scratch, so the common field types must not pay for it)
__device__ __forceinline__ void skip1(Rd& r, uint32_t t) {
  if (const uint32_t fs = fixed_size(t)) {
    if (r.need(fs)) r.pos += fs;
  } else if (t == T_STRING) {
    const uint32_t n = (uint32_t)r.size();
    if (r.need(n)) r.pos += n;
  } else {
    skip(r, t);
  }
}

// ---------------------------------------------------------------- one blob
enum Pass { COUNT = 0, INTERN = 1, FILL = 2 };

struct Ctx {  // per launch
  const uint8_t* bytes;
  const uint64_t* blob_off;
  uint64_t total;  // bytes in `bytes`
  STab T;
  const uint32_t* dom_id;  // [n_seeds]: ID handle of a domain name seed, UNASSIGNED otherwise
  uint32_t n_seeds;
  // pass outputs
  uint32_t* counts;   // COUNT: [4 * n_blobs] events, kvs, rps, strings
  unsigned long long* totals;  // COUNT: string fields, failed blobs
  const uint64_t* bases;  // FILL: [3 * n_blobs] event, kv, rp bases
  int32_t* status;
  cdr_event* events;
  cdr_kv* kvs;
  cdr_reset_point* rps;
};

template <int P>
struct Blob {
  const Ctx C;  // by value: a reference to the kernel argument would copy it to scratch
  Rd r;
  uint32_t n_ev = 0, n_kv = 0, n_rp = 0, n_str = 0;
  uint64_t ev0 = 0, kv0 = 0, rp0 = 0;

  __device__ __forceinline__ Blob(const Ctx& c, uint32_t b) : C(c) {
    r.init(c.bytes, c.blob_off[b], c.blob_off[b + 1], c.total);
    if (P == FILL) {
      ev0 = c.bases[3ull * b];
      kv0 = c.bases[3ull * b + 1];
      rp0 = c.bases[3ull * b + 2];
    }
  }

  // a string / binary value (the field's wire type already checked): its handle
  __device__ __forceinline__ uint32_t str() {
    const uint32_t n = (uint32_t)r.size();
    if (!r.need(n)) return 0;
    const uint64_t at = r.pos;
    r.pos += n;
    if (n == 0) return 0;
    n_str++;
    if (P == COUNT) return 0;
    const uint64_t h = r.hash(at, n);
    if (P == INTERN) {
      tab_insert(C.T, h, at, n, UNASSIGNED);
      return 0;
    }
    return tab_lookup(C.T, h);
  }
  // a whole value of wire type t interned by its bytes (structures kept as one handle)
  __device__ __forceinline__ uint32_t raw(uint32_t t) {
    const uint64_t at = r.pos;
    skip1(r, t);  // (a container: skip())
    if (!r.ok() || r.pos == at) return 0;
    const uint32_t n = (uint32_t)(r.pos - at);
    n_str++;
    if (P == COUNT) return 0;
    const uint64_t h = r.hash(at, n);
    if (P == INTERN) {
      tab_insert(C.T, h, at, n, UNASSIGNED);
      return 0;
    }
    return tab_lookup(C.T, h);
  }
  __device__ __forceinline__ uint32_t domain_id(uint32_t name, bool* missing) {
    const uint32_t id = (P == FILL && name < C.n_seeds) ? C.dom_id[name] : UNASSIGNED;
    *missing = id == UNASSIGNED;
    return id == UNASSIGNED ? 0u : id;
  }
  // iterate the fields of a struct: f(field type, field id) must consume the value
  template <class F>
  __device__ __forceinline__ void fields(F&& f) {
    while (r.ok()) {
      const uint32_t ft = r.u8();
      if (!r.ok() || ft == T_STOP) return;
      const uint32_t fid = r.be16();
      if (!r.ok()) return;
      f(ft, fid);
    }
  }
  __device__ __forceinline__ int64_t i64(uint32_t ft) {
    if (ft != T_I64) {
      skip1(r, ft);
      return 0;
    }
    return (int64_t)r.be64();
  }
  // name of a WorkflowType / TaskList / ActivityType (field 10)
  __device__ __forceinline__ uint32_t name_of(uint32_t ft) {
    if (ft != T_STRUCT) {
      skip1(r, ft);
      return 0;
    }
    uint32_t h = 0;
    fields([&](uint32_t t, uint32_t id) {
      if (id == 10 && t == T_STRING) h = str();
      else skip1(r, t);
    });
    return h;
  }
  // shared.WorkflowExecution{10 workflowId, 20 runId}
  __device__ __forceinline__ void execution(uint32_t ft, uint32_t* wid, uint32_t* rid) {
    if (ft != T_STRUCT) {
      skip1(r, ft);
      return;
    }
    fields([&](uint32_t t, uint32_t id) {
      if (id == 10 && t == T_STRING) *wid = str();
      else if (id == 20 && t == T_STRING) *rid = str();
      else skip1(r, t);
    });
  }
  // RetryPolicy (shared.thrift RetryPolicy): the fields the record keeps
  template <class A>
  __device__ __forceinline__ void retry(A& a) {
    fields([&](uint32_t t, uint32_t id) {
      if (id == 10 && t == T_I32) a.retry_initial_s = (int32_t)r.be32();
      else if (id == 20 && t == T_DOUBLE) a.backoff_coefficient = __longlong_as_double((long long)r.be64());
      else if (id == 30 && t == T_I32) a.retry_max_interval_s = (int32_t)r.be32();
      else if (id == 40 && t == T_I32) a.retry_max_attempts = (int32_t)r.be32();
      else if (id == 60 && t == T_I32) a.retry_expiration_s = (int32_t)r.be32();
      else if (id == 50 && t == T_LIST) {  // nonRetriableErrorReasons: the list's bytes, empty -> 0
        const uint64_t at = r.pos;
        r.u8();
        const int32_t cnt = r.size();
        r.pos = r.ok() ? at : r.pos;
        a.nonretriable = cnt > 0 ? raw(T_LIST) : (skip1(r, T_LIST), 0u);
      } else skip1(r, t);
    });
  }
  // SearchAttributes{10: map<string, binary>} -> kv rows; returns the pair count
  __device__ __forceinline__ uint32_t search_attrs(uint32_t* off) {
    uint32_t cnt = 0;
    *off = (uint32_t)(kv0 + n_kv);
    fields([&](uint32_t t, uint32_t id) {
      if (id != 10 || t != T_MAP) {
        skip1(r, t);
        return;
      }
      const uint32_t kt = r.u8(), vt = r.u8();
      const int32_t n = r.size();
      for (int32_t i = 0; i < n && r.ok(); i++) {
        if (kt == T_STRING && vt == T_STRING) {
          const uint32_t k = str(), v = str();
          if (P == FILL) C.kvs[kv0 + n_kv] = cdr_kv{k, v};
          n_kv++;
          cnt++;
        } else {  // not a map<string, binary>: thriftrw reads no entries
          skip1(r, kt);
          skip1(r, vt);
        }
      }
    });
    return cnt;
  }
  // ResetPoints{10: list<ResetPointInfo>} -> reset-point rows; false when field 10 is absent
  __device__ __forceinline__ bool reset_points(uint32_t* off, uint32_t* len) {
    bool have = false;
    *off = (uint32_t)(rp0 + n_rp);
    *len = 0;
    fields([&](uint32_t t, uint32_t id) {
      if (id != 10 || t != T_LIST) {
        skip1(r, t);
        return;
      }
      const uint32_t et = r.u8();
      const int32_t n = r.size();
      if (et != T_STRUCT) {  // not a list of structs: no points
        for (int32_t i = 0; i < n && r.ok(); i++) skip1(r, et);
        return;
      }
      have = true;
      for (int32_t i = 0; i < n && r.ok(); i++) {
        cdr_reset_point p{};
        fields([&](uint32_t t2, uint32_t id2) {
          if (id2 == 10 && t2 == T_STRING) {
            p.binary_checksum = str();
            p.flags |= CDR_RP_HAS_CHECKSUM;
          } else if (id2 == 20 && t2 == T_STRING) {
            p.run_id = str();
            p.flags |= CDR_RP_HAS_RUN_ID;
          } else if (id2 == 30 && t2 == T_I64) {
            p.first_decision_completed_id = (int64_t)r.be64();
            p.flags |= CDR_RP_HAS_FIRST_DC_ID;
          } else if (id2 == 40 && t2 == T_I64) {
            p.created_time_nano = (int64_t)r.be64();
            p.flags |= CDR_RP_HAS_CREATED;
          } else if (id2 == 50 && t2 == T_I64) {
            p.expiring_time_nano = (int64_t)r.be64();
            p.flags |= CDR_RP_HAS_EXPIRING;
          } else if (id2 == 60 && t2 == T_BOOL) {
            p.flags |= CDR_RP_HAS_RESETTABLE | (r.u8() ? CDR_RP_RESETTABLE : 0u);
          } else skip1(r, t2);
        });
        if (P == FILL) C.rps[rp0 + n_rp] = p;
        n_rp++;
        (*len)++;
      }
    });
    return have;
  }

  // WorkflowExecutionStartedEventAttributes (shared.thrift, field 40 of HistoryEvent)
  __device__ __forceinline__ void started(cdr_attr_wf_started& s) {
    fields([&](uint32_t t, uint32_t id) {
      switch (id) {
        case 10: s.workflow_type = name_of(t); break;
        case 12:
          if (t == T_STRING) {
            bool miss;
            s.flags |= CDR_SF_HAS_PARENT_DOMAIN;
            s.parent_domain_id = domain_id(str(), &miss);
            s.flags |= miss ? CDR_SF_PARENT_DOMAIN_MISSING : 0u;
          } else skip1(r, t);
          break;
        case 14:
          if (t == T_STRUCT) s.flags |= CDR_SF_HAS_PARENT_EXEC;
          execution(t, &s.parent_workflow_id, &s.parent_run_id);
          break;
        case 16:
          if (t == T_I64) {
            s.flags |= CDR_SF_HAS_PARENT_INITIATED;
            s.parent_initiated_id = (int64_t)r.be64();
          } else skip1(r, t);
          break;
        case 20: s.task_list = name_of(t); break;
        case 40: if (t == T_I32) s.exec_timeout_s = (int32_t)r.be32(); else skip1(r, t); break;
        case 50: if (t == T_I32) s.task_timeout_s = (int32_t)r.be32(); else skip1(r, t); break;
        case 54: if (t == T_STRING) s.continued_run_id = str(); else skip1(r, t); break;
        case 55:
          if (t == T_I32) {  // ContinueAsNewInitiator: Decider 0, RetryPolicy 1, CronSchedule 2
            const int32_t v = (int32_t)r.be32();
            s.flags |= CDR_SF_HAS_INITIATOR | (v == 2 ? CDR_SF_CRON_INITIATOR : 0u) |
                       (v == 1 ? CDR_SF_RETRY_INITIATOR : 0u) | (v == 0 ? CDR_SF_DECIDER_INITIATOR : 0u);
          } else skip1(r, t);
          break;
        case 70:
          if (t == T_STRUCT) {
            s.flags |= CDR_SF_HAS_RETRY;
            retry(s);
          } else skip1(r, t);
          break;
        case 80: if (t == T_I32) s.attempt = (int32_t)r.be32(); else skip1(r, t); break;
        case 90: if (t == T_I64) s.expiration_ts = (int64_t)r.be64(); else skip1(r, t); break;
        case 100: if (t == T_STRING) s.cron_schedule = str(); else skip1(r, t); break;
        case 110: if (t == T_I32) s.first_decision_backoff_s = (int32_t)r.be32(); else skip1(r, t); break;
        case 120:
          if (t == T_STRUCT) {
            s.flags |= CDR_SF_HAS_MEMO;
            s.memo = raw(T_STRUCT);
          } else skip1(r, t);
          break;
        case 121:
          if (t == T_STRUCT) {
            s.flags |= CDR_SF_HAS_SEARCH_ATTR;
            s.search_attr_len = search_attrs(&s.search_attr_off);
          } else skip1(r, t);
          break;
        case 130:
          if (t == T_STRUCT) {
            if (reset_points(&s.reset_points_off, &s.reset_points_len)) s.flags |= CDR_SF_HAS_RESET_POINTS;
            else s.reset_points_off = s.reset_points_len = 0;
          } else skip1(r, t);
          break;
        default: skip1(r, t); break;
      }
    });
  }

  // StartChild / SignalExternal / RequestCancelExternal ...Initiated
  __device__ __forceinline__ void external(uint32_t attr, cdr_attr_external& x) {
    // field ids: domain, workflowId (child), WorkflowExecution, workflowType (child),
    // signalName, input, control, childWorkflowOnly, parentClosePolicy
    const bool child = attr == 340, sig = attr == 420;
    const uint32_t f_dom = child ? 10 : 20, f_we = child ? 0 : 30, f_wid = child ? 20 : 0;
    const uint32_t f_in = child ? 50 : (sig ? 50 : 0), f_ctl = child ? 90 : (sig ? 60 : 40);
    const uint32_t f_only = child ? 0 : (sig ? 70 : 50);
    uint32_t dom_name = 0;
    bool have_dom = false;
    fields([&](uint32_t t, uint32_t id) {
      if (id == f_dom && t == T_STRING) {
        dom_name = str();
        have_dom = true;
      } else if (f_we && id == f_we) execution(t, &x.workflow_id, &x.run_id);
      else if (f_wid && id == f_wid && t == T_STRING) x.workflow_id = str();
      else if (child && id == 30) x.workflow_type = name_of(t);
      else if (sig && id == 40 && t == T_STRING) x.signal_name = str();
      else if (f_in && id == f_in && t == T_STRING) x.input = str();
      else if (id == f_ctl && t == T_STRING) x.control = str();
      else if (f_only && id == f_only && t == T_BOOL) x.flags |= r.u8() ? CDR_XF_CHILD_ONLY : 0u;
      else if (child && id == 81 && t == T_I32) x.parent_close_policy = (int32_t)r.be32();
      else skip1(r, t);
    });
    (void)have_dom;
    x.domain = dom_name;
    bool miss;
    x.target_domain_id = domain_id(dom_name, &miss);
    x.flags |= miss ? CDR_XF_DOMAIN_MISSING : 0u;
  }

  // the attribute struct (HistoryEvent field `attr`) into the record's union
  __device__ __forceinline__ void attributes(uint32_t attr, cdr_event& e) {
    // decision / activity events: field ids of scheduledEventId, startedEventId,
    // requestId, activityId, timeoutType, attempt, binaryChecksum (0 = none)
    struct Ids {
      uint16_t attr;
      uint8_t sched, started, req, aid, to, att, cks;
    };
    static constexpr Ids kIds[] = {
        {90, 10, 0, 30, 0, 0, 0, 0},    // DecisionTaskStarted
        {100, 20, 30, 0, 0, 0, 0, 50},  // DecisionTaskCompleted
        {110, 10, 20, 0, 0, 30, 0, 0},  // DecisionTaskTimedOut
        {120, 10, 20, 0, 0, 0, 0, 0},   // DecisionTaskFailed
        {140, 10, 0, 30, 0, 0, 40, 0},  // ActivityTaskStarted
        {150, 20, 30, 0, 0, 0, 0, 0},   // ActivityTaskCompleted
        {160, 30, 40, 0, 0, 0, 0, 0},   // ActivityTaskFailed
        {170, 10, 20, 0, 0, 30, 0, 0},  // ActivityTaskTimedOut
        {200, 0, 0, 0, 10, 0, 0, 0},    // ActivityTaskCancelRequested
        {210, 0, 0, 0, 10, 0, 0, 0},    // RequestCancelActivityTaskFailed
        {220, 30, 40, 0, 0, 0, 0, 0},   // ActivityTaskCanceled
    };
    // child / external closes: initiatedEventId, WorkflowExecution
    struct Ref {
      uint16_t attr;
      uint8_t init, we;
    };
    static constexpr Ref kRef[] = {
        {310, 50, 40}, {320, 10, 30}, {350, 60, 0},  {360, 20, 30}, {370, 50, 30}, {380, 60, 40},
        {390, 50, 30}, {400, 50, 30}, {410, 40, 20}, {430, 50, 40}, {440, 10, 30},
    };
    switch (attr) {
      case 40: started(e.a.started); return;
      case 80:
        fields([&](uint32_t t, uint32_t id) {
          if (id == 10) e.a.dt_sched.task_list = name_of(t);
          else if (id == 20 && t == T_I32) e.a.dt_sched.start_to_close_s = (int32_t)r.be32();
          else if (id == 30 && t == T_I64) e.a.dt_sched.attempt = (int64_t)r.be64();
          else skip1(r, t);
        });
        return;
      case 130: {
        cdr_attr_at_scheduled& a = e.a.at_sched;
        fields([&](uint32_t t, uint32_t id) {
          if (id == 10 && t == T_STRING) a.activity_id = str();
          else if (id == 25 && t == T_STRING) a.domain = str();
          else if (id == 30) a.task_list = name_of(t);
          else if (id == 45 && t == T_I32) a.s2c_s = (int32_t)r.be32();
          else if (id == 50 && t == T_I32) a.s2s_s = (int32_t)r.be32();
          else if (id == 55 && t == T_I32) a.stc_s = (int32_t)r.be32();
          else if (id == 60 && t == T_I32) a.hb_s = (int32_t)r.be32();
          else if (id == 110 && t == T_STRUCT) {
            a.flags |= CDR_AF_HAS_RETRY;
            retry(a);
          } else skip1(r, t);
        });
        if (a.domain) {  // the target domain's ID (refreshTasks, getTargetDomainID)
          bool miss;
          a.target_domain_id = domain_id(a.domain, &miss);
          a.flags |= miss ? CDR_AF_DOMAIN_MISSING : 0u;
        }
        return;
      }
      case 180: case 190: case 230: case 240: {
        cdr_attr_timer& a = e.a.timer;
        fields([&](uint32_t t, uint32_t id) {
          if (id == 10 && t == T_STRING) a.timer_id = str();
          else if (id == 20 && t == T_I64) {
            const int64_t v = (int64_t)r.be64();
            if (attr == 180) a.start_to_fire_s = v;
            else if (attr != 240) a.started_event_id = v;
          } else skip1(r, t);
        });
        return;
      }
      case 300: case 340: case 420: external(attr, e.a.ext); return;
      case 330:
        fields([&](uint32_t t, uint32_t id) {
          if (id == 10 && t == T_STRING) e.a.can.new_execution_run_id = str();
          else skip1(r, t);
        });
        return;
      case 450:
        fields([&](uint32_t t, uint32_t id) {
          if (id == 20 && t == T_STRUCT) e.a.upsert.search_attr_len = search_attrs(&e.a.upsert.search_attr_off);
          else skip1(r, t);
        });
        return;
      default: break;
    }
    for (const Ids& m : kIds) {
      if (m.attr != attr) continue;
      const bool act = attr >= 140;
      fields([&](uint32_t t, uint32_t id) {
        if (m.sched && id == m.sched && t == T_I64) {
          const int64_t v = (int64_t)r.be64();
          if (act) e.a.at.scheduled_event_id = v;
          else e.a.dt.scheduled_event_id = v;
        } else if (m.started && id == m.started && t == T_I64) {
          const int64_t v = (int64_t)r.be64();
          if (act) e.a.at.started_event_id = v;
          else e.a.dt.started_event_id = v;
        } else if (m.req && id == m.req && t == T_STRING) {
          const uint32_t h = str();
          if (act) e.a.at.request_id = h;
          else e.a.dt.request_id = h;
        } else if (m.aid && id == m.aid && t == T_STRING) {
          e.a.at.activity_id = str();
        } else if (m.to && id == m.to && t == T_I32) {
          const int32_t v = (int32_t)r.be32();
          if (act) e.a.at.timeout_type = v;
          else e.a.dt.timeout_type = v;
        } else if (m.att && id == m.att && t == T_I32) {
          e.a.at.attempt = (int32_t)r.be32();
        } else if (m.cks && id == m.cks && t == T_STRING) {
          e.a.dt.binary_checksum = str();
        } else skip1(r, t);
      });
      return;
    }
    for (const Ref& m : kRef) {
      if (m.attr != attr) continue;
      fields([&](uint32_t t, uint32_t id) {
        if (id == m.init && t == T_I64) e.a.ref.initiated_event_id = (int64_t)r.be64();
        else if (m.we && id == m.we) {
          uint32_t wid = 0;
          execution(t, &wid, &e.a.ref.run_id);
        } else skip1(r, t);
      });
      return;
    }
    skip1(r, T_STRUCT);  // an attribute struct the record form does not keep
  }

  // HistoryEvent (shared.thrift:868-916)
  __device__ __forceinline__ void event(bool first) {
    cdr_event e;
    uint64_t* z = reinterpret_cast<uint64_t*>(&e);
#pragma unroll
    for (uint32_t i = 0; i < sizeof(cdr_event) / 8; i++) z[i] = 0;
    fields([&](uint32_t t, uint32_t id) {
      switch (id) {
        case 10: e.event_id = i64(t); break;
        case 20: e.timestamp = i64(t); break;
        case 30: if (t == T_I32) e.type = r.be32(); else skip1(r, t); break;
        case 35: e.version = i64(t); break;
        case 36: e.task_id = i64(t); break;
        default:
          if (t == T_STRUCT && id >= 40 && id <= 450 && id % 10 == 0) attributes(id, e);
          else skip1(r, t);
          break;
      }
    });
    e.flags = first ? CDR_EVF_BATCH_FIRST : 0u;
    if (P == FILL && r.ok()) {
      cdr_event* d = C.events + ev0 + n_ev;
      const uint64_t* s = reinterpret_cast<const uint64_t*>(&e);
      uint64_t* o = reinterpret_cast<uint64_t*>(d);
#pragma unroll
      for (uint32_t i = 0; i < sizeof(cdr_event) / 8; i++) o[i] = s[i];
    }
    n_ev++;
  }

  // codec preamble + History{10: list<HistoryEvent>}
  __device__ __forceinline__ void run() {
    if (r.end <= r.pos) {
      r.err = CDR_DEC_MISSING_VERSION;
      return;
    }
    if (r.u8() != CDR_THRIFT_PREAMBLE_V0) {
      r.err = CDR_DEC_INVALID_VERSION;
      return;
    }
    fields([&](uint32_t t, uint32_t id) {
      if (id != 10 || t != T_LIST) {
        skip1(r, t);
        return;
      }
      const uint32_t et = r.u8();
      const int32_t n = r.size();
      if (et != T_STRUCT) {  // not a list of structs: thriftrw reads no events
        for (int32_t i = 0; i < n && r.ok(); i++) skip1(r, et);
        return;
      }
      // a repeated field 10 replaces the events read so far (FromWire assigns each occurrence)
      n_ev = n_kv = n_rp = 0;
      for (int32_t i = 0; i < n && r.ok(); i++) event(n_ev == 0);
    });
    if (r.ok() && n_ev == 0) r.err = CDR_DEC_NO_EVENTS;
  }
};

// the wave's blobs [wb0, wb0 + 64) into its LDS share when their bytes fit: returns the
// staged address range (lo, n; n = 0: nothing staged)
__device__ void stage_blobs(const Ctx& C, uint32_t n_blobs, uint32_t wb0, uint32_t lane, LDS3 uint4* dst,
                            uint64_t* lo_out, uint64_t* n_out) {
  *lo_out = *n_out = 0;
  if (wb0 >= n_blobs) return;
  const uint32_t wb1 = wb0 + 64 < n_blobs ? wb0 + 64 : n_blobs;
  const uint64_t base = (uint64_t)(uintptr_t)C.bytes;
  const uint64_t A = base + C.blob_off[wb0], E = base + C.blob_off[wb1];
  const uint64_t A16 = A & ~15ull;
  if (E <= A || E - A16 > CDR_INGEST_STAGE) return;
  const uint64_t lim = base + C.total;
  for (uint64_t i = (uint64_t)lane * 16u; A16 + i < E; i += 64u * 16u) {
    const uint64_t a = A16 + i;
    uint4 v;
    if (a >= base && a + 16 <= lim) {
      v = *reinterpret_cast<const uint4*>((uintptr_t)a);
    } else {  // the buffer's first / last partial 16 bytes
      uint32_t w[4] = {0, 0, 0, 0};
      for (uint32_t j = 0; j < 16; j++)
        if (a + j >= base && a + j < lim) w[j >> 2] |= (uint32_t)C.bytes[a + j - base] << (8 * (j & 3));
      v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    LDS3 uint32_t* d4 = (LDS3 uint32_t*)dst + (i >> 2);
    d4[0] = v.x;
    d4[1] = v.y;
    d4[2] = v.z;
    d4[3] = v.w;
  }
  *lo_out = A16;
  *n_out = E - A16;
}

template <int P>
__global__ __launch_bounds__(256) void k_blob(Ctx C, uint32_t n_blobs) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  LDS3 uint4* stage = (LDS3 uint4*)ing_lds + (uint64_t)wv * (CDR_INGEST_STAGE / 16);
  uint64_t s_lo, s_n;
  stage_blobs(C, n_blobs, b - lane, lane, stage, &s_lo, &s_n);
  // the wave's LDS writes complete before any of its lanes reads them (one wave: in order)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  uint64_t n_str = 0;
  uint32_t bad = 0;
  if (b < n_blobs && (P == COUNT || C.status[b] == CDR_DEC_OK)) {  // a failed blob contributes nothing
    Blob<P> x(C, b);
    x.r.sb = (const LDS3 uint8_t*)stage;
    x.r.s_lo = s_lo;
    x.r.s_n = s_n;
    x.run();
    if (P == COUNT) {
      C.counts[4ull * b] = x.r.ok() ? x.n_ev : 0u;
      C.counts[4ull * b + 1] = x.r.ok() ? x.n_kv : 0u;
      C.counts[4ull * b + 2] = x.r.ok() ? x.n_rp : 0u;
      C.counts[4ull * b + 3] = x.n_str;
      C.status[b] = x.r.err;
      n_str = x.n_str;
      bad = x.r.ok() ? 0u : 1u;
    }
  }
  if (P == COUNT) {  // totals: string fields (the table's size) and failed blobs, one atomic per wave
    for (int o = 32; o > 0; o >>= 1) {
      n_str += __shfl_down(n_str, o, 64);
      bad += __shfl_down(bad, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
      if (n_str) atomicAdd(C.totals, (unsigned long long)n_str);
      if (bad) atomicAdd(C.totals + 1, (unsigned long long)bad);
    }
  }
}

__global__ void k_seed(STab T, const uint8_t* bytes, const uint64_t* off, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 || i >= n) return;  // seed 0 is "" (handle 0, never in the table)
  const uint64_t a = off[i], len = off[i + 1] - a;
  if (len == 0) return;
  tab_insert(T, cdr_str_hash(bytes + a, len), a | SEED_REF, (uint32_t)len, i);
}

// seeds may collide with one another only by equal strings; the first claimant keeps its
// handle, the table's value is what lookups return

// the new strings' slots (key set, value UNASSIGNED), in two passes over the table and no
// shared counter: each of COLLECT_WG workgroups counts the new slots of its span of the
// table, the counts are scanned, and each workgroup writes its slots from its offset (one
// atomic per wavefront on a single counter took 8.9 ms: millions of new strings)
constexpr uint32_t COLLECT_WG = 2048;
__device__ __forceinline__ bool is_new(const STab& T, uint64_t i, unsigned long long* k) {
  *k = i <= T.mask ? T.key[i] : 0ull;
  return *k != 0ull && T.val[i] == UNASSIGNED;
}
__global__ __launch_bounds__(256) void k_collect_count(STab T, uint32_t* counts) {
  const uint64_t span = ((T.mask + 1 + COLLECT_WG - 1) / COLLECT_WG + 255) & ~255ull;
  const uint64_t lo = (uint64_t)blockIdx.x * span;
  uint32_t c = 0;
  for (uint64_t i = lo + threadIdx.x; i < lo + span && i <= T.mask; i += 256) {
    unsigned long long k;
    c += is_new(T, i, &k) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o, 64);
  __shared__ uint32_t part[4];
  if ((threadIdx.x & 63u) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}
__global__ __launch_bounds__(256) void k_collect_write(STab T, const uint32_t* offs, unsigned long long* keys,
                                                       uint64_t* idx) {
  const uint64_t span = ((T.mask + 1 + COLLECT_WG - 1) / COLLECT_WG + 255) & ~255ull;
  const uint64_t lo = (uint64_t)blockIdx.x * span;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  __shared__ uint32_t part[4];
  uint32_t base = offs[blockIdx.x];
  for (uint64_t c0 = lo; c0 < lo + span && c0 <= T.mask; c0 += 256) {
    const uint64_t i = c0 + threadIdx.x;
    unsigned long long k;
    const bool take = i < lo + span && is_new(T, i, &k);
    const uint64_t m = __builtin_amdgcn_ballot_w64(take);
    __syncthreads();  // the previous chunk's reads of part[] are done
    if (lane == 0) part[wv] = (uint32_t)__builtin_popcountll(m);
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t v = 0; v < 4; v++) {
      before += v < wv ? part[v] : 0u;
      total += part[v];
    }
    if (take) {
      const uint32_t j = base + before +
                         __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      keys[j] = k;
      idx[j] = i;
    }
    base += total;
  }
}

__global__ void k_rank(STab T, const uint64_t* idx_sorted, uint32_t n_new, uint32_t n_seeds, uint64_t* str_ref,
                       uint32_t* str_len) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_new) return;
  const uint64_t s = idx_sorted[j];
  const uint32_t h = n_seeds + j;
  T.val[s] = h;
  str_ref[h] = T.ref[s];
  str_len[h] = T.len[s];
}

__global__ void k_seed_refs(const uint64_t* off, uint32_t n, uint64_t* str_ref, uint32_t* str_len) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  str_ref[i] = off[i] | SEED_REF;
  str_len[i] = (uint32_t)(off[i + 1] - off[i]);
}

__global__ void k_domains(const uint32_t* map, uint32_t n_dom, uint32_t* dom_id, uint32_t n_seeds) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_dom) return;
  const uint32_t name = map[2 * i], id = map[2 * i + 1];
  if (name < n_seeds) dom_id[name] = id;
}

// per-blob counts (4 per blob) -> per-blob bases (3 per blob) via the scanned columns
__global__ void k_split(const uint32_t* counts, uint64_t* cols, uint32_t n_blobs) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_blobs) return;
  for (int c = 0; c < 3; c++) cols[(uint64_t)c * n_blobs + b] = counts[4ull * b + c];
}
__global__ void k_bases(const uint64_t* scanned, uint64_t* bases, uint32_t n_blobs) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_blobs) return;
  for (int c = 0; c < 3; c++) bases[3ull * b + c] = scanned[(uint64_t)c * n_blobs + b];
}
__global__ void k_entries(const uint32_t* entry_blob0, uint32_t n_entries, const uint64_t* scanned_ev,
                          const uint32_t* counts, uint32_t n_blobs, const int32_t* status, uint64_t* ev_off,
                          int32_t* entry_status) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w > n_entries) return;
  const uint32_t b0 = entry_blob0[w];
  ev_off[w] = b0 < n_blobs ? scanned_ev[b0]
                           : (n_blobs ? scanned_ev[n_blobs - 1] + counts[4ull * (n_blobs - 1)] : 0ull);
  if (w == n_entries) return;
  int32_t st = CDR_DEC_OK;
  for (uint32_t b = b0; b < entry_blob0[w + 1] && st == CDR_DEC_OK; b++) st = status[b];
  entry_status[w] = st;
}

template <class T>
int ws(cdr_ctx* c, int slot, uint64_t n, T** p) {
  *p = (T*)cdr_ws_get(c, slot, n * sizeof(T) + 8);
  return *p ? CDR_API_OK : CDR_API_ENOMEM;
}

}  // namespace

extern "C" int cdr_ingest_decode(cdr_ctx* ctx, const cdr_ingest_in* in, cdr_ingest_out* out, void* stream) {
  if (!ctx || !in || !out || !in->blob_off || !in->entry_blob0 || !in->seed_off || in->n_seeds == 0)
    return CDR_API_EINVAL;
  if (in->n_blobs && !in->blob_bytes) return CDR_API_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipSetDevice(cdr_ctx_device(ctx)));
  const uint32_t nb = in->n_blobs, ne = in->n_entries;
  *out = cdr_ingest_out{};
  int rc;
  uint32_t *counts, *misc;
  int32_t *status, *estatus;
  uint64_t *cols, *scanned, *bases, *ev_off;
  if ((rc = ws(ctx, WS_IN_COUNTS, 4ull * nb + 4, &counts)) || (rc = ws(ctx, WS_IN_STATUS, nb + 1ull, &status)) ||
      (rc = ws(ctx, WS_IN_ESTATUS, ne + 1ull, &estatus)) || (rc = ws(ctx, WS_IN_TMP, 3ull * nb + 3, &cols)) ||
      (rc = ws(ctx, WS_IN_SKEY2, 3ull * nb + 3, &scanned)) || (rc = ws(ctx, WS_IN_BASES, 3ull * nb + 3, &bases)) ||
      (rc = ws(ctx, WS_IN_EVOFF, ne + 1ull, &ev_off)) || (rc = ws(ctx, WS_IN_MISC, 16, &misc)))
    return rc;
  Ctx C{};
  C.bytes = in->blob_bytes;
  C.blob_off = in->blob_off;
  if (nb) {
    HIPCHK(hipMemcpyAsync(&C.total, in->blob_off + nb, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  C.counts = counts;
  C.status = status;
  C.n_seeds = in->n_seeds;
  const dim3 blk(256);
  auto grid = [](uint64_t n) { return dim3((uint32_t)((n + 255) / 256)); };
  // ---- pass 1: counts
  // misc (u32 words): [0] table overflow, [1] new strings; u64 words 2-3: string fields, failed blobs
  uint64_t* tot2 = reinterpret_cast<uint64_t*>(misc) + 2;
  HIPCHK(hipMemsetAsync(misc, 0, 64, st));
  C.totals = reinterpret_cast<unsigned long long*>(tot2);
  if (nb) hipLaunchKernelGGL(k_blob<COUNT>, grid(nb), blk, 4 * CDR_INGEST_STAGE, st, C, nb);
  HIPCHK(hipGetLastError());
  // string fields -> table capacity (2x, power of two)
  uint64_t htot[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(htot, tot2, 16, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const uint64_t n_str_fields = htot[0];
  out->n_bad_blobs = (uint32_t)htot[1];
  uint64_t cap = 1024;
  while (cap < 2 * (n_str_fields + in->n_seeds)) cap <<= 1;
  STab T{};
  T.mask = cap - 1;
  if ((rc = ws(ctx, WS_IN_TKEY, cap, (unsigned long long**)&T.key)) || (rc = ws(ctx, WS_IN_TVAL, cap, &T.val)) ||
      (rc = ws(ctx, WS_IN_TREF, cap, &T.ref)) || (rc = ws(ctx, WS_IN_TLEN, cap, &T.len)))
    return rc;
  T.overflow = misc;
  HIPCHK(hipMemsetAsync(T.key, 0, cap * 8, st));
  C.T = T;
  // ---- pass 2: seeds, then every string of the blobs; rank the new ones by hash
  hipLaunchKernelGGL(k_seed, grid(in->n_seeds), blk, 0, st, T, in->seed_bytes, in->seed_off, in->n_seeds);
  if (nb) hipLaunchKernelGGL(k_blob<INTERN>, grid(nb), blk, 4 * CDR_INGEST_STAGE, st, C, nb);
  HIPCHK(hipGetLastError());
  unsigned long long *k1, *k2;
  uint64_t *i1, *i2;
  if ((rc = ws(ctx, WS_IN_SKEY, n_str_fields + 1, &k1)) || (rc = ws(ctx, WS_IN_SIDX, n_str_fields + 1, &i1)) ||
      (rc = ws(ctx, WS_IN_SIDX2, n_str_fields + 1, &i2)) ||
      (rc = ws(ctx, WS_IN_STRREF, n_str_fields + in->n_seeds + 1, &out->str_ref)) ||
      (rc = ws(ctx, WS_IN_STRLEN, n_str_fields + in->n_seeds + 1, &out->str_len)))
    return rc;
  // the sort's second key buffer (afterwards the seed -> domain ID map)
  if ((rc = ws(ctx, WS_IN_DOM, (n_str_fields + 1) > in->n_seeds ? (n_str_fields + 1) * 2 : in->n_seeds * 2ull,
               &k2)))
    return rc;
  {  // the new strings: per-span counts, their scan, then the slots (k_collect_count / _write)
    uint32_t *ccount, *coffs;
    if ((rc = ws(ctx, WS_IN_GMAX, COLLECT_WG + 1ull, &ccount)) || (rc = ws(ctx, WS_IN_WBASE, COLLECT_WG + 1ull, &coffs)))
      return rc;
    HIPCHK(hipMemsetAsync(ccount + COLLECT_WG, 0, 4, st));
    hipLaunchKernelGGL(k_collect_count, dim3(COLLECT_WG), blk, 0, st, T, ccount);
    size_t tb = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, ccount, coffs, (int)(COLLECT_WG + 1), st));
    void* tmp = cdr_ws_get(ctx, WS_IN_CTMP, tb);
    if (!tmp) return CDR_API_ENOMEM;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, ccount, coffs, (int)(COLLECT_WG + 1), st));
    hipLaunchKernelGGL(k_collect_write, dim3(COLLECT_WG), blk, 0, st, T, coffs, k1, i1);
    HIPCHK(hipMemcpyAsync(misc + 1, coffs + COLLECT_WG, 4, hipMemcpyDeviceToDevice, st));
  }
  HIPCHK(hipGetLastError());
  uint32_t hm[2];
  HIPCHK(hipMemcpyAsync(hm, misc, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (hm[0]) return CDR_API_ENOMEM;  // table overflow: cannot happen at twice the fields
  const uint32_t n_new = hm[1];
  if (n_new) {
    hipcub::DoubleBuffer<unsigned long long> kb(k1, k2);
    hipcub::DoubleBuffer<uint64_t> vb(i1, i2);
    size_t tmp_bytes = 0;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kb, vb, (int)n_new, 0, 64, st));
    // the records' slot is free until pass 3: the sort's temporary storage
    void* sort_tmp = cdr_ws_get(ctx, WS_IN_EVENTS, tmp_bytes);
    if (!sort_tmp) return CDR_API_ENOMEM;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(sort_tmp, tmp_bytes, kb, vb, (int)n_new, 0, 64, st));
    hipLaunchKernelGGL(k_rank, grid(n_new), blk, 0, st, T, vb.Current(), n_new, in->n_seeds, out->str_ref,
                       out->str_len);
  }
  hipLaunchKernelGGL(k_seed_refs, grid(in->n_seeds), blk, 0, st, in->seed_off, in->n_seeds, out->str_ref,
                     out->str_len);
  HIPCHK(hipGetLastError());
  out->n_strings = in->n_seeds + n_new;
  // domain names -> IDs (by seed handle), in the sort's second key buffer (free again)
  uint32_t* dom_id = (uint32_t*)k2;
  HIPCHK(hipMemsetAsync(dom_id, 0xFF, in->n_seeds * 4ull, st));
  if (in->n_domains)
    hipLaunchKernelGGL(k_domains, grid(in->n_domains), blk, 0, st, in->domain_map, in->n_domains, dom_id,
                       in->n_seeds);
  HIPCHK(hipGetLastError());
  C.dom_id = dom_id;
  // ---- offsets: exclusive scans of the per-blob event / kv / reset-point counts
  if (nb) {
    hipLaunchKernelGGL(k_split, grid(nb), blk, 0, st, counts, cols, nb);
    size_t tmp_bytes = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cols, scanned, (int)nb, st));
    void* scan_tmp = cdr_ws_get(ctx, WS_IN_SKEY, tmp_bytes > (n_str_fields + 1) * 8 ? tmp_bytes : 8);
    if (!scan_tmp) return CDR_API_ENOMEM;
    for (int c = 0; c < 3; c++)
      HIPCHK(hipcub::DeviceScan::ExclusiveSum(scan_tmp, tmp_bytes, cols + (uint64_t)c * nb,
                                              scanned + (uint64_t)c * nb, (int)nb, st));
    hipLaunchKernelGGL(k_bases, grid(nb), blk, 0, st, scanned, bases, nb);
  }
  hipLaunchKernelGGL(k_entries, grid(ne + 1ull), blk, 0, st, in->entry_blob0, ne, scanned, counts, nb, status,
                     ev_off, estatus);
  HIPCHK(hipGetLastError());
  // totals
  uint64_t tot[3] = {0, 0, 0};
  if (nb) {
    uint64_t last[3];
    uint32_t lc[4];
    for (int c = 0; c < 3; c++)
      HIPCHK(hipMemcpyAsync(&last[c], scanned + (uint64_t)c * nb + (nb - 1), 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(lc, counts + 4ull * (nb - 1), 16, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (int c = 0; c < 3; c++) tot[c] = last[c] + lc[c];
  }
  if ((rc = ws(ctx, WS_IN_EVENTS, tot[0] + 1, &out->events)) || (rc = ws(ctx, WS_IN_KVS, tot[1] + 1, &out->kvs)) ||
      (rc = ws(ctx, WS_IN_RPS, tot[2] + 1, &out->rps)))
    return rc;
  // ---- pass 3: the records
  C.bases = bases;
  C.events = out->events;
  C.kvs = out->kvs;
  C.rps = out->rps;
  if (nb) hipLaunchKernelGGL(k_blob<FILL>, grid(nb), blk, 4 * CDR_INGEST_STAGE, st, C, nb);
  HIPCHK(hipGetLastError());
  out->ev_off = ev_off;
  out->blob_status = status;
  out->entry_status = estatus;
  out->n_events = tot[0];
  out->n_kvs = tot[1];
  out->n_rps = tot[2];
  HIPCHK(hipStreamSynchronize(st));
  return CDR_API_OK;
}

// ======================================================================== plan + pack
// cdr_plan_caps restated per entry on the device (host.cpp caps_one / task_caps): the
// live sets of the wave kernel's lane tables tracked up to CDR_WAVE_SLOTS + 1 keys (one
// past any bound a flag tests), the reset-point checksum and search-attribute key lists
// of the register-table envelope up to CDR_REG2_NRP / CDR_REG_NSA + 1.
#include "pack_event.h"

namespace {

template <int CAP>
struct Live {
  int64_t k[CAP];
  uint32_t n = 0, max = 0;
  bool over = false;
  __device__ void add(int64_t key, bool unique) {
    if (over) return;
    if (unique)
      for (uint32_t i = 0; i < n; i++)
        if (k[i] == key) return;
    if (n == CAP) {
      over = true;
      max = CAP + 1;
      return;
    }
    k[n++] = key;
    max = n > max ? n : max;
  }
  __device__ void del(int64_t key) {
    if (over) return;
    for (uint32_t i = 0; i < n; i++)
      if (k[i] == key) {
        k[i] = k[--n];
        return;
      }
  }
  __device__ bool has(int64_t key) const {
    for (uint32_t i = 0; i < n; i++)
      if (k[i] == key) return true;
    return false;
  }
  __device__ uint32_t size() const { return over ? CAP + 1 : n; }
};

__global__ __launch_bounds__(64) void k_caps(const cdr_event* events, const uint64_t* ev_off, const cdr_wf_desc* wfs,
                                              const cdr_kv* kvs, const cdr_reset_point* rps, uint32_t n_wfs,
                                              cdr_wf_caps* caps, uint64_t* arena_words) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n_wfs) return;
  const cdr_event* ev = events + ev_off[w];
  const uint64_t n = ev_off[w + 1] - ev_off[w];
  const uint32_t builder = wfs[w].builder;
  cdr_wf_caps c;
  {
    uint64_t* z = reinterpret_cast<uint64_t*>(&c);
    for (uint32_t i = 0; i < sizeof(cdr_wf_caps) / 8; i++) z[i] = 0;
  }
  bool fast = builder != CDR_BUILDER_2DC && n > 0 && ev[0].type == CDR_EV_WF_STARTED;
  bool have_ver = false;
  int64_t last_ver = 0;
  uint32_t vh = 0;
  int64_t live = 0, live_max = 0;
  Live<CDR_WAVE_SLOTS + 1> lv0, lv1, lv2, lv3;  // timers (timer id), children, cancels, signals
  bool reg = n > 0 && n < (1u << 20);
  int64_t last_id = 0;
  uint64_t call_start = 0;
  Live<CDR_REG2_NRP + 1> rp_cks;
  Live<CDR_REG_NSA + 1> sa_keys;
  uint32_t x = 0, t = 0;  // task bounds
  uint64_t aw = 0;
  for (uint64_t k = 0; k < n; k++) {
    const cdr_event& e = ev[k];
    const uint32_t type = e.type;
    if (k == 0 || (e.flags & CDR_EVF_BATCH_FIRST)) call_start = k;
    reg = reg && e.event_id > last_id && e.event_id < (1ll << 31) && e.version < (1ll << 31) &&
          k - call_start < 4096;
    last_id = e.event_id;
    if (type == CDR_EV_WF_STARTED) {  // a second Started resets the row lists
      const cdr_attr_wf_started& a = e.a.started;
      rp_cks = Live<CDR_REG2_NRP + 1>();
      sa_keys = Live<CDR_REG_NSA + 1>();
      if (a.flags & CDR_SF_HAS_RESET_POINTS)
        for (uint32_t q = 0; q < a.reset_points_len; q++) {
          const cdr_reset_point& p = rps[a.reset_points_off + q];
          rp_cks.add((p.flags & CDR_RP_HAS_CHECKSUM) ? p.binary_checksum : 0u, false);
        }
      if (a.flags & CDR_SF_HAS_SEARCH_ATTR)
        for (uint32_t q = 0; q < a.search_attr_len; q++) sa_keys.add(kvs[a.search_attr_off + q].key, false);
    } else if (type == CDR_EV_DT_COMPLETED && e.a.dt.binary_checksum) {
      rp_cks.add(e.a.dt.binary_checksum, true);
    } else if (type == CDR_EV_UPSERT_SA) {
      for (uint32_t q = 0; q < e.a.upsert.search_attr_len && sa_keys.size() <= CDR_REG_NSA; q++)
        sa_keys.add(kvs[e.a.upsert.search_attr_off + q].key, true);
    }
    if (type == CDR_EV_AT_SCHEDULED) {
      ++live;
      live_max = live > live_max ? live : live_max;
    }
    if (type == CDR_EV_AT_COMPLETED || type == CDR_EV_AT_FAILED || type == CDR_EV_AT_TIMED_OUT ||
        type == CDR_EV_AT_CANCELED)
      live = live > 0 ? live - 1 : 0;
    switch (type) {
      case CDR_EV_TIMER_STARTED: lv0.add(e.a.timer.timer_id, true); break;
      case CDR_EV_TIMER_FIRED: case CDR_EV_TIMER_CANCELED: lv0.del(e.a.timer.timer_id); break;
      case CDR_EV_CHILD_INITIATED: lv1.add(e.event_id, false); break;
      case CDR_EV_CHILD_START_FAILED: case CDR_EV_CHILD_COMPLETED: case CDR_EV_CHILD_FAILED:
      case CDR_EV_CHILD_CANCELED: case CDR_EV_CHILD_TIMED_OUT: case CDR_EV_CHILD_TERMINATED:
        lv1.del(e.a.ref.initiated_event_id);
        break;
      case CDR_EV_RCE_INITIATED: lv2.add(e.event_id, false); break;
      case CDR_EV_RCE_FAILED: case CDR_EV_EXT_CANCEL_REQUESTED: lv2.del(e.a.ref.initiated_event_id); break;
      case CDR_EV_SE_INITIATED: lv3.add(e.event_id, false); break;
      case CDR_EV_SE_FAILED: case CDR_EV_EXT_SIGNALED: lv3.del(e.a.ref.initiated_event_id); break;
      default: break;
    }
    fast = fast && type < 64 && (CDR_FAST_TYPES & (1ull << type)) && (k == 0 || type != CDR_EV_WF_STARTED);
    if (!have_ver || e.version > last_ver) {
      vh++;
      last_ver = e.version;
      have_ver = true;
    }
    switch (type) {
      case CDR_EV_WF_STARTED:
        c.rp_cap += e.a.started.reset_points_len;
        c.sa_cap += e.a.started.search_attr_len;
        x += 1;
        t += 2;
        break;
      case CDR_EV_DT_COMPLETED: if (e.a.dt.binary_checksum) c.rp_cap++; break;
      case CDR_EV_AT_SCHEDULED: c.act_cap++; break;
      case CDR_EV_TIMER_STARTED: c.timer_cap++; break;
      case CDR_EV_CHILD_INITIATED: c.child_cap++; break;
      case CDR_EV_RCE_INITIATED: c.cancel_cap++; break;
      case CDR_EV_SE_INITIATED: c.signal_cap++; break;
      case CDR_EV_UPSERT_SA: c.sa_cap += e.a.upsert.search_attr_len; break;
      default: break;
    }
    switch (type) {  // task_caps (host.cpp): transfer / timer tasks an event can append
      case CDR_EV_DT_SCHEDULED: case CDR_EV_DT_TIMED_OUT: case CDR_EV_DT_FAILED: case CDR_EV_CHILD_INITIATED:
      case CDR_EV_RCE_INITIATED: case CDR_EV_SE_INITIATED: case CDR_EV_UPSERT_SA:
        x += 1;
        break;
      case CDR_EV_AT_SCHEDULED: case CDR_EV_WF_COMPLETED: case CDR_EV_WF_FAILED: case CDR_EV_WF_TIMED_OUT:
      case CDR_EV_WF_CANCELED: case CDR_EV_WF_TERMINATED: case CDR_EV_WF_CONTINUED_AS_NEW:
        x += 1;
        t += 1;
        break;
      case CDR_EV_DT_STARTED: case CDR_EV_AT_STARTED: case CDR_EV_AT_COMPLETED: case CDR_EV_AT_FAILED:
      case CDR_EV_AT_TIMED_OUT: case CDR_EV_AT_CANCELED: case CDR_EV_TIMER_STARTED: case CDR_EV_TIMER_FIRED:
      case CDR_EV_TIMER_CANCELED:
        t += 1;
        break;
      default: break;
    }
    aw += cdr_arena_words_for(type);
  }
  c.vh_cap = vh;
  c.act_live = (uint32_t)live_max;
  c.timer_live = lv0.over ? c.timer_cap : lv0.max;  // past the tracked bound: every TimerStarted
  {  // the lane planner's ordering key and the pending tables' row capacities (host.cpp caps_one)
    auto sat = [](uint32_t v, uint32_t bits) { return v < (1u << bits) ? v : (1u << bits) - 1u; };
    c.order_key = sat(c.act_cap, 10) << 22 | sat(c.timer_cap, 11) << 11 |
                  sat(c.child_cap + c.cancel_cap + c.signal_cap, 11);
    c.act_cap = (uint32_t)live_max;
    c.timer_cap = lv0.over ? c.timer_cap : lv0.max;
    c.child_cap = lv1.over ? c.child_cap : lv1.max;
    c.cancel_cap = lv2.over ? c.cancel_cap : lv2.max;
    c.signal_cap = lv3.over ? c.signal_cap : lv3.max;
  }
  c.flags = (fast && live_max <= 1) ? CDR_CAP_FAST : 0u;
  const uint32_t W = CDR_WAVE_SLOTS;
  if (!(c.flags & CDR_CAP_FAST) && live_max <= (int64_t)W && lv0.max <= W && lv1.max <= W && lv2.max <= W &&
      lv3.max <= W)
    c.flags |= CDR_CAP_WAVE;
  if ((c.flags & CDR_CAP_WAVE) && live_max <= (int64_t)CDR_LANE_MAX_ACT && lv0.max <= CDR_LANE_MAX_TIMERS &&
      lv1.max + lv2.max + lv3.max <= CDR_LANE_MAX_EXT && n <= CDR_LANE_MAX_LEN)
    c.flags |= CDR_CAP_LANE;
  reg = reg && !(c.flags & CDR_CAP_FAST) && lv0.max <= CDR_REG_NT && lv1.max <= CDR_REG_NX &&
        lv2.max <= CDR_REG_NX && lv3.max <= CDR_REG_NX && sa_keys.size() <= CDR_REG_NSA;
  if (reg && live_max <= (int64_t)CDR_REG_NA && rp_cks.size() <= CDR_REG_NRP) c.flags |= CDR_CAP_REG;
  else if (reg && live_max <= (int64_t)CDR_REG2_NA && rp_cks.size() <= CDR_REG2_NRP) c.flags |= CDR_CAP_REG2;
  if ((c.flags & CDR_CAP_REG) && live_max <= (int64_t)CDR_REG0_NA && lv0.max <= CDR_REG0_NT &&
      lv1.max <= CDR_REG0_NX && lv2.max <= CDR_REG0_NX && lv3.max <= CDR_REG0_NX)
    c.flags |= CDR_CAP_REG0;
  c.xfer_cap = x + 1;  // + refreshTasks' UpsertWorkflowSearchAttributes task
  c.ttask_cap = t;
  caps[w] = c;
  arena_words[w] = aw;
}

// one thread per lane of a lane slice, one per wave slice (its events in row-major order)
__global__ __launch_bounds__(64) void k_pack(const cdr_event* events, const cdr_wf_desc* wfs, const uint64_t* abase,
                                              const int32_t* lane_wf, const uint32_t* slice_len,
                                              const uint64_t* slice_row0, const uint32_t* slice_flags,
                                              uint8_t* slab, uint64_t* arena) {
  const uint32_t s = blockIdx.x, l = threadIdx.x;
  const uint64_t row0 = slice_row0[s];
  const uint32_t len = slice_len[s];
  uint8_t* blk0 = slab + row0 * CDR_ROW_BYTES;
  if (slice_flags[s] & CDR_SLICE_WAVE) {
    const int32_t w = lane_wf[(uint64_t)s * CDR_SLICE_WIDTH];
    const cdr_event* ev = events + wfs[w].ev_off;
    const uint64_t n = wfs[w].ev_len;
    // one walk in event order (arena positions are the prefix of the entry's records)
    if (l == 0) {
      uint64_t apos = abase[w];
      for (uint64_t k = 0; k < (uint64_t)len * CDR_SLICE_WIDTH; k++)
        cdr_put_event(blk0 + (k / CDR_SLICE_WIDTH) * CDR_ROW_BYTES, (uint32_t)(k % CDR_SLICE_WIDTH),
                      k < n ? ev + k : nullptr, k == 0, &apos, arena);
    }
    return;
  }
  const int32_t w = lane_wf[(uint64_t)s * CDR_SLICE_WIDTH + l];
  uint64_t apos = w >= 0 ? abase[w] : 0;
  const cdr_event* ev = w >= 0 ? events + wfs[w].ev_off : nullptr;
  const uint64_t n = w >= 0 ? wfs[w].ev_len : 0;
  for (uint32_t k = 0; k < len; k++)
    cdr_put_event(blk0 + (uint64_t)k * CDR_ROW_BYTES, l, k < n ? ev + k : nullptr, k == 0, &apos, arena);
}

}  // namespace

extern "C" int cdr_ingest_plan(cdr_ctx* ctx, const cdr_ingest_out* dec, const cdr_batch* meta, uint32_t plan_mode,
                               cdr_dev_batch* db, cdr_wf_caps* caps, cdr_totals* totals, void* stream) {
  if (!ctx || !dec || !meta || !db || !caps || !totals || (meta->n_wfs && !meta->wfs)) return CDR_API_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipSetDevice(cdr_ctx_device(ctx)));
  const uint32_t n = meta->n_wfs;
  int rc;
  // ---- entries with the decode's event ranges
  std::vector<uint64_t> off(n + 1ull);
  HIPCHK(hipMemcpyAsync(off.data(), dec->ev_off, (n + 1ull) * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  std::vector<cdr_wf_desc> wfs(meta->wfs, meta->wfs + n);
  for (uint32_t w = 0; w < n; w++) {
    wfs[w].ev_off = off[w];
    wfs[w].ev_len = off[w + 1] - off[w];
  }
  cdr_wf_desc* d_wfs;
  cdr_wf_caps* d_caps;
  uint64_t *d_aw, *d_abase;
  if ((rc = ws(ctx, WS_PL_WFS, n, &d_wfs)) || (rc = ws(ctx, WS_PL_CAPS, n, &d_caps)) ||
      (rc = ws(ctx, WS_PL_AWORDS, n, &d_aw)) || (rc = ws(ctx, WS_PL_ABASE, n + 1ull, &d_abase)))
    return rc;
  if (n) HIPCHK(hipMemcpyAsync(d_wfs, wfs.data(), n * sizeof(cdr_wf_desc), hipMemcpyHostToDevice, st));
  // ---- capacities and eligibility, one lane per entry
  if (n)
    hipLaunchKernelGGL(k_caps, dim3((n + 63) / 64), dim3(64), 0, st, dec->events, dec->ev_off, d_wfs, dec->kvs,
                       dec->rps, n, d_caps, d_aw);
  HIPCHK(hipGetLastError());
  std::vector<uint64_t> aw(n);
  if (n) {
    HIPCHK(hipMemcpyAsync(caps, d_caps, n * sizeof(cdr_wf_caps), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(aw.data(), d_aw, n * 8ull, hipMemcpyDeviceToHost, st));
  }
  HIPCHK(hipStreamSynchronize(st));
  // ---- offsets (cdr_plan_caps's running sums) and arena bases, on the host
  cdr_totals t{};
  std::vector<uint64_t> abase(n + 1ull, 0);
  for (uint32_t w = 0; w < n; w++) {
    cdr_wf_caps& c = caps[w];
    c.xfer_off = t.xfer;
    t.xfer += c.xfer_cap;
    c.ttask_off = t.ttask;
    t.ttask += c.ttask_cap;
    c.act_off = t.act;
    t.act += c.act_cap;
    c.timer_off = t.timer;
    t.timer += c.timer_cap;
    c.child_off = t.child;
    t.child += c.child_cap;
    c.cancel_off = t.cancel;
    t.cancel += c.cancel_cap;
    c.signal_off = t.signal;
    t.signal += c.signal_cap;
    c.vh_off = t.vh;
    t.vh += c.vh_cap;
    c.rp_off = t.rp;
    t.rp += c.rp_cap;
    c.sa_off = t.sa;
    t.sa += c.sa_cap;
    abase[w + 1] = abase[w] + aw[w];
  }
  *totals = t;
  if (abase[n] >= (1ull << 32)) return CDR_API_EINVAL;  // u32 arena offsets (cdr.h)
  // ---- the slice plan (host, per-entry records only)
  uint32_t ns = 0, n_wave = 0;
  uint64_t rows = 0;
  cdr_internal::plan_vecs pv;  // one planning pass (the C ABI's size query + fill would plan twice)
  if ((rc = cdr_internal::plan_slices_vec(wfs.data(), caps, n, plan_mode, pv, &ns, &rows, &n_wave))) return rc;
  std::vector<int32_t>& lane = pv.lane_wf;
  std::vector<uint32_t>& slen = pv.slice_len;
  std::vector<uint32_t>& sflags = pv.slice_flags;
  std::vector<uint64_t>& row0 = pv.slice_row0;
  std::vector<uint32_t> sc_act(ns), sc_tim(ns);
  std::vector<uint64_t> sc_off(ns);
  uint64_t sc_words = 0;
  uint32_t n_fast = 0;
  if ((rc = cdr_plan_scratch(caps, lane.data(), ns, sc_off.data(), sc_act.data(), sc_tim.data(), sflags.data(),
                             &sc_words, &n_fast)))
    return rc;
  int32_t* d_lane;
  uint32_t *d_slen, *d_sflags, *d_scact, *d_sctim;
  uint64_t *d_row0, *d_scoff, *d_scratch, *d_arena;
  uint8_t* d_slab;
  if ((rc = ws(ctx, WS_PL_LANE, lane.size(), &d_lane)) || (rc = ws(ctx, WS_PL_SLEN, ns, &d_slen)) ||
      (rc = ws(ctx, WS_PL_SFLAGS, ns, &d_sflags)) || (rc = ws(ctx, WS_PL_SCACT, ns, &d_scact)) ||
      (rc = ws(ctx, WS_PL_SCTIM, ns, &d_sctim)) || (rc = ws(ctx, WS_PL_ROW0, ns, &d_row0)) ||
      (rc = ws(ctx, WS_PL_SCOFF, ns, &d_scoff)) || (rc = ws(ctx, WS_PL_SCRATCH, sc_words, &d_scratch)) ||
      (rc = ws(ctx, WS_PL_ARENA, abase[n] + 1, &d_arena)) ||
      (rc = ws(ctx, WS_PL_SLAB, rows * (uint64_t)CDR_ROW_BYTES, &d_slab)))
    return rc;
  auto h2d = [&](void* d, const void* h, uint64_t bytes) -> int {
    if (bytes) HIPCHK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st));
    return CDR_API_OK;
  };
  if ((rc = h2d(d_lane, lane.data(), lane.size() * 4ull)) || (rc = h2d(d_slen, slen.data(), ns * 4ull)) ||
      (rc = h2d(d_sflags, sflags.data(), ns * 4ull)) || (rc = h2d(d_scact, sc_act.data(), ns * 4ull)) ||
      (rc = h2d(d_sctim, sc_tim.data(), ns * 4ull)) || (rc = h2d(d_row0, row0.data(), ns * 8ull)) ||
      (rc = h2d(d_scoff, sc_off.data(), ns * 8ull)) || (rc = h2d(d_abase, abase.data(), (n + 1ull) * 8)) ||
      (rc = h2d(d_caps, caps, n * sizeof(cdr_wf_caps))))
    return rc;
  HIPCHK(hipMemsetAsync(d_scratch, 0, sc_words * 8 + 8, st));
  // ---- the slab and the arena, on the device
  if (ns)
    hipLaunchKernelGGL(k_pack, dim3(ns), dim3(CDR_SLICE_WIDTH), 0, st, dec->events, d_wfs, d_abase, d_lane, d_slen,
                       d_row0, d_sflags, d_slab, d_arena);
  HIPCHK(hipGetLastError());
  cdr_dev_batch b{};
  b.ev.n_slices = ns;
  b.ev.n_rows = rows;
  b.ev.arena_words = abase[n];
  b.ev.slice_row0 = d_row0;
  b.ev.slice_len = d_slen;
  b.ev.lane_wf = d_lane;
  b.ev.slab = d_slab;
  b.ev.arena = d_arena;
  b.ev.slice_scratch_off = d_scoff;
  b.ev.slice_act_slots = d_scact;
  b.ev.slice_tim_slots = d_sctim;
  b.ev.slice_flags = d_sflags;
  b.scratch = d_scratch;
  b.wfs = d_wfs;
  b.caps = d_caps;
  b.kvs = dec->kvs;
  b.rps = dec->rps;
  b.n_wfs = n;
  b.empty_uuid = meta->empty_uuid;
  for (uint32_t i = 0; i < ns; i++) {
    b.max_act_slots = sc_act[i] > b.max_act_slots ? sc_act[i] : b.max_act_slots;
    b.max_tim_slots = sc_tim[i] > b.max_tim_slots ? sc_tim[i] : b.max_tim_slots;
    b.n_reg_slices += (sflags[i] & CDR_SLICE_REG) ? 1u : 0u;
    b.n_reg2_slices += (sflags[i] & CDR_SLICE_REG2) ? 1u : 0u;
    b.n_reg0_slices += (sflags[i] & CDR_SLICE_REG0) ? 1u : 0u;
    b.n_par_slices += (sflags[i] & CDR_SLICE_PAR) ? 1u : 0u;
  }
  cdr_plan_class_ranges(sflags.data(), ns, b.class_lo, b.class_hi);
  b.n_fast_slices = n_fast;
  b.n_wave_slices = n_wave;
  b.cluster = meta->cluster;
  b.now_ns = meta->now_ns;
  b.uuid_seed = meta->uuid_seed;
  b.carry = nullptr;
  // class-sorted blocks of the register-table slices (k_replay_cls), in the plan's own
  // workspace slots (a later host-buffer call on the context must not overwrite them);
  // built when the context asks the packers for them (CDR_CLS_BUILD / CDR_CLS_ALONE, as
  // cdr_replay_batch)
  b.cls_slab = nullptr;
  b.cls_row0 = nullptr;
  b.cls_rows = nullptr;
  if (ctx->cls >= CDR_CLS_ALONE && b.n_reg_slices + b.n_reg2_slices + b.n_reg0_slices + b.n_par_slices > 0) {
    uint32_t* crows = (uint32_t*)cdr_ws_get(ctx, WS_PL_CLS_ROWS, ns * 16ull);
    uint64_t* crow0 = (uint64_t*)cdr_ws_get(ctx, WS_PL_CLS_ROW0, (ns + 1) * 8ull);
    if (!crows || !crow0) return CDR_API_ENOMEM;
    int rc = cdr_cls_plan_async(ctx, &b, crows, crow0, st);
    if (rc != CDR_API_OK) return rc;
    uint64_t total = 0;
    HIPCHK(hipMemcpyAsync(&total, crow0 + ns, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    uint8_t* cslab = (uint8_t*)cdr_ws_get(ctx, WS_PL_CLS_SLAB, total ? total * CDR_ROW_BYTES : 8);
    if (!cslab) return CDR_API_ENOMEM;
    b.cls_slab = cslab;
    b.cls_row0 = crow0;
    b.cls_rows = crows;
    rc = cdr_cls_pack_async(ctx, &b, st);
    if (rc != CDR_API_OK) return rc;
  }
  *db = b;
  HIPCHK(hipStreamSynchronize(st));
  return CDR_API_OK;
}
