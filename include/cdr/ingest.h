/*
 * cdr/ingest.h — on-device decode of persisted histories.
 *
 * The reference reads a workflow's history as history-node rows, one DataBlob per
 * applyEvents batch, each `preambleVersion0` (0x59) followed by a thriftrw
 * binary-protocol shared.History{10: list<HistoryEvent>}
 * (common/persistence/serializer.go:198-250 thriftrwDecode, common/codec/
 * version0Thriftrw.go:45-84 Decode, idl/github.com/uber/cadence/shared.thrift:868-920).
 * cdr_ingest_decode decodes those blobs on the GPU straight into the replay's
 * input records (cdr_event, cdr_kv, cdr_reset_point; schema.h), one lane per blob, so
 * the host never touches an event.
 *
 * Strings.  Every string / binary the replay keeps becomes a u32 handle of the batch's
 * string table.  The caller seeds the table with the strings it already holds (handle
 * i = seed i: its cdr_wf_desc fields, "emptyUuid", domain names and IDs); every other
 * distinct string of the blobs gets handle n_seeds + r, r = its rank among the new
 * strings ordered by their 64-bit hash (cdr_str_hash) — deterministic, independent of
 * decode order.  Strings are identified by that hash (two different strings with equal
 * 64-bit hashes would share a handle).  The empty string is handle 0 (= an absent
 * optional string: Go's GetX() of nil is "").  Values the record form keeps as one
 * handle although the wire value is a structure — Memo, RetryPolicy.nonRetriableErrorReasons
 * (non-empty lists only) — are interned by the bytes of their thrift value.
 *
 * Domains.  The domain cache lookups the replay needs (the parent domain of
 * WorkflowExecutionStarted, the target domain of child / signal / cancel initiations)
 * are resolved against domain_map: pairs (name handle, ID handle) among the seeds; a
 * name not in the map sets CDR_SF_PARENT_DOMAIN_MISSING / CDR_XF_DOMAIN_MISSING.
 *
 * Wire rules (go.uber.org/thriftrw protocol.Binary + generated FromWire): fields in any
 * order, unknown fields skipped, a field of an unexpected wire type skipped, a missing
 * eventType is EventTypeWorkflowExecutionStarted (0), a History whose field 10 is not a
 * list of structs has no events.  The attribute struct present decides the union member
 * (schema.h cdr_event).  Decode failures (missing / wrong preamble, truncated value,
 * nesting deeper than CDR_THRIFT_MAX_DEPTH) are reported per blob and per entry.
 */
#ifndef CDR_INGEST_H
#define CDR_INGEST_H

#include "cdr/cdr.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CDR_THRIFT_PREAMBLE_V0 0x59u
#define CDR_THRIFT_MAX_DEPTH 16
/* per-blob / per-entry decode status (0 = decoded) */
#define CDR_DEC_OK 0
#define CDR_DEC_MISSING_VERSION 1 /* empty blob (codec MissingBinaryEncodingVersion) */
#define CDR_DEC_INVALID_VERSION 2 /* first byte != 0x59 (InvalidBinaryEncodingVersion) */
#define CDR_DEC_TRUNCATED 3       /* a value runs past the blob */
#define CDR_DEC_DEPTH 4           /* nesting deeper than CDR_THRIFT_MAX_DEPTH */
#define CDR_DEC_NO_EVENTS 5       /* a history node without events (applyEvents of an empty history) */
#define CDR_DEC_BAD_SIZE 6        /* negative length / element count */
#define CDR_DEC_BAD_TYPE 7        /* a wire type the binary protocol does not define */

/* 64-bit string identity of the string table (FNV-1a over the bytes, then cdr_mix64
 * with the length); 0 is reserved for "no string" */
CDR_HD uint64_t cdr_str_hash(const uint8_t* p, uint64_t n) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (uint64_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001B3ull;
  h = cdr_mix64(h ^ (n * 0x9E3779B97F4A7C15ull));
  return h ? h : 1u;
}

typedef struct cdr_ingest_in { /* device pointers */
  const uint8_t* blob_bytes;   /* every blob, concatenated */
  const uint64_t* blob_off;    /* [n_blobs + 1]: blob i = blob_bytes[blob_off[i], blob_off[i+1]) */
  const uint32_t* entry_blob0; /* [n_entries + 1]: entry w's calls = blobs [entry_blob0[w], entry_blob0[w+1]) */
  const uint8_t* seed_bytes;   /* the caller's strings: seed i = seed_bytes[seed_off[i], seed_off[i+1]) */
  const uint64_t* seed_off;    /* [n_seeds + 1]; seed 0 must be "" */
  const uint32_t* domain_map;  /* [2 * n_domains]: (name handle, ID handle) */
  uint32_t n_blobs, n_entries, n_seeds, n_domains;
} cdr_ingest_in;

typedef struct cdr_ingest_out { /* device buffers owned by the context, valid until its next ingest */
  cdr_event* events;       /* [n_events]: entry w's events at [ev_off[w], ev_off[w+1]) */
  cdr_kv* kvs;             /* [n_kvs] */
  cdr_reset_point* rps;    /* [n_rps] */
  uint64_t* ev_off;        /* [n_entries + 1] */
  int32_t* blob_status;    /* [n_blobs] CDR_DEC_* */
  int32_t* entry_status;   /* [n_entries]: the first failing blob's status */
  uint64_t* str_ref;       /* [n_strings]: handle h's bytes: (offset into blob_bytes) or (offset into seed_bytes | 1 << 63) */
  uint32_t* str_len;       /* [n_strings] */
  uint64_t n_events, n_kvs, n_rps;
  uint32_t n_strings, n_bad_blobs;
} cdr_ingest_out;

/* Decode every blob on `stream`: three lane-per-blob passes over the bytes (count;
 * intern the strings into a device hash table; fill the records), with the string
 * ranking and the offset scans between them on the device.  Synchronous (the totals
 * size the outputs).  `out` receives device pointers into the context's workspace. */
int cdr_ingest_decode(cdr_ctx* ctx, const cdr_ingest_in* in, cdr_ingest_out* out, void* stream);

/* Plan and pack a decoded batch for the replay, on the device: each entry's capacities
 * and kernel eligibility (cdr_plan_caps restated, one lane per entry: k_caps), the slice
 * plan on the host from those per-entry records alone (cdr_plan_slices_ex,
 * cdr_plan_scratch), then the SELL-64 slab and attribute arena (k_pack, the packer's
 * cdr_put_event per cell).  `meta` gives the entries (meta->wfs[w], n_wfs = the decode's
 * entries; ev_off / ev_len are taken from the decode), cluster, now_ns, uuid_seed and
 * empty_uuid; its events / kvs / rps are not read.  Fills *db with device pointers into
 * the context's workspace (valid until its next ingest) and the host arrays caps[n_wfs]
 * (offsets set) and *totals, which size the replay's outputs.  Entries whose decode
 * failed replay as empty histories (CDR_E_HISTORY_EMPTY): check entry_status.  Not
 * restated from the host planner: the continue-as-new run-id check and the
 * CDR_LANE_MAX tuning override.  Synchronous on `stream`. */
int cdr_ingest_plan(cdr_ctx* ctx, const cdr_ingest_out* dec, const cdr_batch* meta, uint32_t plan_mode,
                    cdr_dev_batch* db, cdr_wf_caps* caps, cdr_totals* totals, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CDR_INGEST_H */
