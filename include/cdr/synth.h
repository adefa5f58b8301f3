/*
 * cdr/synth.h — deterministic synthetic workflow histories (libcdr test/bench
 * utility, not part of the replay path).  Shapes: SURVEY §8(d) configs 1-5 after
 * canary/echo.go:55-79 and common/testing/history_event_util.go:51-960.
 */
#ifndef CDR_SYNTH_H
#define CDR_SYNTH_H
#include "cdr/cdr.h"
#ifdef __cplusplus
extern "C" {
#endif
typedef struct cdr_synth_params {
  int32_t config;       /* 1..5 = SURVEY §8(d) configs; 0 = mixed random walk (tests) */
  uint32_t n_wfs;       /* top-level workflows (continue-as-new runs are added) */
  uint64_t seed;
  uint32_t target_len;  /* median history length (0 = config default) */
  uint32_t max_len;     /* cap (0 = 204800, service.go:264) */
  double error_rate;    /* fraction of workflows with one injected fault */
  int32_t builder;      /* -1 = config default, else cdr_builder */
  int32_t rebuild;      /* set expected_next_event_id (nDCStateRebuilder check) */
  uint32_t fault_kinds; /* bit i allows injected fault kind i (synth.cpp inject_fault); 0 = all */
  uint32_t plan_mode;   /* CDR_PLAN_* of the sliced layout (cdr_plan_slices_ex) */
  const uint32_t* index_map; /* optional [n_wfs]: global index of each generated workflow */
  /* config 5 forks: every workflow's history forks at a batch boundary
   * F (a DeepCopy of the generator with a version bump, nDC_integration_test.go:224-308)
   * into two continuations.  Which part a batch holds: */
  uint32_t ndc_part;  /* CDR_SYNTH_PART_* */
  /* load-balance stress (configs[3]: "skewed lengths up to the history count limit"): if
   * nonzero, every workflow whose global index is long_stride / 2 modulo long_stride is
   * generated at the history count limit (max_len) instead of its drawn length */
  uint32_t long_stride;
} cdr_synth_params;
#define CDR_SYNTH_PART_BASE 0    /* the base branch, whole (default) */
#define CDR_SYNTH_PART_REBUILD 1 /* the base branch's events 1..F (the rebuild path; expected next = F+1) */
#define CDR_SYNTH_PART_FORK_A 2  /* fork A's events F+1.. (version above every base version) */
#define CDR_SYNTH_PART_FORK_B 3  /* fork B's events F+1.. (above fork A's version, or between the
                                    base's version at F and fork A's: half the workflows each) */
typedef struct cdr_synth_sizes {
  uint64_t n_events;
  uint32_t n_entries, _pad;
  uint64_t n_kvs, n_rps, arena_words;
} cdr_synth_sizes;
typedef struct cdr_synth_plan_info {
  uint64_t n_events;
  uint32_t n_entries, n_slices;
  uint64_t n_rows, arena_words, n_kvs, n_rps;
  cdr_totals totals;
} cdr_synth_plan_info;
int cdr_synth_size(const cdr_synth_params* p, cdr_synth_sizes* out);
int cdr_synth_fill(const cdr_synth_params* p, cdr_event* ev, cdr_wf_desc* wfs, cdr_kv* kvs, cdr_reset_point* rps,
                   cdr_batch* b);
int cdr_synth_sliced_plan(const cdr_synth_params* p, cdr_synth_plan_info* info);
int cdr_synth_sliced_fill(const cdr_synth_params* p, cdr_slices* o, cdr_wf_desc* wfs, cdr_wf_caps* caps,
                          cdr_kv* kvs, cdr_reset_point* rps, cdr_batch* meta, int threads);
/* planned event count of workflows 0..n-1 (the walk's target length, drawn without
 * generating the histories): weights of the bench's shard->GPU assignment */
int cdr_synth_weights(const cdr_synth_params* p, uint64_t n, uint32_t* out);
/* The replication tasks that deliver fork A (fork = 0) or B (fork = 1) of every
 * config-5 workflow of `p`: task w's incoming VersionHistory (the base's items up to F
 * then the fork's) at items[w * items_cap ...], first / last event, version and the
 * ForkHistoryBranch token of the branch it would create.  -EINVAL if an item list
 * exceeds items_cap. */
int cdr_synth_ndc_tasks(const cdr_synth_params* p, int fork, cdr_ndc_task* tasks, cdr_vh_item* items,
                        uint32_t items_cap);
/* history shard of synthetic workflow ids "wf-<i>", i in [0, n): farmhash
 * Fingerprint32 % num_shards (common/util.go:249-252) */
int cdr_synth_shards(uint64_t n, int32_t num_shards, int32_t* out);
/* Synthetic persisted histories (cadence_amd/csrc/thrift_enc.cpp): every entry of `b`
 * written as the reference stores it — one blob per applyEvents call, preambleVersion0
 * (0x59) + thriftrw shared.History{10: list<HistoryEvent>} — the input of
 * cdr_ingest_decode (cdr/ingest.h).  Handle h is the string str_bytes[str_off[h],
 * str_off[h+1]) for h < n_str, else "h%08x"; a parent domain is named "dn:" + its ID's
 * string.  Sizes only when blob_bytes is NULL (*n_bytes, *n_blobs); otherwise
 * blob_off[n_blobs + 1] and entry_blob0[n_wfs + 1] are filled too. */
int cdr_synth_encode_history(const cdr_batch* b, const uint8_t* str_bytes, const uint64_t* str_off,
                             uint32_t n_str, uint8_t* blob_bytes, uint64_t* blob_off, uint32_t* entry_blob0,
                             uint64_t* n_bytes, uint32_t* n_blobs, int threads);

#ifdef __cplusplus
}
#endif
#endif
