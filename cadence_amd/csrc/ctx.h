// ctx.h — the replay context (cdr_ctx) shared by replay.hip and api.hip.
//
// One context per device and caller thread / stream (the analogue of one
// stateBuilderProvider, historyReplicator.go:54): kernel-routing switches, timing
// events, the side stream of the wave kernel, and the persistent workspaces of the
// host-buffer entry points (cdr_replay_batch / cdr_rebuild_batch / cdr_replay_one):
// device buffers that only grow, so a warmed-up context replays without hipMalloc,
// and the host-side plan / pack / output buffers of cdr_replay_one.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "cdr/cdr.h"

// k_tasks_merge's occupancy attribute (A/B builds: tools/build_variant.sh -DCDR_MERGE_ATTR=...)
#ifndef CDR_MERGE_ATTR
#define CDR_MERGE_ATTR
#endif
#ifndef CDR_MERGE_D2
#define CDR_MERGE_D2 0 /* 1: each list keeps its head and one record after it (not two) */
#endif

// device workspace slots of the host-buffer pipeline (api.hip replay_host)
enum cdr_ws_slot {
  WS_ROW0, WS_SLEN, WS_LANE, WS_SLAB, WS_ARENA, WS_SFLAGS, WS_SC_OFF, WS_SC_ACT, WS_SC_TIM, WS_SCRATCH,
  WS_WFS, WS_CAPS, WS_KVS, WS_RPS,
  WS_CY_SRC, WS_CY_CAPS, WS_CY_RESULT, WS_CY_EXEC, WS_CY_REPL, WS_CY_VH, WS_CY_ACT, WS_CY_TIMER, WS_CY_CHILD,
  WS_CY_CANCEL, WS_CY_SIGNAL, WS_CY_RP, WS_CY_SA, WS_CY_DESC, WS_CY_INMEM,
  WS_O_RESULT, WS_O_EXEC, WS_O_REPL, WS_O_VH, WS_O_ACT, WS_O_TIMER, WS_O_CHILD, WS_O_CANCEL, WS_O_SIGNAL,
  WS_O_RP, WS_O_SA, WS_O_XFER, WS_O_TTASK, WS_O_NTASKS, WS_O_LD,
  WS_CLS_ROWS, WS_CLS_ROW0, WS_CLS_SLAB,  // class-sorted blocks (cdr_cls_plan_async / cdr_cls_pack_async)
  // cdr_ingest_decode (ingest.hip)
  WS_IN_COUNTS, WS_IN_BASES, WS_IN_STATUS, WS_IN_ESTATUS, WS_IN_EVOFF, WS_IN_TKEY, WS_IN_TVAL, WS_IN_TREF,
  WS_IN_TLEN, WS_IN_SKEY, WS_IN_SIDX, WS_IN_SKEY2, WS_IN_SIDX2, WS_IN_TMP, WS_IN_DOM, WS_IN_EVENTS, WS_IN_KVS,
  WS_IN_RPS, WS_IN_STRREF, WS_IN_STRLEN, WS_IN_MISC, WS_IN_GMAX, WS_IN_WBASE, WS_IN_CTMP,
  // cdr_ingest_plan (ingest.hip)
  WS_PL_CAPS, WS_PL_AWORDS, WS_PL_ABASE, WS_PL_WFS, WS_PL_LANE, WS_PL_SLEN, WS_PL_ROW0, WS_PL_SFLAGS, WS_PL_SCOFF,
  WS_PL_SCACT, WS_PL_SCTIM, WS_PL_SCRATCH, WS_PL_SLAB, WS_PL_ARENA,
  WS_PL_CLS_ROWS, WS_PL_CLS_ROW0, WS_PL_CLS_SLAB,  // the ingested batch's own class-sorted blocks
  // cdr_encode_blobs_async (encode_var.hip)
  WS_ENC_SIZES, WS_ENC_TMP,
  // cdr_ndc_replicate_async (ndc.hip)
  WS_NDC_SKIP_RB, WS_NDC_SKIP_AP, WS_NDC_INMEM, WS_NDC_SRC, WS_NDC_CARRY,
  WS_RETRY,  // the class kernels' retry lists: 8 counters, then a list of n_slices per class
  WS_TSTAGE, WS_THEAD,  // k_replay_cls<TASKS>: staged task records, per-entry headers (k_tasks_merge)
  WS_CLS_MAP,  // the device class sort's per-event (class, position), type word and annotation (k_cls_count -> k_cls_gather)
  WS_NUM
};

// host buffers of cdr_replay_one (valid until the next call on the context)
struct cdr_one_host {
  std::vector<cdr_wf_caps> caps;
  std::vector<cdr_wf_result> result;
  std::vector<cdr_exec_info> exec;
  std::vector<cdr_repl_state> repl;
  std::vector<cdr_vh_item> vh;
  std::vector<cdr_activity_info> act;
  std::vector<cdr_timer_info> timer;
  std::vector<cdr_child_info> child;
  std::vector<cdr_cancel_info> cancel;
  std::vector<cdr_signal_info> signal;
  std::vector<cdr_reset_point> rp;
  std::vector<cdr_kv> sa;
  std::vector<cdr_last_decision> ld;
  cdr_out view{};
};

struct cdr_ctx {
  int device;
  int fast = 1;                        // cdr_set_fast_path
  int reg = 1;                         // cdr_set_reg_path
  int cls = CDR_CLS_ON;                // cdr_set_cls_path (CDR_CLS_*)
  uint32_t plan_mode = CDR_PLAN_WAVE | CDR_PLAN_PAR;  // cdr_set_plan_mode
  hipEvent_t ev[4];
  bool timed;
  // optional per-launch timing ring (bench): event pairs around every replay kernel
  std::vector<hipEvent_t> ring;
  uint32_t ring_used = 0;
  // side streams, one per replay kernel class (wave, 12-activity register, general,
  // small-table register, fast, 6-activity register): the classes' slices co-run instead
  // of one kernel after another (fork/join by events on the caller's stream).
  // Concurrency beyond the HIP runtime's hardware queues (GPU_MAX_HW_QUEUES, default 4)
  // serialises on a shared queue.
  static constexpr int N_SIDE = 7;  // + the PAR slices' stream
  hipStream_t side[N_SIDE] = {};
  hipEvent_t fork = nullptr, join[N_SIDE] = {};
  // class i launches on side[side_of[i]] (N_SIDE: on the caller's stream): every class on
  // its own stream when the runtime has the hardware queues for it (GPU_MAX_HW_QUEUES >= 8),
  // else three side streams and the caller's — the PAR slices; the wave and 12-activity
  // classes; the small-table class; the general, fast and 6-activity classes on the
  // caller's stream — so that with HIP's default 4 queues each stream has a queue of its own
  int side_of[N_SIDE] = {0, 1, 2, 3, 4, 5, 6};
  int concurrent = 1;
  int wait_value = -1;  // hipStreamWaitValue32 usable on the device (-1: not asked yet)
  // grow-only device workspace of the host-buffer calls
  void* ws[WS_NUM] = {};
  // the batch whose class-sort map WS_CLS_MAP holds (cdr_cls_plan_async), checked by cdr_cls_pack_async
  const void* cls_map_slab = nullptr;
  uint64_t cls_map_rows = 0;
  uint64_t ws_bytes[WS_NUM] = {};
  // grow-only pinned host staging of the host-buffer calls (the packed slab and arena):
  // no page faults or zero-fill after the first call, and the H2D copy reads page-locked
  // memory directly
  enum { HS_SLAB, HS_ARENA, HS_NUM };
  void* hs[HS_NUM] = {};
  uint64_t hs_bytes[HS_NUM] = {};
  cdr_one_host one;
};

// pinned host staging `slot` of at least `bytes` (grow-only; contents undefined); nullptr
// when page-locked memory cannot be had (defined in replay.hip)
void* cdr_hs_get(cdr_ctx* c, int slot, uint64_t bytes);

// device buffer `slot` of at least `bytes` (grow-only; contents undefined); nullptr
// when the device is out of memory (defined in replay.hip)
void* cdr_ws_get(cdr_ctx* c, int slot, uint64_t bytes);
extern "C" int cdr_ctx_device(const cdr_ctx* c);  // replay.hip
