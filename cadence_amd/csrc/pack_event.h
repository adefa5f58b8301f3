// pack_event.h — one event into its slab cell and attribute arena (the layout of cdr.h),
// shared by the host packer (host.cpp cdr_pack_slices) and the device packer of
// decoded histories (ingest.hip k_pack), so both produce the same bytes.
#pragma once

#include <stdint.h>

#include "cdr/cdr.h"

// Arena record sizes (8-byte words) of the types that carry one.
CDR_HD uint32_t cdr_arena_words_for(uint32_t type) {
  switch (type) {
    case CDR_EV_WF_STARTED:
      return (sizeof(cdr_attr_wf_started) + 7) / 8;
    case CDR_EV_AT_SCHEDULED:
      return (sizeof(cdr_attr_at_scheduled) + 7) / 8;
    case CDR_EV_CHILD_INITIATED:  // read only by task emission (target execution)
    case CDR_EV_RCE_INITIATED:
    case CDR_EV_SE_INITIATED:
      return (sizeof(cdr_attr_external) + 7) / 8;
    default:
      return 0;
  }
}

// an attribute record into the arena, in whole 8-byte words (the tail word zero-padded)
CDR_HD void cdr_copy_words(uint64_t* dst, const void* src, uint32_t bytes) {
  const uint8_t* s = (const uint8_t*)src;
  for (uint32_t w = 0; w < (bytes + 7) / 8; w++) {
    uint64_t v = 0;
    for (uint32_t j = 0; j < 8 && w * 8 + j < bytes; j++) v |= (uint64_t)s[w * 8 + j] << (8 * j);
    dst[w] = v;
  }
}

// one event (or padding when e == nullptr) into element i of the slab row `row`;
// attribute records go to the arena at *apos
CDR_HD void cdr_put_event(uint8_t* row, uint32_t i, const cdr_event* ep, bool first, uint64_t* apos_p, uint64_t* arena) {
  int64_t* eid = reinterpret_cast<int64_t*>(row + cdr_col_off(CDR_COL_EVENT_ID));
  int64_t* ver = reinterpret_cast<int64_t*>(row + cdr_col_off(CDR_COL_VERSION));
  int64_t* ts = reinterpret_cast<int64_t*>(row + cdr_col_off(CDR_COL_TIMESTAMP));
  int64_t* task = reinterpret_cast<int64_t*>(row + cdr_col_off(CDR_COL_TASK_ID));
  int64_t* key = reinterpret_cast<int64_t*>(row + cdr_col_off(CDR_COL_KEY));
  int64_t* aux = reinterpret_cast<int64_t*>(row + cdr_col_off(CDR_COL_AUX));
  uint32_t* tf = reinterpret_cast<uint32_t*>(row + cdr_col_off(CDR_COL_TYPE_FLAGS));
  uint32_t* hh = reinterpret_cast<uint32_t*>(row + cdr_col_off(CDR_COL_H));
  int32_t* nn = reinterpret_cast<int32_t*>(row + cdr_col_off(CDR_COL_N));
  if (!ep) {
    tf[i] = CDR_EV_PAD;
    eid[i] = ver[i] = ts[i] = task[i] = key[i] = aux[i] = 0;
    hh[i] = 0;
    nn[i] = 0;
    return;
  }
  uint64_t& apos = *apos_p;
  {
    const cdr_event& e = *ep;
    uint32_t flags = (e.flags & CDR_EVF_BATCH_FIRST) || first ? CDR_SEF_BATCH_FIRST : 0;
    if (!first) {  // the entry's events are contiguous: ep - 1 is the previous one
      flags |= (uint64_t)e.event_id == (uint64_t)ep[-1].event_id + 1 ? CDR_SEF_ID_NEXT : 0u;
      flags |= e.version == ep[-1].version ? CDR_SEF_VER_SAME : 0u;
    }
    int64_t kk = 0, ax = 0;
    uint32_t h = 0;
    int32_t n = 0;
    switch (e.type) {
      case CDR_EV_WF_STARTED:
        ax = (int64_t)apos;
        cdr_copy_words(arena + apos, &e.a.started, sizeof(cdr_attr_wf_started));
        apos += cdr_arena_words_for(e.type);
        break;
      case CDR_EV_DT_SCHEDULED:
        ax = e.a.dt_sched.attempt;
        n = e.a.dt_sched.start_to_close_s;
        break;
      case CDR_EV_DT_STARTED:
        kk = e.a.dt.scheduled_event_id;
        h = e.a.dt.request_id;
        break;
      case CDR_EV_DT_COMPLETED:
        kk = e.a.dt.scheduled_event_id;
        ax = e.a.dt.started_event_id;
        h = e.a.dt.binary_checksum;
        break;
      case CDR_EV_DT_TIMED_OUT:
        n = e.a.dt.timeout_type;
        break;
      case CDR_EV_AT_SCHEDULED: {
        // the four timeouts travel in the columns (the replay loop never reads the
        // arena record; only the final emission of a still-pending activity does)
        const cdr_attr_at_scheduled& a = e.a.at_sched;
        kk = (int64_t)((uint64_t)a.activity_id | ((uint64_t)(uint32_t)a.stc_s << 32));
        h = (uint32_t)a.s2c_s;
        n = a.s2s_s;
        ax = (int64_t)((apos & 0xFFFFFFFFull) | ((uint64_t)(uint32_t)a.hb_s << 32));
        cdr_copy_words(arena + apos, &a, sizeof(cdr_attr_at_scheduled));
        apos += cdr_arena_words_for(e.type);
        break;
      }
      case CDR_EV_AT_STARTED:
        kk = e.a.at.scheduled_event_id;
        h = e.a.at.request_id;
        break;
      case CDR_EV_AT_COMPLETED:
      case CDR_EV_AT_FAILED:
      case CDR_EV_AT_TIMED_OUT:
      case CDR_EV_AT_CANCELED:
        kk = e.a.at.scheduled_event_id;
        break;
      case CDR_EV_AT_CANCEL_REQUESTED:
      case CDR_EV_AT_REQ_CANCEL_FAILED:
        kk = e.a.at.activity_id;
        break;
      case CDR_EV_TIMER_STARTED:
        kk = e.a.timer.timer_id;
        ax = e.a.timer.start_to_fire_s;
        break;
      case CDR_EV_TIMER_FIRED:
      case CDR_EV_TIMER_CANCELED:
      case CDR_EV_CANCEL_TIMER_FAILED:
        kk = e.a.timer.timer_id;
        break;
      case CDR_EV_CHILD_INITIATED:
        kk = e.a.ext.domain | ((uint64_t)(apos & 0xFFFFFFFFull) << 32);
        cdr_copy_words(arena + apos, &e.a.ext, sizeof(cdr_attr_external));
        apos += cdr_arena_words_for(e.type);
        ax = e.a.ext.workflow_type;
        h = e.a.ext.workflow_id;
        n = e.a.ext.parent_close_policy;
        if (e.a.ext.flags & CDR_XF_DOMAIN_MISSING) flags |= CDR_SEF_DOMAIN_MISSING;
        break;
      case CDR_EV_RCE_INITIATED:
        kk = e.a.ext.domain | ((uint64_t)(apos & 0xFFFFFFFFull) << 32);
        cdr_copy_words(arena + apos, &e.a.ext, sizeof(cdr_attr_external));
        apos += cdr_arena_words_for(e.type);
        if (e.a.ext.flags & CDR_XF_DOMAIN_MISSING) flags |= CDR_SEF_DOMAIN_MISSING;
        break;
      case CDR_EV_SE_INITIATED:
        kk = e.a.ext.domain | ((uint64_t)(apos & 0xFFFFFFFFull) << 32);
        cdr_copy_words(arena + apos, &e.a.ext, sizeof(cdr_attr_external));
        apos += cdr_arena_words_for(e.type);
        ax = (int64_t)(((uint64_t)e.a.ext.input << 32) | e.a.ext.control);
        h = e.a.ext.signal_name;
        if (e.a.ext.flags & CDR_XF_DOMAIN_MISSING) flags |= CDR_SEF_DOMAIN_MISSING;
        break;
      case CDR_EV_CHILD_STARTED:
        kk = e.a.ref.initiated_event_id;
        h = e.a.ref.run_id;
        break;
      case CDR_EV_CHILD_START_FAILED:
      case CDR_EV_CHILD_COMPLETED:
      case CDR_EV_CHILD_FAILED:
      case CDR_EV_CHILD_CANCELED:
      case CDR_EV_CHILD_TIMED_OUT:
      case CDR_EV_CHILD_TERMINATED:
      case CDR_EV_RCE_FAILED:
      case CDR_EV_EXT_CANCEL_REQUESTED:
      case CDR_EV_SE_FAILED:
      case CDR_EV_EXT_SIGNALED:
        kk = e.a.ref.initiated_event_id;
        break;
      case CDR_EV_UPSERT_SA:
        ax = e.a.upsert.search_attr_off;
        h = e.a.upsert.search_attr_len;
        break;
      case CDR_EV_WF_CONTINUED_AS_NEW:
        h = e.a.can.new_execution_run_id;
        break;
      default:
        break;
    }
    tf[i] = cdr_type_flags(e.type, flags);
    eid[i] = e.event_id;
    ver[i] = e.version;
    ts[i] = e.timestamp;
    task[i] = e.task_id;
    key[i] = kk;
    aux[i] = ax;
    hh[i] = h;
    nn[i] = n;
  }
}

