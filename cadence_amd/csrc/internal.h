// internal.h — helpers shared by the host-side translation units of libcdr.
#pragma once
#include <cstdint>
#include <vector>

#include "cdr/cdr.h"

namespace cdr_internal {

// arena words of the attribute record of `type` (0 if the type has none)
uint32_t arena_words_for(uint32_t type);

// Output capacities of one history (cdr_plan_caps restricted to one workflow);
// offsets are left zero.
// The live rows a loaded state (cdr_carry) starts with: counts (activities, user timers,
// children, request-cancels, signals, reset points, search-attribute keys) and, when the
// state is host-visible, the rows themselves (their keys: a history event that removes a
// loaded row removes it from the simulation too; without rows, the loaded rows count as
// rows no event removes — an upper bound).
struct loaded_rows {
  uint32_t n[7];
  const cdr_timer_info* timer;
  const cdr_child_info* child;
  const cdr_cancel_info* cancel;
  const cdr_signal_info* signal;
  const cdr_reset_point* rp;
  const cdr_kv* sa;
};
// `loaded` (nullable): the entry replays onto that state; its rows count into the peak
// live sets and the register-table envelope.
// upper bounds of the transfer / timer tasks an entry's events append (host.cpp)
void task_caps(const cdr_event* ev, uint64_t n, uint32_t* xfer, uint32_t* ttask);
void caps_one(const cdr_event* ev, uint64_t n, uint32_t builder, cdr_wf_caps* c, const cdr_kv* kvs = nullptr,
              const cdr_reset_point* rps = nullptr, const loaded_rows* loaded = nullptr);

// Pack one workflow's events into lane `lane` of a slice whose first row is row0 and
// whose length is len (rows beyond n are padding).  `apos` is the workflow's arena
// word offset; kv/rp offsets inside the events are rebased by kv_base/rp_base.
void pack_chunked(const cdr_event* ev, uint64_t n_ev, uint64_t row0, uint32_t rows, uint64_t apos,
                  const cdr_slices* o);
void pack_lane(const cdr_event* ev, uint64_t n, uint64_t row0, uint32_t len, uint32_t lane, uint64_t apos,
               const cdr_slices* o);

// cdr_plan_slices_ex in one call, its outputs in vectors sized by the plan (the host-buffer
// pipeline and the device ingest plan once per batch instead of a size query and a fill)
struct plan_vecs {
  std::vector<int32_t> lane_wf;
  std::vector<uint32_t> slice_len;
  std::vector<uint64_t> slice_row0;
  std::vector<uint32_t> slice_flags;
};
int plan_slices_vec(const cdr_wf_desc* wfs, const cdr_wf_caps* caps, uint32_t n_wfs, uint32_t mode, plan_vecs& out,
                    uint32_t* n_slices, uint64_t* n_rows, uint32_t* n_wave);

}  // namespace cdr_internal
