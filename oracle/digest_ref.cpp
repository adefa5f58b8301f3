// oracle/digest_ref.cpp — TEST INFRASTRUCTURE ONLY (full-size parity checker).
//
// Restates the engine's per-entry output digest (cadence_amd/csrc/api.hip k_digest) over
// the oracle's own outputs, so that a 1M-workflow GPU replay can be compared with the CPU
// restatement entry by entry without moving every record off the device: two equal
// digest arrays mean equal result codes / fail event ids and, for every OK entry, equal
// bytes of the persisted projection (mutableStateBuilder.CopyToPersistence,
// service/history/mutableStateBuilder.go:257-270: ExecutionInfo, ReplicationState of a
// 2DC builder, the version-history items, the five pending tables, the reset points and
// the search attributes).  The hash is a fold of cdr_mix64 over the records' 8-byte words.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <thread>
#include <vector>

#include "cdr/schema.h"

namespace {

inline uint64_t fold(uint64_t h, uint64_t v) { return cdr_mix64(h ^ v) + 0x9E3779B97F4A7C15ull; }
inline uint64_t hash_bytes(uint64_t h, const void* p, uint64_t bytes) {
  const uint64_t* q = (const uint64_t*)p;
  for (uint64_t i = 0; i < bytes / 8; i++) h = fold(h, q[i]);
  return h;
}

uint64_t entry_digest(const cdr_batch* b, const cdr_wf_caps* caps, const cdr_out* o, uint32_t w) {
  const cdr_wf_result& r = o->result[w];
  uint64_t h = fold(0x5EED, (uint64_t)(uint32_t)r.code | ((uint64_t)r.flags << 32));
  h = fold(h, (uint64_t)r.fail_event_id);
  if (r.code != CDR_OK) return h;
  const cdr_wf_caps& c = caps[w];
  h = hash_bytes(h, &o->exec[w], sizeof(cdr_exec_info));
  if (b->wfs[w].builder == CDR_BUILDER_2DC) h = hash_bytes(h, &o->repl[w], sizeof(cdr_repl_state));
  h = hash_bytes(h, o->vh + c.vh_off, (uint64_t)r.n_vh * sizeof(cdr_vh_item));
  h = hash_bytes(h, o->act + c.act_off, (uint64_t)r.n_activity * sizeof(cdr_activity_info));
  h = hash_bytes(h, o->timer + c.timer_off, (uint64_t)r.n_timer * sizeof(cdr_timer_info));
  h = hash_bytes(h, o->child + c.child_off, (uint64_t)r.n_child * sizeof(cdr_child_info));
  h = hash_bytes(h, o->cancel + c.cancel_off, (uint64_t)r.n_cancel * sizeof(cdr_cancel_info));
  h = hash_bytes(h, o->signal + c.signal_off, (uint64_t)r.n_signal * sizeof(cdr_signal_info));
  h = hash_bytes(h, o->rp + c.rp_off, (uint64_t)r.n_reset_points * sizeof(cdr_reset_point));
  h = hash_bytes(h, o->sa + c.sa_off, (uint64_t)r.n_search_attr * sizeof(cdr_kv));
  return h;
}

}  // namespace

extern "C" {

// per_entry[w] = digest of entry w (nullable); returns the wrapping sum of all digests
// (the engine's cdr_checksum_async value) through *sum.
int cdro_entry_digests(const cdr_batch* b, const cdr_wf_caps* caps, const cdr_out* out, uint64_t* per_entry,
                       uint64_t* sum, int threads) {
  if (!b || !caps || !out || !sum) return -1;
  const uint32_t n = b->n_wfs;
  if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
  threads = std::min(threads, 64);
  std::atomic<uint64_t> total{0};
  std::atomic<uint32_t> next{0};
  auto work = [&] {
    uint64_t s = 0;
    for (;;) {
      const uint32_t i0 = next.fetch_add(4096);
      if (i0 >= n) break;
      const uint32_t i1 = std::min(n, i0 + 4096);
      for (uint32_t w = i0; w < i1; w++) {
        const uint64_t h = entry_digest(b, caps, out, w);
        if (per_entry) per_entry[w] = h;
        s += h;
      }
    }
    total.fetch_add(s);
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads && n > 4096; t++) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  *sum = total.load();
  return 0;
}

}  // extern "C"
