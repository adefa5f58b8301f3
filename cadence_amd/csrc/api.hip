// api.hip — host pipeline, stream compaction and checksum kernels of libcdr.
//
// cdr_replay_batch is the synchronous "hand me decoded histories, give me mutable
// states" entry point (the batch analogue of stateBuilder.applyEvents); the
// device-resident path used by the benchmark is cdr_replay_sliced_async.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "cdr/cdr.h"
#include "ctx.h"
#include "internal.h"

extern "C" uint32_t cdr_get_plan_mode(const cdr_ctx* ctx);  // replay.hip

#define HIPCHK(x)                                                                                     \
  do {                                                                                                \
    hipError_t _e = (x);                                                                              \
    if (_e != hipSuccess) {                                                                           \
      fprintf(stderr, "cdr: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(_e), __FILE__, __LINE__); \
      return CDR_API_EDEVICE;                                                                         \
    }                                                                                                 \
  } while (0)


namespace {

// float4 stream copy (the bandwidth ceiling bench.py reports beside the replay kernel): one
// 16-B vector per lane, one-shot grid.  Measured on the box (tools/copy_bw.hip, 4 GiB):
// 6.18 TB/s, against 4.7-4.9 TB/s for grid-stride loops of any unroll / grid size
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_stream_copy(const u32x4_t* __restrict__ src, u32x4_t* __restrict__ dst,
                                                     uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

// dense copy of one pending table: one thread per (workflow, row)
template <class Row>
__global__ void k_compact_rows(const cdr_wf_caps* caps, const cdr_wf_result* res, const uint64_t* row_base,
                               uint32_t n_wfs, int table, const Row* src, Row* dst) {
  const uint32_t w = blockIdx.x;
  if (w >= n_wfs) return;
  const cdr_wf_caps c = caps[w];
  const cdr_wf_result r = res[w];
  uint64_t off;
  uint32_t n;
  switch (table) {
    case 0: off = c.act_off; n = r.n_activity; break;
    case 1: off = c.timer_off; n = r.n_timer; break;
    case 2: off = c.child_off; n = r.n_child; break;
    case 3: off = c.cancel_off; n = r.n_cancel; break;
    default: off = c.signal_off; n = r.n_signal; break;
  }
  if (r.code != CDR_OK) n = 0;
  for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) dst[row_base[w] + j] = src[off + j];
}

// exclusive scan of per-workflow counts (single block, chunked; counts are small)
__global__ void k_scan_counts(const cdr_wf_result* res, uint32_t n_wfs, int table, uint64_t* row_base) {
  __shared__ uint64_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (n_wfs + blockDim.x - 1) / blockDim.x;
  const uint32_t b0 = t * per, b1 = min(n_wfs, b0 + per);
  uint64_t sum = 0;
  for (uint32_t w = b0; w < b1; w++) {
    const cdr_wf_result& r = res[w];
    uint32_t n = table == 0 ? r.n_activity : table == 1 ? r.n_timer : table == 2 ? r.n_child
               : table == 3 ? r.n_cancel : r.n_signal;
    sum += r.code == CDR_OK ? n : 0;
  }
  part[t] = sum;
  __syncthreads();
  if (t == 0) {
    uint64_t run = 0;
    for (uint32_t i = 0; i < blockDim.x; i++) {
      uint64_t v = part[i];
      part[i] = run;
      run += v;
    }
    row_base[n_wfs] = run;
  }
  __syncthreads();
  uint64_t run = part[t];
  for (uint32_t w = b0; w < b1; w++) {
    row_base[w] = run;
    const cdr_wf_result& r = res[w];
    uint32_t n = table == 0 ? r.n_activity : table == 1 ? r.n_timer : table == 2 ? r.n_child
               : table == 3 ? r.n_cancel : r.n_signal;
    run += r.code == CDR_OK ? n : 0;
  }
}

__device__ __forceinline__ uint64_t fold(uint64_t h, uint64_t v) { return cdr_mix64(h ^ v) + 0x9E3779B97F4A7C15ull; }
__device__ uint64_t hash_bytes(uint64_t h, const void* p, uint32_t bytes) {
  const uint64_t* q = (const uint64_t*)p;
  for (uint32_t i = 0; i < bytes / 8; i++) h = fold(h, q[i]);
  return h;
}

// per-workflow hash of the whole output record set (restated by oracle/digest_ref.cpp),
// summed (order-independent); per_entry (nullable) receives each entry's hash
__global__ void k_digest(cdr_dev_batch B, cdr_out O, uint64_t* per_entry, unsigned long long* sum) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t h = 0;
  if (w < B.n_wfs) {
    const cdr_wf_result r = O.result[w];
    h = fold(0x5EED, (uint64_t)(uint32_t)r.code | ((uint64_t)r.flags << 32));
    h = fold(h, (uint64_t)r.fail_event_id);
    if (r.code == CDR_OK) {
      const cdr_wf_caps c = B.caps[w];
      h = hash_bytes(h, &O.exec[w], sizeof(cdr_exec_info));
      if (B.wfs[w].builder == CDR_BUILDER_2DC) h = hash_bytes(h, &O.repl[w], sizeof(cdr_repl_state));
      h = hash_bytes(h, O.vh + c.vh_off, r.n_vh * sizeof(cdr_vh_item));
      h = hash_bytes(h, O.act + c.act_off, r.n_activity * sizeof(cdr_activity_info));
      h = hash_bytes(h, O.timer + c.timer_off, r.n_timer * sizeof(cdr_timer_info));
      h = hash_bytes(h, O.child + c.child_off, r.n_child * sizeof(cdr_child_info));
      h = hash_bytes(h, O.cancel + c.cancel_off, r.n_cancel * sizeof(cdr_cancel_info));
      h = hash_bytes(h, O.signal + c.signal_off, r.n_signal * sizeof(cdr_signal_info));
      h = hash_bytes(h, O.rp + c.rp_off, r.n_reset_points * sizeof(cdr_reset_point));
      h = hash_bytes(h, O.sa + c.sa_off, r.n_search_attr * sizeof(cdr_kv));
    }
    if (per_entry) per_entry[w] = h;
  }
  // wave reduction then one atomic per wave
  for (int o = 32; o > 0; o >>= 1) h += __shfl_down(h, o, 64);
  if ((threadIdx.x & 63) == 0 && h) atomicAdd(sum, (unsigned long long)h);
}


}  // namespace

static int replay_host(cdr_ctx* ctx, const cdr_batch* b, const cdr_wf_caps* caps, const cdr_totals* tot,
                       cdr_out* out, bool refresh, uint32_t rflags, hipStream_t st);

extern "C" {

int cdr_stream_copy_async(void* dst, const void* src, uint64_t bytes, void* stream) {
  if (!dst || !src || bytes % 64) return CDR_API_EINVAL;
  const uint64_t n = bytes / 16, grid = (n + 255) / 256;
  if (grid > 0xFFFFFFFFull) return CDR_API_EINVAL;
  hipLaunchKernelGGL(k_stream_copy, dim3((uint32_t)grid), dim3(256), 0, (hipStream_t)stream, (const u32x4_t*)src,
                     (u32x4_t*)dst, n);
  HIPCHK(hipGetLastError());
  return CDR_API_OK;
}

int cdr_compact_async(cdr_ctx* ctx, int table, const cdr_dev_batch* in, const cdr_out* out, void* dense,
                      uint64_t* row_base, void* stream) {
  if (!ctx || !in || !out || table < 0 || table > 4) return CDR_API_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, st, out->result, in->n_wfs, table, row_base);
  HIPCHK(hipGetLastError());
  const dim3 g(in->n_wfs), b(64);
  if (in->n_wfs == 0) return CDR_API_OK;
  switch (table) {
    case 0:
      hipLaunchKernelGGL(k_compact_rows<cdr_activity_info>, g, b, 0, st, in->caps, out->result, row_base, in->n_wfs,
                         table, out->act, (cdr_activity_info*)dense);
      break;
    case 1:
      hipLaunchKernelGGL(k_compact_rows<cdr_timer_info>, g, b, 0, st, in->caps, out->result, row_base, in->n_wfs,
                         table, out->timer, (cdr_timer_info*)dense);
      break;
    case 2:
      hipLaunchKernelGGL(k_compact_rows<cdr_child_info>, g, b, 0, st, in->caps, out->result, row_base, in->n_wfs,
                         table, out->child, (cdr_child_info*)dense);
      break;
    case 3:
      hipLaunchKernelGGL(k_compact_rows<cdr_cancel_info>, g, b, 0, st, in->caps, out->result, row_base, in->n_wfs,
                         table, out->cancel, (cdr_cancel_info*)dense);
      break;
    default:
      hipLaunchKernelGGL(k_compact_rows<cdr_signal_info>, g, b, 0, st, in->caps, out->result, row_base, in->n_wfs,
                         table, out->signal, (cdr_signal_info*)dense);
      break;
  }
  HIPCHK(hipGetLastError());
  return CDR_API_OK;
}

int cdr_entry_digests_async(cdr_ctx* ctx, const cdr_dev_batch* in, const cdr_out* out, uint64_t* per_entry,
                            uint64_t* dev_sum, void* stream) {
  if (!ctx || !in || !out || !dev_sum) return CDR_API_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipMemsetAsync(dev_sum, 0, sizeof(uint64_t), st));
  const uint32_t blocks = (in->n_wfs + 255) / 256;
  if (blocks)
    hipLaunchKernelGGL(k_digest, dim3(blocks), dim3(256), 0, st, *in, *out, per_entry, (unsigned long long*)dev_sum);
  HIPCHK(hipGetLastError());
  return CDR_API_OK;
}

int cdr_checksum_async(cdr_ctx* ctx, const cdr_dev_batch* in, const cdr_out* out, uint64_t* dev_sum, void* stream) {
  return cdr_entry_digests_async(ctx, in, out, nullptr, dev_sum, stream);
}

int cdr_replay_batch(cdr_ctx* ctx, const cdr_batch* b, const cdr_wf_caps* caps, const cdr_totals* tot, cdr_out* out,
                     void* stream) {
  return replay_host(ctx, b, caps, tot, out, false, 0, (hipStream_t)stream);
}

int cdr_rebuild_batch(cdr_ctx* ctx, const cdr_batch* b, const cdr_wf_caps* caps, const cdr_totals* tot, cdr_out* out,
                      uint32_t flags, void* stream) {
  if (!out || !out->transfer || !out->timer_tasks || !out->n_tasks) return CDR_API_EINVAL;
  return replay_host(ctx, b, caps, tot, out, true, flags, (hipStream_t)stream);
}

int cdr_replay_one(cdr_ctx* ctx, const cdr_batch* b, const cdr_out** view, const cdr_wf_caps** caps, void* stream) {
  if (!ctx || !b || !view || !caps || b->n_wfs < 1 || b->n_wfs > 2) return CDR_API_EINVAL;
  if (b->wfs[0].parent >= 0 || (b->n_wfs == 2 && b->wfs[0].newrun != 1)) return CDR_API_EINVAL;
  cdr_one_host& H = ctx->one;
  const uint32_t n = b->n_wfs;
  H.caps.resize(n);
  cdr_totals tot{};
  int rc = cdr_plan_caps(b, H.caps.data(), &tot);
  if (rc) return rc;
  // grow-only host buffers: resize keeps the capacity (records are fully written for
  // OK entries; the replay pipeline downloads every slot)
  auto fit = [](auto& v, uint64_t k) { v.resize(k ? k : 1); return v.data(); };
  cdr_out& o = H.view;
  o = cdr_out{};
  o.result = fit(H.result, n);
  o.exec = fit(H.exec, n);
  o.repl = fit(H.repl, n);
  o.vh = fit(H.vh, tot.vh);
  o.act = fit(H.act, tot.act);
  o.timer = fit(H.timer, tot.timer);
  o.child = fit(H.child, tot.child);
  o.cancel = fit(H.cancel, tot.cancel);
  o.signal = fit(H.signal, tot.signal);
  o.rp = fit(H.rp, tot.rp);
  o.sa = fit(H.sa, tot.sa);
  o.last_decision = fit(H.ld, n);
  rc = replay_host(ctx, b, H.caps.data(), &tot, &o, false, 0, (hipStream_t)stream);
  if (rc) return rc;
  *view = &o;
  *caps = H.caps.data();
  return CDR_API_OK;
}

}  // extern "C"

// plan + pack + H2D + replay (+ refreshTasks) + D2H, on `st` with the context's
// grow-only device workspace
static int replay_host(cdr_ctx* ctx, const cdr_batch* b, const cdr_wf_caps* caps, const cdr_totals* tot,
                       cdr_out* out, bool refresh, uint32_t rflags, hipStream_t st) {
  if (!ctx || !b || !caps || !tot || !out || !out->result) return CDR_API_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));  // the context's device, whatever thread calls
  // ---- plan + pack on the host
  uint32_t ns = 0, n_wave = 0;
  uint64_t rows = 0;
  // stateBuilder task lists are emitted by the general kernel only (no wave slices);
  // the refresher's come from their own kernel after any replay
  const bool tasks = out->transfer != nullptr && !refresh;
  const uint32_t mode = tasks ? 0u : cdr_get_plan_mode(ctx);
  cdr_internal::plan_vecs pv;  // one planning pass (the C ABI's size query + fill would plan twice)
  int rc = cdr_internal::plan_slices_vec(b->wfs, caps, b->n_wfs, mode, pv, &ns, &rows, &n_wave);
  if (rc) return rc;
  std::vector<int32_t>& lane = pv.lane_wf;
  std::vector<uint32_t>& slen = pv.slice_len;
  std::vector<uint32_t>& sflags = pv.slice_flags;
  std::vector<uint64_t>& row0 = pv.slice_row0;
  const uint64_t ne = rows * CDR_SLICE_WIDTH;
  const uint64_t aw = cdr_plan_arena_words(b);
  // the packer writes every cell (padding included) and every arena word it names: staging
  // needs no zero-fill
  uint8_t* slab = (uint8_t*)cdr_hs_get(ctx, cdr_ctx::HS_SLAB, ne * CDR_EL_BYTES);
  uint64_t* arena = (uint64_t*)cdr_hs_get(ctx, cdr_ctx::HS_ARENA, (aw ? aw : 1) * 8ull);
  if (!slab || !arena) return CDR_API_ENOMEM;
  cdr_slices hs{};
  hs.n_slices = ns;
  hs.n_rows = rows;
  hs.arena_words = aw;
  hs.slice_row0 = row0.data();
  hs.slice_len = slen.data();
  hs.lane_wf = lane.data();
  hs.slice_flags = sflags.data();
  hs.slab = slab;
  hs.arena = arena;
  rc = cdr_pack_slices(b, &hs, 0);
  if (rc) return rc;
  std::vector<uint64_t> sc_off(ns);
  std::vector<uint32_t> sc_act(ns), sc_tim(ns);
  uint64_t sc_words = 0;
  uint32_t n_fast = 0;
  rc = cdr_plan_scratch(caps, lane.data(), ns, sc_off.data(), sc_act.data(), sc_tim.data(), sflags.data(), &sc_words,
                        &n_fast);
  if (rc) return rc;

  // ---- device buffers: workspace slots (no allocation once the context is warm);
  // any failed allocation or copy is reported before anything is launched
  bool oom = false, dev_err = false;
  auto up = [&](int slot, const void* src, uint64_t bytes) -> void* {
    void* p = cdr_ws_get(ctx, slot, bytes);
    if (!p) {
      oom = true;
      return nullptr;
    }
    if (bytes && src && hipMemcpyAsync(p, src, bytes, hipMemcpyHostToDevice, st) != hipSuccess) dev_err = true;
    return p;
  };
  auto dz = [&](int slot, uint64_t bytes) -> void* {
    void* p = cdr_ws_get(ctx, slot, bytes);
    if (!p) {
      oom = true;
      return nullptr;
    }
    if (hipMemsetAsync(p, 0, bytes ? bytes : 8, st) != hipSuccess) dev_err = true;
    return p;
  };
  cdr_dev_batch db{};
  db.ev.n_slices = ns;
  db.ev.n_rows = rows;
  db.ev.arena_words = aw;
  db.ev.slice_row0 = (const uint64_t*)up(WS_ROW0, row0.data(), ns * 8ull);
  db.ev.slice_len = (const uint32_t*)up(WS_SLEN, slen.data(), ns * 4ull);
  db.ev.lane_wf = (const int32_t*)up(WS_LANE, lane.data(), lane.size() * 4ull);
  db.ev.slab = (const uint8_t*)up(WS_SLAB, slab, ne * CDR_EL_BYTES);
  db.ev.arena = (const uint64_t*)up(WS_ARENA, arena, (aw ? aw : 1) * 8ull);
  db.ev.slice_flags = (const uint32_t*)up(WS_SFLAGS, sflags.data(), ns * 4ull);
  db.n_fast_slices = n_fast;
  db.n_wave_slices = n_wave;
  for (uint32_t i = 0; i < ns; i++) {
    db.n_reg_slices += (sflags[i] & CDR_SLICE_REG) ? 1u : 0u;
    db.n_reg2_slices += (sflags[i] & CDR_SLICE_REG2) ? 1u : 0u;
    db.n_reg0_slices += (sflags[i] & CDR_SLICE_REG0) ? 1u : 0u;
    db.n_par_slices += (sflags[i] & CDR_SLICE_PAR) ? 1u : 0u;
  }
  cdr_plan_class_ranges(sflags.data(), ns, db.class_lo, db.class_hi);
  db.ev.slice_scratch_off = (const uint64_t*)up(WS_SC_OFF, sc_off.data(), ns * 8ull);
  db.ev.slice_act_slots = (const uint32_t*)up(WS_SC_ACT, sc_act.data(), ns * 4ull);
  db.ev.slice_tim_slots = (const uint32_t*)up(WS_SC_TIM, sc_tim.data(), ns * 4ull);
  for (uint32_t i = 0; i < ns; i++) {
    db.max_act_slots = sc_act[i] > db.max_act_slots ? sc_act[i] : db.max_act_slots;
    db.max_tim_slots = sc_tim[i] > db.max_tim_slots ? sc_tim[i] : db.max_tim_slots;
  }
  db.scratch = (uint64_t*)dz(WS_SCRATCH, sc_words * 8);
  db.wfs = (const cdr_wf_desc*)up(WS_WFS, b->wfs, (uint64_t)b->n_wfs * sizeof(cdr_wf_desc));
  db.caps = (const cdr_wf_caps*)up(WS_CAPS, caps, (uint64_t)b->n_wfs * sizeof(cdr_wf_caps));
  db.kvs = (const cdr_kv*)up(WS_KVS, b->kvs, b->n_kvs * sizeof(cdr_kv));
  db.rps = (const cdr_reset_point*)up(WS_RPS, b->rps, b->n_rps * sizeof(cdr_reset_point));
  cdr_carry dc{};
  if (b->carry && b->carry->src) {  // the loaded states, copied to the device as they are
    const cdr_carry& hc = *b->carry;
    const cdr_totals& t = hc.totals;
    const uint64_t n = hc.n_src;
    dc = hc;
    dc.src = (const int32_t*)up(WS_CY_SRC, hc.src, (uint64_t)b->n_wfs * 4);
    dc.caps = (const cdr_wf_caps*)up(WS_CY_CAPS, hc.caps, n * sizeof(cdr_wf_caps));
    dc.state.result = (cdr_wf_result*)up(WS_CY_RESULT, hc.state.result, n * sizeof(cdr_wf_result));
    dc.state.exec = (cdr_exec_info*)up(WS_CY_EXEC, hc.state.exec, n * sizeof(cdr_exec_info));
    dc.state.repl = (cdr_repl_state*)up(WS_CY_REPL, hc.state.repl, n * sizeof(cdr_repl_state));
    dc.state.vh = (cdr_vh_item*)up(WS_CY_VH, hc.state.vh, t.vh * sizeof(cdr_vh_item));
    dc.state.act = (cdr_activity_info*)up(WS_CY_ACT, hc.state.act, t.act * sizeof(cdr_activity_info));
    dc.state.timer = (cdr_timer_info*)up(WS_CY_TIMER, hc.state.timer, t.timer * sizeof(cdr_timer_info));
    dc.state.child = (cdr_child_info*)up(WS_CY_CHILD, hc.state.child, t.child * sizeof(cdr_child_info));
    dc.state.cancel = (cdr_cancel_info*)up(WS_CY_CANCEL, hc.state.cancel, t.cancel * sizeof(cdr_cancel_info));
    dc.state.signal = (cdr_signal_info*)up(WS_CY_SIGNAL, hc.state.signal, t.signal * sizeof(cdr_signal_info));
    dc.state.rp = (cdr_reset_point*)up(WS_CY_RP, hc.state.rp, t.rp * sizeof(cdr_reset_point));
    dc.state.sa = (cdr_kv*)up(WS_CY_SA, hc.state.sa, t.sa * sizeof(cdr_kv));
    if (hc.in_memory) dc.in_memory = (const uint8_t*)up(WS_CY_INMEM, hc.in_memory, (uint64_t)b->n_wfs);
    dc.state.transfer = dc.state.timer_tasks = nullptr;
    dc.state.n_tasks = nullptr;
    dc.state.last_decision = nullptr;
    db.carry = (const cdr_carry*)up(WS_CY_DESC, &dc, sizeof(dc));
  }
  db.n_wfs = b->n_wfs;
  db.empty_uuid = b->empty_uuid;
  db.cluster = b->cluster;
  db.now_ns = b->now_ns;
  db.uuid_seed = b->uuid_seed;
  cdr_out dout{};
  dout.result = (cdr_wf_result*)dz(WS_O_RESULT, (uint64_t)b->n_wfs * sizeof(cdr_wf_result));
  dout.exec = (cdr_exec_info*)dz(WS_O_EXEC, (uint64_t)b->n_wfs * sizeof(cdr_exec_info));
  dout.repl = (cdr_repl_state*)dz(WS_O_REPL, (uint64_t)b->n_wfs * sizeof(cdr_repl_state));
  dout.vh = (cdr_vh_item*)dz(WS_O_VH, tot->vh * sizeof(cdr_vh_item));
  dout.act = (cdr_activity_info*)dz(WS_O_ACT, tot->act * sizeof(cdr_activity_info));
  dout.timer = (cdr_timer_info*)dz(WS_O_TIMER, tot->timer * sizeof(cdr_timer_info));
  dout.child = (cdr_child_info*)dz(WS_O_CHILD, tot->child * sizeof(cdr_child_info));
  dout.cancel = (cdr_cancel_info*)dz(WS_O_CANCEL, tot->cancel * sizeof(cdr_cancel_info));
  dout.signal = (cdr_signal_info*)dz(WS_O_SIGNAL, tot->signal * sizeof(cdr_signal_info));
  dout.rp = (cdr_reset_point*)dz(WS_O_RP, tot->rp * sizeof(cdr_reset_point));
  dout.sa = (cdr_kv*)dz(WS_O_SA, tot->sa * sizeof(cdr_kv));
  if (out->last_decision)
    dout.last_decision = (cdr_last_decision*)dz(WS_O_LD, (uint64_t)b->n_wfs * sizeof(cdr_last_decision));
  if (tasks || refresh) {
    dout.transfer = (cdr_task*)dz(WS_O_XFER, tot->xfer * sizeof(cdr_task));
    dout.timer_tasks = (cdr_task*)dz(WS_O_TTASK, tot->ttask * sizeof(cdr_task));
    dout.n_tasks = (uint32_t*)dz(WS_O_NTASKS, (uint64_t)b->n_wfs * 2 * sizeof(uint32_t));
    db.task_rows = tot->xfer + tot->ttask;
  }
  if (oom || dev_err) {
    (void)hipStreamSynchronize(st);  // no copy may still read the host vectors
    return oom ? CDR_API_ENOMEM : CDR_API_EDEVICE;
  }
  // class-sorted blocks of the register-table slices (k_replay_cls), packed on the host
  // beside the slab when the context asks for them (CDR_CLS_BUILD / CDR_CLS_ALONE): by
  // default a batch replayed once goes to k_replay_reg, since the block's packing and
  // H2D cost more than the class kernel saves (with task lists: k_replay_cls<TASKS>)
  if (ctx->cls >= CDR_CLS_ALONE && ctx->reg && ctx->fast &&
      db.n_reg_slices + db.n_reg2_slices + db.n_reg0_slices + db.n_par_slices > 0 &&
      b->cluster.n_clusters <= (int)CDR_REG_NCL) {
    // the uploads above read host memory this call owns: pack the blocks meanwhile
    std::vector<uint32_t> crows(ns * 4ull);
    std::vector<uint64_t> crow0(ns + 1ull);
    const cdr_wf_desc* wfs_h = b->wfs;
    rc = cdr_plan_cls(&hs, wfs_h, crows.data(), crow0.data());
    std::vector<uint8_t> cslab;
    if (rc == CDR_API_OK) {
      cslab.resize(crow0[ns] ? crow0[ns] * CDR_ROW_BYTES : 8);
      rc = cdr_pack_cls(&hs, wfs_h, crows.data(), crow0.data(), cslab.data(), 0);
    }
    if (rc == CDR_API_OK) {
      db.cls_rows = (const uint32_t*)up(WS_CLS_ROWS, crows.data(), crows.size() * 4);
      db.cls_row0 = (const uint64_t*)up(WS_CLS_ROW0, crow0.data(), crow0.size() * 8);
      db.cls_slab = (const uint8_t*)up(WS_CLS_SLAB, cslab.data(), cslab.size());
      // the host vectors die with this scope: the copies must land first
      if (hipStreamSynchronize(st) != hipSuccess) dev_err = true;
    }
    if (rc != CDR_API_OK || oom || dev_err) {
      (void)hipStreamSynchronize(st);
      return rc != CDR_API_OK ? rc : oom ? CDR_API_ENOMEM : CDR_API_EDEVICE;
    }
  }
  if (refresh) {  // the replay itself emits no stateBuilder tasks
    cdr_out rout = dout;
    rout.transfer = rout.timer_tasks = nullptr;
    rout.n_tasks = nullptr;
    rc = cdr_replay_sliced_async(ctx, &db, &rout, st);
    if (rc == CDR_API_OK) rc = cdr_refresh_tasks_async(ctx, &db, &dout, b->now_ns, rflags, st);
  } else {
    rc = cdr_replay_sliced_async(ctx, &db, &dout, st);
  }
  auto down = [&](void* dst, const void* src, uint64_t bytes) {
    if (rc == CDR_API_OK && dst && bytes && hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st) != hipSuccess)
      rc = CDR_API_EDEVICE;
  };
  down(out->result, dout.result, (uint64_t)b->n_wfs * sizeof(cdr_wf_result));
  down(out->exec, dout.exec, (uint64_t)b->n_wfs * sizeof(cdr_exec_info));
  down(out->repl, dout.repl, (uint64_t)b->n_wfs * sizeof(cdr_repl_state));
  down(out->vh, dout.vh, tot->vh * sizeof(cdr_vh_item));
  down(out->act, dout.act, tot->act * sizeof(cdr_activity_info));
  down(out->timer, dout.timer, tot->timer * sizeof(cdr_timer_info));
  down(out->child, dout.child, tot->child * sizeof(cdr_child_info));
  down(out->cancel, dout.cancel, tot->cancel * sizeof(cdr_cancel_info));
  down(out->signal, dout.signal, tot->signal * sizeof(cdr_signal_info));
  down(out->rp, dout.rp, tot->rp * sizeof(cdr_reset_point));
  down(out->sa, dout.sa, tot->sa * sizeof(cdr_kv));
  down(out->last_decision, dout.last_decision, (uint64_t)b->n_wfs * sizeof(cdr_last_decision));
  if (tasks || refresh) {
    down(out->transfer, dout.transfer, tot->xfer * sizeof(cdr_task));
    down(out->timer_tasks, dout.timer_tasks, tot->ttask * sizeof(cdr_task));
    down(out->n_tasks, dout.n_tasks, (uint64_t)b->n_wfs * 2 * sizeof(uint32_t));
  }
  // the stream, not the device: other contexts' work is not waited for
  if (hipStreamSynchronize(st) != hipSuccess && rc == CDR_API_OK) rc = CDR_API_EDEVICE;
  return rc;
}
