// encode.hip — persisted-format row encoders: the SQL persistence's thriftrw
// binary-protocol blobs of pending rows.
//
// The sqlblobs structs the row writers build (common/persistence/sql/workflowStateMaps.go
// :239-260 TimerInfo, :504-521 RequestCancelInfo; IDL sqlblobs.thrift:195-206) have every
// field set, so each blob has a fixed size and a fixed field sequence:
//   field = type byte, i16 field ID (big-endian), value; i64 big-endian; string = i32
//   big-endian length + bytes; the struct ends with a 0 stop byte (blob.go:61-73,
//   go.uber.org/thriftrw protocol.Binary; pinned by common/codec/version0Thriftrw_test.go
//   :42-64 through oracle/thrift_binary.py).
// One thread per row slot of the table's (entry, row) space, HBM-bound byte work: a
// TimerInfo row is 40 B in, 45 B out; a RequestCancelInfo row 40 B in, 66 B out.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "cdr/cdr.h"

namespace {

constexpr uint8_t kI64 = 10, kString = 11;

struct Writer {
  uint8_t* p;
  __device__ void byte(uint8_t v) { *p++ = v; }
  __device__ void be(uint64_t v, int n) {
    for (int i = n - 1; i >= 0; i--) byte((uint8_t)(v >> (8 * i)));
  }
  __device__ void header(uint8_t type, int16_t id) {
    byte(type);
    be((uint16_t)id, 2);
  }
  __device__ void i64(int16_t id, int64_t v) {
    header(kI64, id);
    be((uint64_t)v, 8);
  }
  // RFC 4122 text form of (hi, lo): 8-4-4-4-12 lowercase hex
  __device__ void uuid(int16_t id, uint64_t lo, uint64_t hi) {
    header(kString, id);
    be(36, 4);
    for (int k = 0; k < 32; k++) {
      if (k == 8 || k == 12 || k == 16 || k == 20) byte('-');
      const uint64_t w = k < 16 ? hi : lo;
      const uint32_t nib = (uint32_t)(w >> (4 * (15 - (k & 15)))) & 0xFu;
      byte((uint8_t)(nib < 10 ? '0' + nib : 'a' + nib - 10));
    }
  }
};

// entry w's rows of one table; blockIdx.x walks entries, threads the entry's rows
__global__ __launch_bounds__(64) void k_encode_rows(int table, cdr_dev_batch B, cdr_out O, uint8_t* blobs) {
  const uint32_t w = blockIdx.x;
  if (w >= B.n_wfs) return;
  const cdr_wf_result& r = O.result[w];
  if (r.code != CDR_OK) return;
  const cdr_wf_caps& c = B.caps[w];
  if (table == 1) {
    for (uint32_t j = threadIdx.x; j < r.n_timer; j += blockDim.x) {
      const uint64_t row = c.timer_off + j;
      const cdr_timer_info t = O.timer[row];
      Writer W{blobs + row * CDR_BLOB_TIMER_BYTES};
      W.i64(10, t.version);
      W.i64(12, t.started_id);
      W.i64(14, t.expiry_time);  // ExpiryTime.UnixNano()
      W.i64(16, t.task_id);
      W.byte(0);
    }
  } else {
    for (uint32_t j = threadIdx.x; j < r.n_cancel; j += blockDim.x) {
      const uint64_t row = c.cancel_off + j;
      const cdr_cancel_info x = O.cancel[row];
      Writer W{blobs + row * CDR_BLOB_CANCEL_BYTES};
      W.i64(10, x.version);
      W.i64(11, x.initiated_event_batch_id);
      W.uuid(12, x.cancel_request_lo, x.cancel_request_hi);
      W.byte(0);
    }
  }
}

}  // namespace

extern "C" int cdr_encode_rows_async(cdr_ctx* ctx, int table, const cdr_dev_batch* in, const cdr_out* out,
                                     uint8_t* blobs, void* stream) {
  if (!ctx || !in || !out || !blobs || (table != 1 && table != 3) || !out->result) return CDR_API_EINVAL;
  if ((table == 1 && !out->timer) || (table == 3 && !out->cancel)) return CDR_API_EINVAL;
  if (in->n_wfs == 0) return CDR_API_OK;
  hipLaunchKernelGGL(k_encode_rows, dim3(in->n_wfs), dim3(64), 0, (hipStream_t)stream, table, *in, *out, blobs);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    fprintf(stderr, "cdr: k_encode_rows launch failed: %s\n", hipGetErrorString(e));
    return CDR_API_EDEVICE;
  }
  return CDR_API_OK;
}
