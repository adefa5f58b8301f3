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
// One thread per entry (its lane writes the entry's rows one after another), 16-B aligned
// stores into fixed-stride slots;
// HBM-bound byte work: a TimerInfo row is 40 B in, 45 B out; a RequestCancelInfo row
// 40 B in, 66 B out.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "cdr/cdr.h"

namespace {

constexpr uint8_t kI64 = 10, kString = 11;


// the byte at position p of a blob: field headers, big-endian values, the stop byte
__device__ __forceinline__ uint8_t be_byte(uint64_t v, uint32_t q) { return (uint8_t)(v >> (8 * (7 - q))); }

__device__ __forceinline__ uint8_t timer_byte(const cdr_timer_info& t, uint32_t p) {
  if (p == 44) return 0;  // stop
  const uint32_t f = p / 11, q = p % 11;
  if (q == 0) return kI64;
  if (q == 1) return 0;
  if (q == 2) return (uint8_t)(10 + 2 * f);  // field IDs 10, 12, 14, 16
  const uint64_t v = f == 0 ? (uint64_t)t.version : f == 1 ? (uint64_t)t.started_id
                   : f == 2 ? (uint64_t)t.expiry_time : (uint64_t)t.task_id;  // ExpiryTime.UnixNano()
  return be_byte(v, q - 3);
}

__device__ __forceinline__ uint8_t cancel_byte(const cdr_cancel_info& x, uint32_t p) {
  if (p < 22) {
    const uint32_t f = p / 11, q = p % 11;
    if (q == 0) return kI64;
    if (q == 1) return 0;
    if (q == 2) return (uint8_t)(10 + f);  // field IDs 10, 11
    return be_byte(f == 0 ? (uint64_t)x.version : (uint64_t)x.initiated_event_batch_id, q - 3);
  }
  if (p == 22) return kString;
  if (p == 23) return 0;
  if (p == 24) return 12;  // CancelRequestID
  if (p < 29) return p == 28 ? 36 : 0;  // i32 length
  if (p == 65) return 0;  // stop
  // RFC 4122 text of (hi, lo): 8-4-4-4-12 lowercase hex
  const uint32_t c = p - 29;
  if (c == 8 || c == 13 || c == 18 || c == 23) return '-';
  const uint32_t k = c - (c > 8) - (c > 13) - (c > 18) - (c > 23);  // hex digit index 0..31
  const uint64_t w = k < 16 ? x.cancel_request_hi : x.cancel_request_lo;
  const uint32_t nib = (uint32_t)(w >> (4 * (15 - (k & 15)))) & 0xFu;
  return (uint8_t)(nib < 10 ? '0' + nib : 'a' + nib - 10);
}

// one row's blob, by the entry's own lane: assembled in registers (the byte loop unrolls
// to constant positions) and written with aligned 16-B stores into its CDR_BLOB_*_STRIDE
// slot
template <uint32_t BYTES, uint32_t STRIDE, class Row, class ByteFn>
__device__ __forceinline__ void put_blob(const Row& row, uint8_t* dst, ByteFn byte_at) {
  uint4* d = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (uint32_t i = 0; i < STRIDE / 16; i++) {  // one 16-B chunk at a time (few live registers)
    uint32_t q[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t b = 0; b < 16; b++) {
      const uint32_t p = 16 * i + b;
      if (p < BYTES) q[b / 4] |= (uint32_t)byte_at(row, p) << (8 * (b % 4));
    }
    d[i] = make_uint4(q[0], q[1], q[2], q[3]);
  }
}

// one thread per entry: the entry records are read coalesced across a wavefront and an
// entry's rows (a handful) are written by its own lane, blob after blob
__global__ __launch_bounds__(256) void k_encode_rows(int table, cdr_dev_batch B, cdr_out O, uint8_t* blobs) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= B.n_wfs) return;
  const cdr_wf_result& r = O.result[w];
  if (r.code != CDR_OK) return;
  const cdr_wf_caps& c = B.caps[w];
  if (table == 1) {
    const uint32_t n = r.n_timer;
    for (uint32_t j = 0; j < n; j++) {
      const uint64_t row = c.timer_off + j;
      put_blob<CDR_BLOB_TIMER_BYTES, CDR_BLOB_TIMER_STRIDE>(O.timer[row], blobs + row * CDR_BLOB_TIMER_STRIDE,
                                                            timer_byte);
    }
  } else {
    const uint32_t n = r.n_cancel;
    for (uint32_t j = 0; j < n; j++) {
      const uint64_t row = c.cancel_off + j;
      put_blob<CDR_BLOB_CANCEL_BYTES, CDR_BLOB_CANCEL_STRIDE>(O.cancel[row], blobs + row * CDR_BLOB_CANCEL_STRIDE,
                                                              cancel_byte);
    }
  }
}

}  // namespace

extern "C" int cdr_encode_rows_async(cdr_ctx* ctx, int table, const cdr_dev_batch* in, const cdr_out* out,
                                     uint8_t* blobs, void* stream) {
  if (!ctx || !in || !out || !blobs || (table != 1 && table != 3) || !out->result) return CDR_API_EINVAL;
  if ((table == 1 && !out->timer) || (table == 3 && !out->cancel)) return CDR_API_EINVAL;
  if (in->n_wfs == 0) return CDR_API_OK;
  hipLaunchKernelGGL(k_encode_rows, dim3((in->n_wfs + 255) / 256), dim3(256), 0, (hipStream_t)stream, table, *in,
                     *out, blobs);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    fprintf(stderr, "cdr: k_encode_rows launch failed: %s\n", hipGetErrorString(e));
    return CDR_API_EDEVICE;
  }
  return CDR_API_OK;
}
