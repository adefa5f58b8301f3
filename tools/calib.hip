// PMC calibration for the replay kernels' access widths (VERDICT r4 "calibrate first").
//
// MI355X_MICROARCH.md §HBM establishes FETCH_SIZE = 1/2 of the bytes only for 16-B-per-lane
// streaming reads and WRITE_SIZE = the bytes only for 16-B-per-lane streaming stores.  The
// replay kernels read the slab with 4- and 8-B-per-lane buffer loads (one column of one
// 3,840-B row per instruction) and write their records with 8-B stores from lanes 256 B
// apart.  Each kernel here moves a KNOWN byte count in one of those patterns; run it under
// `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes) and
// tools/calib.py divides the counters by the known bytes.
//
// usage: calib [GiB per buffer (default 2)]   -- prints one line per kernel: name bytes ms
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef __amdgpu_buffer_rsrc_t rsrc_t;
static constexpr uint32_t ROW = 3840;  // the slab row (cdr.h CDR_ROW_BYTES)
static constexpr int WG = 256;

__device__ __forceinline__ rsrc_t mk(const void* p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)n, 0x00020000);
}

// ---- streaming reads: one grid-stride pass over n bytes, w bytes per lane per load
__global__ __launch_bounds__(WG) void k_cal_r16(const uint4* p, uint64_t n16, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)WG + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * WG) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;
}
// buffer loads over 1-GiB windows (a descriptor addresses < 4 GiB)
template <int W>
__global__ __launch_bounds__(WG) void k_cal_rbuf(const uint8_t* p, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  const uint64_t win = 1ull << 30;
  for (uint64_t base = 0; base < n; base += win) {
    const uint64_t len = n - base < win ? n - base : win;
    const rsrc_t r = mk(p + base, (uint32_t)len);
    for (uint64_t i = blockIdx.x * (uint64_t)WG + threadIdx.x; i * W < len; i += (uint64_t)gridDim.x * WG) {
      if constexpr (W == 4) {
        acc ^= __builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)(i * 4), 0, 0);
      } else {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)(i * 8), 0, 0);
        acc ^= v[0] ^ v[1];
      }
    }
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;
}
// slab pattern: a wave walks the rows of its slice (rows_per_slice rows, 3,840 B each) and
// per row loads NC8 8-byte columns (512 B each, columns 0..NC8-1) and, if TF, the 4-byte
// type_flags column (256 B at offset 3,072) -- the replay kernels' per-step loads
template <int NC8, bool TF>
__global__ __launch_bounds__(64) void k_cal_slab(const uint8_t* slab, uint32_t nslices, uint32_t rows_per_slice,
                                                 uint32_t* sink) {
  const uint32_t s = blockIdx.x, lane = threadIdx.x;
  if (s >= nslices) return;
  const rsrc_t r = mk(slab + (uint64_t)s * rows_per_slice * ROW, rows_per_slice * ROW);
  uint32_t acc = 0;
  for (uint32_t k = 0; k < rows_per_slice; k++) {
#pragma unroll
    for (int c = 0; c < NC8; c++) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, k * ROW + lane * 8, c * 512, 0);
      acc ^= v[0] ^ v[1];
    }
    if (TF) acc ^= __builtin_amdgcn_raw_buffer_load_b32(r, k * ROW + lane * 4, 3072, 0);
  }
  if (acc == 0x9e3779b9u) sink[s] = acc;
}

// ---- streaming writes
template <int W>
__global__ __launch_bounds__(WG) void k_cal_wstream(uint8_t* p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)WG + threadIdx.x; i * W < n; i += (uint64_t)gridDim.x * WG) {
    if constexpr (W == 16) ((uint4*)p)[i] = make_uint4((uint32_t)i, 1, 2, 3);
    else if constexpr (W == 8) ((uint64_t*)p)[i] = i;
    else ((uint32_t*)p)[i] = (uint32_t)i;
  }
}
// record pattern: lane l owns a 256-B record and writes NF of its 32 8-byte fields, one
// store instruction per field (all lanes field f, then f + 1): 64 records 256 B apart per
// store -- the ExecutionInfo projection's write shape
template <int NF>
__global__ __launch_bounds__(WG) void k_cal_wrec(uint64_t* rec, uint64_t nrec) {
  const uint64_t i = blockIdx.x * (uint64_t)WG + threadIdx.x;
  if (i >= nrec) return;
#pragma unroll
  for (int f = 0; f < NF; f++) {
    rec[i * 32 + f] = i + f;
    asm volatile("" ::: "memory");  // one 8-B store per field, as the replay kernels write them
  }
}
// scattered: each lane stores one 8-byte word into its own 128-B line
__global__ __launch_bounds__(WG) void k_cal_wscat8(uint64_t* p, uint64_t nlines) {
  const uint64_t i = blockIdx.x * (uint64_t)WG + threadIdx.x;
  if (i < nlines) p[i * 16] = i;
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 2.0;
  const uint64_t n = (uint64_t)(gib * (1ull << 30)) & ~(uint64_t)(ROW * 64 - 1);
  uint8_t *a, *b;
  uint32_t* sink;
  CK(hipMalloc(&a, n));
  CK(hipMalloc(&b, n));
  CK(hipMalloc(&sink, 1 << 24));
  CK(hipMemset(a, 1, n));
  CK(hipMemset(b, 2, n));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 8192;
  auto run = [&](const char* name, double bytes, auto&& launch) {
    for (int rep = 0; rep < 3; rep++) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%s %.0f %.4f %.1f\n", name, bytes, ms, bytes / ms / 1e6);
      fflush(stdout);
    }
  };
  // reads alternate between the two buffers so no pass finds the other's lines in the
  // 256-MiB Infinity Cache
  run("k_cal_r16", (double)n, [&] { k_cal_r16<<<grid, WG>>>((const uint4*)a, n / 16, sink); });
  run("k_cal_rbuf<8>", (double)n, [&] { k_cal_rbuf<8><<<grid, WG>>>(b, n, sink); });
  run("k_cal_rbuf<4>", (double)n, [&] { k_cal_rbuf<4><<<grid, WG>>>(a, n, sink); });
  const uint32_t rps = 200;  // rows per slice (a ~200-event history)
  const uint32_t nsl = (uint32_t)(n / ((uint64_t)rps * ROW));
  const double rows = (double)nsl * rps;
  run("k_cal_slab<6,true>", rows * (6 * 512 + 256),
      [&] { k_cal_slab<6, true><<<nsl, 64>>>(b, nsl, rps, sink); });
  run("k_cal_slab<2,true>", rows * (2 * 512 + 256),
      [&] { k_cal_slab<2, true><<<nsl, 64>>>(a, nsl, rps, sink); });
  run("k_cal_slab<0,true>", rows * 256, [&] { k_cal_slab<0, true><<<nsl, 64>>>(b, nsl, rps, sink); });
  run("k_cal_wstream<16>", (double)n, [&] { k_cal_wstream<16><<<grid, WG>>>(a, n); });
  run("k_cal_wstream<8>", (double)n, [&] { k_cal_wstream<8><<<grid, WG>>>(b, n); });
  run("k_cal_wstream<4>", (double)n, [&] { k_cal_wstream<4><<<grid, WG>>>(a, n); });
  const uint64_t nrec = n / 256;
  run("k_cal_wrec<32>", (double)nrec * 256, [&] { k_cal_wrec<32><<<(nrec + WG - 1) / WG, WG>>>((uint64_t*)b, nrec); });
  run("k_cal_wrec<16>", (double)nrec * 128, [&] { k_cal_wrec<16><<<(nrec + WG - 1) / WG, WG>>>((uint64_t*)a, nrec); });
  run("k_cal_wrec<4>", (double)nrec * 32, [&] { k_cal_wrec<4><<<(nrec + WG - 1) / WG, WG>>>((uint64_t*)b, nrec); });
  const uint64_t nl = n / 128;
  run("k_cal_wscat8", (double)nl * 8, [&] { k_cal_wscat8<<<(nl + WG - 1) / WG, WG>>>((uint64_t*)a, nl); });
  CK(hipDeviceSynchronize());
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(sink));
  return 0;
}
