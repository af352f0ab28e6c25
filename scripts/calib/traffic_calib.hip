// traffic_calib.hip — calibrates rocprofv3's memory-side byte counters
// (FETCH_SIZE, TCC_EA0_RDREQ) on gfx950 for the access widths of the score
// kernel (bm25mi_kernels.hip: 64-lane rows of buffer_load_b16 slots and
// buffer_load_b32 scores) against a byte count known exactly.  Dev tool, not
// part of the product.  Each pattern is one dispatch over a buffer far larger
// than the Infinity Cache (2 GiB, each byte read once unless stated):
//   x4      global dwordx4 per lane, 1 KiB per wave-load    (guide: FETCH = 1/2)
//   b32     buffer_load_b32 rows: 256 B per wave-load, consecutive rows
//   b16     buffer_load_b16 rows: 128 B per wave-load, consecutive rows
//   b32mis  b32 rows starting at a 4-B-aligned offset that is not line aligned
//           (row r at byte 256 r + 4 (r % 29)): every row straddles lines
//   pair    a posting row as the kernel reads it: b16 slots + b32 scores of the
//           same 64 postings (6 B per posting, 2 arrays)
//   b32x4waves_distinct  every b32 row read by the 4 waves of one workgroup at
//           once (the distinct bytes are reported; L1/L2 merge the rest)
// Prints one JSON line per pattern with the bytes its loads request.
//   hipcc --offload-arch=gfx950 -O3 -o traffic_calib traffic_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -- ./traffic_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr int kWaves = 4;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, (int)(uint32_t)bytes, 0x00020000);
}

// Rows are dealt to waves round-robin; the sum keeps the loads alive and is
// written once per lane only if it equals an impossible value.
__global__ __launch_bounds__(64 * kWaves) void k_x4(const uint4* __restrict__ p, int64_t n16,
                                                    uint32_t* out) {
  uint32_t s = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const uint4 v = p[i];
    s += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x9E3779B9u) out[threadIdx.x] = s;
}

template <int W>  // 2: b16, 4: b32
__global__ __launch_bounds__(64 * kWaves) void k_rows(const void* __restrict__ base, uint64_t bytes,
                                                      int64_t rows, int mis, int reps,
                                                      uint32_t* out) {
  const auto r = rsrc(base, bytes);
  const uint32_t lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * kWaves;
  uint32_t s = 0;
  // reps > 1: the workgroup's waves all read the same rows (row index from
  // the block, not the wave)
  const int64_t first = reps > 1 ? (int64_t)blockIdx.x : wave;
  const int64_t step = reps > 1 ? (int64_t)gridDim.x : nw;
  for (int64_t row = first; row < rows; row += step) {
    const uint32_t off = (uint32_t)(row * 64 * W + (mis ? 4 * (row % 29) : 0));
    if (W == 2)
      s += __builtin_amdgcn_raw_buffer_load_b16(r, (int)(lane * 2), (int)off, 0);
    else
      s += __builtin_amdgcn_raw_buffer_load_b32(r, (int)(lane * 4), (int)off, 0);
  }
  if (s == 0x9E3779B9u) out[threadIdx.x] = s;
}

// a posting row: slots (u16) and scores (f32) of the same 64 postings
__global__ __launch_bounds__(64 * kWaves) void k_pair(const uint16_t* __restrict__ ldoc,
                                                      const float* __restrict__ val, int64_t n,
                                                      uint32_t* out) {
  const auto rl = rsrc(ldoc, (uint64_t)n * 2);
  const auto rv = rsrc(val, (uint64_t)n * 4);
  const uint32_t lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * kWaves;
  uint32_t s = 0;
  for (int64_t row = wave; row < n / 64; row += nw) {
    const uint32_t p = (uint32_t)(row * 64);
    s += __builtin_amdgcn_raw_buffer_load_b16(rl, (int)(lane * 2), (int)(p * 2), 0);
    s += __builtin_amdgcn_raw_buffer_load_b32(rv, (int)(lane * 4), (int)(p * 4), 0);
  }
  if (s == 0x9E3779B9u) out[threadIdx.x] = s;
}

int main() {
  const uint64_t B = 2ull << 30;  // 2 GiB, 8x the Infinity Cache
  void* buf = nullptr;
  uint32_t* out = nullptr;
  CHECK(hipMalloc(&buf, B + 4096));
  CHECK(hipMalloc(&out, 4096));
  CHECK(hipMemset(buf, 1, B + 4096));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const dim3 grid(cus * 8), blk(64 * kWaves);
  auto report = [](const char* name, double bytes) {
    printf("{\"pattern\": \"%s\", \"requested_bytes\": %.0f}\n", name, bytes);
    fflush(stdout);
  };
  // buffer descriptors take < 4 GiB byte ranges: every pattern stays under 2 GiB
  const uint64_t lim = B - 256;
  k_x4<<<grid, blk>>>((const uint4*)buf, (int64_t)(B / 16), out);
  CHECK(hipDeviceSynchronize());
  report("x4", (double)B);
  const int64_t r32 = (int64_t)(lim / 256);
  k_rows<4><<<grid, blk>>>(buf, B, r32, 0, 1, out);
  CHECK(hipDeviceSynchronize());
  report("b32", (double)r32 * 256);
  const int64_t r16 = (int64_t)(lim / 128);
  k_rows<2><<<grid, blk>>>(buf, B, r16, 0, 1, out);
  CHECK(hipDeviceSynchronize());
  report("b16", (double)r16 * 128);
  k_rows<4><<<grid, blk>>>(buf, B, r32, 1, 1, out);
  CHECK(hipDeviceSynchronize());
  report("b32mis", (double)r32 * 256);
  const int64_t np = (int64_t)(B / 6 / 64 * 64);
  k_pair<<<grid, blk>>>((const uint16_t*)buf, (const float*)((char*)buf + np * 2), np, out);
  CHECK(hipDeviceSynchronize());
  report("pair", (double)np * 6);
  const int64_t r8 = (int64_t)(lim / 4 / 256);  // 512 MiB of rows, each read by 4 waves
  k_rows<4><<<grid, blk>>>(buf, B, r8, 0, kWaves, out);
  CHECK(hipDeviceSynchronize());
  report("b32x4waves_distinct", (double)r8 * 256);
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
