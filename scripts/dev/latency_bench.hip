// Dev micro-benchmark (not part of the product): GPU-side cost of the
// per-batch latency-bound kernels in isolation, next to empty and
// load-chain kernels of the same geometry (1024 waves, 4 per workgroup).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/dev/latency_bench.hip \
//     -o scripts/dev/latency_bench -L mojo-bm25_amd/bm25mi -lbm25mi
#include "../../mojo-bm25_amd/csrc/bm25mi_kernels.hip"
#include <cstdio>
#include <random>
#include <vector>

using namespace bm25mi;

__global__ __launch_bounds__(256) void k_empty(int* out) {
  if (threadIdx.x == 1023) out[0] = 1;
}
__global__ __launch_bounds__(256) void k_load1(const int* in, int* out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  out[i] = in[i] + 1;
}
__global__ __launch_bounds__(256) void k_chain3(const int* in, int* out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  int a = in[i];
  int b = in[(a + i) % n];
  int c = in[(b + i) % n];
  out[i] = c;
}
// one wave per query: load cnt keys, ballot-compact them to the output
__global__ __launch_bounds__(256) void k_copy_list(const uint64_t* list, const int* cnt, int C,
                                                   int k, int* docs, float* scores) {
  const int64_t q = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int n = cnt[q];
  for (int i = lane; i < k; i += 64) {
    const uint64_t x = i < n ? list[q * C + i] : 0ull;
    docs[q * k + i] = x ? (int)(0xFFFFFFFFu - (uint32_t)x) : -1;
    scores[q * k + i] = x ? key_score((uint32_t)(x >> 32)) : 0.f;
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <class F>
float time_it(const char* name, F f, int reps = 200) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) f();
  hipDeviceSynchronize();
  hipEventRecord(a, 0);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  // one launch alone (synchronised before and after)
  float one = 1e9;
  for (int i = 0; i < 20; ++i) {
    hipDeviceSynchronize();
    hipEventRecord(a, 0);
    f();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float m = 0;
    hipEventElapsedTime(&m, a, b);
    one = std::min(one, m);
  }
  printf("{\"kernel\": \"%s\", \"us_back_to_back\": %.2f, \"us_alone_min\": %.2f}\n", name,
         1000.f * ms / reps, 1000.f * one);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms / reps;
}

int main() {
  const int Q = 1024, W = 8, k = 100, S = 80, C = 6400;
  std::mt19937_64 rng(7);
  int *d_i, *d_o;
  CK(hipMalloc(&d_i, sizeof(int) * Q * 256));
  CK(hipMalloc(&d_o, sizeof(int) * Q * 256));
  std::vector<int> hi(Q * 256);
  for (auto& x : hi) x = (int)(rng() % 1000);
  CK(hipMemcpy(d_i, hi.data(), sizeof(int) * hi.size(), hipMemcpyHostToDevice));
  // packed [W][2][Q][k] lists: ~29 real keys per rank and query, padding after
  std::vector<int32_t> pk((size_t)W * 2 * Q * k);
  for (int w = 0; w < W; ++w)
    for (int q = 0; q < Q; ++q) {
      const int n = 10 + (int)(rng() % 40);
      for (int j = 0; j < k; ++j) {
        int32_t* dd = &pk[((size_t)w * 2 * Q + q) * k + j];
        float* ss = reinterpret_cast<float*>(&pk[((size_t)(w * 2 + 1) * Q + q) * k + j]);
        if (j < n) {
          *dd = (int32_t)(w * 1250000 + (rng() % 1250000));
          *ss = 5.f + (float)(rng() % 100000) * 1e-4f;
        } else {
          *dd = -1;
          *reinterpret_cast<uint32_t*>(ss) = 0xFFFFFFFFu;
        }
      }
    }
  int32_t *d_pk, *d_od;
  float* d_os;
  CK(hipMalloc(&d_pk, sizeof(int32_t) * pk.size()));
  CK(hipMemcpy(d_pk, pk.data(), sizeof(int32_t) * pk.size(), hipMemcpyHostToDevice));
  CK(hipMalloc(&d_od, sizeof(int32_t) * Q * k));
  CK(hipMalloc(&d_os, sizeof(float) * Q * k));
  // theta input: [W][Q][S] keys
  std::vector<uint64_t> keys((size_t)W * Q * S);
  for (auto& x : keys) x = make_key(1.f + (float)(rng() % 65536) * 1e-3f, (uint32_t)(rng() % 10000000));
  uint64_t *d_keys, *d_theta;
  int32_t *d_cnt, *d_ctr;
  CK(hipMalloc(&d_keys, sizeof(uint64_t) * keys.size()));
  CK(hipMemcpy(d_keys, keys.data(), sizeof(uint64_t) * keys.size(), hipMemcpyHostToDevice));
  CK(hipMalloc(&d_theta, sizeof(uint64_t) * Q));
  CK(hipMalloc(&d_cnt, sizeof(int32_t) * Q));
  CK(hipMalloc(&d_ctr, sizeof(int32_t) * 64));
  // a list [Q][C] with ~30 keys per query for the copy kernel
  uint64_t* d_list;
  CK(hipMalloc(&d_list, sizeof(uint64_t) * Q * C));
  std::vector<int32_t> hc(Q, 30);
  CK(hipMemcpy(d_cnt, hc.data(), sizeof(int32_t) * Q, hipMemcpyHostToDevice));
  CK(hipMemset(d_list, 0x11, sizeof(uint64_t) * Q * C));

  time_it("empty (256 x 256)", [&] { hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0, d_o); });
  {
    hipEvent_t e1, e2, e3;
    CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming | hipEventReleaseToDevice));
    CK(hipEventCreate(&e3));
    time_it("empty + record(disable timing)", [&] {
      hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0, d_o);
      hipEventRecord(e1, 0);
    });
    time_it("empty + record(disable timing, release to device)", [&] {
      hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0, d_o);
      hipEventRecord(e2, 0);
    });
    time_it("empty + record(default)", [&] {
      hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0, d_o);
      hipEventRecord(e3, 0);
    });
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    time_it("empty + record + wait on 2nd stream + empty there", [&] {
      hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0, d_o);
      hipEventRecord(e1, 0);
      hipStreamWaitEvent(s2, e1, 0);
      hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s2, d_o);
      hipEventRecord(e2, s2);
      hipStreamWaitEvent(0, e2, 0);
    });
    time_it("empty x2 same stream", [&] {
      hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0, d_o);
      hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0, d_o);
    });
  }
  time_it("load1 (256 x 256)", [&] { hipLaunchKernelGGL(k_load1, dim3(Q), dim3(256), 0, 0, d_i, d_o); });
  time_it("chain3 (256 x 256)", [&] { hipLaunchKernelGGL(k_chain3, dim3(Q), dim3(256), 0, 0, d_i, d_o, Q * 256); });
  time_it("copy_list (wave per query)", [&] {
    hipLaunchKernelGGL(k_copy_list, dim3(Q / 4), dim3(256), 0, 0, d_list, d_cnt, C, k, d_od, d_os);
  });
  time_it("merge_sorted W=8 k=100", [&] {
    hipLaunchKernelGGL(merge_sorted_kernel, dim3(Q / kQW), dim3(64 * kQW), 0, 0, d_pk,
                       reinterpret_cast<const float*>(d_pk) + (size_t)Q * k, W, (int64_t)Q, k,
                       (int64_t)2 * Q * k, d_od, d_os);
  });
  time_it("theta_wave W=8 S=80 k=100", [&] {
    hipLaunchKernelGGL(theta_wave_kernel, dim3((Q + kQW - 1) / kQW), dim3(64 * kQW), 0, 0, d_keys,
                       (int64_t)W, (int64_t)Q, (int64_t)S, k, d_theta, d_cnt, C, 1, (int64_t)0,
                       (int64_t)10000000, d_ctr);
  });
  // merge_fast on lists of n keys per query (unsorted shard mode and sorted)
  {
    int32_t *d_fb, *d_nflag, *d_slow, *d_ctrs;
    CK(hipMalloc(&d_fb, sizeof(int32_t) * Q));
    CK(hipMalloc(&d_nflag, sizeof(int32_t) * Q));
    CK(hipMalloc(&d_slow, sizeof(int32_t) * Q));
    CK(hipMalloc(&d_ctrs, sizeof(int32_t) * 64));
    std::vector<uint64_t> th(Q, 1ull << 32);
    CK(hipMemcpy(d_theta, th.data(), sizeof(uint64_t) * Q, hipMemcpyHostToDevice));
    for (int n : {30, 120, 231, 400}) {
      std::vector<uint64_t> lst((size_t)Q * C, 0ull);
      for (int q = 0; q < Q; ++q)
        for (int i = 0; i < n; ++i)
          lst[(size_t)q * C + i] = make_key(2.f + (float)(rng() % 100000) * 1e-4f,
                                            (uint32_t)(rng() % 10000000));
      CK(hipMemcpy(d_list, lst.data(), sizeof(uint64_t) * lst.size(), hipMemcpyHostToDevice));
      std::vector<int32_t> hn(Q, n);
      CK(hipMemcpy(d_cnt, hn.data(), sizeof(int32_t) * Q, hipMemcpyHostToDevice));
      for (int uns = 0; uns < 2; ++uns) {
        Stage sg{};
        sg.theta = d_theta;
        sg.list = d_list;
        sg.list_cnt = d_cnt;
        sg.C = C;
        sg.fb = d_fb;
        sg.fb_cnt = d_ctrs + 2;
        sg.nq_host = Q;
        sg.unsorted = uns != 0;
        Workspace ws{};
        ws.nflag = d_nflag;
        ws.slow = d_slow;
        ws.counters = d_ctrs;
        char name[96];
        snprintf(name, sizeof name, "merge_fast n=%d %s k=100", n, uns ? "unsorted" : "sorted");
        time_it(name, [&] {
          hipLaunchKernelGGL(merge_fast_kernel, dim3(Q / kQW), dim3(64 * kQW), 0, 0, sg, k,
                             (int64_t)0, ws, d_od, d_os);
        });
      }
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
