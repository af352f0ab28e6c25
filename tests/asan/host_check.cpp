// Host-side check of libbm25mi's C-ABI under AddressSanitizer (SURVEY.md:235;
// VERDICT r4 item 8).  Built by tests/test_host.py::test_capi_host_asan with
// every source compiled for the host only (--cuda-host-only) and
// -fsanitize=address, and run where no GPU is visible: every argument check,
// error message and early-exit path of the boundary runs, the device calls
// fail with EHIP, and ASan reports any out-of-bounds or use-after-free on the
// way (the process exits non-zero).
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bm25mi.h"

static int failures = 0;

static void expect(int rc, int want, const char* what, const char* msg_part = nullptr) {
  const std::string msg = bm25_last_error();
  const bool ok = rc == want && (!msg_part || msg.find(msg_part) != std::string::npos);
  if (!ok) {
    std::printf("FAIL %s: rc=%d want=%d msg='%s'\n", what, rc, want, msg.c_str());
    ++failures;
  }
}

int main() {
  if (bm25_abi_version() != BM25MI_ABI_VERSION) ++failures;
  const int ndev = bm25_device_count();
  // a small valid CSC: 3 terms over 5 documents
  std::vector<int64_t> ip = {0, 2, 2, 5};
  std::vector<int32_t> ix = {0, 3, 1, 2, 4};
  std::vector<float> dt = {1.f, 2.f, 0.5f, 0.25f, 3.f};
  bm25_index* h = nullptr;
  expect(bm25_index_create(0, 5, 3, 5, ip.data(), 1, ix.data(), dt.data(), 0, nullptr),
         BM25_EINVAL, "out NULL");
  expect(bm25_index_create(0, -1, 3, 5, ip.data(), 1, ix.data(), dt.data(), 0, &h), BM25_EINVAL,
         "negative", "negative size");
  expect(bm25_index_create(0, 5, 3, 5, nullptr, 1, ix.data(), dt.data(), 0, &h), BM25_EINVAL,
         "NULL indptr", "NULL CSC");
  std::vector<int64_t> bad = {0, 3, 2, 5};
  expect(bm25_index_create(0, 5, 3, 5, bad.data(), 1, ix.data(), dt.data(), 0, &h), BM25_EINVAL,
         "decreasing", "decreases");
  std::vector<int64_t> end = {0, 2, 2, 4};
  expect(bm25_index_create(0, 5, 3, 5, end.data(), 1, ix.data(), dt.data(), 0, &h), BM25_EINVAL,
         "end", "end at nnz");
  std::vector<int32_t> ip32 = {0, 6, 6, 6};
  std::vector<int32_t> ix6(6, 0);
  std::vector<float> dt6(6, 1.f);
  expect(bm25_index_create(0, 5, 3, 6, ip32.data(), 0, ix6.data(), dt6.data(), 0, &h),
         BM25_EINVAL, "column longer than n_docs", "more entries");
  expect(bm25_index_create(0, 5, 3, 5, ip.data(), 1, ix.data(), dt.data(), -4, &h), BM25_EINVAL,
         "doc_offset", "doc_offset");
  expect(bm25_index_create(0, (int64_t)1 << 40, 3, 5, ip.data(), 1, ix.data(), dt.data(), 0, &h),
         BM25_EINVAL, "n_docs range");
  // a wide vocabulary: the host copy of indptr is O(V)
  const int64_t V = 200000;
  std::vector<int64_t> wide(V + 1, 0);
  for (int64_t t = 0; t <= V; ++t) wide[t] = t < 5 ? t : 5;
  if (ndev == 0) {
    expect(bm25_index_create(0, 5, 3, 5, ip.data(), 1, ix.data(), dt.data(), 0, &h), BM25_EHIP,
           "no GPU", "no HIP device");
    std::vector<int32_t> wix = {0, 1, 2, 3, 4};
    expect(bm25_index_create(0, 5, V, 5, wide.data(), 1, wix.data(), dt.data(), 0, &h), BM25_EHIP,
           "no GPU, wide", "no HIP device");
    int devs[2] = {0, 0};
    bm25_sharded* s = nullptr;
    expect(bm25_sharded_create(2, devs, 5, 3, 5, ip.data(), 1, ix.data(), dt.data(), &s),
           BM25_EHIP, "sharded, no GPU", "no HIP device");
    std::vector<int32_t> docs = {0, 1, 1}, terms = {0, 0, 2}, dl = {3, 4};
    std::vector<float> tf = {1.f, 2.f, 1.f};
    std::vector<int64_t> oip(4);
    std::vector<int32_t> oix(3);
    std::vector<float> odt(3);
    expect(bm25_build_scores(0, 2, 3, 3, docs.data(), terms.data(), tf.data(), dl.data(), 3.5, 1.5,
                             0.75, 0, nullptr, oip.data(), oix.data(), odt.data(), nullptr),
           BM25_EHIP, "build, no GPU", "no HIP device");
  }
  int devs[1] = {0};
  bm25_sharded* s = nullptr;
  expect(bm25_sharded_create(0, devs, 5, 3, 5, ip.data(), 1, ix.data(), dt.data(), &s), BM25_EINVAL,
         "sharded n_dev", "at least one device");
  expect(bm25_sharded_create(1, devs, 5, 3, 5, bad.data(), 1, ix.data(), dt.data(), &s),
         BM25_EINVAL, "sharded decreasing", "decreases");
  std::vector<int32_t> docs = {0, 1}, terms = {0, 7};
  std::vector<float> tf = {1.f, 1.f};
  std::vector<int32_t> dl = {1, 1};
  std::vector<int64_t> oip(4);
  std::vector<int32_t> oix(2);
  std::vector<float> odt(2);
  expect(bm25_build_scores(0, -2, 3, 2, docs.data(), terms.data(), tf.data(), dl.data(), 1.0, 1.5,
                           0.75, 0, nullptr, oip.data(), oix.data(), odt.data(), nullptr),
         BM25_EINVAL, "build negative", "negative size");
  expect(bm25_build_scores(0, 2, 3, 2, docs.data(), terms.data(), tf.data(), dl.data(), 1.0, 1.5,
                           0.75, 9, nullptr, oip.data(), oix.data(), odt.data(), nullptr),
         BM25_EINVAL, "build method", "unknown method");
  expect(bm25_build_scores(0, 2, 3, 2, nullptr, terms.data(), tf.data(), dl.data(), 1.0, 1.5, 0.75,
                           0, nullptr, oip.data(), oix.data(), odt.data(), nullptr),
         BM25_EINVAL, "build NULL", "NULL argument");
  // every entry point that takes a handle rejects NULL
  int32_t q[2] = {0, 1}, od[2];
  float os[2];
  double od64[2];
  int64_t v64 = 0, cnt[5];
  int32_t i32 = 0;
  uint32_t u32 = 0;
  expect(bm25_search(nullptr, q, 1, 2, 1, od, os), BM25_EINVAL, "search NULL");
  expect(bm25_search_device(nullptr, q, 1, 2, 1, od, os, nullptr), BM25_EINVAL, "device NULL");
  expect(bm25_scores_dense(nullptr, q, 2, os), BM25_EINVAL, "dense NULL");
  expect(bm25_scores_dense_f64(nullptr, q, 2, od64), BM25_EINVAL, "dense64 NULL");
  expect(bm25_topn_f64(nullptr, q, 2, 1, od, od64), BM25_EINVAL, "topn64 NULL");
  expect(bm25_index_set_values_f64(nullptr, od64), BM25_EINVAL, "values64 NULL");
  expect(bm25_index_fork(nullptr, nullptr), BM25_EINVAL, "fork NULL");
  bm25_index* f = nullptr;
  expect(bm25_index_fork(nullptr, &f), BM25_EINVAL, "fork NULL base", "unbuilt");
  expect(bm25_index_info(nullptr, &v64, &v64, &v64, &i32, &v64, &v64), BM25_EINVAL, "info NULL");
  expect(bm25_index_segments(nullptr, &i32, &v64), BM25_EINVAL, "segments NULL");
  expect(bm25_index_bounds(nullptr, &i32, &v64), BM25_EINVAL, "bounds NULL");
  expect(bm25_index_set_option(nullptr, "flat", 1), BM25_EINVAL, "set_option NULL");
  expect(bm25_index_get_option(nullptr, "flat", &v64), BM25_EINVAL, "get_option NULL");
  expect(bm25_search_dispatch(nullptr, &u32, &i32, &i32, &i32), BM25_EINVAL, "dispatch NULL");
  expect(bm25_search_stats(nullptr, &v64, &v64), BM25_EINVAL, "stats NULL");
  expect(bm25_search_stats_ex(nullptr, &v64, &v64, &v64), BM25_EINVAL, "stats_ex NULL");
  expect(bm25_search_counters(nullptr, cnt, 5), BM25_EINVAL, "counters NULL");
  expect(bm25_profile_enable(nullptr, 1), BM25_EINVAL, "profile NULL");
  expect(bm25_sample_width(nullptr, 10, 1, 10, &v64), BM25_EINVAL, "width NULL");
  expect(bm25_search_sample_device(nullptr, q, 1, 2, 1, 1, 10, nullptr, nullptr), BM25_EINVAL,
         "sample NULL");
  expect(bm25_search_finish_device(nullptr, q, 1, 2, 1, 1, 10, nullptr, od, os, nullptr),
         BM25_EINVAL, "finish NULL");
  expect(bm25_sharded_search(nullptr, q, 1, 2, 1, od, os), BM25_EINVAL, "sharded search NULL");
  expect(bm25_merge_topk_device(0, nullptr, nullptr, 0, 1, 1, od, os, nullptr), BM25_EINVAL,
         "merge W", "bad merge shape");
  expect(bm25_merge_sorted_device(0, nullptr, nullptr, 2, 4, 3, 5, od, os, nullptr), BM25_EINVAL,
         "merge stride", "bad merge shape");
  expect(bm25_index_destroy(nullptr), BM25_OK, "destroy NULL");
  expect(bm25_sharded_destroy(nullptr), BM25_OK, "sharded destroy NULL");
  if (failures) {
    std::printf("%d failures\n", failures);
    return 1;
  }
  std::printf("asan host check ok (%d devices)\n", ndev);
  return 0;
}
