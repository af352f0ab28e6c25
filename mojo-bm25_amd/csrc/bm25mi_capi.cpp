// bm25mi_capi.cpp — the extern "C" boundary of libbm25mi.so (include/bm25mi.h).
//
// Host side of the drop-in: validation with the reference's error behaviour
// (bm25_native.py:105-127), index upload + device layout build, workspace
// management and the search pipeline (score_tiles -> merge -> rescore ->
// merge_final), all on one HIP stream per handle.
#include "../../include/bm25mi.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "bm25mi_internal.h"

using namespace bm25mi;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(e == hipErrorOutOfMemory ? BM25_ENOMEM : BM25_EHIP, "%s: %s (%s)", what,
              hipGetErrorString(e), hipGetErrorName(e));
}

#define HIP_TRY(expr, what)                 \
  do {                                      \
    hipError_t e_ = (expr);                 \
    if (e_ != hipSuccess) return hip_fail(e_, what); \
  } while (0)

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

struct EventPair {
  hipEvent_t a = nullptr, b = nullptr, c = nullptr;  // start, after score pass, end
  bool with_c = false;                                 // c recorded (profiling level 2)
};

// The device arrays of one built index, shared by the handle that built it
// and its forks (bm25_index_fork): freed when the last of them is destroyed.
struct IndexArrays {
  int device = 0;
  std::vector<void*> p;
  ~IndexArrays() {
    hipSetDevice(device);
    for (void* x : p) hipFree(x);
  }
};

}  // namespace

struct bm25_index {
  DevIndex ix;
  std::shared_ptr<IndexArrays> arrays;  // owner of ix's device arrays (null while building)
  hipStream_t stream = nullptr;
  Workspace ws;
  // host-call staging buffers (device)
  int32_t* d_q = nullptr;
  int32_t* d_docs = nullptr;
  float* d_scores = nullptr;
  int64_t cap_q_elems = 0, cap_out_elems = 0;
  std::mutex mu;
  // profiling
  int prof = 0;  // 1: score pass events (a, b) per search; 2: also the search's end (c)
  std::vector<EventPair> ev_pool;
  size_t ev_used = 0;
  double score_ms = 0.0, total_ms = 0.0;
  int64_t score_launches = 0, searches = 0, rescored = 0;
  int64_t device_bytes = 0;
  EventPair* split_ev = nullptr;  // events of a sample/finish search in flight
  hipEvent_t ws_done = nullptr;    // recorded on ws_stream when a search moves to another stream
  hipEvent_t ev_split[2] = {nullptr, nullptr};  // theta -> REST, REST -> select (three streams)
  hipStream_t ws_stream = nullptr; // the stream of the last search that used the workspace
  int32_t* d_maxtok = nullptr;     // bm25_max_token_device result
  bool sampled = false;            // a sample half ran since the last finish half
  // the threshold source (choose_theta_source): host-mapped report of the
  // searches' overflow, the search sequence, the last tile-bound search
  int32_t* report_host = nullptr;
  int32_t* report_dev = nullptr;
  int32_t seq = 0, last_bound_seq = -1, seen_seq = -1, weak_until = 0, backoff = 64;
  int64_t last_bound_q = 0;
  int64_t large_fallback = 0;  // queries of the last large-k list search taken by dense rows
                               // (-1: the dense path served the whole search)
  LargeArena arena;            // the large-k paths' scratch (grown to what they last asked for)
};

namespace {

void free_ws(Workspace& ws) {
  hipFree(ws.cand);
  hipFree(ws.theta);
  hipFree(ws.list);
  hipFree(ws.list_cnt);
  hipFree(ws.fb);
  hipFree(ws.cand2);
  hipFree(ws.flag_tiles);
  hipFree(ws.nflag);
  hipFree(ws.queue);
  hipFree(ws.counters);
  hipFree(ws.slow);
  hipFree(ws.wctr);
  hipFree(ws.seg);
  hipFree(ws.qw);
  hipFree(ws.sub);
  hipFree(ws.sub_ipb);
  hipFree(ws.sub_done);
  ws = Workspace{};
}

// Candidate-list capacity per query: the keys above theta of the non-sample
// tiles number about (P-1)*k; a list that overflows sends its query to the
// exact fallback stage (the list_cap option overrides, for tests).
int32_t list_cap_for(const SearchOpts& o, int64_t k) {
  if (o.list_cap > 0) return o.list_cap;
  return (int32_t)std::min<int64_t>(65536, std::max<int64_t>(2048, 64 * k));
}

// Options of a new handle: the BM25_* environment (include/bm25mi.h).
SearchOpts env_opts() {
  SearchOpts o;
  o.flat = env_int("BM25_FLAT", o.flat) != 0;
  o.flat_bw = env_int("BM25_FLAT_BW", o.flat_bw);
  o.items_per_wave = env_int("BM25_ITEMS_PER_WAVE", o.items_per_wave);
  o.sample_p = env_int("BM25_SAMPLE_P", o.sample_p);
  o.list_cap = env_int("BM25_LIST_CAP", o.list_cap);
  o.claim_ch = env_int("BM25_CLAIM_CH", o.claim_ch);
  o.claim_m = env_int("BM25_CLAIM_M", o.claim_m);
  o.tile_bound = env_int("BM25_TILE_BOUND", o.tile_bound) != 0;
  o.theta_bound = env_int("BM25_THETA_BOUND", o.theta_bound) != 0;
  o.grid_pct = std::min(100, std::max(1, env_int("BM25_GRID_PCT", o.grid_pct)));
  o.count_skips = env_int("BM25_COUNT_SKIPS", o.count_skips) != 0;
  o.large_lists = env_int("BM25_LARGE_LISTS", o.large_lists) != 0;
  o.rest_split = env_int("BM25_REST_SPLIT", o.rest_split) != 0;
  o.bound_pool = env_int("BM25_BOUND_POOL", o.bound_pool) != 0;
  return o;
}

// Sets one option (EINVAL names the accepted values).
int set_opt(SearchOpts& o, const char* name, int64_t v) {
  auto is_pow2 = [](int64_t x) { return x > 0 && (x & (x - 1)) == 0; };
  if (!name) return fail(BM25_EINVAL, "NULL option name");
  const std::string n = name;
  if (n == "flat") {
    if (v != 0 && v != 1) return fail(BM25_EINVAL, "flat must be 0 or 1");
    o.flat = (int)v;
  } else if (n == "flat_bw") {
    if (v != 0 && !(is_pow2(v) && v <= 8)) return fail(BM25_EINVAL, "flat_bw must be 0, 1, 2, 4 or 8");
    o.flat_bw = (int)v;
  } else if (n == "items_per_wave") {
    if (v < 1 || v > 1024) return fail(BM25_EINVAL, "items_per_wave must be in 1..1024");
    o.items_per_wave = (int)v;
  } else if (n == "sample_p") {
    if (!is_pow2(v) || v > 64) return fail(BM25_EINVAL, "sample_p must be a power of two in 1..64");
    o.sample_p = (int)v;
  } else if (n == "list_cap") {
    if (v < 0 || v > (1 << 20)) return fail(BM25_EINVAL, "list_cap must be in 0..2^20");
    o.list_cap = (int)v;
  } else if (n == "claim_ch") {
    if (v < 1 || v > 64) return fail(BM25_EINVAL, "claim_ch must be in 1..64");
    o.claim_ch = (int)v;
  } else if (n == "claim_m") {
    if (v < 1 || v > kClaimM) return fail(BM25_EINVAL, "claim_m must be in 1..%d", kClaimM);
    o.claim_m = (int)v;
  } else if (n == "tile_bound") {
    if (v != 0 && v != 1) return fail(BM25_EINVAL, "tile_bound must be 0 or 1");
    o.tile_bound = (int)v;
  } else if (n == "theta_bound") {
    if (v != 0 && v != 1) return fail(BM25_EINVAL, "theta_bound must be 0 or 1");
    o.theta_bound = (int)v;
  } else if (n == "large_lists") {
    if (v != 0 && v != 1) return fail(BM25_EINVAL, "large_lists must be 0 or 1");
    o.large_lists = (int)v;
  } else if (n == "rest_split") {
    if (v != 0 && v != 1) return fail(BM25_EINVAL, "rest_split must be 0 or 1");
    o.rest_split = (int)v;
  } else if (n == "bound_pool") {
    if (v != 0 && v != 1) return fail(BM25_EINVAL, "bound_pool must be 0 or 1");
    o.bound_pool = (int)v;
  } else if (n == "count_skips") {
    if (v != 0 && v != 1) return fail(BM25_EINVAL, "count_skips must be 0 or 1");
    o.count_skips = (int)v;
  } else if (n == "grid_pct") {
    if (v < 1 || v > 100) return fail(BM25_EINVAL, "grid_pct must be in 1..100");
    o.grid_pct = (int)v;
  } else {
    return fail(BM25_EINVAL, "unknown option '%s'", name);
  }
  return BM25_OK;
}

int get_opt(const SearchOpts& o, const char* name, int64_t* v) {
  if (!name || !v) return fail(BM25_EINVAL, "NULL argument");
  const std::string n = name;
  if (n == "flat") *v = o.flat;
  else if (n == "flat_bw") *v = o.flat_bw;
  else if (n == "items_per_wave") *v = o.items_per_wave;
  else if (n == "sample_p") *v = o.sample_p;
  else if (n == "list_cap") *v = o.list_cap;
  else if (n == "claim_ch") *v = o.claim_ch;
  else if (n == "claim_m") *v = o.claim_m;
  else if (n == "tile_bound") *v = o.tile_bound;
  else if (n == "theta_bound") *v = o.theta_bound;
  else if (n == "grid_pct") *v = o.grid_pct;
  else if (n == "count_skips") *v = o.count_skips;
  else if (n == "large_lists") *v = o.large_lists;
  else if (n == "rest_split") *v = o.rest_split;
  else if (n == "bound_pool") *v = o.bound_pool;
  else return fail(BM25_EINVAL, "unknown option '%s'", name);
  return BM25_OK;
}

// The workspace for a search of Q queries of T terms at k, enqueued on st.
// A (re)allocated workspace's counters are zeroed on st itself, so they are
// ordered before the search's first kernel on any stream, blocking or not
// (they were zeroed on the null stream once, which a non-blocking stream does
// not wait for: a fork's first search on a part stream read a half-zeroed
// claim counter and skipped items).
int ensure_ws(bm25_index* h, int64_t Q, int64_t T, int k, hipStream_t st) {
  Workspace& ws = h->ws;
  const int64_t need_seg = seg_entries(h->ix, std::max(Q, ws.cap_q), T);
  if (Q <= ws.cap_q && k <= ws.cap_k) {
    if (need_seg <= ws.cap_seg) return BM25_OK;
    // a wider query batch on a sparse index: only the segment table grows
    hipFree(ws.seg);
    ws.seg = nullptr;
    ws.cap_seg = 0;
    HIP_TRY(hipMalloc(&ws.seg, sizeof(uint64_t) * need_seg), "hipMalloc(seg)");
    ws.cap_seg = need_seg;
    return BM25_OK;
  }
  const int64_t q = std::max(Q, ws.cap_q);
  const int64_t kk = std::max<int64_t>(k, ws.cap_k);
  free_ws(ws);
  const int64_t nt = h->ix.ntiles;
  const int64_t mf = maxflag_for((int)kk, nt);
  const int32_t C = list_cap_for(h->ix.opt, kk);
  HIP_TRY(hipMalloc(&ws.cand, sizeof(uint64_t) * q * nt * kTileM), "hipMalloc(cand)");
  HIP_TRY(hipMalloc(&ws.theta, sizeof(uint64_t) * q), "hipMalloc(theta)");
  HIP_TRY(hipMalloc(&ws.list, sizeof(uint64_t) * q * C), "hipMalloc(list)");
  HIP_TRY(hipMalloc(&ws.list_cnt, sizeof(int32_t) * q), "hipMalloc(list_cnt)");
  HIP_TRY(hipMalloc(&ws.fb, sizeof(int32_t) * q), "hipMalloc(fb)");
  HIP_TRY(hipMalloc(&ws.cand2, sizeof(uint64_t) * q * mf * kk), "hipMalloc(cand2)");
  HIP_TRY(hipMalloc(&ws.flag_tiles, sizeof(int32_t) * q * mf), "hipMalloc(flag_tiles)");
  HIP_TRY(hipMalloc(&ws.nflag, sizeof(int32_t) * q), "hipMalloc(nflag)");
  HIP_TRY(hipMalloc(&ws.queue, sizeof(int32_t) * q * mf), "hipMalloc(queue)");
  HIP_TRY(hipMalloc(&ws.counters, sizeof(int32_t) * kCounters), "hipMalloc(counters)");
  HIP_TRY(hipMemsetAsync(ws.counters, 0, sizeof(int32_t) * kCounters, st), "hipMemsetAsync(counters)");
  HIP_TRY(hipMalloc(&ws.slow, sizeof(int32_t) * q), "hipMalloc(slow)");
  HIP_TRY(hipMalloc(&ws.wctr, sizeof(int32_t) * kWctrRegions * kWctrInts), "hipMalloc(wctr)");
  // claim counters start at 0; each flat launch's last wave re-zeroes its region
  HIP_TRY(hipMemsetAsync(ws.wctr, 0, sizeof(int32_t) * kWctrRegions * kWctrInts, st),
          "hipMemsetAsync(wctr)");
  // the split-item table of the REST pass (bound_keys_kernel builds it; its
  // finished-block count resets itself)
  HIP_TRY(hipMalloc(&ws.qw, sizeof(uint32_t) * q), "hipMalloc(qw)");
  HIP_TRY(hipMalloc(&ws.sub, sizeof(uint32_t) * q * 8), "hipMalloc(sub)");
  HIP_TRY(hipMalloc(&ws.sub_ipb, sizeof(int32_t)), "hipMalloc(sub_ipb)");
  HIP_TRY(hipMalloc(&ws.sub_done, sizeof(int32_t)), "hipMalloc(sub_done)");
  HIP_TRY(hipMemsetAsync(ws.sub_done, 0, sizeof(int32_t), st), "hipMemsetAsync(sub_done)");
  ws.cap_seg = need_seg;
  if (ws.cap_seg > 0) HIP_TRY(hipMalloc(&ws.seg, sizeof(uint64_t) * ws.cap_seg), "hipMalloc(seg)");
  ws.list_cap = C;
  ws.cap_q = q;
  ws.cap_k = kk;
  return BM25_OK;
}

int ensure_io(bm25_index* h, int64_t q_elems, int64_t out_elems) {
  if (q_elems > h->cap_q_elems) {
    hipFree(h->d_q);
    h->d_q = nullptr;
    HIP_TRY(hipMalloc(&h->d_q, sizeof(int32_t) * std::max<int64_t>(q_elems, 1)), "hipMalloc(queries)");
    h->cap_q_elems = q_elems;
  }
  if (out_elems > h->cap_out_elems) {
    hipFree(h->d_docs);
    hipFree(h->d_scores);
    h->d_docs = nullptr;
    h->d_scores = nullptr;
    HIP_TRY(hipMalloc(&h->d_docs, sizeof(int32_t) * std::max<int64_t>(out_elems, 1)), "hipMalloc(docs)");
    HIP_TRY(hipMalloc(&h->d_scores, sizeof(float) * std::max<int64_t>(out_elems, 1)), "hipMalloc(scores)");
    h->cap_out_elems = out_elems;
  }
  return BM25_OK;
}

void harvest_events(bm25_index* h) {
  if (h->ev_used == 0) return;
  for (size_t i = 0; i < h->ev_used; ++i) {
    float ms1 = 0.f, ms2 = 0.f;
    const bool tot = h->ev_pool[i].with_c;
    hipEventSynchronize(tot ? h->ev_pool[i].c : h->ev_pool[i].b);  // (maybe a caller's stream)
    hipEventElapsedTime(&ms1, h->ev_pool[i].a, h->ev_pool[i].b);
    if (tot) hipEventElapsedTime(&ms2, h->ev_pool[i].a, h->ev_pool[i].c);
    h->score_ms += ms1;
    h->total_ms += tot ? ms2 : ms1;
  }
  h->ev_used = 0;
}

EventPair* next_events(bm25_index* h) {
  if (!h->prof) return nullptr;
  if (h->ev_used == h->ev_pool.size()) {
    if (h->ev_pool.size() < 512) {
      EventPair p;
      hipEventCreate(&p.a);
      hipEventCreate(&p.b);
      hipEventCreate(&p.c);
      h->ev_pool.push_back(p);
    } else {
      harvest_events(h);
    }
  }
  EventPair* e = &h->ev_pool[h->ev_used++];
  e->with_c = h->prof >= 2;
  return e;
}

// Records the search's end event of a profiled search (level 2 only: every
// event record is a marker packet the device spends ~4 us on).
hipError_t record_end(bm25_index* h, EventPair* ev, hipStream_t st) {
  return (ev && ev->with_c) ? hipEventRecord(ev->c, st) : hipSuccess;
}

// The workspace is shared by every search on the handle: a search enqueued
// on another stream than the previous one first waits for everything
// enqueued on that stream so far (ws_done, recorded there now).  Searches
// that stay on one stream record nothing: an event record costs the device
// a marker packet (~4 us, measured: scripts/dev/latency_bench.hip), a
// cross-stream wait more.  The previous search's stream must still exist
// (torch's pooled streams do).
hipError_t order_ws(bm25_index* h, hipStream_t st) {
  if (h->ws_stream == nullptr || st == h->ws_stream) {
    h->ws_stream = st;
    return hipSuccess;
  }
  if (!h->ws_done) {
    const hipError_t e = hipEventCreateWithFlags(&h->ws_done, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  hipError_t e = hipEventRecord(h->ws_done, h->ws_stream);
  if (e == hipSuccess) e = hipStreamWaitEvent(st, h->ws_done, 0);
  h->ws_stream = st;
  return e;
}

// The host waits for the workspace's last search (its stream).
void ws_wait_host(bm25_index* h) {
  if (h->ws_stream) hipStreamSynchronize(h->ws_stream);
}

// The threshold source of the handle's next search (DevIndex::bound_weak).
// A search that took the tile-bound threshold and sent more than 1/16 of its
// queries to the exact fallback stage — their candidate lists overflowed:
// the single-term tile maxima sit far below the best sums, as on an index
// whose terms all weigh alike — turns that threshold off for the next
// `backoff` searches (64, doubling while it keeps failing, at most 4096),
// which take the sampled threshold instead.  The overflow comes from the
// host-mapped report merge_tail_kernel writes at the end of a search: no
// wait — a report not written yet leaves the choice as it is.  Every choice
// is exact; only the cost differs.  Caller holds h->mu.
void choose_theta_source(bm25_index* h) {
  ++h->seq;
  if (h->report_host && h->last_bound_seq >= 0 && h->seen_seq != h->last_bound_seq) {
    const int32_t r = __atomic_load_n(h->report_host + 1, __ATOMIC_ACQUIRE);
    if (r == h->last_bound_seq) {
      h->seen_seq = r;
      const int64_t nf = __atomic_load_n(h->report_host, __ATOMIC_RELAXED);
      if (nf * 16 > h->last_bound_q) {
        h->weak_until = h->seq + h->backoff;
        h->backoff = std::min(2 * h->backoff, 4096);
      } else {
        h->backoff = 64;
      }
    }
  }
  h->ix.bound_weak = h->seq < h->weak_until;
}

// The search's report slot and sequence number in the workspace (after
// ensure_ws, which may rebuild it); P = 0: it took the tile-bound threshold.
void arm_report(bm25_index* h, int P, int64_t Q) {
  h->ws.report = h->report_dev;
  h->ws.seq = h->seq;
  if (h->ix.bound_weak) h->ix.disp.kernels |= kKBoundOff;
  if (P == 0) {
    h->last_bound_seq = h->seq;
    h->last_bound_q = Q;
  }
}

void alloc_report(bm25_index* h) {
  if (hipHostMalloc((void**)&h->report_host, 2 * sizeof(int32_t), hipHostMallocMapped) !=
      hipSuccess) {
    (void)hipGetLastError();
    h->report_host = nullptr;
    return;
  }
  h->report_host[0] = 0;
  h->report_host[1] = -1;
  if (hipHostGetDevicePointer((void**)&h->report_dev, h->report_host, 0) != hipSuccess) {
    (void)hipGetLastError();
    hipHostFree(h->report_host);
    h->report_host = h->report_dev = nullptr;
  }
}

// Device pipeline on stream st; caller holds h->mu and has set the device.
// shard: bm25_search_shard_device — the collection's threshold from the
// world bounds and this shard's keys >= it, unsorted, for the W-way merge.
int run_search(bm25_index* h, const int32_t* d_queries, int64_t Q, int64_t T, int k,
               int32_t* d_docs, float* d_scores, hipStream_t st, bool shard = false) {
  if (Q == 0 || k == 0) return BM25_OK;
  if (k > kMaxK) {  // any k up to n_docs: the large-k path (bm25mi_large.hip)
    // the list path when it applies (no dense score rows), else dense rows
    const bool lists = h->ix.opt.large_lists && k <= kLargeListMaxK && k <= h->ix.n_docs &&
                       large_list_supported(h->ix, T, Q) && large_geom(h->ix, k).P > 0;
    if (lists) {
      const int rc = ensure_ws(h, Q, T, 1, st);  // claim counters, counters, segment table
      if (rc) return rc;
    }
    // the scratch the large-k paths last asked for, allocated once for the
    // next ones (the device is done with the old arena: its last search is)
    if (h->arena.need > h->arena.bytes) {
      if (h->ws_stream) HIP_TRY(hipStreamSynchronize(h->ws_stream), "hipStreamSynchronize");
      hipFree(h->arena.base);
      h->arena.base = nullptr;
      h->arena.bytes = 0;
      HIP_TRY(hipMalloc((void**)&h->arena.base, h->arena.need), "hipMalloc(large-k scratch)");
      h->arena.bytes = h->arena.need;
    }
    h->arena.used = 0;
    h->ws.arena = &h->arena;
    HIP_TRY(order_ws(h, st), "workspace order");
    // this search selects without the counters: the stats read as zero, not
    // as the previous search's
    if (h->ws.counters)
      HIP_TRY(hipMemsetAsync(h->ws.counters, 0, sizeof(int32_t) * kCounters, st), "hipMemsetAsync");
    h->ix.disp = Dispatch{};
    h->ix.disp.sample_p = 1;
    EventPair* ev = next_events(h);
    if (ev) HIP_TRY(hipEventRecord(ev->a, st), "hipEventRecord");
    if (lists) {
      int64_t nfb = 0;
      HIP_TRY(launch_search_large_lists(h->ix, d_queries, Q, T, k, h->ws, d_docs, d_scores, &nfb, st),
              "large-k list search");
      h->large_fallback = nfb;
    } else {
      h->large_fallback = -1;
      HIP_TRY(launch_search_large(h->ix, d_queries, Q, T, k, d_docs, d_scores, st, &h->arena),
              "large-k search launch");
    }
    if (ev) {
      HIP_TRY(hipEventRecord(ev->b, st), "hipEventRecord");
      HIP_TRY(record_end(h, ev, st), "hipEventRecord");
    }
    if (h->prof) {
      h->score_launches += 1;
      h->searches += 1;
    }
    return BM25_OK;
  }
  int rc = ensure_ws(h, Q, T, k, st);
  if (rc) return rc;
  HIP_TRY(order_ws(h, st), "workspace order");
  h->large_fallback = 0;  // (counter [5] belongs to the last search: no large-k rows here)
  choose_theta_source(h);
  const int P = shard_geom_world(h->ix, k, T, shard).P;
  h->ix.disp = Dispatch{};
  h->ix.disp.sample_p = P;
  arm_report(h, P, Q);
  EventPair* ev = next_events(h);
  if (ev) HIP_TRY(hipEventRecord(ev->a, st), "hipEventRecord");
  HIP_TRY(launch_score(h->ix, d_queries, Q, T, k, h->ws, st, shard), "score launch");
  if (ev) HIP_TRY(hipEventRecord(ev->b, st), "hipEventRecord");
  HIP_TRY(launch_select(h->ix, d_queries, Q, T, k, P, h->ws, d_docs, d_scores, st, shard),
          "select launch");
  HIP_TRY(record_end(h, ev, st), "hipEventRecord");
  if (h->prof) {
    h->score_launches += 1;
    h->searches += 1;
  }
  return BM25_OK;
}

// Counters of the last search (caller holds h->mu); the search may run on a
// caller's stream: wait for that stream, not for the device.
void read_counters(bm25_index* h, int32_t (&cnt)[kCounters]) {
  if (!h->ws.counters) return;
  ws_wait_host(h);
  hipMemcpyAsync(cnt, h->ws.counters, sizeof cnt, hipMemcpyDeviceToHost, h->stream);
  hipStreamSynchronize(h->stream);
}

// shard = true: the index is one doc shard of a larger collection, whose
// [Q, k] lists are padded (doc -1, score bits ~0) where it holds fewer than k
// documents; otherwise k > n_docs is numpy's argpartition error (the
// reference's behaviour, bm25_native.py:205).
int check_k(const bm25_index* h, int64_t k, bool shard = false) {
  if (k < 0) return fail(BM25_EINVAL, "negative dimensions are not allowed (top_k=%lld)", (long long)k);
  if (!shard && k > h->ix.n_docs)
    return fail(BM25_EINVAL, "kth(=%lld) out of bounds (%lld)", (long long)(h->ix.n_docs - k),
                (long long)h->ix.n_docs);
  return BM25_OK;
}

}  // namespace

extern "C" {

int bm25_abi_version(void) { return BM25MI_ABI_VERSION; }

const char* bm25_last_error(void) { return g_err.c_str(); }

int bm25_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int bm25_index_create(int device, int64_t n_docs, int64_t n_terms, int64_t nnz,
                      const void* indptr, int indptr_is_i64, const int32_t* indices,
                      const float* data, int64_t doc_offset, bm25_index** out) {
  if (!out) return fail(BM25_EINVAL, "out is NULL");
  *out = nullptr;
  if (n_docs < 0 || n_terms < 0 || nnz < 0)
    return fail(BM25_EINVAL, "negative size (n_docs=%lld n_terms=%lld nnz=%lld)",
                (long long)n_docs, (long long)n_terms, (long long)nnz);
  if (n_docs > INT32_MAX) return fail(BM25_EINVAL, "n_docs=%lld exceeds int32 doc ids", (long long)n_docs);
  if (doc_offset < 0 || doc_offset + n_docs > (int64_t)INT32_MAX + 1)
    return fail(BM25_EINVAL, "doc_offset=%lld out of int32 range", (long long)doc_offset);
  if (!indptr || (nnz > 0 && (!indices || !data)))
    return fail(BM25_EINVAL, "NULL CSC array");
  // indptr on the host: int64, validated O(V)
  std::vector<int64_t> ip(n_terms + 1);
  for (int64_t t = 0; t <= n_terms; ++t)
    ip[t] = indptr_is_i64 ? ((const int64_t*)indptr)[t] : (int64_t)((const int32_t*)indptr)[t];
  if (ip[0] != 0 || ip[n_terms] != nnz)
    return fail(BM25_EINVAL, "indptr must start at 0 and end at nnz (got %lld..%lld, nnz=%lld)",
                (long long)ip[0], (long long)ip[n_terms], (long long)nnz);
  for (int64_t t = 0; t < n_terms; ++t) {
    if (ip[t + 1] < ip[t]) return fail(BM25_EINVAL, "indptr decreases at column %lld", (long long)t);
    if (ip[t + 1] - ip[t] > n_docs)
      return fail(BM25_EINVAL, "column %lld has more entries than n_docs", (long long)t);
  }
  const int shift = build_tile_shift();
  const int64_t ntiles = (n_docs + (1LL << shift) - 1) >> shift;
  if (ntiles > 65536) return fail(BM25_EINVAL, "n_docs=%lld needs %lld tiles (> 65536)", (long long)n_docs, (long long)ntiles);

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(BM25_EHIP, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(BM25_EINVAL, "device %d out of range (%d visible)", device, ndev);
  HIP_TRY(hipSetDevice(device), "hipSetDevice");

  bm25_index* h = new bm25_index();
  DevIndex& ix = h->ix;
  ix.opt = env_opts();
  ix.device = device;
  ix.n_docs = n_docs;
  ix.n_terms = n_terms;
  ix.nnz = nnz;
  ix.doc_offset = doc_offset;
  ix.tile_shift = shift;
  ix.ntiles = ntiles;
  int32_t* d_indices = nullptr;
  int32_t* d_err = nullptr;
  auto cleanup = [&](int rc) {
    hipFree(d_indices);
    hipFree(d_err);
    if (rc != BM25_OK) bm25_index_destroy(h);
    return rc;
  };
  hipError_t e;
#define TRYC(expr, what)                                          \
  do {                                                            \
    e = (expr);                                                   \
    if (e != hipSuccess) return cleanup(hip_fail(e, what));       \
  } while (0)
  TRYC(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking), "hipStreamCreate");
  alloc_report(h);
  // segment table form (DevIndex): BM25_SEGMENTS=dense|sparse; by default the
  // dense V x (ntiles+1) table (O(1) lookups, no per-search table: config 5's
  // 24 GB per rank ran 6 % faster than the tile lists) unless it would
  // outgrow both twice the posting arrays (6 B per posting) and 1/8 of the
  // device's memory — then the O(pairs) tile lists
  const int64_t rel_elems = n_terms * (ntiles + 1);
  {
    const char* m = getenv("BM25_SEGMENTS");
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) total_b = 0;
    const int64_t rel_bytes = rel_elems * 4;
    if (m && !strcmp(m, "sparse")) ix.sparse = true;
    else if (m && !strcmp(m, "dense")) ix.sparse = false;
    else ix.sparse = rel_bytes > 2 * 6 * std::max<int64_t>(nnz, 1) &&
                     rel_bytes > (int64_t)(total_b / 8);
  }
  TRYC(hipMalloc(&ix.indptr, sizeof(int64_t) * (n_terms + 1)), "hipMalloc(indptr)");
  if (!ix.sparse)
    TRYC(hipMalloc(&ix.rel, sizeof(uint32_t) * std::max<int64_t>(rel_elems, 1)), "hipMalloc(rel)");
  TRYC(hipMalloc(&ix.ldoc, sizeof(uint16_t) * (nnz + kPostingPad)), "hipMalloc(ldoc)");
  TRYC(hipMalloc(&ix.val, sizeof(float) * (nnz + kPostingPad)), "hipMalloc(val)");
  TRYC(hipMemsetAsync(ix.ldoc + nnz, 0, sizeof(uint16_t) * kPostingPad, h->stream), "hipMemset");
  TRYC(hipMemsetAsync(ix.val + nnz, 0, sizeof(float) * kPostingPad, h->stream), "hipMemset");
  TRYC(hipMalloc(&d_indices, sizeof(int32_t) * std::max<int64_t>(nnz, 1)), "hipMalloc(indices)");
  TRYC(hipMalloc(&d_err, sizeof(int32_t)), "hipMalloc(err)");
  h->device_bytes = (int64_t)(sizeof(int64_t) * (n_terms + 1) +
                              (ix.sparse ? 0 : sizeof(uint32_t) * rel_elems) +
                              (sizeof(uint16_t) + sizeof(float)) * nnz);
  TRYC(hipMemsetAsync(d_err, 0, sizeof(int32_t), h->stream), "hipMemset");
  TRYC(hipMemcpyAsync(ix.indptr, ip.data(), sizeof(int64_t) * (n_terms + 1), hipMemcpyHostToDevice, h->stream), "H2D indptr");
  if (nnz > 0) {
    TRYC(hipMemcpyAsync(d_indices, indices, sizeof(int32_t) * nnz, hipMemcpyHostToDevice, h->stream), "H2D indices");
    TRYC(hipMemcpyAsync(ix.val, data, sizeof(float) * nnz, hipMemcpyHostToDevice, h->stream), "H2D data");
  }
  if (!ix.sparse) {
    TRYC(launch_build_tables(ix, d_indices, d_err, h->stream), "build_tables launch");
  } else {  // tile lists: count per term, scan on the host, fill
    int64_t* d_cnt = nullptr;
    TRYC(hipMalloc(&d_cnt, sizeof(int64_t) * std::max<int64_t>(n_terms, 1)), "hipMalloc(cnt)");
    std::vector<int64_t> cnt(n_terms + 1, 0);
    e = launch_count_tiles(ix, d_indices, d_cnt, d_err, h->stream);
    if (e == hipSuccess && n_terms > 0)
      e = hipMemcpyAsync(cnt.data() + 1, d_cnt, sizeof(int64_t) * n_terms, hipMemcpyDeviceToHost,
                         h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    hipFree(d_cnt);
    if (e != hipSuccess) return cleanup(hip_fail(e, "count_tiles"));
    for (int64_t t = 0; t < n_terms; ++t) cnt[t + 1] += cnt[t];
    ix.n_pairs = cnt[n_terms];
    TRYC(hipMalloc(&ix.tl_ptr, sizeof(int64_t) * (n_terms + 1)), "hipMalloc(tl_ptr)");
    TRYC(hipMalloc(&ix.tl_tile, sizeof(uint16_t) * std::max<int64_t>(ix.n_pairs, 1)), "hipMalloc(tl_tile)");
    TRYC(hipMalloc(&ix.tl_start, sizeof(uint32_t) * std::max<int64_t>(ix.n_pairs, 1)), "hipMalloc(tl_start)");
    TRYC(hipMemcpyAsync(ix.tl_ptr, cnt.data(), sizeof(int64_t) * (n_terms + 1), hipMemcpyHostToDevice, h->stream), "H2D tl_ptr");
    TRYC(launch_fill_tiles(ix, d_indices, h->stream), "fill_tiles launch");
    TRYC(hipStreamSynchronize(h->stream), "fill_tiles");
    h->device_bytes += (int64_t)(sizeof(int64_t) * (n_terms + 1) +
                                 (sizeof(uint16_t) + sizeof(uint32_t)) * ix.n_pairs);
  }
  // values 0 or normal positive (no NaN, no denormal): every doc's running
  // sum only grows and is 0 or >= FLT_MIN, which lets the REST pass flag
  // candidates while adding and complete rare queries with zero-score docs
  // (bm25mi_kernels.hip)
  ix.nonneg = true;
  for (int64_t p = 0; p < nnz && ix.nonneg; ++p)
    ix.nonneg = data[p] == 0.0f || data[p] >= 1.17549435e-38f;
  // tile bounds of the REST pass (dense table, non-negative index); without
  // the memory the search simply runs without them
  if (!ix.sparse && ix.nonneg && n_terms > 0 && ntiles > 0) {
    if (hipMalloc(&ix.bmax, sizeof(uint16_t) * n_terms * bmax_stride(ntiles)) == hipSuccess) {
      TRYC(launch_build_bmax(ix, h->stream), "build_bmax launch");
      h->device_bytes += (int64_t)(sizeof(uint16_t) * n_terms * bmax_stride(ntiles));
      // the pooled copy of the threshold kernel (a quarter of the bytes; optional)
      const int64_t ps = bmax_stride((ntiles + kPool - 1) / kPool);
      if (hipMalloc(&ix.bpool, sizeof(uint16_t) * n_terms * ps) == hipSuccess) {
        ix.pstride = ps;
        TRYC(launch_pool_bounds(ix.bmax, n_terms, bmax_stride(ntiles), ix.bpool, ps, h->stream),
             "pool_bounds launch");
        h->device_bytes += (int64_t)(sizeof(uint16_t) * n_terms * ps);
      } else {
        (void)hipGetLastError();
        ix.bpool = nullptr;
      }
    } else {
      (void)hipGetLastError();
      ix.bmax = nullptr;
    }
  }
  int32_t herr = 0;
  TRYC(hipMemcpyAsync(&herr, d_err, sizeof(int32_t), hipMemcpyDeviceToHost, h->stream), "D2H err");
  TRYC(hipStreamSynchronize(h->stream), "build sync");
#undef TRYC
  if (herr)
    return cleanup(fail(BM25_EINVAL,
                        "indices must be sorted, unique and in [0, n_docs) within every column "
                        "(canonical CSC)"));
  h->arrays = std::make_shared<IndexArrays>();
  h->arrays->device = device;
  h->arrays->p = {ix.indptr, ix.rel, ix.tl_ptr, ix.tl_tile, ix.tl_start, ix.ldoc, ix.val, ix.bmax,
                  ix.bpool};
  *out = h;
  return cleanup(BM25_OK);
}

int bm25_index_destroy(bm25_index* h) {
  if (!h) return BM25_OK;
  hipSetDevice(h->ix.device);
  if (h->stream) hipStreamSynchronize(h->stream);
  // a search on a caller's stream (which the caller may have destroyed since:
  // the device, not the stream)
  if (h->ws_stream) hipDeviceSynchronize();
  for (auto& p : h->ev_pool) {
    hipEventDestroy(p.a);
    hipEventDestroy(p.b);
    hipEventDestroy(p.c);
  }
  if (h->ws_done) hipEventDestroy(h->ws_done);
  for (hipEvent_t e : h->ev_split)
    if (e) hipEventDestroy(e);
  free_ws(h->ws);
  hipFree(h->arena.base);
  hipFree(h->d_q);
  hipFree(h->d_docs);
  hipFree(h->d_scores);
  hipFree(h->d_maxtok);
  if (h->report_host) hipHostFree(h->report_host);
  if (h->arrays) {
    h->arrays.reset();  // the index arrays go with the last handle sharing them
  } else {              // a create that failed part-way
    for (void* x : {(void*)h->ix.indptr, (void*)h->ix.rel, (void*)h->ix.tl_ptr,
                    (void*)h->ix.tl_tile, (void*)h->ix.tl_start, (void*)h->ix.ldoc,
                    (void*)h->ix.val, (void*)h->ix.bmax, (void*)h->ix.bpool})
      hipFree(x);
  }
  hipFree(h->ix.wbpool);  // (the handle's own pooled world bounds)
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return BM25_OK;
}

static int pool_world(bm25_index* h);

int bm25_index_fork(bm25_index* base, bm25_index** out) {
  if (!out) return fail(BM25_EINVAL, "out is NULL");
  *out = nullptr;
  if (!base || !base->arrays) return fail(BM25_EINVAL, "NULL or unbuilt index");
  std::lock_guard<std::mutex> lk(base->mu);
  HIP_TRY(hipSetDevice(base->ix.device), "hipSetDevice");
  bm25_index* h = new bm25_index();
  h->ix = base->ix;  // the same device arrays and options; its own dispatch report
  h->ix.disp = Dispatch{};
  h->ix.wbpool = nullptr;  // (the base's own; the fork pools the world table itself, below)
  h->arrays = base->arrays;
  h->device_bytes = base->device_bytes;
  const hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    bm25_index_destroy(h);
    return hip_fail(e, "hipStreamCreate");
  }
  alloc_report(h);
  if (h->ix.wbmax) {
    const int rc = pool_world(h);
    if (rc) {
      bm25_index_destroy(h);
      return rc;
    }
  }
  *out = h;
  return BM25_OK;
}

int bm25_index_info(const bm25_index* h, int64_t* n_docs, int64_t* n_terms, int64_t* nnz,
                    int32_t* tile_docs, int64_t* n_tiles, int64_t* device_bytes) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  if (n_docs) *n_docs = h->ix.n_docs;
  if (n_terms) *n_terms = h->ix.n_terms;
  if (nnz) *nnz = h->ix.nnz;
  if (tile_docs) *tile_docs = 1 << h->ix.tile_shift;
  if (n_tiles) *n_tiles = h->ix.ntiles;
  if (device_bytes) *device_bytes = h->device_bytes;
  return BM25_OK;
}

int bm25_index_segments(const bm25_index* h, int32_t* sparse, int64_t* n_pairs) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  if (sparse) *sparse = h->ix.sparse ? 1 : 0;
  if (n_pairs) *n_pairs = h->ix.n_pairs;
  return BM25_OK;
}

int bm25_index_bounds(const bm25_index* h, int32_t* has_bounds, int64_t* bytes) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  const bool on = h->ix.bmax != nullptr;
  if (has_bounds) *has_bounds = on ? 1 : 0;
  if (bytes) *bytes = on ? (int64_t)sizeof(uint16_t) * h->ix.n_terms * bmax_stride(h->ix.ntiles) : 0;
  return BM25_OK;
}

int bm25_search(bm25_index* h, const int32_t* queries, int64_t Q, int64_t T, int32_t k,
                int32_t* out_docs, float* out_scores) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  if (Q < 0 || T < 0) return fail(BM25_EINVAL, "negative query shape");
  int rc = check_k(h, k);
  if (rc) return rc;
  if (Q == 0 || k == 0) return BM25_OK;
  if (T > 0 && !queries) return fail(BM25_EINVAL, "NULL queries");
  if (!out_docs || !out_scores) return fail(BM25_EINVAL, "NULL output");
  // bm25_native.py:116-121: max(initial=0) >= n_terms -> ValueError
  int64_t mx = 0;
  for (int64_t i = 0; i < Q * T; ++i) mx = std::max<int64_t>(mx, queries[i]);
  if (mx >= h->ix.n_terms)
    return fail(BM25_EINVAL,
                "The maximum token ID in the query (%lld) is higher than the number of tokens in "
                "the index.",
                (long long)mx);
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  rc = ensure_io(h, Q * T, Q * (int64_t)k);
  if (rc) return rc;
  if (Q * T > 0)
    HIP_TRY(hipMemcpyAsync(h->d_q, queries, sizeof(int32_t) * Q * T, hipMemcpyHostToDevice, h->stream), "H2D queries");
  rc = run_search(h, h->d_q, Q, T, k, h->d_docs, h->d_scores, h->stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out_docs, h->d_docs, sizeof(int32_t) * Q * k, hipMemcpyDeviceToHost, h->stream), "D2H docs");
  HIP_TRY(hipMemcpyAsync(out_scores, h->d_scores, sizeof(float) * Q * k, hipMemcpyDeviceToHost, h->stream), "D2H scores");
  HIP_TRY(hipStreamSynchronize(h->stream), "search sync");
  return BM25_OK;
}

int bm25_search_device(bm25_index* h, const int32_t* d_queries, int64_t Q, int64_t T, int32_t k,
                       int32_t* d_docs, float* d_scores, void* stream) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  if (Q < 0 || T < 0) return fail(BM25_EINVAL, "negative query shape");
  int rc = check_k(h, k);
  if (rc) return rc;
  if (Q == 0 || k == 0) return BM25_OK;
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  return run_search(h, d_queries, Q, T, k, d_docs, d_scores, (hipStream_t)stream);
}

int bm25_index_bounds_export(bm25_index* h, uint16_t* d_out, int64_t stride, void* stream) {
  if (!h || !d_out) return fail(BM25_EINVAL, "NULL argument");
  std::lock_guard<std::mutex> lk(h->mu);
  if (!h->ix.bmax)
    return fail(BM25_EINVAL, "the index keeps no tile bounds (a dense, non-negative index does)");
  const int64_t bs = bmax_stride(h->ix.ntiles);
  if (stride < bs || stride % 4 != 0)
    return fail(BM25_EINVAL, "stride %lld: a multiple of 4, >= %lld", (long long)stride, (long long)bs);
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  const hipStream_t st = (hipStream_t)stream;
  const int64_t V = h->ix.n_terms;
  if (V == 0) return BM25_OK;
  if (stride > bs) HIP_TRY(hipMemsetAsync(d_out, 0, sizeof(uint16_t) * V * stride, st), "hipMemsetAsync");
  if (bs > 0)
    HIP_TRY(hipMemcpy2DAsync(d_out, sizeof(uint16_t) * stride, h->ix.bmax, sizeof(uint16_t) * bs,
                             sizeof(uint16_t) * bs, V, hipMemcpyDeviceToDevice, st),
            "hipMemcpy2DAsync");
  return BM25_OK;
}

// The pooled world table (DevIndex::wbpool) of a handle with world bounds,
// built on the handle's stream once the device is idle (the caller's table
// finished on whatever stream wrote it) and owned by the handle; without the
// memory, none (the per-tile table serves).
static int pool_world(bm25_index* h) {
  DevIndex& ix = h->ix;
  const int64_t ps = bmax_stride(ix.wstride / kPool);
  const int64_t rows = (int64_t)ix.wW * ix.n_terms;
  if (rows > 0 && hipMalloc(&ix.wbpool, sizeof(uint16_t) * rows * ps) == hipSuccess) {
    // the caller's table may still be in flight on any of its streams (the
    // exports, the all-gather): the whole device first — a setup call
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    HIP_TRY(launch_pool_bounds(ix.wbmax, rows, ix.wstride, ix.wbpool, ps, h->stream), "pool_bounds launch");
    HIP_TRY(hipStreamSynchronize(h->stream), "pool_bounds");
    ix.wpstride = ps;
    // (a lower estimate of the collection's groups: each shard has ceil(its
    // tiles / kPool) of them)
    ix.wgroups = std::min<int64_t>((ix.wtiles + kPool - 1) / kPool, (int64_t)ix.wW * ps);
  } else {
    (void)hipGetLastError();
    ix.wbpool = nullptr;
    ix.wpstride = ix.wgroups = 0;
  }
  return BM25_OK;
}

int bm25_index_set_world_bounds(bm25_index* h, const uint16_t* d_world, int32_t world,
                                int64_t stride, int64_t world_tiles) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  std::lock_guard<std::mutex> lk(h->mu);
  auto clear = [&]() {
    if (h->ix.wbpool) {  // (searches still reading it: on the handle's last stream)
      if (h->ws_stream) hipStreamSynchronize(h->ws_stream);
      hipStreamSynchronize(h->stream);
      hipFree(h->ix.wbpool);
    }
    h->ix.wbmax = nullptr;
    h->ix.wbpool = nullptr;
    h->ix.wW = 0;
    h->ix.wstride = h->ix.wtiles = h->ix.wpstride = h->ix.wgroups = 0;
  };
  if (!d_world) {
    HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
    clear();
    return BM25_OK;
  }
  if (!h->ix.bmax)
    return fail(BM25_EINVAL, "the index keeps no tile bounds (a dense, non-negative index does)");
  if (world < 1 || stride % 4 != 0 || stride < bmax_stride(h->ix.ntiles) || world_tiles < 1 ||
      world_tiles > (int64_t)world * stride)
    return fail(BM25_EINVAL, "bad world bounds (world %d, stride %lld, tiles %lld)", world,
                (long long)stride, (long long)world_tiles);
  if ((int64_t)world * stride > kBoundMaxTiles + 4 * (int64_t)world)
    return fail(BM25_EINVAL, "world bounds of %lld tiles exceed the %lld one block selects over",
                (long long)((int64_t)world * stride), (long long)kBoundMaxTiles);
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  clear();
  h->ix.wbmax = d_world;
  h->ix.wW = world;
  h->ix.wstride = stride;
  h->ix.wtiles = world_tiles;
  return pool_world(h);
}

int bm25_search_shard_device(bm25_index* h, const int32_t* d_queries, int64_t Q, int64_t T,
                             int32_t k, int32_t* d_docs, float* d_scores, void* stream) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  if (Q < 0 || T < 0) return fail(BM25_EINVAL, "negative query shape");
  int rc = check_k(h, k, true);
  if (rc) return rc;
  if (Q == 0 || k == 0) return BM25_OK;
  std::lock_guard<std::mutex> lk(h->mu);
  if (!h->ix.wbmax) return fail(BM25_EINVAL, "no world bounds: bm25_index_set_world_bounds first");
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  h->sampled = false;
  // k > 4096: this shard's exact top-k (padded past its documents)
  return run_search(h, d_queries, Q, T, k, d_docs, d_scores, (hipStream_t)stream, k <= kMaxK);
}

int bm25_max_token_device(bm25_index* h, const int32_t* d_queries, int64_t Q, int64_t T,
                          int32_t* max_token, void* stream) {
  if (!h || !max_token) return fail(BM25_EINVAL, "NULL argument");
  if (Q < 0 || T < 0) return fail(BM25_EINVAL, "negative query shape");
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  if (!h->d_maxtok) HIP_TRY(hipMalloc(&h->d_maxtok, sizeof(int32_t)), "hipMalloc");
  const hipStream_t st = (hipStream_t)stream;
  HIP_TRY(launch_max_token(d_queries, Q * T, h->d_maxtok, st), "max_token_kernel");
  HIP_TRY(hipMemcpyAsync(max_token, h->d_maxtok, sizeof(int32_t), hipMemcpyDeviceToHost, st),
          "hipMemcpyAsync");
  HIP_TRY(hipStreamSynchronize(st), "hipStreamSynchronize");
  return BM25_OK;
}

// Two-phase search of W doc shards with a global threshold (bm25mi.h).
// (T = 0: the width alone — the same for every T, search_geom)
static SampleGeom shard_geom(const bm25_index* h, int64_t shard_docs_max, int32_t world, int k,
                             int64_t T = 0) {
  const int64_t D = 1ll << h->ix.tile_shift;
  const int64_t nt = std::max<int64_t>((std::max<int64_t>(shard_docs_max, h->ix.n_docs) + D - 1) / D, 1);
  return search_geom(h->ix, nt, k, std::max(world, 1), T);
}

int bm25_sample_width(const bm25_index* h, int64_t shard_docs_max, int32_t world, int32_t k,
                      int64_t* width) {
  if (!h || !width) return fail(BM25_EINVAL, "NULL argument");
  if (world < 1 || k < 0) return fail(BM25_EINVAL, "bad world=%d or k=%d", world, k);
  // k > kMaxK: no sample (each shard's exact top-k, bm25mi_large.hip)
  *width = (k == 0 || k > kMaxK) ? 0 : shard_geom(h, shard_docs_max, world, k).S;
  return BM25_OK;
}

int bm25_search_sample_device(bm25_index* h, const int32_t* d_queries, int64_t Q, int64_t T,
                              int32_t k, int32_t world, int64_t shard_docs_max, uint64_t* d_keys,
                              void* stream) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  if (Q < 0 || T < 0 || world < 1) return fail(BM25_EINVAL, "bad shape");
  int rc = check_k(h, k, true);
  if (rc) return rc;
  if (Q == 0 || k == 0 || k > kMaxK) return BM25_OK;  // k > kMaxK: no sample half
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  const hipStream_t st = (hipStream_t)stream;
  rc = ensure_ws(h, Q, T, k, st);
  if (rc) return rc;
  HIP_TRY(order_ws(h, st), "workspace order");
  h->large_fallback = 0;
  h->split_ev = next_events(h);
  if (h->split_ev) HIP_TRY(hipEventRecord(h->split_ev->a, st), "hipEventRecord");
  choose_theta_source(h);  // (the finish half keeps this choice)
  const SampleGeom g = shard_geom(h, shard_docs_max, world, k, T);
  h->ix.disp = Dispatch{};
  h->ix.disp.sample_p = g.P;
  arm_report(h, g.P, Q);
  h->sampled = true;
  HIP_TRY(launch_sample(h->ix, d_queries, Q, T, g, d_keys, h->ws, st), "sample launch");
  return BM25_OK;
}

// The finish half on up to three streams: theta on st_theta, the REST pass
// on st_rest (after theta: an event), the merges on st_sel (after REST).  One
// stream for all three is bm25_search_finish_device.
static int finish_impl(bm25_index* h, const int32_t* d_queries, int64_t Q, int64_t T, int32_t k,
                       int32_t world, int64_t shard_docs_max, const uint64_t* d_all_keys,
                       int32_t* d_docs, float* d_scores, hipStream_t st, hipStream_t st_rest,
                       hipStream_t st_sel) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  if (Q < 0 || T < 0 || world < 1) return fail(BM25_EINVAL, "bad shape");
  int rc = check_k(h, k, true);
  if (rc) return rc;
  if (Q == 0 || k == 0) return BM25_OK;
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  for (hipEvent_t& e : h->ev_split)
    if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  // st_sel continues after everything enqueued on st (an event; none if equal)
  auto join = [&](hipStream_t from, hipStream_t to, hipEvent_t e) -> hipError_t {
    if (from == to) return hipSuccess;
    hipError_t x = hipEventRecord(e, from);
    return x != hipSuccess ? x : hipStreamWaitEvent(to, e, 0);
  };
  if (k > kMaxK) {  // this shard's exact top-k (padded past its documents)
    h->sampled = false;
    rc = run_search(h, d_queries, Q, T, k, d_docs, d_scores, st);
    if (rc) return rc;
    HIP_TRY(join(st, st_sel, h->ev_split[1]), "stream join");
    if (st_sel != st) h->ws_stream = st_sel;  // (after the join: st_sel waits for st)
    return BM25_OK;
  }
  rc = ensure_ws(h, Q, T, k, st);
  if (rc) return rc;
  HIP_TRY(order_ws(h, st), "workspace order");
  h->large_fallback = 0;
  if (!h->sampled) choose_theta_source(h);  // no sample half ran for this search (S = 0)
  const SampleGeom g = shard_geom(h, shard_docs_max, world, k, T);
  if (!h->sampled) {
    h->ix.disp = Dispatch{};
    h->ix.disp.sample_p = g.P;
    arm_report(h, g.P, Q);
  } else {
    h->ws.report = h->report_dev;  // (ensure_ws may have rebuilt the workspace)
    h->ws.seq = h->seq;
  }
  h->sampled = false;
  EventPair* ev = h->split_ev;
  h->split_ev = nullptr;
  // on three streams the score pass is timed on its own stream, from the
  // REST pass's start (the sample half and theta ran on another stream)
  HIP_TRY(launch_finish(h->ix, d_queries, Q, T, k, g, world, d_all_keys, h->ws, st, st_rest,
                        h->ev_split[0], (ev && st_rest != st) ? ev->a : nullptr),
          "finish launch");
  if (ev) HIP_TRY(hipEventRecord(ev->b, st_rest), "hipEventRecord");
  HIP_TRY(join(st_rest, st_sel, h->ev_split[1]), "stream join");
  // world > 1: this shard's list goes to the W-way merge, which sorts (no
  // sorted list needed here); world = 1 is a plain search: sorted
  HIP_TRY(launch_select(h->ix, d_queries, Q, T, k, g.P, h->ws, d_docs, d_scores, st_sel,
                        world > 1),
          "select launch");
  HIP_TRY(record_end(h, ev, st_sel), "hipEventRecord");
  h->ws_stream = st_sel;  // (the next search on another stream waits for this one)
  if (h->prof) {
    h->score_launches += 1;
    h->searches += 1;
  }
  return BM25_OK;
}

int bm25_search_finish_device(bm25_index* h, const int32_t* d_queries, int64_t Q, int64_t T,
                              int32_t k, int32_t world, int64_t shard_docs_max,
                              const uint64_t* d_all_keys, int32_t* d_docs, float* d_scores,
                              void* stream) {
  const hipStream_t st = (hipStream_t)stream;
  return finish_impl(h, d_queries, Q, T, k, world, shard_docs_max, d_all_keys, d_docs, d_scores,
                     st, st, st);
}

int bm25_search_finish_streams_device(bm25_index* h, const int32_t* d_queries, int64_t Q,
                                      int64_t T, int32_t k, int32_t world,
                                      int64_t shard_docs_max, const uint64_t* d_all_keys,
                                      int32_t* d_docs, float* d_scores, void* stream_theta,
                                      void* stream_rest, void* stream_select) {
  return finish_impl(h, d_queries, Q, T, k, world, shard_docs_max, d_all_keys, d_docs, d_scores,
                     (hipStream_t)stream_theta, (hipStream_t)stream_rest,
                     (hipStream_t)stream_select);
}

int bm25_build_scores(int device, int64_t n_docs, int64_t n_terms, int64_t n_triples,
                      const int32_t* docs, const int32_t* terms, const float* tfs,
                      const int32_t* doc_len, double avgdl, double k1, double b, int method,
                      const float* idf, int64_t* out_indptr, int32_t* out_indices,
                      float* out_data, double* out_data64) {
  if (n_docs < 0 || n_terms < 0 || n_triples < 0)
    return fail(BM25_EINVAL, "negative size (n_docs=%lld n_terms=%lld n=%lld)", (long long)n_docs,
                (long long)n_terms, (long long)n_triples);
  if (n_docs > INT32_MAX || n_terms > INT32_MAX || n_triples > INT32_MAX)
    return fail(BM25_EINVAL, "sizes above int32 are built per shard");
  if (method != kLucene && method != kBm25Py) return fail(BM25_EINVAL, "unknown method %d", method);
  if (!out_indptr || (n_triples > 0 && (!docs || !terms || !tfs || !doc_len || !out_indices ||
                                         !out_data)))
    return fail(BM25_EINVAL, "NULL argument");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(BM25_EHIP, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(BM25_EINVAL, "device %d out of range (%d visible)", device, ndev);
  HIP_TRY(hipSetDevice(device), "hipSetDevice");
  const size_t n = (size_t)std::max<int64_t>(n_triples, 1);
  int32_t *d_docs = nullptr, *d_terms = nullptr, *d_dl = nullptr, *d_ix = nullptr, *d_err = nullptr;
  float *d_tf = nullptr, *d_idf = nullptr, *d_dt = nullptr;
  double* d_dt64 = nullptr;
  int64_t* d_ip = nullptr;
  hipStream_t st = nullptr;
  auto cleanup = [&](int rc) {
    if (st) hipStreamSynchronize(st);
    for (void* p : {(void*)d_docs, (void*)d_terms, (void*)d_dl, (void*)d_ix, (void*)d_err,
                    (void*)d_tf, (void*)d_idf, (void*)d_dt, (void*)d_dt64, (void*)d_ip})
      hipFree(p);
    if (st) hipStreamDestroy(st);
    return rc;
  };
  hipError_t e;
#define TRYB(expr, what)                                    \
  do {                                                      \
    e = (expr);                                             \
    if (e != hipSuccess) return cleanup(hip_fail(e, what)); \
  } while (0)
  TRYB(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
  TRYB(hipMalloc(&d_docs, sizeof(int32_t) * n), "hipMalloc(docs)");
  TRYB(hipMalloc(&d_terms, sizeof(int32_t) * n), "hipMalloc(terms)");
  TRYB(hipMalloc(&d_tf, sizeof(float) * n), "hipMalloc(tf)");
  TRYB(hipMalloc(&d_dl, sizeof(int32_t) * std::max<int64_t>(n_docs, 1)), "hipMalloc(doc_len)");
  TRYB(hipMalloc(&d_ix, sizeof(int32_t) * n), "hipMalloc(indices)");
  TRYB(hipMalloc(&d_dt, sizeof(float) * n), "hipMalloc(data)");
  TRYB(hipMalloc(&d_ip, sizeof(int64_t) * (n_terms + 1)), "hipMalloc(indptr)");
  TRYB(hipMalloc(&d_err, sizeof(int32_t)), "hipMalloc(err)");
  if (out_data64) TRYB(hipMalloc(&d_dt64, sizeof(double) * n), "hipMalloc(data64)");
  if (idf) {
    TRYB(hipMalloc(&d_idf, sizeof(float) * std::max<int64_t>(n_terms, 1)), "hipMalloc(idf)");
    TRYB(hipMemcpyAsync(d_idf, idf, sizeof(float) * n_terms, hipMemcpyHostToDevice, st), "H2D idf");
  }
  TRYB(hipMemsetAsync(d_err, 0, sizeof(int32_t), st), "hipMemset");
  if (n_triples > 0) {
    TRYB(hipMemcpyAsync(d_docs, docs, sizeof(int32_t) * n_triples, hipMemcpyHostToDevice, st), "H2D docs");
    TRYB(hipMemcpyAsync(d_terms, terms, sizeof(int32_t) * n_triples, hipMemcpyHostToDevice, st), "H2D terms");
    TRYB(hipMemcpyAsync(d_tf, tfs, sizeof(float) * n_triples, hipMemcpyHostToDevice, st), "H2D tf");
    TRYB(hipMemcpyAsync(d_dl, doc_len, sizeof(int32_t) * n_docs, hipMemcpyHostToDevice, st), "H2D doc_len");
  }
  TRYB(build_scores(n_docs, n_terms, n_triples, d_docs, d_terms, d_tf, d_dl, avgdl, k1, b, method,
                    d_idf, d_ip, d_ix, d_dt, d_dt64, d_err, st), "build_scores");
  int32_t herr = 0;
  TRYB(hipMemcpyAsync(&herr, d_err, sizeof(int32_t), hipMemcpyDeviceToHost, st), "D2H err");
  TRYB(hipStreamSynchronize(st), "build sync");
  if (herr & 1) return cleanup(fail(BM25_EINVAL, "doc or term id out of range"));
  if (herr & 2) return cleanup(fail(BM25_EINVAL, "term frequencies must be positive and finite"));
  if (herr & 4) return cleanup(fail(BM25_EINVAL, "duplicate (doc, term) triple"));
  TRYB(hipMemcpyAsync(out_indptr, d_ip, sizeof(int64_t) * (n_terms + 1), hipMemcpyDeviceToHost, st), "D2H indptr");
  if (n_triples > 0) {
    TRYB(hipMemcpyAsync(out_indices, d_ix, sizeof(int32_t) * n_triples, hipMemcpyDeviceToHost, st), "D2H indices");
    TRYB(hipMemcpyAsync(out_data, d_dt, sizeof(float) * n_triples, hipMemcpyDeviceToHost, st), "D2H data");
    if (out_data64)
      TRYB(hipMemcpyAsync(out_data64, d_dt64, sizeof(double) * n_triples, hipMemcpyDeviceToHost, st), "D2H data64");
  }
  TRYB(hipStreamSynchronize(st), "build sync");
#undef TRYB
  return cleanup(BM25_OK);
}

int bm25_scores_dense(bm25_index* h, const int32_t* query, int64_t T, float* out_scores) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  if (T < 0) return fail(BM25_EINVAL, "negative query length");
  if (!out_scores) return fail(BM25_EINVAL, "NULL output");
  int64_t mx = 0;
  for (int64_t i = 0; i < T; ++i) mx = std::max<int64_t>(mx, query[i]);
  if (mx >= h->ix.n_terms)
    return fail(BM25_EINVAL,
                "The maximum token ID in the query (%lld) is higher than the number of tokens in "
                "the index.",
                (long long)mx);
  if (h->ix.n_docs == 0) return BM25_OK;
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  float* d_out = nullptr;
  int32_t* d_qq = nullptr;
  HIP_TRY(hipMalloc(&d_out, sizeof(float) * h->ix.n_docs), "hipMalloc(dense)");
  hipError_t e = hipMalloc(&d_qq, sizeof(int32_t) * std::max<int64_t>(T, 1));
  if (e == hipSuccess && T > 0)
    e = hipMemcpyAsync(d_qq, query, sizeof(int32_t) * T, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = launch_scores_dense(h->ix, d_qq, T, d_out, h->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(out_scores, d_out, sizeof(float) * h->ix.n_docs, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  hipFree(d_out);
  hipFree(d_qq);
  if (e != hipSuccess) return hip_fail(e, "scores_dense");
  return BM25_OK;
}

int bm25_index_set_values_f64(bm25_index* h, const double* data64) {
  if (!h || (h->ix.nnz > 0 && !data64)) return fail(BM25_EINVAL, "NULL argument");
  if (!h->arrays) return fail(BM25_EINVAL, "unbuilt index");
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  if (!h->ix.val64) {
    HIP_TRY(hipMalloc(&h->ix.val64, sizeof(double) * std::max<int64_t>(h->ix.nnz, 1)),
            "hipMalloc(val64)");
    h->arrays->p.push_back(h->ix.val64);  // freed with the index arrays
  }
  if (h->ix.nnz > 0)
    HIP_TRY(hipMemcpyAsync(h->ix.val64, data64, sizeof(double) * h->ix.nnz, hipMemcpyHostToDevice,
                           h->stream), "H2D val64");
  HIP_TRY(hipStreamSynchronize(h->stream), "val64 sync");
  return BM25_OK;
}

// Device query + f64 dense sums of one query on h's stream (caller holds
// h->mu and has set the device); *d_q / *d_out are freed by the caller.
static int dense_f64_query(bm25_index* h, const int32_t* query, int64_t T, int32_t** d_q,
                           double** d_out) {
  if (T < 0) return fail(BM25_EINVAL, "negative query length");
  if (T > 0 && !query) return fail(BM25_EINVAL, "NULL query");
  if (!h->ix.val64) return fail(BM25_EINVAL, "no float64 values: bm25_index_set_values_f64 first");
  int64_t mx = 0;
  for (int64_t i = 0; i < T; ++i) mx = std::max<int64_t>(mx, query[i]);
  if (mx >= h->ix.n_terms)
    return fail(BM25_EINVAL,
                "The maximum token ID in the query (%lld) is higher than the number of tokens in "
                "the index.",
                (long long)mx);
  HIP_TRY(hipMalloc(d_q, sizeof(int32_t) * std::max<int64_t>(T, 1)), "hipMalloc(query)");
  HIP_TRY(hipMalloc(d_out, sizeof(double) * std::max<int64_t>(h->ix.n_docs, 1)), "hipMalloc(dense)");
  if (T > 0)
    HIP_TRY(hipMemcpyAsync(*d_q, query, sizeof(int32_t) * T, hipMemcpyHostToDevice, h->stream),
            "H2D query");
  HIP_TRY(launch_dense_f64(h->ix, h->ix.val64, *d_q, T, *d_out, h->stream), "dense f64 launch");
  return BM25_OK;
}

int bm25_scores_dense_f64(bm25_index* h, const int32_t* query, int64_t T, double* out_scores) {
  if (!h || !out_scores) return fail(BM25_EINVAL, "NULL argument");
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  int32_t* d_q = nullptr;
  double* d_out = nullptr;
  int rc = dense_f64_query(h, query, T, &d_q, &d_out);
  hipError_t e = hipSuccess;
  if (rc == BM25_OK && h->ix.n_docs > 0)
    e = hipMemcpyAsync(out_scores, d_out, sizeof(double) * h->ix.n_docs, hipMemcpyDeviceToHost,
                       h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  hipFree(d_q);
  hipFree(d_out);
  if (rc) return rc;
  if (e != hipSuccess) return hip_fail(e, "scores_dense_f64");
  return BM25_OK;
}

int bm25_topn_f64(bm25_index* h, const int32_t* query, int64_t T, int64_t n, int32_t* out_docs,
                  double* out_scores) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  if (n < 0 || n > h->ix.n_docs)
    return fail(BM25_EINVAL, "n=%lld must be in 0..n_docs (%lld)", (long long)n,
                (long long)h->ix.n_docs);
  if (n > 0 && (!out_docs || !out_scores)) return fail(BM25_EINVAL, "NULL output");
  if (n == 0) return BM25_OK;
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  int32_t* d_q = nullptr;
  double* d_out = nullptr;
  void* scratch = nullptr;
  int32_t* d_docs = nullptr;
  double* d_sc = nullptr;
  int rc = dense_f64_query(h, query, T, &d_q, &d_out);
  hipError_t e = hipSuccess;
  if (rc == BM25_OK) {
    e = hipMalloc(&scratch, topn_f64_scratch_bytes(h->ix.n_docs));
    if (e == hipSuccess) e = hipMalloc(&d_docs, sizeof(int32_t) * n);
    if (e == hipSuccess) e = hipMalloc(&d_sc, sizeof(double) * n);
    if (e == hipSuccess)
      e = launch_topn_f64(d_out, h->ix.n_docs, n, scratch, d_docs, d_sc, h->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(out_docs, d_docs, sizeof(int32_t) * n, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(out_scores, d_sc, sizeof(double) * n, hipMemcpyDeviceToHost, h->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  else hipStreamSynchronize(h->stream);
  for (void* p : {(void*)d_q, (void*)d_out, scratch, (void*)d_docs, (void*)d_sc}) hipFree(p);
  if (rc) return rc;
  if (e != hipSuccess) return hip_fail(e, "topn_f64");
  return BM25_OK;
}

int bm25_merge_topk_device(int device, const int32_t* d_docs, const float* d_scores, int64_t W,
                           int64_t Q, int32_t k, int32_t* d_out_docs, float* d_out_scores,
                           void* stream) {
  if (W < 1 || Q < 0 || k < 0) return fail(BM25_EINVAL, "bad merge shape W=%lld Q=%lld k=%d", (long long)W, (long long)Q, k);
  HIP_TRY(hipSetDevice(device), "hipSetDevice");
  HIP_TRY(launch_merge_lists(d_docs, d_scores, W, Q, k, Q * (int64_t)k, false, d_out_docs, d_out_scores, (hipStream_t)stream), "merge_lists launch");
  return BM25_OK;
}

int bm25_merge_sorted_device(int device, const int32_t* d_docs, const float* d_scores, int64_t W,
                             int64_t Q, int32_t k, int64_t rank_stride, int32_t* d_out_docs,
                             float* d_out_scores, void* stream) {
  if (W < 1 || Q < 0 || k < 0 || rank_stride < Q * (int64_t)k)
    return fail(BM25_EINVAL, "bad merge shape W=%lld Q=%lld k=%d stride=%lld", (long long)W,
                (long long)Q, k, (long long)rank_stride);
  HIP_TRY(hipSetDevice(device), "hipSetDevice");
  HIP_TRY(launch_merge_lists(d_docs, d_scores, W, Q, k, rank_stride, true, d_out_docs,
                             d_out_scores, (hipStream_t)stream),
          "merge_sorted launch");
  return BM25_OK;
}

int bm25_profile_enable(bm25_index* h, int on) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  std::lock_guard<std::mutex> lk(h->mu);
  hipSetDevice(h->ix.device);
  harvest_events(h);
  h->prof = on < 0 ? 0 : (on > 2 ? 2 : on);
  h->score_ms = h->total_ms = 0.0;
  h->score_launches = h->searches = h->rescored = 0;
  return BM25_OK;
}

int bm25_profile_read(bm25_index* h, double* score_ms_total, int64_t* score_launches,
                      double* total_ms, int64_t* searches, int64_t* rescored_tiles) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  std::lock_guard<std::mutex> lk(h->mu);
  hipSetDevice(h->ix.device);
  harvest_events(h);
  int32_t cnt[kCounters] = {};
  read_counters(h, cnt);
  if (score_ms_total) *score_ms_total = h->score_ms;
  if (score_launches) *score_launches = h->score_launches;
  if (total_ms) *total_ms = h->total_ms;
  if (searches) *searches = h->searches;
  if (rescored_tiles) *rescored_tiles = cnt[3];  // tiles re-scored by the last search
  return BM25_OK;
}

int bm25_search_stats(bm25_index* h, int64_t* rescored_tiles, int64_t* fallback_queries) {
  return bm25_search_stats_ex(h, rescored_tiles, fallback_queries, nullptr);
}

int bm25_search_stats_ex(bm25_index* h, int64_t* rescored_tiles, int64_t* fallback_queries,
                         int64_t* bound_skipped) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  int32_t cnt[kCounters] = {};
  read_counters(h, cnt);
  if (rescored_tiles) *rescored_tiles = cnt[3];
  if (fallback_queries) *fallback_queries = cnt[2];
  if (bound_skipped) *bound_skipped = (h->ix.disp.kernels & kKCountSkips) ? cnt[5] : -1;
  return BM25_OK;
}

int bm25_search_counters(bm25_index* h, int64_t* out, int32_t n) {
  if (!h || !out) return fail(BM25_EINVAL, "NULL argument");
  if (n < 1 || n > 6) return fail(BM25_EINVAL, "n=%d must be in 1..6", n);
  std::lock_guard<std::mutex> lk(h->mu);
  HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
  int32_t cnt[kCounters] = {};
  read_counters(h, cnt);
  uint64_t post = 0;
  std::memcpy(&post, cnt + 6, sizeof post);  // counters[6..7]: a u64 (score_flat_kernel)
  // (the skipped pairs and postings: counted by the count_skips build only, else -1)
  const bool counted = (h->ix.disp.kernels & kKCountSkips) != 0;
  const int64_t v[6] = {cnt[3], cnt[2], counted ? cnt[5] : -1, counted ? (int64_t)post : -1,
                        cnt[4], h->large_fallback};
  for (int i = 0; i < n; ++i) out[i] = v[i];
  return BM25_OK;
}

int bm25_index_set_option(bm25_index* h, const char* name, int64_t value) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  std::lock_guard<std::mutex> lk(h->mu);
  const int old_cap = h->ix.opt.list_cap;
  const int rc = set_opt(h->ix.opt, name, value);
  if (rc) return rc;
  if (h->ix.opt.list_cap != old_cap && h->ws.cap_q > 0) {  // the list capacity is sized in
    hipSetDevice(h->ix.device);                            // the workspace: rebuild it
    ws_wait_host(h);
    free_ws(h->ws);
  }
  return BM25_OK;
}

int bm25_index_get_option(const bm25_index* h, const char* name, int64_t* value) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  bm25_index* m = const_cast<bm25_index*>(h);  // the mutex only: set_option writes under it
  std::lock_guard<std::mutex> lk(m->mu);
  return get_opt(h->ix.opt, name, value);
}

int bm25_search_dispatch(bm25_index* h, uint32_t* kernels, int32_t* term_lanes,
                         int32_t* band_tiles, int32_t* sample_p) {
  if (!h) return fail(BM25_EINVAL, "NULL index");
  std::lock_guard<std::mutex> lk(h->mu);
  const Dispatch& d = h->ix.disp;
  if (kernels) *kernels = d.kernels;
  if (term_lanes) *term_lanes = d.term_lanes;
  if (band_tiles)
    for (int i = 0; i < 3; ++i) band_tiles[i] = d.band_tiles[i];
  if (sample_p) *sample_p = d.sample_p;
  return BM25_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Doc-sharded index over several devices of one process:
// shard s owns the tile-aligned doc range [lo_s, hi_s) as an ordinary index
// (doc_offset = lo_s) on devices[s].  A search is the global-threshold
// protocol of the multi-process path (bm25mi.dist.sharded_search) with peer
// copies over xGMI in place of the collectives:
//   1. every shard samples on its own stream -> keys_s [Q][S];
//   2. every shard's keys are copied into every shard's all_keys [W][Q][S]
//      (peer copies on the destination's stream, after the source's event);
//   3. every shard: theta = the k-th best key of the whole sample, then its
//      keys >= theta as a padded [Q, k] list (global doc ids);
//   4. the lists are copied to shard 0's device and merged there with the
//      same (score desc, doc asc) rule, so the result equals a single-index
//      search.
// One process owns every device here, so no RCCL communicator is involved
// (the multi-process path runs its all-gathers over RCCL).
// ---------------------------------------------------------------------------
struct bm25_sharded {
  std::vector<bm25_index*> shards;
  std::vector<int64_t> lo, hi;
  std::vector<hipEvent_t> sampled;  // per shard: its sample keys are written
  std::vector<hipEvent_t> keyed;    // per shard: its all_keys copies landed
  std::vector<hipEvent_t> done;     // per shard: its [Q, k] list is written
  std::vector<uint64_t*> keys;      // per shard (own device): [Q][S]
  std::vector<uint64_t*> all_keys;  // per shard (own device): [W][Q][S]
  int64_t cap_keys = 0;
  int64_t n_docs = 0, n_terms = 0, shard_docs_max = 0;
  int32_t* g_docs = nullptr;     // [W][Q][k] on shard 0's device
  float* g_scores = nullptr;
  int32_t* m_docs = nullptr;     // [Q][k]
  float* m_scores = nullptr;
  int64_t cap_g = 0, cap_m = 0;
  std::mutex mu;
};

namespace {

int sharded_free(bm25_sharded* s) {
  if (!s) return BM25_OK;
  if (!s->shards.empty() && s->shards[0]) {
    hipSetDevice(s->shards[0]->ix.device);
    hipFree(s->g_docs);
    hipFree(s->g_scores);
    hipFree(s->m_docs);
    hipFree(s->m_scores);
  }
  for (size_t i = 0; i < s->shards.size(); ++i) {
    if (!s->shards[i]) continue;
    hipSetDevice(s->shards[i]->ix.device);
    hipStreamSynchronize(s->shards[i]->stream);
    for (auto* v : {&s->sampled, &s->keyed, &s->done})
      if (i < v->size() && (*v)[i]) hipEventDestroy((*v)[i]);
    if (i < s->keys.size()) hipFree(s->keys[i]);
    if (i < s->all_keys.size()) hipFree(s->all_keys[i]);
    bm25_index_destroy(s->shards[i]);
  }
  delete s;
  return BM25_OK;
}

}  // namespace

extern "C" {

int bm25_sharded_create(int n_dev, const int* devices, int64_t n_docs, int64_t n_terms,
                        int64_t nnz, const void* indptr, int indptr_is_i64,
                        const int32_t* indices, const float* data, bm25_sharded** out) {
  if (!out) return fail(BM25_EINVAL, "out is NULL");
  *out = nullptr;
  if (n_dev < 1 || !devices) return fail(BM25_EINVAL, "need at least one device");
  if (n_docs < 0 || n_terms < 0 || nnz < 0) return fail(BM25_EINVAL, "negative size");
  if (!indptr || (nnz > 0 && (!indices || !data))) return fail(BM25_EINVAL, "NULL CSC array");
  std::vector<int64_t> ip(n_terms + 1);
  for (int64_t t = 0; t <= n_terms; ++t)
    ip[t] = indptr_is_i64 ? ((const int64_t*)indptr)[t] : (int64_t)((const int32_t*)indptr)[t];
  if (ip[0] != 0 || ip[n_terms] != nnz)
    return fail(BM25_EINVAL, "indptr must start at 0 and end at nnz");
  for (int64_t t = 0; t < n_terms; ++t)
    if (ip[t + 1] < ip[t]) return fail(BM25_EINVAL, "indptr decreases at column %lld", (long long)t);
  bm25_sharded* s = new bm25_sharded();
  s->n_docs = n_docs;
  s->n_terms = n_terms;
  const int64_t align = 2048;
  auto bound = [&](int64_t r) -> int64_t {
    if (r >= n_dev) return n_docs;
    const int64_t x = n_docs * r / n_dev;
    return std::min(n_docs, (x + align / 2) / align * align);
  };
  std::vector<int64_t> sip(n_terms + 1);
  std::vector<int32_t> six;
  std::vector<float> sdt;
  for (int r = 0; r < n_dev; ++r) {
    const int64_t lo = bound(r), hi = bound(r + 1);
    // the shard's CSC: per column, the entries with lo <= doc < hi (columns are
    // sorted; unsorted input is rejected by the shard's own build check)
    sip[0] = 0;
    for (int64_t t = 0; t < n_terms; ++t) {
      const int32_t* b = indices + ip[t];
      const int32_t* e = indices + ip[t + 1];
      const int32_t* p0 = std::lower_bound(b, e, (int32_t)std::min<int64_t>(lo, INT32_MAX));
      const int32_t* p1 = std::lower_bound(p0, e, (int32_t)std::min<int64_t>(hi, INT32_MAX));
      sip[t + 1] = sip[t] + (p1 - p0);
    }
    six.resize(std::max<int64_t>(sip[n_terms], 1));
    sdt.resize(std::max<int64_t>(sip[n_terms], 1));
    for (int64_t t = 0; t < n_terms; ++t) {
      const int32_t* b = indices + ip[t];
      const int32_t* e = indices + ip[t + 1];
      const int32_t* p0 = std::lower_bound(b, e, (int32_t)std::min<int64_t>(lo, INT32_MAX));
      for (int64_t i = 0; i < sip[t + 1] - sip[t]; ++i) {
        six[sip[t] + i] = p0[i] - (int32_t)lo;
        sdt[sip[t] + i] = data[(p0 - indices) + i];
      }
    }
    bm25_index* h = nullptr;
    const int rc = bm25_index_create(devices[r], hi - lo, n_terms, sip[n_terms], sip.data(), 1,
                                     six.data(), sdt.data(), lo, &h);
    if (rc) {
      const std::string msg = g_err;
      sharded_free(s);
      return fail(rc, "shard %d (device %d): %s", r, devices[r], msg.c_str());
    }
    s->shards.push_back(h);
    s->lo.push_back(lo);
    s->hi.push_back(hi);
    s->keys.push_back(nullptr);
    s->all_keys.push_back(nullptr);
    s->shard_docs_max = std::max(s->shard_docs_max, hi - lo);
    hipSetDevice(devices[r]);
    for (auto* v : {&s->sampled, &s->keyed, &s->done}) {
      hipEvent_t ev = nullptr;
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
        sharded_free(s);
        return fail(BM25_EHIP, "hipEventCreate");
      }
      v->push_back(ev);
    }
  }
  *out = s;
  return BM25_OK;
}

int bm25_sharded_destroy(bm25_sharded* s) { return sharded_free(s); }

int bm25_sharded_search(bm25_sharded* s, const int32_t* queries, int64_t Q, int64_t T,
                        int32_t k, int32_t* out_docs, float* out_scores) {
  if (!s) return fail(BM25_EINVAL, "NULL index");
  if (Q < 0 || T < 0) return fail(BM25_EINVAL, "negative query shape");
  if (k < 0) return fail(BM25_EINVAL, "negative dimensions are not allowed (top_k=%d)", k);
  if (k > s->n_docs)
    return fail(BM25_EINVAL, "kth(=%lld) out of bounds (%lld)", (long long)(s->n_docs - k),
                (long long)s->n_docs);
  if (Q == 0 || k == 0) return BM25_OK;
  if (T > 0 && !queries) return fail(BM25_EINVAL, "NULL queries");
  if (!out_docs || !out_scores) return fail(BM25_EINVAL, "NULL output");
  int64_t mx = 0;
  for (int64_t i = 0; i < Q * T; ++i) mx = std::max<int64_t>(mx, queries[i]);
  if (mx >= s->n_terms)
    return fail(BM25_EINVAL,
                "The maximum token ID in the query (%lld) is higher than the number of tokens in "
                "the index.",
                (long long)mx);
  const int64_t W = (int64_t)s->shards.size();
  std::lock_guard<std::mutex> lk(s->mu);
  bm25_index* h0 = s->shards[0];
  const int64_t out = Q * (int64_t)k;
  HIP_TRY(hipSetDevice(h0->ix.device), "hipSetDevice");
  if (W * out > s->cap_g) {
    hipFree(s->g_docs);
    hipFree(s->g_scores);
    s->g_docs = nullptr;
    s->g_scores = nullptr;
    HIP_TRY(hipMalloc(&s->g_docs, sizeof(int32_t) * W * out), "hipMalloc(shard lists)");
    HIP_TRY(hipMalloc(&s->g_scores, sizeof(float) * W * out), "hipMalloc(shard lists)");
    s->cap_g = W * out;
  }
  if (out > s->cap_m) {
    hipFree(s->m_docs);
    hipFree(s->m_scores);
    s->m_docs = nullptr;
    s->m_scores = nullptr;
    HIP_TRY(hipMalloc(&s->m_docs, sizeof(int32_t) * out), "hipMalloc(merged)");
    HIP_TRY(hipMalloc(&s->m_scores, sizeof(float) * out), "hipMalloc(merged)");
    s->cap_m = out;
  }
  // sample width: the same on every shard (bm25_sample_width's rule)
  int64_t S = 0;
  int rc = bm25_sample_width(h0, s->shard_docs_max, (int32_t)W, k, &S);
  if (rc) return rc;
  if (Q * S > s->cap_keys) {
    for (int64_t r = 0; r < W; ++r) {
      HIP_TRY(hipSetDevice(s->shards[r]->ix.device), "hipSetDevice");
      hipStreamSynchronize(s->shards[r]->stream);
      hipFree(s->keys[r]);
      hipFree(s->all_keys[r]);
      s->keys[r] = s->all_keys[r] = nullptr;
      HIP_TRY(hipMalloc(&s->keys[r], sizeof(uint64_t) * Q * S), "hipMalloc(sample keys)");
      HIP_TRY(hipMalloc(&s->all_keys[r], sizeof(uint64_t) * W * Q * S), "hipMalloc(all keys)");
    }
    s->cap_keys = Q * S;
  }
  // 1. every shard: H2D queries + its sample keys, on its own stream
  for (int64_t r = 0; r < W; ++r) {
    bm25_index* h = s->shards[r];
    HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
    {
      std::lock_guard<std::mutex> lh(h->mu);
      rc = ensure_io(h, Q * T, out);
      if (rc) return rc;
      if (Q * T > 0)
        HIP_TRY(hipMemcpyAsync(h->d_q, queries, sizeof(int32_t) * Q * T, hipMemcpyHostToDevice,
                               h->stream), "H2D queries");
    }
    if (S > 0) {
      rc = bm25_search_sample_device(h, h->d_q, Q, T, k, (int32_t)W, s->shard_docs_max,
                                     s->keys[r], h->stream);
      if (rc) return rc;
    }
    HIP_TRY(hipEventRecord(s->sampled[r], h->stream), "hipEventRecord");
  }
  // 2. every shard's keys into every shard's all_keys (destination stream)
  if (S > 0) {
    for (int64_t d = 0; d < W; ++d) {
      bm25_index* hd = s->shards[d];
      HIP_TRY(hipSetDevice(hd->ix.device), "hipSetDevice");
      for (int64_t r = 0; r < W; ++r) {
        bm25_index* hr = s->shards[r];
        HIP_TRY(hipStreamWaitEvent(hd->stream, s->sampled[r], 0), "hipStreamWaitEvent");
        HIP_TRY(hipMemcpyPeerAsync(s->all_keys[d] + r * Q * S, hd->ix.device, s->keys[r],
                                   hr->ix.device, sizeof(uint64_t) * Q * S, hd->stream),
                "peer copy (sample keys)");
      }
      HIP_TRY(hipEventRecord(s->keyed[d], hd->stream), "hipEventRecord");
    }
  }
  // 3. every shard: global theta, REST, its padded [Q, k] list (a shard's
  // keys buffer is rewritten only by the next search, and this one waits for
  // every keyed[*] event before it returns)
  for (int64_t r = 0; r < W; ++r) {
    bm25_index* h = s->shards[r];
    HIP_TRY(hipSetDevice(h->ix.device), "hipSetDevice");
    rc = bm25_search_finish_device(h, h->d_q, Q, T, k, (int32_t)W, s->shard_docs_max,
                                   S > 0 ? s->all_keys[r] : nullptr, h->d_docs, h->d_scores,
                                   h->stream);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(s->done[r], h->stream), "hipEventRecord");
  }
  // gather on shard 0's stream (peer copies after each shard's event), merge, D2H
  HIP_TRY(hipSetDevice(h0->ix.device), "hipSetDevice");
  for (int64_t r = 0; r < W; ++r) {
    bm25_index* h = s->shards[r];
    HIP_TRY(hipStreamWaitEvent(h0->stream, s->done[r], 0), "hipStreamWaitEvent");
    HIP_TRY(hipMemcpyPeerAsync(s->g_docs + r * out, h0->ix.device, h->d_docs, h->ix.device,
                               sizeof(int32_t) * out, h0->stream), "peer copy");
    HIP_TRY(hipMemcpyPeerAsync(s->g_scores + r * out, h0->ix.device, h->d_scores, h->ix.device,
                               sizeof(float) * out, h0->stream), "peer copy");
  }
  HIP_TRY(launch_merge_lists(s->g_docs, s->g_scores, W, Q, k, Q * (int64_t)k, true, s->m_docs, s->m_scores, h0->stream),
          "merge_lists launch");
  HIP_TRY(hipMemcpyAsync(out_docs, s->m_docs, sizeof(int32_t) * out, hipMemcpyDeviceToHost,
                         h0->stream), "D2H docs");
  HIP_TRY(hipMemcpyAsync(out_scores, s->m_scores, sizeof(float) * out, hipMemcpyDeviceToHost,
                         h0->stream), "D2H scores");
  HIP_TRY(hipStreamSynchronize(h0->stream), "sharded search sync");
  // every shard's stream has drained its copies of the others' keys
  for (int64_t r = 0; r < W; ++r) {
    HIP_TRY(hipSetDevice(s->shards[r]->ix.device), "hipSetDevice");
    HIP_TRY(hipEventSynchronize(s->keyed[r]), "hipEventSynchronize");
  }
  return BM25_OK;
}

int bm25_sharded_info(const bm25_sharded* s, int64_t* n_shards, int64_t* shard_lo,
                      int64_t* shard_hi) {
  if (!s) return fail(BM25_EINVAL, "NULL index");
  if (n_shards) *n_shards = (int64_t)s->shards.size();
  for (size_t i = 0; i < s->shards.size(); ++i) {
    if (shard_lo) shard_lo[i] = s->lo[i];
    if (shard_hi) shard_hi[i] = s->hi[i];
  }
  return BM25_OK;
}

}  // extern "C"
