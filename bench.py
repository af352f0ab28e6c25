"""bench.py — batched BM25 CSC search throughput on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

A step = one search of the whole query batch (config c3: 1024 queries, k=100)
over the 10M-doc / 200k-term / 640M-posting synthetic CSC index, inputs already
resident in HBM.  With N GPUs the doc axis is sharded (one contiguous doc range
per rank); every rank samples its shard, the sample keys are
all-gathered over RCCL (one global threshold), every rank lists its keys above
it, and the per-shard [Q, k] lists are all-gathered and merged on the GPU, so
every step returns the same global top-k as one GPU would.  Total work is fixed as N
grows ("scaling": "strong").  ``--mode replica`` is the comparison point of
SURVEY.md §8(e): every rank holds the whole index and searches its Q/N slice of
the batch with no collective (``--replica-of R`` at N=1 runs rank 0's slice of an
R-way replica job on one GPU).  ``--config c2`` (a 25.6 MB index, resident in the
256 MB Infinity Cache) labels its roofline as effective bandwidth.

Printed by rank 0: ONE JSON line with the metric (value = steps x Q / the
barrier-bracketed wall time, max over ranks), the per-step median from HIP
events, the roofline of the dominant kernel (the score pass, timed with HIP
events on its stream over the timed region), the end-to-end host-buffer time
(bm25_search: H2D queries -> D2H results, median of --e2e-batches, N=1) and
the CPU baseline (the reference's scipy/numpy call sequence,
oracle.search_faithful, on a seeded 64-query sample: one process, and a fork
pool over the job's cores; rank 0 at N=1, run before the GPU is touched).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(REPO, "mojo-bm25_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(indptr: np.ndarray, queries: np.ndarray, k: int) -> int:
    """B(q) = sum_{distinct t in q, t>=0} (8 df(t) + 8) + 4T + 8k."""
    df = np.diff(indptr)
    total = 0
    for row in queries:
        t = np.unique(row[row >= 0])
        total += int((8 * df[t] + 8).sum()) + 4 * len(row) + 8 * k
    return total


def query_postings(indptr: np.ndarray, queries: np.ndarray) -> int:
    """Postings the batch reads query by query: sum over queries of the
    distinct terms' document frequencies (the posting part of B(q))."""
    df = np.diff(indptr)
    return int(sum(int(df[np.unique(row[row >= 0])].sum()) for row in queries))


def batch_distinct_postings(indptr: np.ndarray, queries: np.ndarray) -> int:
    """Postings of the batch's DISTINCT terms (SURVEY.md:381, BASELINE.md:49):
    what one read of every posting list the batch needs would move — the
    floor under the per-query algorithmic bytes once L2/MALL reuse across the
    batch's queries is perfect."""
    df = np.diff(indptr)
    t = np.unique(queries[queries >= 0])
    return int(df[t].sum())


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def load_traffic(path: str, config: str, shift: int, terms: int):
    """HBM bytes per score pass measured offline with rocprofv3 --pmc
    (profiles/) — used only if it matches this workload."""
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    for e in t.get("entries", [t]):
        if (e.get("config") == config and int(e.get("tile_shift", -1)) == shift
                and int(e.get("terms_per_query", 8)) == terms):
            return dict(e, method=t.get("method", e.get("method")),
                        source=t.get("source", e.get("source")))
    return None


def cpu_quota():
    """CPUs this job may use: the cgroup v2 CPU quota (cpu.max) when one is
    set, else the affinity mask."""
    aff = len(os.sched_getaffinity(0))
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, min(aff, int(int(q) // int(period)))), aff, f"cgroup cpu.max {q} {period}"
    except (OSError, ValueError):
        pass
    return aff, aff, "no cgroup quota"


def cpu_baseline(args, n_docs, indptr, indices, data, queries, k):
    """BASELINE.md CPU legs on a seeded query sample: (i) one process, one
    core; (ii) a fork-based process pool over the cores this job may use
    (BASELINE.md:54 names the affinity mask; the GPU box gives one GPU's job
    a cgroup quota of 16 CPUs — the pool is sized to the quota, or to the
    affinity mask when no quota is set; BM25_CPU_SHARE caps it explicitly —
    and the per-core rate scaled to the whole affinity mask is reported
    beside it, labelled as an extrapolation).  The port is oracle.search_faithful — the reference's
    scipy/numpy call sequence (bm25_native.py:147-158, 204-214)."""
    from oracle import oracle  # the checker / CPU baseline (test infrastructure)
    Q = queries.shape[0]
    quota, aff, why = cpu_quota()
    share = int(os.environ.get("BM25_CPU_SHARE", "0"))  # explicit cap only
    procs = args.cpu_procs if args.cpu_procs > 0 else (min(quota, share) if share > 0 else quota)
    nq1 = min(args.cpu_queries, Q)                 # single-core leg
    nqp = min(Q, max(nq1, 4 * procs))              # pool leg: 4 queries per process
    rng = np.random.default_rng(20240601)
    order = rng.permutation(Q)
    sample1 = queries[np.sort(order[:nq1])]
    samplep = queries[np.sort(order[:nqp])]
    m = oracle.faithful_matrix(n_docs, indptr, indices, data)
    log(f"[rank 0] CPU baseline: {nq1} sampled queries, 1 process ...")
    t0 = time.perf_counter()
    d1, s1 = oracle.search_faithful_m(m, sample1, k)
    t1 = time.perf_counter() - t0
    log(f"[rank 0] CPU baseline: {nqp} sampled queries, pool of {procs} processes ...")
    d2, s2, t2 = oracle.search_faithful_pool(m, samplep, k, procs)
    pos = np.searchsorted(np.sort(order[:nqp]), np.sort(order[:nq1]))
    if not np.array_equal(s1.view(np.uint32), s2[pos].view(np.uint32)):
        raise RuntimeError("CPU baseline legs disagree")
    per_core = nqp / t2 / procs
    return {"value": round(nqp / t2, 3), "unit": "queries/s", "cores": procs, "kind": "port",
            "sample": f"{nqp} queries drawn (seed 20240601) from the {Q}-query bench batch, same "
                      f"index, k={k}; leg (ii): fork pool of {procs} processes (this job's CPU "
                      f"share), batch split evenly; {t2:.2f} s; host {cpu_model()}, "
                      f"os.cpu_count()={os.cpu_count()}, affinity {aff} cpus, {why}",
            "single_core": {"value": round(nq1 / t1, 3), "unit": "queries/s", "cores": 1,
                            "queries": nq1, "seconds": round(t1, 2)},
            "affinity_extrapolation": {
                "value": round(per_core * aff, 1), "unit": "queries/s", "cores": aff,
                "note": f"EXTRAPOLATION: the pool's per-process rate ({per_core:.3f} q/s) x the "
                        f"{aff} cpus of the affinity mask (BASELINE.md:54); not measured — the "
                        f"job's CPU share is {procs}"},
            "batch_s_extrapolated": {"single_core": round(t1 / nq1 * Q, 1),
                                     "pool": round(t2 / nqp * Q, 1),
                                     "note": f"EXTRAPOLATION: sample time x {Q}/sample"}}


def launch_ranks(n: int) -> int:
    """`--gpus N` (N > 1) run without a launcher: start the N ranks as a
    child torch.distributed.run on 127.0.0.1 (this process has not touched
    the GPU and is not replaced: it waits for the child and returns its exit
    status), so the line reports n_gpus = N or the run fails — never a
    silent one-GPU measurement."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] --gpus {n} without WORLD_SIZE: launching {n} ranks: {' '.join(cmd)}")
    rc = subprocess.run(cmd).returncode
    if rc != 0:
        log(f"[bench] the {n}-rank run failed (exit status {rc})")
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", help="c3 (headline), c2, c5 (100M docs: one GPU "
                    "runs one rank's doc shard, see --c5-rank); side lines: c3u (config 3 with "
                    "uniform weights: terms weigh alike), c3l (config 3's postings with "
                    "lucene scores: tf saturation and document lengths, built on the GPU)")
    ap.add_argument("--c5-rank", type=int, default=0,
                    help="config 5 at N=1: which of the 8 doc shards of the 8-GPU job to run")
    ap.add_argument("--cpu-queries", type=int, default=64,
                    help="CPU baseline: seeded query sample size (0 = skip)")
    ap.add_argument("--cpu-procs", type=int, default=-1,
                    help="CPU baseline pool leg: worker processes (default: the cgroup CPU "
                         "quota, 16 on the GPU box, else the affinity mask)")
    ap.add_argument("--terms", type=int, default=0,
                    help="terms per query (default: the config's, 8); e.g. 16 for the "
                         "long-query workload line")
    ap.add_argument("--k", type=int, default=0,
                    help="top-k (default: the config's); k > 4096 takes the large-k path")
    ap.add_argument("--e2e-batches", type=int, default=20,
                    help="host-buffer searches (H2D queries -> D2H results) timed for the "
                         "end-to-end median")
    ap.add_argument("--threads", type=int, default=16, help="host threads for index generation")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--backend", default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL; gloo only for "
                         "rehearsing several ranks on one GPU)")
    ap.add_argument("--mode", default="shard", choices=("shard", "replica"),
                    help="N > 1: shard = the doc axis split over the ranks (global threshold, "
                         "two all-gathers); replica = every rank holds the whole index and "
                         "searches its Q/N slice of the batch, no collective (SURVEY.md §8(e) "
                         "comparison point)")
    ap.add_argument("--protocol", default="auto", choices=("auto", "one", "two"),
                    help="N > 1 shard mode: one = every rank keeps the world's tile bounds "
                         "(one all-gather at setup) and each batch needs ONE collective, the "
                         "[Q, k] lists; two = the sample-key all-gather + theta + the lists; "
                         "auto = one where the collection's tile bounds allow it")
    ap.add_argument("--parts", type=int, default=1,
                    help="N > 1 shard mode: pipeline each batch as this many row ranges over "
                         "forks of the rank's index on their own streams (bm25mi.dist."
                         "_search_parts): one part's collectives and merges overlap another's "
                         "score pass")
    ap.add_argument("--replica-of", type=int, default=0,
                    help="replica mode at N=1: run rank 0's slice of an R-way replica job "
                         "(Q/R queries on the whole index) — the one-GPU proxy of the N=R line")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if args.replica_of > 1:
        args.mode = "replica"

    import torch
    from bm25mi import synth
    from bm25mi.index import GpuIndex
    from bm25mi.dist import sharded_search

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch "
                         f"--nproc-per-node {args.gpus}, or pass --gpus {world}")
    cfg = synth.CONFIGS[args.config]
    import dataclasses
    if args.terms > 0:
        cfg = dataclasses.replace(cfg, terms_per_query=args.terms)
    if args.k > 0:
        cfg = dataclasses.replace(cfg, k=args.k)
    # config 5 holds 6.4B postings: one GPU runs one of the 8 ranks' shards
    # (800M postings, int64 global indptr cut per rank by the generator)
    emul = 8 if (args.config == "c5" and world == 1) else 0
    replica = args.mode == "replica"
    if replica and args.config == "c5":
        raise SystemExit("replica mode holds the whole index per GPU: config 5 does not fit")
    if emul:
        lo, hi = synth.shard_bounds(cfg.n_docs, emul, args.c5_rank)
    elif replica:
        lo, hi = 0, cfg.n_docs
    else:
        lo, hi = synth.shard_bounds(cfg.n_docs, world, rank)
    t0 = time.time()
    if cfg.weights == "lucene" and args.cpu_queries > 0:
        # its scores are built on the GPU (bm25_build_scores), and the CPU
        # baseline's process pool must fork before this process touches it
        log("note: --config c3l builds its scores on the GPU: no CPU baseline (--cpu-queries 0)")
        args.cpu_queries = 0
    local0 = local % max(torch.cuda.device_count(), 1)
    indptr, indices, data = synth.make_index(cfg, lo, hi, threads=args.threads, device=local0)
    log(f"[rank {rank}] shard docs [{lo},{hi}) nnz={int(indptr[-1])} generated in "
        f"{time.time() - t0:.1f}s")
    queries = synth.make_queries(cfg)
    q_all = queries.shape[0]
    if replica:  # this rank's contiguous slice of the batch
        R = args.replica_of if (args.replica_of > 1 and world == 1) else world
        r = 0 if args.replica_of > 1 else rank
        queries = np.ascontiguousarray(queries[q_all * r // R:q_all * (r + 1) // R])
    else:
        R = 1

    # CPU baseline first (rank 0 at N=1): its process pool forks before this
    # process touches the GPU
    cpu = None
    if rank == 0 and world == 1 and args.cpu_queries > 0:
        cpu = cpu_baseline(args, hi - lo, indptr, indices, data, queries, cfg.k)

    dist = None
    local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    t0 = time.time()
    index = GpuIndex(indptr, indices, data, hi - lo, device=local, doc_offset=lo)
    info = index.info()
    log(f"[rank {rank}] index on cuda:{local} in {time.time() - t0:.1f}s: {info}")
    Q, T, k = queries.shape[0], queries.shape[1], cfg.k
    dq = torch.from_numpy(queries).to(dev)
    d_docs = torch.empty((Q, k), dtype=torch.int32, device=dev)
    d_scores = torch.empty((Q, k), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)

    sdm = max(b - a for a, b in (synth.shard_bounds(cfg.n_docs, world, r) for r in range(world)))
    one_coll = False
    if world > 1 and not replica and args.protocol != "two" and args.parts <= 1:
        from bm25mi.dist import setup_world_bounds
        one_coll = setup_world_bounds(index)
        if args.protocol == "one" and not one_coll:
            raise SystemExit("--protocol one: the collection's tile bounds do not allow it")
        log(f"[rank {rank}] doc-shard protocol: {'one collective (world tile bounds)' if one_coll else 'two collectives'}")

    def step():
        if world > 1 and not replica:  # global theta: RCCL all-gathers of sample keys and [Q, k] lists (bm25mi.dist)
            sharded_search(index, dq, k, sdm, d_docs, d_scores, None, stream, parts=args.parts)
        else:
            index.search_device(dq, k, d_docs, d_scores, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    index.profile_enable(True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t_start = time.perf_counter()
    for i in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    prof = index.profile_read()
    dispatch = index.last_dispatch()
    stats = index.search_stats()  # the last timed search's selection counters
    # per-step times for the median: the same steps again with an event
    # between steps (every event record costs the device ~4 us, so not in the
    # timed region above)
    index.profile_enable(False)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    evs[0].record(stream)
    for i in range(args.steps):
        step()
        evs[i + 1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    if info.get("tile_bounds") and (world == 1 or replica):
        # the (query, tile) pairs the tile bound skipped and their postings:
        # counted by the count_skips REST build (registers the timed build does
        # without), in one extra search of the same batch after the timed ones
        # (not in a doc-sharded run: its search is collective, and the extra
        # one must not depend on a rank's own index)
        index.set_option("count_skips", 1)
        step()
        torch.cuda.synchronize(dev)
        counted = index.search_stats()
        stats["bound_skipped_tiles"] = counted["bound_skipped_tiles"]
        stats["bound_skipped_postings"] = counted["bound_skipped_postings"]
        index.set_option("count_skips", 0)
    step_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
    # end-to-end (N=1): the host-buffer entry point bm25_search — H2D of the
    # query batch, the search, D2H of the [Q, k] results — timed per call
    e2e = None
    if world == 1 and args.e2e_batches > 0:
        for _ in range(3):
            index.search(queries, k)
        ts = []
        for _ in range(args.e2e_batches):
            t0 = time.perf_counter()
            index.search(queries, k)
            ts.append(1000.0 * (time.perf_counter() - t0))
        e2e = {"median_ms": round(float(np.median(ts)), 4), "min_ms": round(min(ts), 4),
               "queries_per_s": round(Q / (float(np.median(ts)) * 1e-3), 1),
               "batches": args.e2e_batches,
               "what": "bm25_search host buffers: H2D queries -> search -> D2H docs+scores, "
                       "host clock around the synchronous call"}
    nnz_total = int(indptr[-1])
    q_done = Q  # queries one step searches on this rank
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        if replica:  # every rank holds the whole index; the batch is split
            z = torch.tensor([Q], dtype=torch.int64, device=dev)
            dist.all_reduce(z)
            q_done = int(z.item())
        else:
            z = torch.tensor([nnz_total], dtype=torch.int64, device=dev)
            dist.all_reduce(z)  # the realised postings of every rank's shard
            nnz_total = int(z.item())

    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    qps = q_done * args.steps / elapsed
    # roofline of the dominant kernel on this rank (rank 0 reports its own)
    alg_bytes = algorithmic_bytes(indptr, queries, k)
    kern_ms = prof["score_ms"] / max(prof["score_launches"], 1)
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    shift = int(np.log2(info["tile_docs"]))
    default_k = cfg.k == synth.CONFIGS[args.config].k
    traffic = (load_traffic(args.traffic, args.config, shift, T)
               if world == 1 and not replica and default_k else None)
    large_k = "large_k" in dispatch["kernels"]
    # an index that fits the 256 MB Infinity Cache (MALL) is not HBM-bound:
    # its rate is effective bandwidth over algorithmic bytes (config 2)
    mall = info["device_bytes"] < 256 * 2**20
    # the bytes beside the algorithmic ones: what the
    # tile-bound skip spared (the kernel never reads those postings, so the
    # algorithmic rate is partly an effective rate), the batch's distinct
    # posting bytes (the reuse floor) and the counter-measured bytes
    skip_post = max(0, int(stats.get("bound_skipped_postings", 0)))
    n_post = query_postings(indptr, queries)
    distinct = batch_distinct_postings(indptr, queries)
    read_bytes = alg_bytes - 8 * skip_post
    phys = (traffic.get("hbm_bytes_per_launch") / (kern_ms * 1e-3) / 1e9) if traffic else None
    from bm25mi import _capi

    if rank == 0:
        out = {
            "metric": ("queries/sec + achieved HBM GB/s, 10M-doc CSC index, batch=1024, k=100"
                       if args.config == "c3" and not (replica and world == 1 and R > 1) else
                       (f"queries/sec per rank, {cfg.name}, rank {args.c5_rank} of 8 "
                        "(standalone shard search)" if emul else
                        (f"queries/sec per rank, {cfg.name}, rank 0 of a {R}-way replica job "
                         f"({Q} of {q_all} queries on the whole index)"
                         if replica and world == 1 and R > 1 else f"queries/sec, {cfg.name}"))),
            "value": round(qps, 2),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "ms_per_step_median": round(float(np.median(step_ms)), 4),
            "higher_is_better": True,
            "scaling": "strong",
            "native_lib": os.path.relpath(_capi.LIB, REPO),
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded Zipf CSC index + df^0.75 queries, csrc/synth.cpp; "
                    f"weights: {cfg.weights})",
            "config": {
                "workload": f"{args.config}: {cfg.name}, {T} terms per query" + (
                    f"; one rank's doc shard [{lo}, {hi}) of the 8-GPU job" if emul else "") + (
                    f"; replica mode: {Q} of the {q_all} queries per GPU" if replica else ""),
                "segments": "sparse" if info.get("sparse") else "dense",
                "n_docs": cfg.n_docs, "n_terms": cfg.n_terms, "nnz": nnz_total,
                "batch": Q, "terms_per_query": T, "k": k,
                "tile_docs": info["tile_docs"],
                "parallelism": (f"replica x{world} (whole index per GPU, batch split, no "
                                "collective)" if replica else f"doc-shard x{world}" + (
                    (f" + ONE {'RCCL' if args.backend == 'nccl' else args.backend} all-gather "
                     "per batch (packed [Q, k] lists; every rank keeps the world's tile bounds, "
                     "all-gathered once at setup)" if one_coll else
                     f" + {'RCCL' if args.backend == 'nccl' else args.backend} all-gathers "
                     "(sample keys, packed [Q, k] lists)") + (
                        f", batch pipelined as {args.parts} parts on forked contexts"
                        if args.parts > 1 else "") if world > 1 else "")),
                "score_kernels": sorted(dispatch["kernels"]),
                "term_lanes": dispatch["term_lanes"],
                "tiles_per_item": dispatch["band_tiles"],
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
                "traffic_source": (f"profiles/traffic.json ({traffic.get('source')}): "
                                   f"{traffic.get('method')}; L2 hit rate "
                                   f"{traffic.get('l2_hit_rate')}") if traffic else None,
                "kernel": (("large-k list path (score_flat_kernel SAMPLE slice maxima + "
                            "row_kth_kernel theta + score_flat_kernel REST crossing lists into "
                            "per-tile slots + slot_pack / row_kth / list_compact + LDS row sort)")
                           if large_k and "flat_rest" in dispatch["kernels"] else
                           "large-k search (scores_batch_kernel dense sums + lk_* radix "
                           "selection + row sort)" if large_k else
                           "score pass (bound_keys_kernel tile-bound threshold + "
                           "score_flat_kernel REST)" if "bound_keys" in dispatch["kernels"] else
                           "score pass (score_flat_kernel SAMPLE + theta_wave_kernel + "
                           "score_flat_kernel REST)"),
                "kernel_ms": round(kern_ms, 4),
                "alg_bytes_per_launch": alg_bytes,
                "achieved_kind": ("effective: algorithmic bytes (SURVEY.md §8(d)) over the pass "
                                  "time, including postings the REST tile skip never reads"
                                  if skip_post > 0 else
                                  "algorithmic bytes (SURVEY.md §8(d)) over the pass time"),
                "bound_skip": {"pairs": max(0, int(stats.get("bound_skipped_tiles", 0))),
                               "postings": skip_post,
                               "share_of_postings": round(skip_post / max(n_post, 1), 4),
                               "read_bytes": read_bytes,
                               "read_frac": round(read_bytes / (kern_ms * 1e-3) / 1e9
                                                  / HBM_PEAK_GBPS, 4),
                               "note": "postings of the (query, tile) pairs whose term-maxima "
                                       "sum stayed below theta (counted in one more search "
                                       "of the batch by the count_skips build); read_bytes = "
                                       "algorithmic minus 8 B per skipped posting"},
                "batch_distinct_bytes": {"postings": distinct, "at_6B": 6 * distinct,
                                         "at_8B": 8 * distinct,
                                         "reuse": round(n_post / max(distinct, 1), 2),
                                         "note": "every distinct term of the batch read once: "
                                                 "6 B/posting in this engine's layout (u16 slot "
                                                 "+ f32), 8 B on disk"},
                "physical_GBps": round(phys, 1) if phys else None,
                "physical_frac": round(phys / HBM_PEAK_GBPS, 4) if phys else None,
                "scope": ("rank 0's query slice" if replica else
                          "rank 0's shard" if world > 1 else "the whole index"),
                "note": (f"index of {info['device_bytes'] / 2**20:.1f} MiB fits the 256 MB "
                         "Infinity Cache (MALL): effective GB/s over algorithmic bytes, not an "
                         "HBM-bound rate" if mall else None),
            },
            "cpu_baseline": cpu,
            "e2e": e2e,
        }
        if cfg.k != synth.CONFIGS[args.config].k:  # a --k side line, not the config's metric
            out["metric"] = f"queries/sec, {args.config} index ({cfg.n_docs} docs) at k={cfg.k}"
            out["config"]["workload"] += f"; k={cfg.k} instead of the config's " \
                                         f"{synth.CONFIGS[args.config].k}"
        print(json.dumps(out), flush=True)
    index.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
