"""Doc-sharded search across ranks.

One process per GPU.  Rank r owns the contiguous document range
``shard_bounds(N, W, r)`` (bm25mi.shard) as an independent index whose ``doc_offset``
is the global id of its first document, and searches the whole (replicated)
query batch on it.  The path has two exchanges, both all-gathers (RCCL over
xGMI with the ``nccl`` backend): every rank's sample keys (global doc ids),
from which each rank takes the same global threshold, and every rank's
[Q, k] list of keys above it (global doc ids + scores), merged by the same
(score desc, doc asc) rule — so the result is exactly the single-index top-k.

The reference has no multi-device path (``DEVICE_ID = 0`` at
main.py:205); this module is the build's only collective.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist

from .shard import shard_bounds  # noqa: F401  (the one definition; re-exported here)

# merge(g_docs [W,Q,k] int32, g_scores [W,Q,k] f32) -> (docs [Q,k], scores [Q,k])
MergeFn = Callable[[torch.Tensor, torch.Tensor], Tuple[torch.Tensor, torch.Tensor]]


def _all_gather(x: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """[...] on every rank -> [W, ...] (rank-major).  RCCL (backend "nccl")
    gathers device tensors in place over xGMI; gloo (CPU tests, several ranks
    sharing one GPU) has no into-tensor form and no device all_gather, so
    device tensors are staged through host memory there."""
    world = dist.get_world_size(group)
    x = x.contiguous()
    if dist.get_backend(group) != "gloo":
        out = torch.empty((world,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x, group=group)
        return out
    h = x.cpu()
    out = torch.empty((world,) + tuple(h.shape), dtype=h.dtype)
    dist.all_gather(list(out.unbind(0)), h, group=group)
    return out.to(x.device)


def all_gather_lists(docs: torch.Tensor, scores: torch.Tensor,
                     group: Optional[dist.ProcessGroup] = None
                     ) -> Tuple[torch.Tensor, torch.Tensor]:
    """All ranks' [Q, k] lists -> [W, Q, k] (rank-major), on every rank."""
    return _all_gather(docs, group), _all_gather(scores, group)


def sharded_topk(docs: torch.Tensor, scores: torch.Tensor, merge: MergeFn,
                 group: Optional[dist.ProcessGroup] = None
                 ) -> Tuple[torch.Tensor, torch.Tensor]:
    """This rank's [Q, k] list (global doc ids) -> the global [Q, k] top-k."""
    if dist.get_world_size(group) == 1:
        return docs, scores
    g_docs, g_scores = all_gather_lists(docs, scores, group)
    return merge(g_docs, g_scores)


def gpu_merge(device: int, stream=None) -> MergeFn:
    """The HIP merge (bm25_merge_topk_device) as a MergeFn, on ``stream``."""
    from .index import merge_topk_device

    def merge(g_docs: torch.Tensor, g_scores: torch.Tensor):
        W, Q, k = g_docs.shape
        out_d = torch.empty((Q, k), dtype=torch.int32, device=g_docs.device)
        out_s = torch.empty((Q, k), dtype=torch.float32, device=g_docs.device)
        merge_topk_device(device, g_docs, g_scores, W, Q, k, out_d, out_s, stream)
        return out_d, out_s

    return merge


def _group_key(group):
    return dist.group.WORLD if group is None else group


def _global_docs(index, device, group=None) -> int:
    """Documents of the whole collection: the sum of every rank's shard,
    all-reduced once per process group and cached on the index object."""
    cache = index.__dict__.setdefault("_bm25_global_docs", {})
    n = cache.get(_group_key(group))
    if n is None:
        if dist.get_world_size(group) == 1:
            n = int(index.n_docs)
        else:
            backend = dist.get_backend(group)
            t = torch.tensor([int(index.n_docs)], dtype=torch.int64,
                             device="cpu" if backend == "gloo" else device)
            dist.all_reduce(t, group=group)
            n = int(t.item())
        cache[_group_key(group)] = n
    return n


def _agree_width(index, S: int, k: int, device, group=None) -> None:
    """Every rank must sample the same width S (the key all-gather has one
    shape): it depends on k, the world and the handle's ``sample_p`` and
    ``theta_bound`` options (and on the shard having tile bounds), which each
    rank sets on its own.  Checked once per (group, k) by one
    all-reduce of (S, -S) with MAX; every rank raises the same ValueError when
    they differ.  GpuIndex.set_option drops the cache, so a changed option
    is re-checked on the next search — every rank must change it together."""
    seen = index.__dict__.setdefault("_bm25_width_ok", set())
    key = (_group_key(group), int(k))
    if key in seen:
        return
    backend = dist.get_backend(group)
    t = torch.tensor([S, -S], dtype=torch.int64, device="cpu" if backend == "gloo" else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    lo, hi = -int(t[1].item()), int(t[0].item())
    if lo != hi:
        raise ValueError(f"ranks disagree on the sample width at k={k} (min {lo}, max {hi}): "
                         "set the same sample_p and theta_bound options on every rank's index "
                         "(theta_bound needs every shard's tile bounds: dense, non-negative)")
    seen.add(key)


BOUND_MAX_TILES = 30720  # tiles one block selects a threshold over (kBoundMaxTiles)


def setup_world_bounds(index, group: Optional[dist.ProcessGroup] = None, stream=None,
                       device=None) -> bool:
    """The one-collective protocol's setup (include/bm25mi.h,
    bm25_search_shard_device): every rank exports its shard's tile bounds, the
    ranks all-gather them once, and each rank's handle keeps the world's
    [W, n_terms, stride] table, so a search takes the whole collection's
    tile-bound threshold without the per-batch key exchange.  Collective:
    every rank calls it; False (on every rank) when a shard keeps no tile
    bounds or the collection has more tiles than one block selects over
    (config 5: the two-exchange protocol stays).  ~2 GB per rank at config 3."""
    world = dist.get_world_size(group)
    info = index.info()
    dev = torch.device(device) if device is not None else torch.device("cuda", index.device)
    backend = dist.get_backend(group)
    tdev = "cpu" if backend == "gloo" else dev
    # (no bounds anywhere -> 1, widest stride) by one MAX all-reduce; tiles by a SUM
    t = torch.tensor([0 if info["tile_bounds"] else 1, index.bounds_stride()], dtype=torch.int64,
                     device=tdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    n = torch.tensor([int(info["n_tiles"])], dtype=torch.int64, device=tdev)
    dist.all_reduce(n, group=group)
    missing, stride, tiles = int(t[0].item()), int(t[1].item()), int(n.item())
    if missing or world * stride > BOUND_MAX_TILES + 4 * world or tiles < 1:
        return False
    local = torch.empty((index.n_terms, stride), dtype=torch.int16, device=dev)
    st = (stream if stream is not None else torch.cuda.current_stream(dev)) if dev.type == "cuda" \
        else None
    index.bounds_export(local, stride, st)
    with _stream_ctx(st):  # (as int32 pairs: RCCL and gloo move no int16)
        g = _all_gather(local.view(torch.int32), group).view(torch.int16)  # [W, n_terms, stride]
    if st is not None:
        st.synchronize()
    index.set_world_bounds(g, world, stride, tiles)
    return True


def gather_keys(keys: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """All ranks' [Q, S] sample keys -> [W, Q, S] (rank-major), on every rank."""
    return _all_gather(keys, group)


def _forks(index, parts: int):
    """The index and parts - 1 forks of it (bm25_index_fork: shared device
    arrays, own workspaces), created once and cached on the index.  Options
    are copied at fork time; set_option on the index drops the cache."""
    forks = index.__dict__.setdefault("_bm25_forks", [])
    while len(forks) < parts - 1:
        forks.append(index.fork())
    return [index] + forks[:parts - 1]


def _part_streams(index, parts: int, device):
    """One torch stream per part (cached on the index), or None on the CPU."""
    if device.type != "cuda":
        return [None] * parts
    st = index.__dict__.setdefault("_bm25_part_streams", [])
    while len(st) < parts:
        st.append(torch.cuda.Stream(device=device))
    return st[:parts]


def _stream_ctx(s):
    import contextlib
    return torch.cuda.stream(s) if s is not None else contextlib.nullcontext()


def _search_parts(index, d_queries, k, shard_docs_max, d_docs, d_scores, stream, group, world,
                  S, parts):
    """sharded_search over `parts` contiguous row ranges of the batch, each
    on its own fork of the index and its own stream, issued phase by phase
    (every part's sample half, every part's key all-gather, every finish
    half, every list all-gather, every W-way merge).  The device then runs one
    part's collectives and its latency-bound kernels (threshold, merges: one
    wavefront per query) beside another part's score pass — the per-batch
    fixed costs of a doc shard overlap instead of adding up.
    Collectives keep one issue order on every rank.  The result is the
    unsplit search's, row for row."""
    from .index import merge_sorted_device
    Q = d_queries.shape[0]
    cuts = [Q * i // parts for i in range(parts + 1)]
    rows = [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
    ctxs = _forks(index, len(rows))
    dev = d_queries.device
    streams = _part_streams(index, len(rows), dev)
    if streams[0] is not None:  # the parts start after the caller's stream
        ev = torch.cuda.Event()
        ev.record(stream)
        for s in streams:
            s.wait_event(ev)
    qs = [d_queries[a:b] for a, b in rows]
    keys, all_keys, packed, gathered = [], [], [], []
    for i, (a, b) in enumerate(rows):
        with _stream_ctx(streams[i]):
            kk = (torch.empty if S > 0 else torch.zeros)((b - a, max(S, 1)), dtype=torch.int64,
                                                        device=dev)
            if S > 0:
                ctxs[i].search_sample_device(qs[i], k, world, shard_docs_max, kk, streams[i])
            keys.append(kk)
    for i in range(len(rows)):
        with _stream_ctx(streams[i]):
            all_keys.append(gather_keys(keys[i], group) if world > 1 and S > 0
                            else keys[i].unsqueeze(0))
    for i, (a, b) in enumerate(rows):
        with _stream_ctx(streams[i]):
            pk = torch.empty((2, b - a, k), dtype=torch.int32, device=dev)
            ctxs[i].search_finish_device(qs[i], k, world, shard_docs_max, all_keys[i], pk[0],
                                         pk[1].view(torch.float32), streams[i])
            packed.append(pk)
    for i in range(len(rows)):
        with _stream_ctx(streams[i]):
            gathered.append(_all_gather(packed[i], group) if world > 1 else packed[i].unsqueeze(0))
    for i, (a, b) in enumerate(rows):
        with _stream_ctx(streams[i]):
            g = gathered[i]
            merge_sorted_device(dev.index, g, g[:, 1].view(torch.float32), world, b - a, k,
                                2 * (b - a) * k, d_docs[a:b], d_scores[a:b], streams[i])
    if streams[0] is not None:  # the caller's stream continues after every part
        for s in streams:
            ev = torch.cuda.Event()
            ev.record(s)
            stream.wait_event(ev)
    return d_docs, d_scores


def sharded_search(index, d_queries: torch.Tensor, k: int, shard_docs_max: int,
                   d_docs: torch.Tensor, d_scores: torch.Tensor,
                   merge: Optional[MergeFn] = None, stream=None,
                   group: Optional[dist.ProcessGroup] = None,
                   exchange: Optional[Callable[[torch.Tensor], torch.Tensor]] = None,
                   n_docs_total: Optional[int] = None, parts: int = 1
                   ) -> Tuple[torch.Tensor, torch.Tensor]:
    """One rank's doc-sharded search with a GLOBAL threshold (bm25_search_
    sample/finish_device): this shard's sample keys are all-gathered, theta =
    the k-th best key of the whole sample, the shard lists its keys >= theta,
    and the lists are all-gathered and merged.  Two collectives per batch:
    W*Q*S*8 B of sample keys (S ~ 2k/W: ~200 KB per rank at config 3) and the
    [Q, k] lists — docs and scores in one packed [2, Q, k] buffer, merged by
    the W-way merge of best-first lists (bm25_merge_sorted_device) unless a
    ``merge`` of the two gathered arrays is given.  ``exchange`` replaces the
    key all-gather (tests).

    Everything — kernels and collectives — is enqueued on ``stream`` (default:
    the current stream; a torch.cuda.Stream or a raw hipStream_t handle): the
    collectives order against torch's current stream, so the body runs with
    ``stream`` made current.

    ``k`` is checked against the whole collection's document count, as the
    single-index search checks it (numpy's argpartition error,
    bm25_native.py:205): ``n_docs_total``, or one all-reduce of the shards'
    counts on the first search (cached on ``index``).

    ``parts`` > 1 (packed lists, no ``merge`` / ``exchange``): the batch's
    rows are searched as that many parts pipelined over forks of the index
    on their own streams (``_search_parts``) — the same result."""
    world = int(exchange.world) if exchange is not None else dist.get_world_size(group)
    total = n_docs_total if n_docs_total is not None else (
        _global_docs(index, d_queries.device, group) if exchange is None else None)
    if total is not None and k > total:
        raise ValueError(f"kth(={total - k}) out of bounds ({total})")
    # (k > 4096: S = 0, every shard's exact top-k — bm25mi_large.hip)
    S = index.sample_width(k, world, shard_docs_max)
    if exchange is None and world > 1:
        _agree_width(index, S, k, d_queries.device, group)
    cuda = d_queries.device.type == "cuda"
    if not cuda:
        stream = None
    elif stream is None:
        stream = torch.cuda.current_stream(d_queries.device)
    elif not isinstance(stream, torch.cuda.Stream):
        stream = torch.cuda.ExternalStream(int(stream), device=d_queries.device)
    if (merge is None and exchange is None and parts <= 1
            and index.__dict__.get("_bm25_world_bounds") is not None):
        # one collective: the shard's keys >= the collection's threshold (its
        # own from the world bounds), all-gathered and merged
        with _stream_ctx(stream):
            Q = d_queries.shape[0]
            pk = torch.empty((2, Q, k), dtype=torch.int32, device=d_queries.device)
            index.search_shard_device(d_queries, k, pk[0], pk[1].view(torch.float32), stream)
            g = _all_gather(pk, group) if world > 1 else pk.unsqueeze(0)
            from .index import merge_sorted_device
            merge_sorted_device(d_queries.device.index, g, g[:, 1].view(torch.float32), world, Q,
                                k, 2 * Q * k, d_docs, d_scores, stream)
            return d_docs, d_scores
    if parts > 1 and merge is None and exchange is None:
        return _search_parts(index, d_queries, k, shard_docs_max, d_docs, d_scores, stream,
                             group, world, S, parts)
    if not cuda:
        raise ValueError("sharded_search runs on the GPU (parts > 1 for CPU protocol tests)")
    with torch.cuda.stream(stream):
        Q = d_queries.shape[0]
        # S > 0: the sample pass writes every key of its own width
        keys = (torch.empty if S > 0 else torch.zeros)((Q, max(S, 1)), dtype=torch.int64,
                                                       device=d_queries.device)
        if S > 0:
            index.search_sample_device(d_queries, k, world, shard_docs_max, keys, stream)
        if exchange is not None:
            all_keys = exchange(keys)
        elif world > 1 and S > 0:
            all_keys = gather_keys(keys, group)
        else:
            all_keys = keys.unsqueeze(0)
        packed = merge is None and exchange is None and world > 1
        if not packed:
            index.search_finish_device(d_queries, k, world, shard_docs_max, all_keys, d_docs,
                                       d_scores, stream)
            if exchange is not None or world == 1:
                return d_docs, d_scores
            return sharded_topk(d_docs, d_scores, merge, group)
        pk = torch.empty((2, Q, k), dtype=torch.int32, device=d_queries.device)
        index.search_finish_device(d_queries, k, world, shard_docs_max, all_keys, pk[0],
                                   pk[1].view(torch.float32), stream)
        g = _all_gather(pk, group)  # [W, 2, Q, k]: one collective for docs and scores
        # the merge reads rank w's docs at w * 2Qk and its scores Qk later
        assert tuple(g.shape) == (world, 2, Q, k) and g.is_contiguous(), tuple(g.shape)
        from .index import merge_sorted_device
        merge_sorted_device(d_queries.device.index, g, g[:, 1].view(torch.float32), world, Q, k,
                            2 * Q * k, d_docs, d_scores, stream)
        return d_docs, d_scores
