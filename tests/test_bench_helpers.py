"""bench.py's host-side helpers (no GPU): the per-workload PMC traffic lookup
behind roofline.traffic and the SURVEY.md §8(d) algorithmic byte count
behind roofline.achieved."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_traffic_entries_match_their_workload():
    path = os.path.join(REPO, "profiles", "traffic.json")
    seen = {}
    for config, terms in (("c3", 8), ("c3", 16), ("c5", 8)):
        t = bench.load_traffic(path, config, 11, terms)
        assert t is not None, (config, terms)
        assert t["config"] == config and t["terms_per_query"] == terms
        assert abs(t["hbm_bytes_per_launch"] - t["read_bytes"] - t["write_size_bytes"]) <= 2
        assert t["hbm_bytes_per_launch"] > 0
        assert 0.0 < t["l2_hit_rate"] < 1.0 and t["method"] and t["source"]
        seen[(config, terms)] = t["hbm_bytes_per_launch"]
    # 16-term queries read about twice the postings of 8-term ones (more of
    # them L2 hits: the moved bytes grow less), and every entry stays below
    # its workload's algorithmic bytes (17.9 GB at 8 terms, 34.7 GB at 16)
    assert seen[("c3", 16)] > 1.2 * seen[("c3", 8)]
    assert seen[("c3", 8)] < 17.9e9 and seen[("c3", 16)] < 34.7e9
    assert bench.load_traffic(path, "c3", 12, 8) is None  # other tile size
    assert bench.load_traffic(path, "c2", 11, 8) is None  # never profiled


def test_traffic_single_entry_file(tmp_path):
    """The round-2 layout (one workload at the top level) still loads."""
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"config": "c3", "tile_shift": 11, "hbm_bytes_per_launch": 5,
                             "method": "m"}))
    assert bench.load_traffic(str(p), "c3", 11, 8)["hbm_bytes_per_launch"] == 5
    assert bench.load_traffic(str(p), "c3", 11, 16) is None
    assert bench.load_traffic(str(tmp_path / "missing.json"), "c3", 11, 8) is None


def test_algorithmic_bytes_formula():
    # terms 0..3 with df 2, 0, 5, 1; padding and a repeated term count once
    indptr = np.array([0, 2, 2, 7, 8], np.int64)
    q = np.array([[0, 2, 2, -1], [3, -1, -1, -1]], np.int32)
    k = 10
    want = ((8 * 2 + 8) + (8 * 5 + 8) + 4 * 4 + 8 * k) + ((8 * 1 + 8) + 4 * 4 + 8 * k)
    assert bench.algorithmic_bytes(indptr, q, k) == want


def test_posting_counts_per_query_and_batch_distinct():
    # terms 0..3 with df 2, 0, 5, 1; query 0 = {0, 2} (2 repeated), query 1 = {3},
    # query 2 = {2, 3}: per query 7 + 1 + 6, batch-distinct {0, 2, 3} = 8
    indptr = np.array([0, 2, 2, 7, 8], np.int64)
    q = np.array([[0, 2, 2, -1], [3, -1, -1, -1], [2, 3, -5, -1]], np.int32)
    assert bench.query_postings(indptr, q) == 14
    assert bench.batch_distinct_postings(indptr, q) == 8
    assert bench.batch_distinct_postings(indptr, np.full((2, 3), -1, np.int32)) == 0


def test_gpus_n_without_launcher_launches_ranks():
    """`bench.py --gpus 2` with no WORLD_SIZE starts the
    two ranks itself (a child torch.distributed.run on 127.0.0.1): the line
    reports n_gpus 2, or — here, with no GPU — the run fails non-zero.  It
    never silently measures one GPU."""
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--backend", "gloo", "--config", "c2", "--steps", "1", "--warmup", "0",
                        "--cpu-queries", "0", "--e2e-batches", "0", "--threads", "4"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert "launching 2 ranks" in r.stderr, r.stderr[-2000:]
    if r.returncode == 0:
        line = json.loads(r.stdout.strip().splitlines()[-1])
        assert line["n_gpus"] == 2
    else:
        assert r.returncode != 0


def test_gpus_mismatch_with_world_size_fails():
    """--gpus N under a launcher of another world size is an error, not a note."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--cpu-queries", "0"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr, r.stderr[-2000:]
