"""Multi-rank path on CPU (gloo, world_size 2 and 3): hypothesis sharding + the one all-reduce that
combines per-rank best keys (minicv_amd/dist.py) must reproduce the single-process sequential
RANSAC answer, including the sampler-failure `break`. The per-rank "device" evaluation is played
by precomputed per-hypothesis counts (from the oracle), reduced like mcv_best_* does."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from minicv_amd import dist as MD


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def local_key(counts, begin, count, m=4, slots=1):
    """What mcv_best_partial/final compute for one rank's range (slot indices when slots > 1)."""
    begin, count = begin * slots, count * slots
    seg = counts[begin:begin + count]
    fail = np.nonzero(seg == -2)[0]
    lim = int(fail[0]) if len(fail) else count
    first_fail = begin + int(fail[0]) if len(fail) else MD.NO_FAIL
    valid = seg[:lim] >= m
    if not valid.any():
        return 0, first_fail
    c = int(seg[:lim].max())
    i = int(np.nonzero(seg[:lim] == c)[0][0])
    return (c << 32) | (0xFFFFFFFF - (begin + i)), first_fail


def _worker_replay(rank, world, port, counts, q, n, m, conf, max_iters, fixed, slots):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    evaluated = []

    def evaluate_counts(begin, count):
        evaluated.append((begin, count))
        return counts[begin * slots:(begin + count) * slots]

    res = MD.global_replay(evaluate_counts, n, m, conf, max_iters, rank, world, MD.torch_allgather(dist),
                           fixed=fixed, slots=slots)
    q.put((rank, (res, sum(c for _, c in evaluated))))
    dist.destroy_process_group()


def run_replay(world, counts, n, m, conf, max_iters, fixed, slots=1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_replay, args=(r, world, port, counts, q, n, m, conf, max_iters, fixed, slots))
          for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return out


def _worker(rank, world, port, counts, q, m=4, slots=1):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def evaluate(begin, count):
        return local_key(counts, begin, count, m, slots)

    def allreduce_max(vals):
        t = torch.tensor(vals, dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [int(v) for v in t]

    res = MD.global_best(evaluate, len(counts) // slots, rank, world, allreduce_max, slots=slots)
    q.put((rank, res))
    dist.destroy_process_group()


def run_ranks(world, counts, m=4, slots=1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, counts, q, m, slots)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return out


def test_shard_covers_range():
    for total in (1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [MD.shard(total, r, world) for r in range(world)]
            assert spans[0][0] == 0
            assert sum(c for _, c in spans) == total
            for (b0, c0), (b1, _) in zip(spans, spans[1:]):
                assert b0 + c0 == b1


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_best_matches_sequential(oracle, world):
    from minicv_amd import synthetic as S
    src, dst, _ = S.homography_problem(500, 31)
    pts4 = oracle.pack4(src, dst)
    counts = oracle.h_counts(pts4, 31, 0, 3000, float(np.float32(5e-3 ** 2)))
    best, bc = oracle.replay(counts, 500, 4, 0.995, len(counts), fixed=True)
    out = run_ranks(world, counts)
    for r in range(world):
        assert out[r][0] == bc and out[r][1] == best


def test_distributed_sampler_failure_break(oracle):
    rng = np.random.default_rng(5)
    counts = rng.integers(0, 100, size=1000).astype(np.int32)
    counts[700] = 500          # global max lies after the failure ...
    counts[400] = -2           # ... which stops the sequential loop at 400
    counts[100] = 99
    counts[:100] = np.minimum(counts[:100], 50)
    best, bc = oracle.replay(counts, 1000, 4, 0.99, len(counts), fixed=True)
    assert best < 400
    out = run_ranks(2, counts)
    for r in range(2):
        assert out[r][0] == bc and out[r][1] == best and out[r][2] == 400


def test_distributed_essential_slots(oracle):
    """Multi-model hypotheses (five-point: <= 10 E per sample): slot-indexed keys over 2 ranks equal
    the sequential replay, also when a sampler failure truncates the stream."""
    from minicv_amd import synthetic as S
    a, b, *_ = S.essential_problem(400, seed=8, outlier_frac=0.5)
    p = oracle.pack_e(a, b, 800.0, (640.0, 360.0))
    counts = oracle.e_counts(p, 8, 0, 600, float(np.float32((1.0 / 800.0) ** 2)))
    best, bc = oracle.replay_slots(counts, 600, 400, 5, 0.999, 600, True)
    out = run_ranks(2, counts, m=5, slots=10)
    for r in range(2):
        assert out[r][0] == bc and out[r][1] == best
    c2 = counts.copy()
    c2[10 * 450] = -2
    c2[10 * 500] = 400           # best after the failure must be ignored
    best2, bc2 = oracle.replay_slots(c2, 600, 400, 5, 0.999, 600, True)
    out = run_ranks(2, c2, m=5, slots=10)
    for r in range(2):
        assert out[r][0] == bc2 and out[r][1] == best2 and out[r][2] == 4500


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_adaptive_replay_matches_sequential(oracle, world):
    """Adaptive termination across ranks (no FIXED_ITERS): chunked sharding + all-gather of the counts
    + the sequential replay on every rank equals the single-process replay (winner and stopping
    point); the ranks evaluate no more than the chunks up to the stop."""
    from minicv_amd import synthetic as S
    n = 2000
    src, dst, _ = S.homography_problem(n, 33, outlier_frac=0.6)
    pts4 = oracle.pack4(src, dst)
    max_iters = 20000
    counts = oracle.h_counts(pts4, 33, 0, max_iters, float(np.float32(5e-3 ** 2)))
    best, bc = oracle.replay(counts, n, 4, 0.995, max_iters, fixed=False)
    out = run_replay(world, counts, n, 4, 0.995, max_iters, False)
    total = sum(v[1] for v in out.values())
    assert total < max_iters          # stopped early, like the sequential loop
    for r in range(world):
        assert out[r][0] == (bc, best)
    best_f, bc_f = oracle.replay(counts, n, 4, 0.995, 3000, fixed=True)
    out = run_replay(world, counts[:3000], n, 4, 0.995, 3000, True)
    for r in range(world):
        assert out[r][0] == (bc_f, best_f)


def test_distributed_adaptive_replay_essential_slots_and_failure(oracle):
    from minicv_amd import synthetic as S
    a, b, *_ = S.essential_problem(400, seed=9, outlier_frac=0.5)
    p = oracle.pack_e(a, b, 800.0, (640.0, 360.0))
    counts = oracle.e_counts(p, 9, 0, 1000, float(np.float32((1.0 / 800.0) ** 2)))
    best, bc = oracle.replay_slots(counts, 1000, 400, 5, 0.999, 1000, False)
    out = run_replay(2, counts, 400, 5, 0.999, 1000, False, slots=10)
    for r in range(2):
        assert out[r][0] == (bc, best)
    c2 = counts.copy()
    c2[10 * 37] = -2                      # sampler failure: the loop breaks there
    best2, bc2 = oracle.replay_slots(c2, 1000, 400, 5, 0.999, 1000, False)
    out = run_replay(3, c2, 400, 5, 0.999, 1000, False, slots=10)
    for r in range(3):
        assert out[r][0] == (bc2, best2)
