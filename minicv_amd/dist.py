"""Multi-GPU RANSAC: hypothesis batches sharded over ranks, one all-reduce for the global best.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on ROCm). Every rank
holds a full replica of the N correspondences (1.6 MB at N = 100k) and evaluates its own
contiguous range of hypothesis indices with the same counter-based sampler, so the union over
ranks is exactly the hypothesis stream a single GPU would evaluate. The exchange step is a
single all-reduce(MAX) over two int64 words per rank:
    word 0 = packed key (count << 32 | 0xFFFFFFFF - hypIndex)   -> global "first strictly greater"
    word 1 = -(first sampler failure index)                      -> global first failure (as MAX)
If the global winner lies after the global first sampler failure (degenerate input only),
the ranks re-evaluate their ranges truncated at the failure and reduce once more, reproducing
the sequential loop's `break`. That path is exact for fixed-iteration calls (MCV_FLAG_FIXED_ITERS).

Adaptive calls (OpenCV's niters shrinking with the best inlier ratio) need the counts in order:
`global_replay` evaluates the hypothesis stream in chunks (the same chunk schedule as the
single-process ransac_search), shards each chunk over the ranks, all-gathers the per-hypothesis
counts (4 B per model slot: 256 KB for a 65536-hypothesis chunk) and runs the sequential replay
(mcvReplayChunkModels, host code of libMiniCVNative.so) identically on every rank — the answer of
the single-GPU sequential loop, including where it stops.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, List, Tuple

import numpy as np

NO_FAIL = (1 << 63) - 1
CHUNK_FIRST = 4096        # ransac_search's chunk schedule (plan.h: kChunkFirst, doubling to kChunkMax)
CHUNK_MAX = 1 << 20


def shard(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [begin, begin + count) share of `total` hypotheses for `rank`."""
    base, rem = divmod(total, world)
    begin = rank * base + min(rank, rem)
    return begin, base + (1 if rank < rem else 0)


def unpack(key: int) -> Tuple[int, int]:
    key &= 0xFFFFFFFFFFFFFFFF
    if key == 0:
        return 0, -1
    return key >> 32, 0xFFFFFFFF - (key & 0xFFFFFFFF)


def global_best(evaluate: Callable[[int, int], Tuple[int, int]], total: int, rank: int, world: int,
                allreduce_max: Callable[[list], list], slots: int = 1, fixed: bool = True) -> Tuple[int, int, int]:
    """evaluate(begin, count) -> (key, first_fail) for this rank's range of hypotheses (device work);
    allreduce_max([a, b]) -> elementwise MAX over ranks. Returns (count, index, first_fail).
    With multi-model hypotheses (essential: slots = 10) keys, index and first_fail are slot indices
    (hypothesis h owns slots h * slots .. h * slots + slots - 1). Exact only for fixed-iteration
    calls: an adaptive call (fixed=False) is refused — use global_replay."""
    if not fixed:
        raise ValueError("global_best ignores the adaptive iteration bound; use global_replay for adaptive RANSAC")
    begin, count = shard(total, rank, world)
    key, fail = evaluate(begin, count) if count > 0 else (0, NO_FAIL)
    g = allreduce_max([key, -fail])
    gkey, gfail = g[0], -g[1]
    cnt, idx = unpack(gkey)
    if gfail != NO_FAIL and idx >= 0 and idx > gfail:
        end = min(begin + count, gfail // slots)
        key2, _ = evaluate(begin, end - begin) if end > begin else (0, NO_FAIL)
        g2 = allreduce_max([key2, 0])
        cnt, idx = unpack(g2[0])
    elif gfail != NO_FAIL and idx < 0:
        cnt, idx = 0, -1
    return cnt, idx, gfail


def global_replay(evaluate_counts: Callable[[int, int], np.ndarray], n_corr: int, model_points: int,
                  confidence: float, max_iters: int, rank: int, world: int,
                  allgather: Callable[[np.ndarray, List[int]], List[np.ndarray]], fixed: bool = False,
                  slots: int = 1) -> Tuple[int, int]:
    """Multi-rank RANSAC with OpenCV's sequential semantics, adaptive termination included.

    evaluate_counts(begin, count) -> int32 counts of this rank's hypotheses [begin, begin + count)
    (count * slots entries: >= 0 inliers, -1 no model, -2 sampler failure); allgather(arr, lens) ->
    the arrays of all ranks in rank order (lens: every rank's entry count). Returns (best count, best index) with index a slot index when
    slots > 1 (-1 when no model reaches the minimal sample size)."""
    from . import native as N
    lib = N.lib()
    st = N.ReplayState()
    lib.mcvReplayInit(C.byref(st), int(max_iters))
    begin = 0
    chunk = min(max(int(st.niters), 1), CHUNK_FIRST)
    while not st.stopped:
        remaining = int(st.niters) - begin
        if remaining <= 0:
            break
        cnt = min(remaining, chunk)
        b, c = shard(cnt, rank, world)
        local = np.ascontiguousarray(evaluate_counts(begin + b, c) if c > 0 else np.zeros(0, np.int32),
                                     dtype=np.int32)
        if local.shape[0] != c * slots:
            raise ValueError(f"evaluate_counts returned {local.shape[0]} entries, expected {c * slots}")
        parts = allgather(local, [shard(cnt, r, world)[1] * slots for r in range(world)])
        counts = np.ascontiguousarray(np.concatenate(parts), dtype=np.int32)
        if counts.shape[0] != cnt * slots:
            raise ValueError("all-gathered counts do not cover the chunk")
        lib.mcvReplayChunkModels(C.byref(st), counts.ctypes.data, begin, cnt, slots, n_corr, model_points,
                                 float(confidence), 1 if fixed else 0)
        begin += cnt
        chunk = min(chunk * 2, CHUNK_MAX)
    return int(st.bestCount), int(st.bestIndex)


def torch_allgather(dist, device=None):
    """allgather for global_replay over torch.distributed (RCCL over xGMI with device tensors, gloo on
    CPU): the int32 arrays padded to the longest shard (shards differ by at most one hypothesis),
    one all_gather per chunk."""
    import torch

    def gather(arr: np.ndarray, lens: List[int]) -> List[np.ndarray]:
        m = max(lens)
        buf = torch.full((max(m, 1),), -1, dtype=torch.int32, device=device)
        if arr.shape[0]:
            buf[:arr.shape[0]] = torch.from_numpy(arr).to(device)
        outs = [torch.empty_like(buf) for _ in lens]
        dist.all_gather(outs, buf)
        return [o[:l].cpu().numpy() for o, l in zip(outs, lens)]

    return gather
