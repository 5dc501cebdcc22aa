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
the sequential loop's `break`.
"""
from __future__ import annotations

from typing import Callable, Tuple

NO_FAIL = (1 << 63) - 1


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
                allreduce_max: Callable[[list], list], slots: int = 1) -> Tuple[int, int, int]:
    """evaluate(begin, count) -> (key, first_fail) for this rank's range of hypotheses (device work);
    allreduce_max([a, b]) -> elementwise MAX over ranks. Returns (count, index, first_fail).
    With multi-model hypotheses (essential: slots = 10) keys, index and first_fail are slot indices
    (hypothesis h owns slots h * slots .. h * slots + slots - 1)."""
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
