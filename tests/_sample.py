"""Hypothesis-range samples for the full-size parity tests (test infrastructure).

bench.py runs F / E / PnP at 2^20 hypotheses per call and splits them over up to 8 ranks in
contiguous shares (rank r: [r 2^20 / R, (r + 1) 2^20 / R)). A full-range oracle count at the
bench's sizes costs minutes of CPU, so the tests compare a sample of 262144 hypotheses (a quarter) over
the whole range: the first and last `edge` hypotheses of every 8-rank share, `strided` blocks at
evenly spaced offsets between them, and a window around each named hypothesis (the bench's
reported winners, the device's own argmax).
"""


def bench_sample(total=1 << 20, ranks=8, edge=1024, strided=240, block=1024, around=(), window=64):
    """Sorted, merged [begin, end) ranges inside [0, total)."""
    share = total // ranks
    rng = []
    for r in range(ranks):
        rng.append((r * share, r * share + edge))
        rng.append(((r + 1) * share - edge, (r + 1) * share))
    step = total // strided
    for i in range(strided):
        b = i * step + (step // 2 // block) * block
        rng.append((b, b + block))
    for h in around:
        rng.append((max(0, h - window // 2), min(total, h + window // 2)))
    rng.sort()
    out = []
    for b, e in rng:
        b, e = max(0, b), min(total, e)
        if out and b <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], e))
        else:
            out.append((b, e))
    return out


def describe(ranges):
    n = sum(e - b for b, e in ranges)
    return f"{n} hypotheses in {len(ranges)} ranges: " + ", ".join(f"[{b},{e})" for b, e in ranges)
