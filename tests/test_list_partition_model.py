"""CPU model of the ragged-list work split (engine.cpp list_stream + crc_kernels.hip
crc32_list_stream_kernel): the host cuts the list's sequence of 4 KiB groups evenly
over the waves and gives each wave its first buffer, its first group in it and its group range; the
kernel walks forward from there.  The model replays both sides and checks that every group of every
buffer is scanned by exactly one wave, that every buffer without a main region is folded by exactly
one wave, and that the parts of a buffer add up to its group count (the completion rule of the
per-buffer accumulator)."""
import random

import pytest

GB = 4096


def host_split(groups, nw):
    """list_stream: wbuf / woff / wq for nw waves (groups[b] = 4 KiB groups of buffer b)."""
    count = len(groups)
    gp = [0]
    for g in groups:
        gp.append(gp[-1] + g)
    ng = gp[-1]
    wbuf, woff, wq = [], [], []
    b = 0
    for w in range(nw + 1):
        q0 = ng if w == nw else w * ng // nw
        if w == nw:
            b = count
        else:
            while b < count and gp[b + 1] <= q0 and not (gp[b + 1] == gp[b] and gp[b] >= q0):
                b += 1
        wbuf.append(b)
        wq.append(q0)
        woff.append(q0 - gp[b] if b < count and gp[b + 1] > gp[b] else 0)
    return wbuf, woff, wq


def kernel_walk(groups, wbuf, woff, wq, w):
    """one wave of crc32_list_stream_kernel: (buffer, group) pairs scanned, buffers folded whole,
    and the parts it finishes as (buffer, first group, end group)"""
    count = len(groups)
    b0, b_end, g0, nq = wbuf[w], wbuf[w + 1], woff[w], wq[w + 1] - wq[w]
    scanned, empties, parts = [], [], []
    sc = b0
    if b0 < b_end or nq:
        while groups[sc] == 0:
            empties.append(sc)
            if nq == 0 and sc + 1 >= b_end:
                break
            sc += 1
    if nq == 0:
        return scanned, empties, parts
    g, ga, q = g0, g0, 0
    while q < nq:
        scanned.append((sc, g))
        q += 1
        g += 1
        if g == groups[sc] or q == nq:
            parts.append((sc, ga, g))
            if q < nq:
                while True:
                    sc += 1
                    assert sc < count
                    if groups[sc]:
                        break
                    empties.append(sc)
                g = ga = 0
    while sc + 1 < b_end:
        sc += 1
        assert groups[sc] == 0
        empties.append(sc)
    return scanned, empties, parts


def check(groups, nw):
    wbuf, woff, wq = host_split(groups, nw)
    seen, folded, done = {}, {}, {}
    for w in range(nw):
        scanned, empties, parts = kernel_walk(groups, wbuf, woff, wq, w)
        for k in scanned:
            assert k not in seen, (k, w, seen.get(k))
            seen[k] = w
        for e in empties:
            assert e not in folded
            folded[e] = w
        for b, ga, gz in parts:
            assert 0 <= ga < gz <= groups[b]
            done[b] = done.get(b, 0) + (gz - ga)
    want = {(b, g) for b, n in enumerate(groups) for g in range(n)}
    assert set(seen) == want
    assert set(folded) == {b for b, n in enumerate(groups) if n == 0}
    assert done == {b: n for b, n in enumerate(groups) if n}
    # the split is even: every wave scans floor or ceil of the mean
    per = [wq[w + 1] - wq[w] for w in range(nw)]
    assert max(per) - min(per) <= 1


@pytest.mark.parametrize("seed", range(40))
def test_list_split_random(seed):
    rng = random.Random(seed)
    count = rng.choice([1, 2, 3, 17, 300, 4096])
    groups = [rng.choice([0, 0, 1, 2, 8, 9, 16, 24, 100]) for _ in range(count)]
    if not any(groups):
        groups[rng.randrange(count)] = 1
    nw = rng.choice([8, 64, 512, 4096])
    check(groups, nw)


@pytest.mark.parametrize("groups,nw", [
    ([0, 5, 0, 0, 3, 0], 8),           # empties on every edge, more waves than groups
    ([16] * 4096, 4096),               # one buffer per wave (C2-like lists)
    ([262144], 4096),                  # one 1 GiB buffer cut into 4096 parts
    ([0] * 100 + [1] + [0] * 100, 16),  # a single group among empties
    ([8, 24] * 2048, 4096),            # ragged 32-96 KiB-like
    ([8], 8),                          # a wave whose buffer range is empty but which has groups
    ([0, 0, 8, 0], 64),
])
def test_list_split_edges(groups, nw):
    check(groups, nw)
