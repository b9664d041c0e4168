"""CPU model of crc32_stream_kernel's XCD-window tile order (ScanParams::xcd_order, round 4) and of the
engine's conditions for taking it (engine.cpp scan_batches): the waves of XCD x = blockIdx mod 8 take
tiles j, j + nwx, ... of the x-th eighth of the launch's tiles.  Checked here for the shapes the
engine accepts: every tile is scanned exactly once; a buffer's T tiles are scanned at the same step by
T consecutive waves of one workgroup, whose LDS slot index (step * WAVES / T + wave / T) is the same
for all T and below the 128 slots, and distinct across the workgroup's buffers.
"""
import pytest

WAVES = 8
XO_TILE = 16384
SLOTS = 128


def geometry(cus, ntiles, total_main):
    """engine.cpp scan_geometry for W = 32: 512-thread workgroups, two per CU from 256 MiB"""
    per_cu = 2 if total_main >= 256 << 20 else 1
    return min((ntiles + WAVES - 1) // WAVES, cus * per_cu)


def accepted(cus, ml, count):
    if ml <= 0 or ml % XO_TILE or ml // XO_TILE > 8:
        return None
    T = ml // XO_TILE
    if T & (T - 1):
        return None
    nt = T * count
    blocks = geometry(cus, nt, ml * count)
    nwx = blocks * WAVES // 8
    rounds = -(-(nt // 8) // nwx) if nwx else 0
    if blocks % 8 or nt % (8 * T) or rounds * (WAVES // T) > SLOTS:
        return None
    return T, nt, blocks


def walk(T, nt, blocks):
    """{tile: (block, wave, step, slot)} as the kernel assigns them"""
    nw = blocks * WAVES
    nwx = nw // 8
    seen = {}
    for b in range(blocks):
        x = b & 7
        xlo, xhi = x * nt // 8, (x + 1) * nt // 8
        for wv in range(WAVES):
            t0 = xlo + (b >> 3) * WAVES + wv
            ntw = (xhi - t0 + nwx - 1) // nwx if t0 < xhi else 0
            for n in range(ntw):
                t = t0 + n * nwx
                assert t not in seen
                seen[t] = (b, wv, n, n * (WAVES // T) + wv // T)
    return seen


@pytest.mark.parametrize("cus,ml,count", [(256, 65536, 20 * 1024), (256, 65536, 1024), (256, 16384, 4096),
                                          (256, 32768, 8192), (256, 131072, 2048), (256, 65536, 2048 * 3),
                                          (8, 65536, 96), (16, 32768, 200)])
def test_walk_covers_and_groups_buffers(cus, ml, count):
    acc = accepted(cus, ml, count)
    if acc is None:
        pytest.skip("shape not taken by the XCD-window order")
    T, nt, blocks = acc
    seen = walk(T, nt, blocks)
    assert sorted(seen) == list(range(nt))
    slots_used = {}
    for buf in range(count):
        where = [seen[buf * T + k] for k in range(T)]
        assert len({w[0] for w in where}) == 1  # one workgroup
        assert len({w[2] for w in where}) == 1  # one step
        assert [w[1] for w in where] == list(range(where[0][1], where[0][1] + T))  # consecutive waves, tile order
        slot = {w[3] for w in where}
        assert len(slot) == 1 and next(iter(slot)) < SLOTS
        key = (where[0][0], next(iter(slot)))
        assert key not in slots_used  # a slot holds one buffer per launch
        slots_used[key] = buf


def test_c2_headline_shape_is_taken():
    # the driver's 20-batch launch of C2 buffers (20 x 1024 x 64 KiB) on 256 CUs
    acc = accepted(256, 65536, 20 * 1024)
    assert acc == (4, 81920, 512)
