"""CPU model of the lane scans' conflict-free slice-by-8 fold (crc_kernels.hip LaneW8, round 4): the
plain tables T_t[e] = e * x^(8(t+1)) in the 8-copy LDS image (entry e's 256-byte row holds table t at
32 t, copy c at 4 c) looked up with the per-lane byte rotation of crc32_stream_kernel's tables.

Checked: the image built as lane_w8_tables builds it; every lane's eight-lookup word step equals the
slice-by-8 step (so a lane scan equals zlib's CRC32 / the SSE4.2 CRC32C); the byte step reads T_0;
and in each of the eight lookup slots the 32 lanes of a ds_read_b32 half-wave meet 32 distinct banks
((address / 4) mod 32) for any data.
"""
import random
import zlib

import pytest

M32 = 0xFFFFFFFF
POLYS = {"crc32": 0xEDB88320, "crc32c": 0x82F63B78}


def table_entry(e, t, poly):
    """T_t[e]: the byte e advanced over t + 1 zero bytes (gf2_table_entry)"""
    c = e
    for _ in range(8 * (t + 1)):
        c = (c >> 1) ^ (poly if c & 1 else 0)
    return c


def image(poly):
    """dword index (e * 64 + t * 8 + c) -> T_t[e]"""
    T = [[table_entry(e, t, poly) for e in range(256)] for t in range(8)]
    img = [0] * (256 * 64)
    for e in range(256):
        for t in range(8):
            for c in range(8):
                img[e * 64 + t * 8 + c] = T[t][e]
    return img, T


def schedule(lane):
    """(byte offsets) cst8[k] and the byte q of the dword each slot reads: LaneW8::init"""
    j, c = (lane >> 3) & 3, lane & 7
    slots = []
    for k in range(4):
        q = (k + j) & 3
        slots.append(("lo", q, ((7 - q) << 5) | (c << 2)))
    for k in range(4):
        q = (k + j) & 3
        slots.append(("hi", q, ((3 - q) << 5) | (c << 2)))
    return slots


def word_step(img, lane, s, v):
    lo, hi = (v & M32) ^ s, v >> 32
    acc = 0
    for half, q, cst in schedule(lane):
        dw = lo if half == "lo" else hi
        addr = (((dw >> (8 * q)) & 0xFF) << 8) | cst
        acc ^= img[addr // 4]
    return acc


def byte_step(img, lane, s, b):
    return (s >> 8) ^ img[((((s ^ b) & 0xFF) << 8) | ((lane & 7) << 2)) // 4]


@pytest.mark.parametrize("name", sorted(POLYS))
def test_word_and_byte_steps_match_slice_by_8(name):
    poly = POLYS[name]
    img, T = image(poly)
    rnd = random.Random(7)
    for lane in range(64):
        for _ in range(8):
            s, v = rnd.getrandbits(32), rnd.getrandbits(64)
            x = v ^ s
            ref = 0
            for i in range(8):
                ref ^= T[7 - i][(x >> (8 * i)) & 0xFF]
            assert word_step(img, lane, s, v) == ref
            b = rnd.getrandbits(8)
            assert byte_step(img, lane, s, b) == (s >> 8) ^ T[0][(s ^ b) & 0xFF]


def lane_scan(img, lane, s, data):
    """lane_scan's word path on an 8-aligned buffer (head / tail bytes through the byte step)"""
    n8 = len(data) // 8
    for i in range(n8):
        s = word_step(img, lane, s, int.from_bytes(data[8 * i:8 * i + 8], "little"))
    for b in data[8 * n8:]:
        s = byte_step(img, lane, s, b)
    return s


def test_lane_scan_is_zlib_crc32():
    img, _ = image(POLYS["crc32"])
    rnd = random.Random(3)
    for lane in (0, 9, 31, 42, 63):
        for n in (0, 1, 7, 8, 15, 64, 100, 517):
            data = bytes(rnd.getrandbits(8) for _ in range(n))
            assert (~lane_scan(img, lane, M32, data)) & M32 == zlib.crc32(data)


def test_half_waves_meet_distinct_banks():
    rnd = random.Random(11)
    for _ in range(200):
        lo = [rnd.getrandbits(32) for _ in range(64)]
        hi = [rnd.getrandbits(32) for _ in range(64)]
        for k in range(8):
            for h in (0, 32):
                banks = set()
                for lane in range(h, h + 32):
                    half, q, cst = schedule(lane)[k]
                    dw = lo[lane] if half == "lo" else hi[lane]
                    addr = (((dw >> (8 * q)) & 0xFF) << 8) | cst
                    banks.add((addr // 4) % 32)
                assert len(banks) == 32
