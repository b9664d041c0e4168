"""Event-stream framing CRCs (aws_crt_amd/eventstream.py).

The framing (prelude CRC32 over 8 bytes, message CRC32 over every byte before the trailer) is the
aws-c-event-stream wire format; that library is absent from the reference checkout (initialised at
source/Api.cpp:51), so the span layout is checked here against its definition and the CRC values
against the oracle.  Parity of the message CRC with a real event-stream encoder: unpinned.
"""
import random
import struct

import pytest

from aws_crt_amd.eventstream import MIN_MESSAGE_BYTES, frame_spans


def test_frame_spans_layout():
    offs, lens = frame_spans([0, 100, 300], [16, 200, 4096])
    assert offs == [0, 0, 100, 100, 300, 300]
    assert lens == [8, 12, 8, 196, 8, 4092]
    assert frame_spans([], []) == ([], [])


def test_frame_spans_rejects_short_and_mismatched():
    with pytest.raises(ValueError):
        frame_spans([0], [MIN_MESSAGE_BYTES - 1])
    with pytest.raises(ValueError):
        frame_spans([0, 1], [16])


def _messages(n, seed):
    """n well-formed messages (prelude, prelude CRC placeholder, random body, trailer placeholder)."""
    rng = random.Random(seed)
    blob, offs, lens = bytearray(), [], []
    for _ in range(n):
        total = rng.choice([16, 17, 31, 64, 255, 1000, rng.randint(16, 5000)])
        hdr = rng.randint(0, total - 16)
        offs.append(len(blob))
        lens.append(total)
        blob += struct.pack(">II", total, hdr) + bytes(rng.getrandbits(8) for _ in range(total - 8))
        blob += bytes(rng.randrange(16))  # gaps: every start alignment mod 16
    return bytes(blob), offs, lens


@pytest.mark.gpu
def test_frame_crcs_vs_oracle(engine):
    import numpy as np
    import torch

    from aws_crt_amd.eventstream import FrameBatch, frame_crcs
    from oracle import oracle

    blob, offs, lens = _messages(1500, 0xE5)
    d = torch.from_numpy(np.frombuffer(blob, dtype=np.uint8).copy()).cuda()
    out = frame_crcs(d, offs, lens)
    torch.cuda.synchronize()
    got = engine.as_unsigned(out)
    want = []
    for o, n in zip(offs, lens):
        pre = oracle.crc("crc32", blob[o: o + 8])
        msg = oracle.crc("crc32", blob[o: o + n - 4])
        assert msg == oracle.crc("crc32", blob[o + 8: o + n - 4], pre)  # the running form
        want += [pre, msg]
    assert got == want
    # the prepared batch replays on another stream with the same result
    s = torch.cuda.Stream()
    again = FrameBatch(d, offs, lens).run(stream=s)
    torch.cuda.synchronize()
    assert engine.as_unsigned(again) == want


def _slice8_model(poly, width, data, seed=0):
    """Python model of crc_lanes_kernel's arithmetic (byte steps to 8-byte alignment, slice-by-8 words,
    tail bytes) for an aligned start; checked against the oracle's bitwise tier."""
    mask = (1 << width) - 1
    t0 = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ (poly if c & 1 else 0)
        t0.append(c)
    tabs = [t0]
    for _ in range(7):
        tabs.append([(c >> 8) ^ t0[c & 0xFF] for c in tabs[-1]])
    s = ~seed & mask
    n8 = len(data) // 8 * 8
    for k in range(0, n8, 8):
        x = int.from_bytes(data[k:k + 8], "little") ^ s
        s = 0
        for j in range(8):
            s ^= tabs[7 - j][(x >> (8 * j)) & 0xFF]
    for byte in data[n8:]:
        s = (s >> 8) ^ t0[(s ^ byte) & 0xFF]
    return ~s & mask


@pytest.mark.parametrize("name,poly,width", [("crc32", 0xEDB88320, 32), ("crc32c", 0x82F63B78, 32),
                                             ("crc64nvme", 0x9A6C9329AC4BC9B5, 64)])
def test_lane_slice8_model(name, poly, width):
    from oracle import oracle

    rng = random.Random(width + poly % 97)
    for n in [0, 1, 7, 8, 9, 15, 16, 17, 100, 257]:
        data = bytes(rng.getrandbits(8) for _ in range(n))
        seed = rng.getrandbits(width)
        assert _slice8_model(poly, width, data, seed) == oracle.crc(name, data, seed, tier="bitwise")


@pytest.mark.gpu
def test_check_frames_device(engine):
    """aws_crt_amd_eventstream_crcs: lengths read from the preludes on the device, stored CRCs
    compared; corrupted prelude CRCs, corrupted bodies and malformed / truncated lengths flagged."""
    import numpy as np
    import torch

    from aws_crt_amd.eventstream import STATUS_MALFORMED, STATUS_MESSAGE_OK, STATUS_PRELUDE_OK, check_frames
    from oracle import oracle

    blob, offs, lens = _messages(2000, 0xE6)
    blob = bytearray(blob)
    rng = random.Random(7)
    want = []
    for i, (o, n) in enumerate(zip(offs, lens)):
        pre = oracle.crc("crc32", bytes(blob[o: o + 8]))
        blob[o + 8: o + 12] = struct.pack(">I", pre)
        msg = oracle.crc("crc32", bytes(blob[o: o + n - 4]))
        blob[o + n - 4: o + n] = struct.pack(">I", msg)
        st = STATUS_PRELUDE_OK | STATUS_MESSAGE_OK
        kind = i % 7
        if kind == 1:  # stored prelude CRC wrong: the prelude CRC itself is still computed over bytes 0..7
            blob[o + 8] ^= 0x01
            msg = oracle.crc("crc32", bytes(blob[o: o + n - 4]))  # the stored prelude CRC is part of the body
            st = STATUS_MESSAGE_OK
            blob[o + n - 4: o + n] = struct.pack(">I", msg)
        elif kind == 2 and n > 16:  # body byte flipped after the message CRC was stored
            blob[o + rng.randrange(12, n - 4)] ^= 0x40
            msg = oracle.crc("crc32", bytes(blob[o: o + n - 4]))
            st = STATUS_PRELUDE_OK
        want.append((pre, msg, st))
    # malformed: a length below 16 and one past the end of the buffer
    extra = []
    for total in (15, len(blob) + 100):
        extra.append(len(blob))
        blob += struct.pack(">II", total, 0) + bytes(8)
        want.append((0, 0, STATUS_MALFORMED))
    # headers_length > total_length - 16 (aws-c-event-stream refuses it), even with both CRCs right
    extra.append(len(blob))
    bad = struct.pack(">II", 40, 25) + bytes(28)
    bad = bad[:8] + struct.pack(">I", oracle.crc("crc32", bad[:8])) + bad[12:36]
    bad += struct.pack(">I", oracle.crc("crc32", bad))
    blob += bad
    want.append((0, 0, STATUS_MALFORMED))
    extra.append(len(blob) - 4)  # fewer than 16 bytes left
    want.append((0, 0, STATUS_MALFORMED))
    d = torch.from_numpy(np.frombuffer(bytes(blob), dtype=np.uint8).copy()).cuda()
    o_t = torch.tensor(offs + extra, dtype=torch.int64, device="cuda")
    pre, msg, st = check_frames(d, o_t)
    torch.cuda.synchronize()
    got = list(zip(engine.as_unsigned(pre), engine.as_unsigned(msg), engine.as_unsigned(st)))
    assert got == want


def test_check_frames_argument_types():
    """check_frames refuses offsets that are not int64 (the kernel reads u64 offsets) before any
    device work; the byte limit is taken from the buffer's size in bytes, not its element count."""
    import torch

    from aws_crt_amd.eventstream import check_frames

    base = torch.zeros(64, dtype=torch.uint8)
    with pytest.raises(TypeError):
        check_frames(base, torch.zeros(2, dtype=torch.int32))
    with pytest.raises(TypeError):
        check_frames(base, torch.zeros(4, dtype=torch.int64)[::2])


def _packed(lens, seed, lead=0, corrupt=False):
    """messages packed back to back after `lead` bytes (a stream of frames, eventstream_flat_kernel's
    shape), with correct stored CRCs unless corrupted; returns blob, offsets, expected (pre, msg, st)"""
    import zlib

    rng = random.Random(seed)
    blob = bytearray(rng.randbytes(lead))
    offs, want = [], []
    for i, total in enumerate(lens):
        offs.append(len(blob))
        m = bytearray(struct.pack(">II", total, rng.randint(0, total - 16)) + bytes(4) + rng.randbytes(total - 12))
        pre = zlib.crc32(bytes(m[:8]))
        m[8:12] = struct.pack(">I", pre)
        msg = zlib.crc32(bytes(m[:total - 4]))
        m[total - 4:] = struct.pack(">I", msg)
        st = 3
        if corrupt and i % 5 == 1:  # stored prelude CRC wrong
            m[9] ^= 0x10
            msg = zlib.crc32(bytes(m[:total - 4]))
            m[total - 4:] = struct.pack(">I", msg)
            st = 2
        elif corrupt and i % 5 == 2:  # body flipped after the message CRC was stored
            m[rng.randrange(12, total - 4) if total > 16 else 12] ^= 0x04
            msg = zlib.crc32(bytes(m[:total - 4]))
            st = 1
        elif corrupt and i % 5 == 3:  # stored message CRC wrong
            m[total - 1] ^= 0x80
            st = 1
        blob += m
        want.append((pre, msg, st))
    blob += rng.randbytes(64)
    return blob, offs, want


def _run_frames(blob, offs, order=None):
    import numpy as np
    import torch

    from aws_crt_amd.eventstream import check_frames

    d = torch.from_numpy(np.frombuffer(bytes(blob), dtype=np.uint8).copy()).cuda()
    o_t = torch.tensor(offs if order is None else [offs[i] for i in order], dtype=torch.int64, device="cuda")
    pre, msg, st = check_frames(d, o_t)
    torch.cuda.synchronize()
    u = lambda t: [int(x) & 0xFFFFFFFF for x in t.cpu().tolist()]  # noqa: E731
    return list(zip(u(pre), u(msg), u(st)))


@pytest.mark.gpu
def test_check_frames_packed(engine):
    """packed streams (the balanced flat kernel): every start alignment of the first message, random
    16..1024-byte mixes with a partial last wave, the shortest messages (several ends per 64-byte block),
    messages spanning many chunks, corrupted CRCs, all against zlib"""
    rng = random.Random(0xF1A)
    for lead in (0, 1, 7, 8, 13, 31, 47, 63):
        lens = [rng.randint(16, 1024) for _ in range(64 * 6 + 5)]
        blob, offs, want = _packed(lens, lead, lead, corrupt=lead % 2 == 1)
        assert _run_frames(blob, offs) == want, lead
    for lens in ([16] * 640, [rng.randint(16, 40) for _ in range(640)], [16 + i % 9 for i in range(640)],
                 [rng.choice([16, 17, 4000, 20000, 70000]) for _ in range(200)]):
        blob, offs, want = _packed(lens, len(lens), 5, corrupt=True)
        assert _run_frames(blob, offs) == want


@pytest.mark.gpu
def test_check_frames_packed_fallbacks(engine):
    """waves the flat kernel must leave to the lane path: a malformed frame inside a packed wave, offsets
    out of order, a region beyond the flat kernel's bound; every other wave unaffected"""
    rng = random.Random(0xF1B)
    lens = [rng.randint(16, 1024) for _ in range(64 * 5)]
    blob, offs, want = _packed(lens, 11, 3)
    # headers_length > total - 16 in wave 1 (the frame stays packed): malformed
    o = offs[70]
    blob[o + 4:o + 8] = struct.pack(">I", lens[70] - 15)
    want[70] = (0, 0, 4)
    # wave 3's offsets swapped: not back to back
    order = list(range(len(offs)))
    order[200], order[201] = 201, 200
    got = _run_frames(blob, offs, order)
    assert got == [want[i] for i in order]
    # one wave spanning more than 256 KiB (a 300 KB message): lane path
    lens = [rng.randint(16, 1024) for _ in range(64 * 3)]
    lens[100] = 300000
    blob, offs, want = _packed(lens, 12, 9)
    assert _run_frames(blob, offs) == want
