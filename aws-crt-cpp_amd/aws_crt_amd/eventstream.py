"""Event-stream framing CRCs as one ragged batch.

aws-c-event-stream (initialised by the reference at source/Api.cpp:51; the library itself is an
absent submodule) frames every message as

    prelude   total_length (u32 BE) | headers_length (u32 BE)       8 bytes
    prelude_crc  CRC32 of the prelude                                 4 bytes
    headers, payload
    message_crc  CRC32 of every byte before it (prelude .. payload)   4 bytes

so a stream of N messages is 2N independent CRC32 buffers: [m, m+8) and [m, m+total_length-4).
Both go to the engine as one list batch (aws_crt_amd_checksum_list); the descriptor arrays are built
once per message layout (`FrameBatch`) so repeated stream chunks with the same framing pay only the
launch.  Every byte is read by the gfx950 ragged scan -- no host CRC.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

from . import CRC32, _check, _stream_handle, lib

PRELUDE_BYTES = 8
TRAILER_BYTES = 4
MIN_MESSAGE_BYTES = PRELUDE_BYTES + 4 + TRAILER_BYTES  # empty headers and payload


def frame_spans(offsets: Sequence[int], total_lengths: Sequence[int]):
    """(ptr offsets, lengths) of the 2N CRC spans: entry 2i = prelude of message i, 2i+1 = its body."""
    if len(offsets) != len(total_lengths):
        raise ValueError("offsets and total_lengths differ in length")
    offs, lens = [], []
    for o, n in zip(offsets, total_lengths):
        if n < MIN_MESSAGE_BYTES:
            raise ValueError(f"event-stream message of {n} bytes is shorter than {MIN_MESSAGE_BYTES}")
        offs += [o, o]
        lens += [PRELUDE_BYTES, n - TRAILER_BYTES]
    return offs, lens


class FrameBatch:
    """Prepared descriptors for a fixed framing of a device buffer (`base`: torch uint8 tensor or raw
    address).  `run()` returns a 2N int32 tensor: [prelude_crc_0, message_crc_0, prelude_crc_1, ...]."""

    def __init__(self, base, offsets: Sequence[int], total_lengths: Sequence[int]):
        import torch

        addr = base.data_ptr() if hasattr(base, "data_ptr") else int(base)
        self.device = base.device if hasattr(base, "device") else torch.device("cuda")
        offs, lens = frame_spans(offsets, total_lengths)
        self.n = len(lens)
        self.payload_bytes = sum(lens)
        self._ptrs = (ctypes.c_void_p * self.n)(*[addr + o for o in offs])
        self._lens = (ctypes.c_size_t * self.n)(*lens)

    def run(self, out=None, stream=None):
        import torch

        if out is None:
            out = torch.empty(self.n, dtype=torch.int32, device=self.device)
        if self.n:
            _check(lib().aws_crt_amd_checksum_list(CRC32, self._ptrs, self._lens, self.n, None, out.data_ptr(),
                                                    _stream_handle(stream)))
        return out


def frame_crcs(base, offsets: Sequence[int], total_lengths: Sequence[int], stream=None):
    """Prelude and message CRC32s of N framed messages at `offsets` of device buffer `base`."""
    return FrameBatch(base, offsets, total_lengths).run(stream=stream)


STATUS_PRELUDE_OK, STATUS_MESSAGE_OK, STATUS_MALFORMED = 1, 2, 4


def check_frames(base, offsets, limit=None, stream=None):
    """Device-side framing check (aws_crt_amd_eventstream_crcs): `base` is a torch uint8 device tensor
    holding the messages, `offsets` a device int64 tensor of message starts.  Each message's length
    comes from its own prelude.  Returns (prelude_crc, message_crc, status) int32 device tensors;
    status bits: STATUS_PRELUDE_OK, STATUS_MESSAGE_OK, STATUS_MALFORMED (length outside the buffer,
    total_length < 16, or headers_length > total_length - 16)."""
    import torch

    L = lib()
    f = L.aws_crt_amd_eventstream_crcs
    vp = ctypes.c_void_p
    f.argtypes = [vp, ctypes.c_uint64, vp, ctypes.c_size_t, vp, vp, vp, vp]
    if offsets.dtype != torch.int64 or not offsets.is_contiguous():
        raise TypeError("offsets must be a contiguous int64 tensor (the kernel reads u64 offsets)")
    if not base.is_contiguous():
        raise TypeError("base must be contiguous")
    if offsets.device != base.device:
        raise ValueError("base and offsets must be on the same device")
    n = offsets.numel()
    pre, msg, st = (torch.empty(n, dtype=torch.int32, device=base.device) for _ in range(3))
    nbytes = base.numel() * base.element_size()
    lim = nbytes if limit is None else min(int(limit), nbytes)
    _check(f(base.data_ptr(), lim, offsets.data_ptr(), n, pre.data_ptr(), msg.data_ptr(), st.data_ptr(),
             _stream_handle(stream)))
    return pre, msg, st
