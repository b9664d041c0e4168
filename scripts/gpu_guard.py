"""Debug (-DAMDCRC_GUARD builds): run streaming-scan shapes, check parity and the guard record."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "aws-crt-cpp_amd")]
import torch  # noqa: E402
import aws_crt_amd as eng  # noqa: E402
from oracle import oracle  # noqa: E402

eng.init()
L = eng.lib()
g = (ctypes.c_ulonglong * 4)()
for (n, blen) in [(1, 4096), (5, 4096), (1, 1 << 20), (1024, 65536), (16, 1 << 20), (4096, 8192)]:
    d = torch.randint(0, 256, (n * blen,), dtype=torch.uint8, device="cuda")
    out = eng.checksum_strided(eng.CRC32C, d, blen, blen, n)
    torch.cuda.synchronize()
    rc = L.amdcrc_debug_guard(g)
    h = d.cpu().numpy()
    want = [oracle.crc("crc32c", h[i * blen:(i + 1) * blen]) for i in range(n)]
    print(n, blen, "guard rc", rc, [hex(x) for x in g], "parity", eng.as_unsigned(out) == want, flush=True)
