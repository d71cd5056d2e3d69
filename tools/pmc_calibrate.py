"""FETCH_SIZE calibration on gfx950: read 256 MiB once with 4-, 12- and 16-byte lane accesses
(dirt_debug_read_bytes) so that rocprofv3 FETCH_SIZE (KB) can be converted to bytes per access width.
Run under rocprofv3 --pmc FETCH_SIZE (tools/gpu_final.sh and tools/gpu_traffic.sh do); the buffer exceeds the 256 MiB
Infinity Cache together with the flush buffer, so the reads come from HBM."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dirt_amd import _lib  # noqa: E402


def main():
    lib = _lib.load()
    fn = lib.dirt_debug_read_bytes
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    nbytes = 256 << 20
    src = torch.rand(nbytes // 4, device="cuda")
    flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
    out = torch.zeros(4, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for width in (4, 12, 16):
        for _ in range(3):
            flush.fill_(1)  # evict the source from the Infinity Cache
            _lib.check(fn(width, src.data_ptr(), nbytes - nbytes % width, out.data_ptr(), stream))
    torch.cuda.synchronize()
    print("calibration reads done: 3 x {4, 12, 16}-byte widths of %d bytes" % nbytes)


if __name__ == "__main__":
    main()
