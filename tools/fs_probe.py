#!/usr/bin/env python3
"""Device transcript kernel cost by shape: sezkp_fs_xof (phases 0-3 of
k_fs_point: the stream's chunk chaining from byte 0, per-challenge tails and
stack merges, XOF blocks) over stream lengths and challenge counts, 5 launches
each. Run under `rocprofv3 --kernel-trace`; the launches appear in this order."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "streaming-zero-knowledge-proofs_amd"))
import torch  # noqa: E402,F401
from sezkp_amd._lib import lib  # noqa: E402


def main():
    order = []
    for L in (64, 1024, 4096, 16384, 39000):
        for nch in (1, 8, 16):
            stream = bytes((i * 7 + 3) & 255 for i in range(L))
            pos = (C.c_uint32 * nch)(*[max(0, L - 64 * j) for j in range(nch)])
            sl = (C.c_uint32 * nch)(*([20] * nch))
            ol = (C.c_uint32 * nch)(*([64] * nch))
            sfx = bytes(20 * nch)
            out = C.create_string_buffer(64 * nch)
            for _ in range(5):
                assert lib.sezkp_fs_xof(stream, L, pos, sfx, sl, ol, nch, out, None) == 0
                order.append((L, nch))
    print(json.dumps(order))


if __name__ == "__main__":
    main()
