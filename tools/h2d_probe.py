"""Host -> device copy bandwidth from page-locked memory, the transfer the
staged uploads make (67 MB per T = 2^21 proof): one copy at a time, and 2 / 3
copies on concurrent streams (the contexts in flight each stage on their own
copy stream). Run under HSA_ENABLE_SDMA=0 for the blit-kernel path.
  python3 tools/h2d_probe.py [MB] [reps]"""
import os
import sys
import time

import torch


def main():
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 67
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    n = mb << 20
    hs = [torch.empty(n, dtype=torch.uint8).pin_memory() for _ in range(3)]
    ds = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(3)]
    ss = [torch.cuda.Stream() for _ in range(3)]
    for h in hs:
        h.fill_(7)
    res = {"MB": mb, "sdma": os.environ.get("HSA_ENABLE_SDMA", "default")}
    for k in (1, 2, 3):
        for _ in range(2):
            for i in range(k):
                with torch.cuda.stream(ss[i]):
                    ds[i].copy_(hs[i], non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            for i in range(k):
                with torch.cuda.stream(ss[i]):
                    ds[i].copy_(hs[i], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[f"streams{k}_GBs"] = round(k * reps * n / dt / 1e9, 2)
    print(res)


if __name__ == "__main__":
    main()
