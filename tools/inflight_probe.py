"""Throughput of independent proofs in flight on one GPU.
--mode threads: one Python thread per context calling prove_view (ctypes
releases the GIL); --mode async: the contexts' native workers
(sezkp_ctx_prove_async / sezkp_ctx_wait), waited round-robin.
--distinct: each context proves its own trace (seeds 42, 43, ...).
Usage: python tools/inflight_probe.py [--log-t 21] [--proofs 48] [--max 4]"""
import argparse
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "streaming-zero-knowledge-proofs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-t", type=int, default=21)
    ap.add_argument("--proofs", type=int, default=48)
    ap.add_argument("--max", type=int, default=4)
    ap.add_argument("--modes", default="threads,async")
    ap.add_argument("--distinct", action="store_true")
    a = ap.parse_args()
    import torch
    from sezkp_amd import ProverContext, reference_blocks
    T = 1 << a.log_t
    ctxs, roots, refs = [], [], []
    for i in range(a.max):
        bl = reference_blocks(T, 512, 8, 42 + i if a.distinct else 42)
        c = ProverContext(0)
        c.upload(bl)
        r = bl.manifest_root()
        c.prove(r)
        ctxs.append(c)
        roots.append(r)
        refs.append(bytes(c.prove_view(r)))

    def run_threads(k, per):
        ok = [None] * k

        def run(i):
            for _ in range(per):
                v = ctxs[i].prove_view(roots[i])
            ok[i] = bytes(v) == refs[i]
        th = [threading.Thread(target=run, args=(i,)) for i in range(k)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        return all(ok)

    def run_async(k, per):
        total, ok = per * k, True
        for i in range(k):
            ctxs[i].prove_async(roots[i])
        sub, done = k, 0
        while done < total:
            i = done % k
            ok = ok and bytes(ctxs[i].wait_view()) == refs[i]
            done += 1
            if sub < total:
                ctxs[i].prove_async(roots[i])
                sub += 1
        return ok

    for mode in a.modes.split(","):
        fn = run_threads if mode == "threads" else run_async
        for k in list(range(1, a.max + 1)) + [1]:
            per = a.proofs // k
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ok = fn(k, per)
            dt = time.perf_counter() - t0
            print(f"{mode} distinct={a.distinct} inflight={k} proofs={per * k} ms/proof={dt / (per * k) * 1e3:.3f} "
                  f"G elem/s={8 * T * per * k / dt / 1e9:.3f} same_bytes={ok}", flush=True)


if __name__ == "__main__":
    main()
