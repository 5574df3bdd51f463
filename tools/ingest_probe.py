#!/usr/bin/env python3
"""Per-rank time of the sliced JSONL ingest (sezkp_amd.ingest) without a GPU:
P gloo ranks on this host read one blocks.jsonl of T = 2^log_t rows (written
once to /tmp), each decoding its metadata share and its own row slice, as the
sharded launcher does before upload. Usage: tools/ingest_probe.py [log_t] [P]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "streaming-zero-knowledge-proofs_amd"))


def worker(rank, world, port, path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("SEZKP_HOST_THREADS", str(max(1, (os.cpu_count() or 1) // world)))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sezkp_amd.ingest import TorchComm, sliced_ingest
    dist.barrier()
    tw = time.perf_counter()
    if os.environ.get("PROBE_WARM"):
        box = [None] * world
        dist.all_gather_object(box, bytes(int(os.environ["PROBE_WARM"])))
    tw = time.perf_counter() - tw
    if os.environ.get("PROBE_TENSOR"):
        import torch
        n = int(os.environ["PROBE_TENSOR"])
        tl = []
        for _ in range(3):
            t1 = time.perf_counter()
            outs = [torch.empty(n, dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(outs, torch.zeros(n, dtype=torch.uint8))
            tl.append(round(time.perf_counter() - t1, 3))
        print(rank, "tensor allgather", tl, flush=True)
    runs = []
    for _ in range(2):  # the first call also pays gloo's first-collective setup
        t0 = time.perf_counter()
        r = sliced_ingest(path, rank, world, TorchComm(), None, None, frontier=True)
        runs.append((time.perf_counter() - t0, r["seconds"]))
        dist.barrier()
    q.put((rank, runs[0][0], runs[0][1], r["nrows"], runs[1][0], runs[1][1], tw))
    dist.destroy_process_group()


def main():
    log_t = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    path = f"/tmp/ingest_probe_{log_t}.jsonl"
    if not os.path.exists(path):
        import sezkp_amd
        jl = sezkp_amd.synthetic_blocks(1 << log_t, 512, 8, 42).to_jsonl()
        open(path, "wb").write(jl)
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, port, path, q)) for r in range(P)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join()
    print(json.dumps({"log_t": log_t, "P": P, "file_MB": os.path.getsize(path) / 1e6,
                      "load_s": [round(x[1], 3) for x in res],
                      "stages_rank0": {k: round(v, 3) for k, v in res[0][2].items()},
                      "decode_own_s": [round(x[2]["decode_own"], 3) for x in res],
                      "second_call_load_s": [round(x[4], 3) for x in res],
                      "second_call_stages_rank0": {k: round(v, 3) for k, v in res[0][5].items()},
                      "warm_allgather_s": [round(x[6], 3) for x in res],
                      "nrows": [x[3] for x in res]}))


if __name__ == "__main__":
    main()
