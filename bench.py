#!/usr/bin/env python3
"""Headline benchmark: STARK v1 prove throughput on MI355X.

Metric (BASELINE.json): "STARK prove field-elements/sec (NTT+FRI+Merkle),
2^24 domain". One step = one complete `prove_v1` (column commitments, AIR
composition, INTT + coset LDE + DEEP, layer-0 and all FRI layer trees, query
paths and column openings, bincode proof bytes back on the host) of a
T = 2^21-row, tau = 8 trace (N = 8T = 2^24 LDE points), with the trace image
already resident in HBM. value = N * steps * ranks / max-over-ranks time.

Multi-GPU (--gpus N, launched by torch.distributed.run): one process per GPU,
each proving its own copy of the workload (independent proofs, weak scaling,
no data-path collective); the barrier / max-time reduction runs over RCCL.

Extra objects on the JSON line:
  roofline     — dominant kernel (k_layer16: the BLAKE3 Merkle tree over the
                 2^24-point LDE, one launch per prove) timed live with HIP
                 events bracketing exactly that launch on the prover's
                 stream; achieved = SURVEY §8(d) algorithmic bytes per launch
                 (72 B per leaf) / mean launch time. The kernel is VALU-bound
                 (BLAKE3), so `valu` reports compressions/s against the
                 CDNA4 integer-VALU ceiling next to the HBM fraction.
  ntt_lde      — the HBM-bound LDE NTT (3 LDS passes) against SURVEY's
                 9 B per LDE point compulsory traffic and against its own
                 moved bytes.
  cpu_baseline — the C oracle (single-thread restatement of the reference's
                 compute path) timed on this host on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "streaming-zero-knowledge-proofs_amd"))

METRIC = "STARK prove field-elements/sec (NTT+FRI+Merkle), 2^24 domain, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# BLAKE3 compression = 7 rounds x 8 G x 12 VALU ops + finalisation ~ 690 ops;
# 256 CU x 64 lanes x 2.4 GHz = 39.3 T int32 ops/s -> 57 G compressions/s
# (tools/b3_ceiling.hip measures 57.4 G/s for 64-byte parent blocks).
VALU_B3_PEAK = 57.0e9


def alg_bytes(n: int, tau: int) -> dict:
    """SURVEY.md §8(d) compulsory traffic, per LDE element N = 8n:
    179 + 9*(3+7tau) B total; the column commitments account for
    72 B per column cell (8 B value + 64 B of tree nodes) = 9*(3+7tau) per LDE element."""
    N = 8 * n
    ncols = 3 + 7 * tau
    return {"total": (179 + 9 * ncols) * N, "col_commit": 72 * ncols * n}


def load_pmc(kernel: str):
    p = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p)).get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_baseline(T_sample: int, tau: int, T_mt: int):
    """The C oracle's compute-once prover on this host: the
    OpenMP build on the host's cores (`value`, the fair multi-core baseline)
    and the single-thread build, each on a bounded sample of the workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ctypes as O
    from sezkp_amd import reference_blocks
    O.build()
    blocks = reference_blocks(T_sample, 512, tau)
    root = blocks.manifest_root()
    t0 = time.perf_counter()
    O.prove_v1(blocks, root)
    dt = time.perf_counter() - t0
    N = 8 * T_sample
    # reference-faithful structure repeats the layer-0 LDE pass 1 + 2*30*k times
    t_pass = O.time_lde_pass(blocks, root)
    k = N.bit_length() - 1
    single = {"value": N / dt, "cores": 1,
              "sample": f"oracle compute-once prove_v1, 1 thread, T=2^{T_sample.bit_length()-1} (N=2^{k}), "
                        f"tau={tau}; {dt:.2f} s"}
    threads = min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1))
    used = O.use_mt(threads)
    bl = reference_blocks(T_mt, 512, tau)
    r = bl.manifest_root()
    t1 = time.perf_counter()
    O.prove_v1(bl, r)
    dt_mt = time.perf_counter() - t1
    Nm = 8 * T_mt
    return {"value": Nm / dt_mt, "unit": "field-elements/s", "cores": used, "kind": "port",
            "sample": f"oracle compute-once prove_v1 (C restatement, OpenMP, {used} threads), "
                      f"T=2^{T_mt.bit_length()-1} (N=2^{Nm.bit_length()-1}), tau={tau}; {dt_mt:.2f} s",
            "single_thread": single,
            "reference_faithful_est_elems_per_s": N / (dt + 60 * k * t_pass),
            "reference_faithful_note": f"1 thread, +{60*k} layer-0 LDE passes of {t_pass:.3f} s each "
                                       f"(prover.rs:312-398), as the reference runs"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--log-t", type=int, default=21, help="trace rows T = 2^log_t (N = 8T)")
    ap.add_argument("--tau", type=int, default=8)
    ap.add_argument("--b", type=int, default=512)
    ap.add_argument("--stagger-ms", type=float, default=-1.0,
                    help="start offset between the in-flight pipelines (-1 = one proof time / inflight)")
    ap.add_argument("--pace", type=float, default=0.0,
                    help="minimum gap between proof starts, in units of the stagger (single proof / inflight)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="independent proofs in flight per GPU (one resident context each, sezkp_ctx_prove_async)")
    ap.add_argument("--cpu-sample-log-t", type=int, default=18)
    ap.add_argument("--cpu-mt-log-t", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the BASELINE config 2 (2^20 NTT) and config 3 (T=2^18 prove) objects")
    ap.add_argument("--no-sharded", action="store_true",
                    help="N>1: skip the extra sharded (one proof over all GPUs) measurement")
    ap.add_argument("--sharded-steps", type=int, default=3)
    ap.add_argument("--sharded-timeout", type=float, default=240.0,
                    help="watchdog: print the main line and exit if the sharded measurement stalls")
    ap.add_argument("--dntt-log-n", type=int, default=26,
                    help="distributed four-step NTT sub-measurement size (BASELINE config 4: 2^26); 0 = skip")
    ap.add_argument("--dntt-steps", type=int, default=5)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)

    from sezkp_amd import ProverContext, reference_blocks
    T = 1 << args.log_t
    dev = local if world > 1 else 0
    # `inflight` resident contexts, each with its own trace: context 0 holds
    # exactly `sezkp-cli simulate`'s blocks (seed 42), the others the same
    # generator at seeds 43.. (independent proofs, nothing shared)
    K = max(1, args.inflight)
    ctxs, roots = [], []
    for i in range(K):
        bl = reference_blocks(T, args.b, args.tau, 42 + i)
        c = ProverContext(dev)
        c.upload(bl)  # trace image resident in HBM before timing
        ctxs.append(c)
        roots.append(bl.manifest_root())
        if i == 0:
            blocks, mroot = bl, roots[0]
        del bl
    ctx = ctxs[0]

    def barrier():
        if dist:
            dist.barrier()
        torch.cuda.synchronize()

    # stagger: context i starts i/K of a proof later, so the K pipelines run
    # different stages (VALU-bound trees beside memory/latency-bound NTT,
    # openings, compose) instead of the same stage at the same time
    ctx.prove_async(mroot)
    ctx.wait_view()
    t_s = time.perf_counter()
    ctx.prove_async(mroot)
    ctx.wait_view()
    stagger = (args.stagger_ms * 1e-3 if args.stagger_ms >= 0 else (time.perf_counter() - t_s) / K)

    # timed: steps x K proofs, K in flight: one persistent host thread per
    # context keeps its context busy (prove_async / wait, each proof on the
    # context's own worker thread; the ctypes calls release the GIL). The same
    # threads run the warmup proofs, so no first-call cost of a new thread
    # lands in the timed region.
    total = args.steps * K
    l0_conc, done_t, per_proof = [], [], []
    timeline = bool(os.environ.get("SEZKP_BENCH_TIMELINE"))
    import gc
    import threading
    lock = threading.Lock()
    left = [total]  # shared work queue: a context takes the next proof when it is free
    warm = threading.Barrier(K + 1)
    go = threading.Barrier(K + 1)

    def take():
        with lock:
            if left[0] == 0:
                return False
            left[0] -= 1
            return True

    # optional start pacing: a proof never starts within `pace` of the
    # previous start (keeps the contexts out of the same stage)
    pace = args.pace * stagger
    last_start = [0.0]

    def paced_start(i):
        with lock:
            wait = last_start[0] + pace - time.perf_counter()
            if wait > 0:
                time.sleep(wait)
            last_start[0] = time.perf_counter()
        ctxs[i].prove_async(roots[i])

    def pipeline(i):
        for _ in range(max(1, args.warmup)):
            ctxs[i].prove_async(roots[i])
            ctxs[i].wait_view()
            ctxs[i].stage_times_ms()
        warm.wait()
        go.wait()
        if i and stagger > 0:
            time.sleep(i * stagger)
        while take():
            paced_start(i)
            ctxs[i].wait_view()
            st_i = ctxs[i].stage_times_ms()
            l0_conc.append(st_i.get("layer0_tree", float("nan")))
            done_t.append(time.perf_counter())
            if timeline:
                per_proof.append((i, done_t[-1], st_i))

    workers = [threading.Thread(target=pipeline, args=(i,)) for i in range(K)]
    for w in workers:
        w.start()
    warm.wait()
    gc.collect()
    gc.disable()  # no collector pauses in the host threads while proofs are in flight
    barrier()
    c0 = time.process_time()
    t0 = time.perf_counter()
    go.wait()
    for w in workers:
        w.join()
    barrier()
    dt = time.perf_counter() - t0
    cpu_frac = (time.process_time() - c0) / dt  # host CPU seconds per wall second (all threads)
    gc.enable()
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    N = 8 * T
    value = N * total * world / dt
    # one proof at a time on context 0: latency, stage split and roofline
    # (kernel timings without a concurrent proof sharing the chip)
    stage_sum = {}
    barrier()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        proof = ctx.prove_view(mroot)
        for k, v in ctx.stage_times_ms().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
    barrier()
    dt1 = time.perf_counter() - t1
    proof_len = len(proof)
    stages = {k: v / args.steps for k, v in stage_sum.items()}
    # PCIe-inclusive (never `value`): blocks in host memory -> proof bytes,
    # i.e. re-upload (device allocation + trace image over PCIe) + prove
    barrier()
    t1 = time.perf_counter()
    ctx.upload(blocks)
    torch.cuda.synchronize()
    t_up = time.perf_counter() - t1
    ctx.prove(mroot)
    torch.cuda.synchronize()
    t_host = time.perf_counter() - t1
    # the same from a fresh context (stream, twiddle tables, workspace allocation)
    t1 = time.perf_counter()
    cold = ProverContext(dev)
    cold.upload(blocks)
    cold.prove(mroot)
    torch.cuda.synchronize()
    t_cold = time.perf_counter() - t1
    cold.close()
    del cold

    if rank == 0:
        ab = alg_bytes(T, args.tau)
        t_l0 = stages.get("layer0_tree", float("nan")) * 1e-3
        l0_bytes = 72 * N  # layer-0 Merkle = 8 B value + 64 B of nodes per leaf
        achieved = l0_bytes / t_l0 / 1e9
        roof = {"bound": "hbm", "kernel": "k_layer16", "achieved": achieved, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": load_pmc("k_layer16"),
                "alg_bytes_per_launch": l0_bytes, "mean_launch_ms": t_l0 * 1e3,
                "measured_on": "single-proof pass (HIP events around the launch on the prover stream)",
                "concurrent_mean_launch_ms": sum(l0_conc) / len(l0_conc),
                "valu": {"compressions_per_launch": 2 * N - N // 4096,
                         "achieved_per_s": (2 * N - N // 4096) / t_l0, "peak_per_s": VALU_B3_PEAK,
                         "frac": (2 * N - N // 4096) / t_l0 / VALU_B3_PEAK},
                "note": "layer-0 FRI Merkle tree over the LDE (2^24 leaves); BLAKE3 is VALU-bound on CDNA4, "
                        "so the HBM fraction is structurally low (SURVEY 8(d) caveat); traffic = PMC "
                        "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE per launch from profiles/pmc_summary.json"}
        t_lde = stages.get("lde_ntt", float("nan")) * 1e-3
        moved = 16 * N * 3 - 8 * (N - T)  # 3 passes read+write, the first reads only the n coefficients
        ntt = {"kernel": "k_ntt4<DIT> x3 (coset LDE 2^%d, four-step register passes)" % (N.bit_length() - 1),
               "alg_bytes": 9 * N, "achieved_alg_GBs": 9 * N / t_lde / 1e9,
               "moved_bytes": moved, "achieved_moved_GBs": moved / t_lde / 1e9,
               "frac_moved": moved / t_lde / 1e9 / HBM_PEAK_GBS, "ms": t_lde * 1e3}
        whole = {"alg_bytes_per_proof": ab["total"], "achieved_GBs": ab["total"] * total / dt / 1e9}
        whole["frac"] = whole["achieved_GBs"] / HBM_PEAK_GBS  # per GPU: rank 0 proved `total` in dt
        out = {
            "metric": METRIC, "value": value, "unit": "field-elements/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "proofs_per_step": K, "ms_per_proof": dt / total * 1e3,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": f"synthetic: the blocks `sezkp-cli simulate --t {T} --b {args.b} --tau {args.tau}` writes "
                    f"(reference generator + partition, bit-exact restatement)",
            "config": {"workload": f"stark-v1 prove, T=2^{args.log_t} rows (N=2^{args.log_t + 3} LDE domain), "
                                   f"b={args.b}, tau={args.tau}, trace resident in HBM",
                       "T": T, "N": N, "tau": args.tau, "b": args.b, "proof_bytes": proof_len,
                       "proofs_in_flight_per_gpu": K,
                       "parallelism": f"replicas x{world}, {K} independent proofs in flight per GPU"},
            "halves_ms_per_proof": halves(done_t, t0),
            **({"done_ms": [round((t - t0) * 1e3, 3) for t in sorted(done_t)], "host_cpu_per_wall": cpu_frac,
                "slowest": [{"ctx": i, "at_ms": round((t - t0) * 1e3, 2),
                             **{k: round(v, 3) for k, v in st.items()}}
                            for i, t, st in sorted(per_proof, key=lambda x: -x[2].get("host_wall", 0))[:4]]}
               if timeline else {}),
            "single_proof": {"value": N * args.steps / dt1, "unit": "field-elements/s",
                             "ms_per_proof": dt1 / args.steps * 1e3,
                             "note": "one proof at a time on one context (rank 0): the latency view; "
                                     "stages_ms and roofline come from this pass"},
            "roofline": roof, "ntt_lde": ntt, "whole_prove_hbm": whole, "stages_ms": stages,
            "pcie_inclusive": {"value": N / t_host, "unit": "field-elements/s", "ms": t_host * 1e3,
                               "upload_ms": t_up * 1e3, "fresh_context_ms": t_cold * 1e3,
                               "note": "rank 0, one proof from blocks in host memory: ctx.upload on a context that "
                                       "held a trace of this shape (workspace reused, step arrays over PCIe "
                                       "and transposed on the device) + prove; not `value`"},
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(1 << args.cpu_sample_log_t, args.tau, 1 << args.cpu_mt_log_t)
    for c in ctxs:
        c.close()
    del blocks, ctxs, ctx

    def guarded(key, fn):
        # extra measurements are reported beside the main line; a watchdog
        # keeps a stalled collective from costing it
        import threading

        def _bail():
            if rank == 0:
                out[key] = {"error": f"watchdog: no result within {args.sharded_timeout:.0f} s"}
                print(json.dumps(out), flush=True)
            os._exit(0)
        wd = threading.Timer(args.sharded_timeout, _bail)
        wd.daemon = True
        wd.start()
        try:
            res = fn()
        except Exception as e:  # reported, never fatal to the main line
            res = {"error": f"{type(e).__name__}: {e}"}
        wd.cancel()
        if rank == 0:
            out[key] = res

    if rank == 0 and not args.no_configs:
        guarded("configs", lambda: measure_configs(args, torch))
    if args.dntt_log_n:
        # BASELINE config 4 (at N = 8): 2^26-point four-step NTT over all ranks
        guarded("dist_ntt", lambda: measure_dist_ntt(args, world, rank, local, dist, torch))
    if world > 1 and not args.no_sharded:
        # ONE proof over all ranks (weak: 2^log_t rows per GPU)
        guarded("sharded", lambda: measure_sharded(args, world, rank, local, dist, torch))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def halves(done_t, t0):
    """ms per proof over the first and the second half of the timed proofs
    (a slow first half would mean the warmup is too short)."""
    ts = sorted(done_t)
    if len(ts) < 4:
        return None
    h = len(ts) // 2
    return [(ts[h - 1] - t0) / h * 1e3, (ts[-1] - ts[h - 1]) / (len(ts) - h) * 1e3]


def det_vec(n: int, seed: int):
    """crates/sezkp-ffts/benches/ntt.rs:21-34: LCG (A=1664525, C=1013904223,
    mod 2^32) started at A*seed + C, stepped before each use; value
    (a_i ^ i*0x9E3779B97F4A7C15) mod p. Vectorised with the affine powers
    f^(j+1)(x) = mul_j x + add_j (mod 2^32) per block of 4096."""
    import numpy as np
    P = 0xFFFFFFFF00000001
    A, Cc, M32 = 1664525, 1013904223, 0xFFFFFFFF
    blk = 1 << 12
    mul = np.empty(blk, dtype=np.uint64)
    add = np.empty(blk, dtype=np.uint64)
    m, c = 1, 0
    for j in range(blk):
        m, c = (A * m) & M32, (A * c + Cc) & M32
        mul[j], add[j] = m, c
    a = np.empty(n, dtype=np.uint64)
    x = (A * seed + Cc) & M32
    for lo in range(0, n, blk):
        hi = min(n, lo + blk)
        a[lo:hi] = (mul[: hi - lo] * np.uint64(x) + add[: hi - lo]) & np.uint64(M32)
        x = (int(mul[-1]) * x + int(add[-1])) & M32
    v = a ^ (np.arange(n, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
    return np.where(v >= np.uint64(P), v - np.uint64(P), v)


def measure_configs(args, torch):
    """BASELINE configs 2 and 3 on this GPU: the 2^20-point forward + inverse
    NTT of det_vec(2^20, 2024) through sezkp_gl_ntt (round trip checked), and
    the full T = 2^18 prove (one proof at a time and 3 in flight)."""
    from sezkp_amd import ProverContext, reference_blocks
    from sezkp_amd._lib import lib
    out = {}
    n = 1 << 20
    x = torch.from_numpy(det_vec(n, 2024).view("int64")).cuda()
    d, s = x.clone(), torch.empty_like(x)
    for _ in range(3):
        assert lib.sezkp_gl_ntt(d.data_ptr(), s.data_ptr(), 20, 1, None) == 0
        assert lib.sezkp_gl_ntt(d.data_ptr(), s.data_ptr(), 20, -1, None) == 0
    torch.cuda.synchronize()
    ok = bool(torch.equal(d, x))
    reps = 50
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        lib.sezkp_gl_ntt(d.data_ptr(), s.data_ptr(), 20, 1, None)
        lib.sezkp_gl_ntt(d.data_ptr(), s.data_ptr(), 20, -1, None)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    out["c2_ntt_2e20"] = {"workload": "2^20-point Goldilocks NTT, forward + inverse (natural order in and out), "
                                      "det_vec(2^20, 2024) input, sezkp_gl_ntt",
                          "ms_fwd_plus_inv": ms, "value": 2 * n / (ms * 1e-3), "unit": "field-elements/s",
                          "roundtrip_ok": ok and bool(torch.equal(d, x))}
    # config 3: T = 2^18 full prove
    T = 1 << 18
    ctxs, roots = [], []
    for i in range(3):
        bl = reference_blocks(T, args.b, args.tau, 42 + i)
        c = ProverContext(0)
        c.upload(bl)
        ctxs.append(c)
        roots.append(bl.manifest_root())
    for c, r in zip(ctxs, roots):
        c.prove_view(r)
    torch.cuda.synchronize()
    steps = 20
    t0 = time.perf_counter()
    for _ in range(steps):
        ctxs[0].prove_view(roots[0])
    t1 = (time.perf_counter() - t0) / steps
    import threading
    lock = threading.Lock()
    left = [3 * steps]

    def pipe(i):
        while True:
            with lock:
                if left[0] == 0:
                    return
                left[0] -= 1
            ctxs[i].prove_async(roots[i])
            ctxs[i].wait_view()
    t0 = time.perf_counter()
    ws = [threading.Thread(target=pipe, args=(i,)) for i in range(3)]
    for w in ws:
        w.start()
    for w in ws:
        w.join()
    t3 = (time.perf_counter() - t0) / (3 * steps)
    for c in ctxs:
        c.close()
    N = 8 * T
    out["c3_prove_2e18"] = {"workload": f"stark-v1 prove T=2^18 (N=2^21), b={args.b}, tau={args.tau}",
                            "single_proof_ms": t1 * 1e3, "value_single": N / t1,
                            "inflight3_ms_per_proof": t3 * 1e3, "value_inflight3": N / t3,
                            "unit": "field-elements/s"}
    return out


def measure_dist_ntt(args, world, rank, local, dist, torch):
    """sezkp_ctx_dist_ntt: n = 2^dntt_log_n points split over the ranks
    (strong scaling: fixed n), forward + inverse per step on the context
    stream; one RCCL all-to-all per transform. Round trip checked."""
    from sezkp_amd import ProverContext, ShardedProverContext
    ctx = ShardedProverContext(rank, world, device=local, comm="rccl") if world > 1 else ProverContext(0)
    log_n = args.dntt_log_n
    M = (1 << log_n) // world
    g = torch.Generator(device="cuda")
    g.manual_seed(1234 + rank)
    x = torch.randint(0, 0xFFFFFFFF00000001 >> 1, (M,), dtype=torch.int64, device="cuda", generator=g)
    d = x.clone()
    scratch = torch.empty_like(d)
    for _ in range(2):
        ctx.dist_ntt(d, scratch)
        ctx.dist_ntt(d, scratch, inverse=True)
    ok = bool(torch.equal(d, x))
    st = torch.cuda.ExternalStream(ctx.stream)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.dntt_steps):
        ctx.dist_ntt(d, scratch, sync=False)
        ctx.dist_ntt(d, scratch, inverse=True, sync=False)
    st.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        oks = [None] * world
        dist.all_gather_object(oks, ok)
        ok = all(oks)
    ctx.close()
    n = 1 << log_n
    per = dt / (2 * args.dntt_steps)
    alg = 16 * M / per / 1e9  # read + write each local element once, per GPU
    return {"workload": f"2^{log_n}-point Goldilocks NTT over {world} GPU(s), forward + inverse (four-step: "
                        f"local 2^{log_n - (world.bit_length() - 1)} NTT, twiddle, "
                        f"{'1 RCCL all-to-all' if world > 1 else 'no exchange'}, {world}-point DFTs)",
            "value": n / per, "unit": "field-elements/s", "ms_per_transform": per * 1e3, "steps": args.dntt_steps,
            "scaling": "strong", "roundtrip_ok": ok, "alg_GBs_per_gpu": alg, "frac_hbm_alg": alg / HBM_PEAK_GBS}


def measure_sharded(args, world, rank, local, dist, torch):
    from sezkp_amd import ShardedProverContext, reference_blocks
    T = (1 << args.log_t) * world
    blocks = reference_blocks(T, args.b, args.tau)
    mroot = blocks.manifest_root()
    ctx = ShardedProverContext(rank, world, device=local, comm="rccl")
    ctx.upload(blocks)
    del blocks
    ctx.prove(mroot)  # warmup
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stage_sum = {}
    for _ in range(args.sharded_steps):
        view = ctx.prove_view(mroot)
        for k, v in ctx.stage_times_ms().items():
            stage_sum[k] = stage_sum.get(k, 0.0) + v
    dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    digest = __import__("hashlib").sha256(view).hexdigest()
    plen = len(view)
    ds = [None] * world
    dist.all_gather_object(ds, digest)
    ctx.close()
    N = 8 * T
    return {"metric": METRIC, "value": N * args.sharded_steps / dt, "unit": "field-elements/s",
            "ms_per_step": dt / args.sharded_steps * 1e3, "steps": args.sharded_steps, "scaling": "weak",
            "config": {"workload": f"ONE stark-v1 proof over {world} GPUs, T=2^{T.bit_length() - 1} rows "
                                   f"(N=2^{N.bit_length() - 1}), b={args.b}, tau={args.tau}",
                       "parallelism": f"sharded x{world}: coset-split LDE, 1 RCCL all-to-all, allgathered "
                                      f"Merkle caps, byte-sum proof assembly"},
            "ranks_agree": len(set(ds)) == 1, "proof_bytes": plen,
            "stages_ms_rank0": {k: v / args.sharded_steps for k, v in stage_sum.items()}}


if __name__ == "__main__":
    main()
