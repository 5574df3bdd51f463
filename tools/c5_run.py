#!/usr/bin/env python3
"""BASELINE config 5 at full size on the box: T = 2^22 (N = 2^25) blocks ->
blocks.jsonl -> `sezkp_amd.launch prove` single-GPU and sharded (P ranks, one
GPU, host collectives); both artifacts must be identical. Prints timings."""
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "streaming-zero-knowledge-proofs_amd")
sys.path.insert(0, PKG)


def manifest_cbor(root: bytes, n: int) -> bytes:
    def head(major, v):
        if v < 24:
            return bytes([major << 5 | v])
        for nb, code in ((1, 24), (2, 25), (4, 26), (8, 27)):
            if v < 1 << (8 * nb):
                return bytes([major << 5 | code]) + v.to_bytes(nb, "big")
    out = b"\xa2" + head(3, 4) + b"root" + head(4, 32) + b"".join(head(0, x) for x in root)
    return out + head(3, 8) + b"n_leaves" + head(0, n)


def main():
    log_t = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    out = os.path.join(ROOT, "gpurun_out", "c5")
    os.makedirs(out, exist_ok=True)
    import sezkp_amd
    t0 = time.time()
    blocks = sezkp_amd.synthetic_blocks(1 << log_t, 512, 8, 42)
    jl = blocks.to_jsonl()
    bpath, mpath = "/tmp/c5_blocks.jsonl", "/tmp/c5_manifest.cbor"
    open(bpath, "wb").write(jl)
    open(mpath, "wb").write(manifest_cbor(blocks.manifest_root(), int(blocks.block_id.size)))
    print(f"T=2^{log_t}: jsonl {len(jl)/1e6:.0f} MB written in {time.time()-t0:.1f} s", flush=True)
    del jl, blocks
    res = {}
    for name, extra in (("single", ["--gpus", "1"]), (f"sharded_host_x{P}", ["--gpus", str(P), "--comm", "host"]),
                        (f"sharded_host_x{P}_full_ingest", ["--gpus", str(P), "--comm", "host", "--full-ingest"])):
        o = f"/tmp/c5_{name}.cbor"
        t1 = time.time()
        pr = subprocess.Popen([sys.executable, "-m", "sezkp_amd.launch", "prove", "--blocks", bpath, "--manifest",
                               mpath, "--out", o, "--stream"] + extra, cwd=PKG, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True)
        while True:  # a heartbeat line every 30 s (a silent run looks hung)
            try:
                out, err = pr.communicate(timeout=30)
                break
            except subprocess.TimeoutExpired:
                print(f"{name}: running, {time.time() - t1:.0f} s", flush=True)
                if time.time() - t1 > 1500:
                    pr.kill()
        dt = time.time() - t1
        js = [x for x in out.splitlines() if x.startswith("{")]
        print(name, pr.returncode, js[-1] if js else out.strip()[-300:], "" if pr.returncode == 0 else err.strip()[-500:],
              f"wall {dt:.1f} s", flush=True)
        res[name] = hashlib.sha256(open(o, "rb").read()).hexdigest() if pr.returncode == 0 else None
    print(json.dumps(res))
    print("identical" if len(set(res.values())) == 1 and None not in res.values() else "DIFFERENT")


if __name__ == "__main__":
    main()
