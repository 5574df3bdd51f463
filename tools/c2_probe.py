"""Config 2 probe: the 2^20-point forward + inverse NTT through sezkp_gl_ntt,
timed with events over many round trips (as bench.py's `configs` does), so a
rocprofv3 kernel trace of this script shows whether the round trip is bound
by the kernels or by launch submission. Usage (GPU box, repo root):
  rocprofv3 --kernel-trace --stats -d gpurun_out/c2 -o run -- python3 tools/c2_probe.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "streaming-zero-knowledge-proofs_amd"))
import torch  # noqa: E402  (one HIP runtime: torch first)

if os.environ.get("SEZKP_PROBE_LIB"):  # A/B: another build of the library (same C ABI)
    import ctypes
    lib = ctypes.CDLL(os.environ["SEZKP_PROBE_LIB"])
    lib.sezkp_gl_ntt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_void_p]
    lib.sezkp_gl_ntt.restype = ctypes.c_int32
else:
    from sezkp_amd._lib import lib  # noqa: E402


def main():
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    n = 1 << log_n
    g = torch.Generator().manual_seed(2024)
    x = torch.randint(0, 2**62, (n,), generator=g, dtype=torch.int64).cuda()
    d = x.clone()
    s = torch.empty_like(x)
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        assert lib.sezkp_gl_ntt(d.data_ptr(), s.data_ptr(), log_n, 1, stream) == 0
        assert lib.sezkp_gl_ntt(d.data_ptr(), s.data_ptr(), log_n, -1, stream) == 0
    torch.cuda.synchronize()
    assert torch.equal(d, x)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(reps):
        lib.sezkp_gl_ntt(d.data_ptr(), s.data_ptr(), log_n, 1, stream)
        lib.sezkp_gl_ntt(d.data_ptr(), s.data_ptr(), log_n, -1, stream)
    t_sub = time.perf_counter() - t0
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"2^{log_n} fwd+inv: {ms * 1e3:.1f} us per round trip (events); host submission {t_sub / reps * 1e6:.1f} us "
          f"per round trip; round trip ok {bool(torch.equal(d, x))}")


if __name__ == "__main__":
    main()
