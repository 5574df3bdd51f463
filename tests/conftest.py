"""Shared test setup: paths, the `gpu` marker, oracle/product handles.

CPU tests (-m "not gpu") exercise the oracle against the reference fixtures,
the host codec/ABI of the product, and the Python-vs-C oracle cross-check.
GPU tests (-m gpu) are the parity tests proper: HIP path vs oracle through the
C ABI.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "streaming-zero-knowledge-proofs_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def free_port() -> int:
    """A TCP port for a multi-process test's rendezvous, drawn outside Linux's
    ephemeral range (32768-60999): a port found by binding port 0 comes from
    that range and can go to another connection (an earlier test's gloo pairs)
    before the store listens on it (EADDRINUSE, seen once on the GPU box)."""
    import random
    import socket
    rng = random.SystemRandom()
    for _ in range(500):
        p = rng.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
        except OSError:
            continue
        finally:
            s.close()
        return p
    raise RuntimeError("no free TCP port in 20000-32000")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def insert_zero_step_blocks(blocks, at):
    """A BlockSoA with zero-step blocks (step_hi = step_lo - 1, no steps)
    inserted before the block indices in `at` (n_blocks = after the last),
    copying a neighbour's windows and offsets. The reference gives them 0 rows
    and skips them (columns.rs:254-257,281-284; RowIter openings.rs:209-238),
    so with the same manifest root the proof is the one of `blocks`."""
    import numpy as np
    import sezkp_amd
    nb, tau = blocks.n_blocks, blocks.tau
    src, lo = [], []
    for i in range(nb + 1):
        for _ in range(at.count(i)):
            src.append(-1 - min(i, nb - 1))  # a zero-step copy of block min(i, nb - 1)
            lo.append(int(blocks.step_hi[i - 1]) + 1 if i else int(blocks.step_lo[0]))
        if i < nb:
            src.append(i)
            lo.append(None)
    arr = {}
    for f in ("version", "block_id", "step_lo", "step_hi", "ctrl_in", "ctrl_out", "in_head_in", "in_head_out"):
        a = getattr(blocks, f)
        arr[f] = np.array([a[j if j >= 0 else -1 - j] for j in src], dtype=a.dtype)
    for k, j in enumerate(src):
        if j < 0:
            arr["block_id"][k] = 1000 + k
            arr["step_lo"][k] = np.uint64(lo[k])
            arr["step_hi"][k] = np.uint64(lo[k]) - np.uint64(1)
    for f in ("win_left", "win_right", "off_in", "off_out"):
        a = getattr(blocks, f).reshape(nb, tau)
        arr[f] = np.concatenate([a[j if j >= 0 else -1 - j][None] for j in src]).reshape(-1)
    ss = [0]
    for j in src:
        ss.append(ss[-1] + (int(blocks.step_start[j + 1] - blocks.step_start[j]) if j >= 0 else 0))
    arr["step_start"] = np.array(ss, np.uint64)
    for f in ("input_mv", "mv", "has_write", "wsym"):
        arr[f] = getattr(blocks, f)
    return sezkp_amd.BlockSoA(tau, **arr)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def oracle():
    import oracle_ctypes
    oracle_ctypes.build()
    return oracle_ctypes


@pytest.fixture(scope="session")
def product():
    import sezkp_amd
    return sezkp_amd


@pytest.fixture(scope="session")
def gpu_ok():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    return torch
