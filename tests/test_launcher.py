"""The multi-GPU launcher's failure handling (sezkp_amd/launch.py), on CPU:
the first rank that reports an error stops the others (which would block in
a collective forever), a rank that dies silently is noticed, and the overall
timeout ends the job. No GPU needed: the workers are stand-ins."""
import multiprocessing as mp
import time

from conftest import PKG  # noqa: F401  (puts the package on sys.path)
from sezkp_amd.launch import _collect


def _ok(rank, q):
    q.put((rank, None, 10, 0.0, 0.0))


def _fail(rank, q):
    q.put((rank, "RuntimeError: boom", 0, 0.0, 0.0))


def _hang(rank, q):
    time.sleep(600)


def _die(rank, q):
    import os
    os._exit(3)


def _spawn(targets):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=t, args=(r, q), daemon=True) for r, t in enumerate(targets)]
    for p in ps:
        p.start()
    return ps, q


def test_all_ranks_ok():
    ps, q = _spawn([_ok, _ok])
    res, err = _collect(ps, q, 60)
    assert err is None and [r[0] for r in res] == [0, 1]


def test_first_error_stops_blocked_ranks():
    ps, q = _spawn([_hang, _fail, _hang])
    t0 = time.monotonic()
    res, err = _collect(ps, q, 120)
    assert err == "rank 1: RuntimeError: boom"
    assert time.monotonic() - t0 < 60
    assert not any(p.is_alive() for p in ps)


def test_silent_death_is_noticed():
    ps, q = _spawn([_hang, _die])
    res, err = _collect(ps, q, 120)
    assert err.startswith("rank 1 exited with code 3")
    assert not any(p.is_alive() for p in ps)


def test_timeout_ends_the_job():
    ps, q = _spawn([_ok, _hang])
    # long enough for the spawned rank to start and report under a loaded
    # test run (a spawn child imports the launcher's module)
    res, err = _collect(ps, q, 20)
    assert err.startswith("timeout after 20 s (1 of 2 ranks reported)")
    assert not any(p.is_alive() for p in ps)
