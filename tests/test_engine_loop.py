"""The native negotiation loop (csrc/engine/loop.cc, ``_mvcore.EngineLoop``):
cycle/wake-up behaviour, local fusion, issue-order position, shutdown — and the
Python engine running on it."""
import threading
import time

import pytest
import torch

from mivod import _mvcore

F32 = "torch.float32"


def _req(name, n=4, dtype=F32, op=0):
    return (name, 0, dtype, [n], -1, op, -1, 4 * n)


def _loop(cycle=0.0):
    c = _mvcore.ControllerConfig()
    c.rank, c.size = 0, 1
    ctl = _mvcore.Controller(c)
    return ctl, _mvcore.EngineLoop(ctl, 1, cycle)


def test_loop_fuses_and_reports_position():
    ctl, loop = _loop()
    loop.set_position(7)
    loop.submit([_req("a"), _req("b"), _req("c", dtype="torch.float16")])
    r = loop.wait(5.0)
    assert r is not None
    responses, all_shutdown, exec_at, err = r
    assert err == "" and not all_shutdown and exec_at == 7
    assert [names for _, names, _ in responses] == [["a", "b"], ["c"]]
    assert loop.requests == 3 and loop.cycles >= 1
    loop.request_shutdown()
    r = loop.wait(5.0)
    assert r is not None and r[1] is True        # the final all-shutdown cycle
    assert loop.wait(0.1) is None and loop.finished
    loop.join()
    ctl.close()


def test_loop_wakes_on_submit_without_waiting_for_the_cycle():
    ctl, loop = _loop(cycle=0.0)
    time.sleep(0.05)
    t0 = time.perf_counter()
    loop.submit([_req("x")])
    r = loop.wait(5.0)
    dt = time.perf_counter() - t0
    assert r is not None and r[0][0][1] == ["x"]
    assert dt < 0.5, dt
    loop.request_shutdown()
    loop.join()


def test_loop_waits_release_the_gil():
    """A Python thread keeps running while the executor blocks in wait()."""
    ctl, loop = _loop()
    ticks = []
    stop = threading.Event()

    def spin():
        while not stop.is_set():
            ticks.append(1)
            time.sleep(0.001)

    th = threading.Thread(target=spin)
    th.start()
    assert loop.wait(0.3) is None
    stop.set()
    th.join()
    assert len(ticks) > 20
    loop.request_shutdown()
    loop.join()


def test_submit_after_shutdown_raises():
    ctl, loop = _loop()
    loop.request_shutdown()
    loop.join()
    with pytest.raises(RuntimeError):
        loop.submit([_req("late")])


def test_engine_runs_named_ops_on_the_native_loop():
    import mivod.torch as hvd
    hvd.init()
    try:
        from mivod.common import basics
        eng = basics.state().engine
        assert eng.native and eng.loop is not None
        hs = [hvd.allreduce_async(torch.full((5,), float(i)), name=f"nl.{i}") for i in range(6)]
        outs = [hvd.synchronize(h) for h in hs]
        for i, o in enumerate(outs):
            assert torch.equal(o, torch.full((5,), float(i)))
        assert eng.loop.requests >= 6
    finally:
        hvd.shutdown()
