"""CPU-tier tests of round-2 plumbing:

* the cross-rank issue-order protocol (mivod/parallel/order.py) under random
  thread timing, against a simulated coordinator — every simulated rank must
  issue the identical collective sequence;
* bench.py's self-launch (``--gpus N`` without a launcher environment);
* fault kinds ``hang`` and ``raise``: every rank exits non-zero, within the
  stall-shutdown time, instead of the job hanging.
"""
import os
import random
import subprocess
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ------------------------------------------------------------------ order
class _Coordinator:
    """Cycle barrier for N simulated ranks: gathers (names, position), answers
    with the names every rank has submitted (first-submission order) and
    exec_at = max position — the contract of csrc/engine/controller.cc."""

    def __init__(self, n):
        self.n = n
        self.lock = threading.Condition()
        self.round = 0
        self.inbox = {}
        self.table = {}          # name -> set(ranks)
        self.order = []
        self.out = None

    def negotiate(self, rank, names, position):
        with self.lock:
            my_round = self.round
            self.inbox[rank] = (names, position)
            if len(self.inbox) == self.n:
                for r in range(self.n):
                    for nm in self.inbox[r][0]:
                        if nm not in self.table:
                            self.table[nm] = set()
                            self.order.append(nm)
                        self.table[nm].add(r)
                ready = [nm for nm in self.order if len(self.table[nm]) == self.n]
                for nm in ready:
                    del self.table[nm]
                    self.order.remove(nm)
                self.out = (ready, max(p for _, p in self.inbox.values()))
                self.inbox = {}
                self.round += 1
                self.lock.notify_all()
            else:
                while self.round == my_round:
                    self.lock.wait()
            return self.out


def _sim_rank(rank, program, coord, logs, seed, stop):
    from mivod.parallel.order import IssueOrder
    rng = random.Random(seed)
    order = IssueOrder()
    order.reset(enabled=True)
    log = logs[rank]
    pending, plock = [], threading.Lock()
    done = {}

    def engine():
        while not stop.is_set():
            time.sleep(rng.random() * 0.002)
            with plock:
                batch, pending[:] = list(pending), []
            pos = order.position()
            ready, exec_at = coord.negotiate(rank, batch, pos)
            fns = []
            for nm in ready:
                def fn(nm=nm):
                    with order.issue(negotiated=True):
                        log.append(("n", nm))
                    done[nm].set()
                fns.append(fn)
            if ready:
                order.responded(exec_at, len(ready), fns)

    th = threading.Thread(target=engine, daemon=True)
    th.start()
    for kind, arg, sync in program:
        time.sleep(rng.random() * 0.003)
        if kind == "d":
            with order.issue():
                log.append(("d", arg))
        else:
            done[arg] = threading.Event()
            order.submitted(1)
            with plock:
                pending.append(arg)
            if sync:
                assert done[arg].wait(20), f"rank {rank}: named op {arg} never ran"
    for nm, ev in done.items():
        assert ev.wait(20), f"rank {rank}: named op {nm} never ran"
    return th


@pytest.mark.parametrize("trial", range(6))
def test_issue_order_protocol_agrees_across_ranks(trial):
    rng = random.Random(1000 + trial)
    program = []
    k = 0
    for i in range(40):
        if rng.random() < 0.3:
            program.append(("n", f"op{k}", rng.random() < 0.5))
            k += 1
        else:
            program.append(("d", i, False))
    n = 3
    coord = _Coordinator(n)
    logs = [[] for _ in range(n)]
    stop = threading.Event()
    errs = []

    def run(r):
        try:
            _sim_rank(r, program, coord, logs, seed=trial * 10 + r, stop=stop)
        except BaseException as e:  # pragma: no cover - reported below
            errs.append(e)

    ths = [threading.Thread(target=run, args=(r,)) for r in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(60)
    # let the engines' last cycles finish (they keep cycling until stopped)
    stop.set()
    assert not errs, errs
    assert all(len(lg) == len(program) for lg in logs), [len(lg) for lg in logs]
    assert logs[0] == logs[1] == logs[2]


# --------------------------------------------------------- bench launcher
def test_bench_self_launch_needs_enough_gpus():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "HOROVOD_RANK", "MIVOD_BENCH_SHARE_GPUS")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stdout + r.stderr
    assert "only 0 GPU(s) are visible" in r.stderr


def test_bench_self_launch_spawns_ranks(monkeypatch):
    import importlib.util

    import torch

    import mivod.run.launcher as L
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    seen = {}

    def fake_launch(slots, cmd, env, tag_output=None, **kw):
        seen.update(slots=slots, cmd=cmd, env=env, tag=tag_output)
        return 0

    monkeypatch.setattr(L, "launch", fake_launch)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert bench.self_launch(["--gpus", "8", "--steps", "3"], 8) == 0
    assert [s.rank for s in seen["slots"]] == list(range(8))
    assert [s.local_rank for s in seen["slots"]] == list(range(8))
    assert seen["cmd"][1].endswith("bench.py") and seen["cmd"][2:] == ["--gpus", "8", "--steps",
                                                                       "3"]
    assert seen["tag"] is False and "MIVOD_TRANSPORT" not in seen["env"]
    # rehearsal on fewer GPUs: shared GPUs over the gloo-gpu wire
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setenv("MIVOD_BENCH_SHARE_GPUS", "1")
    monkeypatch.delenv("MIVOD_TRANSPORT", raising=False)
    assert bench.self_launch(["--gpus", "2"], 2) == 0
    assert seen["env"]["MIVOD_TRANSPORT"] == "gloo-gpu" and len(seen["slots"]) == 2


# ------------------------------------------------------------------ faults
@pytest.mark.parametrize("kind,step", [("hang", 3), ("raise", 3)])
def test_fault_kinds_end_the_job(kind, step):
    env = dict(os.environ, MIVOD_TRANSPORT="gloo", PYTHONPATH=ROOT,
               MIVOD_FAULT=f"1:{step}:{kind}", HOROVOD_STALL_SHUTDOWN_TIME_SECONDS="6",
               OMP_NUM_THREADS="1")
    t0 = time.time()
    r = subprocess.run([sys.executable, "-m", "mivod.run", "-np", "2", sys.executable,
                        os.path.join(ROOT, "tests", "mp_workers.py"), "fault_run"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    took = time.time() - t0
    assert r.returncode != 0, r.stdout + r.stderr
    assert "OK 0" not in r.stdout and "OK 1" not in r.stdout
    assert took < 60, took
    if kind == "hang":
        assert "timed out" in r.stderr or "stall" in r.stderr.lower(), r.stderr[-3000:]
    else:
        assert "injected fault" in r.stderr


def test_rccl_cta_autotune_picks_fastest_and_closes_the_rest(tmp_path):
    """tune_rccl_ctas: one communicator per candidate, the (rank-MAX) fastest kept,
    every other closed, one CSV row per candidate."""
    from mivod.parallel.autotune import tune_rccl_ctas

    class FakeComm:
        def __init__(self, c):
            self.c, self.closed = c, False

        def close(self):
            self.closed = True

    times = {0: 3.0, 4: 2.5, 8: 1.0, 16: 1.5, 32: 1.0}
    made = []

    def make(c):
        made.append(FakeComm(c))
        return made[-1]

    log = tmp_path / "at.csv"
    best, c, res = tune_rccl_ctas(make, lambda comm: times[comm.c], log_path=str(log))
    assert c == 8 and best.c == 8 and not best.closed      # first of the tied minimum
    assert [m.closed for m in made] == [True, True, False, True, True]
    assert res == [(0, 3.0), (4, 2.5), (8, 1.0), (16, 1.5), (32, 1.0)]
    rows = log.read_text().splitlines()
    assert rows[0] == "rccl_ctas,allreduce_s" and len(rows) == 6
