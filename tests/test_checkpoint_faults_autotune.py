"""Checkpoint/resume, fault injection (launcher teardown), bucket autotune — CPU tier."""
import os
import subprocess
import sys

import torch

import mivod.torch as hvd
from mivod.optim import FusedAdam, FusedSGD
from mivod.utils import checkpoint as ckpt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _net(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))


def _train(m, opt, steps=3):
    for _ in range(steps):
        opt.zero_grad()
        torch.nn.functional.mse_loss(m(torch.randn(5, 8)), torch.randn(5, 4)).backward()
        opt.step()


def test_checkpoint_roundtrip_fused_and_torch(tmp_path):
    hvd.init()
    for make in (lambda p: FusedAdam(p, lr=1e-2), lambda p: torch.optim.SGD(p, lr=0.1,
                                                                            momentum=0.9)):
        m = _net()
        opt = make(m.parameters())
        _train(m, opt)
        path = str(tmp_path / "checkpoint-3.safetensors")
        ckpt.save_checkpoint(path, m, opt, epoch=3, extra={"note": "x"})
        m2 = _net(seed=5)
        opt2 = make(m2.parameters())
        _train(m2, opt2, 1)
        start = ckpt.resume_from(str(tmp_path), m2, opt2)
        assert start == 4
        for a, b in zip(m.state_dict().values(), m2.state_dict().values()):
            torch.testing.assert_close(a, b)
        torch.manual_seed(11)
        _train(m, opt, 2)
        torch.manual_seed(11)
        _train(m2, opt2, 2)
        for a, b in zip(m.parameters(), m2.parameters()):
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
        os.remove(path)


def test_autotune_replans_and_logs(tmp_path, monkeypatch):
    log = tmp_path / "autotune.csv"
    monkeypatch.setenv("HOROVOD_AUTOTUNE", "1")
    monkeypatch.setenv("HOROVOD_AUTOTUNE_LOG", str(log))
    hvd.shutdown()
    hvd.init()
    try:
        m = torch.nn.Sequential(*[torch.nn.Linear(256, 256) for _ in range(6)])
        opt = hvd.DistributedOptimizer(FusedSGD(m.parameters(), lr=0.01))
        tuner = opt._mvd_autotune
        assert tuner is not None
        plans = set()
        total = len(tuner.seed) + tuner.bo_iters
        for _ in range(total * (tuner.warmup + tuner.trial + 1) + 2):
            opt.zero_grad()
            m(torch.randn(4, 256)).sum().backward()
            opt.step()
            plans.add(tuple(b.nbytes for b in opt._mvd_buckets))
        assert tuner.done and tuner.best in [c for c, _ in tuner.results]
        assert len(plans) > 1
        rows = log.read_text().strip().splitlines()
        assert rows[0].startswith("first_bucket_mb") and len(rows) == total + 1
        assert sum(",bayes," in r for r in rows) == tuner.bo_iters
    finally:
        hvd.shutdown()
        monkeypatch.delenv("HOROVOD_AUTOTUNE")
        hvd.init()


PROG = r'''
import os, sys
sys.path.insert(0, %r)
import torch, mivod.torch as hvd
from mivod.optim import FusedSGD
hvd.init()
m = torch.nn.Linear(4, 4)
opt = hvd.DistributedOptimizer(FusedSGD(m.parameters(), lr=0.1))
for step in range(10):
    opt.zero_grad()
    m(torch.randn(2, 4)).sum().backward()
    opt.step()
print("finished", hvd.rank())
''' % ROOT


def test_fault_injection_crash_tears_down_job(tmp_path):
    f = tmp_path / "prog.py"
    f.write_text(PROG)
    env = dict(os.environ, MIVOD_TRANSPORT="gloo", PYTHONPATH=ROOT, MIVOD_FAULT="1:3:crash")
    r = subprocess.run([sys.executable, "-m", "mivod.run", "-np", "2", sys.executable, str(f)],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 17, r.stdout + r.stderr
    assert "rank 1 exited with code 17" in r.stderr
    assert "finished 0" not in r.stdout


def test_bayesian_autotuner_finds_the_optimum_of_a_synthetic_step_time():
    """Seed design + GP/expected-improvement rounds on a smooth bowl in log2 space
    (minimum at first=2 MB, bucket=64 MB): the winner lands near the optimum and
    beats every seed candidate."""
    import math

    from mivod.parallel.autotune import BucketAutotuner

    def step_time(c):
        f, b = math.log2(c[0]), math.log2(c[1])
        return 0.1 + 0.01 * ((f - 1.0) ** 2 + 0.5 * (b - 6.0) ** 2)

    t = [0.0]
    tuner = BucketAutotuner(warmup=1, trial=3, bo_iters=8, clock=lambda: t[0])
    while not tuner.done:
        t[0] += step_time(tuner.current())
        tuner.on_step_end(lambda: None)
    best = tuner.best
    seed_best = min(step_time(c) for c in tuner.seed)
    assert step_time(best) < seed_best
    assert abs(math.log2(best[0]) - 1.0) <= 0.75 and abs(math.log2(best[1]) - 6.0) <= 1.0, best
