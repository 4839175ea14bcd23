"""Launcher (mivodrun / horovodrun parity) — CPU tier."""
import os
import subprocess
import sys

import pytest

from mivod.run.launcher import (assign_slots, build_parser, exported_env, parse_hostfile,
                                parse_hosts, tuning_env)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_hosts_and_hostfile(tmp_path):
    assert parse_hosts("a:4,b:2,c") == [("a", 4), ("b", 2), ("c", 1)]
    hf = tmp_path / "hostfile"
    hf.write_text("# comment\nnode1 slots=4\nnode2:2\nnode3\n")
    assert parse_hostfile(str(hf)) == [("node1", 4), ("node2", 2), ("node3", 1)]


def test_assign_slots_topology():
    s = assign_slots([("a", 2), ("b", 2)], 4)
    assert [(x.host, x.rank, x.local_rank, x.local_size) for x in s] == [
        ("a", 0, 0, 2), ("a", 1, 1, 2), ("b", 2, 0, 2), ("b", 3, 1, 2)]
    assert [(x.cross_rank, x.cross_size) for x in s] == [(0, 2), (0, 2), (1, 2), (1, 2)]
    with pytest.raises(ValueError):
        assign_slots([("a", 1)], 2)


def test_mpirun_flags_tolerated_and_tuning_mapped():
    # the reference's mpirun line (README.md:57) with mpirun -> mivodrun
    argv = ("--allow-run-as-root -np 1 --hostfile /generated/hostfile -bind-to none -map-by slot "
            "-x NCCL_DEBUG=INFO -mca pml ob1 -mca btl ^openib --fusion-threshold-mb 32 "
            "--cycle-time-ms 2 --timeline-filename /tmp/tl.json --no-stall-check "
            "python keras_mnist.py --epochs 1").split()
    a = build_parser().parse_args(argv)
    assert a.np == 1 and a.hostfile == "/generated/hostfile"
    assert a.command == ["python", "keras_mnist.py", "--epochs", "1"]
    env = tuning_env(a)
    assert env["HOROVOD_FUSION_THRESHOLD"] == str(32 * 2 ** 20)
    assert env["HOROVOD_CYCLE_TIME"] == "2"
    assert env["HOROVOD_TIMELINE"] == "/tmp/tl.json"
    assert env["HOROVOD_STALL_CHECK_DISABLE"] == "1"
    assert exported_env(a.export) == {"NCCL_DEBUG": "INFO"}


SCRIPT = r'''
import os, sys
sys.path.insert(0, %r)
import torch
import mivod as hvd
hvd.init()
x = hvd.allreduce(torch.tensor([float(hvd.rank())]), op=hvd.Sum)
print("rank", hvd.rank(), "size", hvd.size(), "local", hvd.local_rank(), "sum", float(x),
      "nccl_debug", os.environ.get("NCCL_DEBUG"))
from mivod.common import basics
print("store", basics.state().store_kind, flush=True)
hvd.shutdown()
''' % ROOT


def test_launch_two_local_ranks(tmp_path):
    f = tmp_path / "prog.py"
    f.write_text(SCRIPT)
    env = dict(os.environ, MIVOD_TRANSPORT="gloo", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "mivod.run", "-np", "2", "-H", "localhost:2",
                        "-x", "NCCL_DEBUG=INFO", "python", str(f)], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "[0]<stdout>:rank 0 size 2 local 0 sum 1.0 nccl_debug INFO" in r.stdout, r.stdout
    assert "[1]<stdout>:rank 1 size 2 local 1 sum 1.0 nccl_debug INFO" in r.stdout, r.stdout
    # the gloo world, rings and engine bootstrapped through the launcher's native store
    assert "[0]<stdout>:store native" in r.stdout and "[1]<stdout>:store native" in r.stdout


def test_native_rendezvous_store():
    """csrc/engine/store.cc: blocking get, counters, wait/check, compare-set, delete,
    timeouts — and as a torch.distributed.Store for a 3-rank gloo world."""
    import threading
    import time

    from mivod.run.store import NativeStore, serve
    srv = serve("127.0.0.1", 0)
    try:
        a = NativeStore("127.0.0.1", srv.port, 5.0)
        b = NativeStore("127.0.0.1", srv.port, 5.0)
        got = []
        t = threading.Thread(target=lambda: got.append(b.get("k")))
        t.start()
        time.sleep(0.2)
        a.set("k", "v1")                   # wakes the blocked get (server-side wait, no polling)
        t.join(5)
        assert got == [b"v1"]
        assert a.add("n", 3) == 3 and b.add("n", 2) == 5
        assert a.check(["k", "n"]) and not a.check(["missing"])
        assert a.compare_set("k", b"v1", b"v2") == b"v2" and b.get("k") == b"v2"
        assert a.compare_set("k", b"zz", b"v3") == b"v2"
        assert a.num_keys() == 2 and a.delete_key("k") and not a.check(["k"])
        import datetime
        t0 = time.time()
        try:
            a.wait(["never"], datetime.timedelta(seconds=0.3))
            raise AssertionError("wait did not time out")
        except RuntimeError as e:
            assert "timed out" in str(e) and time.time() - t0 < 3
        script = ("import sys, torch, torch.distributed as dist; sys.path.insert(0, %r)\n"
                  "from mivod.run.store import NativeStore\n"
                  "r = int(sys.argv[1]); st = NativeStore('127.0.0.1', %d, 30.0)\n"
                  "dist.init_process_group('gloo', store=st, rank=r, world_size=3)\n"
                  "x = torch.tensor([r + 1.0]); dist.all_reduce(x); print('sum', x.item())\n"
                  "dist.destroy_process_group()\n") % (ROOT, srv.port)
        ps = [subprocess.Popen([sys.executable, "-c", script, str(r)], stdout=subprocess.PIPE,
                               stderr=subprocess.STDOUT, text=True) for r in range(3)]
        outs = [p.communicate(timeout=120)[0] for p in ps]
        assert all(p.returncode == 0 and "sum 6.0" in o for p, o in zip(ps, outs)), outs
        assert srv.requests > 10
    finally:
        srv.close()


def test_launch_failure_kills_all(tmp_path):
    f = tmp_path / "fail.py"
    f.write_text("import os, time, sys\n"
                 "r = int(os.environ['HOROVOD_RANK'])\n"
                 "time.sleep(0.5)\n"
                 "sys.exit(3) if r == 1 else time.sleep(120)\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bin", "horovodrun"), "-np", "2",
                        sys.executable, str(f)], cwd=ROOT, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 3, r.stdout + r.stderr
    assert "rank 1 exited with code 3" in r.stderr


def test_bucket_plan_orders_by_readiness():
    """Buckets launch in the order their last gradient arrives; the mixed
    bf16-conv / fp32-BN ResNet-50 layout must not let the BN bucket (which
    holds the stem BN) block the conv buckets."""
    import mivod.torch as hvd
    from mivod.models.resnet import resnet50, to_mixed_bf16
    from mivod.optim import FusedSGD
    hvd.init()
    m = to_mixed_bf16(resnet50())
    opt = hvd.DistributedOptimizer(FusedSGD(m.parameters(), lr=0.1, momentum=0.9),
                                   named_parameters=m.named_parameters())
    names = [n for n, _ in m.named_parameters()]
    pos = {n: len(names) - 1 - i for i, n in enumerate(names)}      # backward position
    plan = opt.bucket_plan()
    ready = [max(pos[p] for p in ps) for _, _, ps in plan]
    assert ready == sorted(ready)
    assert plan[0][1] <= 4 * 2 ** 20            # small first bucket
    assert plan[-1][1] <= 5 * 2 ** 20           # small exposed tail
    assert sum(b for _, b, _ in plan) >= 25557032 * 2 * 0.99


def test_config_file_maps_sections_and_flags_win(tmp_path):
    from mivod.run.launcher import config_file_env, main
    cfg = tmp_path / "hvd.yaml"
    cfg.write_text("params:\n  fusion_threshold_mb: 16\n  cycle_time_ms: 3\n"
                   "  hierarchical_allreduce: true\n"
                   "timeline:\n  filename: /tmp/t.json\n  mark_cycles: true\n"
                   "stall_check:\n  enabled: false\n  warning_time_seconds: 30\n"
                   "logging:\n  level: debug\n")
    env = config_file_env(str(cfg))
    assert env["HOROVOD_FUSION_THRESHOLD"] == str(16 * 2 ** 20)
    assert env["HOROVOD_CYCLE_TIME"] == "3" and env["HOROVOD_HIERARCHICAL_ALLREDUCE"] == "1"
    assert env["HOROVOD_TIMELINE"] == "/tmp/t.json" and env["HOROVOD_TIMELINE_MARK_CYCLES"] == "1"
    assert env["HOROVOD_STALL_CHECK_DISABLE"] == "1"
    assert env["HOROVOD_STALL_CHECK_TIME_SECONDS"] == "30" and env["HOROVOD_LOG_LEVEL"] == "debug"
    bad = tmp_path / "bad.yaml"
    bad.write_text("params:\n  no_such_knob: 1\n")
    with pytest.raises(ValueError):
        config_file_env(str(bad))
    # the file feeds the ranks; a command-line flag overrides it
    prog = tmp_path / "show.py"
    prog.write_text("import os; print('FT', os.environ['HOROVOD_FUSION_THRESHOLD'], "
                    "'CT', os.environ['HOROVOD_CYCLE_TIME'], 'CC', os.environ['HOROVOD_CACHE_CAPACITY'])\n")
    r = subprocess.run([sys.executable, "-m", "mivod.run", "-np", "1", "--config-file", str(cfg),
                        "--cycle-time-ms", "7", "--disable-cache", "--output-filename",
                        str(tmp_path / "logs"), sys.executable, str(prog)],
                       cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert f"FT {16 * 2 ** 20} CT 7 CC 0" in r.stdout
    assert f"FT {16 * 2 ** 20} CT 7 CC 0" in (tmp_path / "logs" / "rank.0" / "stdout").read_text()


def test_check_build_lists_backends():
    r = subprocess.run([sys.executable, "-m", "mivod.run", "--check-build"], cwd=ROOT,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "[X] PyTorch" in r.stdout and "Available Tensor Operations:" in r.stdout
    assert "[ ] MPI" in r.stdout and "[X] Gloo" in r.stdout


FAKE_SSH = r'''#!/bin/bash
# test double for ssh: record the call, drop options, run the remote command locally.
# "fakenode" stands in for a remote host name (no DNS here): map it to loopback.
echo "$@" >> "%(log)s"
while [[ "$1" == -* ]]; do
  case "$1" in -o|-p) shift 2 ;; *) shift ;; esac
done
host="$1"; shift
remote="$*"
exec bash -c "${remote//fakenode/127.0.0.1}"
'''


def test_launch_remote_hosts_over_ssh(tmp_path):
    """-H with a non-local host goes through ssh: options, port, cwd and the rank env
    (HOROVOD_*, MASTER_*, -x exports) are carried on the remote command line."""
    log = tmp_path / "ssh.log"
    bindir = tmp_path / "bin"
    bindir.mkdir()
    ssh = bindir / "ssh"
    ssh.write_text(FAKE_SSH % {"log": log})
    ssh.chmod(0o755)
    f = tmp_path / "prog.py"
    f.write_text(SCRIPT)
    env = dict(os.environ, MIVOD_TRANSPORT="gloo", PYTHONPATH=ROOT,
               PATH=f"{bindir}{os.pathsep}{os.environ['PATH']}")
    r = subprocess.run([sys.executable, "-m", "mivod.run", "-np", "2", "-H", "fakenode:2",
                        "--ssh-port", "2222", "-x", "NCCL_DEBUG=INFO", "-x", "PYTHONPATH",
                        "-x", "MIVOD_TRANSPORT", sys.executable, str(f)],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "[0]<stdout>:rank 0 size 2 local 0 sum 1.0 nccl_debug INFO" in r.stdout, r.stdout
    assert "[1]<stdout>:rank 1 size 2 local 1 sum 1.0 nccl_debug INFO" in r.stdout, r.stdout
    calls = log.read_text().splitlines()
    assert len(calls) == 2
    for c in calls:
        assert "-p 2222" in c and "BatchMode=yes" in c and " fakenode " in c
        assert f"cd {ROOT}" in c and "HOROVOD_SIZE=2" in c and "MASTER_ADDR=fakenode" in c
