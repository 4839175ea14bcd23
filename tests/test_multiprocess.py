"""Multi-process CPU tier (T2): N local ranks over gloo, as horovod's own tests
run `mpirun -np 2 pytest`.  Scenarios live in tests/mp_workers.py."""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_ranks(scenario, n=2, timeout=240, extra_env=None, local_size=None, expect_ok=True):
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        ls = local_size or n
        env.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(r),
                    "WORLD_SIZE": str(n), "LOCAL_RANK": str(r % ls), "LOCAL_WORLD_SIZE": str(ls),
                    "MIVOD_TRANSPORT": "gloo", "OMP_NUM_THREADS": "1",
                    "PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", "")})
        env.pop("HOROVOD_RANK", None)
        if extra_env:
            env.update(extra_env)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "mp_workers.py"),
                                       scenario], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append(out)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    if not expect_ok:
        return [p.returncode for p in procs], outs
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0 and f"OK {r}" in out, f"rank {r} rc={p.returncode}\n{out}"
    return outs


def test_basics_2ranks():
    run_ranks("basics", 2)


def test_basics_4ranks():
    run_ranks("basics", 4)


def test_basics_2ranks_python_engine_loop():
    """The Python fallback of the negotiation loop (MIVOD_ENGINE=python) still works."""
    run_ranks("basics", 2, extra_env={"MIVOD_ENGINE": "python"})


def test_negotiation_errors():
    run_ranks("errors", 2)


def test_out_of_order_submission():
    run_ranks("out_of_order", 3)


def test_stall_inspector():
    run_ranks("stall", 2)


def test_distributed_optimizer_matches_averaged_reference():
    run_ranks("dist_optimizer", 2, timeout=400)


def test_broadcast_parameters_and_optimizer_state():
    run_ranks("broadcast_state", 2)


def test_adasum_4ranks():
    run_ranks("adasum", 4)


def test_timeline(tmp_path):
    path = str(tmp_path / "timeline.json")
    run_ranks("timeline", 2, extra_env={"HOROVOD_TIMELINE": path})
    assert os.path.getsize(path) > 0


def test_keras_tf2_style_2ranks():
    outs = run_ranks("keras_tf2", 2, timeout=400)
    assert "finished gradual learning rate warmup" in outs[0]


def test_keras_static_schedule_2ranks():
    """Keras gradients on the static schedule == the negotiated protocol."""
    run_ranks("keras_static", 2, timeout=300)


def test_hierarchical_allreduce_2x2():
    run_ranks("hierarchical", 4, local_size=2)


def test_horovod_namespace_2ranks():
    """``import horovod.torch as hvd`` scripts run unchanged on mivod."""
    run_ranks("horovod_namespace", 2)


def test_horovod_tensorflow_api_2ranks():
    """horovod.tensorflow surface (U18): sparse allreduce, global-variable broadcast,
    DistributedOptimizer.compute_gradients, DistributedGradientTape."""
    run_ranks("tensorflow_api", 2)


@pytest.mark.parametrize("n", [2, 3, 4])
def test_native_tcp_ring(n):
    """C++ ring allreduce / broadcast / allgatherv on CPU tensors (all dtypes incl.
    fp16 via F16C and bf16), bitwise identical across ranks, odd world sizes."""
    run_ranks("ring", n)


def test_schedule_mismatch_raises_on_all_ranks():
    """SURVEY §7.4 risk 4: a differing static bucket schedule raises everywhere."""
    outs = run_ranks("schedule_mismatch", 2)
    assert all(f"raised {r}" in o for r, o in enumerate(outs))


# ---- round 2: data-plane features -------------------------------------------
def test_adasum_vector_halving_4ranks():
    run_ranks("adasum_vhdd", 4)


def test_adasum_vector_halving_2ranks():
    run_ranks("adasum_vhdd", 2)


def test_overflow_guard_skips_bucket_on_every_rank():
    run_ranks("overflow_guard", 2)


def test_overflow_guard_step_mode_skips_whole_step():
    run_ranks("overflow_guard", 2, extra_env={"MIVOD_GUARD_MODE": "step"})


def test_timeline_records_bucket_phases(tmp_path):
    run_ranks("timeline_buckets", 2, extra_env={"HOROVOD_TIMELINE": str(tmp_path / "tl.json")})


def test_prescale_factors_are_not_fused_together():
    run_ranks("prescale_fusion", 2)


@pytest.mark.parametrize("cap", [0, 4, 1024])
def test_response_cache_capacity(cap):
    run_ranks("cache_capacity", 2, extra_env={"HOROVOD_CACHE_CAPACITY": str(cap)})


def test_checkpoint_resume_keeps_fp32_master_bf16(tmp_path):
    run_ranks("ckpt_bf16_resume", 2, extra_env={"MIVOD_TEST_DIR": str(tmp_path)})
