"""Multi-rank GPU hook path on ONE MI355X: 2 ranks share cuda:0 with a gloo wire
(MIVOD_TRANSPORT=gloo-gpu; RCCL refuses two ranks on one device).  Exercises the
pack kernel, the comm-stream collective and the fused update kernel with a real
2-rank reduction — the path the 8-GPU RCCL run takes, minus RCCL itself."""
import pytest

from test_multiprocess import run_ranks

pytestmark = pytest.mark.gpu


def test_gpu_hook_path_two_ranks_one_gpu(cuda):
    run_ranks("gpu_dist", 2, timeout=180, extra_env={"MIVOD_TRANSPORT": "gloo-gpu"})


def test_gpu_adasum_fp16_two_ranks_one_gpu(cuda):
    """Config-5 path (fp16 wire + Adasum + FusedAdamW) with 2 real ranks on one GPU."""
    run_ranks("gpu_adasum", 2, timeout=180, extra_env={"MIVOD_TRANSPORT": "gloo-gpu"})


def test_gpu_named_ops_during_backward_share_one_order(cuda):
    """hvd.allreduce from a backward hook and between backward and step, on the
    same communicator/stream as the bucket schedule: no hang, correct averages,
    bit-identical ranks."""
    run_ranks("gpu_order", 2, timeout=180, extra_env={"MIVOD_TRANSPORT": "gloo-gpu"})


def test_gpu_rccl_communicator_world1(cuda):
    """mivod's own RCCL communicator (csrc/comm) at world size 1 with the
    size-1 shortcut disabled: RCCL kernels really run for every collective."""
    run_ranks("gpu_rccl_single", 1, timeout=180,
              extra_env={"MIVOD_TRANSPORT": "rccl", "MIVOD_FORCE_COLLECTIVES": "1"})


def test_gpu_rccl_watchdog_aborts_a_stuck_collective(cuda):
    """Failure detection on hardware: the RCCL watchdog (csrc/comm/comm.cc) aborts a
    communicator whose collective outlives MIVOD_RCCL_TIMEOUT_S and later calls raise."""
    run_ranks("gpu_rccl_watchdog", 1, timeout=120,
              extra_env={"MIVOD_TRANSPORT": "rccl", "MIVOD_FORCE_COLLECTIVES": "1",
                         "MIVOD_RCCL_TIMEOUT_S": "1"})


def test_gpu_xgmi_mesh_one_shot_allreduce(cuda):
    """K7: the HIP-IPC mesh allreduce kernel between two processes on one GPU."""
    run_ranks("gpu_mesh", 2, timeout=180,
              extra_env={"MIVOD_TRANSPORT": "gloo-gpu", "MIVOD_MESH_MAX_MB": "1"})


def test_gpu_xgmi_mesh_two_shot_and_staged_pack(cuda):
    """K7 two-shot (mesh reduce-scatter + all-gather through IPC result buffers)
    for every bucket above 1 KB, and the bucket pack writing straight into the
    mesh staging slot: bitwise equal to the gloo wire, ranks identical."""
    run_ranks("gpu_mesh", 2, timeout=180,
              extra_env={"MIVOD_TRANSPORT": "gloo-gpu", "MIVOD_MESH_MAX_MB": "1",
                         "MIVOD_MESH_ONESHOT_KB": "1"})


def test_gpu_xgmi_mesh_timeout_exits_both_ranks(cuda):
    """A rank that never arrives: the waiting rank's mesh kernel times out, poisons
    its output and the watcher exits the process; the other rank then fails too."""
    rcs, outs = run_ranks("gpu_mesh_timeout", 2, timeout=120, expect_ok=False,
                          extra_env={"MIVOD_TRANSPORT": "gloo-gpu", "MIVOD_MESH_MAX_MB": "1",
                                     "MIVOD_MESH_TIMEOUT_S": "3"})
    assert rcs[0] != 0 and rcs[1] != 0, (rcs, outs)
    assert "did not arrive within" in outs[0], outs[0]
    assert "was not stopped" not in outs[0] and "passed a barrier" not in outs[1]


def test_gpu_xgmi_mesh_timeout_poisons_and_raises(cuda):
    run_ranks("gpu_mesh_timeout_raise", 2, timeout=120,
              extra_env={"MIVOD_TRANSPORT": "gloo-gpu", "MIVOD_MESH_MAX_MB": "1",
                         "MIVOD_MESH_TIMEOUT_S": "2", "MIVOD_MESH_TIMEOUT_EXIT": "0"})


def test_gpu_rccl_cta_config_and_autotune(cuda):
    """ncclCommInitRankConfig with a CTA range, and the CTA autotune loop over real
    communicators (world 1: the sweep mechanics, not the timing, are what is tested)."""
    import torch

    from mivod.parallel.autotune import tune_rccl_ctas
    from mivod.parallel.transport import RcclTransport
    made = []

    def make(c):
        t = RcclTransport.create(0, 1, cuda, min_ctas=c, max_ctas=c)
        made.append(t)
        return t

    best, c, res = tune_rccl_ctas(make, lambda t: t.time_allreduce([2 ** 20, 4 * 2 ** 20], iters=2),
                                  candidates=(0, 4, 8))
    assert [r[0] for r in res] == [0, 4, 8] and all(r[1] >= 0 for r in res)
    assert best.ctas == (c, c)
    x = torch.arange(1000, dtype=torch.float32, device=cuda)
    best.allreduce_(x)
    torch.cuda.synchronize()
    assert torch.equal(x, torch.arange(1000, dtype=torch.float32, device=cuda))
    best.close()


# ---- real multi-GPU RCCL (skipped on a 1-GPU box: RCCL refuses 2 ranks per device)
def _gpus():
    import torch
    return torch.cuda.device_count()


_MULTI = pytest.mark.skipif(_gpus() < 2, reason="needs >= 2 GPUs")


@_MULTI
@pytest.mark.parametrize("scenario", ["gpu_dist", "gpu_adasum", "gpu_order"])
def test_rccl_two_gpus(cuda, scenario):
    """The hook path, fp16-wire Adasum and the one-issue-order protocol over mivod's
    own RCCL communicator, one rank per GPU."""
    run_ranks(scenario, 2, timeout=240, extra_env={"MIVOD_TRANSPORT": "rccl"})


@_MULTI
def test_xgmi_mesh_two_gpus(cuda):
    """K7 one-shot allreduce between two GPUs' IPC-mapped staging buffers."""
    run_ranks("gpu_mesh", 2, timeout=240,
              extra_env={"MIVOD_TRANSPORT": "rccl", "MIVOD_MESH_MAX_MB": "1"})
