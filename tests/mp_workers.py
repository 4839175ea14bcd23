"""Multi-rank scenarios, run as `python tests/mp_workers.py <scenario>` by
tests/test_multiprocess.py in N processes (gloo on CPU).  Each scenario asserts
and prints "OK <rank>" at the end.  Reference behaviour: horovod's
test_torch.py style (rank-seeded tensors, sum == size * x, average == x, error
cases raise on every rank rather than hang)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import mivod.torch as hvd  # noqa: E402


def _close(a, b, tol=1e-5):
    torch.testing.assert_close(a, b, rtol=tol, atol=tol)


def basics():
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    assert n == int(os.environ["WORLD_SIZE"]) and r == int(os.environ["RANK"])
    assert hvd.local_rank() == r and hvd.local_size() == n
    assert hvd.cross_size() == 1 and hvd.cross_rank() == 0
    for dt in (torch.float32, torch.float64, torch.int32, torch.int64, torch.float16,
               torch.bfloat16):
        for dims in (1, 2, 3):
            torch.manual_seed(1234)
            x = (torch.rand([17] * dims) * 100).to(dt)
            s = hvd.allreduce(x, op=hvd.Sum, name=f"sum.{dt}.{dims}")
            tol = 1e-2 if dt in (torch.float16, torch.bfloat16) else 1e-5
            _close(s.double(), (x.double() * n), tol=tol * 100 if dt == torch.bfloat16 else tol)
            if dt.is_floating_point:
                a = hvd.allreduce(x, name=f"avg.{dt}.{dims}")
                _close(a.double(), x.double(), tol=tol * 10)
    # rank-dependent average
    x = torch.full((5,), float(r))
    _close(hvd.allreduce(x), torch.full((5,), (n - 1) / 2.0))
    # in-place + async + many names (fusion)
    hs = [hvd.allreduce_async_(torch.full((100 + i,), float(r + i)), name=f"fused.{i}",
                               op=hvd.Sum) for i in range(20)]
    for i, h in enumerate(hs):
        out = hvd.synchronize(h)
        _close(out, torch.full((100 + i,), float(sum(rr + i for rr in range(n)))))
    # compression
    y = torch.randn(1000)
    z = hvd.allreduce(y, compression=hvd.Compression.fp16, name="fp16c")
    _close(z, y.half().float(), tol=1e-3)
    # pre/post scale
    p = hvd.allreduce(torch.ones(4), op=hvd.Sum, prescale_factor=2.0, postscale_factor=0.5)
    _close(p, torch.full((4,), float(n)))
    # allgather, ragged first dim
    g = hvd.allgather(torch.full((r + 1, 3), float(r)), name="ag")
    assert g.shape == (sum(range(1, n + 1)), 3)
    off = 0
    for rr in range(n):
        _close(g[off:off + rr + 1], torch.full((rr + 1, 3), float(rr)))
        off += rr + 1
    # broadcast
    b = hvd.broadcast(torch.full((3,), float(r)), root_rank=n - 1, name="bc")
    _close(b, torch.full((3,), float(n - 1)))
    t = torch.full((2, 2), float(r))
    hvd.broadcast_(t, 0)
    _close(t, torch.zeros(2, 2))
    # alltoall
    a2a = hvd.alltoall(torch.arange(n * 2, dtype=torch.float32) + 100 * r)
    exp = torch.cat([torch.arange(2 * r, 2 * r + 2, dtype=torch.float32) + 100 * rr
                     for rr in range(n)])
    _close(a2a, exp)
    # autograd through allreduce
    w = torch.ones(3, requires_grad=True)
    hvd.allreduce(w * (r + 1), op=hvd.Sum).sum().backward()
    # d/dw sum(allreduce_sum(w*(r+1))) = allreduce_sum(ones) * (r+1) = n*(r+1)
    _close(w.grad, torch.full((3,), float(n * (r + 1))))
    # objects
    o = hvd.broadcast_object({"rank": r, "v": [1, 2]}, root_rank=0)
    assert o == {"rank": 0, "v": [1, 2]}
    objs = hvd.allgather_object(r * 10)
    assert objs == [rr * 10 for rr in range(n)]
    hvd.shutdown()
    print("OK", r)


def errors():
    hvd.init()
    r = hvd.rank()
    # mismatched shapes -> error on every rank, no hang
    try:
        hvd.allreduce(torch.ones(3 + r), name="bad.shape")
        raise AssertionError("expected failure")
    except hvd.HorovodInternalError as e:
        assert "Mismatched allreduce tensor shapes" in str(e), str(e)
    try:
        hvd.allreduce(torch.ones(3, dtype=torch.float32 if r == 0 else torch.float64),
                      name="bad.dtype")
        raise AssertionError("expected failure")
    except hvd.HorovodInternalError as e:
        assert "Mismatched data types" in str(e), str(e)
    try:
        hvd.broadcast(torch.ones(3), root_rank=r, name="bad.root")
        raise AssertionError("expected failure")
    except hvd.HorovodInternalError as e:
        assert "root rank" in str(e), str(e)
    # the engine still works afterwards
    _close(hvd.allreduce(torch.ones(3), name="good"), torch.ones(3))
    hvd.shutdown()
    print("OK", r)


def out_of_order():
    """Ranks submit the same names in different orders; negotiation matches them."""
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    names = [f"t{i}" for i in range(8)]
    order = names if r % 2 == 0 else list(reversed(names))
    hs = {nm: hvd.allreduce_async(torch.full((10,), float(r * 10 + int(nm[1:]))), name=nm,
                                  op=hvd.Sum) for nm in order}
    for nm in names:
        i = int(nm[1:])
        _close(hvd.synchronize(hs[nm]), torch.full((10,), float(sum(rr * 10 + i
                                                                      for rr in range(n)))))
    hvd.shutdown()
    print("OK", r)


def stall():
    os.environ["HOROVOD_STALL_CHECK_TIME_SECONDS"] = "1"
    hvd.init()
    r = hvd.rank()
    from mivod.common import basics
    eng = basics.state().engine
    if r == 0:
        h = hvd.allreduce_async(torch.ones(2), name="late")
        time.sleep(2.5)
        stalls = eng.controller.last_stalls()
        assert any(s[0] == "late" and 1 in s[1] for s in stalls), stalls
        _close(hvd.synchronize(h), torch.ones(2))
    else:
        time.sleep(3.0)
        _close(hvd.allreduce(torch.ones(2), name="late"), torch.ones(2))
    hvd.shutdown()
    print("OK", r)


def _toy(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8), torch.nn.ReLU(),
                               torch.nn.Flatten(), torch.nn.Linear(8 * 6 * 6, 10))


def _make_opt(kind, params):
    from mivod.optim import FusedAdam, FusedLARS, FusedSGD
    if kind == "fused_sgd":
        return FusedSGD(params, lr=0.1, momentum=0.9, weight_decay=1e-4)
    if kind == "fused_adam":
        return FusedAdam(params, lr=1e-2)
    if kind == "fused_lars":
        return FusedLARS(params, lr=0.5, momentum=0.9, weight_decay=1e-4)
    if kind == "torch_sgd":
        return torch.optim.SGD(params, lr=0.1, momentum=0.9, weight_decay=1e-4)
    if kind == "torch_adam":
        return torch.optim.Adam(params, lr=1e-2)
    raise ValueError(kind)


def dist_optimizer():
    """Params after k steps equal a single-process run on the averaged gradient
    (BN in train mode sees each rank's own batch, exactly as in DP)."""
    import copy
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    for kind in ("fused_sgd", "torch_sgd", "fused_adam", "torch_adam", "fused_lars"):
        comps = (hvd.Compression.none,) if "adam" in kind else (hvd.Compression.none,
                                                                  hvd.Compression.fp16)
        # (Adam normalises each coordinate, so fp16 rounding of tiny gradients is
        # not comparable elementwise; fp16 wire is covered with SGD / LARS.)
        for comp in comps:
            base = _toy(0)
            m = copy.deepcopy(base)
            opt = hvd.DistributedOptimizer(_make_opt(kind, m.parameters()),
                                           named_parameters=m.named_parameters(),
                                           compression=comp, bucket_mb=0.005,
                                           first_bucket_mb=0.001)
            hvd.broadcast_parameters(m.state_dict(), 0)
            # reference: same model, per-rank grads averaged by hand
            ref = copy.deepcopy(base)
            ref_opt = _make_opt(kind, ref.parameters())
            data = []
            for rr in range(n):
                g = torch.Generator().manual_seed(100 + rr)
                data.append((torch.randn(4, 3, 8, 8, generator=g), torch.randint(0, 10, (4,),
                                                                                  generator=g)))
            for step in range(3):
                x, y = data[r]
                opt.zero_grad()
                torch.nn.functional.cross_entropy(m(x), y).backward()
                opt.step()
                grads = None
                for rr in range(n):
                    refc = copy.deepcopy(ref)
                    refc.zero_grad()
                    torch.nn.functional.cross_entropy(refc(data[rr][0]), data[rr][1]).backward()
                    gs = [p.grad.clone() for p in refc.parameters()]
                    if comp is hvd.Compression.fp16:
                        gs = [g.half().float() for g in gs]
                    grads = gs if grads is None else [a + b for a, b in zip(grads, gs)]
                    if rr == r:
                        ref.load_state_dict(refc.state_dict())  # own BN running stats
                for p, g in zip(ref.parameters(), grads):
                    p.grad = g / n
                ref_opt.step()
            tol = 2e-3 if comp is hvd.Compression.fp16 else 2e-5
            for (nm, p), q in zip(m.named_parameters(), ref.parameters()):
                torch.testing.assert_close(p.detach(), q.detach(), rtol=tol, atol=tol,
                                           msg=lambda s: f"{kind} {comp.__name__} {nm}: {s}")
            # all ranks bit-identical
            flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
            allf = hvd.allgather(flat.unsqueeze(0))
            assert torch.equal(allf[0], allf[-1]), kind
    hvd.shutdown()
    print("OK", r)


def broadcast_state():
    import copy
    hvd.init()
    r = hvd.rank()
    for kind in ("fused_sgd", "torch_sgd", "torch_adam", "fused_adam"):
        m = _toy(seed=r)  # different init per rank
        opt = _make_opt(kind, m.parameters())
        opt.param_groups[0]["lr"] = 0.1 * (r + 1)
        # take a local step so state differs per rank
        torch.nn.functional.cross_entropy(m(torch.randn(2, 3, 8, 8)), torch.tensor([1, 2])).backward()
        opt.step()
        hvd.broadcast_parameters(m.state_dict(), root_rank=0)
        hvd.broadcast_optimizer_state(opt, root_rank=0)
        sd = copy.deepcopy(m.state_dict())
        allsd = hvd.allgather_object({k: v.clone() for k, v in sd.items()})
        for k in sd:
            assert torch.equal(allsd[0][k], allsd[-1][k]), (kind, k)
        assert abs(opt.param_groups[0]["lr"] - 0.1) < 1e-12, opt.param_groups[0]["lr"]
        st = opt.state_dict()["state"]
        allst = hvd.allgather_object({k: {kk: (vv.clone() if torch.is_tensor(vv) else vv)
                                          for kk, vv in v.items()} for k, v in st.items()})
        for pid in allst[0]:
            for kk, vv in allst[0][pid].items():
                ov = allst[-1][pid][kk]
                if torch.is_tensor(vv):
                    assert torch.equal(vv, ov), (kind, pid, kk)
    hvd.shutdown()
    print("OK", r)


def adasum():
    import numpy as np
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    vecs = [np.random.RandomState(7 + rr).randn(1000).astype(np.float64) for rr in range(n)]

    def comb(a, b):
        d = a @ b
        na, nb = a @ a, b @ b
        return (1 - d / (2 * na)) * a + (1 - d / (2 * nb)) * b

    cur = list(vecs)
    while len(cur) > 1:
        cur = [comb(cur[i], cur[i + 1]) for i in range(0, len(cur), 2)]
    out = hvd.allreduce(torch.tensor(vecs[r], dtype=torch.float32), op=hvd.Adasum, name="ada")
    np.testing.assert_allclose(out.numpy(), cur[0], rtol=1e-4, atol=1e-4)
    # identical gradients: adasum(g, g) = g
    g = torch.ones(50)
    _close(hvd.allreduce(g, op=hvd.Adasum, name="ada2"), g)
    # orthogonal gradients: sum
    e = torch.zeros(n * 4)
    e[r * 4:(r + 1) * 4] = 1.0
    _close(hvd.allreduce(e, op=hvd.Adasum, name="ada3"), torch.ones(n * 4))
    hvd.shutdown()
    print("OK", r)


def timeline():
    path = os.environ["HOROVOD_TIMELINE"]
    hvd.init()
    for i in range(3):
        hvd.allreduce(torch.ones(10) * i, name=f"tl.{i}")
    hvd.shutdown()
    from mivod.utils import timeline as TL
    TL.stop_timeline()
    if hvd_rank() == 0:
        import json
        ev = json.load(open(path))
        names = {e.get("name") for e in ev}
        assert "NEGOTIATE_allreduce" in names, names
        assert "QUEUE" in names and ("GLOO_ALLREDUCE" in names or "NCCL_ALLREDUCE" in names), names
    print("OK", hvd_rank())


def keras_tf2():
    """Config 2 (TF2-style Keras MNIST, 2 ranks): broadcast at batch 0, averaged
    gradients, MetricAverageCallback, LR warmup -> identical weights and logs."""
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    os.environ["PS_MODEL_PATH"] = tempfile.mkdtemp()
    from keras_mnist_tf2_style import main
    hist, model = main(["--epochs", "4", "--steps", "15"])
    r = hvd.rank()
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    allf = hvd.allgather(flat.unsqueeze(0))
    assert torch.equal(allf[0], allf[1])
    logs = hvd.allgather_object(hist.history)
    assert logs[0]["loss"] == logs[1]["loss"], logs       # averaged in place, identical
    assert logs[0]["loss"][-1] < logs[0]["loss"][0], logs[0]["loss"]
    assert abs(logs[0]["lr"][-1] - 0.001 * hvd.size()) < 1e-9, logs[0]["lr"]
    hvd.shutdown()
    print("OK", r)


def hierarchical():
    """2 'nodes' x 2 local ranks: HOROVOD_HIERARCHICAL_ALLREDUCE gives the same
    result as the flat allreduce; local/cross topology exposed."""
    os.environ["HOROVOD_HIERARCHICAL_ALLREDUCE"] = "1"
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    assert hvd.local_size() == 2 and hvd.cross_size() == 2
    assert hvd.local_rank() == r % 2 and hvd.cross_rank() == r // 2
    from mivod.common import basics
    assert basics.state().local_pg is not None and basics.state().cross_pg is not None
    x = torch.arange(7, dtype=torch.float32) + r
    _close(hvd.allreduce(x, op=hvd.Sum, name="h1"), torch.arange(7, dtype=torch.float32) * n +
           sum(range(n)))
    _close(hvd.allreduce(x, name="h2"), torch.arange(7, dtype=torch.float32) + (n - 1) / 2)
    # Max / Min are never summed by the two-level schedule (they run flat): the
    # Keras plan check MAX-reduces int64 hashes with hierarchical on
    from mivod.parallel import collectives as C
    h = torch.tensor([1000 + r, -r], dtype=torch.int64)
    C.allreduce_(h, C.Max)
    assert h.tolist() == [1000 + n - 1, 0], h
    m = torch.tensor([float(r), -float(r)])
    C.allreduce_(m, C.Min)
    assert m.tolist() == [0.0, -float(n - 1)], m
    m = torch.tensor([float(r)])
    C.hierarchical_allreduce_(m, C.Max)
    assert m.tolist() == [float(n - 1)], m
    hvd.shutdown()
    print("OK", r)


def horovod_namespace():
    """An unmodified horovod-style PyTorch script: ``import horovod.torch as hvd``."""
    import horovod.torch as hvd2
    hvd2.init()
    r, n = hvd2.rank(), hvd2.size()
    torch.manual_seed(r)                       # different init per rank ...
    m = torch.nn.Linear(5, 3)
    opt = torch.optim.SGD(m.parameters(), lr=0.1 * n)
    opt = hvd2.DistributedOptimizer(opt, named_parameters=m.named_parameters())
    hvd2.broadcast_parameters(m.state_dict(), root_rank=0)   # ... made identical
    hvd2.broadcast_optimizer_state(opt, root_rank=0)
    x = torch.randn(8, 5, generator=torch.Generator().manual_seed(10 + r))
    for _ in range(2):
        opt.zero_grad()
        m(x).pow(2).mean().backward()
        opt.step()
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    allf = hvd2.allgather(flat.unsqueeze(0))
    assert torch.equal(allf[0], allf[-1])
    avg = hvd2.allreduce(torch.tensor([float(r)]), name="ns.avg")
    _close(avg, torch.tensor([(n - 1) / 2]))
    hvd2.shutdown()
    print("OK", r)


def ring():
    """Native TCP ring data plane (csrc/engine/ring.cc) on CPU tensors."""
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    from mivod.common import basics as B
    st = B.state()
    assert st.rings is not None and len(st.rings) == 2, "native ring not active"
    from mivod.parallel import collectives as C
    for dt in (torch.float32, torch.float64, torch.float16, torch.bfloat16, torch.int32,
               torch.int64):
        for cnt in (0, 1, 7, n - 1, 1000, (1 << 20) + 3):
            g = torch.Generator().manual_seed(cnt)
            parts = [(torch.randn(cnt, generator=g) * 4).to(dt) for _ in range(n)]
            t = parts[r].clone()
            C.allreduce_(t, C.Sum)
            exp = sum(p.double() for p in parts) if cnt else torch.zeros(0, dtype=torch.float64)
            tol = {torch.float16: 0.06, torch.bfloat16: 0.3}.get(dt, 1e-4)
            assert t.dtype == dt and t.shape == (cnt,)
            if cnt:
                err = (t.double() - exp).abs().max().item()
                assert err <= tol * max(1.0, exp.abs().max().item() / 8), (dt, cnt, err)
            # bitwise identical on every rank
            chk = C.allgather(t.view(1, -1) if cnt else t.view(1, 0))
            assert all(torch.equal(chk[0], chk[i]) for i in range(n)), (dt, cnt)
    a = torch.full((5,), float(r + 1))
    C.allreduce_(a, C.Average)
    assert torch.allclose(a, torch.full((5,), (n + 1) / 2))
    b = torch.tensor([True, False, r == 0])
    C.allreduce_(b, C.Sum)
    assert b.tolist() == [True, False, True]
    for root in range(n):
        x = torch.arange(3 * (1 << 19) + 5, dtype=torch.float32) * (r + 1)
        C.broadcast_(x, root)
        assert torch.equal(x, torch.arange(3 * (1 << 19) + 5, dtype=torch.float32) * (root + 1))
    y = torch.full((r + 1, 3), float(r), dtype=torch.float16)
    g = C.allgather(y)
    assert g.shape == (sum(range(1, n + 1)), 3)
    o = 0
    for k in range(n):
        assert torch.all(g[o:o + k + 1] == k)
        o += k + 1
    # engine ring (named async ops) runs on its own sockets
    h = hvd.allreduce_async(torch.ones(4) * r, name="ring.async", op=hvd.Sum)
    _close(hvd.synchronize(h), torch.ones(4) * sum(range(n)))
    assert st.rings[0].ring.bytes_sent > 0 and st.rings[1].ring.bytes_sent > 0
    hvd.shutdown()
    print("OK", r)


def gpu_dist():
    """2 ranks sharing one GPU (MIVOD_TRANSPORT=gloo-gpu: GPU compute, gloo wire): the
    GPU hook path — pack kernel, comm-stream collective, fused update kernel — with a
    real multi-rank reduction.  fp32 toy model vs hand-averaged reference, then a
    bf16 ResNet with fused BN must stay bitwise identical across ranks."""
    import copy
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    dev = hvd.device()
    assert dev.type == "cuda"
    from mivod.optim import FusedSGD
    for comp in (hvd.Compression.none, hvd.Compression.fp16):
        base = _toy(0).to(dev)
        m = copy.deepcopy(base)
        opt = hvd.DistributedOptimizer(FusedSGD(m.parameters(), lr=0.1, momentum=0.9,
                                                weight_decay=1e-4),
                                       named_parameters=m.named_parameters(), compression=comp,
                                       bucket_mb=0.005, first_bucket_mb=0.001)
        assert len(opt.bucket_plan()) > 1
        ref = copy.deepcopy(base)
        ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        data = []
        for rr in range(n):
            g = torch.Generator().manual_seed(100 + rr)
            data.append((torch.randn(4, 3, 8, 8, generator=g).to(dev),
                         torch.randint(0, 10, (4,), generator=g).to(dev)))
        for step in range(3):
            x, y = data[r]
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            opt.step()
            grads = None
            for rr in range(n):
                refc = copy.deepcopy(ref)
                refc.zero_grad()
                torch.nn.functional.cross_entropy(refc(data[rr][0]), data[rr][1]).backward()
                gs = [p.grad.clone() for p in refc.parameters()]
                if comp is hvd.Compression.fp16:
                    gs = [q.half().float() for q in gs]
                grads = gs if grads is None else [a + b for a, b in zip(grads, gs)]
                if rr == r:
                    ref.load_state_dict(refc.state_dict())
            for p, g in zip(ref.parameters(), grads):
                p.grad = g / n
            ref_opt.step()
        torch.cuda.synchronize()
        tol = 2e-3 if comp is hvd.Compression.fp16 else 1e-4
        for (nm, p), q in zip(m.named_parameters(), ref.parameters()):
            torch.testing.assert_close(p.detach(), q.detach(), rtol=tol, atol=tol,
                                       msg=lambda s: f"{comp.__name__} {nm}: {s}")
        flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
        allf = hvd.allgather(flat.unsqueeze(0))
        assert torch.equal(allf[0], allf[-1])
    # bf16 ResNet, fused BN, per-rank data: parameters bitwise identical across ranks
    from mivod.models.resnet import ResNet, to_mixed_bf16
    torch.manual_seed(r)                                   # different init ...
    net = to_mixed_bf16(ResNet((1, 1, 1, 1), num_classes=10, zero_init_residual=True)).to(dev)
    o = hvd.DistributedOptimizer(FusedSGD(net.parameters(), lr=0.05, momentum=0.9),
                                 named_parameters=net.named_parameters())
    hvd.broadcast_parameters(net.state_dict(), 0)          # ... made identical
    g = torch.Generator(device=dev).manual_seed(7 + r)
    x = torch.rand(8, 3, 64, 64, device=dev, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=dev, generator=g)
    for _ in range(3):
        torch.nn.functional.cross_entropy(net(x).float(), y).backward()
        o.step()
        o.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().float().reshape(-1) for p in net.parameters()])
    allf = hvd.allgather(flat.unsqueeze(0))
    assert torch.isfinite(allf).all(), "non-finite parameters"
    bad = [nm for k, (nm, p) in enumerate(net.named_parameters())]
    if not torch.equal(allf[0], allf[-1]):
        d = (allf[0] - allf[-1]).abs()
        off = 0
        bad = []
        for nm, p in net.named_parameters():
            k = p.numel()
            if d[off:off + k].max() > 0:
                bad.append((nm, float(d[off:off + k].max())))
            off += k
        raise AssertionError(f"ranks differ: {bad[:10]}")
    hvd.shutdown()
    print("OK", r)


def gpu_adasum():
    """BASELINE config 5 path on GPU with 2 real ranks (gloo-gpu wire): Adasum kernels
    (seg_dot3 / adasum_combine) vs a float64 reference, then DistributedOptimizer with
    fp16 wire compression + Adasum + FusedAdamW keeps the ranks bit-identical."""
    import numpy as np
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    dev = hvd.device()
    vecs = [np.random.RandomState(7 + rr).randn(1000) for rr in range(n)]

    def comb(a, b):
        d = a @ b
        return (1 - d / (2 * (a @ a))) * a + (1 - d / (2 * (b @ b))) * b

    cur = list(vecs)
    while len(cur) > 1:
        cur = [comb(cur[i], cur[i + 1]) for i in range(0, len(cur), 2)]
    out = hvd.allreduce(torch.tensor(vecs[r], dtype=torch.float32, device=dev), op=hvd.Adasum,
                        name="gada")
    np.testing.assert_allclose(out.cpu().numpy(), cur[0], rtol=1e-4, atol=1e-4)
    from mivod.optim import FusedAdamW
    torch.manual_seed(0)
    m = _toy(0).to(dev)
    opt = hvd.DistributedOptimizer(FusedAdamW(m.parameters(), lr=1e-3),
                                   named_parameters=m.named_parameters(),
                                   compression=hvd.Compression.fp16, op=hvd.Adasum,
                                   bucket_mb=0.005, first_bucket_mb=0.001)
    g = torch.Generator().manual_seed(100 + r)
    x, y = torch.randn(4, 3, 8, 8, generator=g).to(dev), torch.randint(0, 10, (4,), generator=g).to(dev)
    before = [p.detach().clone() for p in m.parameters()]
    for _ in range(3):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    torch.cuda.synchronize()
    assert any((p.detach() - q).abs().max() > 0 for p, q in zip(m.parameters(), before))
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    allf = hvd.allgather(flat.unsqueeze(0))
    assert torch.isfinite(allf).all() and torch.equal(allf[0], allf[-1])
    hvd.shutdown()
    print("OK", r)


def schedule_mismatch():
    """Rank 1 wraps a different model: every rank raises (no hang, no silent mixing)."""
    hvd.init()
    r = hvd.rank()
    m = torch.nn.Linear(4, 4) if r == 0 else torch.nn.Linear(4, 5)
    try:
        hvd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1),
                                 named_parameters=m.named_parameters())
    except ValueError as e:
        assert "schedule differs across ranks" in str(e), e
        print("raised", r)
    else:
        raise AssertionError("schedule mismatch not detected")
    m2 = torch.nn.Linear(4, 4)
    hvd.DistributedOptimizer(torch.optim.SGD(m2.parameters(), lr=0.1),
                             named_parameters=m2.named_parameters())   # equal plans pass
    hvd.shutdown()
    print("OK", r)


def tensorflow_api():
    """``import horovod.tensorflow as hvd`` (U18): dense / IndexedSlices / sparse allreduce,
    broadcast_global_variables over every live model, DistributedOptimizer.compute_gradients
    and DistributedGradientTape return rank-averaged gradients."""
    import horovod.tensorflow as htf
    from mivod import kerasfw as keras
    htf.init()
    r, n = htf.rank(), htf.size()
    x = torch.full((6,), float(r + 1))
    _close(htf.allreduce(x), torch.full((6,), (n + 1) / 2.0))
    _close(htf.allreduce(x, average=False), torch.full((6,), n * (n + 1) / 2.0))
    _close(htf.allreduce(x, compression=htf.Compression.fp16), torch.full((6,), (n + 1) / 2.0),
           tol=1e-3)
    # IndexedSlices -> allgather of values + indices, values / size when averaging
    sl = htf.IndexedSlices(torch.full((1, 3), float(r + 1)), torch.tensor([r]), (n, 3))
    out = htf.allreduce(sl)
    assert isinstance(out, htf.IndexedSlices) and out.indices.tolist() == list(range(n))
    dense = out.to_dense()
    for rr in range(n):
        _close(dense[rr], torch.full((3,), (rr + 1) / n))
    sp = torch.sparse_coo_tensor(torch.tensor([[0]]), torch.full((1, 2), 2.0), (n, 2))
    d = htf.allreduce(sp, average=False)
    assert d.is_sparse
    _close(d.to_dense()[0], torch.full((2,), 2.0 * n))
    # broadcast_global_variables: every live model (no model argument, as in TF1)
    torch.manual_seed(100 + r)
    m1 = keras.Sequential([keras.layers.Dense(4, input_shape=(3,))])
    m1.build((None, 3))
    m2 = keras.Sequential([keras.layers.Dense(2, input_shape=(5,))])
    m2.build((None, 5))
    htf.broadcast_global_variables(0)
    gv = htf.global_variables()
    assert len(gv) >= 4
    flat = torch.cat([v.detach().reshape(-1) for v in gv])
    allf = htf.allgather(flat.unsqueeze(0))
    assert torch.equal(allf[0], allf[-1])
    # DistributedOptimizer.compute_gradients: averaged; apply_gradients keeps ranks in sync
    opt = htf.DistributedOptimizer(keras.optimizers.SGD(lr=0.1))
    w = list(m1.trainable_weights)
    inp = torch.full((2, 3), float(r + 1))
    gv_pairs = opt.compute_gradients(m1(inp).sum(), w)
    local = torch.autograd.grad(m1(inp).sum(), w)
    every = htf.allgather(torch.cat([g.reshape(-1) for g in local]).unsqueeze(0))
    _close(torch.cat([g.reshape(-1) for g, _ in gv_pairs]), every.mean(0))
    opt.apply_gradients(gv_pairs)
    flat = torch.cat([v.detach().reshape(-1) for v in m1.trainable_weights]).unsqueeze(0)
    allf = htf.allgather(flat)
    assert torch.equal(allf[0], allf[-1])
    # DistributedGradientTape
    v = torch.tensor([1.0, 2.0], requires_grad=True)
    with htf.DistributedGradientTape(htf.GradientTape()) as tape:
        loss = (v * float(r + 1)).sum()
    g = tape.gradient(loss, v)
    _close(g, torch.full((2,), (n + 1) / 2.0))
    htf.shutdown()
    print("OK", r)

def adasum_vhdd():
    """Vector-halving / distance-doubling Adasum (mivod.parallel.adasum) on a fused
    multi-tensor buffer equals the full-vector recursive-doubling reference within
    fp32 tolerance, sends <= 2*S*(N-1)/N bytes per rank, and leaves every rank with
    identical bits — fp32 and bf16 wires, odd segment sizes."""
    from mivod.ops import kernels as K
    from mivod.parallel import adasum as A
    from mivod.parallel import collectives as C
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    sizes = [1, 63, 4096 + 5, 130, 9000, 7]
    offs, o = [], 0
    for sz in sizes:
        offs.append(o)
        o += (sz + 63) // 64 * 64
    S = o
    table = K.make_chunk_table(sizes, "cpu", offs)
    vecs = []
    for rr in range(n):
        v = torch.zeros(S)
        g = torch.Generator().manual_seed(31 + rr)
        for sz, off in zip(sizes, offs):
            v[off:off + sz] = torch.randn(sz, generator=g) * (1 + rr)
        vecs.append(v)
    ref = A.adasum_reference(vecs, table)
    for dt, tol in ((torch.float32, 2e-5), (torch.bfloat16, 3e-2)):
        buf = vecs[r].to(dt).clone()
        C.allreduce_(buf, C.Adasum, adasum_table=table)
        es = buf.element_size()
        bound = 2 * S * (n - 1) / n * es + 2 * A.LAST["levels"] * A.ALIGN * es
        assert A.LAST["exchange_bytes"] <= bound, (A.LAST, bound)
        # Gram partials are summed inside each level's 2^(i+1) group only:
        # (i+1) exchanges of nseg*3 fp32 at level i, independent of the world size
        L = A.LAST["levels"]
        assert A.LAST["dot_bytes"] == sum(i + 1 for i in range(L)) * len(sizes) * 3 * 4, A.LAST
        wire_ref = A.adasum_reference([v.to(dt).float() for v in vecs], table)
        err = (buf.float() - wire_ref).abs().max().item()
        scale = wire_ref.abs().max().item()
        assert err <= tol * scale, (dt, err, scale)
        if dt == torch.float32:
            torch.testing.assert_close(buf, ref, rtol=2e-5, atol=2e-5 * scale)
        allb = C.allgather(buf.float().unsqueeze(0))
        assert all(torch.equal(allb[0], allb[i]) for i in range(n)), dt
    # fresh tables with the SAME total but different segment layouts, built and
    # dropped one after another (CPython may reuse the address): each call must
    # use its own segment boundaries (the clipped-table cache lives on the table)
    for lay in ([64, 128], [128, 64], [64, 128]):
        tab = K.make_chunk_table(lay, "cpu")
        vs = [torch.randn(192, generator=torch.Generator().manual_seed(7 + q)) * (q + 1)
              for q in range(n)]
        x = vs[r].clone()
        C.allreduce_(x, C.Adasum, adasum_table=tab)
        torch.testing.assert_close(x, A.adasum_reference(vs, tab), rtol=2e-5, atol=2e-5)
        del tab
    # identical inputs: adasum(g, ..., g) = g ; orthogonal inputs: the sum
    g = torch.linspace(-1, 1, 300)
    t1 = K.make_chunk_table([300], "cpu")
    x = g.clone()
    C.allreduce_(x, C.Adasum, adasum_table=t1)
    _close(x, g)
    e = torch.zeros(n * 64)
    e[r * 64:(r + 1) * 64] = 1.0
    C.allreduce_(e, C.Adasum, adasum_table=K.make_chunk_table([n * 64], "cpu"))
    _close(e, torch.ones(n * 64))
    hvd.shutdown()
    print("OK", r)


def overflow_guard():
    """fp16 wire + FusedSGD: rank 1 injects inf into one gradient at step 2.  The
    reduced bucket holding it is non-finite on EVERY rank (the scan of the reduced
    bucket sets the same flag everywhere, no extra collective):
    MIVOD_GUARD_MODE=bucket (default) skips that bucket's update on every rank
    while the other buckets' updates (already overlapped with backward) apply;
    MIVOD_GUARD_MODE=step skips the whole step.  Parameters stay identical
    across ranks and finite, a warning is logged, the saved optimizer state
    does not count a fully skipped step, and training continues afterwards."""
    import warnings
    from mivod.optim import FusedSGD
    mode = os.environ.get("MIVOD_GUARD_MODE", "bucket")
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    torch.manual_seed(0)
    m = _toy(0)
    opt = hvd.DistributedOptimizer(FusedSGD(m.parameters(), lr=0.1, momentum=0.9),
                                   named_parameters=m.named_parameters(),
                                   compression=hvd.Compression.fp16,
                                   bucket_mb=0.005, first_bucket_mb=0.001)
    gs = opt.guard_stats()
    assert gs["enabled"] and gs["mode"] == mode
    plan = opt.bucket_plan()
    assert len(plan) > 1
    names = [nm for nm, _ in m.named_parameters()]
    first = names[0]
    poisoned = next(i for i, (_, _, ps) in enumerate(plan) if first in ps)
    in_poisoned = [nm in plan[poisoned][2] for nm in names]
    assert not all(in_poisoned)
    g = torch.Generator().manual_seed(100 + r)
    x, y = torch.randn(4, 3, 8, 8, generator=g), torch.randint(0, 10, (4,), generator=g)
    snap = {}
    inject = [False]

    def poison(gr):               # the fused path frees p.grad after packing: poison
        if inject[0]:             # the gradient on its way into the accumulator
            gr = gr.clone()
            gr.view(-1)[0] = float("inf")
        return gr

    next(iter(m.parameters())).register_hook(poison)
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        for step in range(1, 5):
            inject[0] = step == 2 and r == 1
            before = [p.detach().clone() for p in m.parameters()]
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            opt.step()
            snap[step] = (before, [p.detach().clone() for p in m.parameters()])
            if step == 2:
                sd = opt.state_dict()          # resolves the step-2 flags first
    b2, a2 = snap[2]
    same = [torch.equal(p, q) for p, q in zip(b2, a2)]
    if mode == "step":
        assert all(same), "overflow step was not skipped"
        steps = {int(v["step"]) for v in sd["state"].values() if "step" in v}
        assert steps == {1}, steps          # the skipped step is not counted
    else:
        assert all(s_ for s_, ip in zip(same, in_poisoned) if ip), "poisoned bucket applied"
        assert not all(s_ for s_, ip in zip(same, in_poisoned) if not ip), \
            "clean buckets were not applied"
    b3, a3 = snap[3]
    assert any(not torch.equal(p, q) for p, q in zip(b3, a3)), "training did not resume"
    assert opt.guard_stats()["skipped_steps"] == 1, opt.guard_stats()
    assert any("skipped on every rank" in str(w.message) for w in caught)
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    allf = hvd.allgather(flat.unsqueeze(0))
    assert torch.isfinite(allf).all() and torch.equal(allf[0], allf[-1])
    hvd.shutdown()
    print("OK", r)


def timeline_buckets():
    """HOROVOD_TIMELINE records every bucket of the static gradient schedule with
    its pack / collective / fused-step phases as complete events."""
    import json
    from mivod.optim import FusedSGD
    path = os.environ["HOROVOD_TIMELINE"]
    hvd.init()
    r = hvd.rank()
    m = _toy(0)
    opt = hvd.DistributedOptimizer(FusedSGD(m.parameters(), lr=0.1, momentum=0.9),
                                   named_parameters=m.named_parameters(),
                                   bucket_mb=0.005, first_bucket_mb=0.001)
    nb = len(opt.bucket_plan())
    assert nb > 1
    g = torch.Generator().manual_seed(r)
    x, y = torch.randn(4, 3, 8, 8, generator=g), torch.randint(0, 10, (4,), generator=g)
    for _ in range(2):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    hvd.shutdown()
    from mivod.utils import timeline as TL
    TL.stop_timeline()
    if r == 0:
        ev = json.load(open(path))
        rows = {e["pid"]: e["args"]["name"] for e in ev if e.get("name") == "process_name"}
        per = {}
        for e in ev:
            if e.get("ph") == "X":
                per.setdefault(rows[e["pid"]], []).append(e["name"])
                assert e["dur"] >= 0 and e["ts"] >= 0
        for k in range(nb):
            phases = per.get(f"bucket.{k}", [])
            for ph in ("MEMCPY_IN_FUSION_BUFFER", "RING_ALLREDUCE", "OPTIMIZER_STEP"):
                assert phases.count(ph) == 2, (k, ph, phases)
    print("OK", r)


def prescale_fusion():
    """Two allreduces with different prescale factors submitted in one cycle are
    never fused under one factor (the coordinator keys fusion on them); equal
    factors fuse; mismatched factors across ranks raise on every rank."""
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    a = torch.full((5,), float(r + 1))
    b = torch.full((7,), float(r + 1))
    ha = hvd.allreduce_async(a, name="ps.a", op=hvd.Sum, prescale_factor=0.5)
    hb = hvd.allreduce_async(b, name="ps.b", op=hvd.Sum, prescale_factor=2.0, postscale_factor=3.0)
    tot = n * (n + 1) / 2
    _close(hvd.synchronize(ha), torch.full((5,), 0.5 * tot))
    _close(hvd.synchronize(hb), torch.full((7,), 6.0 * tot))
    hs = [hvd.allreduce_async(torch.full((3,), float(r)), name=f"ps.eq{i}", op=hvd.Sum,
                              prescale_factor=0.25) for i in range(3)]
    for h in hs:
        _close(hvd.synchronize(h), torch.full((3,), 0.25 * sum(range(n))))
    try:
        hvd.allreduce(torch.ones(2), name="ps.bad", op=hvd.Sum, prescale_factor=1.0 + r)
    except Exception as e:
        assert "prescale" in str(e), e
    else:
        raise AssertionError("mismatched prescale not detected")
    hvd.shutdown()
    print("OK", r)


def cache_capacity():
    """HOROVOD_CACHE_CAPACITY bounds the response cache (FIFO slots, mirrored on
    the coordinator); all-hit cycles travel as bit vectors; 0 disables the cache.
    Results stay correct throughout."""
    from mivod.common import basics as B
    cap = int(os.environ["HOROVOD_CACHE_CAPACITY"])
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    for it in range(12):
        names = [f"cc.{(it + k) % 6}" for k in range(3)]
        hs = [hvd.allreduce_async(torch.full((4,), float(r + k)), name=nm, op=hvd.Sum)
              for k, nm in enumerate(names)]
        for k, h in enumerate(hs):
            _close(hvd.synchronize(h), torch.full((4,), float(sum(range(n)) + n * k)))
    # a burst of repeated names submitted together -> all-hit cycles
    for it in range(20):
        hs = [hvd.allreduce_async(torch.ones(2), name=f"bv.{k}", op=hvd.Sum) for k in range(12)]
        for h in hs:
            _close(hvd.synchronize(h), torch.full((2,), float(n)))
    ctl = B.state().engine.controller.ctl
    assert ctl.cache_size <= cap, (ctl.cache_size, cap)
    if cap == 0:
        assert ctl.cache_size == 0 and ctl.cache_hits == 0
    if r == 0 and cap >= 12:
        assert ctl.cache_hits > 0
    hvd.shutdown()
    print("OK", r)


def ckpt_bf16_resume():
    """Resume of a bf16 model with a fused optimizer keeps the checkpointed fp32
    master weights bit-for-bit on every rank (broadcast_parameters followed by
    broadcast_optimizer_state must not re-seed the master from the bf16 copy)."""
    import tempfile
    from mivod.optim import FusedAdam
    from mivod.utils.checkpoint import load_checkpoint, save_checkpoint
    hvd.init()
    r = hvd.rank()
    d = os.environ.get("MIVOD_TEST_DIR") or tempfile.mkdtemp()
    path = os.path.join(d, "checkpoint-3.safetensors")

    def make(seed):
        torch.manual_seed(seed)
        m = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Linear(5, 3)).to(torch.bfloat16)
        o = hvd.DistributedOptimizer(FusedAdam(m.parameters(), lr=1e-2),
                                     named_parameters=m.named_parameters())
        return m, o

    m, o = make(0)
    hvd.broadcast_parameters(m.state_dict(), 0)
    x = torch.randn(4, 6, generator=torch.Generator().manual_seed(r)).to(torch.bfloat16)
    for _ in range(3):
        o.zero_grad()
        m(x).float().pow(2).mean().backward()
        o.step()
    master = torch.cat([a.master.clone() for a in o._mv_arenas])
    save_checkpoint(path, m, o, epoch=3)
    hvd.allreduce(torch.zeros(1), name="ck.barrier")
    m2, o2 = make(100 + r)                            # different weights per rank
    info = load_checkpoint(path, m2, o2)
    assert info["epoch"] == 3
    o2._mv_begin_step()                               # what the next step does first
    got = torch.cat([a.master.clone() for a in o2._mv_arenas])
    assert torch.equal(got, master), (got - master).abs().max()
    allm = hvd.allgather(got.unsqueeze(0))
    assert torch.equal(allm[0], allm[-1])
    hvd.shutdown()
    print("OK", r)


def fault_run():
    """Training loop for the fault-injection tests (MIVOD_FAULT set by the test)."""
    from mivod.optim import FusedSGD
    hvd.init()
    m = _toy(0)
    opt = hvd.DistributedOptimizer(FusedSGD(m.parameters(), lr=0.01),
                                   named_parameters=m.named_parameters())
    x, y = torch.randn(4, 3, 8, 8), torch.randint(0, 10, (4,))
    for _ in range(6):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    hvd.shutdown()
    print("OK", hvd_rank())


def gpu_order():
    """ONE communicator, two producers: the hook-driven bucket schedule and named
    ops submitted (a) from a backward hook in the middle of backward and (b) between
    backward and step (metric averaging) — every rank runs them in the same order,
    results match the reference and ranks stay bit-identical (2 ranks on one GPU,
    gloo-gpu wire; the same protocol orders RCCL on 8 GPUs)."""
    from mivod.optim import FusedSGD
    from mivod.parallel.order import ORDER
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    dev = hvd.device()
    assert ORDER.enabled
    torch.manual_seed(0)
    m = _toy(0).to(dev)
    opt = hvd.DistributedOptimizer(FusedSGD(m.parameters(), lr=0.05, momentum=0.9),
                                   named_parameters=m.named_parameters(),
                                   bucket_mb=0.002, first_bucket_mb=0.001)
    assert len(opt.bucket_plan()) >= 3
    seen = []

    def hook(mod, gin, gout):
        v = hvd.allreduce(torch.full((3,), float(r + 1), device=dev), name=f"mid.{len(seen)}")
        seen.append(v)

    bn = [mm for mm in m.modules() if isinstance(mm, torch.nn.BatchNorm2d)][0]
    bn.register_full_backward_hook(hook)           # fires in the middle of backward
    g = torch.Generator().manual_seed(100 + r)
    x, y = torch.randn(4, 3, 8, 8, generator=g).to(dev), torch.randint(0, 10, (4,), generator=g).to(dev)
    for step in range(4):
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(m(x), y)
        loss.backward()
        avg = hvd.allreduce(loss.detach().reshape(1), name=f"loss.{step}")   # between bwd and step
        opt.step()
        la = hvd.allgather(loss.detach().reshape(1))
        _close(avg, la.mean().reshape(1), tol=1e-5)
    torch.cuda.synchronize()
    for v in seen:
        _close(v, torch.full((3,), (n + 1) / 2.0, device=dev))
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    allf = hvd.allgather(flat.unsqueeze(0))
    assert torch.equal(allf[0], allf[-1])
    hvd.shutdown()
    print("OK", r)


def gpu_rccl_single():
    """MIVOD_FORCE_COLLECTIVES=1 at world size 1: mivod's own RCCL communicator
    (csrc/comm) is created and EVERY collective really launches on the GPU —
    allreduce sum/avg/premul over the dtypes, broadcast, allgather, Adasum, and a
    DistributedOptimizer step whose bucket allreduce rides RCCL on the comm stream."""
    from mivod.common import basics as B
    from mivod.optim import FusedSGD
    from mivod.parallel import collectives as C
    hvd.init()
    st = B.state()
    assert st.gpu is not None and st.gpu.name == "rccl", st.backend
    dev = hvd.device()
    calls0 = C.gpu_stats()["calls"]
    for dt in (torch.float32, torch.bfloat16, torch.float16, torch.int32, torch.int64):
        x = (torch.arange(1000, device=dev) % 17).to(dt)
        y = x.clone()
        C.allreduce_(y, C.Sum)
        assert torch.equal(y, x), dt
        C.allreduce_(y, C.Average)
        assert torch.equal(y, x), dt
        if dt.is_floating_point:
            z = x.clone()
            C.allreduce_(z, C.Sum, prescale=0.5)
            torch.testing.assert_close(z.float(), x.float() * 0.5)
    b = torch.arange(10, device=dev, dtype=torch.float32)
    C.broadcast_(b, 0)
    assert torch.equal(b, torch.arange(10, device=dev, dtype=torch.float32))
    import copy
    m = _toy(0).to(dev)
    twin = copy.deepcopy(m)
    ref = [p.detach().clone() for p in m.parameters()]
    opt = hvd.DistributedOptimizer(FusedSGD(m.parameters(), lr=0.1),
                                   named_parameters=m.named_parameters())
    g = torch.Generator().manual_seed(0)
    x, yy = torch.randn(4, 3, 8, 8, generator=g).to(dev), torch.randint(0, 10, (4,), generator=g).to(dev)
    torch.nn.functional.cross_entropy(twin(x), yy).backward()
    grads = [p.grad.detach().clone() for p in twin.parameters()]   # fused path frees p.grad
    torch.nn.functional.cross_entropy(m(x), yy).backward()
    opt.step()
    torch.cuda.synchronize()
    for p, q, gr in zip(m.parameters(), ref, grads):
        torch.testing.assert_close(p.detach(), q - 0.1 * gr, rtol=1e-5, atol=1e-6)
    calls = C.gpu_stats()["calls"] - calls0
    assert calls >= 14, calls
    # the hierarchical branch (reduce-scatter / cross allreduce / allgather on
    # ncclCommSplit children) with 1-rank local and cross comms
    st.gpu_local = st.gpu.split(0, 0)
    st.gpu_cross = st.gpu.split(0, 0)
    assert st.gpu_local.size == 1 and st.gpu_cross.size == 1
    for n in (1000, 4097):
        h = torch.arange(n, device=dev, dtype=torch.float32) % 13
        ref = h.clone()
        C._hierarchical_gpu_(h, C.Sum, 0.5)
        torch.testing.assert_close(h, ref * 0.5)
        C._hierarchical_gpu_(h, C.Average, 1.0)
        torch.testing.assert_close(h, ref * 0.5)
    st.gpu_local.close()
    st.gpu_cross.close()
    st.gpu_local = st.gpu_cross = None
    st.gpu.check()
    hvd.shutdown()
    print("OK", 0)


def gpu_mesh():
    """xGMI mesh one-shot allreduce (csrc/comm/mesh.hip) with 2 real ranks on one GPU
    (HIP IPC between the two processes): bitwise equal to the reference wire
    (gloo-gpu), deterministic across repeats, identical on both ranks; then a
    DistributedOptimizer whose small buckets ride the mesh keeps ranks identical."""
    from mivod.common import basics as B
    from mivod.optim import FusedSGD
    from mivod.parallel import collectives as C
    from mivod.parallel import transport as T
    hvd.init()
    r, n = hvd.rank(), hvd.size()
    dev = hvd.device()
    st = B.state()
    assert st.mesh is not None, "mesh not created"
    for dt in (torch.float32, torch.bfloat16, torch.float16):
        for cnt in (1, 7, 8, 64, 1000, 65536 + 3, 200000):
            g = torch.Generator().manual_seed(cnt * 10 + r)
            x = (torch.randn(cnt, generator=g) * 3).to(dt).to(dev)
            ref = x.clone()
            st.gpu.allreduce_(ref, T.SUM)                   # the gloo-gpu wire, no mesh
            y = x.clone()
            calls = st.mesh.mesh.calls
            C.allreduce_(y, C.Sum)
            assert st.mesh.mesh.calls == calls + 1, "allreduce did not take the mesh"
            torch.cuda.synchronize()
            assert torch.equal(y, ref), (dt, cnt, (y.float() - ref.float()).abs().max())
            y2 = x.clone()
            C.allreduce_(y2, C.Sum)
            assert torch.equal(y, y2), "mesh not deterministic"
            a = x.clone()
            C.allreduce_(a, C.Average)
            torch.testing.assert_close(a.float(), ref.float() / n, rtol=1e-2, atol=1e-2)
            allb = hvd.allgather(y.float().unsqueeze(0))
            assert torch.equal(allb[0], allb[-1])
    big = torch.ones(2 * 2 ** 20, device=dev)                   # 8 MB > 1 MB: RCCL/gloo path
    calls = st.mesh.mesh.calls
    C.allreduce_(big, C.Sum)
    assert st.mesh.mesh.calls == calls and float(big[0]) == n
    torch.manual_seed(0)
    m = _toy(0).to(dev)
    opt = hvd.DistributedOptimizer(FusedSGD(m.parameters(), lr=0.05, momentum=0.9),
                                   named_parameters=m.named_parameters(),
                                   bucket_mb=0.002, first_bucket_mb=0.001)
    gg = torch.Generator().manual_seed(100 + r)
    x, y = torch.randn(4, 3, 8, 8, generator=gg).to(dev), torch.randint(0, 10, (4,), generator=gg).to(dev)
    calls = st.mesh.mesh.calls
    for _ in range(3):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
    torch.cuda.synchronize()
    assert st.mesh.mesh.calls >= calls + 3 * len(opt.bucket_plan())
    # the bucket pack kernel wrote straight into the IPC staging slot (no copy)
    assert st.mesh.mesh.copies_saved >= 3 * len(opt.bucket_plan()), st.mesh.stats()
    if int(os.environ.get("MIVOD_MESH_ONESHOT_KB", "1024")) < 64:
        assert st.mesh.mesh.two_shot_calls > 0, st.mesh.stats()
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    allf = hvd.allgather(flat.unsqueeze(0))
    assert torch.equal(allf[0], allf[-1])
    assert st.mesh.status() == 0
    hvd.shutdown()
    print("OK", r)


def gpu_mesh_timeout():
    """A peer that never arrives: rank 1 skips the mesh allreduce.  Rank 0's
    kernel waits MIVOD_MESH_TIMEOUT_S, poisons the output with NaN, sets the
    host-mapped status word, and the native watcher ends rank 0 with a
    diagnosis (exit 1).  Rank 1 sits in a gloo barrier and fails when rank 0's
    connection drops: both ranks exit non-zero, nobody trains on a local gradient."""
    import time
    import torch.distributed as dist
    from mivod.common import basics as B
    from mivod.parallel import collectives as C
    hvd.init()
    r = hvd.rank()
    dev = hvd.device()
    st = B.state()
    assert st.mesh is not None and st.mesh.mesh.timeout_s <= 5
    if r == 0:
        x = torch.ones(1000, device=dev)
        C.allreduce_(x, C.Sum)
        torch.cuda.synchronize()
        time.sleep(20)              # the watcher exits the process long before this
        print("rank 0 was not stopped by the mesh watcher", flush=True)
        sys.exit(0)
    dist.barrier(group=st.cpu_pg)   # never completes: rank 0 dies
    print("rank 1 passed a barrier rank 0 never reached", flush=True)
    sys.exit(0)


def gpu_mesh_timeout_raise():
    """MIVOD_MESH_TIMEOUT_EXIT=0: the timed-out allreduce leaves NaN in the output
    (not the local gradient), status() reports it, and every later mesh call raises."""
    import time
    import torch.distributed as dist
    from mivod.common import basics as B
    from mivod.parallel import collectives as C
    hvd.init()
    r = hvd.rank()
    dev = hvd.device()
    st = B.state()
    if r == 0:
        x = torch.ones(1000, device=dev)
        C.allreduce_(x, C.Sum)
        torch.cuda.synchronize()
        assert bool(torch.isnan(x).all()), x[:8]
        t0 = time.time()
        while not st.mesh.mesh.failed() and time.time() - t0 < 5:
            time.sleep(0.02)
        assert st.mesh.status() == 1 and st.mesh.mesh.failed()
        try:
            C.allreduce_(torch.ones(8, device=dev), C.Sum)
            raise AssertionError("a failed mesh accepted another allreduce")
        except RuntimeError as e:
            assert "timed out" in str(e), e
    dist.barrier(group=st.cpu_pg)
    print("OK", r, flush=True)
    os._exit(0)                     # skip shutdown: the mesh epochs are out of step


def gpu_mesh_bench():
    """Timing of the mesh allreduce (for rocprof): 2 ranks on one GPU, 64 KB - 4 MB."""
    from mivod.common import basics as B
    from mivod.parallel import collectives as C
    hvd.init()
    r = hvd.rank()
    dev = hvd.device()
    assert B.state().mesh is not None
    for kb in (64, 256, 1024, 4096):
        x = torch.randn(kb * 256, device=dev).to(torch.bfloat16)     # kb KiB of bf16 x2
        for _ in range(5):
            C.allreduce_(x, C.Sum)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            C.allreduce_(x, C.Sum)
        e1.record()
        torch.cuda.synchronize()
        if r == 0:
            print(f"mesh allreduce {kb * 512 // 1024} KiB bf16: {e0.elapsed_time(e1) / 50 * 1000:.1f} us",
                  flush=True)
    assert B.state().mesh.status() == 0
    hvd.shutdown()
    print("OK", r)


def hvd_rank():
    return int(os.environ.get("RANK", "0"))



def keras_static():
    """Keras DistributedOptimizer on the static schedule: one plan (checked across
    ranks) reused every step, same weights as the negotiated per-tensor protocol,
    identical on every rank; a mismatched gradient set is refused."""
    import numpy as np

    import mivod.keras as hk
    import mivod.kerasfw as keras
    hvd.init()
    r = hvd.rank()
    rng = np.random.default_rng(100 + r)
    xs = rng.standard_normal((6, 16, 8)).astype(np.float32)
    ys = rng.integers(0, 4, (6, 16)).astype(np.int64)

    def train(negotiated):
        os.environ["MIVOD_KERAS_NEGOTIATED"] = "1" if negotiated else "0"
        torch.manual_seed(0)
        model = keras.Sequential([keras.layers.Dense(16, activation="relu"),
                                  keras.layers.Dense(4)])
        opt = hk.DistributedOptimizer(keras.optimizers.SGD(0.1, momentum=0.9))
        model.compile(loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=opt)
        for x, y in zip(xs, ys):
            model.train_on_batch(x, y)
        flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        return flat, opt

    fs, opt_s = train(False)
    fn, _ = train(True)
    assert opt_s._hvd_static.plans == 1, opt_s._hvd_static.plans
    torch.testing.assert_close(fs, fn, rtol=1e-5, atol=1e-6)
    allf = hvd.allgather(fs.unsqueeze(0))
    assert torch.equal(allf[0], allf[1])
    # a rank-dependent gradient list must be refused by the plan check
    from mivod.keras._static import StaticGradientReducer
    red = StaticGradientReducer("Bad", hk.Average, hk.Compression.none)
    gs = [torch.ones(3 + r)]
    try:
        red(gs)
    except RuntimeError as e:
        assert "differ across ranks" in str(e)
    else:
        raise AssertionError("mismatched plans were not detected")
    hvd.shutdown()
    print("OK", r)


def keras_overlap():
    """Keras DistributedOptimizer with the reduction overlapping the backward
    (OverlappedGradientReducer: tensor hooks during autograd.grad -> pack -> comm
    stream): several buckets, most launched INSIDE autograd.grad, one plan, same
    weights as the static (after-backward) reducer, identical on every rank; then
    the TF2-style example (config 2) on it: identical weights, averaged metrics,
    and HOROVOD_TIMELINE collective phases per bucket."""
    import json
    import tempfile

    import numpy as np

    import mivod.keras as hk
    import mivod.kerasfw as keras
    tl = os.path.join(tempfile.mkdtemp(), "timeline.json")
    os.environ["HOROVOD_TIMELINE"] = tl
    os.environ["MIVOD_BUCKET_MB"] = "0.05"            # several buckets for a small model
    os.environ["MIVOD_FIRST_BUCKET_MB"] = "0.01"
    os.environ["MIVOD_LAST_BUCKET_MB"] = "0.01"
    hvd.init()
    r = hvd.rank()
    rng = np.random.default_rng(100 + r)
    xs = rng.standard_normal((6, 16, 32)).astype(np.float32)
    ys = rng.integers(0, 4, (6, 16)).astype(np.int64)

    def train(overlap):
        os.environ["MIVOD_KERAS_OVERLAP"] = "1" if overlap else "0"
        torch.manual_seed(0)
        model = keras.Sequential([keras.layers.Dense(64, activation="relu"),
                                  keras.layers.Dense(64, activation="relu"),
                                  keras.layers.Dense(64, activation="relu"),
                                  keras.layers.Dense(4)])
        opt = hk.DistributedOptimizer(keras.optimizers.SGD(0.1, momentum=0.9))
        model.compile(loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=opt)
        for x, y in zip(xs, ys):
            model.train_on_batch(x, y)
        flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        return flat, opt

    fo, opt_o = train(True)
    fs, opt_s = train(False)
    red = opt_o._hvd_overlap
    assert red.plans == 1 and red.steps == len(xs), (red.plans, red.steps)
    assert len(red.buckets) > 2, len(red.buckets)
    assert red.launched_in_backward >= len(xs) * (len(red.buckets) - 1), \
        (red.launched_in_backward, len(red.buckets))
    assert opt_s._hvd_static.plans == 1 and opt_o._hvd_static.plans == 0
    torch.testing.assert_close(fo.cpu(), fs.cpu(), rtol=1e-5, atol=1e-6)
    allf = hvd.allgather(fo.unsqueeze(0))
    assert torch.equal(allf[0], allf[1])
    # config 2 (TF2-style example) on the overlapped path
    os.environ["MIVOD_KERAS_OVERLAP"] = "1"
    os.environ["MIVOD_BUCKET_MB"] = "1"
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    os.environ["PS_MODEL_PATH"] = tempfile.mkdtemp()
    from keras_mnist_tf2_style import main
    hist, model = main(["--epochs", "2", "--steps", "10"])
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    allf = hvd.allgather(flat.unsqueeze(0))
    assert torch.equal(allf[0], allf[1])
    logs = hvd.allgather_object(hist.history)
    assert logs[0]["loss"] == logs[1]["loss"], logs
    assert model.optimizer._hvd_overlap.steps == 20
    hvd.shutdown()
    from mivod.utils import timeline as TL
    TL.stop_timeline()
    if r == 0:
        ev = json.load(open(tl))
        names = {e.get("name") for e in ev if e.get("ph") == "X"}
        assert names & {"NCCL_ALLREDUCE", "RING_ALLREDUCE"}, names
    print("OK", r)


def gpu_rccl_watchdog():
    """The communicator watchdog: a collective that cannot complete within
    MIVOD_RCCL_TIMEOUT_S (here: queued behind a ~3 s spin kernel) makes the watchdog
    thread abort the communicator (ncclCommAbort); the next collective raises."""
    import time as _t

    from mivod.common import basics as B
    from mivod.parallel import collectives as C
    hvd.init()
    st = B.state()
    assert st.gpu is not None and st.gpu.name == "rccl"
    dev = hvd.device()
    x = torch.ones(4096, device=dev)
    torch.cuda._sleep(int(6e9))            # bounded spin on the current stream
    C.allreduce_(x, C.Sum)                 # its completion event is stuck behind the spin
    t0, err = _t.time(), ""
    while _t.time() - t0 < 30:
        err = st.gpu.comm.error()
        if err:
            break
        _t.sleep(0.1)
    assert "did not complete" in err, err
    try:
        C.allreduce_(x, C.Sum)
    except RuntimeError as e:
        assert "aborted" in str(e), e
    else:
        raise AssertionError("a collective on an aborted communicator did not raise")
    torch.cuda.synchronize()
    print("OK", 0, flush=True)
    os._exit(0)      # the aborted communicator is not destroyed again at exit



if __name__ == "__main__":
    globals()[sys.argv[1]]()
