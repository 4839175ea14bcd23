"""Model families on CPU (eager fallbacks of the fused ops): BERT pre-training
and ResNet shapes / parameter counts, one training step each, and the
transformer op fallbacks' semantics."""
import torch
import torch.nn.functional as F

from mivod.models.bert import BertConfig, BertForPreTraining, count_params, synthetic_batch
from mivod.models.resnet import resnet50
from mivod.ops.transformer import bias_dropout_add_ln, bias_gelu, dropout_keep_mask


def test_bert_large_parameter_count():
    with torch.device("meta"):
        m = BertForPreTraining(BertConfig.large())
    assert count_params(m) == 336_226_108


def test_resnet50_parameter_count():
    with torch.device("meta"):
        m = resnet50()
    assert count_params(m) == 25_557_032


def test_bert_tiny_trains_on_cpu():
    torch.manual_seed(0)
    c = BertConfig.tiny()
    model = BertForPreTraining(c)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    batch = synthetic_batch(c, 4, 32, "cpu", generator=torch.Generator().manual_seed(0))
    losses = []
    for _ in range(8):
        opt.zero_grad()
        loss = model(*batch)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0]


def test_transformer_fallbacks_match_composition():
    torch.manual_seed(1)
    x = torch.randn(6, 16)
    b = torch.randn(16)
    torch.testing.assert_close(bias_gelu(x, b), F.gelu(x + b))
    ln = torch.nn.LayerNorm(16)
    res = torch.randn(6, 16)
    torch.testing.assert_close(bias_dropout_add_ln(x, b, res, ln, p=0.5, training=False),
                               ln(res + x + b))


def test_dropout_keep_mask_rate_and_determinism():
    k1 = dropout_keep_mask(256, 1024, 0.1, 99)
    k2 = dropout_keep_mask(256, 1024, 0.1, 99)
    k3 = dropout_keep_mask(256, 1024, 0.1, 100)
    assert torch.equal(k1, k2) and not torch.equal(k1, k3)
    assert abs((1 - k1.float().mean().item()) - 0.1) < 0.01


def test_resnet_zero_init_residual_survives_generic_init():
    m = resnet50(zero_init_residual=True)
    assert all(float(b.bn3.weight.abs().sum()) == 0.0 for b in m.modules() if hasattr(b, "bn3"))
    assert float(m.bn1.weight.sum()) == 64.0


def test_gram_stats_formula_with_a_torch_backend():
    """ops.bn._gram_stats' algebra (sum z = W colsum(x), sum z^2 = rowsum((W G) * W), both
    around a shift) with the two native calls replaced by their fp32 torch definitions:
    equals the direct statistics of z = x W^T (the GPU test checks the kernels)."""
    from mivod.ops import bn as B

    class Nat:
        @staticmethod
        def wgrad1x1(x, dy, stride, fp32):
            x2 = x.permute(0, 2, 3, 1).reshape(-1, x.shape[1]).double()
            return (x2.t() @ x2).float().view(x.shape[1], x.shape[1], 1, 1)

        @staticmethod
        def gram_stats(w, g, xsum, shift, m):
            wf = w.double()
            u = wf @ xsum.double()
            q = ((wf @ g.view(w.shape[1], w.shape[1]).double()) * wf).sum(1)
            sh = shift.double()
            return torch.stack((u - m * sh, q - 2 * sh * u + m * sh * sh)).float().unsqueeze(0)

    torch.manual_seed(0)
    x = torch.relu(torch.randn(3, 16, 5, 7) + 0.5).contiguous(memory_format=torch.channels_last)
    w = torch.randn(32, 16) / 4
    shift = torch.randn(32) * 0.2
    m = 3 * 5 * 7
    cs = torch.stack((x.sum((0, 2, 3)) * 0.25, x.sum((0, 2, 3)) * 0.75))   # [P, cin] partials
    part = B._gram_stats(Nat, x, w, cs, shift, m)
    z = x.permute(0, 2, 3, 1).reshape(m, 16).double() @ w.double().t() - shift.double()
    torch.testing.assert_close(part[0, 0].double(), z.sum(0), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(part[0, 1].double(), (z * z).sum(0), rtol=1e-5, atol=1e-4)


def test_fused_stem_path_declines_off_gpu(monkeypatch):
    """models.resnet.stem_bn_relu_maxpool (the fused stem forward/backward) only takes a
    channels_last bf16 224 x 224 GPU image in training mode; elsewhere it returns None and
    the model runs its composed stem."""
    from mivod.models.resnet import ResNet, stem_bn_relu_maxpool
    m = ResNet((1, 1, 1, 1), num_classes=10)
    x = torch.rand(2, 3, 224, 224).contiguous(memory_format=torch.channels_last)
    assert stem_bn_relu_maxpool(m.conv1, m.bn1, m.maxpool, x) is None
    monkeypatch.setenv("MIVOD_STEM_POOL_FUSE", "0")
    assert stem_bn_relu_maxpool(m.conv1, m.bn1, m.maxpool, x) is None
    out = m(torch.rand(2, 3, 64, 64))
    assert out.shape == (2, 10) and torch.isfinite(out).all()
