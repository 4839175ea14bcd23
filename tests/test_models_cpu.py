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
