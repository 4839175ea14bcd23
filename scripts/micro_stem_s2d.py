"""Microbenchmark: ResNet-50 stem (7x7/2, 4 -> 64, NHWC bf16) as is vs as a space-to-depth
4x4/1 conv on 16 channels (x_pad[c, 2s+p, 2t+q] -> X[(p, q, c), s, t]; W padded to 8x8 ->
W'[o, (p, q, c), a, b] = W[o, c, 2a+p, 2b+q]) — fwd and fwd+wgrad, MIOpen find NORMAL."""
import os
import time

import torch
import torch.nn.functional as F

os.environ.setdefault("MIOPEN_FIND_MODE", "NORMAL")
dev = torch.device("cuda")
N = int(os.environ.get("BS", 2048))
C = 4


def bench(fn, iters=8):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def s2d_input(x):          # [N, C, 224, 224] channels_last -> [N, 4C, 115, 115] channels_last
    xn = F.pad(x.permute(0, 2, 3, 1), (0, 0, 3, 3, 3, 3))          # NHWC, 230 x 230
    n, h, w, c = xn.shape
    xs = xn.view(n, h // 2, 2, w // 2, 2, c).permute(0, 1, 3, 2, 4, 5).reshape(n, h // 2, w // 2, 4 * c)
    return xs.permute(0, 3, 1, 2)


def s2d_weight(w):         # [O, C, 7, 7] -> [O, 4C, 4, 4]
    o, c = w.shape[:2]
    wp = F.pad(w, (0, 1, 0, 1))
    return wp.view(o, c, 4, 2, 4, 2).permute(0, 3, 5, 1, 2, 4).reshape(o, 4 * c, 4, 4).contiguous(
        memory_format=torch.channels_last)


x = torch.rand(N, C, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
x[:, 3] = 0
w = (torch.randn(64, C, 7, 7, device=dev) * 0.05).to(torch.bfloat16).contiguous(
    memory_format=torch.channels_last).requires_grad_()
gy = torch.randn(N, 64, 112, 112, device=dev, dtype=torch.bfloat16).contiguous(
    memory_format=torch.channels_last)

y0 = F.conv2d(x, w, stride=2, padding=3)
xs = s2d_input(x)
y1 = F.conv2d(xs, s2d_weight(w))
print("shapes", tuple(y0.shape), tuple(y1.shape), "max|diff|", float((y0.float() - y1.float()).abs().max()),
      "max|y|", float(y0.float().abs().max()), flush=True)
y0.backward(gy)
g0 = w.grad.clone()
w.grad = None
F.conv2d(xs, s2d_weight(w)).backward(gy)
print("wgrad rel diff", float((w.grad.float() - g0.float()).norm() / g0.float().norm()), flush=True)


def a_fwd():
    return F.conv2d(x, w, stride=2, padding=3)


def a_all():
    F.conv2d(x, w, stride=2, padding=3).backward(gy)


def b_fwd():
    return F.conv2d(s2d_input(x), s2d_weight(w))


def b_all():
    F.conv2d(s2d_input(x), s2d_weight(w)).backward(gy)


def b_in():
    return s2d_input(x).contiguous(memory_format=torch.channels_last)


print(f"7x7/2 C4 : fwd {bench(a_fwd):8.1f} us  fwd+wgrad {bench(a_all):8.1f} us", flush=True)
print(f"s2d 4x4 C16: fwd {bench(b_fwd):8.1f} us  fwd+wgrad {bench(b_all):8.1f} us  (input s2d alone {bench(b_in):7.1f} us)", flush=True)
