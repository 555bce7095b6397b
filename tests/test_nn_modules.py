"""Autograd modules over the kernels (splitlearning_amd/nn.py) vs plain torch.nn."""
import pytest
import torch
import torch.nn.functional as F

from splitlearning_amd import nn as snn


def _devices():
    return ["cpu"] + (["cuda"] if torch.cuda.is_available() else [])


def _check_linear(dev, M, K, N, relu):
    torch.manual_seed(0)
    lin = snn.FusedLinear(K, N, relu=relu).to(dev)
    ref = torch.nn.Linear(K, N).to(dev)
    ref.load_state_dict(lin.state_dict())
    x = torch.randn(M, K, device=dev, requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    y = lin(x)
    yr = ref(x2)
    if relu:
        yr = F.relu(yr)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(lin.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(lin.bias.grad, ref.bias.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M,K,N,relu", [(16, 64, 40, True), (5, 30, 7, False), (200, 128, 33, True)])
def test_fused_linear_cpu(M, K, N, relu):
    _check_linear("cpu", M, K, N, relu)


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,N,relu", [(16, 5408, 1000, True), (5, 30, 7, False), (200, 128, 33, True)])
def test_fused_linear_gpu(cuda, M, K, N, relu):
    _check_linear(cuda, M, K, N, relu)


def test_fused_linear_dropout_is_inverted_and_masked():
    lin = snn.FusedLinear(32, 64, relu=True, dropout=0.5, seed=3)
    x = torch.randn(16, 32, requires_grad=True)
    y = lin(x)
    ref = F.relu(F.linear(x, lin.weight, lin.bias))
    kept = y != 0
    frac = kept.float().mean().item() / (ref > 0).float().mean().item()    # dropout keep rate
    assert 0.4 < frac < 0.6
    torch.testing.assert_close(y[kept], 2 * ref[kept], rtol=1e-5, atol=1e-5)
    y.sum().backward()
    assert lin.weight.grad is not None
    lin.eval()
    torch.testing.assert_close(lin(x), ref, rtol=1e-5, atol=1e-5)


def _check_conv(dev):
    torch.manual_seed(1)
    m = snn.FusedConvFront().to(dev)
    conv = torch.nn.Conv2d(1, 32, 3).to(dev)
    conv.load_state_dict({k.split(".", 2)[-1]: v for k, v in m.state_dict().items()})
    x = torch.randint(0, 256, (6, 1, 28, 28), device=dev).float()
    y = m(x)
    yr = F.max_pool2d(F.relu(conv(x)), 2, 2).flatten(1)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-3)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    c = m.conv_layers[0]
    torch.testing.assert_close(c.weight.grad, conv.weight.grad, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(c.bias.grad, conv.bias.grad, rtol=1e-4, atol=1e-3)


def test_fused_conv_front_cpu():
    _check_conv("cpu")


@pytest.mark.gpu
def test_fused_conv_front_gpu(cuda):
    _check_conv(cuda)


@pytest.mark.parametrize("dev", _devices())
def test_softmax_cross_entropy(dev):
    logits = torch.randn(16, 100, device=dev, requires_grad=True)
    labels = torch.randint(0, 10, (16,), device=dev)
    labels[3] = -100
    l2 = logits.detach().clone().requires_grad_(True)
    loss = snn.softmax_cross_entropy(logits, labels)
    ref = F.cross_entropy(l2, labels)
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-5)
    loss.backward()
    ref.backward()
    torch.testing.assert_close(logits.grad, l2.grad, rtol=1e-5, atol=1e-6)
