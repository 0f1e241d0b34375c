"""CPU: the split-K dense autograd functions equal torch's own linear/conv1d (pure torch
code, so it is checkable here)."""
import torch
import torch.nn as nn
import torch.nn.functional as F

import dense


def test_linear_splitk_matches_torch():
    torch.manual_seed(0)
    x = torch.randn(3, 5000, 2, 37, dtype=torch.float64, requires_grad=True)
    lin = nn.Linear(37, 19).double()
    y = dense.linear(x, lin.weight, lin.bias)
    gy = torch.randn_like(y)
    y.backward(gy)
    gx, gw, gb = x.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone()
    x.grad = None
    lin.zero_grad()
    F.linear(x, lin.weight, lin.bias).backward(gy)
    torch.testing.assert_close(gx, x.grad)
    torch.testing.assert_close(gw, lin.weight.grad)
    torch.testing.assert_close(gb, lin.bias.grad)
    assert dense._chunks(30000, 19 * 37) > 1  # the split path was exercised


def test_conv1x1_splitk_matches_torch():
    torch.manual_seed(1)
    x = torch.randn(4, 11, 8192, dtype=torch.float64, requires_grad=True)
    conv = nn.Conv1d(11, 7, 1).double()
    y = dense.conv1x1(x, conv)
    gy = torch.randn_like(y)
    y.backward(gy)
    gx, gw, gb = x.grad.clone(), conv.weight.grad.clone(), conv.bias.grad.clone()
    x.grad = None
    conv.zero_grad()
    conv(x).backward(gy)
    torch.testing.assert_close(gx, x.grad)
    torch.testing.assert_close(gw, conv.weight.grad)
    torch.testing.assert_close(gb, conv.bias.grad)
