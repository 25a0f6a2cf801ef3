"""A ResNet-style conv-net tenant (torch.nn, hand-built: torchvision is not in
the image) and its pod-server program.

``ResNet`` is the ResNet-18/34 topology -- 7x7/2 stem + BN + ReLU + 3x3/2
max-pool, four stages of BasicBlocks (3x3 conv-BN-ReLU, 3x3 conv-BN, the
identity or a 1x1/2 conv-BN projection added, ReLU), global average pool,
fc -- with random-init weights and perturbed BatchNorm statistics (so BN
folding is exercised, not multiplied by ones).  :func:`resnet_tenant`
exports it with :func:`nos_amd.podserver.export.export`; on the server every
conv + BN (+ residual) (+ ReLU) becomes ONE implicit-GEMM h3 kernel
(ops.tenant.conv2d).
"""
from __future__ import annotations

import torch
import torch.nn as nn


class BasicBlock(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu1 = nn.ReLU()
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))
        self.relu2 = nn.ReLU()

    def forward(self, x):
        y = self.relu1(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        idn = x if self.down is None else self.down(x)
        return self.relu2(y + idn)


class ResNet(nn.Module):
    def __init__(self, layers=(2, 2, 2, 2), widths=(64, 128, 256, 512), num_classes: int = 1000):
        super().__init__()
        self.stem = nn.Conv2d(3, widths[0], 7, 2, 3, bias=False)
        self.bn = nn.BatchNorm2d(widths[0])
        self.relu = nn.ReLU()
        self.pool = nn.MaxPool2d(3, 2, 1)
        blocks = []
        cin = widths[0]
        for i, (n, w) in enumerate(zip(layers, widths)):
            for j in range(n):
                blocks.append(BasicBlock(cin, w, 2 if (j == 0 and i > 0) else 1))
                cin = w
        self.blocks = nn.Sequential(*blocks)
        self.avg = nn.AdaptiveAvgPool2d(1)
        self.flat = nn.Flatten()
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        x = self.pool(self.relu(self.bn(self.stem(x))))
        x = self.blocks(x)
        return self.fc(self.flat(self.avg(x)))

    @torch.no_grad()
    def randomize(self, seed: int = 0) -> "ResNet":
        """Random init with non-trivial BatchNorm statistics and affine terms."""
        g = torch.Generator().manual_seed(seed)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                fan = m.weight[0].numel()
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / fan) ** 0.5)
            elif isinstance(m, nn.BatchNorm2d):
                c = m.num_features
                m.weight.copy_(1 + 0.1 * torch.randn(c, generator=g))
                m.bias.copy_(0.1 * torch.randn(c, generator=g))
                m.running_mean.copy_(0.1 * torch.randn(c, generator=g))
                m.running_var.copy_(1 + 0.2 * torch.rand(c, generator=g))
            elif isinstance(m, nn.Linear):
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) / m.in_features ** 0.5)
                m.bias.copy_(0.01 * torch.randn(m.bias.shape, generator=g))
        return self.eval()


def resnet18(num_classes: int = 1000, seed: int = 0) -> ResNet:
    return ResNet((2, 2, 2, 2), (64, 128, 256, 512), num_classes).randomize(seed)


def resnet_tiny(seed: int = 0) -> ResNet:
    """The tests' small variant (2 stages, narrow)."""
    return ResNet((1, 1), (16, 32), num_classes=10).randomize(seed)


def resnet_tenant(dtype: str = "fp32", seed: int = 0, small: bool = True, hw: tuple[int, int] = (224, 224),
                  batch: int = 1) -> tuple[dict, bytes]:
    """(program, weights) of the conv-net tenant: ResNet-18 on a
    ``[batch, 3, *hw]`` image (``small=False``: the tiny test variant at 32x32)."""
    from ..podserver.export import export

    m = resnet18(seed=seed) if small else resnet_tiny(seed)
    hw = hw if small else (32, 32)
    name = f"resnet18-{dtype}" if small else f"resnet-tiny-{dtype}"
    return export(m, torch.zeros(batch, 3, *hw), name=name, dtype=dtype)


__all__ = ["ResNet", "BasicBlock", "resnet18", "resnet_tiny", "resnet_tenant"]
