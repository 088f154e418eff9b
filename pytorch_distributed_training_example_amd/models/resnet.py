"""ResNet (v1.5, torchvision-compatible) for the ResNet-50 north-star config.

Not in the reference (its only model is LeNet, /root/reference/cnn.py); BASELINE.json's headline
metric is ResNet-50 DDP images/sec. Parameter and buffer names match
``torchvision.models.resnet50`` exactly (``conv1``, ``bn1``, ``layer{1-4}.{i}.conv{1,2,3}``,
``bn{1,2,3}``, ``downsample.{0,1}``, ``fc``) so checkpoints interchange; torchvision itself is
not needed at run time.

MI355X-first layout: the model runs channels_last (NHWC) so every convolution is an
implicit GEMM with C contiguous (MIOpen / hipBLASLt MFMA kernels) and every BatchNorm is the
fused NHWC bf16 HIP kernel (ops/batchnorm.py). ReLU is fused into bn1/bn2, and the bottleneck
tail ``relu(bn3(conv3) + identity)`` is ONE kernel.
"""
from __future__ import annotations

import os
from typing import List, Optional, Type

import torch
from torch import nn

from ..ops.batchnorm import BatchNorm2d, BNGradLink, ResidualGradLink
from ..config import SW
from ..ops._native import disabled as native_disabled
from ..ops.conv import Conv1x1, SplitConv2d, linked_conv, prepare_weights, stem_block
from ..ops.linear import Linear


def conv3x3(inp: int, out: int, stride: int = 1, groups: int = 1, dilation: int = 1) -> nn.Conv2d:
    cls = SplitConv2d if _norm_kind[0] == "pdt" else nn.Conv2d  # ours: weight grad on a side stream
    return cls(inp, out, 3, stride=stride, padding=dilation, groups=groups, bias=False, dilation=dilation)


def conv1x1(inp: int, out: int, stride: int = 1) -> nn.Conv2d:
    if _norm_kind[0] == "pdt":  # our path: autotuned MIOpen / hipBLASLt GEMM (ops/conv.py)
        return Conv1x1(inp, out, stride)
    return nn.Conv2d(inp, out, 1, stride=stride, bias=False)


class _Downsample(nn.Sequential):
    """conv1x1 + BN (no ReLU); indices 0/1 as in torchvision."""


_NORM = {"pdt": BatchNorm2d, "torch": nn.BatchNorm2d}
RESIDUAL_GRAD_LINK = [True]  # identity-block residual gradient accumulated in conv1's dgrad GEMM
DS_MASKED_GRAD = [True]  # downsample blocks: bn3 hands the shortcut gradient to the shortcut BN as (dy, mask)
# downsample blocks: the shortcut BN's apply is deferred into bn3's (a_ds x_ds + b_ds added there):
# its output is never written (+0.9 % ResNet-50, in-process A/B at 512/GPU). Skipped automatically
# when the shortcut BN has forward hooks (they must see its real output)
DS_DEFER_APPLY = [os.environ.get("PDT_DS_DEFER", "1") != "0"]
# the shortcut BN's backward apply deferred into the shortcut conv's fused backward (where its shape allows)
DS_FUSED_BWD = [os.environ.get("PDT_DS_FUSED_BWD", "1") != "0"]
_norm_kind = ["pdt"]
# the backward weight transforms of all convs (1x1 W^T, 3x3 flips) made in one launch at the start of the
# training forward (csrc/kernels/weight_prep.hip) instead of 53 per-conv launches in the backward
PREP_WEIGHTS = [os.environ.get("PDT_PREP_WEIGHTS", "1") != "0"]


def _bn(c: int, fused_relu: bool = False) -> nn.Module:
    if _norm_kind[0] == "pdt":
        return BatchNorm2d(c, fused_relu=fused_relu)
    return nn.BatchNorm2d(c)


def _bn_trains(bn: nn.Module) -> bool:
    """``bn`` is our BatchNorm and will take batch_norm_act's training (batch-statistics) path."""
    return isinstance(bn, BatchNorm2d) and (bn.training or not bn.track_running_stats)


def bn_act(bn: nn.Module, x, residual=None, relu: bool = False):
    """relu?(bn(x) + residual?) — one fused kernel for our BN, three ops for torch's."""
    if isinstance(bn, BatchNorm2d):
        return bn(x, residual=residual, relu=relu)
    y = bn(x)
    if residual is not None:
        y = y + residual
    return torch.relu(y) if relu else y


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = _bn(planes, fused_relu=True)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = _bn(planes)
        self.downsample = downsample
        self.stride = stride
        # >= 2: this block's output also feeds the next stage's strided 1x1 shortcut — its bn3 apply writes that
        # subsample too (set by ResNet; the shortcut's gather pass never runs)
        self.emit_sub = 0

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = bn_act(self.bn1, self.conv1(x), relu=True)
        return bn_act(self.bn2, self.conv2(out), residual=identity, relu=True)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = _bn(width, fused_relu=True)
        self.conv2 = conv3x3(width, width, stride, groups, dilation)
        self.bn2 = _bn(width, fused_relu=True)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = _bn(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride
        # >= 2: this block's output also feeds the next stage's strided 1x1 shortcut — its bn3 apply writes that
        # subsample too (set by ResNet; the shortcut's gather pass never runs)
        self.emit_sub = 0

    def forward(self, x):
        # The linked path needs bn3 on its native kernel (bf16): only that path deposits the shortcut
        # gradient into the link. With any other BatchNorm path conv1's backward would find the link
        # empty, park its dx there for a partner that never comes, and the conv1 branch's gradient
        # would be lost (fp32 ResNet-50 on the GPU lost it in every block until round 5).
        # The BatchNorms that deposit into the links must run batch_norm_act's training path (a frozen /
        # eval-mode BN runs _BNEvalFn, which returns the shortcut gradient through autograd instead).
        ds_bn0 = self.downsample[1] if self.downsample is not None else None
        if (RESIDUAL_GRAD_LINK[0] and self.training and x.requires_grad and torch.is_grad_enabled()
                and x.dtype == torch.bfloat16 and not native_disabled()
                and isinstance(self.conv1, Conv1x1) and _bn_trains(self.bn3)
                and (ds_bn0 is None or not isinstance(ds_bn0, BatchNorm2d) or _bn_trains(ds_bn0))
                and self.conv1.gemm_eligible(x) and x.shape[1] % 64 == 0):
            # the two gradients of x (conv1 branch, shortcut) meet in conv1's data-gradient GEMM
            # (beta = 1) instead of an autograd add kernel (ops/batchnorm.py ResidualGradLink)
            # identity blocks: bn3's backward may hand the shortcut gradient over as (dy, mask); conv1's
            # backward always runs after bn3's there (consumer_last: never parks its dx)
            link = ResidualGradLink(lazy=self.downsample is None and self.conv1.masked_residual_ok(x),
                                    consumer_last=self.downsample is None)
            out = bn_act(self.bn1, self.conv1(x, res_link=link), relu=True)
            z2 = self.conv2(out)  # same shape / layout as bn2's output: decides conv3's paths
            ds_bn = self.downsample[1] if self.downsample is not None else None
            # conv3 + bn3 backward as one kernel: bn3 hands its input gradient to conv3 in deferred form
            # (or the ALG backward for the shapes the fused kernel does not take: ops/conv.py _bwd_alg)
            alg3 = self.conv3.alg_bwd_ok(z2)
            fused3 = self.conv3.fused_bwd_ok(z2) and not (SW.bwd_alg_first and SW.bwd_alg >= 2 and alg3)
            blink = BNGradLink(needs_masked=not fused3) if ((fused3 or alg3) and not self.bn3.has_hooks()
                                     and (link.lazy or (isinstance(ds_bn, BatchNorm2d) and DS_MASKED_GRAD[0]))) \
                else None
            if (blink is not None and fused3 and SW.bn2_defer and isinstance(self.bn2, BatchNorm2d)
                    and not self.bn2.has_hooks()):
                # bn2 -> conv3: statistics only here; conv3's GEMM reads relu(a z2 + b) on load and its fused
                # backward recomputes that operand (ops/batchnorm.py DeferredReLUBN): bn2's output never exists
                out = self.bn2._forward_deferred_relu(z2)
            else:
                out = bn_act(self.bn2, z2, relu=True)
            out = self.conv3(out, bwd_link=blink)
            if self.downsample is None:  # identity: bn3's backward deposits the shortcut gradient
                return self.bn3(out, residual=x, relu=True, res_link=link, out_link=blink, sub_stride=self.emit_sub)
            # shortcut built AFTER the main branch so its backward nodes run first (higher
            # autograd sequence numbers): the shortcut conv deposits, conv1 accumulates. Either
            # order is correct (whichever branch finishes second adds), this one saves a pass.
            if isinstance(ds_bn, BatchNorm2d) and DS_MASKED_GRAD[0]:
                # bn3's backward hands the shortcut gradient to the downsample BN as (dy, ReLU mask):
                # the masked copy dres is never written
                glink = ResidualGradLink(lazy=True)
                dconv = self.downsample[0]
                # the shortcut conv's backward as one fused kernel too (layer 1's stride-1 256x64 shortcut):
                # ds_bn hands it (dy, x, mask, coefficients) and never writes its input gradient
                # or the shortcut conv + BN on the ALG backward (PDT_DS_ALG: ops/batchnorm.py _alg_ds_prelude) when
                # bn3 runs it too (bn3's bias gradient is the shortcut BN's sum(g): same output gradient)
                ds_ok = DS_DEFER_APPLY[0] and not ds_bn.has_hooks() and isinstance(dconv, Conv1x1)
                if ds_ok and blink is not None and not fused3 and dconv.ds_alg_ok(x):
                    dlink = BNGradLink(needs_masked=True)
                elif ds_ok and DS_FUSED_BWD[0] and dconv.fused_bwd_ok(x):
                    dlink = BNGradLink()
                else:
                    dlink = None
                xs = linked_conv(dconv, x, link, bwd_link=dlink)
                if DS_DEFER_APPLY[0] and not ds_bn.has_hooks():
                    # statistics only: an internal DeferredBNOutput handle that only bn3's fused
                    # apply consumes (a_ds x_ds + b_ds added there, the shortcut output never written)
                    identity = ds_bn._forward_stats_only(xs, grad_link=glink, out_link=dlink)
                else:
                    identity = ds_bn(xs, grad_link=glink)
                return self.bn3(out, residual=identity, relu=True, res_link=glink, out_link=blink,
                                sub_stride=self.emit_sub)
            identity = bn_act(ds_bn, linked_conv(self.downsample[0], x, link))
            return bn_act(self.bn3, out, residual=identity, relu=True)  # (blink unused: conv3 gets a dense gy)
        identity = x if self.downsample is None else self.downsample(x)
        out = bn_act(self.bn1, self.conv1(x), relu=True)
        out = bn_act(self.bn2, self.conv2(out), relu=True)
        return bn_act(self.bn3, self.conv3(out), residual=identity, relu=True)


class ResNet(nn.Module):
    def __init__(self, block: Type[nn.Module], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = False, groups: int = 1, width_per_group: int = 64,
                 norm: str = "pdt"):
        super().__init__()
        _norm_kind[0] = norm
        self.inplanes = 64
        self.dilation = 1
        self.groups = groups
        self.base_width = width_per_group
        stem = SplitConv2d if norm == "pdt" else nn.Conv2d
        self.conv1 = stem(3, self.inplanes, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = _bn(self.inplanes, fused_relu=True)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        # ours: the head's bias gradient on the colsum kernel (ops/linear.py Linear: aten's reduction
        # there replays wrong under hipGraph capture at 1024/GPU)
        # (PDT_HEAD_COLSUM=0: aten's nn.Linear, for A/B)
        head = Linear if norm == "pdt" and os.environ.get("PDT_HEAD_COLSUM", "1") != "0" else nn.Linear
        self.fc = head(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        _norm_kind[0] = "pdt"
        # a stage's last block writes the stride-2 subsample the next stage's strided 1x1 shortcut reads
        stages = [self.layer1, self.layer2, self.layer3, self.layer4]
        for prev, nxt in zip(stages[:-1], stages[1:]):
            ds = getattr(nxt[0], "downsample", None)
            if (isinstance(prev[-1], Bottleneck) and ds is not None and isinstance(ds[0], Conv1x1)
                    and ds[0].stride[0] > 1 and ds[0].stride[0] == ds[0].stride[1]):
                prev[-1].emit_sub = ds[0].stride[0]
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = _Downsample(conv1x1(self.inplanes, planes * block.expansion, stride),
                                     _bn(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width))
        return nn.Sequential(*layers)

    def _prep_convs(self):
        """The convs whose data gradients read transformed weights (1x1: W^T, 3x3: flipped)."""
        convs = getattr(self, "_pdt_prep_convs", None)
        if convs is None:
            convs = [m for m in self.modules() if isinstance(m, (Conv1x1, SplitConv2d)) and m is not self.conv1
                     and m.kernel_size in ((1, 1), (3, 3))]
            self._pdt_prep_convs = convs
        return convs

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if (PREP_WEIGHTS[0] and self.training and torch.is_grad_enabled() and x.is_cuda
                and x.dtype == torch.bfloat16 and not native_disabled()):
            # every conv's backward weight transform for this step, in one launch (ops/conv.py)
            prepare_weights(self._prep_convs())
        y = stem_block(self.conv1, self.bn1, x)  # one node: the BN's backward apply goes into the wgrad
        if y is not None:
            x = y
        elif hasattr(self.bn1, "forward_relu_maxpool"):  # fused BN+ReLU+pool: stem output never stored
            x = self.bn1.forward_relu_maxpool(self.conv1(x))
        else:
            x = self.maxpool(bn_act(self.bn1, self.conv1(x), relu=True))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if x.is_cuda and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] > 1:
            from ..ops.batchnorm import grad_stats_source_of
            x = _GlobalAvgPoolFn.apply(x, grad_stats_source_of(x) if self.training and torch.is_grad_enabled() else None)
        else:
            x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


class _GlobalAvgPoolFn(torch.autograd.Function):
    """Global average pool of a channels_last [N, C, H, W] tensor -> [N, C]. Its backward writes the
    broadcast gradient straight into a channels_last tensor: nn.AdaptiveAvgPool2d's backward made
    an NCHW gradient that the channels_last BatchNorm backward then had to transpose (a 166 us
    copy + 37 us scale of the [512, 2048, 7, 7] gradient per ResNet-50 step, profiles/r2). On the GPU the
    gradient is written by our kernel (batchnorm.hip gap_bwd_kernel, ``PDT_GAP_NATIVE``), which also takes the
    pooled BatchNorm's backward reduction."""

    @staticmethod
    def forward(ctx, x, gsrc=None):
        ctx.shape = x.shape
        ctx.gsrc = gsrc  # x is a BatchNorm output: our gradient kernel can take that BN's backward reduction
        return x.mean(dim=(2, 3))

    @staticmethod
    def backward(ctx, gy):
        n, c, h, w = ctx.shape
        if (gy.dtype == torch.bfloat16 and gy.is_cuda and c % 8 == 0 and SW.gap_native
                and not native_disabled()):
            from ..ops._native import native
            gs = ctx.gsrc if (ctx.gsrc is not None and ctx.gsrc.ready()) else None
            r = native().gap_bwd(gy.contiguous(), h, w, **(gs.bn_kwargs() if gs else {}))
            if gs is not None and len(r) == 2:  # the last bn3's backward skips its reduce pass
                gs.deposit(r[1], r[0], masked=gs.mask is not None, sum_only=gs.sum_only)
            return r[0], None
        g = (gy * (1.0 / (h * w))).view(n, c, 1, 1).expand(n, c, h, w)
        return g.contiguous(memory_format=torch.channels_last), None


def resnet18(**kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet50(**kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)
