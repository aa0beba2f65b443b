"""ResNet-18/34/50/101/152 on the MI355X engine.

Module names, shapes, dtypes and initialisation follow torchvision's ``resnet*`` exactly, so a
``state_dict`` is key-for-key compatible with the reference checkpoints
(/root/reference/pytorch/resnet/main.py:40-41 builds ``torchvision.models.resnet18`` with a
replaced 10-class ``fc``; BASELINE.json targets ResNet-50/152 at 224x224).

Forward/backward run as an explicit engine schedule (models/engine.py): stem conv7x7+BN+ReLU,
maxpool, bottleneck/basic blocks with the residual add and ReLU fused into the last BN-apply,
global average pool and the fc GEMM (fp32 logits).  ``forward_torch`` is the plain eager-PyTorch
path of the same parameters (stock PyTorch baseline and test oracle).
"""
from __future__ import annotations


import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.act import Act, padc
from .engine import PendingApply, BwdFuse, ConvUnit, EngineModule, S2DConvUnit, record_on, resolve


def conv3x3(i, o, stride=1):
    return nn.Conv2d(i, o, 3, stride, 1, bias=False)


def conv1x1(i, o, stride=1):
    return nn.Conv2d(i, o, 1, stride, 0, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward_torch(self, x):
        idn = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + idn)

    def units(self, ar):
        u = [ConvUnit(ar, self.conv1, self.bn1, relu=True), ConvUnit(ar, self.conv2, self.bn2, relu=True)]
        ud = ConvUnit(ar, self.downsample[0], self.downsample[1], relu=False) if self.downsample is not None else None
        return u, ud


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        width = planes
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = conv3x3(width, width, stride)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward_torch(self, x):
        idn = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + idn)

    def units(self, ar):
        u = [ConvUnit(ar, self.conv1, self.bn1, relu=True), ConvUnit(ar, self.conv2, self.bn2, relu=True),
             ConvUnit(ar, self.conv3, self.bn3, relu=True)]
        # 1x1 stride-1 convs: data gradient over [dy | z] without materialising dz (engine.DUAL_DGRAD)
        u[0].dual = u[2].dual = True
        ud = ConvUnit(ar, self.downsample[0], self.downsample[1], relu=False) if self.downsample is not None else None
        return u, ud


# The downsample branch stream is joined right before the residual is first read (the last unit's
# BN-apply in the forward, conv1's data gradient in the backward), and its BN output is applied inside
# the block's last BN-apply (Deferred.bn) instead of a pass of its own (profiles/r2_ds_fuse).
# (Starting the branch after a fused conv1 instead measured slower: profiles/r3_ds_after_conv1_rejected.)
_LATE_JOIN = True
_DS_FUSE = True


class _BlockExec:
    """Forward/backward schedule of one residual block (basic or bottleneck)."""

    def __init__(self, units, ds):
        self.u, self.ud = units, ds

    def fwd(self, be, x: Act, train, save):
        """The downsample branch (1x1 conv + BN) depends only on the block input: with a branch
        stream it runs beside conv1 -> conv2 and joins before the residual add of conv3's BN."""
        ctxs = []
        lazy = train and save   # the block output's BN-apply may run inside its consumer (PendingApply)
        first = None
        if self.ud is not None:   # the branch reads the whole block input
            if isinstance(x, PendingApply) and self.u[0].can_fuse_apply(be, x, train, save):
                # the previous block's BN-apply runs inside conv1 (which stores it); the branch reads
                # the stored output after conv1 instead of both reading a separate apply pass's output
                first = self.u[0].fwd(be, x, train, save=save, lazy=lazy)
            x = resolve(be, x)
        # the downsample BN output is read once, as the residual of the last unit's BN-apply: applied
        # there on the fly (Deferred.bn), which removes its own apply pass (read z_ds + write idn)
        ds_defer = "bn" if (_DS_FUSE and train and save) else False
        br = getattr(be, "branch_stream", None) if self.ud is not None else None
        main = torch.cuda.current_stream() if br is not None else None

        def branch_fwd(xb):
            if br is not None:
                br.wait_stream(main)
                with torch.cuda.stream(br):
                    out = self.ud.fwd(be, xb, train, save=save, defer_apply=ds_defer)
                record_on(br, xb)
                return out
            return self.ud.fwd(be, xb, train, save=save, defer_apply=ds_defer)

        if br is not None:
            idn, cd = branch_fwd(x)
        h = x
        if first is not None:
            h = first[0]
            ctxs.append(first[1])
        for u in self.u[1 if first is not None else 0:-1]:
            h, c = u.fwd(be, h, train, save=save, lazy=lazy)
            ctxs.append(c)
        join = None
        if br is not None:
            def join():   # the residual is first read by the last unit's BN-apply, after its GEMM
                main.wait_stream(br)
                record_on(main, idn, cd)
            if not _LATE_JOIN:
                join()
                join = None
        elif self.ud is not None:
            idn, cd = self.ud.fwd(be, x, train, save=save, defer_apply=ds_defer)
        else:   # identity: the block input, complete once conv1 has consumed it
            idn, cd = resolve(be, x), None
        y, c = self.u[-1].fwd(be, h, train, res=idn, save=save, before_res=join, lazy=lazy)
        ctxs.append(c)
        return y, (ctxs, cd)

    def fuse_spec(self, st):
        """(block output y, BN input of the last conv, BN input of the downsample conv | None): the
        previous schedule step fuses this block's BN-backward reductions into its dgrad epilogue."""
        ctxs, cd = st
        return ConvUnit.fuse_spec(ctxs[-1], z2=cd[1] if cd is not None else None)

    def out_slot(self, st):
        """Where the block-output gradient should be written (the last unit's dy_slot) or None."""
        return self.u[-1].dy_slot(st[0][-1])

    def bwd(self, be, st, dy: Act, pre=None, fuse_prev=None, fuse_inner=False, dx_out=None):
        """dy: gradient of the block output.  With ``pre`` (partials from the producer's dgrad
        epilogue) dy is already ReLU-masked.  With ``fuse_prev`` the block-input gradient is
        produced masked for the previous block and returned with its partials.  dx_out: where to
        write the block-input gradient (the previous block's out_slot)."""
        ctxs, cd = st
        slot = lambda k: self.u[k].dy_slot(ctxs[k])   # noqa: E731
        ylast = ctxs[-1][2]
        n = len(self.u)
        spec = lambda k: ConvUnit.fuse_spec(ctxs[k])   # noqa: E731
        if pre is not None:
            # the masked dy is the identity-path gradient; the downsample BN reads row 2 of `pre`.
            # With a branch stream the downsample backward (BN backward + 1x1 data gradient) runs
            # beside the main branch and joins before conv1's data gradient adds it.
            br = getattr(be, "branch_stream", None) if self.ud is not None else None
            if br is not None:
                main = torch.cuda.current_stream()
                br.wait_stream(main)
                with torch.cuda.stream(br):
                    dres = self.ud.bwd(be, cd, dy, pre=pre, k2=2)
                record_on(br, dy, pre)
            dh, part = self.u[-1].bwd(be, ctxs[-1], dy, pre=pre, k2=1, fuse_next=spec(n - 2), dx_out=slot(n - 2))
            for k in range(n - 2, 0, -1):
                dh, part = self.u[k].bwd(be, ctxs[k], dh, pre=part, fuse_next=spec(k - 1), dx_out=slot(k - 1))
            join = None
            if br is not None:
                def join():   # dres is first read by conv1's data-gradient GEMM, after its BN backward
                    main.wait_stream(br)
                    record_on(main, dres)
                if not _LATE_JOIN:
                    join()
                    join = None
            elif self.ud is not None:
                dres = self.ud.bwd(be, cd, dy, pre=pre, k2=2)
            else:
                dres = dy
            return self.u[0].bwd(be, ctxs[0], dh, dx_res=dres, pre=part, fuse_next=fuse_prev, before_res=join,
                                 dx_out=dx_out)
        # fused BN-backward partials for the inner units also when the block's output gradient comes
        # without them (the last block, behind the average-pool backward); required when their BN +
        # ReLU output was deferred (never stored: ctx y is None), so the mask is recomputed from z
        inner = fuse_inner or any(c[2] is None for c in ctxs[:-1])
        if self.ud is None:
            dyr = Act.empty(dy.N, dy.H, dy.W, dy.C, be.act_dtype, dy.device)   # identity-path grad
            dh = self.u[-1].bwd(be, ctxs[-1], dy, dyr_out=dyr, fuse_next=spec(n - 2) if inner else None,
                                dx_out=slot(n - 2))
        else:
            dyr = None
            dh = self.u[-1].bwd(be, ctxs[-1], dy, fuse_next=spec(n - 2) if inner else None, dx_out=slot(n - 2))
        part = None
        if inner:
            dh, part = dh
        for k in range(n - 2, 0, -1):
            if inner:
                dh, part = self.u[k].bwd(be, ctxs[k], dh, pre=part, fuse_next=spec(k - 1), dx_out=slot(k - 1))
            else:
                dh = self.u[k].bwd(be, ctxs[k], dh, dx_out=slot(k - 1))
        if self.ud is not None:
            # downsample BN sees the same relu-masked output grad as the main branch
            dres = self.ud.bwd(be, cd, dy, ymask=ylast)
        else:
            dres = dyr
        out = self.u[0].bwd(be, ctxs[0], dh, dx_res=dres, pre=part, fuse_next=fuse_prev, dx_out=dx_out)
        return out


class ResNet(EngineModule):
    def __init__(self, block, layers, num_classes=1000, in_channels=3):
        super().__init__()
        self.inplanes = 64
        self.in_channels = in_channels
        self.conv1 = nn.Conv2d(in_channels, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    # ------------------------------------------------------------------ eager torch path
    def forward_torch(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for b in layer:
                x = b.forward_torch(x)
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)

    # ------------------------------------------------------------------ engine
    def _grad_ready_names(self):
        """Backward order (_BlockExec.bwd): fc, then per block (last first) its last conv unit,
        the middle units, the downsample branch (joined before conv1's data gradient), conv1;
        finally the stem."""
        un = self.unit_ready_names
        names = un("fc", None, conv_bias=self.fc.bias is not None)
        for li in (4, 3, 2, 1):
            layer = getattr(self, f"layer{li}")
            for bi in range(len(layer) - 1, -1, -1):
                p = f"layer{li}.{bi}"
                nconv = 3 if isinstance(layer[bi], Bottleneck) else 2
                for k in range(nconv, 1, -1):
                    names += un(f"{p}.conv{k}", f"{p}.bn{k}")
                if layer[bi].downsample is not None:
                    names += un(f"{p}.downsample.0", f"{p}.downsample.1")
                names += un(f"{p}.conv1", f"{p}.bn1")
        return names + un("conv1", "bn1")

    def _build_units(self, ar):
        self.cin_pad = padc(self.in_channels)
        if self.in_channels <= S2DConvUnit.CS:
            # 7x7/s2 stem as a 4x4/s1 conv over a 2x2 space-to-depth image (engine.py:S2DConvUnit)
            self.u_stem = S2DConvUnit(ar, self.conv1, self.bn1, relu=True)
        else:
            self.u_stem = ConvUnit(ar, self.conv1, self.bn1, relu=True, cin_pad=self.cin_pad, need_dgrad=False)
        self.u_stem.wgrad_main = True   # the step's last weight gradient (engine.WGRAD_TAIL_MAIN)
        self.blocks = []
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for b in layer:
                self.blocks.append(_BlockExec(*b.units(ar)))
        self.u_fc = ConvUnit(ar, self.fc, None, relu=False)
        # (no split weight recast, ar.mark_cast_group: on the side stream beside the stem conv or beside
        # layer 1 it slowed those memory-heavy kernels by as much as it saved or more, profiles/r6_recast)

    def _engine_forward(self, x, train, save):
        be = self._be
        N = x.shape[0]
        a0 = self.u_stem.prep_input(be, x)
        # training with the fused BN backward: the stem BN-apply + ReLU runs inside the max-pool
        # (h is then the BN input z; the backward needs only z, scale and shift)
        defer = train and save and self.fuse_bn_bwd and self.bn1 is not None
        h, cs = self.u_stem.fwd(be, a0, train, save=save, defer_apply=defer)
        OH, OW = (h.H + 2 - 3) // 2 + 1, (h.W + 2 - 3) // 2 + 1
        p = Act.empty(N, OH, OW, h.C, be.act_dtype, x.device)
        idx = be.maxpool_fwd(h, 3, 2, 1, p, bn=(cs[5], cs[6]) if defer else None)
        st_blocks = []
        a = p
        for blk in self.blocks:
            a, st = blk.fwd(be, a, train, save)
            st_blocks.append(st)
        a = resolve(be, a)
        pooled = Act.empty(N, 1, 1, a.C, be.act_dtype, x.device)
        be.avgpool_fwd(a, pooled)
        K = self.fc.out_features
        logits = torch.empty(N, K, dtype=be.dt, device=x.device)
        la = Act(logits, N, 1, 1, K)
        _, cf = self.u_fc.fwd(be, pooled, train, out=la, save=save)
        state = (cs, h, p, idx, st_blocks, a, pooled, cf) if save else None
        return logits, state

    def _engine_backward(self, state, gout):
        be = self._be
        cs, h, p, idx, st_blocks, a, pooled, cf = state
        N, K = gout.shape
        dl = be.nchw_to_nhwc(gout.reshape(N, K, 1, 1), self.u_fc.Kp)
        x_fc, _ = cf
        dpool = self.u_fc.bwd(be, (x_fc, None), dl)
        da = Act.empty(a.N, a.H, a.W, a.C, be.act_dtype, a.device)
        be.avgpool_bwd(dpool, da)
        pre = None
        for i in range(len(self.blocks) - 1, -1, -1):
            fuse_prev = self.blocks[i - 1].fuse_spec(st_blocks[i - 1]) if (i > 0 and self.fuse_bn_bwd) else None
            out = self.blocks[i].bwd(be, st_blocks[i], da, pre=pre, fuse_prev=fuse_prev, fuse_inner=self.fuse_bn_bwd,
                                     dx_out=self.blocks[i - 1].out_slot(st_blocks[i - 1]) if i > 0 else None)
            da, pre = out if fuse_prev is not None else (out, None)
        dh = Act.empty(h.N, h.H, h.W, h.C, be.act_dtype, h.device)
        if self.fuse_bn_bwd:   # stem BN-backward statistics in the max-pool backward (mask from z)
            part = be.maxpool_bwd(da, idx, h, 3, 2, 1, dh, fuse=ConvUnit.fuse_spec(cs))
            self.u_stem.bwd(be, cs, dh, need_dx=False, pre=part)
        else:
            be.maxpool_bwd(da, idx, h, 3, 2, 1, dh)
            self.u_stem.bwd(be, cs, dh, need_dx=False)


def resnet18(num_classes=1000, **kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, **kw)


def resnet34(num_classes=1000, **kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes, **kw)


def resnet50(num_classes=1000, **kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, **kw)


def resnet101(num_classes=1000, **kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes, **kw)


def resnet152(num_classes=1000, **kw):
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes, **kw)


ARCHS = {"resnet18": resnet18, "resnet34": resnet34, "resnet50": resnet50, "resnet101": resnet101,
         "resnet152": resnet152}
