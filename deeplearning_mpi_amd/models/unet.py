"""UNet (4-level encoder/decoder) on the MI355X engine.

Same module tree, parameter names and defaults as /root/reference/pytorch/unet/model.py:5-81
(``DoubleConv`` = (Conv3x3 with bias -> BN -> ReLU) x 2, ``DownBlock``, ``UpBlock`` with
ConvTranspose2d(k2,s2) or bilinear Upsample, ``conv_last`` 1x1), so checkpoints load both ways.
Extension (BASELINE.json config 5): ``in_channels`` (the reference hard-codes 3).

Engine schedule (MI355X-first):
* the skip concatenation is free: each encoder level's second BN-apply writes the skip tensor
  straight into channel slice [C_up, C_up+C_skip) of the decoder's preallocated concat buffer,
  and the decoder's ConvTranspose2d writes the up-sampled tensor into slice [0, C_up)
  (torch.cat at model.py:47 disappears);
* ConvTranspose2d(k2, s2) is 4 sub-pixel GEMM phases with a strided-store epilogue;
* backward: the concat-buffer gradient is produced by ONE data-gradient GEMM, the skip slice of it
  is added inside the 2x2 max-pool backward kernel (no separate add).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.act import Act, padc
from .engine import ConvTUnit, ConvUnit, EngineModule

# Training forward: each encoder DoubleConv's last BN-apply + ReLU runs inside the 2x2 max-pool that
# reads it, which also stores it as the skip (pool.hip maxpool_fwd_fixed_kernel, ys): one pass over the
# BN input instead of the apply pass plus the pool re-reading its output (profiles/r5_poolapply).
FUSE_POOL_APPLY = True
# Training forward: the last decoder BN-apply + ReLU is applied inside the 1x1 head kernel and the
# head's weight gradient (operand prologue) instead of a stored pass (profiles/r5_poolapply).
FUSE_HEAD_APPLY = True



class DoubleConv(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.double_conv = nn.Sequential(
            nn.Conv2d(in_channels, out_channels, kernel_size=3, padding=1),
            nn.BatchNorm2d(out_channels),
            nn.ReLU(inplace=True),
            nn.Conv2d(out_channels, out_channels, kernel_size=3, padding=1),
            nn.BatchNorm2d(out_channels),
            nn.ReLU(inplace=True),
        )

    def forward(self, x):
        return self.double_conv(x)

    def units(self, ar, cin_pad=None, need_dgrad=True):
        s = self.double_conv
        return (ConvUnit(ar, s[0], s[1], relu=True, cin_pad=cin_pad, need_dgrad=need_dgrad),
                ConvUnit(ar, s[3], s[4], relu=True))


class DownBlock(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.double_conv = DoubleConv(in_channels, out_channels)
        self.down_sample = nn.MaxPool2d(2)

    def forward(self, x):
        skip_out = self.double_conv(x)
        return self.down_sample(skip_out), skip_out


class UpBlock(nn.Module):
    def __init__(self, in_channels, out_channels, up_sample_mode):
        super().__init__()
        if up_sample_mode == "conv_transpose":
            self.up_sample = nn.ConvTranspose2d(in_channels - out_channels, in_channels - out_channels, kernel_size=2,
                                                stride=2)
        elif up_sample_mode == "bilinear":
            self.up_sample = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
        else:
            raise ValueError("Unsupported `up_sample_mode` (can take one of `conv_transpose` or `bilinear`)")
        self.double_conv = DoubleConv(in_channels, out_channels)

    def forward(self, down_input, skip_input):
        x = self.up_sample(down_input)
        x = torch.cat([x, skip_input], dim=1)
        return self.double_conv(x)


class UNet(EngineModule):
    def __init__(self, out_classes=2, up_sample_mode="conv_transpose", in_channels=3):
        super().__init__()
        self.up_sample_mode = up_sample_mode
        self.in_channels = in_channels
        self.out_classes = out_classes
        self.down_conv1 = DownBlock(in_channels, 64)
        self.down_conv2 = DownBlock(64, 128)
        self.down_conv3 = DownBlock(128, 256)
        self.down_conv4 = DownBlock(256, 512)
        self.double_conv = DoubleConv(512, 1024)
        self.up_conv4 = UpBlock(512 + 1024, 512, self.up_sample_mode)
        self.up_conv3 = UpBlock(256 + 512, 256, self.up_sample_mode)
        self.up_conv2 = UpBlock(128 + 256, 128, self.up_sample_mode)
        self.up_conv1 = UpBlock(128 + 64, 64, self.up_sample_mode)
        self.conv_last = nn.Conv2d(64, out_classes, kernel_size=1)

    # ------------------------------------------------------------------ eager torch path
    def forward_torch(self, x):
        x, s1 = self.down_conv1(x)
        x, s2 = self.down_conv2(x)
        x, s3 = self.down_conv3(x)
        x, s4 = self.down_conv4(x)
        x = self.double_conv(x)
        x = self.up_conv4(x, s4)
        x = self.up_conv3(x, s3)
        x = self.up_conv2(x, s2)
        x = self.up_conv1(x, s1)
        return self.conv_last(x)

    # ------------------------------------------------------------------ engine
    def _grad_ready_names(self):
        """Backward order (_engine_backward): the head, each decoder level from the top (its
        DoubleConv's second then first unit, then its ConvTranspose2d), the bottleneck, the
        encoder from the bottom."""
        un = self.unit_ready_names

        def dc(prefix):
            b = f"{prefix}.double_conv"
            return un(f"{b}.3", f"{b}.4", conv_bias=True) + un(f"{b}.0", f"{b}.1", conv_bias=True)

        names = un("conv_last", None, conv_bias=self.conv_last.bias is not None)
        for k in (1, 2, 3, 4):
            names += dc(f"up_conv{k}.double_conv")
            if self.up_sample_mode == "conv_transpose":
                names += un(f"up_conv{k}.up_sample", None, conv_bias=True)
        names += dc("double_conv")
        for k in (4, 3, 2, 1):
            names += dc(f"down_conv{k}.double_conv")
        return names

    def _build_units(self, ar):
        self.cin_pad = padc(self.in_channels)
        downs = [self.down_conv1, self.down_conv2, self.down_conv3, self.down_conv4]
        ups = [self.up_conv1, self.up_conv2, self.up_conv3, self.up_conv4]   # level 1..4
        self.enc = []
        for k, d in enumerate(downs):
            self.enc.append(d.double_conv.units(ar, cin_pad=self.cin_pad if k == 0 else None, need_dgrad=k != 0))
            if k == 0:   # the input DoubleConv's weights recast first; the rest beside its forward
                ar.mark_cast_group()
        self.bott = self.double_conv.units(ar)
        self.skip_ch = [64, 128, 256, 512]
        self.up_ch = [128, 256, 512, 1024]   # channels arriving from below at levels 1..4
        self.dec = [u.double_conv.units(ar, cin_pad=self.up_ch[k] + self.skip_ch[k]) for k, u in enumerate(ups)]
        self.upT = [ConvTUnit(ar, u.up_sample) if self.up_sample_mode == "conv_transpose" else None for u in ups]
        self.u_last = ConvUnit(ar, self.conv_last, None, relu=False)
        # level 1 (64 -> 64): the first conv's BN-apply inside the second conv's streaming kernel
        self.enc[0][1].fuse3 = True
        self.dec[0][1].fuse3 = True

    def _engine_forward(self, x, train, save):
        be = self._be
        N, _, H, W = x.shape
        assert H % 16 == 0 and W % 16 == 0, "UNet input must be a multiple of 16 (reference model.py:71-79)"
        dt, dev = be.act_dtype, x.device
        a = be.nchw_to_nhwc(x, self.cin_pad)
        cats, ctx_enc, idxs, skips = [], [], [], []
        h, w = H, W
        for k in range(4):
            ccat = self.up_ch[k] + self.skip_ch[k]
            cat = Act.empty(N, h, w, ccat, dt, dev)
            cats.append(cat)
            ua, ub = self.enc[k]
            # lazy: the BN-apply may run inside ub (the level-1 64 -> 64 conv: FUSE_APPLY_3X3)
            t, ca = ua.fwd(be, a, train, save=save, lazy=train and save)
            if k == 0:   # the deeper layers' weight recast beside the 64-channel 3x3 conv (compute-bound)
                self._arena.launch_cast()
            skip = cat.slice(self.up_ch[k], self.skip_ch[k])
            down = Act.empty(N, h // 2, w // 2, self.skip_ch[k], dt, dev)
            # (only with the fused BN backward: its data gradient takes the ReLU mask from z, the unfused
            # bn_bwd needs the stored y in the saved context)
            if FUSE_POOL_APPLY and train and save and self.fuse_bn_bwd:
                # the skip's BN-apply runs inside the pool, which stores it (one pass over z, not two)
                z, cb = ub.fwd(be, t, train, out=skip, save=save, defer_apply=True)
                idx = be.maxpool_fwd(z, 2, 2, 0, down, bn=(cb[5], cb[6]), store=skip)
            else:
                _, cb = ub.fwd(be, t, train, out=skip, save=save)
                idx = be.maxpool_fwd(skip, 2, 2, 0, down)
            ctx_enc.append((ca, cb))
            idxs.append(idx)
            skips.append(skip)
            a = down
            h, w = h // 2, w // 2
        ua, ub = self.bott
        t, cba = ua.fwd(be, a, train, save=save)
        a, cbb = ub.fwd(be, t, train, save=save)
        ctx_dec = [None] * 4
        for k in range(3, -1, -1):
            cat = cats[k]
            up = cat.slice(0, self.up_ch[k])
            if self.upT[k] is not None:
                self.upT[k].fwd(be, a, up)
            else:
                be.upsample_fwd(a, up)
            below = a
            ua, ub = self.dec[k]
            t, ca = ua.fwd(be, cat, train, save=save, lazy=train and save)
            # level 1's output is read only by the 1x1 head (forward and weight gradient): never stored
            # (the head's weight gradient rebuilds it in an operand prologue: bf16 backends only)
            head_defer = k == 0 and FUSE_HEAD_APPLY and self.fuse_bn_bwd and getattr(be, "prologue", False)
            a, cb = ub.fwd(be, t, train, save=save, defer_apply="act" if head_defer else False)
            ctx_dec[k] = (below, ca, cb)
        K = self.out_classes
        out = torch.empty(N, H, W, K, dtype=be.dt, device=dev)
        _, cl = self.u_last.fwd(be, a, train, out=Act(out.view(N * H * W, K), N, H, W, K), save=save)
        logits = out.permute(0, 3, 1, 2)
        state = (cats, ctx_enc, idxs, skips, (cba, cbb), ctx_dec, cl) if save else None
        return logits, state

    def _engine_backward(self, state, gout):
        """Reverse schedule.  With ``fuse_bn_bwd`` every data-gradient GEMM whose output is the
        gradient of a BN+ReLU output (inside each DoubleConv, and the 1x1 head into the last
        decoder DoubleConv) masks it and emits that BN's backward partials in its epilogue."""
        be = self._be
        fuse = self.fuse_bn_bwd
        cats, ctx_enc, idxs, skips, (cba, cbb), ctx_dec, cl = state

        def spec(ctx):
            return ConvUnit.fuse_spec(ctx) if fuse else None

        def double_bwd(units, ca, cb, dy, pre=None, need_dx=True, colsum=False):
            ua, ub = units
            out = ub.bwd(be, cb, dy, pre=pre, fuse_next=spec(ca))
            dt_, part = out if fuse else (out, None)
            return ua.bwd(be, ca, dt_, pre=part, need_dx=need_dx, colsum=colsum)

        dl = be.nchw_to_nhwc(gout, self.u_last.Kp)
        out = self.u_last.bwd(be, (cl[0], None), dl, fuse_next=spec(ctx_dec[0][2]))
        da, pre = out if fuse else (out, None)
        for k in range(4):                    # decoder, level 1 (last executed) first
            below, ca, cb = ctx_dec[k]
            up_t = self.upT[k]
            # with a ConvTranspose2d up-sampling, the concat-gradient GEMM also emits its column sums:
            # those of the up-sampling slice are the ConvTranspose bias gradient (no extra pass)
            out = double_bwd(self.dec[k], ca, cb, da, pre=pre, colsum=up_t is not None and up_t.m.bias is not None)
            dcat, cpart = out if isinstance(out, tuple) else (out, None)
            pre = None
            dup = dcat.slice(0, self.up_ch[k])
            if up_t is not None:
                # the ConvTranspose data-gradient is the gradient of the BN+ReLU output below it
                # (the next decoder level's, or the bottleneck's, second conv): masked + partials
                below_ctx = ctx_dec[k + 1][2] if k < 3 else cbb
                out = up_t.bwd(be, below, dup, fuse_next=spec(below_ctx),
                               bias_part=cpart)
                da, pre = out if fuse else (out, None)
            else:
                da = Act.empty(below.N, below.H, below.W, below.C, be.act_dtype, below.device)
                be.upsample_bwd(dup, da)
            ctx_dec[k] = dcat                 # keep the skip-slice gradient for the encoder
        da = double_bwd(self.bott, cba, cbb, da, pre=pre)
        for k in range(3, -1, -1):
            skip = skips[k]
            dskip = Act.empty(skip.N, skip.H, skip.W, skip.C, be.act_dtype, skip.device)
            ca, cb = ctx_enc[k]
            # gradient of the encoder output = pool backward + its skip-concat slice; with the
            # fusion the pool backward also masks it and emits the encoder BN's partials
            part = be.maxpool_bwd(da, idxs[k], skip, 2, 2, 0, dskip,
                                  add=ctx_dec[k].slice(self.up_ch[k], self.skip_ch[k]), fuse=spec(cb))
            da = double_bwd(self.enc[k], ca, cb, dskip, pre=part, need_dx=k != 0)
