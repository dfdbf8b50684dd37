"""Implicit-GEMM convolutions with fused BatchNorm for the ResNet-50 bottleneck
(csrc/kernels/convgemm.hip).

A bottleneck block -- conv1x1 -> BN -> ReLU -> conv3x3 -> BN -> ReLU -> conv1x1 -> BN (+ identity
or downsample conv1x1 -> BN) -> ReLU -- runs as ONE autograd Function whose 1x1 layers are our
MFMA GEMMs with the neighbouring BatchNorm passes folded into them:

  forward   z1 = conv1(x)            + bn1 statistics        (GEMM epilogue)
            y1 = relu(bn1(z1))                               (one apply pass)
            z2 = conv2(y1)           + bn2 statistics        (GEMM epilogue)
            z3 = conv3(relu(bn2(z2))) + bn3 statistics       (bn2 + ReLU in the GEMM prologue:
                                                              bn2's output is never written)
            zd = downsample(x)       + bn_d statistics       (stride-2 rows gathered in-kernel)
            out = relu(bn3(z3) + x  or  bn_d(zd))            (one pass)
  backward  bn3 backward (ReLU mask from 1-bit-per-element output bits); the masked gradient is
            also the identity-branch gradient, recomputed from (dout, bits) where consumed
            conv3 data grad -> ReLU mask + bn2 backward sums (GEMM epilogue), conv3 weight grad
            with relu(bn2(z2)) recomputed in the GEMM prologue, bn2 apply
            conv2 data grad -> ReLU mask + bn1 backward sums (GEMM epilogue; stride 2 as four
            phase GEMMs), weight grad (wide split-K kernel from 256 channels, the patch kernel
            at 64 / 128: no MIOpen solver left)
            conv1 data grad + identity (dout masked by the bits) / downsample gradient (GEMM
            epilogue), weight grads.

Across blocks: block i's conv1 data-grad epilogue also runs block i-1's bn3 backward reduce
(epilogues 6/7/8: mask by block i-1's output bits, sums against its z3), so block i-1's bn3
backward is one apply pass -- or, at 256 channels, no pass at all: block i-1's conv3 data-grad GEMM
applies it while staging its A tile from (gradient, z3) and stores dz3 for the weight gradient.  The hand-off is a ``_Link`` set up in forward when block i's input
IS block i-1's output; block i-1 uses the partials only if the gradient it receives is exactly
the tensor block i produced (same storage, same version) -- any other consumer of the block
output makes autograd sum into a different tensor and the plain reduce runs instead.

Per block that removes the statistics passes of bn1 / bn3 / bn_d, bn2's output write + re-read,
bn2's backward reduce pass and the residual-gradient add, and replaces MIOpen's 1x1 solvers (and
their zero-fill / cast side kernels).  Anything else -- CPU tensors, eval mode, fp32, channel
counts that are not multiples of 64 -- runs the module-by-module path, which is also the numerics
oracle in tests/test_convgemm_gpu.py.  ``PS_AMD_DISABLE=fused_block`` turns the fused path off
(ps_amd/knobs.py).
"""
from __future__ import annotations

import contextlib
import threading
import weakref
from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import knobs
from . import side_stream as _side
from ._ext import native


def rows(x: torch.Tensor) -> torch.Tensor:
    """NCHW channels_last tensor -> its [N*H*W, C] row view (a copy only if not channels_last)."""
    n, c, h, w = x.shape
    if not x.is_contiguous(memory_format=torch.channels_last):
        x = x.contiguous(memory_format=torch.channels_last)
    return x.permute(0, 2, 3, 1).reshape(n * h * w, c)


def image(y2: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
    """[N*H*W, C] rows -> NCHW channels_last view."""
    return y2.view(n, h, w, -1).permute(0, 3, 1, 2)


def geo(h: int, w: int, ks: int = 1, stride: int = 1, pad: int = 0) -> List[int]:
    """Geometry vector [H, W, OH, OW, ks, stride, pad] of a square-kernel NHWC convolution."""
    return [h, w, (h + 2 * pad - ks) // stride + 1, (w + 2 * pad - ks) // stride + 1, ks, stride, pad]


def conv_gemm(a, b, g, pro=None, epi=0, aux=None, kshift=None, mc=None, mean=None, invstd=None, bits=None):
    """c [M, N] = epilogue(sum_k f(a[src(m, k)]) b[n, k]) -> (c, folded BN partials [2, G, N] or None).

    a: [images*H*W, C] bf16 rows; b: [N, ks*ks*C] (channels_last weight order; a strided view is
    copied contiguous once); g: ``geo(...)``;
    pro: [scale | shift] applied with ReLU to ``a`` while staging; epi: 0 store, 1 + BN statistics
    (about ``kshift``), 2 + ``aux`` rows, 3 ReLU mask from ``aux`` * mc + shift and BN-backward sums,
    4 + ``aux`` of the stride-2 map at even (h, w), 5 + ``aux`` masked by ReLU ``bits``."""
    return native().conv_gemm(a, b, g, pro, epi, aux, kshift, mc, mean, invstd, bits)


def conv_wgrad(dz, x, g, pro=None):
    """dW [N, ks*ks*C] bf16 = sum_m dz[m]^T f(x[src(m, k)])."""
    return native().conv_wgrad(dz, x, g, pro)


def _momentum(bn: nn.BatchNorm2d) -> float:
    return float(bn.momentum if bn.momentum is not None else 0.1)


def _finalize(part, kshift, nrows, bn):
    return native().bn_finalize_sums(part, kshift, nrows, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                     _momentum(bn), float(bn.eps))


def _mat(w: torch.Tensor) -> torch.Tensor:
    """1x1 conv weight [N, C, 1, 1] -> [N, C] view."""
    return w.reshape(w.shape[0], w.shape[1])


def _mat3(w: torch.Tensor) -> torch.Tensor:
    """3x3 conv weight [N, C, 3, 3] -> [N, 9C] in (kh, kw, c) order (a view for channels_last)."""
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)


def _mat3_dgrad(w: torch.Tensor) -> torch.Tensor:
    """The weight of the stride-1 3x3 data gradient as a forward conv over dz: wt[c][kh][kw][n] =
    w[n][c][2 - kh][2 - kw] -> [C, 9N]."""
    return w.flip(2, 3).permute(1, 2, 3, 0).reshape(w.shape[1], -1)


_PHASE_IDX: dict = {}


def _phase_weights(w: torch.Tensor) -> List[torch.Tensor]:
    """Weights of the four stride-2 data-gradient phases (csrc conv_dgrad_s2): input pixel
    (2i + a, 2j + b) takes dz row i with tap kh = 1 (a = 0), or dz rows i, i + 1 with taps kh = 2, 0
    (a = 1); likewise for the width.  Phase (a, b): [C1, nh * nw * C2] in (dh, dw, c2) order.
    One gather from the (kh, kw, c1)-ordered weight into a phase-major buffer (the index is
    built once per shape), so each phase weight is a contiguous view."""
    c2, c1 = w.shape[0], w.shape[1]
    key = (c2, c1, w.device)
    idx = _PHASE_IDX.get(key)
    if idx is None:
        parts = []
        ar2 = torch.arange(c2).view(1, 1, 1, c2)
        ar1 = torch.arange(c1).view(c1, 1, 1, 1)
        for a in (0, 1):
            for b in (0, 1):
                kh = torch.tensor([1] if a == 0 else [2, 0]).view(1, -1, 1, 1)
                kw = torch.tensor([1] if b == 0 else [2, 0]).view(1, 1, -1, 1)
                parts.append((((ar2 * 3 + kh) * 3 + kw) * c1 + ar1).reshape(-1))  # [c1, dh, dw, c2]
        idx = _PHASE_IDX[key] = torch.cat(parts).to(w.device)
    flat = w.permute(0, 2, 3, 1).reshape(-1)[idx]  # (c2, kh, kw, c1) source order
    out, o = [], 0
    for nh, nw in ((1, 1), (1, 2), (2, 1), (2, 2)):
        k = nh * nw * c2
        out.append(flat[o:o + c1 * k].view(c1, k))
        o += c1 * k
    return out


def _dgrad_s2_min_c() -> int:
    """Stride-2 data gradients on the phase GEMMs from 128 channels up: at 256 / 512 channels they
    beat MIOpen's kernel alone; at 128 (56x56) the four phases (747 us) trail its kernel (728 us)
    but not its zero fill + the separate bn1 reduce (profiles/r2_probe_dgrad_s2.jsonl: bench A/B
    13.53-13.56K vs 13.52K img/s)."""
    return 128


WGRAD3X3_MIN_C = 256


def _patch_wgrad_ok(h: int, w: int, c1: int, c2: int, s: int) -> bool:
    """The shapes csrc conv_wgrad_patch_kernel takes (mirrors convgemm.hip patch_ok): 3x3 / pad 1,
    stride 1 on 56- or 28-wide input maps, stride 2 on a 56-wide one (whole 112-pixel stages),
    c1 <= 128."""
    if not (c1 % 64 == 0 and c2 % 64 == 0 and c1 <= 128):
        return False
    if s == 1:
        return w in (56, 28) and h % (112 // w) == 0
    return s == 2 and w == 56 and h % 8 == 0


def _conv3x3_enabled() -> bool:
    return knobs.enabled("conv3x3")


class _Link:
    """bn3 backward hand-off from block i (consumer of this block's output) to this block."""

    __slots__ = ("out_ref", "z3", "bits", "mean", "invstd", "part", "dx_ptr", "dx_version", "dx_keep", "zd", "md",
                 "idd")

    def __init__(self, z3, bits, mean, invstd, zd=None, md=None, idd=None):
        self.out_ref = None
        self.z3, self.bits, self.mean, self.invstd = z3, bits, mean, invstd
        # a downsample block also hands its downsample BN (input zd, batch stats): the consumer's
        # epilogue 9 reduces that BN's backward sum next to bn3's
        self.zd, self.md, self.idd = zd, md, idd
        self.part = None
        self.dx_ptr = self.dx_version = self.dx_keep = None


FOLD_STATS = {"used": 0, "ds": 0, "resp": 0}  # bn3 / downsample-BN backward passes that took the consumer's
# partials; block outputs applied in the consumer's conv1 prologue ("resp")


class _Deferred:
    """A block output left unapplied: relu(bn3(z3) + r), r = the block input (identity) or the
    downsample BN's output.  The next fused block's conv1 applies it while staging its A tile and
    writes the output rows / ReLU bits into ``out`` / ``bits`` (block-output prologue, PRO 3):
    the separate apply pass and conv1's re-read of the output are gone."""

    __slots__ = ("out_ref", "z3", "cf3", "res", "cfd", "out", "bits")

    def __init__(self, z3, cf3, res, cfd, out, bits):
        self.out_ref = None
        self.z3, self.cf3, self.res, self.cfd, self.out, self.bits = z3, cf3, res, cfd, out, bits

    def flush(self) -> None:
        """Materialise the output with the apply pass (a consumer that cannot take the prologue)."""
        y, b = native().bn_apply_coef(self.z3, self.cf3, self.res, self.cfd, 1, True)
        with torch.no_grad():
            self.out.copy_(y)
            self.bits.copy_(b)


def _resp_enabled(c: int) -> bool:
    """Block outputs are applied in the consumer's conv1 prologue (which consumers take it:
    models/resnet.py ResNet.forward, resp_consumer_ok) unless PS_AMD_DISABLE=block_out."""
    return knobs.enabled("block_out")


def twosrc_glds_min_nk() -> int:
    """Mirror of csrc convgemm.hip kTwosrcGldsMinNk: two-source prologues with K >= 64 x this run
    on the LDS-DMA variant."""
    return 4


def big_tile(m: int, n: int, k: int, src2: int = 0, epi: int = 1, pro: bool = False) -> bool:
    """Whether conv_gemm runs this 1x1 stride-1 GEMM ([m, k] x [k, n]) on the 256 x 256 tiles of
    csrc/kernels/conv_big.hip (src2: 1 the block-output prologue, 2 the BN-backward prologue):
    there a prologue stages and transforms the A rows once per 256-channel tile, and the tiles of
    one pixel tile share an XCD, so the re-read that limits the 128-wide tiles to N <= 128 is gone."""
    return tuple(native().conv_gemm_plan(m, n, k, [m, 1, m, 1, 1, 1, 0], pro, epi, src2)[:2]) == (256, 256)


def resp_consumer_ok(blk: nn.Module, m: int = 0) -> bool:
    """Whether the block-output prologue pays on ``blk``'s conv1: with one channel tile (N <= 128,
    _twosrc_max_n) -- the layer-1 and layer-2 blocks and the layer-1 -> 2 boundary (LDS-DMA
    variant: 1.01 vs 1.21 ms at 256 -> 64 channels, 0.53 vs 0.62 ms at 512 -> 128); with two or
    more tiles each re-reads both sources and the apply pass + plain GEMM is faster
    (profiles/r4_twosrc_probe.txt)."""
    c1 = blk.conv1
    if m > 0 and big_tile(m, c1.out_channels, c1.in_channels, src2=1):  # m: the consumer's input pixels
        return True
    return c1.out_channels <= _twosrc_max_n() and (
        c1.in_channels >= 64 * twosrc_glds_min_nk() or c1.out_channels <= 64)


def flush_deferred() -> None:
    """Apply a pending deferred block output now (a consumer outside the fused path)."""
    pend = getattr(_tls, "pend", None)
    _tls.pend = None
    if pend is not None and pend.out_ref is not None and pend.out_ref() is not None:
        pend.flush()


def _twosrc_max_n() -> int:
    """Two-source prologues pay while the GEMM has ONE channel tile (N <= 128): every further tile
    re-reads both row sources (scripts/probe_twosrc.py, profiles/r4_twosrc_probe.txt: conv3 data
    grad 0.51 vs 0.64 ms at N = 128, 0.36 vs 0.25 ms at N = 512)."""
    return 128


def _bwd_prologue_enabled(c3: int, n: int = 0) -> bool:
    """bn3 backward applied in the conv3 data-gradient prologue (one channel tile).  At 256 channels (4 K-stages, persistent
    grid) the prologue stages A through registers from TWO row sources and replaces the apply
    pass + the LDS-DMA GEMM (1.29 -> 1.05-1.08 ms per layer-1 block); deeper K (512-2048
    channels, where the register-staged GEMM was 2-6x slower: profiles/r3_bn_bwd_prologue_ab.txt)
    runs the LDS-DMA two-source variant: both row sources land in LDS by DMA and one in-place pass
    per stage applies the BN backward (csrc convgemm.hip TWO_GLDS, scripts/probe_twosrc.py)."""
    return n <= _twosrc_max_n()


def _pro_fuse_max_k() -> int:
    """conv3's forward applies bn2 + ReLU while staging up to this many input channels; deeper
    (layer 4, 512) the apply pass + plain GEMM is faster: 0.16 vs 0.21 ms (layer 3: 0.26 either
    way; profiles/r4_twosrc_probe.txt, bn_relu_prologue rows)."""
    return 256


def _conv3_bwd_fused(ci: int, co: int) -> bool:
    """conv3's data AND weight gradient in one pass with bn3's backward in the prologue
    (csrc/kernels/conv_bwd_fused.hip): dz3 never reaches HBM and z2 is read once.
    PS_AMD_DISABLE=conv3_bwd_fused keeps the two-kernel chain (prologue data gradient storing dz3 +
    the weight-gradient GEMM re-reading it)."""
    return knobs.enabled("conv3_bwd_fused") and bool(native().conv11_bwd_fused_supported(ci, co))


def _ds_bwd_fused(ci: int, co: int, s: int) -> bool:
    """The downsample branch's data AND weight gradient in one pass with its BN backward in the
    prologue (the PLAIN mode of conv_bwd_fused.hip; stride 1, layer 1's 64 -> 256): dzd never
    reaches HBM and the block input is read once.  PS_AMD_DISABLE=ds_bwd_fused keeps the apply
    pass + weight-gradient GEMM + data-gradient GEMM."""
    return (s == 1 and knobs.enabled("ds_bwd_fused")
            and bool(native().conv11_bwd_fused_supported(ci, co, True)))


def _fold_enabled() -> bool:
    return knobs.enabled("fold_bn3")


def _fold_ds_enabled() -> bool:
    """Downsample BN's backward reduce in the consumer block's conv1 data-gradient epilogue (9)."""
    return knobs.enabled("fold_bn_ds")


class _BottleneckFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, g1, b1, w2, g2, b2, w3, g3, b3, wd, gd, bd, blk, link_in, pend_in):
        nat = native()
        n, cin, h, w = x.shape
        s = blk.conv2.stride[0]
        oh, ow = (h - 1) // s + 1, (w - 1) // s + 1
        gi, go = geo(h, w), geo(oh, ow)
        x2 = rows(x)
        bn1, bn2, bn3 = blk.bn1, blk.bn2, blk.bn3
        # shift of the statistics sums (~ the batch mean): the running mean itself -- the finalize
        # kernel reads channel c's shift before it updates that channel's running mean
        k1 = bn1.running_mean
        if pend_in is not None:  # the previous block's output is applied (and stored) while staging
            z1, p1 = nat.conv_gemm(pend_in.z3, _mat(w1), gi, pend_in.cf3, 1, None, k1, a2=pend_in.res,
                                   pro2=pend_in.cfd, aout=x2, abits=pend_in.bits)
            FOLD_STATS["resp"] += 1
        else:
            z1, p1 = nat.conv_gemm(x2, _mat(w1), gi, None, 1, None, k1)
        m1, i1, cf1 = _finalize(p1, k1, n * h * w, bn1)
        y1 = nat.bn_apply_coef(z1, cf1, None, None, 1)[0]
        if _conv3x3_enabled():
            # our implicit GEMM (LDS-DMA staging at this depth) with bn2's statistics in the epilogue
            k2 = bn2.running_mean
            z2r, p2s = nat.conv_gemm(y1, _mat3(w2), geo(h, w, 3, s, 1), None, 1, None, k2)
            m2, i2, cf2 = _finalize(p2s, k2, n * oh * ow, bn2)
        else:
            z2r = rows(F.conv2d(image(y1, n, h, w), w2, None, s, 1))
            m2, i2, cf2 = nat.bn_stats(z2r, g2, b2, bn2.running_mean, bn2.running_var, True, _momentum(bn2),
                                       float(bn2.eps))
        k3 = bn3.running_mean
        if z2r.shape[1] <= _pro_fuse_max_k():
            z3, p3 = nat.conv_gemm(z2r, _mat(w3), go, cf2, 1, None, k3)  # bn2 + ReLU in the prologue
        else:  # the apply pass + plain LDS-DMA GEMM is faster at this depth
            z3, p3 = nat.conv_gemm(nat.bn_apply_coef(z2r, cf2, None, None, 1)[0], _mat(w3), go, None, 1, None, k3)
        m3, i3, cf3 = _finalize(p3, k3, n * oh * ow, bn3)
        cfd = None
        if wd is not None:
            bnd = blk.downsample[1]
            kd = bnd.running_mean
            zd, pd = nat.conv_gemm(x2, _mat(wd), geo(h, w, 1, s), None, 1, None, kd)
            md, idd, cfd = _finalize(pd, kd, n * oh * ow, bnd)
        else:
            zd = md = idd = None
        if (getattr(blk, "_defer_out", False) and getattr(_tls, "pending", None) is not None
                and _resp_enabled(z3.shape[1])):
            # the next fused block applies this output in its conv1 prologue and fills out / obits
            # (handed over through the thread-local, which also works under no_grad)
            out = torch.empty_like(z3)
            obits = torch.empty(z3.numel() // 8, dtype=torch.uint8, device=z3.device)
            _tls.pend_new = _Deferred(z3, cf3, zd if wd is not None else x2, cfd, out, obits)
        else:
            out, obits = nat.bn_apply_coef(z3, cf3, zd if wd is not None else x2, cfd, 1, True)
        # the block output's ReLU mask is kept as 1 bit per element (the output itself is the
        # next block's input; the backward reads 1/16 of its bytes)
        ctx.save_for_backward(x2, w1, w2, w3, wd, g1, g2, g3, gd, z1, y1, z2r, z3, obits, zd,
                              m1, i1, cf1, m2, i2, cf2, m3, i3, md, idd)
        ctx.dims = (n, h, w, s, oh, ow)
        ctx.prep = _prep_for(blk, w1, w2, w3)  # backward weight layouts built for this forward
        ctx.link_in = link_in  # block i-1's bn3: its reduce runs in our conv1 data-grad epilogue
        ctx.link_out = (_Link(z3, obits, m3, i3, zd if _fold_ds_enabled() else None, md, idd)
                        if _fold_enabled() else None)
        return image(out, n, oh, ow)

    @staticmethod
    def backward(ctx, dout):
        nat = native()
        (x2, w1, w2, w3, wd, g1, g2, g3, gd, z1, y1, z2r, z3, obits, zd,
         m1, i1, cf1, m2, i2, cf2, m3, i3, md, idd) = ctx.saved_tensors
        n, h, w, s, oh, ow = ctx.dims
        gi, go = geo(h, w), geo(oh, ow)
        d2 = rows(dout)
        # weight gradients run on the side stream, overlapped with this data-gradient chain
        sd = _side.Fork(d2.device, (w1, w2, w3, wd), images=n)
        pw = ctx.prep
        w3t = pw[1] if pw else _mat(w3).t()
        lk = ctx.link_out
        dz3 = dw3f = None
        ds_part = None  # [2, G, C] downsample-BN sums from the consumer's epilogue 9
        if (lk is not None and lk.part is not None and d2.data_ptr() == lk.dx_ptr
                and d2._version == lk.dx_version):
            # the consumer block already masked dout and reduced bn3's backward sums
            if lk.part.shape[0] == 3:
                ds_part = lk.part[0::2]  # sum(g), sum(g * xhat_d): a strided view, no copy
                lk.part = lk.part[:2]
                FOLD_STATS["ds"] += 1
            if (_bwd_prologue_enabled(z3.shape[1], w3.shape[1])
                    or big_tile(d2.shape[0], w3.shape[1], z3.shape[1], src2=2, epi=3)):
                # bn3's backward runs in the conv3 data-grad prologue, which also stores dz3 for
                # the weight gradient: no separate apply pass over the widest tensors
                dg3, db3, cb3 = nat.bn_bwd_coef(lk.part, g3, m3, i3, d2.shape[0])
                if _conv3_bwd_fused(w3.shape[1], w3.shape[0]):
                    # data + weight gradient in ONE pass: dz3 stays in LDS, z2 is read once
                    gy2, p2, dw3f = nat.conv11_bwd_fused(d2, z3, cb3, w3t.contiguous(), z2r, cf2, m2, i2)
                    FOLD_STATS["conv3_fused"] = FOLD_STATS.get("conv3_fused", 0) + 1
                else:
                    gy2, p2, dz3 = nat.conv_gemm(d2, w3t, go, None, 3, z2r, None, cf2, m2, i2, a2=z3, bwd=cb3)
            else:
                dz3, dg3, db3 = nat.bn_bwd_partials(d2, z3, lk.part, g3, m3, i3)
                gy2 = None
            FOLD_STATS["used"] += 1
        else:
            # bn3 with the ReLU mask from the output bits; the masked gradient dout * relu' is
            # also the identity-branch gradient -- recomputed where needed, never stored
            dz3, _, dg3, db3 = nat.bn_act_bwd(d2, None, z3, g3, m3, i3, 3, False, True, None, obits)
            gy2 = None
        if lk is not None:
            lk.part = lk.dx_keep = None
        # conv3: data grad with bn2's ReLU mask + backward sums in the epilogue, weight grad with
        # relu(bn2(z2)) recomputed in the prologue
        if dw3f is not None:
            dw3 = _side._match_layout(dw3f, w3)
        else:
            sd.fork()
            dw3 = sd.run(lambda: nat.conv_wgrad(dz3, z2r, go, cf2), dz3, z2r, cf2, like=w3)
        if gy2 is None:
            gy2, p2 = nat.conv_gemm(dz3, w3t, go, None, 3, z2r, None, cf2, m2, i2)
        dz2, dg2, db2 = nat.bn_bwd_partials(gy2, z2r, p2, g2, m2, i2)
        c1, c2 = w2.shape[1], w2.shape[0]
        ours_dgrad = _conv3x3_enabled() and (s == 1 or (s == 2 and h % 2 == 0 and w % 2 == 0
                                                         and w2.shape[1] >= _dgrad_s2_min_c()))
        # weight grad on the wide-tile kernel from 256 input channels up (on par with / faster than
        # MIOpen there: profiles/r2_wgrad_probe.jsonl), on the patch kernel at 64 / 128 channels
        # (csrc conv_wgrad_patch_kernel: 2.4x / 1.6x MIOpen, profiles/r3_wgrad_probe_patch.jsonl)
        ours_wgrad = _conv3x3_enabled() and (c1 >= WGRAD3X3_MIN_C or _patch_wgrad_ok(h, w, c1, c2, s))
        dy1 = dw2 = None
        sd.fork()
        if ours_wgrad:
            dw2 = sd.run(lambda: nat.conv_wgrad(dz2, y1, geo(h, w, 3, s, 1)).view(w2.shape[0], 3, 3, c1)
                         .permute(0, 3, 1, 2), dz2, y1, like=w2)
        else:
            dw2 = sd.run(lambda: torch.ops.aten.convolution_backward(
                image(dz2, n, oh, ow), image(y1, n, h, w), w2, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1,
                [False, True, False])[1], dz2, y1, like=w2)
        if not ours_dgrad:
            dy1 = torch.ops.aten.convolution_backward(image(dz2, n, oh, ow), image(y1, n, h, w), w2, None,
                                                      [s, s], [1, 1], [1, 1], False, [0, 0], 1,
                                                      [True, False, False])[0]
        if ours_dgrad:
            # data grad = the forward GEMM over dz2 with the flipped, transposed weight; its epilogue
            # applies bn1's ReLU mask and reduces bn1's backward sums (no separate reduce pass)
            if s == 1:
                gy1, p1b = nat.conv_gemm(dz2, pw[2] if pw else _mat3_dgrad(w2), geo(oh, ow, 3, 1, 1), None, 3, z1,
                                         None, cf1, m1, i1)
            else:  # four stride-1 phase GEMMs, each writing every other dx row (no zero fill)
                gy1, p1b = nat.conv_dgrad_s2(dz2, pw[2] if pw else _phase_weights(w2), h, w, 3, z1, cf1, m1, i1)
        li = ctx.link_in
        fold = li is not None and _fold_enabled()
        fkw = dict(mean=li.mean, invstd=li.invstd, aux2=li.z3, bits2=li.bits) if fold else {}
        if wd is not None:
            e1 = (8 if s == 2 else 7) if fold else (4 if s == 2 else 2)
        else:
            e1 = (9 if li.zd is not None else 6) if fold else 5
        # (bn1's backward as the conv1 data-gradient prologue on the 256 x 256 tiles cost more than
        # the apply pass it removes at K = 256 / 512 in the round-5 A/B, scripts/probe_conv_big.py; removed)
        if ours_dgrad:
            dz1, dg1, db1 = nat.bn_bwd_partials(gy1, z1, p1b, g1, m1, i1)
        else:
            dz1, _, dg1, db1 = nat.bn_act_bwd(rows(dy1), None, z1, g1, m1, i1, 1, False, True, cf1)
        sd.fork()
        dw1 = sd.run(lambda: nat.conv_wgrad(dz1, x2, gi), dz1, x2, like=w1)
        a1 = dz1
        w1t = pw[0] if pw else _mat(w1).t()
        dwd = dgd = dbd = None
        if wd is not None:
            wdt = pw[3] if pw else _mat(wd).t()
            if ds_part is not None and _ds_bwd_fused(wd.shape[1], wd.shape[0], s):
                # d2 is masked already and the downsample BN's sums came with it: its backward
                # coefficients, then ONE pass = data gradient t + weight gradient (dzd stays in LDS)
                dgd, dbd, cbd = nat.bn_bwd_coef(ds_part, gd, md, idd, d2.shape[0])
                t, _, dwdf = nat.conv11_bwd_fused(d2, zd, cbd, wdt.contiguous(), x2)
                dwd = _side._match_layout(dwdf, wd)
                FOLD_STATS["ds_fused"] = FOLD_STATS.get("ds_fused", 0) + 1
            else:
                if ds_part is not None:  # d2 is masked already; sum(g), sum(g * xhat_d) came with it
                    dzd, dgd, dbd = nat.bn_bwd_partials(d2, zd, ds_part, gd, md, idd)
                else:
                    dzd, _, dgd, dbd = nat.bn_act_bwd(d2, None, zd, gd, md, idd, 3, False, True, None, obits)
                sd.fork()
                dwd = sd.run(lambda: nat.conv_wgrad(dzd, x2, geo(h, w, 1, s)), dzd, x2, like=wd)
                t = nat.conv_gemm(dzd, wdt, go)[0]
            r1 = nat.conv_gemm(a1, w1t, gi, None, e1, t, **fkw)
        elif e1 == 9:  # the producer has a downsample BN: its sum rides along
            r1 = nat.conv_gemm(a1, w1t, gi, None, 9, d2, bits=obits, aux3=li.zd, mean2=li.md, invstd2=li.idd,
                               **fkw)
        else:
            r1 = nat.conv_gemm(a1, w1t, gi, None, e1, d2, bits=obits, **fkw)
        dx2, part = r1[0], r1[1]
        if fold:
            # dx_keep pins a second reference on dx2's storage, so autograd cannot sum another
            # consumer's gradient into it in place (it would not bump the version): a summed
            # gradient always lands in a different buffer and fails the pointer check
            li.part, li.dx_ptr, li.dx_version, li.dx_keep = part, dx2.data_ptr(), dx2._version, dx2
        return (image(dx2, n, h, w), dw1, dg1, db1, dw2, dg2, db2, dw3, dg3, db3,
                dwd, dgd, dbd, None, None, None)


def fused_block_ok(blk: nn.Module, x: torch.Tensor) -> bool:
    """True when ``blk`` (models.resnet.Bottleneck) can run the fused path on ``x``."""
    if knobs.disabled("fused_block") or not getattr(blk, "fuse_block", False):
        return False
    if not (blk.training and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4):
        return False
    ds = blk.downsample
    bns = [blk.bn1, blk.bn2, blk.bn3] + ([ds[1]] if ds is not None else [])
    for bn in bns:
        if not (bn.track_running_stats and bn.affine and bn.weight.dtype == torch.float32
                and bn.running_mean is not None and bn.running_mean.dtype == torch.float32):
            return False
    c1, c2, c3 = blk.conv1, blk.conv2, blk.conv3
    convs = [c1, c2, c3] + ([ds[0]] if ds is not None else [])
    if any(not isinstance(c, nn.Conv2d) or c.weight.dtype != torch.bfloat16 or c.bias is not None or c.groups != 1
           for c in convs):
        return False
    if c1.kernel_size != (1, 1) or c1.stride != (1, 1) or c3.kernel_size != (1, 1) or c3.stride != (1, 1):
        return False
    if (c2.kernel_size != (3, 3) or c2.padding != (1, 1) or c2.dilation != (1, 1)
            or c2.stride[0] != c2.stride[1] or c2.stride[0] not in (1, 2)):
        return False
    if ds is not None:
        if len(ds) != 2 or ds[0].kernel_size != (1, 1) or ds[0].stride != c2.stride or ds[0].padding != (0, 0):
            return False
        if getattr(ds[1], "act", "none") != "none":
            return False
    elif c2.stride != (1, 1) or x.shape[1] != c3.out_channels:
        return False
    return all(c % 64 == 0 for c in (x.shape[1], c1.out_channels, c3.out_channels))


_tls = threading.local()

# Backward weight layouts (transposed 1x1, flipped / phase-split 3x3) of every fused block, built
# in ONE kernel per forward (csrc weight_prep) instead of ~70 copy / flip / gather kernels per step.
# Cache: weight storage pointers -> (job table, per-block output tensors); the PS binds weights to
# fixed slot views, so the table is built once per slot.
_PREP_CACHE: "dict" = {}


def _prep_ok(blk: nn.Module) -> bool:
    ws = [blk.conv1.weight, blk.conv2.weight, blk.conv3.weight] + (
        [blk.downsample[0].weight] if blk.downsample is not None else [])
    return (getattr(blk, "fuse_block", False) and all(w.is_cuda and w.dtype == torch.bfloat16 for w in ws)
            and blk.conv2.weight.is_contiguous(memory_format=torch.channels_last)
            and all(w.is_contiguous() for w in [blk.conv1.weight, blk.conv3.weight] + ws[3:]))


def prepare_backward_weights(blocks) -> None:
    """Build the backward weight layouts of ``blocks`` (the fused bottlenecks of one forward) in
    one launch; _BottleneckFn picks them up through the thread-local set (cleared when the
    enclosing ``deferred_bn_counters`` context ends)."""
    if knobs.disabled("weight_prep"):
        return
    blks = [b for b in blocks if _prep_ok(b)]
    if not blks:
        return
    key = tuple((id(b), b.conv1.weight.data_ptr(), b.conv2.weight.data_ptr(), b.conv3.weight.data_ptr(),
                 b.downsample[0].weight.data_ptr() if b.downsample is not None else 0) for b in blks)
    ent = _PREP_CACHE.get(key)
    if ent is None:
        rows, outs, nblk = [], {}, [1]
        dev = blks[0].conv1.weight.device

        def job(src, kind, a, b):
            n = (1 if kind == 0 else 9) * a * b
            dst = torch.empty(n, dtype=torch.bfloat16, device=dev)
            rows.append([src.data_ptr(), dst.data_ptr(), kind | (a << 32), b])
            nblk[0] = max(nblk[0], (1 if kind == 0 else 9) * ((a + 63) // 64) * ((b + 63) // 64))
            return dst

        for b in blks:
            w1, w2, w3 = b.conv1.weight, b.conv2.weight, b.conv3.weight
            c2, c1 = w2.shape[0], w2.shape[1]
            w1t = job(w1, 0, w1.shape[0], w1.shape[1]).view(w1.shape[1], w1.shape[0])
            w3t = job(w3, 0, w3.shape[0], w3.shape[1]).view(w3.shape[1], w3.shape[0])
            if b.conv2.stride[0] == 1:
                w2d = job(w2, 1, c2, c1).view(c1, 9 * c2)
            else:
                flat = job(w2, 2, c2, c1)
                w2d, o = [], 0
                for nh, nw in ((1, 1), (1, 2), (2, 1), (2, 2)):
                    k = nh * nw * c2
                    w2d.append(flat[o:o + c1 * k].view(c1, k))
                    o += c1 * k
            wdt = None
            if b.downsample is not None:
                wd = b.downsample[0].weight
                wdt = job(wd, 0, wd.shape[0], wd.shape[1]).view(wd.shape[1], wd.shape[0])
            outs[id(b)] = (w1t, w3t, w2d, wdt, (w1.data_ptr(), w2.data_ptr(), w3.data_ptr()))
        ent = (torch.tensor(rows, dtype=torch.int64).to(dev), outs, nblk[0])
        if len(_PREP_CACHE) >= 4:
            _PREP_CACHE.pop(next(iter(_PREP_CACHE)))
        _PREP_CACHE[key] = ent
    native().weight_prep(ent[0], ent[2])
    _tls.prep = ent[1]


def _prep_for(blk, w1, w2, w3):
    prep = getattr(_tls, "prep", None)
    ent = prep.get(id(blk)) if prep else None
    if ent is None or ent[4] != (w1.data_ptr(), w2.data_ptr(), w3.data_ptr()):
        return None
    return ent


@contextlib.contextmanager
def deferred_bn_counters():
    """Collect the BN ``num_batches_tracked`` increments of the fused blocks run inside and apply
    them as one multi-tensor add on exit (53 one-element kernels per ResNet-50 step otherwise)."""
    prev = getattr(_tls, "pending", None)
    _tls.pending = []
    _tls.last = None  # bn3 hand-off chain starts fresh every forward
    _tls.pend = None
    try:
        yield
    finally:
        flush_deferred()  # (a deferred output nobody consumed -- never on the ResNet path)
        _tls.last = None
        _tls.prep = None
        pending, _tls.pending = _tls.pending, prev
        if pending:
            torch._foreach_add_(pending, 1)


def fused_bottleneck(blk: nn.Module, x: torch.Tensor) -> torch.Tensor:
    ds = blk.downsample
    counters = [bn.num_batches_tracked for bn in [blk.bn1, blk.bn2, blk.bn3] + ([ds[1]] if ds is not None else [])]
    pending = getattr(_tls, "pending", None)
    if pending is not None:
        pending.extend(counters)
    else:
        torch._foreach_add_(counters, 1)
    wd, gd, bd = (ds[0].weight, ds[1].weight, ds[1].bias) if ds is not None else (None, None, None)
    last = getattr(_tls, "last", None)
    link_in = last if last is not None and last.out_ref is not None and last.out_ref() is x else None
    _tls.pend_new = None
    pend = getattr(_tls, "pend", None)
    pend_in = None
    if pend is not None:
        if pend.out_ref is not None and pend.out_ref() is x:
            pend_in = pend
            _tls.pend = None
        else:
            flush_deferred()
    y = _BottleneckFn.apply(x, blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight,
                            blk.bn2.bias, blk.conv3.weight, blk.bn3.weight, blk.bn3.bias, wd, gd, bd, blk, link_in,
                            pend_in)
    gf = y.grad_fn
    lk = gf.link_out if gf is not None and hasattr(gf, "link_out") else None
    if lk is not None and hasattr(_tls, "pending") and _tls.pending is not None:
        lk.out_ref = weakref.ref(y)
        _tls.last = lk
    po = getattr(_tls, "pend_new", None)
    _tls.pend_new = None
    if po is not None:
        po.out_ref = weakref.ref(y)
        _tls.pend = po
    return y
