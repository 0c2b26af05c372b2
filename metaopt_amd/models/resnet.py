"""ResNet-20 populations on CIFAR-shaped data (BASELINE.json config 3: TPE over ResNet-20,
trial-parallel over 8 GPUs with the RCCL metric all-gather).

Architecture (He et al. 2016, CIFAR variant): 3x3 conv 16 -> 3 stages x 3 basic blocks (16, 32,
64 channels; stride 2 at stages 2 and 3 with the parameter-free "option A" shortcut: subsample +
zero-pad channels) -> global average pool -> linear 64 -> 10; ~0.27M parameters per trial.
Activations are NHWC bf16 with the population folded into the batch; images carry 8 channels
(3 real + 5 zero) so every kernel moves 16-byte vectors.  Convolutions: direct halo-tiled MFMA
kernels (ops/conv.py -> csrc/conv_direct.hip: forward with the BatchNorm batch statistics in its
epilogue, stride-1 data gradient, weight gradient), the implicit GEMM of csrc/pgemm.hip for the
stride-2 data gradient; BatchNorm (+ residual + ReLU) fused HIP kernels with per-trial batch
and running statistics; SGD-momentum with per-trial lr / momentum / weight decay (fused K5).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import ClassVar, Dict, Optional

import numpy as np
import torch

from ..ops import conv as cops
from ..ops.population import MemberConfig
from .flatpop import FlatPopulation

IN_CH = 8          # 3 image channels + 5 zero channels
STAGES = (16, 32, 64)
NCLS = 10
NCLS_PAD = 16      # head width padded to a multiple of 8 (only the first 10 logits are used)


def resnet20_layout(blocks_per_stage: int = 3):
    """[(conv name, cin, cout, stride)] in forward order (BN after each conv)."""
    convs = [("conv0", IN_CH, STAGES[0], 1)]
    cin = STAGES[0]
    for si, cout in enumerate(STAGES):
        for b in range(blocks_per_stage):
            stride = 2 if (si > 0 and b == 0) else 1
            convs.append((f"s{si}b{b}c1", cin, cout, stride))
            convs.append((f"s{si}b{b}c2", cout, cout, 1))
            cin = cout
    return convs


class PopulationResNet(FlatPopulation):
    optimizer = "sgd"
    secondary = "acc"

    def __init__(self, capacity: int, batch_size: int = 128, device="cuda",
                 blocks_per_stage: int = 3, image_size: int = 32, use_graph: bool = True):
        self.batch_size = int(batch_size)
        self.blocks = int(blocks_per_stage)
        self.image_size = int(image_size)
        self.layout = resnet20_layout(self.blocks)
        super().__init__(capacity, device=device, use_graph=use_graph)

    # ------------------------------------------------------------------ structure
    def param_specs(self):
        specs = []
        for name, cin, cout, _ in self.layout:
            specs.append((f"{name}.w", (9 * cin, cout), ("kaiming", 9 * cin)))
            specs.append((f"{name}.g", (cout,), ("ones",)))
            specs.append((f"{name}.b", (cout,), ("zeros",)))
        specs.append(("fc.w", (STAGES[-1], NCLS_PAD), ("normal", 1.0 / math.sqrt(STAGES[-1]))))
        specs.append(("fc.b", (NCLS_PAD,), ("zeros",)))
        return specs

    def direct_grads(self):
        # conv weights (wgrad kernels), BatchNorm gamma / beta (BN backward) and the classifier
        # (the fused head kernel): every gradient is written in full by a HIP kernel
        return {f"{name}.{k}" for name, _, _, _ in self.layout for k in ("w", "g", "b")} | \
            {"fc.w", "fc.b"}

    def aux_specs(self):
        return [(f"{name}.running", 2 * cout) for name, _, cout, _ in self.layout]

    def aux_fill_specs(self):
        # running mean 0, running var 1 of every BatchNorm (one launch with the parameters)
        out = []
        for name, _, cout, _ in self.layout:
            out += [(f"{name}.running", 0, cout, 0.0), (f"{name}.running", cout, cout, 1.0)]
        return out

    def init_aux(self, slot: int) -> None:
        for name, _, cout, _ in self.layout:
            r = self.A[f"{name}.running"][slot].view(2, cout)
            r[0].zero_()
            r[1].fill_(1.0)

    def rows_per_batch(self, x) -> int:
        return int(x.shape[0])

    # ------------------------------------------------------------------ forward
    def _conv_bn(self, name, x, stride, train, res=None, relu=True, arena=None, **mail):
        P, W = self.capacity, self.W
        w = W[f"{name}.w"]
        running = self.A[f"{name}.running"].view(P, 2, w.shape[-1])
        return cops.conv_bn_act(x, w, W[f"{name}.g"], W[f"{name}.b"], running, P, stride, train,
                                res=res, relu=relu, arena=arena, **mail)

    def _block_fused(self, n1, n2, h, pend, s1, identity, arena, box):
        """One training basic block on the HIP path.  Its input is either materialised (``h``)
        or still ``pend``-ing: the previous block's BatchNorm 2 + shortcut + ReLU (or the stem's
        BatchNorm + ReLU), which conv 1 then forms while staging its input bands and writes out
        once (``bn_res_conv3x3``; the materialised fallback runs the apply pass and links that
        BatchNorm's backward into conv 1's data gradient).  Conv 1 (+ its BatchNorm's batch
        sums), BatchNorm 1 + ReLU applied inside conv 2 (``bn_relu_conv3x3``) when the shapes
        allow, and this block's BatchNorm 2 + shortcut + ReLU left pending for the next
        consumer; the shortcut's gradient joins conv 1's data gradient in its epilogue
        (``box``).  Returns (the block input h, this block's PendingBN or its output)."""
        P, W = self.capacity, self.W
        w1, w2 = W[f"{n1}.w"], W[f"{n2}.w"]
        c1, c2 = w1.shape[-1], w2.shape[-1]
        run1 = self.A[f"{n1}.running"].view(P, 2, c1)
        run2 = self.A[f"{n2}.running"].view(P, 2, c2)
        if pend is not None and cops.bn_res_conv_ok(pend, w1, s1):
            y1, st1, h = cops.bn_res_conv3x3(pend, w1, P, s1, arena, conv_mailbox=box)
        else:
            link = None
            if pend is not None:
                link = {}
                h = pend.materialize(arena, link=link)
            y1, st1 = cops.conv_stats(h, w1, P, s1, True, arena=arena, mailbox=box,
                                      bn_link=link)
        if cops.bn_into_conv_ok(y1, w2, P, 1, True, arena, st1 is not None):
            y2, st2 = cops.bn_relu_conv3x3(y1, W[f"{n1}.g"], W[f"{n1}.b"], run1, w2, P, st1,
                                           arena)
        else:
            t = cops.bn_act(y1, W[f"{n1}.g"], W[f"{n1}.b"], run1, P, True, sums=st1,
                            arena=arena)
            y2, st2 = cops.conv_stats(t, w2, P, 1, True, arena=arena)
        out = cops.PendingBN(y2, st2, W[f"{n2}.g"], W[f"{n2}.b"], run2, P, res=h.detach(),
                             res_sub2=not identity, mailbox=box)
        if st2 is None:       # no batch sums from conv 2: the BatchNorm runs its own reduction
            return h, out.materialize(arena)
        return h, out

    @staticmethod
    def _shortcut(x, cout, stride):
        if stride == 1 and x.shape[-1] == cout:
            return x
        return cops.option_a_shortcut(x, cout)

    def _loss(self, x, y, train: bool):
        P, W = self.capacity, self.W
        # [P*B, H, W, 8]: the evaluation / CPU path's input (training on the HIP path reads the
        # shared batch in place, cops.shared_conv_stats)
        h = self._expand(x, torch.bfloat16).view(-1, *x.shape[1:]) \
            if not (train and x.device.type == "cuda") else None
        B = x.shape[0]
        # one zero fill per step for every layer's BatchNorm sums (forward and backward)
        arena = (cops.ZeroArena(sum(4 * P * c for _, _, c, _ in self.layout), x.device)
                 if train and x.device.type == "cuda" else None)
        it = iter(self.layout)
        name, _, cout, stride = next(it)
        # training on the HIP path: every BatchNorm whose output feeds a convolution is left
        # pending (cops.PendingBN) and formed inside that convolution's input staging, its
        # backward's masking and reductions in that convolution's data gradient
        pend = None
        if arena is not None:
            W0 = self.W[f"{name}.w"]
            # the stem reads the shared minibatch itself, not the P-fold expanded copy
            shared = cops.shared_conv_stats(x.to(self.device, torch.bfloat16), W0, P, arena) \
                if stride == 1 else None
            if shared is None:
                h = self._expand(x, torch.bfloat16).view(-1, *x.shape[1:])
                shared = cops.conv_stats(h, W0, P, stride, True, arena=arena)
            y0, st0 = shared
            pend = cops.PendingBN(y0, st0, W[f"{name}.g"], W[f"{name}.b"],
                                  self.A[f"{name}.running"].view(P, 2, cout), P)
            if st0 is None:
                h, pend = pend.materialize(arena), None
        else:
            h = self._conv_bn(name, h, stride, train, arena=arena)
        for si in range(len(STAGES)):
            for b in range(self.blocks):
                n1, _, c1, s1 = next(it)
                n2, _, c2, _ = next(it)
                cin = pend.x.shape[-1] if pend is not None else h.shape[-1]
                identity = s1 == 1 and cin == c2
                if train and arena is not None and (identity or s1 == 2):
                    # the shortcut's gradient joins the first conv's data gradient in that
                    # kernel's epilogue (no separate add over the block input); an option-A
                    # shortcut is also read in place (no padded copy)
                    box = {}
                    h, out = self._block_fused(n1, n2, h if pend is None else None, pend, s1,
                                               identity, arena, box)
                    pend, h = (out, None) if isinstance(out, cops.PendingBN) else (None, out)
                    continue
                if pend is not None:
                    h, pend = pend.materialize(arena), None
                r = self._shortcut(h, c2, s1)
                t = self._conv_bn(n1, h, s1, train, arena=arena)
                h = self._conv_bn(n2, t, 1, train, res=r, arena=arena)
        labels = self._expand(y, torch.long).reshape(-1)
        if pend is not None and cops.bn_head_ok(pend, W["fc.w"], W["fc.b"], labels):
            # the last block's output is formed inside the head, never written
            return cops.bn_resnet_head(pend, W["fc.w"], W["fc.b"], labels, NCLS, arena,
                                       scale=1.0 / B)
        if pend is not None:          # the last block's output feeds the head
            h = pend.materialize(arena)
        if x.device.type == "cuda":
            # pool + linear + cross-entropy (+ its backward) in one HIP kernel; the classifier's
            # dW / db land in the flat gradient buffer (direct gradients), mean-loss scaled
            return cops.resnet_head(h, W["fc.w"], W["fc.b"], labels, P, NCLS, train,
                                    scale=1.0 / B)
        loss, correct, _ = cops.head_ref(h, W["fc.w"], W["fc.b"], labels, P, NCLS)
        if train:
            loss = _GradScale.apply(loss, 1.0 / B)
        return loss, correct


class _GradScale(torch.autograd.Function):
    """Identity forward, scales the gradient (loss SUMS are reported, mean-loss gradients used)."""

    @staticmethod
    def forward(ctx, x, s):
        ctx.s = s
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return g * ctx.s, None


class SyntheticCIFAR:
    """CIFAR-shaped synthetic classification that ResNet-20 can learn: each 32x32x3 image (NHWC,
    padded to 8 channels, bf16) is a texture -- N(0, 1) noise filtered by its class's fixed
    random 3x3 colour filter -- mixed with a weaker texture of another class (a distractor)
    and white noise.  The class is a translation-invariant property of the image (its local
    colour / spatial correlations), which a conv net with a global average pool reads at every
    position.  Round 6: the former teacher on position-specific 4x4-pooled pixels was nearly
    unlearnable through the final global pool (the best of 224 trials reached 2.145 nats against
    H(y) = 2.286), which left TPE-vs-random comparisons at noise level.  ``mix`` = (class,
    distractor, white) amplitudes sets the difficulty."""

    def __init__(self, n_train: int = 50048, n_val: int = 1024, batch_size: int = 128,
                 seed: int = 0, device=None, image_size: int = 32,
                 mix: tuple = (1.0, 0.7, 0.5)):
        g = torch.Generator().manual_seed(seed)
        S = image_size
        filt = torch.randn(NCLS, 3, 3, 3, 3, generator=g)          # [class][out][in][3][3]
        filt = filt / filt.flatten(2).norm(dim=2).view(NCLS, 3, 1, 1, 1)
        dev = torch.device(device) if device is not None else torch.device("cpu")
        a, b, c = mix

        def texture(cls, n):
            z = torch.randn(n, 3, S, S, generator=g)
            out = torch.empty(n, 3, S, S)
            for k in range(NCLS):   # one grouped conv per class
                idx = (cls == k).nonzero().flatten()
                if len(idx):
                    out[idx] = torch.nn.functional.conv2d(z[idx], filt[k], padding=1)
            return out

        def draw(n):
            y = torch.randint(0, NCLS, (n,), generator=g)
            other = (y + torch.randint(1, NCLS, (n,), generator=g)) % NCLS
            x = a * texture(y, n) + b * texture(other, n) + \
                c * torch.randn(n, 3, S, S, generator=g)
            xp = torch.zeros(n, S, S, IN_CH)
            xp[..., :3] = x.permute(0, 2, 3, 1)
            return xp.to(torch.bfloat16).to(dev), y.to(dev)

        self.batch_size = batch_size
        n_train = n_train // batch_size * batch_size
        self.train_x, self.train_y = draw(n_train)
        self.val_x, self.val_y = draw(n_val)
        self.n_batches = n_train // batch_size

    def batch(self, step: int):
        i = step % self.n_batches
        sl = slice(i * self.batch_size, (i + 1) * self.batch_size)
        return self.train_x[sl], self.train_y[sl]

    def validation(self):
        return self.val_x, self.val_y


RESNET_TPE_PRIORS = {
    "/lr": "loguniform(0.01, 0.5)",
    "/momentum": "uniform(0.5, 0.99)",
    "/weight_decay": "loguniform(1e-5, 1e-2)",
}


@dataclass
class ResNetSweepTask:
    """Trial parameters -> ResNet population members (SGD lr / momentum / weight decay); trials
    train a fixed budget of ``steps`` unless the space has a fidelity dimension."""

    priors: Dict[str, str] = field(default_factory=lambda: dict(RESNET_TPE_PRIORS))
    # key(params) == param_key(params, fidelity): the sweep may derive it from points directly
    key_by_params: ClassVar[bool] = True
    fidelity: str = "/steps"
    steps: int = 390
    secondary_stat: str = "val_acc"

    def member_config(self, params: Dict, seed: int) -> MemberConfig:
        return MemberConfig(width=0, lr=float(params["/lr"]),
                            momentum=float(params.get("/momentum", 0.9)),
                            weight_decay=float(params.get("/weight_decay", 5e-4)),
                            seed=int(seed) & 0x7FFFFFFF)

    def budget(self, params: Dict) -> int:
        return int(params.get(self.fidelity, self.steps))

    def key(self, params: Dict) -> str:
        from .mlp import param_key
        return param_key(params, self.fidelity)

    @staticmethod
    def seed_of(key: str) -> int:
        return int(key[:8], 16)
