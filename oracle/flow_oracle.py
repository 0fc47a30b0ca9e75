"""oracle/flow_oracle.py -- TEST INFRASTRUCTURE ONLY.

A functional torch-fp32 CPU restatement of the reference's integer-discrete
flow (IDF) hot path, driven by a state_dict (the reference's key names) and the
reference YAML model config.  It is the checker for the HIP flow kernels and the
flow leg of bench.py's cpu_baseline; the product path never imports it.

Pinned against tests/golden/flow_*.npz and imagenet64_b2.npz, which were
produced by the reference's own modules (tests/golden/make_golden.py).

Reference map:
  dequant              trainer.py:101,131-136   (ToTensor k/255, Round(nbits=8))
  round8               roundlib.py:27-38        (rint(x*2^n)/2^n, ties to even)
  dense_layer          nnlayer.py:42-51         (1x1 c->c, 3x3 c->g pad 1, act, cat)
  dense_block          nnblock.py:24-56         (depth layers + 1x1 head)
  couple_fwd / _bwd    couplelib.py:47-61       (zb = xb + Round(NN(xa)))
  permute_fwd / _bwd   invertible.py:38-48      (F.linear with 0/1 P == channel gather)
  extend_fwd / _bwd    extenddim.py:23-37       (space-to-depth)
  prior                priorlib.py:36-47
  idflows_forward      flows.py:87-116
  cond_forward         flows.py:303-327
  generated_from_latents flows.py:139-152
  decode_levels        flows.py:118-137 with rANS decode in place of sampling
  log_likelihood       flows.py:154-169, distlib.py:40-55
"""
from __future__ import annotations

import copy

import torch
import torch.nn.functional as F

LEAKY_SLOPE = 0.01  # nn.LeakyReLU() default (nnlayer.py:37)


def dequant(u8: torch.Tensor) -> torch.Tensor:
    x = u8.to(torch.float32) / 255.0
    return torch.round(x * 256) / 256


def round8(x: torch.Tensor, nbits: int = 8) -> torch.Tensor:
    bins = 2 ** nbits
    return torch.round(x * bins) / bins


def _act(h, act):
    if act == "ReLU":
        return F.relu(h)
    if act == "LeakyReLU":
        return F.leaky_relu(h, LEAKY_SLOPE)
    if act == "Tanh":
        return torch.tanh(h)
    raise ValueError(act)


def dense_layer(x, sd, p, act):
    t = F.conv2d(x, sd[p + "layers.0.weight"], sd[p + "layers.0.bias"])
    h = F.conv2d(t, sd[p + "layers.1.weight"], sd[p + "layers.1.bias"], padding=1)
    return torch.cat((x, _act(h, act)), dim=1)


def dense_block(x, sd, p, depth, act):
    for i in range(depth):
        x = dense_layer(x, sd, f"{p}layers.{i}.", act)
    return F.conv2d(x, sd[f"{p}layers.{depth}.weight"], sd[f"{p}layers.{depth}.bias"])


def perm_ids(P: torch.Tensor) -> torch.Tensor:
    """y = F.linear(x, P) with P[i, ids[i]] = 1  ==>  y[:, i] = x[:, ids[i]]."""
    return torch.argmax(P, dim=1)


def permute_fwd(x, P):
    return x[:, perm_ids(P)]


def permute_bwd(y, P):
    ids = perm_ids(P)
    x = torch.empty_like(y)
    x[:, ids] = y
    return x


def extend_fwd(x, s):
    B, C, H, W = x.shape
    x = x.view(B, C, H // s, s, W // s, s).permute(0, 1, 3, 5, 2, 4).contiguous()
    return x.view(B, C * s * s, H // s, W // s)


def extend_bwd(x, s):
    B, C, H, W = x.shape
    x = x.view(B, C // s // s, s, s, H, W).permute(0, 1, 4, 2, 5, 3).contiguous()
    return x.view(B, C // s // s, H * s, W * s)


class FlowOracle:
    """Holds a reference state_dict + model config; runs the hot path on CPU fp32."""

    def __init__(self, cfg: dict, state_dict: dict):
        cfg = copy.deepcopy(cfg)
        self.name = cfg.get("name", "IDFlows")
        self.nflows = cfg["nflows"]
        self.nsplit = cfg["nsplit"]
        self.nbits = cfg.get("nbits", 8)
        self.C, self.H, self.W = cfg["C"], cfg["H"], cfg["W"]
        self.scale = cfg["extenddim"]["scale"]
        self.split = cfg["couple"].get("split", 0.75)
        self.c_depth = cfg["couple"]["nn"]["depth"]
        self.c_act = cfg["couple"]["nn"]["layer"].get("act", "ReLU")
        self.p_depth = cfg["prior"]["nn"]["depth"]
        self.p_act = cfg["prior"]["nn"]["layer"].get("act", "ReLU")
        self.conv_for_cond = bool(cfg.get("conv_for_cond", False))
        self.sd = {k: (v if isinstance(v, torch.Tensor) else torch.as_tensor(v)).float()
                   for k, v in state_dict.items()}
        # per-level channel geometry (flows.py:57-83)
        self.level_ch = []
        ch = self.C
        for lvl in range(self.nsplit):
            ch *= self.scale * self.scale
            self.level_ch.append(ch)
            if lvl < self.nsplit - 1:
                ch -= ch // 2
        self.prior_cond = [int(self.sd[f"blocks.{l}.prior.NN.layers.0.layers.0.weight"].shape[1])
                           for l in range(self.nsplit)]

    # -- pieces --------------------------------------------------------------
    def coupling_nn(self, lvl, k, xa):
        return dense_block(xa, self.sd, f"blocks.{lvl}.flows.{2 * k + 1}.dense.", self.c_depth,
                           self.c_act)

    def couple_fwd(self, lvl, k, x):
        a = int(x.shape[1] * self.split)
        xa, xb = x[:, :a], x[:, a:]
        return torch.cat([xa, xb + round8(self.coupling_nn(lvl, k, xa), self.nbits)], dim=1)

    def couple_bwd(self, lvl, k, z):
        a = int(z.shape[1] * self.split)
        za, zb = z[:, :a], z[:, a:]
        return torch.cat([za, zb - round8(self.coupling_nn(lvl, k, za), self.nbits)], dim=1)

    def flows_fwd(self, lvl, x):
        for k in range(self.nflows):
            x = permute_fwd(x, self.sd[f"blocks.{lvl}.flows.{2 * k}.P"])
            x = self.couple_fwd(lvl, k, x)
        return permute_fwd(x, self.sd[f"blocks.{lvl}.flows.{2 * self.nflows}.P"])

    def flows_bwd(self, lvl, x):
        x = permute_bwd(x, self.sd[f"blocks.{lvl}.flows.{2 * self.nflows}.P"])
        for k in reversed(range(self.nflows)):
            x = self.couple_bwd(lvl, k, x)
            x = permute_bwd(x, self.sd[f"blocks.{lvl}.flows.{2 * k}.P"])
        return x

    def prior(self, lvl, inp):
        """priorlib.py:36-47. `inp` is what the reference passes to Prior.forward."""
        out_ch = self.sd[f"blocks.{lvl}.prior.NN.layers.{self.p_depth}.weight"].shape[0] // 2
        cond_ch = self.prior_cond[lvl]
        is_cond = self.name == "ConditionalFlows" or (lvl < self.nsplit - 1)
        x = inp if is_cond else torch.zeros_like(inp)
        del cond_ch
        params = dense_block(x, self.sd, f"blocks.{lvl}.prior.NN.", self.p_depth, self.p_act)
        return params[:, :out_ch], params[:, out_ch:]

    def cond_at(self, lvl, cond):
        if self.conv_for_cond:
            return F.conv2d(cond, self.sd[f"convs.{lvl}.weight"], self.sd[f"convs.{lvl}.bias"],
                            stride=2, padding=1)
        return extend_fwd(cond, self.scale)

    # -- model-level ---------------------------------------------------------
    @torch.no_grad()
    def forward(self, x, cond=None):
        """flows.py:87-116 (IDFlows) / :303-327 (ConditionalFlows)."""
        latents, means, logscales = [], [], []
        for lvl in range(self.nsplit):
            x = extend_fwd(x, self.scale)
            if cond is not None:
                cond = self.cond_at(lvl, cond)
            x = self.flows_fwd(lvl, x)
            if lvl < self.nsplit - 1:
                z, x = x[:, : x.shape[1] // 2], x[:, x.shape[1] // 2:]
                pin = x if cond is None else torch.cat((x, cond), 1)
            else:
                z = x
                pin = x if cond is None else torch.cat((torch.zeros_like(x), cond), 1)
            m, ls = self.prior(lvl, pin)
            latents.append(z)
            means.append(m)
            logscales.append(ls)
        return latents, means, logscales

    @torch.no_grad()
    def generated_from_latents(self, latents):
        """flows.py:139-152 (no priors: decoder given the latents)."""
        x = None
        for lvl in reversed(range(self.nsplit)):
            z = latents[lvl]
            x = z if lvl == self.nsplit - 1 else torch.cat((z, x), 1)
            x = self.flows_bwd(lvl, x)
            x = extend_bwd(x, self.scale)
        return x

    @torch.no_grad()
    def decode_levels(self, B, decode_level, cond=None):
        """True hierarchical decoder (flows.py:118-137 order, sampling replaced by
        `decode_level(lvl, mean, logscale) -> z`).  Returns the image and the
        per-level (mean, logscale) the decoder saw."""
        conds = []
        if cond is not None:
            c = cond
            for lvl in range(self.nsplit):
                c = self.cond_at(lvl, c)
                conds.append(c)
        x = None
        params = [None] * self.nsplit
        for lvl in reversed(range(self.nsplit)):
            if lvl == self.nsplit - 1:
                h, w = self.level_hw(lvl)
                zeros = torch.zeros((B, self.level_ch[lvl], h, w))
                pin = zeros if not conds else torch.cat((zeros, conds[lvl]), 1)
            else:
                pin = x if not conds else torch.cat((x, conds[lvl]), 1)
            m, ls = self.prior(lvl, pin)
            z = decode_level(lvl, m, ls)
            x = z if lvl == self.nsplit - 1 else torch.cat((z, x), 1)
            params[lvl] = (m, ls)
            x = self.flows_bwd(lvl, x)
            x = extend_bwd(x, self.scale)
        return x, params

    def level_hw(self, lvl):
        s = self.scale ** (lvl + 1)
        return self.H // s, self.W // s

    @torch.no_grad()
    def log_likelihood(self, latents, means, logscales):
        """flows.py:154-169 with DLogistic.log_prob (distlib.py:40-55)."""
        bins = 2 ** self.nbits
        lp = torch.zeros(latents[0].shape[0])
        for z, m, ls in zip(latents, means, logscales):
            s = torch.exp(ls)
            xp = (z + 0.5 / bins - m) / s
            xn = (z - 0.5 / bins - m) / s
            lfp, lfn = F.logsigmoid(xp), F.logsigmoid(xn)
            logp = lfp + torch.log(1 - torch.exp(lfn - lfp) + 1e-8)
            lp += logp.sum(dim=(1, 2, 3))
        return lp / (self.H * self.W * self.C)
