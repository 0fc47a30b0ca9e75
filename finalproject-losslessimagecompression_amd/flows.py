"""Flow models (mirror of flows.py:19-361): IDFlows and ConditionalFlows with the
reference's constructor kwargs, registry names, submodule tree and parameter
creation order -- the same YAML configs build them, the same state_dicts load,
and `random.seed(0); torch.manual_seed(0)` gives the same initial weights.

forward / generated_from_latents / log_likelihood keep the reference
signatures; the whole pass runs in idfcodec.FlowEngine (HIP kernels, pixel-major
activations, one feature buffer per DenseBlock).  encode / decode -- empty
placeholders in the reference (flows.py:177-181) -- are the real lossless codec
here: uint8 images <-> rANS bitstreams (idfcodec.codec).

TwoLevelFlows (flows.py:184-274) is not used by any north-star config and is
out of scope; it is registered so configs naming it fail with a
clear message.
"""
from copy import deepcopy

import torch
from torch import nn

import moduleregister
from couplelib import NNCouple  # noqa: F401  (registers AdditiveCouple)
from distlib import NNDistribution
from extenddim import ExtendDim, NNExtendDim
from invertible import InvertibleModuleList, Permute
from priorlib import NNPrior
from roundlib import NNRound, Round  # noqa: F401
from idfcodec._lib import require_device


class NNFlows(moduleregister.Register):
    def __init__(self):
        super().__init__()


@NNFlows.register
class IDFlows(nn.Module):
    def __init__(self, nflows=8, nbits=8, nsplit=3, H=64, W=64, C=3, couple=None, extenddim=None,
                 prior=None, distribution=None, round=None, batch_squeeze=0):
        super().__init__()
        self.nflows = nflows
        self.nbits = nbits
        self.nsplit = nsplit
        self.blocks = nn.ModuleList()
        self.latents_shape = []
        self.C, self.H, self.W = C, H, W
        couple, extenddim, prior = dict(couple), dict(extenddim), dict(prior)
        distribution, round = dict(distribution), dict(round)
        self.couple_type = NNCouple.get(couple.pop("name"))
        self.prior_type = NNPrior.get(prior.pop("name"))
        self.extenddim_type = NNExtendDim.get(extenddim.pop("name"))
        self.dist_type = NNDistribution.get(distribution.pop("name"))
        self.round_type = NNRound.get(round.pop("name"))
        self.batch_squeeze = batch_squeeze
        channel = C * batch_squeeze if batch_squeeze else C
        h, w = H, W
        s = extenddim.get("scale")
        for split_level in range(nsplit):
            channel *= s * s
            h //= s
            w //= s
            flow_module = InvertibleModuleList()
            for _ in range(nflows):
                flow_module.append(Permute(dim=channel))
                flow_module.append(self.couple_type(channel=channel, **deepcopy(couple)))
            flow_module.append(Permute(dim=channel))
            if split_level < nsplit - 1:
                prior_nn = self.prior_type(channel // 2, channel - channel // 2, **deepcopy(prior))
                self.latents_shape.append((channel // 2, h, w))
                channel -= channel // 2
            else:
                prior_nn = self.prior_type(channel, 0, **deepcopy(prior))
                self.latents_shape.append((channel, h, w))
            self.blocks.append(nn.ModuleDict(dict(
                extend=self.extenddim_type(**deepcopy(extenddim)), flows=flow_module, prior=prior_nn)))
        self.dist = self.dist_type(**distribution)
        self.round = self.round_type(**round)
        self._engine = None
        self._engine_key = None

    # ------------------------------------------------------------ engine
    def engine(self):
        """The device engine for the current parameters (rebuilt when they change)."""
        from idfcodec.engine import FlowEngine
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("idfcodec: move the model to the HIP device (.cuda()) first; "
                               "there is no CPU path")
        key = tuple((p.data_ptr(), p._version) for p in self.parameters()) + (
            getattr(self, "idf_precision", "f32"),)
        if self._engine is None or self._engine_key != key:
            self._engine = FlowEngine(self, dev)
            self._engine_key = key
        return self._engine

    def codec(self):
        from idfcodec.codec import ImageCodec
        eng = self.engine()
        if getattr(self, "_codec", None) is None or self._codec.engine is not eng:
            self._codec = ImageCodec(eng)
        return self._codec

    def _check_batch_squeeze(self):
        if self.batch_squeeze:
            raise NotImplementedError("batch_squeeze (flows.py:92-95) is not used by the north-star "
                                      "configs and is not implemented")

    # ------------------------------------------------------------ reference API
    def forward(self, x, logv):
        """flows.py:87-116 -> (latents, means, logscales, logv), NCHW per level."""
        require_device(x, "IDFlows input")
        self._check_batch_squeeze()
        eng = self.engine()
        B = x.shape[0]
        ws = eng.load_nchw(x)
        eng.forward_pm(B)
        lat = [t.clone() for t in eng.level_views(ws, B, "lat")]
        mean = [t.clone() for t in eng.level_views(ws, B, "mean")]
        logs = [t.clone() for t in eng.level_views(ws, B, "logscale")]
        return lat, mean, logs, logv

    def generated_from_latents(self, latents):
        """flows.py:139-152: invert the flows given every level's latent."""
        self._check_batch_squeeze()
        eng = self.engine()
        B = latents[0].shape[0]

        def put(l, ws):
            eng.level_views(ws, B, "lat")[l].copy_(latents[l])

        ws = eng.inverse_pm(B, put, priors=False)
        return eng.image_nchw(ws, B)

    def generated_from_noise(self, latents):
        """flows.py:118-137 (sampling/visualisation; not on the coding path)."""
        eng = self.engine()
        B = latents[0].shape[0]

        def put(l, ws):
            m = eng.level_views(ws, B, "mean")[l]
            ls = eng.level_views(ws, B, "logscale")[l]
            z = latents[l].to(m.device) * torch.exp(ls) + m
            eng.level_views(ws, B, "lat")[l].copy_(torch.round(z * 256) / 256)

        ws = eng.inverse_pm(B, put, priors=True)
        return eng.image_nchw(ws, B)

    def log_likelihood(self, latents, means, logscales):
        """flows.py:154-169: per image, the log-probabilities of every level summed (per-level
        means in log_Ps), divided by H*W*C -- one idf_log_prob launch per level, the
        per-(level, image) sums reduced on the device in a fixed order (f64)."""
        from distlib import DLogistic, dlogistic_log_prob
        if not isinstance(self.dist, DLogistic):
            raise NotImplementedError("log_likelihood supports the DLogistic prior only")
        B = latents[0].shape[0]
        dev = latents[0].device
        require_device(latents[0], "latents")
        total = torch.zeros(B, dtype=torch.float64, device=dev)
        log_Ps = []
        for z, m, ls in zip(latents, means, logscales):
            z, m, ls = torch.broadcast_tensors(z.to(dev), m.to(dev), ls.to(dev))
            sums = dlogistic_log_prob(z, m, ls, self.nbits, groups=B)
            log_Ps.append((sums / (z.numel() // B)).float())
            total += sums
        return (total / (self.H * self.W * self.C)).float(), log_Ps

    def inverse(self):
        for block in self.blocks:
            block["extend"].inverse()
            for flow in block["flows"]:
                flow.inverse()

    # ------------------------------------------------------------ the codec
    def encode(self, x):
        """uint8 images [B, C, H, W] (device) -> idfcodec.Bitstream."""
        return self.codec().encode(x)

    def decode(self, bitstream, verify=True):
        """Bitstream -> (uint8 images, info) -- exact inverse of encode()."""
        return self.codec().decode(bitstream, verify=verify)


@NNFlows.register
class TwoLevelFlows(nn.Module):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("TwoLevelFlows (flows.py:184-274) is out of scope: no north-star "
                                  "config uses it (SURVEY.md 2)")


@NNFlows.register
class ConditionalFlows(IDFlows):
    """flows.py:277-361: priors see cat(x, cond) where cond is the VQ-VAE
    reconstruction squeezed (conv_for_cond False) or passed through stride-2
    convs (conv_for_cond True)."""

    def __init__(self, conv_for_cond=False, *args, **kwargs):
        super().__init__(*args, **kwargs)
        ch = self.C
        self.conv_for_cond = conv_for_cond
        if conv_for_cond:
            self.convs = nn.ModuleList()
        # the reference's IDFlows.__init__ popped 'name' from kwargs['prior'] in place
        prior_kw = {k: v for k, v in dict(kwargs.get("prior")).items() if k != "name"}
        for split_level in range(self.nsplit):
            block = self.blocks[split_level]
            scale = block["extend"].scale
            ch *= scale * scale
            prior = block["prior"]
            block["prior"] = self.prior_type(
                prior.out_channel,
                prior.cond_channel + ch if prior.cond_channel > 0 else prior.out_channel + ch,
                **deepcopy(prior_kw))
            if conv_for_cond:
                self.convs.append(nn.Conv2d(ch // scale // scale, ch, 4, 2, 1))

    def forward(self, x, logv, cond):
        require_device(x, "ConditionalFlows input")
        eng = self.engine()
        B = x.shape[0]
        ws = eng.load_nchw(x)
        eng.forward_pm(B, cond=cond.contiguous().float())
        lat = [t.clone() for t in eng.level_views(ws, B, "lat")]
        mean = [t.clone() for t in eng.level_views(ws, B, "mean")]
        logs = [t.clone() for t in eng.level_views(ws, B, "logscale")]
        return lat, mean, logs, logv

    def encode(self, x, cond):
        return self.codec().encode(x, cond=cond.contiguous().float())

    def decode(self, bitstream, cond, verify=True):
        return self.codec().decode(bitstream, cond=cond.contiguous().float(), verify=verify)
