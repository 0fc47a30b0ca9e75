"""End-to-end lossless codec on the GPU: uint8 images <-> rANS bitstreams.

encode: dequant (trainer.py:101) -> IDF forward + priors (flows.py:87-116) ->
        rANS encode of every (image, level) stream (rans.pyx:37-67, the
        trainer's per-level reset contract trainer.py:310-315, one stream per
        image) -> word compaction.
decode: per level, top first: prior -> rANS decode (rans.pyx:69-110) -> flow
        inverse (flows.py:118-152) -> unsqueeze; then exact re-quantisation.

Streams are ordered level-major, image-minor; stream (l, b) covers the symbols
latents[l][b].reshape(-1) (NCHW order) exactly as a reference encode() call on
that slice would, and is bit-identical to it.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr

RANS_L = 1 << 32
MAGIC = b"IDFB"
VERSION = 2         # 2: flags always carry the conv arithmetic; version-1 files still read
FLAG_CONV_X3 = 1
# container flags bits 0-3: the conv arithmetic the flow ran (engine.conv_family); the decoder
# must run the same one.  Version 1 wrote 0 both for exact-f32 Winograd and for every engine
# that predates the field (halo / gemm / unfold / bf16): a version-1 file with flags 0 reads as
# conv "unrecorded", which any engine but a split-f16 one may decode (the pre-field behaviour).
# 6: round 4's dx3 (direct split-f16 only at widths a multiple of 16: engine mode 'dx3w16'; a
#    file the round-4 build wrote decodes exactly today: tests/golden/imagenet64_code6_r4.npz);
# 7: dx3 on every geometry conv3_dx3.hip packs (imagenet64's 8x8 level too); 8: bf16 engines on
# the bf16 direct conv (engine mode 'dxb'; 5 = conv3_bf16.hip)
CONV_CODES = {"f32": 0, "x3": 1, "halo": 2, "gemm": 3, "unfold": 4, "bf16": 5, "dx3w16": 6,
              "dx3": 7, "dxb": 8}
# the modes one engine switches between per bitstream (engine.can_run says which it has):
# split-f16 / exact-f32 for fp32 engines (engine.CONV_MODES), dxb / bf16 for bf16 engines
SWITCHABLE = ("dx3", "dx3w16", "x3", "f32", "dxb", "bf16")
SPLIT_F16 = ("dx3", "dx3w16", "x3")
CONV_NAMES = {v: k for k, v in CONV_CODES.items()}


@dataclass
class Bitstream:
    """Per-stream final rANS states + word counts + the concatenated words.
    Tensors live on the device that produced them (or the host after from_bytes)."""
    n_images: int
    level_shapes: list            # [(c, h, w)] per level
    states: torch.Tensor          # int64 view of u64 final states [n_streams]
    nwords: torch.Tensor          # int64 [n_streams]
    words: torch.Tensor           # int32 view of u32 words, stream-major, push order
    status: torch.Tensor | None = None
    meta: dict = field(default_factory=dict)
    # host (CPU int64) copy of nwords when the producer already had one (encode's compaction,
    # from_bytes, the multi-GPU exchanges): sizes and checks then never wait on the device.
    # It must equal nwords: assigning nwords drops it (the next nwords_host() reads the device
    # table again), and a copy whose length differs from nwords is dropped at construction.
    host_nwords: torch.Tensor | None = None

    def __post_init__(self):
        hn = self.host_nwords
        if hn is not None and hn.numel() != self.nwords.numel():
            object.__setattr__(self, "host_nwords", None)

    def __setattr__(self, name, value):
        object.__setattr__(self, name, value)
        if name == "nwords" and "host_nwords" in self.__dict__:
            object.__setattr__(self, "host_nwords", None)  # a new table: its host copy is stale

    def nwords_host(self) -> torch.Tensor:
        """nwords on the host: the kept copy, else one device->host read (cached)."""
        if self.host_nwords is None or self.host_nwords.numel() != self.nwords.numel():
            self.host_nwords = self.nwords.detach().to("cpu", torch.int64)
        return self.host_nwords

    @property
    def n_streams(self) -> int:
        return int(self.states.numel())

    def total_words(self) -> int:
        return int(self.words.numel())

    def bits(self) -> int:
        """The reference's accounting (trainer.py:326-327): 64 bits of state per
        stream + 32 bits per word."""
        return 64 * self.n_streams + 32 * self.total_words()

    def n_subpixels(self) -> int:
        return self.meta.get("n_subpixels", 0)

    def bpd(self) -> float:
        n = self.n_subpixels()
        return self.bits() / n if n else float("nan")

    def word_offsets(self) -> torch.Tensor:
        off = torch.zeros_like(self.nwords)
        if self.nwords.numel() > 1:
            off[1:] = torch.cumsum(self.nwords, 0)[:-1]
        return off

    # ---- container (the reference has no file format)
    def to_bytes(self) -> bytes:
        # flags bit 0: the flow's Winograd convs ran as split-f16 products (meta conv 'x3');
        # 0: exact-f32 (every stream written before the flag existed)
        conv = self.meta.get("conv", "f32")
        if conv not in CONV_CODES:
            raise ValueError(f"unknown conv mode {conv!r}"
                             + (": a version-1 file without the conv field cannot be rewritten"
                                " as version 2; re-encode it" if conv == "unrecorded" else ""))
        flags = CONV_CODES[conv]
        hdr = struct.pack("<4sHHIII", MAGIC, VERSION, flags, self.n_images, len(self.level_shapes),
                          self.n_streams)
        shapes = b"".join(struct.pack("<III", *s) for s in self.level_shapes)
        meta = struct.pack("<Q", self.n_subpixels())
        st = self.states.detach().cpu().numpy().astype("<i8").tobytes()
        nw = self.nwords.detach().cpu().numpy().astype("<u4").tobytes()
        w = self.words.detach().cpu().numpy().astype("<i4").tobytes()
        return hdr + shapes + meta + st + nw + w

    @classmethod
    def from_bytes(cls, buf: bytes, device=None) -> "Bitstream":
        magic, ver, flags, n_img, n_lvl, n_str = struct.unpack_from("<4sHHIII", buf, 0)
        if magic != MAGIC or ver not in (1, VERSION):
            raise ValueError("not an IDF bitstream")
        o = struct.calcsize("<4sHHIII")
        shapes = [struct.unpack_from("<III", buf, o + 12 * i) for i in range(n_lvl)]
        o += 12 * n_lvl
        (nsub,) = struct.unpack_from("<Q", buf, o)
        o += 8
        st = np.frombuffer(buf, "<i8", n_str, o).copy()
        o += 8 * n_str
        nw = np.frombuffer(buf, "<u4", n_str, o).astype(np.int64)
        o += 4 * n_str
        w = np.frombuffer(buf, "<i4", int(nw.sum()), o).copy()
        t = lambda a: torch.from_numpy(a).to(device) if device else torch.from_numpy(a)  # noqa: E731
        if (flags & 0xF) not in CONV_NAMES or flags >> 4:
            raise ValueError(f"unknown bitstream flags {flags:#x}")
        conv = "unrecorded" if ver == 1 and flags == 0 else CONV_NAMES[flags & 0xF]
        return cls(n_img, [tuple(s) for s in shapes], t(st), t(nw), t(w),
                   meta={"n_subpixels": int(nsub), "conv": conv},
                   host_nwords=torch.from_numpy(nw))


class StreamCoder:
    """Batched rANS over the engine's flat latent layout."""

    def __init__(self, engine):
        self.engine = engine
        self._off = {}
        self._lvl = {}
        self._dws = {}  # decode scratch per workspace slot (lanes decode concurrently)
        # when a list: (kind, n_symbols, n_streams, start, end) timing events around every
        # rANS launch pair (prep + serial pass) on the launch stream (bench.py)
        self.trace = None

    def _mark(self):
        if self.trace is None:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def sym_off(self, B: int) -> torch.Tensor:
        t = self._off.get(B)
        if t is None:
            offs = [0]
            for L in self.engine.levels:
                offs += [offs[-1] + L.n_sym * (b + 1) for b in range(B)]
            t = torch.tensor(offs, dtype=torch.int64, device=self.engine.device)
            self._off = {B: t}
        return t

    def encode(self, ws, B: int, compact: bool = True) -> Bitstream:
        eng = self.engine
        dev = eng.device
        s = _lib.stream_ptr(dev)
        off = self.sym_off(B)
        ns = off.numel() - 1
        nsym = B * eng.n_sym_img
        init = torch.full((ns,), RANS_L, dtype=torch.int64, device=dev)
        final = torch.empty(ns, dtype=torch.int64, device=dev)
        nwords = torch.empty(ns, dtype=torch.int64, device=dev)
        status = torch.empty(ns, dtype=torch.int32, device=dev)
        scratch = ws.get("words")
        if scratch is None or scratch.numel() < nsym:
            scratch = ws["words"] = torch.empty(nsym, dtype=torch.int32, device=dev)
        wbytes = lib().idf_rans_encode_workspace_bytes(nsym)
        wsp = ws.get("rans_ws")
        if wsp is None or wsp.numel() < wbytes:
            wsp = ws["rans_ws"] = torch.empty(wbytes, dtype=torch.uint8, device=dev)
        e0 = self._mark()
        check(lib().idf_rans_encode_streams(s, ns, nsym, ptr(off), ptr(ws["lat"]), ptr(ws["mean"]),
                                            ptr(ws["scale"]), ptr(init), ptr(final), ptr(scratch),
                                            ptr(nwords), ptr(status), ptr(wsp), wbytes),
              "rans encode")
        if e0 is not None:
            self.trace.append(("encode", nsym, ns, e0, self._mark()))
        shapes = [(L.z, L.h, L.w) for L in eng.levels]
        meta = {"n_subpixels": B * eng.C * eng.H * eng.W}
        if not compact:
            return Bitstream(B, shapes, final, nwords, scratch, status,
                             meta=dict(meta, scratch_offsets=off[:-1]))
        dst_off = torch.zeros_like(nwords)
        dst_off[1:] = torch.cumsum(nwords, 0)[:-1]
        nw_host = nwords.to("cpu")  # the one sync: the compacted size
        total = int(nw_host.sum())
        words = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
        check(lib().idf_gather_words(s, ns, ptr(off), ptr(nwords), ptr(dst_off), ptr(scratch),
                                     ptr(words)), "gather words")
        return Bitstream(B, shapes, final, nwords, words[:total], status, meta=meta,
                         host_nwords=nw_host)

    def level_encoder(self, B: int):
        """Per-level rANS encode overlapped with the flow: forward_pm calls .level(l, ws)
        once level l's latents and prior are written; that level's streams are encoded on a
        side stream while the flow computes the next levels (their buffers are disjoint).
        .finish(ws, compact) joins the side stream and compacts.  The streams are the same
        launches on the same data as encode(), per level, so the bitstream is identical."""
        return _LevelEncoder(self, B)

    def level_streams(self, B: int, l: int):
        """(first symbol of level l, its symbol count, device int64[B+1] stream offsets
        relative to that first symbol) -- a level's decode touches only its own symbols."""
        key = (B, l)
        hit = self._lvl.get(key)
        if hit is None:
            base = B * sum(L.n_sym for L in self.engine.levels[:l])
            n = self.engine.levels[l].n_sym
            rel = torch.arange(B + 1, dtype=torch.int64, device=self.engine.device) * n
            hit = (base, B * n, rel)
            self._lvl[key] = hit
        return hit

    def decode_level(self, bs: Bitstream, B: int, l: int, ws, word_off, out_state, out_status,
                     img0: int = 0, n_img: int | None = None, slot: int = 0):
        """Decodes level l of images [img0, img0 + n_img) of the B-image bitstream bs into
        ws (a workspace laid out for n_img images)."""
        eng = self.engine
        s = _lib.stream_ptr(eng.device)
        nb = B if n_img is None else n_img
        base, nsym, rel = self.level_streams(nb, l)
        k0 = l * B + img0
        wbytes = lib().idf_rans_decode_workspace_bytes(nsym)
        dws = self._dws.get(slot)
        if dws is None or dws.numel() < wbytes:
            dws = self._dws[slot] = torch.empty(wbytes, dtype=torch.uint8, device=eng.device)
        e0 = self._mark()
        check(lib().idf_rans_decode_streams(
            s, nb, nsym, ptr(rel), ptr(word_off) + 8 * k0, ptr(bs.nwords) + 8 * k0, ptr(bs.words),
            ptr(ws["mean"]) + 4 * base, ptr(ws["scale"]) + 4 * base, ptr(bs.states) + 8 * k0,
            ptr(out_state) + 8 * k0, ptr(ws["lat"]) + 4 * base, ptr(out_status) + 4 * k0,
            ptr(dws), wbytes), "rans decode")
        if e0 is not None:
            self.trace.append(("decode", nsym, nb, e0, self._mark()))


class _LevelEncoder:
    def __init__(self, coder: StreamCoder, B: int):
        self.coder, self.B = coder, B
        eng = coder.engine
        dev = eng.device
        self.off = coder.sym_off(B)
        ns = self.off.numel() - 1
        self.init = torch.full((ns,), RANS_L, dtype=torch.int64, device=dev)
        self.final = torch.empty(ns, dtype=torch.int64, device=dev)
        self.nwords = torch.empty(ns, dtype=torch.int64, device=dev)
        self.status = torch.empty(ns, dtype=torch.int32, device=dev)
        if getattr(coder, "_side", None) is None:
            coder._side = _lib.new_stream(dev)
        self.side = coder._side
        self.main = torch.cuda.current_stream(dev)
        self.scratch = self.wsp = None
        # every level's stream offsets are built here, on the main stream, before the first
        # event the side stream waits on: built lazily inside level() they would be written
        # after that event and the side-stream encode could read them unwritten
        for l in range(len(eng.levels)):
            coder.level_streams(B, l)

    def level(self, l: int, ws):
        coder, B = self.coder, self.B
        eng = coder.engine
        dev = eng.device
        nsym_all = B * eng.n_sym_img
        if self.scratch is None:  # on the main stream, before the first side launch
            sc = ws.get("words")
            if sc is None or sc.numel() < nsym_all:
                sc = ws["words"] = torch.empty(nsym_all, dtype=torch.int32, device=dev)
            self.scratch = sc
            nmax = B * max(L.n_sym for L in eng.levels)
            wb = lib().idf_rans_encode_workspace_bytes(nmax)
            wsp = ws.get("rans_ws")
            if wsp is None or wsp.numel() < wb:
                wsp = ws["rans_ws"] = torch.empty(wb, dtype=torch.uint8, device=dev)
            self.wsp = wsp
        base, nsym, rel = coder.level_streams(B, l)  # cached in __init__: no launch here
        ev = torch.cuda.Event()
        ev.record(self.main)
        self.side.wait_event(ev)
        k0 = l * B
        wbytes = lib().idf_rans_encode_workspace_bytes(nsym)
        with torch.cuda.stream(self.side):
            s = _lib.stream_ptr(dev)
            e0 = coder._mark()
            check(lib().idf_rans_encode_streams(
                s, B, nsym, ptr(rel), ptr(ws["lat"]) + 4 * base, ptr(ws["mean"]) + 4 * base,
                ptr(ws["scale"]) + 4 * base, ptr(self.init) + 8 * k0, ptr(self.final) + 8 * k0,
                ptr(self.scratch) + 4 * base, ptr(self.nwords) + 8 * k0,
                ptr(self.status) + 4 * k0, ptr(self.wsp), wbytes), "rans encode")
            if e0 is not None:
                coder.trace.append(("encode", nsym, B, e0, coder._mark()))

    def level_lane(self, l: int, ws, img0: int, n_img: int, wsp):
        """Level l of images [img0, img0 + n_img) from an encode lane's workspace (laid out
        for n_img images), encoded on the current (lane) stream into this encoder's stream
        arrays and word scratch at the images' places in the B-image layout: per stream the
        same launch arithmetic as level(), so the bitstream is identical."""
        coder, B = self.coder, self.B
        eng = coder.engine
        base, nsym, rel = coder.level_streams(n_img, l)  # lane-local symbols
        gbase = coder.level_streams(B, l)[0] + img0 * eng.levels[l].n_sym
        k0 = l * B + img0
        wbytes = lib().idf_rans_encode_workspace_bytes(nsym)
        s = _lib.stream_ptr(eng.device)
        e0 = coder._mark()
        check(lib().idf_rans_encode_streams(
            s, n_img, nsym, ptr(rel), ptr(ws["lat"]) + 4 * base, ptr(ws["mean"]) + 4 * base,
            ptr(ws["scale"]) + 4 * base, ptr(self.init) + 8 * k0, ptr(self.final) + 8 * k0,
            ptr(self.scratch) + 4 * gbase, ptr(self.nwords) + 8 * k0,
            ptr(self.status) + 4 * k0, ptr(wsp), wbytes), "rans encode")
        if e0 is not None:
            coder.trace.append(("encode", nsym, n_img, e0, coder._mark()))

    def join(self):
        """The main stream waits for every side-stream launch issued so far."""
        self.main.wait_stream(self.side)

    def finish(self, compact: bool = True) -> Bitstream:
        self.join()
        eng = self.coder.engine
        B, off, final, nwords, status = self.B, self.off, self.final, self.nwords, self.status
        scratch = self.scratch
        shapes = [(L.z, L.h, L.w) for L in eng.levels]
        meta = {"n_subpixels": B * eng.C * eng.H * eng.W}
        if not compact:
            return Bitstream(B, shapes, final, nwords, scratch, status,
                             meta=dict(meta, scratch_offsets=off[:-1]))
        ns = off.numel() - 1
        dst_off = torch.zeros_like(nwords)
        dst_off[1:] = torch.cumsum(nwords, 0)[:-1]
        nw_host = nwords.to("cpu")  # the one sync: the compacted size
        total = int(nw_host.sum())
        words = torch.empty(max(total, 1), dtype=torch.int32, device=eng.device)
        check(lib().idf_gather_words(_lib.stream_ptr(eng.device), ns, ptr(off), ptr(nwords),
                                     ptr(dst_off), ptr(scratch), ptr(words)), "gather words")
        return Bitstream(B, shapes, final, nwords, words[:total], status, meta=meta,
                         host_nwords=nw_host)


class ImageCodec:
    """uint8 NCHW images <-> Bitstream with a FlowEngine (IDFlows configs).

    Decode lanes (IDF_LANES / `lanes`, default 2): a batch of B >= 2 * LANE_MIN images
    decodes as `lanes` equal sub-batches, each on its own non-blocking HIP stream and
    workspace slot, lane i+1 waiting for lane i's top-level decode.  The rANS decode is a
    serial chain per stream that holds a few CUs for milliseconds; staggered lanes run one
    lane's decode beside the other lane's flow convs (imagenet64 B=256: decode 37.8 ->
    35.8 ms).  More than 2 lanes exceed the process's concurrent hardware queues
    (GPU_MAX_HW_QUEUES=4, one taken by the default stream) and serialize.  Exact: the convs
    are batch-invariant, so every stream decodes identically to the single-lane decode
    (tests/test_gpu_lanes.py)."""

    LANE_MIN = 8

    def __init__(self, engine, lanes: int | None = None):
        self.engine = engine
        self.coder = StreamCoder(engine)
        self.lanes = int(os.environ.get("IDF_LANES", "2")) if lanes is None else int(lanes)
        # encode lanes (IDF_ENC_LANES): the flow of a batch as equal sub-batches on the lanes'
        # streams (_encode_lanes); 1 = the one-pass encode with the side-stream level encode
        self.enc_lanes = int(os.environ.get("IDF_ENC_LANES", "1"))
        self._enc_scratch = None  # encode lanes: the B-image word scratch
        self._enc_wsp = []        # encode lanes: one rANS encode workspace per lane
        # per-level rANS encode on a side stream, overlapped with the next levels' flow
        self.overlap_encode = os.environ.get("IDF_ENC_OVERLAP", "1") == "1"
        self._streams = []
        self.lane_marks = None
        # resident workspace sets: every decode lane's, the pipelined encode's (ENC_SLOT) and
        # one more, so a pipelined step never evicts and reallocates a full-batch set
        if engine is not None:
            engine.ws_keep = max(engine.ws_keep, max(self.lanes, self.enc_lanes) + 2)

    # engine workspace slot of an encode that may run beside a decode on another stream (the
    # pipelined steps of bench.py run_steps_pipelined): the decode lanes and encode lanes hold
    # slots 0 .. lanes - 1, so this key is one no lane uses.  Shared between the two streams
    # (the caller must not switch conv modes while the other stream still enqueues): the
    # engine's block descriptors and conv mode (set_conv_mode, host state read at enqueue time),
    # its range_flag word, and the per-mode top-prior cache (engine._top_prior: kept for the
    # engine's lifetime, its users wait on the event recorded where it was computed).
    ENC_SLOT = -1

    @torch.no_grad()
    def encode(self, img_u8: torch.Tensor, cond=None, compact: bool = True,
               slot: int = 0) -> Bitstream:
        """slot: the engine workspace set the flow runs in (ENC_SLOT, a different one from the
        decode lanes', lets an encode overlap a decode on another stream: bench.py
        run_steps_pipelined; ENC_SLOT's comment lists the state the two share)."""
        _lib.require_device(img_u8, "image batch")
        if img_u8.dtype != torch.uint8:
            raise TypeError("ImageCodec.encode expects uint8 images")
        B = img_u8.shape[0]
        img_u8 = img_u8.contiguous()
        return self._encode_guarded(lambda: self.engine.load_u8(img_u8, slot), B, cond, compact,
                                    lanes_img=img_u8 if slot == 0 else None, slot=slot)

    def _encode_lanes(self, img_u8, B: int, nl: int, compact: bool) -> Bitstream:
        """Encode lanes (IDF_ENC_LANES): the batch's flow as nl equal sub-batches on the
        decode lanes' streams and workspace slots, their launches enqueued interleaved (one
        coupling of each lane in turn), each lane rANS-encoding its levels on its own stream
        into the shared B-image stream arrays; one lane's HBM-bound coupling heads and
        serial rANS chains then run beside the other lane's convs.  The convs are
        batch-invariant, so the bitstream equals the one-lane encode's bit for bit."""
        eng = self.engine
        dev = eng.device
        sz = [B // nl] * nl
        off = [sum(sz[:i]) for i in range(nl)]
        streams = self._lane_streams(nl)
        enc = self.coder.level_encoder(B)
        # everything the lanes share is built on the main stream before they fork: the word
        # scratch, per-lane rANS workspaces, every (size, level) stream-offset table, the top
        # prior
        nsym_all = B * eng.n_sym_img
        if self._enc_scratch is None or self._enc_scratch.numel() < nsym_all:
            self._enc_scratch = torch.empty(nsym_all, dtype=torch.int32, device=dev)
        enc.scratch = self._enc_scratch
        wb = lib().idf_rans_encode_workspace_bytes(sz[0] * max(L.n_sym for L in eng.levels))
        wsps = self._enc_wsp
        while len(wsps) < nl:
            wsps.append(torch.empty(0, dtype=torch.uint8, device=dev))
        for i in range(nl):
            if wsps[i].numel() < wb:
                wsps[i] = torch.empty(wb, dtype=torch.uint8, device=dev)
        self._enc_wsp = wsps
        for l in range(len(eng.levels)):
            self.coder.level_streams(sz[0], l)
        eng.ensure_top_prior(eng.workspace(sz[0], 0), _lib.stream_ptr(dev))
        main = torch.cuda.current_stream(dev)
        go = torch.cuda.Event()
        go.record(main)
        gens = []
        for i, st in enumerate(streams):
            st.wait_event(go)
            with torch.cuda.stream(st):
                eng.load_u8(img_u8[off[i]:off[i] + sz[i]], slot=i)
                gens.append(eng.forward_pm_steps(
                    sz[i], slot=i, on_level=lambda l, ws, i=i: enc.level_lane(
                        l, ws, off[i], sz[i], wsps[i])))
        live = list(range(nl))
        while live:
            for i in list(live):
                with torch.cuda.stream(streams[i]):
                    try:
                        next(gens[i])
                    except StopIteration:
                        live.remove(i)
        for st in streams:
            main.wait_stream(st)
        return enc.finish(compact=compact)

    def _encode_guarded(self, load, B, cond, compact, lanes_img=None, slot: int = 0):
        """Encode in the engine's conv mode; if the split-f16 range guard tripped (a value
        beyond its f16 range), recompute the batch with the exact-f32 convs.  The mode that
        produced the streams is recorded in the bitstream (meta['conv'], container flag)."""
        eng = self.engine
        mode = eng.conv_family
        if mode in SPLIT_F16:
            eng.clear_range_flag()
        nl = 1
        if lanes_img is not None and cond is None and not eng.conditional:
            nl = max(1, self.enc_lanes)
            while nl > 1 and (B % nl or B // nl < self.LANE_MIN):
                nl -= 1
            if nl > 1:
                try:
                    self._lane_streams(nl)
                except (OSError, AttributeError, _lib.IdfError):
                    nl = 1  # no separate HIP streams: one lane (same bitstream)
        enc = None
        if self.overlap_encode and nl == 1:
            try:
                enc = self.coder.level_encoder(B)
            except (OSError, AttributeError, _lib.IdfError):
                # no separate HIP stream available: the one-pass encode (same bitstream)
                self.overlap_encode = False
        if nl > 1:
            bs = self._encode_lanes(lanes_img, B, nl, compact)
        elif enc is not None:
            load()
            try:
                eng.forward_pm(B, cond=cond, slot=slot, on_level=enc.level)
            finally:
                # never free or reuse main-stream buffers while side launches may run
                enc.join()
            bs = enc.finish(compact=compact)
        else:
            ws = load()
            eng.forward_pm(B, cond=cond, slot=slot)
            bs = self.coder.encode(ws, B, compact=compact)
        if mode in SPLIT_F16 and eng.range_flag_tripped():
            eng.set_conv_mode("f32")
            try:
                ws = load()
                eng.forward_pm(B, cond=cond, slot=slot)
                bs = self.coder.encode(ws, B, compact=compact)
            finally:
                eng.set_conv_mode(mode)
            mode = "f32"
        bs.meta["conv"] = mode
        return bs

    @torch.no_grad()
    def encode_nchw(self, x: torch.Tensor, cond=None, compact: bool = True) -> Bitstream:
        """float NCHW input on the 1/256 grid (e.g. the residual data - rec of the residual
        configs, trainer.py:608) -> Bitstream."""
        _lib.require_device(x, "flow input")
        B = x.shape[0]
        xf = x.float().contiguous()
        return self._encode_guarded(lambda: self.engine.load_nchw(xf), B, cond, compact)

    @torch.no_grad()
    def decode_nchw(self, bs: Bitstream, cond=None, verify: bool = True):
        """inverse of encode_nchw -> (float NCHW, info)."""
        eng = self.engine
        x = torch.empty((bs.n_images, eng.C, eng.H, eng.W), dtype=torch.float32,
                        device=eng.device)
        info = self._decode_lanes(bs, cond,
                                  lambda i, b0, n, ws: eng.image_nchw(ws, n, out=x[b0:b0 + n]))
        if verify:
            info["ok"] = bool((info["final_states"] == RANS_L).all().item()) and not bool(
                (info["status"] & ~_lib.STREAM_WORDS_LEFT).any().item())
        return x, info

    def _n_lanes(self, B: int) -> int:
        n = max(1, self.lanes)
        while n > 1 and (B % n or B // n < self.LANE_MIN):
            n -= 1
        return n

    def _lane_sizes(self, B: int, n: int):
        """Images per lane: equal (measured best), or with 2 lanes lane 0 takes IDF_LANE_SPLIT
        of the batch (a smaller lane 0 runs ahead of lane 1; 112/144 decoded 1 ms slower)."""
        f = float(os.environ.get("IDF_LANE_SPLIT", "0.5"))
        if n == 2 and f != 0.5:
            n0 = max(self.LANE_MIN, min(B - self.LANE_MIN, int(round(B * f))))
            return [n0, B - n0]
        return [B // n] * n

    def _lane_streams(self, n: int):
        # IDF_LANE_PRIO=1: lane 0's stream at the device's greatest priority (timing A/B)
        prio = os.environ.get("IDF_LANE_PRIO", "0") == "1"
        while len(self._streams) < n:
            p = -1 if (prio and not self._streams) else None
            self._streams.append(_lib.new_stream(self.engine.device, priority=p))
        return self._streams[:n]

    def check_bitstream(self, bs: Bitstream):
        """Raises ValueError unless bs was produced by an engine of this geometry: the
        rANS decode indexes streams, word offsets and states by (level, image), so a
        truncated or foreign container would otherwise read device memory out of bounds."""
        eng = self.engine
        want = [(L.z, L.h, L.w) for L in eng.levels]
        if [tuple(int(v) for v in s) for s in bs.level_shapes] != want:
            raise ValueError(f"bitstream level shapes {bs.level_shapes} do not match the "
                             f"model's {want}")
        if bs.n_images < 0 or bs.n_streams != len(eng.levels) * bs.n_images:
            raise ValueError(f"bitstream holds {bs.n_streams} streams, expected "
                             f"{len(eng.levels)} levels x {bs.n_images} images")
        if bs.nwords.numel() != bs.n_streams:
            raise ValueError("bitstream word-count table does not match its stream count")
        nw_host = bs.nwords_host()
        if bool((nw_host < 0).any()):
            raise ValueError("bitstream has a negative word count")
        if "scratch_offsets" not in bs.meta:
            total = int(nw_host.sum()) if bs.n_streams else 0
            if total != bs.words.numel():
                raise ValueError(f"bitstream word table sums to {total} words, "
                                 f"{bs.words.numel()} present")
        conv, have = bs.meta.get("conv", "f32"), eng.conv_family
        if conv == "unrecorded":  # version-1 file, flags 0: any engine but split-f16
            if have in SPLIT_F16:
                raise ValueError("bitstream predates the conv field (version 1, flags 0) and "
                                 "was not coded with split-f16 convs; decode it with "
                                 "engine.set_conv_mode('f32') or the engine that wrote it")
            return
        if conv not in CONV_CODES:
            raise ValueError(f"unknown conv mode {conv!r}")
        switchable = conv in SWITCHABLE and have in SWITCHABLE and eng.can_run(conv)
        if conv != have and not switchable:
            raise ValueError(f"bitstream was coded with {conv!r} convs; this engine runs "
                             f"{have!r} (IDF_FOLD / IDF_WINO / IDF_HALO / precision differ): "
                             "its couplings would not invert bit-exactly")

    def _prep_decode(self, bs: Bitstream):
        self.check_bitstream(bs)
        dev = self.engine.device
        if bs.states.device != dev:
            bs = Bitstream(bs.n_images, bs.level_shapes, bs.states.to(dev), bs.nwords.to(dev),
                           bs.words.to(dev), None, bs.meta, bs.host_nwords)
        word_off = bs.meta.get("scratch_offsets")
        if word_off is None:
            word_off = bs.word_offsets()
        if bs.words.numel() == 0:
            bs.words = torch.zeros(1, dtype=torch.int32, device=dev)
        out_state = torch.empty_like(bs.states)
        out_status = torch.zeros(bs.n_streams, dtype=torch.int32, device=dev)
        return bs, word_off, out_state, out_status

    def _decode_lanes(self, bs: Bitstream, cond, finish):
        """Runs the top-down decode of bs in lanes; finish(i, img0, n, ws) is issued on lane
        i's stream after its flows.  Returns the decode info."""
        eng = self.engine
        B = bs.n_images
        bs, word_off, out_state, out_status = self._prep_decode(bs)
        nl = self._n_lanes(B)
        if nl > 1:
            try:
                self._lane_streams(nl)
            except (OSError, AttributeError, _lib.IdfError):
                nl = 1  # no separate HIP streams: decode in one lane (same bits)
        sz = self._lane_sizes(B, nl)
        off = [sum(sz[:i]) for i in range(nl)]
        # the convs must run as the encoder ran them (bit-identical couplings)
        mode, prev = bs.meta.get("conv", "f32"), eng.conv_mode
        if mode not in SWITCHABLE:  # a fixed family, checked equal in check_bitstream
            mode = prev
        if mode != prev:
            eng.set_conv_mode(mode)
        try:
            if nl == 1:
                def dec(l, ws):
                    self.coder.decode_level(bs, B, l, ws, word_off, out_state, out_status)
                ws = eng.inverse_pm(B, dec, cond=cond)
                finish(0, 0, B, ws)
            else:
                main = torch.cuda.current_stream(eng.device)
                eng.ensure_top_prior(eng.workspace(sz[0], 0), _lib.stream_ptr(eng.device))
                # every lane's per-level stream offsets are built here, on the main stream,
                # before `go`: built lazily, lane 0 would create the (size, level) entry on its
                # own stream and lane 1 -- same size -- read it from another stream, unordered
                # (level 0 of lane 1 decoded from unwritten offsets: a race seen at 2 x 1024)
                for n_i in set(sz):
                    for l in range(eng.nsplit):
                        self.coder.level_streams(n_i, l)
                go = torch.cuda.Event()
                go.record(main)
                top = eng.nsplit - 1
                # IDF_LANE_STAGGER: "top" -- lane i+1 starts after lane i's top-level
                # rANS decode; "levels" -- also every other level's decode waits for lane i's
                # decode of that level; "none" -- no cross-lane order.  The lanes drift
                # together after the top level (the GPU ran only rANS kernels for 3.7 ms of a
                # 31 ms decode), but neither "levels", a high-priority lane 0 nor unequal lanes
                # (IDF_LANE_SPLIT) shortened the decode (profiles/r02/lanes/order_ab.txt).
                # "flows0": as "top", and at the bottom level lane i's couplings start when lane
                # i-1's are done, so lane i's longest rANS decode runs beside lane i-1's
                # couplings (round 3's default: +0.5-0.9% bench with four streams per decode
                # block, profiles/r03/lanes_flows); "flows" orders every level so (-2.7%).
                # "top" is the default again since the decode runs two streams per block (a
                # faster chain, profiles/r04/rans_wpb): back-to-back decode 27.6 vs 28.0 ms,
                # bench +0.7% pipelined / +1.2% back to back, same box
                # (profiles/r04/lane_stagger/).
                stagger = os.environ.get("IDF_LANE_STAGGER", "top")
                # The host enqueues the lanes interleaved -- one step (a level's rANS decode, or
                # one coupling) of each lane in turn -- so that every lane's launches reach the
                # GPU early: enqueued lane after lane, the second lane's first kernel waited for
                # the host to issue all ~500 launches of the first (profiles/r02/lanes/).  Every
                # lane has the same steps, so lane i-1's decode of a level is enqueued (its
                # event recorded) before lane i's waits on it.
                gens, streams = [], self._lane_streams(nl)
                done = [dict() for _ in range(nl)]  # done[i][l]: lane i decoded level l
                prior_done = [None] * nl  # flows: lane i's bottom-level prior enqueued
                flows = stagger.startswith("flows")
                together = stagger == "none" or stagger == "flows"  # every top decode at once
                for i, st in enumerate(streams):
                    st.wait_event(go if (not together or i == 0) else first)
                    if i == 0:
                        first = go
                    if self.lane_marks is not None:  # lane start times (tools/lanes_probe.py)
                        m = torch.cuda.Event(enable_timing=True)
                        m.record(st)
                        self.lane_marks.append(m)
                    staggered = torch.cuda.Event()

                    def dec(l, ws, i=i, st=st, ev=staggered):
                        if flows and l == 0 and i + 1 < nl:  # the next lane's bottom prior
                            prior_done[i] = torch.cuda.Event()
                            prior_done[i].record(st)
                        if stagger == "levels" and i > 0 and l != top:
                            st.wait_event(done[i - 1][l])
                        self.coder.decode_level(bs, B, l, ws, word_off, out_state, out_status,
                                                img0=off[i], n_img=sz[i], slot=i)
                        if l == top:
                            ev.record(st)
                        elif stagger == "levels":
                            done[i][l] = torch.cuda.Event()
                            done[i][l].record(st)
                    def pre(l, i=i, st=st):
                        # flows orders: lane i's bottom prior after lane i-1's, so it runs
                        # beside lane i-1's bottom rANS decode instead of beside its prior
                        if flows and l == 0 and i > 0 and top > 0:
                            st.wait_event(prior_done[i - 1])
                    ci = None if cond is None else cond[off[i]:off[i] + sz[i]].contiguous()
                    gens.append(eng.inverse_pm_steps(sz[i], dec, cond=ci, slot=i, pre_prior=pre))
                    # lane i's first step (its top level's rANS decode) is enqueued before lane
                    # i + 1 waits on the event it records
                    with torch.cuda.stream(st):
                        next(gens[i])
                    go = staggered
                live = list(range(nl)) if not flows else []
                if flows:
                    # "flows": lane i's couplings of a level start once lane i-1's couplings of
                    # that level are done, so a lane's prior + rANS decode of the next level
                    # runs beside the other lane's couplings instead of beside its own rANS
                    # decode (the lanes otherwise drift into phase and both decode a level's
                    # streams at once, with the chip idle: profiles/r03/lanes_q).  Host order:
                    # level by level, lane by lane.  "flows0": only the bottom level (the
                    # longest rANS chains, the largest couplings) is ordered so; the others
                    # step round-robin as in "top".
                    flows_done = [None] * nl
                    for lv in range(eng.nsplit):
                        ordered = stagger == "flows" or top - lv == 0
                        if ordered:
                            for i, st in enumerate(streams):
                                with torch.cuda.stream(st):
                                    if lv:  # the previous level's unsqueeze, this level's decode
                                        next(gens[i])
                                    if i:
                                        st.wait_event(flows_done[i - 1])
                                    for _ in range(eng.nflows):
                                        next(gens[i])
                                    flows_done[i] = torch.cuda.Event()
                                    flows_done[i].record(st)
                        else:  # round robin, one step of each lane in turn
                            for k in range(eng.nflows + (1 if lv else 0)):
                                for i, st in enumerate(streams):
                                    with torch.cuda.stream(st):
                                        next(gens[i])
                    for i, st in enumerate(streams):
                        with torch.cuda.stream(st):
                            try:
                                next(gens[i])
                                raise RuntimeError("decode lane did not finish after its levels")
                            except StopIteration as lane_done:
                                finish(i, off[i], sz[i], lane_done.value)
                while live:
                    for i in list(live):
                        with torch.cuda.stream(streams[i]):
                            try:
                                next(gens[i])
                            except StopIteration as lane_done:
                                # the lane's own workspace (a fresh cache lookup could hand
                                # back a different, uninitialised set once the cache evicts)
                                finish(i, off[i], sz[i], lane_done.value)
                                live.remove(i)
                for st in streams:
                    main.wait_stream(st)
        finally:
            if mode != prev:
                eng.set_conv_mode(prev)
        return {"final_states": out_state, "status": out_status}

    @torch.no_grad()
    def decode(self, bs: Bitstream, cond=None, verify: bool = True):
        eng = self.engine
        img = torch.empty((bs.n_images, eng.C, eng.H, eng.W), dtype=torch.uint8,
                          device=eng.device)
        bad = torch.zeros(1, dtype=torch.int32, device=eng.device)
        info = self._decode_lanes(
            bs, cond, lambda i, b0, n, ws: eng.image_u8(ws, n, out=img[b0:b0 + n], bad=bad))
        info["off_grid"] = bad
        if verify:
            ok = bool((info["final_states"] == RANS_L).all().item()) and int(bad.item()) == 0
            info["ok"] = ok and not bool((info["status"] & ~_lib.STREAM_WORDS_LEFT).any().item())
        return img, info
