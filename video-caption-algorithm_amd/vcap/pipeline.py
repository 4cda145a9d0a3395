"""Two-stream caption pipeline: the ViT encode of batch k+1 overlaps the GPT-2 decode of batch k.

The encode is MFMA-bound and fills the chip; the decode is a latency-bound chain of small
kernels (one hipGraph per batch) that leaves most CUs idle.  Running them on separate HIP
streams lets the decode graph's workgroups interleave with the encode GEMMs, so steady-state
time per batch approaches max(encode, decode) instead of their sum.  Every batch still gets its
full encode + prefix + decode; double-buffered prefix/ids buffers and events keep batch k+2's
encode from overwriting buffers batch k's decode still reads.

`dec_lanes` > 1 keeps that many decodes in flight at once (decode group g on lane g % dec_lanes,
each lane its own stream, KV/scratch workspace and captured graph).  A decode is a chain of ~60
dependent launches per token that occupies a fraction of the CUs it is given, so a second
independent chain fills the gaps of the first.

`dec_group` > 1 decodes that many consecutive encode batches together as one decode of
dec_group * B rows: the decode step is latency-bound, so 16 rows cost ~8 % more than 8 rows per
token step (every step streams the 247 MB of weights once instead of once per batch).  Rows are
independent in every decode kernel (per-row MFMA outputs, per-row processors), so a batch's ids
are bit-identical whichever group it is decoded in (tests/test_gpu_bf16.py).  The price is latency:
a batch waits for the next batch's encode before its decode starts.

`enc_group` > 1 (a divisor of dec_group) encodes that many consecutive batches as one encode of
enc_group * B videos: each submitted batch is copied into a staging buffer and the group's last
submission launches the encode.  The ViT's N = 768 GEMMs (attn-proj, fc2) leave most of a
second 256-tile round idle at B = 8 (297 tiles on 256 CUs); at 16 videos the rounds fill.  Every
encode kernel computes each row independently of M (the CLS-tail split-K plan depends on K only),
so a video's prefix - and its caption - is bit-identical whichever batch it is encoded in.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

import atexit
import ctypes as C

import torch

from . import _native as N
from . import trace
from .model import GenConfig, HipGPT2Decoder, HipPrefix, HipViTEncoder, _Workspace


# One set of streams per (device, reservation, confinement, lanes) for the whole process, reused by
# every pipeline with that schedule.  Measured: pipelines that each created fresh streams after
# earlier ones had been closed sometimes ran serialised - an 8-video schedule following another in
# one bench process read 291 instead of ~1090 captions/s (profiles/r04_stream_reuse.txt) - most
# likely their encode stream and a decode lane sharing one of the process's 4 hardware queues
# (streams are spread over them in creation order).  Reusing the first set keeps the queue layout
# every measurement was taken with.
_STREAM_SETS: dict = {}


def _device_index(device) -> int:
    d = torch.device(device)
    return d.index if d.index is not None else torch.cuda.current_device()


def _stream_set(device, reserve_cus: int, confine_decode, lanes: int):
    """confine_decode: False = decode lanes unmasked; True = masked to the reserved CUs; an int n > 1 =
    masked to the first n CUs (the reserved ones plus n - reserve_cus of the encode's)."""
    device = torch.device("cuda", _device_index(device))   # 'cuda' = the current device, resolved once
    ndec = reserve_cus if confine_decode is True else int(confine_decode or 0)
    key = (device.index, reserve_cus, ndec, lanes)
    if key in _STREAM_SETS:
        return _STREAM_SETS[key][:2]
    lo, hi = torch.cuda.Stream.priority_range()
    handles = []
    with torch.cuda.device(device):
        if reserve_cus > 0:
            # the encode kept off `reserve_cus` CUs (a CU-masked stream) so the decode always finds some
            h = C.c_void_p()
            N.check(N.lib().vcap_stream_create_cu_reserved(int(reserve_cus), C.byref(h)), "masked stream")
            handles.append(h.value)
            s_enc = torch.cuda.ExternalStream(h.value, device=device)
        else:
            s_enc = torch.cuda.Stream(device, priority=lo)
        if ndec > 0:
            # decode streams masked to the reserved CUs (plus, for ndec > reserve_cus, some of the
            # encode's): decode workgroups never take the other encode CUs between two GEMM workgroups
            words = (torch.cuda.get_device_properties(device).multi_processor_count + 31) // 32
            mask = (C.c_uint32 * words)()
            for c in range(ndec):
                mask[c // 32] |= 1 << (c % 32)
            s_decs = []
            for _ in range(lanes):
                h = C.c_void_p()
                N.check(N.lib().vcap_stream_create_cu_mask(mask, words, C.byref(h)), "decode stream")
                handles.append(h.value)
                s_decs.append(torch.cuda.ExternalStream(h.value, device=device))
        else:
            # the decode chain is latency-bound: its lanes get the higher priority (normal priority
            # measured the same, 1224-1228 captions/s either way, r03)
            s_decs = [torch.cuda.Stream(device, priority=hi) for _ in range(lanes)]
    _STREAM_SETS[key] = (s_enc, s_decs, handles)
    return s_enc, s_decs


def release_streams() -> None:
    """Destroy the CU-masked streams of every cached stream set (after all pipelines are closed).
    Registered with atexit when the first set is created; callers may run it earlier."""
    for s_enc, s_decs, handles in _STREAM_SETS.values():
        s_enc.synchronize()
        for s in s_decs:
            s.synchronize()
        for h in handles:
            N.check(N.lib().vcap_stream_destroy(h), "stream destroy")
    _STREAM_SETS.clear()


def _release_at_exit() -> None:
    try:
        if _STREAM_SETS and torch.cuda.is_initialized():
            release_streams()
    except Exception:   # interpreter shutdown: never turn a clean exit into a failure
        pass


atexit.register(_release_at_exit)


class CaptionPipeline:
    def __init__(self, encoder: HipViTEncoder, prefix: HipPrefix, decoder: HipGPT2Decoder, cfg: GenConfig,
                 batch: int, prompt_ids: Sequence[int], device, depth: int = 2, gather=None,
                 reserve_cus: int = 0, dec_lanes: int = 1, confine_decode: Union[bool, int] = False, dec_group: int = 1,
                 enc_group: int = 1):
        self.enc, self.pre, self.dec, self.cfg = encoder, prefix, decoder, cfg
        self.prompt_ids = list(prompt_ids)
        self.device = torch.device("cuda", _device_index(device))
        if dec_lanes < 1 or dec_group < 1 or enc_group < 1:
            raise ValueError("dec_lanes, dec_group and enc_group must be >= 1")
        if dec_group % enc_group:
            raise ValueError(f"enc_group ({enc_group}) must divide dec_group ({dec_group})")
        self.lanes = int(dec_lanes)
        self.group = int(dec_group)
        self.egroup = int(enc_group)
        self._stage = None            # [enc_group * B, T, 3, H, W] staging buffer (enc_group > 1)
        self._staged = 0              # batches copied into it since the last encode
        self._pending_mid: List[torch.cuda.Event] = []
        self.batch = int(batch)
        depth = max(int(depth), self.lanes + 1)   # one slot being encoded + one per decoding lane
        self.depth = depth
        # The decode chain is latency-bound: give its stream the higher priority so its small
        # workgroups are dispatched as soon as encode GEMM workgroups retire, and optionally keep
        # the encode off `reserve_cus` CUs (a CU-masked stream) so the decode always finds some.
        self.s_enc, self.s_decs = _stream_set(self.device, int(reserve_cus),
                                              confine_decode if isinstance(confine_decode, bool) else int(confine_decode),
                                              self.lanes)
        self.s_dec = self.s_decs[0]
        # the encoder / decoder workspaces are shared with serial calls made on the creating stream:
        # nothing of the pipeline may start before that stream's pending work has finished
        cur = torch.cuda.current_stream(self.device)
        for st in [self.s_enc] + self.s_decs:
            st.wait_stream(cur)
        self.dec_ws = [decoder.ws] + [_Workspace(self.device) for _ in range(self.lanes - 1)]
        E = decoder.arch.n_embd
        G = self.group
        # slot = one decode group: G consecutive batches' prefixes side by side, decoded as G*B rows
        self.group_prefix = [torch.empty(G * batch, prefix.prefix_len, E, device=self.device) for _ in range(depth)]
        self.group_ids = [torch.empty(G * batch, cfg.max_new_tokens, dtype=torch.int32, device=self.device)
                          for _ in range(depth)]
        self.enc_done = [torch.cuda.Event() for _ in range(depth)]
        self.dec_done: List[Optional[torch.cuda.Event]] = [None] * depth
        self.gather = gather          # optional callable(ids, first_k) -> ids, run on the decode stream
        self.outputs: List[Optional[torch.Tensor]] = [None] * (depth * G)
        self._pending_end: List[torch.cuda.Event] = []
        self.k = 0

    @property
    def prefix_bufs(self) -> List[torch.Tensor]:
        """Per-submission-slot prefix views (slot = k % (depth * dec_group))."""
        B = self.batch
        return [gp[j * B:(j + 1) * B] for gp in self.group_prefix for j in range(self.group)]

    def submit(self, video: torch.Tensor, t_start: Optional[torch.cuda.Event] = None,
               t_mid: Optional[torch.cuda.Event] = None, t_end: Optional[torch.cuda.Event] = None) -> int:
        """Encode one batch; launch the decode of its group once the group's last batch is encoded.
        Returns the submission slot for result() (k % (depth * dec_group)).  With dec_group > 1,
        t_end of a batch is recorded after its GROUP's decode; `gather(ids, first_k)` receives the
        group's [G*B, L] ids and the submission index of its first batch."""
        G, B, E = self.group, self.batch, self.egroup
        g, j = divmod(self.k, G)
        slot = g % self.depth
        with torch.cuda.stream(self.s_enc):
            if j == 0 and self.dec_done[slot] is not None:
                self.s_enc.wait_event(self.dec_done[slot])   # buffers of group g-depth are free
            if t_start is not None:
                t_start.record()
            if t_mid is not None:
                self._pending_mid.append(t_mid)
            if E == 1:
                self._encode(video, slot, j, 1)
            else:
                if self._stage is None or self._stage.shape[1:] != video.shape[1:] or self._stage.dtype != video.dtype:
                    self._stage = torch.empty((E * B,) + tuple(video.shape[1:]), dtype=video.dtype, device=self.device)
                self._stage[self._staged * B:(self._staged + 1) * B].copy_(video)
                self._staged += 1
                if self._staged == E:
                    self._encode(self._stage, slot, j - E + 1, E)
        if t_end is not None:
            self._pending_end.append(t_end)
        self.k += 1
        self.last_slot = slot * G + j
        if j == G - 1:
            self._decode_group(g)
        return self.last_slot

    def _encode(self, video: torch.Tensor, slot: int, j0: int, n: int) -> None:
        """Encode n staged batches (on the encode stream) into submission positions j0.. of slot."""
        B = self.batch
        # (roctx, off unless trace.enable(): the fused encode also runs the Cross_Modal_Alignment
        # kernels - final LN, proj, engine LN-scale, mapper - at its tail)
        with trace.range(trace.VIT):
            self.enc.encode(video[:n * B], self.pre, out_prefix=self.group_prefix[slot][j0 * B:(j0 + n) * B])
        for ev in self._pending_mid:
            ev.record()
        self._pending_mid = []
        self.enc_done[slot].record()
        self._staged = 0

    def flush(self) -> None:
        """Decode a partially filled group now (its unfilled rows hold stale prefixes; their ids
        are ignored).  Called before waiting on results when k is not a multiple of dec_group."""
        if self.k % self.group:
            g = self.k // self.group
            if self._staged:
                with torch.cuda.stream(self.s_enc):
                    j = self.k % self.group
                    self._encode(self._stage, g % self.depth, j - self._staged, self._staged)
            self.k = (g + 1) * self.group
            self._decode_group(g)

    def _decode_group(self, g: int) -> None:
        G, B = self.group, self.batch
        slot, lane = g % self.depth, g % self.lanes
        s_dec = self.s_decs[lane]
        with torch.cuda.stream(s_dec):
            s_dec.wait_event(self.enc_done[slot])
            with trace.range(trace.DECODE):
                self.dec.generate_ids(self.group_prefix[slot], self.prompt_ids, self.cfg, out=self.group_ids[slot],
                                      workspace=self.dec_ws[lane])
            out = self.group_ids[slot]
            if self.gather is not None:
                out = self.gather(out, g * G)
            for i in range(G):
                self.outputs[slot * G + i] = out[i * B:(i + 1) * B]
            for ev in self._pending_end:
                ev.record()
            self._pending_end = []
            ev = torch.cuda.Event()
            ev.record()
            self.dec_done[slot] = ev

    def result(self, slot: int) -> torch.Tensor:
        if self.k % self.group and slot // self.group == (self.k // self.group) % self.depth:
            self.flush()   # the slot's group has not been decoded yet
        self.dec_done[slot // self.group].synchronize()
        return self.outputs[slot]

    def synchronize(self) -> None:
        self.flush()
        self.s_enc.synchronize()
        for s in self.s_decs:
            s.synchronize()

    def close(self) -> None:
        """Drain the streams.  The streams themselves stay in the per-process set (_stream_set) for the
        next pipeline with the same schedule; release_streams() destroys them."""
        self.synchronize()
