"""Batch-level pipelining of the hot path over HIP streams.

The backbone's late blocks run one workgroup per CU at low occupancy and the head/decode kernels are small, so
a single stream leaves the GPU partly idle at the end of every batch. ``StreamPipeline`` keeps up to ``depth``
batches in flight, batch k on stream k % depth with its own SPEF context (workspace), so batch k's tail kernels
overlap batch k+1's front kernels. Weights are loaded into every context from the same blob (13.5 MB each for
the fp16 URSONet model -- nothing next to 288 GB of HBM).

This is the serving-side counterpart of the reference's evaluation loop (``tools/evaluation.py:63-90``), which
runs ``SPETorch.predict`` batch after batch; each submitted batch is still the complete forward + decode.

``use_graphs()`` (optional) records each (stream, input batch) pair's forward + decode once as a HIP graph and
replays it on later submits of the same input tensor: one graph launch per batch instead of ~20 kernel launches.
Its decode outputs then live in the graph's memory and are overwritten when that pair is submitted again. A recorded
graph holds fixed device addresses (the engine's workspace, the stream's output buffers, the decode tables), so its
key carries the engine's ``epoch`` (bumped by every workspace reallocation and state change) and the output buffers'
addresses, and a stream's graphs are dropped as soon as either moves.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from . import _lib as L
from .engine import Engine


class StreamPipeline:
    def __init__(self, blob, device, depth: int = 3, ori_bins: Optional[np.ndarray] = None,
                 pos_grid: Optional[np.ndarray] = None, comm=None, root: int = 0):
        """``blob``: the packed weights (host bytes or device tensor). With ``comm`` (a ``shard.RcclComm``), only
        rank ``root`` passes a blob (the others None) and every context receives the root's weights over RCCL
        (``spef_bcast_weights``, collective)."""
        assert depth >= 1
        self.device = torch.device(device)
        self.depth = depth
        self.engines: List[Engine] = [Engine(blob, self.device) for _ in range(depth)]
        if comm is not None:
            for e in self.engines:
                e.bcast_weights(comm, root)
        for e in self.engines:
            e.set_decode_tables(ori_bins, pos_grid)
        self.streams = [torch.cuda.Stream(self.device) for _ in range(depth)]
        self._bufs = [None] * depth
        self._next = 0
        self.graphs = False
        self._graphs = {}

    def use_graphs(self, on: bool = True) -> None:
        self.graphs = bool(on)
        if not on:
            self._graphs.clear()

    @property
    def engine(self) -> Engine:
        return self.engines[0]

    def reserve(self, B: int, H: int, W: int) -> None:
        for e in self.engines:
            e.reserve(B, H, W)

    def submit(self, frames: torch.Tensor, ori_mode: int = L.CLASSIFICATION, pos_mode: int = L.REGRESSION,
               want_soft: bool = True) -> dict:
        """Enqueue forward + decode of one batch on the next stream; returns the decode dict (device tensors,
        valid once that stream reaches them -- ``synchronize()`` or the dict's 'event')."""
        i = self._next
        self._next = (i + 1) % self.depth
        eng, s = self.engines[i], self.streams[i]
        B = frames.shape[0]
        buf = self._bufs[i]
        if buf is None or buf[0].shape[0] != B:
            buf = (torch.empty((B, eng.n_out0), dtype=torch.float32, device=self.device),
                   torch.empty((B, eng.n_out1), dtype=torch.float32, device=self.device) if eng.n_out1 else None)
            self._bufs[i] = buf
            self._drop_graphs(i)                                 # recorded against the previous buffers
        s.wait_stream(torch.cuda.current_stream(self.device))   # frames were produced on the caller's stream
        if self.graphs:
            return self._submit_graph(i, eng, s, buf, frames, ori_mode, pos_mode, want_soft)
        with torch.cuda.stream(s):
            frames.record_stream(s)
            raw0, raw1 = eng.forward(frames, *buf)
            dec = eng.decode(ori_mode, pos_mode, raw0, raw1, want_soft=want_soft)
            ev = torch.cuda.Event()
            ev.record(s)
        dec['raw0'], dec['raw1'] = raw0, raw1
        dec['event'] = ev
        return dec

    def _drop_graphs(self, i: int) -> None:
        for k in [k for k in self._graphs if k[0] == i]:
            del self._graphs[k]

    def _submit_graph(self, i, eng, s, buf, frames, ori_mode, pos_mode, want_soft) -> dict:
        _, B, H, W = eng._layout(frames)
        eng.reserve(B, H, W)                                     # any reallocation happens before the key is taken
        bufkey = tuple(0 if t is None else t.data_ptr() for t in buf)
        key = (i, frames.data_ptr(), tuple(frames.shape), frames.dtype, ori_mode, pos_mode, want_soft, eng.epoch,
               bufkey)
        stale = [k for k in self._graphs if k[0] == i and (k[7] != eng.epoch or k[8] != bufkey)]
        for k in stale:                                          # their workspace / buffers may be freed memory now
            del self._graphs[k]
        ent = self._graphs.get(key)
        if ent is None:
            with torch.cuda.stream(s):   # one eager pass first: lazily set kernel attributes stay out of the capture
                raw0, raw1 = eng.forward(frames, *buf)
                eng.decode(ori_mode, pos_mode, raw0, raw1, want_soft=want_soft)
            s.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                raw0, raw1 = eng.forward(frames, *buf)
                dec = eng.decode(ori_mode, pos_mode, raw0, raw1, want_soft=want_soft)
            ent = self._graphs[key] = (g, dec)
        g, dec0 = ent
        with torch.cuda.stream(s):
            frames.record_stream(s)
            g.replay()
            ev = torch.cuda.Event()
            ev.record(s)
        dec = dict(dec0)
        dec['raw0'], dec['raw1'] = buf
        dec['event'] = ev
        return dec

    def set_keypoints(self, kp3d: np.ndarray, K: np.ndarray, nu: float, nv: float, dist=None) -> None:
        for e in self.engines:
            e.set_keypoints(kp3d, K, nu, nv, dist)

    def submit_keypoints(self, frames: torch.Tensor) -> dict:
        """Keypoint mode: forward (KeypointRegressionHead) + sigmoid + batched EPnP of one batch on the next stream;
        returns the decode dict of Engine.decode_keypoints plus 'raw' and 'event' (as submit())."""
        i = self._next
        self._next = (i + 1) % self.depth
        eng, s = self.engines[i], self.streams[i]
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            frames.record_stream(s)
            raw, _ = eng.forward(frames)   # allocated on s: every returned tensor belongs to this batch alone
            dec = eng.decode_keypoints(raw)
            ev = torch.cuda.Event()
            ev.record(s)
        dec['raw'] = raw
        dec['event'] = ev
        return dec

    def synchronize(self) -> None:
        for s in self.streams:
            s.synchronize()

    def close(self) -> None:
        self.synchronize()
        self._graphs.clear()
        for e in self.engines:
            e.close()
        self.engines = []
