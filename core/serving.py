"""Request batching for the serving path.

Reference: server/services/inference_service.py:46-63 (request -> config -> engine -> infer under
the GPU gate), server/services/model_registry.py:12-44 (one engine per config, keyed by
json.dumps(asdict(config), sort_keys=True, default=str), created under a lock) and
server/services/task_manager.py:7-22 (a Semaphore(1) around GPU work).  The reference runs one
/infer request per engine call (batch 1).  Here concurrent requests whose configs map to the same
engine are coalesced - up to `max_batch` of them, waiting at most `max_wait_ms` for company - into
one InferenceEngine.infer_batch call: one fused encode for all videos and one batched decode per
caption candidate, so the GPU sees batch-8 work instead of eight batch-1 calls.  Results and
errors come back per request through futures; the registry and the GPU gate keep the reference's
semantics.

A request must fail alone, as it would in the reference's one-request-per-call service: videos
are loaded per request (a bad frames_dir fails only its own request), grouped by shape (frame
count and size: torch.cat of different clips would fail the whole call), cut into chunks the
decoder takes in one call (engine.max_batch_videos(): B * (prefix + prompt) <= vcap_gpt2_max_rows()
= 512 decode rows, and one full device beam chunk: <= 8 sequences, B * beams * (prefix + prompt) <= 512),
and a chunk whose engine call fails is retried one request at a time so only the offending
request gets the error.
"""
from __future__ import annotations

import json
import queue
import threading
import time
from collections import deque
from concurrent.futures import Future
from contextlib import contextmanager
from dataclasses import asdict
from pathlib import Path
from typing import Callable, Deque, Dict, List, Optional, Tuple


def engine_key(config) -> str:
    """Stable key for one model/runtime configuration (model_registry.py:12-15)."""
    return json.dumps(asdict(config), sort_keys=True, default=str)


class ModelRegistry:
    """One engine per configuration key, created once under a lock (model_registry.py:18-41)."""

    def __init__(self, factory: Optional[Callable] = None):
        self._engines: Dict[str, object] = {}
        self._lock = threading.Lock()
        self._factory = factory

    def get_engine(self, config):
        key = engine_key(config)
        with self._lock:
            engine = self._engines.get(key)
            if engine is None:
                if self._factory is None:
                    from core.engine import InferenceEngine
                    engine = InferenceEngine.from_config(config)
                else:
                    engine = self._factory(config)
                self._engines[key] = engine
            return engine


class GpuTaskManager:
    """Serial GPU execution gate (task_manager.py:7-22)."""

    def __init__(self, max_concurrent_tasks: int = 1):
        self._sem = threading.Semaphore(max_concurrent_tasks)

    @contextmanager
    def acquire(self):
        self._sem.acquire()
        try:
            yield
        finally:
            self._sem.release()


_Item = Tuple[str, object, str, Future]


class BatchingInferenceService:
    """submit(frames_dir, config) -> Future[InferenceResult]; one worker thread batches requests."""

    def __init__(self, registry: Optional[ModelRegistry] = None, gate: Optional[GpuTaskManager] = None,
                 max_batch: int = 8, max_wait_ms: float = 5.0):
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        self.registry = registry or ModelRegistry()
        self.gate = gate or GpuTaskManager(1)
        self.max_batch = max_batch
        self.max_wait = max_wait_ms / 1e3
        self._q: "queue.Queue[Optional[_Item]]" = queue.Queue()
        self._held: Deque[_Item] = deque()  # requests of other engines seen while filling a batch
        self._closed = False
        self.batches: List[int] = []        # sizes of the engine calls made (observability / tests)
        self._worker = threading.Thread(target=self._run, name="vcap-batcher", daemon=True)
        self._worker.start()

    def submit(self, frames_dir: str, config) -> Future:
        """Validate like InferenceService.infer (inference_service.py:50-55), then enqueue."""
        d = Path(frames_dir)
        if not d.exists() or not d.is_dir():
            raise FileNotFoundError(f"frames_dir not found: {d}")
        if getattr(config, "ckpt", "") and not Path(config.ckpt).exists():
            raise FileNotFoundError(f"ckpt not found: {config.ckpt}")
        if self._closed:
            raise RuntimeError("BatchingInferenceService is closed")
        fut: Future = Future()
        self._q.put((engine_key(config), config, str(d), fut))
        return fut

    def infer(self, frames_dir: str, config):
        return self.submit(frames_dir, config).result()

    def close(self, timeout: float = 60.0) -> None:
        """Finish every request already submitted, then stop the worker."""
        self._closed = True
        self._q.put(None)
        self._worker.join(timeout)

    # ---- worker
    def _take(self, timeout: float) -> Optional[_Item]:
        if self._held:
            return self._held.popleft()
        return self._q.get(timeout=timeout)

    def _run(self) -> None:
        stopping = False
        while True:
            try:
                first = self._take(0.05)
            except queue.Empty:
                if stopping:
                    return
                continue
            if first is None:
                stopping = True
                continue
            batch = [first]
            deadline = time.monotonic() + self.max_wait
            other: List[_Item] = []
            while len(batch) < self.max_batch:  # same-engine requests from the held list first
                same = [h for h in self._held if h[0] == first[0]]
                if not same:
                    break
                self._held.remove(same[0])
                batch.append(same[0])
            while len(batch) < self.max_batch and not stopping:
                left = deadline - time.monotonic()
                if left <= 0:
                    break
                try:
                    item = self._q.get(timeout=left)
                except queue.Empty:
                    break
                if item is None:
                    stopping = True
                    break
                (batch if item[0] == first[0] else other).append(item)
            self._held.extend(other)
            self._execute(first[1], batch)

    def _execute(self, config, batch: List[_Item]) -> None:
        try:
            engine = self.registry.get_engine(config)
        except BaseException as e:  # noqa: BLE001  (no engine: every request of this config fails)
            for b in batch:
                b[3].set_exception(e)
            return
        if not hasattr(engine, "load_video"):
            self._call(lambda items: engine.infer_batch([b[2] for b in items]), batch)
            return
        groups: Dict[tuple, List[Tuple[_Item, object]]] = {}
        for b in batch:
            try:
                with self.gate.acquire():
                    v = engine.load_video(b[2])
            except BaseException as e:  # noqa: BLE001
                b[3].set_exception(e)
                continue
            groups.setdefault(tuple(v.shape[1:]), []).append((b, v))
        cap = max(1, min(self.max_batch, int(engine.max_batch_videos())))
        for members in groups.values():
            for i in range(0, len(members), cap):
                chunk = members[i:i + cap]
                vids = {id(b): v for b, v in chunk}

                def run(items, vids=vids):
                    import torch
                    return engine.infer_videos(torch.cat([vids[id(b)] for b in items], dim=0))
                self._call(run, [b for b, _ in chunk])

    def _call(self, fn, items: List[_Item]) -> None:
        """One engine call for `items`; on failure retry each request alone (only the request that
        fails on its own gets the error)."""
        try:
            with self.gate.acquire():
                results = fn(items)
            if len(results) != len(items):
                raise RuntimeError(f"engine returned {len(results)} results for {len(items)} requests")
        except BaseException as e:  # noqa: BLE001
            if len(items) == 1:
                items[0][3].set_exception(e)
            else:
                for it in items:
                    self._call(fn, [it])
            return
        self.batches.append(len(items))
        for it, r in zip(items, results):
            it[3].set_result(r)
