"""Request coalescing: concurrent single-item calls -> one device batch.

The reference API is one query per request: each ``/searches`` request embeds
one query (llm/embed/embedding_service.py:114) and runs one ``collection.query``
(vectorstore/seekdb_connector.py:103-107).  A GPU wants batches.  ``Coalescer`` batches "while
busy": a call that finds the device idle runs at once, alone (no timer, no added latency); calls
that arrive while a batch is running queue up and the next batch takes all of them (up to
``max_batch``).  Leadership is handed to the first queued caller when a batch ends, so no caller
keeps serving other callers' requests after its own result is ready.  Results are per item and
identical to running the items one by one (the batched kernels are row-independent).
"""
from __future__ import annotations

import threading
from typing import Any, Callable, List, Sequence


class _Slot:
    __slots__ = ("item", "result", "error", "done", "lead", "event")

    def __init__(self, item):
        self.item = item
        self.result = None
        self.error = None
        self.done = False
        self.lead = False
        self.event = threading.Event()


class Coalescer:
    def __init__(self, run_batch: Callable[[Sequence[Any]], List[Any]], max_batch: int = 256):
        self._run = run_batch
        self.max_batch = max(1, int(max_batch))
        self._lock = threading.Lock()
        self._queue: List[_Slot] = []
        self._busy = False
        self.batches = 0        # number of device batches run (diagnostics)
        self.items = 0          # number of items served

    def __call__(self, item):
        slot = _Slot(item)
        with self._lock:
            self._queue.append(slot)
            if not self._busy:
                self._busy = True
                slot.lead = True
        while not slot.lead and not slot.done:
            slot.event.wait()
            slot.event.clear()
        if not slot.done:
            self._lead()
        if slot.error is not None:
            raise slot.error
        return slot.result

    def _lead(self) -> None:
        with self._lock:
            batch = self._queue[: self.max_batch]
            del self._queue[: self.max_batch]
        try:
            results = self._run([s.item for s in batch])
            if len(results) != len(batch):
                raise RuntimeError(f"coalesced batch returned {len(results)} results for "
                                   f"{len(batch)} items")
            for s, r in zip(batch, results):
                s.result = r
        except BaseException as e:  # noqa: BLE001 - every caller of the batch sees the failure
            for s in batch:
                s.error = e
        with self._lock:
            self.batches += 1
            self.items += len(batch)
            nxt = None
            if self._queue:
                nxt = self._queue[0]
                nxt.lead = True
            else:
                self._busy = False
        for s in batch:
            s.done = True
            s.event.set()
        if nxt is not None:
            nxt.event.set()
