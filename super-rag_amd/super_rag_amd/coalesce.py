"""Request coalescing: concurrent single-item calls -> one device batch.

The reference API is one query per request: each ``/searches`` request embeds
one query (llm/embed/embedding_service.py:114) and runs one ``collection.query``
(vectorstore/seekdb_connector.py:103-107).  A GPU wants batches.  ``Coalescer`` batches "while
busy": a call that finds the device idle runs at once, alone (no timer, no added latency); calls
that arrive while a batch is running queue up and the next batch takes all of them (up to
``max_batch``).  Leadership is handed to the first queued caller when a batch ends, so no caller
keeps serving other callers' requests after its own result is ready.  Results are per item and
identical to running the items one by one (the batched kernels are row-independent).

``acall`` is the same queue for coroutines: a waiting coroutine holds no thread (its slot carries
an asyncio future, completed with one ``call_soon_threadsafe`` per event loop per batch).  The
batches of coroutine slots are led by ONE daemon thread the coalescer owns, which keeps leading
while the next queued slot is a coroutine's.  With one worker thread blocked per waiting request
(``asyncio.to_thread`` around ``__call__``), every finished batch woke its ~30 callers' threads,
which then contended for the interpreter lock.  The leader is not a worker of the caller's event
loop: that loop's executor may be full of sync callers blocked on this same coalescer, or the loop
thread itself may be blocked in a sync ``__call__`` (the reference calls ``embed_query`` on the
loop: nodeflow/runners/vector_search.py:76), and either would leave the queue led by nobody.
"""
from __future__ import annotations

import asyncio
import logging
import threading
import time
from typing import Any, Callable, List, Sequence


logger = logging.getLogger(__name__)


class _Slot:
    __slots__ = ("item", "result", "error", "done", "lead", "event", "loop", "fut")

    def __init__(self, item, loop=None):
        self.item = item
        self.result = None
        self.error = None
        self.done = False
        self.lead = False
        self.loop = loop                                   # acall: the caller's event loop
        self.fut = loop.create_future() if loop is not None else None
        self.event = threading.Event() if loop is None else None


def _finish(slots) -> None:
    """(in the slots' event loop) complete the futures of one batch's coroutine slots."""
    for s in slots:
        if s.fut.done():  # cancelled by its caller
            continue
        if s.error is not None:
            s.fut.set_exception(s.error)
        else:
            s.fut.set_result(s.result)


class Coalescer:
    def __init__(self, run_batch: Callable[[Sequence[Any]], List[Any]], max_batch: int = 256,
                 min_fill: int = 1, max_wait_s: float = 0.0):
        self._run = run_batch
        self.max_batch = max(1, int(max_batch))
        # fill wait: a leader that finds fewer than min_fill items queued waits up to max_wait_s
        # for more before running the batch (1 / 0: run at once, the batch-while-busy default)
        self.min_fill = max(1, int(min_fill))
        self.max_wait_s = max(0.0, float(max_wait_s))
        self._lock = threading.Lock()
        self._more = threading.Condition(self._lock)
        self._queue: List[_Slot] = []
        self._busy = False
        self.batches = 0        # number of device batches run (diagnostics)
        self.items = 0          # number of items served
        # the owned leader of coroutine batches: started on first use, woken by _wake_leader
        self._cv = threading.Condition(threading.Lock())
        self._wake = False
        self._leader = None

    def __call__(self, item):
        slot = _Slot(item)
        with self._lock:
            self._queue.append(slot)
            self._more.notify()
            if not self._busy:
                self._busy = True
                slot.lead = True
        while not slot.lead and not slot.done:
            slot.event.wait()
            slot.event.clear()
        if not slot.done:
            self._lead(caller=True)
        if slot.error is not None:
            raise slot.error
        return slot.result

    async def acall(self, item):
        """``__call__`` for a coroutine: same batches, same per-item results, no thread held while
        the item waits for its batch."""
        slot = _Slot(item, asyncio.get_running_loop())
        lead = False
        with self._lock:
            self._queue.append(slot)
            self._more.notify()
            if not self._busy:
                self._busy = True
                lead = True
        if lead:
            self._wake_leader()
        return await slot.fut

    def _wake_leader(self) -> None:
        """Hand the lead (this caller holds it: _busy is set) to the owned leader thread.  If that
        thread cannot be started (interpreter shutdown), lead here instead: _busy must never stay
        set with nobody leading."""
        try:
            with self._cv:
                if self._leader is None or not self._leader.is_alive():
                    t = threading.Thread(target=self._leader_loop, name="coalescer-leader", daemon=True)
                    t.start()
                    self._leader = t
                self._wake = True
                self._cv.notify()
        except BaseException:  # noqa: BLE001 - no leader thread: serve the queue inline
            self._lead()

    def _leader_loop(self) -> None:
        while True:
            with self._cv:
                while not self._wake:
                    self._cv.wait()
                self._wake = False
            try:
                self._lead()
            except BaseException as e:  # noqa: BLE001 - _lead_one reports batch failures itself
                logger.error("coalescer leader failed: %r", e)

    def _lead(self, caller: bool = False) -> None:
        """Run batches while the queue's next slot is a coroutine's (it has no thread of its own
        to lead with); hand over to a queued thread caller, or go idle.  A thread CALLER that led
        (caller=True) does not serve coroutines after its own batch: the owned leader thread takes
        over, so the caller returns."""
        while self._lead_one(caller):
            pass

    def _lead_one(self, caller: bool = False) -> bool:
        with self._lock:
            if self.min_fill > 1 and self.max_wait_s > 0 and len(self._queue) < self.min_fill:
                deadline = time.monotonic() + self.max_wait_s
                while len(self._queue) < self.min_fill:
                    rem = deadline - time.monotonic()
                    if rem <= 0:
                        break
                    self._more.wait(rem)
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
            keep = False
            hand_off = False
            if self._queue:
                nxt = self._queue[0]
                if nxt.fut is None:
                    nxt.lead = True
                elif caller:
                    hand_off = True  # the owned leader thread leads the coroutines' batches
                    nxt = None
                else:
                    keep = True  # a coroutine's slot: this worker runs the next batch too
                    nxt = None
            else:
                self._busy = False
        by_loop = {}
        for s in batch:
            s.done = True
            if s.fut is None:
                s.event.set()
            else:
                by_loop.setdefault(s.loop, []).append(s)
        for loop, slots in by_loop.items():
            try:
                loop.call_soon_threadsafe(_finish, slots)
            except RuntimeError:  # the caller's loop has closed: nobody awaits these
                pass
        if nxt is not None:
            nxt.event.set()
        if hand_off:
            self._wake_leader()
        return keep
